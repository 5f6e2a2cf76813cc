"""Worker of tests/test_node_barrier.py (launched by torch.distributed.run): every rank goes
through the node barrier R times, recording when it arrived and when it left; rank 0 gathers
the records and writes them as JSON to argv[1]."""
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd.parallel.dist import init_distributed  # noqa: E402

ctx = init_distributed()
rounds = int(sys.argv[2])
rng = random.Random(ctx.rank)
arr, dep = [], []
for i in range(rounds):
    # uneven arrival: up to 2 ms of skew per round
    t_end = time.perf_counter() + rng.random() * 2e-3
    while time.perf_counter() < t_end:
        pass
    arr.append(time.perf_counter())
    ctx.node_barrier()
    dep.append(time.perf_counter())
recs = ctx.gather_objects({"rank": ctx.rank, "arr": arr, "dep": dep, "shm": ctx._shm_state})
if ctx.rank == 0:
    with open(sys.argv[1], "w") as f:
        json.dump(recs, f)
ctx.shutdown()
