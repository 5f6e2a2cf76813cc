"""Worker of test_gpu_halo_wait_sees_a_late_neighbour (run by torch.distributed.run, 2 ranks on one
GPU): two row strips through the direct IPC pipeline; rank 1 starts its second run 50 ms late, so
rank 0's halo units wait for its pushes — the halo-wait counters must show it."""
import json
import os
import sys
import time

import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
dist.init_process_group("gloo")
rank = dist.get_rank()
e = n.Engine(256, 1024, gridx=2, gridy=1, tblock=7, device=0, ranks=[rank], transport=n.TRANSPORT_IPC,
             halo_timeout_s=10.0, persistent=0)
hs = [None, None]
dist.all_gather_object(hs, e.ipc_handle())
e.ipc_open(hs)
dist.barrier()
e.ipc_prime()
dist.barrier()
e.run(14)
e.synchronize()
dist.barrier()
e.reset_halo_wait()
dist.barrier()
if rank == 1:
    time.sleep(0.05)
e.run(28)
e.synchronize()
hw = e.halo_wait()
print(json.dumps({"rank": rank, **hw}), flush=True)
dist.barrier()
dist.destroy_process_group()
