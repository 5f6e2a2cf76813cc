"""Worker of test_gpu_persistent_two_processes (torch.distributed.run, 2 ranks on one GPU): row
strips through the direct IPC pipeline with the persistent kernel on both ranks (small tiles, so
both launches' waves fit on the GPU together); every rank's tile is compared with the oracle.
Argument `conv`: with the fused convergence check every 20 steps (the chunks between checks are
persistent launches, the decision goes through the IPC all-reduce); the run must stop at the
oracle's step with the oracle's grid; after a re-prime the next run converges again at that
step (it starts on the converged check's step) with the same grid."""
import json
import os
import sys

import numpy as np
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402

n = native()
dist.init_process_group("gloo")
rank = dist.get_rank()
nx, ny, K, steps = 2 * 192 + 1, 2048, 8, 5 * 8 + 3
conv = len(sys.argv) > 1 and sys.argv[1] == "conv"
kw = {}
if conv:
    # converges at the check of step 60 (between the residuals of the checks at 40 and 60)
    r = [n.oracle_run(nx, ny, s, convergence=True, interval=20, sensitivity=0.0)["residual"] for s in (40, 60)]
    kw = dict(convergence=True, interval=20, sensitivity=0.5 * (r[0] + r[1]))
    steps = 200
e = n.Engine(nx, ny, gridx=2, gridy=1, tblock=K, device=0, ranks=[rank], transport=n.TRANSPORT_IPC,
             halo_timeout_s=10.0, persistent=1, pstream_cols=128,
             debug_kernel=int(os.environ.get("H2D_DEBUG_KERNEL", "0")), **kw)
# Both ranks' persistent launches share the GPU and each needs all of its waves resident: run
# only if the two plans fit on the device together, else report a skip.
blocks = (len(e.pstream_units(K)) + 3) // 4
allb = [None, None]
dist.all_gather_object(allb, blocks)
cap = n.device_props(0)["multiprocessor_count"] * n.pstream_blocks_per_cu(K, 0, 2)
if sum(allb) > cap:
    print(json.dumps({"rank": rank, "skip": f"plans need {sum(allb)} blocks, the GPU holds {cap}"}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0)
hs = [None, None]
dist.all_gather_object(hs, e.ipc_handle())
e.ipc_open(hs)
dist.barrier()
e.ipc_prime()
dist.barrier()
st = e.run(steps)
e.synchronize()
g = e.geom(0)
full = n.oracle_run(nx, ny, steps, **kw)
ref = full["grid"][g["gx0"]:g["gx0"] + g["xcell"], :]
got = e.download(0)
ok = bool(np.array_equal(got, ref))
if conv:
    ok = ok and bool(st["converged"]) and full["converged"] and st["steps_done"] == full["steps_done"]
    steps = int(full["steps_done"])
    dist.barrier()
    e.ipc_prime()  # a converged run leaves the neighbours' receive buffers one chunk ahead
    dist.barrier()


def where(got, ref):
    bad = got != ref
    if not bad.any():
        return None
    r, c = np.nonzero(bad)
    return [int(bad.sum()), int(r.min()), int(r.max()), int(c.min()), int(c.max()), sorted(set(r.tolist()))[:12]]


bad1 = where(got, ref)
dist.barrier()
st2 = e.run(2 * K)
e.synchronize()
ref2 = ref if conv else n.oracle_run(nx, ny, steps + 2 * K)["grid"][g["gx0"]:g["gx0"] + g["xcell"], :]
got2 = e.download(0)
ok2 = bool(np.array_equal(got2, ref2))
if conv:
    ok2 = ok2 and bool(st2["converged"]) and st2["steps_done"] == steps
print(json.dumps({"rank": rank, "ok": ok, "ok2": ok2, "launches": e.pstream_launches(),
                  "steps_done": int(e.steps_done())}), flush=True)
if not (ok and ok2):
    print(f"rank {rank} xcell {g['xcell']}: first run wrong {bad1}; second {where(got2, ref2)}", flush=True)
dist.barrier()
dist.destroy_process_group()
