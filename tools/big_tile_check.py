"""Huge-tile validation (the BASELINE's ~288 GB/GPU weak-scaling tile): 64-bit indexing, unit
planning and throughput at N×N with N≈180k (2 fp32 buffers ≈ 259 GB), plus a correctness
check of a 2^31+-cell tile against the PyTorch reference on a cropped window."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import heat2d_amd  # noqa: E402
from heat2d_amd.ops import reference as R  # noqa: E402

n = heat2d_amd.native()
p = n.device_props(0)
print("device", p["name"], p["gcn_arch"], "mem GB", p["total_global_mem"] / 1e9, flush=True)

# (1) correctness beyond 2^31 cells: 49152 x 49152 = 2.4e9 cells, fixed edges, 16 steps.
N1 = int(os.environ.get("BIG_N1", "49152"))
e = n.Engine(N1, N1, device=0, tblock=8)
e.run(16)
t = e.download(0)  # host copy (9.6 GB)
top = torch.from_numpy(t[:64, :64].copy())
ref = R.run(R.center_hot(N1, N1)[:80, :80].contiguous(), 16)[:64, :64]  # window far from other edges
print("2^31+ tile corner bit-exact:", torch.equal(top, ref), flush=True)
bot = torch.from_numpy(t[N1 - 64:, N1 - 64:].copy())
full_corner = R.center_hot(N1, N1)[N1 - 80:, N1 - 80:].contiguous()
refb = R.run(full_corner, 16)[16:, 16:]
print("far corner bit-exact:", torch.equal(bot, refb), flush=True)
del e, t

# (2) the 288 GB-class tile: throughput over a few chunks
N2 = int(os.environ.get("BIG_N2", "180000"))
t0 = time.perf_counter()
e = n.Engine(N2, N2, device=0, tblock=8)
print(f"{N2}^2 tile: setup {time.perf_counter() - t0:.1f} s, units(K=8) {e.num_units(8)}", flush=True)
e.run(8)
st = e.run(32)
cells = N2 * N2 * 32
print(f"{N2}^2: {st['device_ms'] / 32:.2f} ms/step, {cells / (st['device_ms'] / 1e3):.3e} cell-updates/s", flush=True)
