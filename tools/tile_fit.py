"""Per-launch time of the LDS-tiled kernel against steps per launch K (fixed tile shape):
fits T_launch = F + c·K to split the fixed launch cost F from the per-level cost c.
  python tools/tile_fit.py NX NY RY TX NT CPL [K,K,...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import heat2d_amd  # noqa: E402

n = heat2d_amd.native()
nx, ny, ry, tx, nt, cpl = (int(v) for v in sys.argv[1:7])
ks = [int(v) for v in sys.argv[7].split(",")] if len(sys.argv) > 7 else [1, 2, 4, 6, 8, 12]
pts = []
for K in ks:
    steps = 960
    e = n.Engine(nx, ny, device=0, tiled=1, tile_width=ry, tile_k=K, tile_rows=tx, tile_threads=nt, tile_cpl=cpl,
                 small_grid_lds=False)
    e.run(steps)
    us = min(e.run(steps)["device_ms"] for _ in range(3)) * 1e3 / steps
    pts.append((K, us * K))
    print(f"{nx}x{ny} RY={ry} TX={tx} NT={nt} CPL={cpl} K={K:2d}: {us:.3f} us/step, {us * K:.2f} us/launch", flush=True)
k_mean = sum(k for k, _ in pts) / len(pts)
t_mean = sum(t for _, t in pts) / len(pts)
c = sum((k - k_mean) * (t - t_mean) for k, t in pts) / sum((k - k_mean) ** 2 for k, _ in pts)
print(f"fit: F = {t_mean - c * k_mean:.2f} us per launch, c = {c:.3f} us per level")
