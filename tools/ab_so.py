"""A/B of two builds of the native extension on the headline shape (4096^2, ref, depth 7):
python tools/ab_so.py DIR_A DIR_B — each DIR holds a _heat2d*.so; every measurement runs in its
own process (alternating A, B, A, B, ...), 1000-step and 20-step median times."""
import os
import subprocess
import sys

CHILD = r'''
import importlib.machinery, importlib.util, sys, time, glob
so = glob.glob(sys.argv[1] + "/_heat2d*.so")[0]
spec = importlib.util.spec_from_file_location("_heat2d", so)
n = importlib.util.module_from_spec(spec); spec.loader.exec_module(n)
e = n.Engine(4096, 4096, tblock=7, device=0, small_grid_lds=False, tiled=0, sync_mode=2)
t_end = time.perf_counter() + 1.5
while time.perf_counter() < t_end:
    e.run(140); e.synchronize()
out = []
for steps in (1000, 20):
    ts = []
    for _ in range(5):
        e.synchronize(); t0 = time.perf_counter(); e.run(steps); e.synchronize(); ts.append(time.perf_counter() - t0)
    out.append(sorted(ts)[2] / steps * 1e6)
print("%.4f %.4f" % tuple(out))
'''

res = {}
for rnd in range(3):
    for d in sys.argv[1:3]:
        r = subprocess.run([sys.executable, "-c", CHILD, d], capture_output=True, text=True, timeout=240)
        v = r.stdout.strip().split()
        res.setdefault(d, []).append(v)
        print(f"{os.path.basename(d.rstrip('/'))} round {rnd}: us/step 1000 steps {v[0] if v else '?'}, 20 steps "
              f"{v[1] if len(v) > 1 else '?'} {r.stderr[-200:] if r.returncode else ''}", flush=True)
