"""Interleaved A/B timing of engine variants on one GPU.

usage: python tools/ab_kernel.py NX NY STEPS ROUNDS 'name:opt=v,opt=v' 'name:opt=v' ...

Every variant gets its own engine (built once, warmed up); the rounds alternate A, B, ... so that
clock and thermal drift hit every variant alike.  Prints each variant's median and best us/step
(host wall time around Engine.run, the device synchronised on both sides) and its ratio to the
first variant.  Example: the per-wave integrity preamble against none (debug_kernel bit 2):
  python tools/ab_kernel.py 4096 4096 1000 7 'checks:tblock=7' 'nochecks:tblock=7,debug_kernel=2'
"""
import os
import statistics
import sys
import time

import torch  # noqa: F401  (the shared HIP runtime)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from heat2d_amd._native import native  # noqa: E402


def parse(spec):
    name, _, opts = spec.partition(":")
    kw = {}
    for kv in filter(None, opts.split(",")):
        k, v = kv.split("=")
        kw[k] = float(v) if "." in v else int(v)
    return name, kw


def main(argv):
    nx, ny, steps, rounds = (int(v) for v in argv[:4])
    n = native()
    variants = [parse(s) for s in argv[4:]]
    engines = []
    for name, kw in variants:
        kw = dict(dict(device=0, small_grid_lds=False), **kw)
        e = n.Engine(nx, ny, **kw)
        e.run(max(steps, 200))  # warm: every plan, block and code object
        engines.append((name, e))
    times = {name: [] for name, _ in engines}
    for _ in range(rounds):
        for name, e in engines:
            e.synchronize()
            t0 = time.perf_counter()
            e.run(steps)
            e.synchronize()
            times[name].append((time.perf_counter() - t0) / steps * 1e6)
    base = statistics.median(times[engines[0][0]])
    for name, _ in engines:
        med = statistics.median(times[name])
        print(f"{name:16s} {nx}x{ny} {steps} steps: median {med:8.3f} us/step  best {min(times[name]):8.3f}  "
              f"x{med / base:6.3f}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
