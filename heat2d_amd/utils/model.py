"""Analytic cost models: the reference report's strips-vs-blocks model and an MI355X model of
this framework's temporally-blocked, halo-overlapped execution.

Reference model (Report.pdf p.10-11, "Σχεδιασμός διαμοιρασμού δεδομένων"; SURVEY C-DOC-2):
``T = Tcomp + Tcomm`` with a message costing ``Tmsg = ts + tw·L``.  For an M×N grid on P
processes (M >= N):

* strips (P strips of columns):   ``T = tc·M·(⌊N/P⌋ + 1) + 2·ts + 4·M·tw``
* blocks (√P × √P):               ``T = 4·ts + (4·tw + tc)·(⌊M/√P⌋ + 1)·(⌊N/√P⌋ + 1)``

(the blocks line is printed that way in the report — its communication term 2(ts + 2tw(⌊M/√P⌋+1))
+ 2(ts + 2tw(⌊N/√P⌋+1)) was folded into the area term; we reproduce the report as published).
Speedup and efficiency are model against model, ``S(P) = T(1)/T(P)``, ``E = S/P``
(Tables 14-19, p.29-32: e.g. blocks, 2560×2048, P=160 -> 0.119 s, E = 0.997).  Measured
constants (mpptest): tc = 0.025 µs, ts = 0.6 µs, tw = 0.9 µs (p.11).

MI355X model (this framework, ``docs/MODEL.md``).  One GPU per rank; the tile of a rank is
X rows × Y columns; time advances in chunks of K fused steps (one kernel launch each).  The
streaming kernel gives every wave a 256-column strip of ``R = round_up(K,4)`` lead columns per
side (``ceil((Y - 2R)/(256 - 2R))`` strips, edge-aligned at fixed edges) and ``h`` rows, with
one wave per SIMD (VALU-bound).  A unit of ``h`` rows costs ``K·(h + K - 1)`` level-rows
(the K-cone), each ``t_lr`` on its SIMD; a launch adds ``F``:

    T_chunk(X, Y, K) = F + max(K·(h + K − 1)·t_lr, 8·X·Y / BW),   h = X·strips / SIMDs
    T_step = T_chunk / K

Halo exchange (direct IPC pipeline): halo units push their first G rows into the neighbour's
receive buffer as soon as those rows are final and the neighbour's next chunk waits for them
in-kernel, so the exposed communication per chunk is ``max(0, t_sig + L_xgmi − T_chunk)``
(zero when a chunk is longer than the hand-off latency).  Constants are fitted to MI355X
measurements (profiles/strong_proxy_r2.txt): ``t_lr`` ≈ 99 ns (ref precision), F ≈ 3.2 µs
(an empty launch of the stream kernel in the kernel trace), L_xgmi a few µs (placeholder until
the 8-GPU SCALE run measures it).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Iterable, List, Tuple

# ---- the report's model ----------------------------------------------------------------------

REPORT_TC_US = 0.025
REPORT_TS_US = 0.6
REPORT_TW_US = 0.9


def report_time_strips(M: int, N: int, P: int, tc: float = REPORT_TC_US, ts: float = REPORT_TS_US,
                       tw: float = REPORT_TW_US) -> float:
    """Report model, strips: T in µs (Report.pdf p.10)."""
    M, N = max(M, N), min(M, N)
    return tc * M * (N // P + 1) + 2 * ts + 4 * M * tw


def report_time_blocks(M: int, N: int, P: int, tc: float = REPORT_TC_US, ts: float = REPORT_TS_US,
                       tw: float = REPORT_TW_US) -> float:
    """Report model, √P×√P blocks: T in µs (Report.pdf p.11)."""
    M, N = max(M, N), min(M, N)
    r = math.sqrt(P)
    return 4 * ts + (4 * tw + tc) * (math.floor(M / r) + 1) * (math.floor(N / r) + 1)


def report_tables(grids: Iterable[Tuple[int, int]], procs: Iterable[int], kind: str = "blocks") -> Dict:
    """{(M, N): [(P, T_s, S, E), ...]} in the report's units (T printed in seconds = µs·1e-6)."""
    f = report_time_blocks if kind == "blocks" else report_time_strips
    out = {}
    for M, N in grids:
        t1 = f(M, N, 1)
        rows = []
        for P in procs:
            t = f(M, N, P)
            s = t1 / t
            rows.append((P, t * 1e-6, s, s / P))
        out[(M, N)] = rows
    return out


REPORT_GRIDS = [(80, 64), (160, 128), (320, 256), (640, 512), (1280, 1024), (2560, 2048)]
REPORT_PROCS = [1, 4, 16, 64, 128, 160]  # the measured tables' task counts (nodes/tasks 1/1 .. 20/160)

# ---- MI355X model ------------------------------------------------------------------------------


@dataclass
class Mi355xConstants:
    simds: int = 1024          # 256 CUs x 4 SIMDs: one resident stencil wave per SIMD
    t_lr_ns: float = 99.0      # one level-row (256 columns x 1 row x 1 time level) of one wave, ref precision
    launch_us: float = 3.2     # fixed cost of one chunk launch (empty stream-kernel launch, kernel trace)
    wave_cols: int = 256
    l_xgmi_us: float = 5.0     # halo hand-off latency between GPUs (push + release + remote flag): placeholder
    host_us: float = 15.0      # fixed host cost of one timed run (first dispatch + final sync)
    hbm_tbs: float = 4.5       # streaming bandwidth when both buffers exceed the 256 MiB Infinity Cache
    mall_tbs: float = 10.0     # ... when they fit in it
    mall_bytes: float = 256 * 2**20


def lead(K: int) -> int:
    return (K + 3) // 4 * 4


def strips(Y: int, K: int, fixed: bool = True, wave_cols: int = 256) -> int:
    R = lead(K)
    if fixed and Y >= wave_cols:  # edge-aligned end strips output 256 - R columns
        inner = max(0, Y - 2 * (wave_cols - R))
        return 2 + math.ceil(inner / (wave_cols - 2 * R))
    return max(1, math.ceil(Y / (wave_cols - 2 * R)))


def chunk_time_us(X: int, Y: int, K: int, c: Mi355xConstants = Mi355xConstants(), fixed: bool = True) -> float:
    """Model time of one K-step launch on an X×Y tile (µs)."""
    s = strips(Y, K, fixed, c.wave_cols)
    units = min(c.simds, max(s, s * max(1, X // 8)))  # units never go below 8 rows
    h = X * s / units
    compute = K * (h + K - 1) * c.t_lr_ns * 1e-3
    # each launch reads the tile once and writes it once (+ the cone rows)
    nbytes = 2 * 4.0 * X * Y
    bw = c.mall_tbs if nbytes <= c.mall_bytes else c.hbm_tbs
    memory = nbytes / (bw * 1e12) * 1e6
    return c.launch_us + max(compute, memory)


def step_time_us(X: int, Y: int, K: int, c: Mi355xConstants = Mi355xConstants(), exchange: bool = False) -> float:
    """Model time per step (µs) of one rank; with `exchange`, adds the exposed halo latency of
    the direct pipeline (the hand-off overlaps the chunk: only what exceeds it is exposed)."""
    tc = chunk_time_us(X, Y, K, c)
    exposed = max(0.0, c.l_xgmi_us + 0.3 * tc - tc) if exchange else 0.0
    return (tc + exposed) / K


def best_k(X: int, Y: int, ks=(2, 3, 4, 5, 6, 7, 8, 10, 12, 16), c: Mi355xConstants = Mi355xConstants(),
           exchange: bool = False) -> Tuple[int, float]:
    return min(((k, step_time_us(X, Y, k, c, exchange)) for k in ks), key=lambda kv: kv[1])


def strong_scaling(side: int, gpus: Iterable[int], layout: str = "rows", steps: int = 1000,
                   c: Mi355xConstants = Mi355xConstants()) -> List[dict]:
    """Predicted time / speedup / efficiency of a side×side grid on 1..N GPUs (strong scaling),
    the per-rank tile at its best K, `steps` steps plus the host's fixed cost of the run."""
    out = []
    t1 = None
    for n in gpus:
        if layout == "rows":
            X, Y = math.ceil(side / n), side
        else:
            gx = int(math.isqrt(n))
            while n % gx:
                gx -= 1
            gy = n // gx
            X, Y = math.ceil(side / gx), math.ceil(side / gy)
        k, us = best_k(X, Y, c=c, exchange=n > 1)
        t = (us * steps + c.host_us) * 1e-6
        if t1 is None:
            t1 = t
        s = t1 / t
        out.append(dict(gpus=n, tile=(X, Y), K=k, us_per_step=us, time_s=t, speedup=s, efficiency=s / n,
                        cups=side * side * steps / t))
    return out
