"""Banners and metrics, byte-compatible with the reference programs' stdout (C-IO-4).

Sources: ``grad1612_mpi_heat.c:66-69,192,287``; ``grad1612_hybrid_heat.c:70,204,318``;
``mpi_heat2Dn.c:79-83,113-114,130-133,174,206``; ``grad1612_cuda_heat.cu:73,89``.
The JSON line is an extension (metrics/observability).
"""
from __future__ import annotations

import json
import sys
from typing import Optional, TextIO


def cfmt_e(x: float) -> str:
    """C's ``%e``."""
    return "%e" % x


class Reporter:
    def __init__(self, style: str, enabled: bool = True, out: Optional[TextIO] = None):
        self.style = style
        self.enabled = enabled
        self.out = out or sys.stdout

    def _p(self, s: str) -> None:
        if self.enabled:
            self.out.write(s)
            self.out.flush()

    # ---- before the loop -----------------------------------------------------------------
    def start(self, *, nprocs: int, nx: int, ny: int, xcell: int, ycell: int, steps: int, convergence: bool,
              interval: int, numthreads: int = 4, strips: Optional[list] = None) -> None:
        st = self.style
        if st in ("grad", "hybrid"):
            if st == "grad":
                self._p("Starting with %d processes\n" % nprocs)
            else:
                self._p("Starting with %d processes and %d threads\n" % (nprocs, numthreads))
            self._p("Problem size:%dx%d\nEach process will take: %dx%d\nAmount of iterations: %d\n"
                    % (nx, ny, xcell, ycell, steps))
            if convergence:
                self._p("Check for convergence every %d iterations\n" % interval)
        elif st == "heat2dn":
            self._p("Starting mpi_heat2D with %d worker tasks.\n" % nprocs)
            self._p("Grid size: X= %d  Y= %d  Time steps= %d\n" % (nx, ny, steps))
            self._p("Initializing grid and writing initial.dat file...\n")
            for s in strips or []:
                self._p("Sent to task %d: rows= %d offset= %d left= %d right= %d\n"
                        % (s["task"], s["rows"], s["offset"], s["left"], s["right"]))
        elif st == "cuda":
            self._p("Problem size: %dx%d\nAmount of iterations: %d\n" % (nx, ny, steps))

    def writing_initial(self) -> None:
        if self.style in ("grad", "hybrid"):
            self._p("Writing initial.dat ...\n")

    def begin_steps(self, strips: Optional[list] = None) -> None:
        if self.style == "heat2dn":
            for s in strips or []:
                self._p("Task %d received work. Beginning time steps...\n" % s["task"])

    # ---- after the loop ------------------------------------------------------------------
    def finish(self, *, steps_done: int, elapsed_s: float, writes_final: bool) -> None:
        st = self.style
        if st in ("grad", "hybrid"):
            self._p("Exiting after %d iterations\nElapsed time: %s sec\n" % (steps_done, cfmt_e(elapsed_s)))
            if writes_final:
                self._p("Writing final.dat ...\n")
        elif st == "heat2dn":
            self._p("Elapsed time: %s sec\n" % cfmt_e(elapsed_s))
            self._p("Writing final.dat file and generating graph...\n")
            self._p("Click on MORE button to view initial/final states.\n")
            self._p("Click on EXIT button to quit program.\n")
        elif st == "cuda":
            self._p("Elapsed time: %s sec\n" % cfmt_e(elapsed_s))

    def debug_neighbors(self, rank: int, nb: dict, host: str) -> None:
        # grad1612_mpi_heat.c:170-175
        self._p("I am %d and my neighbors are North=%d, South=%d, East=%d, West=%d (Running on %s)\n"
                % (rank, nb["N"], nb["S"], nb["E"], nb["W"], host))

    def json_line(self, payload: dict) -> None:
        self._p(json.dumps(payload, sort_keys=True) + "\n")


def metrics(nx: int, ny: int, steps: int, elapsed_s: float, **extra) -> dict:
    cells = float(nx) * float(ny) * float(steps)
    cups = cells / elapsed_s if elapsed_s > 0 else float("nan")
    d = {
        "grid": [nx, ny],
        "steps": steps,
        "elapsed_s": elapsed_s,
        "cell_updates_per_s": cups,
        # a 1-read + 1-write per cell-step streaming roofline figure, comparable with the
        # report's CUDA numbers; temporal blocking moves fewer real bytes.
        "effective_gbps_8B_per_cell": cups * 8.0 / 1e9 if elapsed_s > 0 else float("nan"),
    }
    d.update(extra)
    return d
