"""Device report (``--debug``), the equivalent of ``detailsGPU`` (``grad1612_cuda_heat.cu:24-37``)."""
from __future__ import annotations

from .._native import native


def device_report() -> str:
    n = native()
    lines = []
    kb, mb = 1024, 1024 * 1024
    for i in range(n.device_count()):
        p = n.device_props(i)
        lines.append("%s (%s):   %d.%d" % (p["name"], p["gcn_arch"], p["major"], p["minor"]))
        lines.append("Global memory:   %d mb" % (p["total_global_mem"] // mb))
        lines.append("Shared memory:   %d kb" % (p["shared_mem_per_block"] // kb))
        lines.append("Constant memory: %d kb" % (p["total_const_mem"] // kb))
        lines.append("Block registers: %d" % p["regs_per_block"])
        lines.append("Warp size:         %d" % p["warp_size"])
        lines.append("Threads per block: %d" % p["max_threads_per_block"])
        lines.append("Compute units:     %d" % p["multiprocessor_count"])
        lines.append("Max block dimensions: [%d, %d, %d]" % tuple(p["max_threads_dim"]))
        lines.append("Max grid dimensions: [%d, %d, %d]" % tuple(p["max_grid_size"]))
        lines.append("")
    return "\n".join(lines) + ("\n" if lines else "")
