"""In-tree build of the native runtime (``heat2d_amd/_heat2d*.so``) and the ``heat2d`` CLI.

Every translation unit is compiled by ``hipcc --offload-arch=gfx950`` with
``-ffp-contract=off`` (the bit-exact numerics contract).  The streaming
stencil is instantiated once per temporal-block depth K in its own translation unit so the
objects compile in parallel.  Objects are rebuilt only when the source or a header it includes is newer.

Usage: ``python -m heat2d_amd._build [--force] [--jobs N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import re
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(os.path.dirname(ROOT), "build", "obj")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("HEAT2D_ARCH", "gfx950")

EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
EXT_PATH = os.path.join(ROOT, "_heat2d" + EXT_SUFFIX)
CLI_PATH = os.path.join(ROOT, "bin", "heat2d")

# Sources of the Python extension (bindings + runtime) and of the CLI (runtime + main).
RUNTIME_SOURCES = [
    "decomposition.cpp",
    "cpu_reference.cpp",
    "io.cpp",
    "engine.cpp",
    "kernels.hip",
    "tile_kernel.hip",
] + [f"stream_k{k}.hip" for k in (1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 16)]
EXT_SOURCES = RUNTIME_SOURCES + ["bindings.cpp"]
CLI_SOURCES = RUNTIME_SOURCES + ["heat2d_main.cpp"]

COMMON_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-ffp-contract=off",
    "-Wall",
    "-Wno-unused-result",
    "-Wno-unused-function",
]


def _hipcc() -> str:
    p = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    if not os.path.exists(p):
        raise RuntimeError("hipcc not found; the native runtime needs ROCm")
    return p


def _py_includes() -> list[str]:
    import pybind11

    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


_INCLUDE_RE = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _deps_mtime(src: str, seen: set | None = None) -> float:
    """Newest mtime over `src` and the in-tree headers it includes, transitively."""
    seen = set() if seen is None else seen
    path = os.path.join(CSRC, src)
    if src in seen or not os.path.exists(path):
        return 0.0
    seen.add(src)
    m = os.path.getmtime(path)
    with open(path, encoding="utf-8", errors="replace") as f:
        for inc in _INCLUDE_RE.findall(f.read()):
            m = max(m, _deps_mtime(inc, seen))
    return m


def _obj_for(src: str) -> str:
    return os.path.join(BUILD, os.path.splitext(src)[0] + ".o")


def _compile(src: str, force: bool) -> tuple[str, bool]:
    path = os.path.join(CSRC, src)
    obj = _obj_for(src)
    if not force and os.path.exists(obj):
        if os.path.getmtime(obj) >= _deps_mtime(src):
            return obj, False
    cmd = [_hipcc(), *COMMON_FLAGS, f"-I{CSRC}"]
    if src == "bindings.cpp":
        cmd += _py_includes()
    cmd += ["-c", path, "-o", obj + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(obj + ".tmp", obj)
    return obj, True


def _link(objs: list[str], out: str, shared: bool) -> None:
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-fPIC"]
    if shared:
        cmd.append("-shared")
    cmd += objs + ["-o", out + ".tmp", f"-L{ROCM}/lib", "-lrccl", "-lamdhip64", f"-Wl,-rpath,{ROCM}/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(out + ".tmp", out)


def build(force: bool = False, jobs: int | None = None, cli: bool = True, verbose: bool = False) -> str:
    """Compile (incrementally) and link the extension and the CLI.  Returns the extension path."""
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(os.path.dirname(CLI_PATH), exist_ok=True)
    srcs = sorted(set(EXT_SOURCES + (CLI_SOURCES if cli else [])))
    srcs = [s for s in srcs if os.path.exists(os.path.join(CSRC, s))]
    jobs = jobs or max(1, min(8, os.cpu_count() or 1))
    rebuilt = []
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = {ex.submit(_compile, s, force): s for s in srcs}
        for f in cf.as_completed(futs):
            obj, did = f.result()
            if did:
                rebuilt.append(futs[f])
    if verbose and rebuilt:
        print("compiled:", ", ".join(sorted(rebuilt)), file=sys.stderr)
    ext_objs = [_obj_for(s) for s in EXT_SOURCES]
    if rebuilt or not os.path.exists(EXT_PATH) or any(os.path.getmtime(o) > os.path.getmtime(EXT_PATH) for o in ext_objs):
        _link(ext_objs, EXT_PATH, shared=True)
    if cli and os.path.exists(os.path.join(CSRC, "heat2d_main.cpp")):
        cli_objs = [_obj_for(s) for s in CLI_SOURCES]
        if not os.path.exists(CLI_PATH) or any(os.path.getmtime(o) > os.path.getmtime(CLI_PATH) for o in cli_objs):
            _link(cli_objs, CLI_PATH, shared=False)
    return EXT_PATH


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--no-cli", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force, jobs=a.jobs, cli=not a.no_cli, verbose=True))


if __name__ == "__main__":
    main()
