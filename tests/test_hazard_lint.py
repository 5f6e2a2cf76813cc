"""The store-data hazard lint (tools/hazard_lint.py) as a CPU test.

A VMEM store wider than 64 bits reads its data VGPRs after it issues; a VALU write of those
registers within 2 wait states can change what it stores, and ROCm 7.2's hipcc does not always pad
it (docs/ARCHITECTURE.md, "Store-data hazard lint").  The stencil kernels avoid the pattern by
construction (soffset-0 write-through stores, `s_nop 1` guards, stream_kernel.hpp); this test
disassembles every built code object so that a kernel edit that brings the pattern back fails the
CPU suite, and checks on a deliberately unguarded store that the lint does catch it.
"""
import concurrent.futures
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LLVM = "/opt/rocm/lib/llvm/bin"
HIPCC = "/opt/rocm/bin/hipcc"

pytestmark = pytest.mark.skipif(not (os.path.exists(f"{LLVM}/llvm-objcopy") and os.path.exists(HIPCC)),
                                reason="ROCm LLVM tools absent")


def test_built_code_objects_have_no_store_data_hazard():
    import hazard_lint

    objs = sorted(glob.glob(os.path.join(ROOT, "build", "obj", "*.o")))
    if not objs:
        pytest.skip("native runtime not built (python -m heat2d_amd._build)")
    def dis(o):
        try:
            return o, hazard_lint.disassemble(o)
        except subprocess.CalledProcessError:
            return o, None  # host-only object

    dev = stores = 0
    bad = []
    with concurrent.futures.ThreadPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        listings = list(ex.map(dis, objs))
    for o, ins in listings:
        if ins is None:
            continue
        dev += 1
        stores += sum(1 for line in ins if hazard_lint.WIDE.match(line.split()[0]))
        bad += [(os.path.basename(o), st, w) for _, st, w in hazard_lint.findings(ins)]
    assert dev >= 40 and stores > 1000, (dev, stores)  # every stencil variant was disassembled
    assert not bad, f"{len(bad)} wide store(s) followed by a VALU write of their data: {bad[:5]}"


def test_lint_catches_an_unguarded_wide_store(tmp_path):
    import hazard_lint

    src = tmp_path / "bad.hip"
    # one asm block, so the compiler cannot pad between the store and the write of its data
    src.write_text(
        "#include <hip/hip_runtime.h>\n"
        "__global__ void bad_store() {\n"
        "  asm volatile(\"v_mov_b32 v10, 0\\n\\tv_mov_b32 v11, 0\\n\\t\"\n"
        "               \"global_store_dwordx4 v[10:11], v[12:15], off\\n\\tv_mov_b32 v13, 1\"\n"
        "               ::: \"v10\", \"v11\", \"v12\", \"v13\", \"v14\", \"v15\", \"memory\");\n"
        "}\n")
    obj = tmp_path / "bad.o"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O2", "-c", str(src), "-o", str(obj)], check=True,
                   capture_output=True)
    f = hazard_lint.findings(hazard_lint.disassemble(str(obj)))
    assert len(f) == 1 and "global_store_dwordx4" in f[0][1] and "v13" in f[0][2], f
    # and the guarded form (the s_nop the kernels use) passes
    src.write_text(src.read_text().replace("off\\n\\tv_mov_b32 v13", "off\\n\\ts_nop 1\\n\\tv_mov_b32 v13"))
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O2", "-c", str(src), "-o", str(obj)], check=True,
                   capture_output=True)
    assert "s_nop 1" in src.read_text()
    assert hazard_lint.findings(hazard_lint.disassemble(str(obj))) == []


def test_stencil_kernels_use_global_memory_instructions():
    """The stencil kernels read their pointers from device-resident argument blocks, which the
    compiler sees as generic (flat) pointers; `gp()` (stream_kernel.hpp) marks them global.  A flat
    access would complete out of order with the buffer loads/stores (the persistent kernel's
    counted `s_waitcnt vmcnt(N)` relies on in-order completion), add lgkmcnt waits, and turn each
    write-through row store's buffer resource into a readfirstlane waterfall — measured +4 % VALU
    instructions in the K=7 steady loop when it happened (round 5)."""
    import hazard_lint

    objs = sorted(glob.glob(os.path.join(ROOT, "build", "obj", "stream_k*.o")) +
                  glob.glob(os.path.join(ROOT, "build", "obj", "pstream_k*.o")) +
                  glob.glob(os.path.join(ROOT, "build", "obj", "tile_kernel.o")))
    if not objs:
        pytest.skip("native runtime not built (python -m heat2d_amd._build)")

    def flat_ops(o):
        return o, sum(1 for line in hazard_lint.disassemble(o) if line.split()[0].startswith("flat_"))

    with concurrent.futures.ThreadPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        bad = [(os.path.basename(o), n) for o, n in ex.map(flat_ops, objs) if n]
    assert not bad, f"flat memory instructions in stencil kernels: {bad}"
