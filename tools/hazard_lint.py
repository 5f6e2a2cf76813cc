"""Store-data hazard lint of the built device code (gfx950).

A VMEM/FLAT store of more than 64 bits reads its data VGPRs after it issues: an instruction that
writes one of those VGPRs within 2 wait states of the store can change what the store writes
(the MI355X guide: an asm `..._store_dwordx3/x4` ends with `s_nop 1`).  ROCm 7.2's hipcc did not
pad such a write when it was a packed-FP32 VALU op (`v_pk_add_f32` right after a
`buffer_store_dwordx4`): lanes of the stored row came out wrong under memory load, intermittently.

This lint disassembles every device code object of the build (build/obj/*.o, .hip_fatbin) and
reports each wide store followed, within 2 wait states, by a VALU instruction that writes one of
its data VGPRs.  Usage: python tools/hazard_lint.py [objects...]  (exit 1 on a finding).
"""
from __future__ import annotations

import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
WIDE = re.compile(r"^(buffer|global|flat|scratch)_store_(dwordx3|dwordx4|b96|b128)\b")


def vregs(tok: str) -> set:
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def disassemble(obj: str) -> list:
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb"), os.path.join(d, "co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(d, "x")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--targets={TARGET}", f"--input={fb}",
                        f"--output={co}", "--unbundle"], check=True, capture_output=True)
        out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True, capture_output=True,
                             text=True).stdout
    ins = []
    for line in out.splitlines():
        line = line.split("//")[0].strip()
        if not line or line.endswith(":") or line.startswith(("Disassembly", ".")):
            continue
        ins.append(line)
    return ins


def findings(ins: list) -> list:
    bad = []
    for i, l in enumerate(ins):
        p = l.replace(",", " ").split()
        if not WIDE.match(p[0]):
            continue
        data = vregs(p[1] if p[0].startswith("buffer") else p[2])
        ws = 0
        for j in range(i + 1, min(len(ins), i + 8)):
            q = ins[j].replace(",", " ").split()
            if q[0] == "s_endpgm":
                break  # the wave ends here: what follows in the listing is another block
            if q[0] == "s_nop":
                ws += int(q[1], 0) + 1
            else:
                # VALU writers only: a vector-memory load issues behind the store in the same memory
                # pipeline and returns its data hundreds of cycles later
                if len(q) > 1 and q[0].startswith("v_") and vregs(q[1]) & data:
                    bad.append((ws, l, ins[j]))
                    break
                ws += 1
            if ws >= 2:
                break
    return bad


def main(argv: list) -> int:
    objs = argv or sorted(glob.glob(os.path.join(ROOT, "build", "obj", "*.o")))
    total = stores = dev = 0
    for o in objs:
        try:
            ins = disassemble(o)
        except subprocess.CalledProcessError:
            continue  # host-only object
        dev += 1
        stores += sum(1 for l in ins if WIDE.match(l.split()[0]))
        f = findings(ins)
        total += len(f)
        for ws, st, w in f[:3]:
            print(f"{os.path.basename(o)}: {ws} wait state(s): {st}  ->  {w}")
        if len(f) > 3:
            print(f"{os.path.basename(o)}: ... {len(f)} findings")
    print(f"hazard_lint: {total} finding(s); {stores} wide stores in {dev} device code object(s)")
    return 1 if total or dev == 0 else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
