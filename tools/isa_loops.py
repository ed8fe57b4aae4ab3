"""Instruction counts of the loops of one kernel (static ISA), to compare
builds of the DFS step:  python tools/isa_loops.py csrc/compact.hip compact_searchILj2ELb0ENS_12_GLOBAL__N_13G32
Prints each back-edge range with its VALU / SALU / LDS / v_mov counts."""

import re
import subprocess
import sys

src, sym = sys.argv[1], sys.argv[2]
min_len = int(sys.argv[3]) if len(sys.argv) > 3 else 150
asm = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I../include", "-Icsrc",
                      "-S", "--cuda-device-only", src, "-o", "-"], capture_output=True, text=True).stdout
lines = asm.split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l and l.endswith(":") is False or
             (l.startswith("_Z") and sym in l))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
L = lines[start:end]
lab = {}
for i, l in enumerate(L):
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        lab[m.group(1)] = i
seen = set()
for i, l in enumerate(L):
    m = re.search(r"(s_cbranch_\w+|s_branch)\s+(\.LBB\w+)", l)
    if m and m.group(2) in lab and lab[m.group(2)] < i:
        s = lab[m.group(2)]
        body = [x.strip() for x in L[s:i + 1] if x.startswith("\t") and not x.startswith("\t.") and not x.strip().startswith(";")]
        if len(body) < min_len or (s, i) in seen:
            continue
        seen.add((s, i))
        nv = sum(1 for x in body if x.startswith("v_"))
        nm = sum(1 for x in body if x.startswith("v_mov"))
        ns = sum(1 for x in body if x.startswith("s_"))
        nd = sum(1 for x in body if x.startswith("ds_"))
        print(f"{m.group(2):12s} [{s:5d},{i:5d}] instr {len(body):4d}  valu {nv:4d} (mov {nm:3d})  salu {ns:4d}  lds {nd:3d}")
