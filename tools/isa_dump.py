"""Dump one loop (by its header label) of one kernel:  python tools/isa_dump.py SRC SYM LABEL"""
import re
import subprocess
import sys

src, sym, label = sys.argv[1:4]
asm = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I../include", "-Icsrc",
                      "-S", "--cuda-device-only", src, "-o", "-"], capture_output=True, text=True).stdout
L = asm.split("\n")
st = next(i for i, l in enumerate(L) if l.startswith("_Z") and sym in l)
L = L[st:]
s = next(i for i, l in enumerate(L) if l.startswith(label + ":"))
e = max(i for i in range(s, min(len(L), s + 3000)) if "s_cbranch" in L[i] and label in L[i] or "s_branch" in L[i] and label in L[i])
for l in L[s:e + 1]:
    t = l.strip()
    if t and not t.startswith(";") and not t.startswith(".loc") and not t.startswith(".Ltmp"):
        print(l.split(";")[0].rstrip())
