"""Loop census of a device assembly file (diagnostic): for one kernel of a
`hipcc --cuda-device-only -S` output, every backward branch's loop body with
its instruction mix (v_ / s_ / ds_ / global_ / waitcnt).

    python tools/asm_loops.py file.s <kernel-substring>
"""
import re
import sys
from collections import Counter


def main():
    path, pat = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and pat in l)
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith("s_endpgm"))
    body = lines[start:end + 1]
    labels = {}
    ins = []                                   # (index in body, text)
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB[\w_]+):", l)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        t = l.split(";")[0].strip()
        if t and not t.startswith(".") and not t.endswith(":"):
            ins.append(t)
    for k, t in enumerate(ins):
        m = re.match(r"s_(cbranch_\w+|branch)\s+(\.LBB[\w_]+)", t)
        if m and labels.get(m.group(2), 1 << 30) <= k:
            lo = labels[m.group(2)]
            seg = ins[lo:k + 1]
            c = Counter()
            for s in seg:
                op = s.split()[0]
                kind = ("waitcnt" if op.startswith("s_waitcnt") else op.split("_")[0])
                c[kind] += 1
            print(f"loop {m.group(2)} [{lo}..{k}] {len(seg)} insts: {dict(c)}")


if __name__ == "__main__":
    main()
