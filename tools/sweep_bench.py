"""Repeated bench runs over a list of argument sets (diagnostic): prints the
median value and device times per set.

    python tools/sweep_bench.py rounds "ARGS1" "ARGS2" ...
"""
import json
import os
import shlex
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    rounds = int(sys.argv[1])
    sets = sys.argv[2:]
    res = {s: [] for s in sets}
    for r in range(rounds):
        for s in (sets if r % 2 == 0 else sets[::-1]):
            out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-extra",
                                  *shlex.split(s)], capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:], file=sys.stderr)
                sys.exit(out.returncode)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            res[s].append((d["value"] / 1e9, d["device_ms"]["stage0_mean"], d["device_ms"]["call_mean"]))
            print(f"round {r} [{s}]: {res[s][-1]}", flush=True)
    for s in sets:
        v = list(zip(*res[s]))
        print(f"MEDIAN [{s}]: value {statistics.median(v[0]):.3f}e9 stage0 {statistics.median(v[1]):.4f} "
              f"call {statistics.median(v[2]):.4f}", flush=True)


if __name__ == "__main__":
    main()
