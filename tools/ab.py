"""A/B timing of two builds of libqsmd.so on the GPU box (diagnostic).

    python tools/ab.py libA.so libB.so [rounds] [bench args...]

Runs bench.py alternately with each library (QSMD_LIB_PATH), `rounds`
times, and prints the stage-0 and call device times and the value of every
run plus the medians per library.
"""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    libs = sys.argv[1:3]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    extra = sys.argv[4:] or ["--steps", "50", "--warmup", "5", "--inflight", "1"]
    res = {lib: [] for lib in libs}
    for r in range(rounds):
        for lib in (libs if r % 2 == 0 else libs[::-1]):
            env = dict(os.environ, QSMD_LIB_PATH=os.path.abspath(lib))
            out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-extra",
                                  *extra], env=env, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:], file=sys.stderr)
                sys.exit(out.returncode)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            al = d["device_ms"]["alone"]
            row = (d["value"] / 1e9, al["stage0_mean"], al["heavy_mean"] or 0.0, al["call_mean"])
            res[lib].append(row)
            print(f"round {r} {os.path.basename(lib)}: value {row[0]:.3f}e9 alone: stage0 {row[1]:.4f} ms "
                  f"heavy {row[2]:.4f} ms call {row[3]:.4f} ms", flush=True)
    for lib in libs:
        v = list(zip(*res[lib]))
        print(f"MEDIAN {os.path.basename(lib)}: value {statistics.median(v[0]):.3f}e9 alone: stage0 "
              f"{statistics.median(v[1]):.4f} ms heavy {statistics.median(v[2]):.4f} ms call "
              f"{statistics.median(v[3]):.4f} ms", flush=True)


if __name__ == "__main__":
    main()
