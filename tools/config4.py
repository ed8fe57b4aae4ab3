"""BASELINE config 4 timing (diagnostic): one adversarial TicketDispenser
8 x 64 history (gen.adversarial_ticket), QSMD_FLAG_MEMO, through the host
entry point, per qsmd_set_param setting; verdict against the oracle's memo
mode.
    python tools/config4.py [--reps 20] [--bug 0|1] "name=value,..." ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

import oracle_c  # noqa: E402
from qsmd import device, gen  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--bug", type=int, default=1)
    ap.add_argument("cases", nargs="*", default=[""])
    args = ap.parse_args()
    h, e, _ = gen.adversarial_ticket(8, 64, bug=bool(args.bug))
    st_o, nd_o, _ = oracle_c.check_batch(1, h, e, memo=True)
    t, k = time.perf_counter(), 0
    while time.perf_counter() - t < 1.0:                 # the CPU point: the oracle's memo mode, 1 thread
        oracle_c.check_batch(1, h, e, memo=True)
        k += 1
    print(json.dumps({"cpu_ms_per_history": round(1e3 * (time.perf_counter() - t) / k, 4), "calls": k}), flush=True)
    for case in args.cases:
        ctx = device.Context(0)
        for kv in filter(None, case.split(",")):
            k, v = kv.split("=")
            ctx.set_param(k, int(v))
        times = []
        ctx.timing_reset()
        for _ in range(args.reps):
            t = time.perf_counter()
            st, nd, _, _ = ctx.check_arrays(1, h, e, flags=device.QSMD_FLAG_EXHAUSTIVE | device.QSMD_FLAG_MEMO)
            times.append(time.perf_counter() - t)
        _, call_ms = ctx.timing_read()
        ctx.close()
        print(json.dumps({"case": case or "default", "bug": args.bug, "ms_median": round(1e3 * float(np.median(times[2:])), 3),
                          "device_ms_median": round(float(np.median(call_ms[2:])), 3),
                          "verdict": int(st[0]), "oracle": int(st_o[0]), "explored": int(nd[0]),
                          "oracle_explored": int(nd_o[0])}), flush=True)


if __name__ == "__main__":
    main()
