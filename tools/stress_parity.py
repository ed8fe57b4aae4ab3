"""Randomised parity sweep (test infrastructure): generated batches with
random generator parameters and random any-shape histories, through the
cascade with witnesses and, per batch, random stage budgets and heavy-stage
mode (--knobs; the default cascade otherwise), against the C oracle.
Prints one JSON summary line; exits 1 on any mismatch.
    python tools/stress_parity.py [--batches 40] [--seed 1] [--knobs] [--wide]"""

import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (our library shares torch's HIP runtime)

import histgen  # noqa: E402
import oracle_c  # noqa: E402
from qsmd import codec, device, gen, models  # noqa: E402

KNOBS = {"stage0_budget": [0, 4, 16, 32, 40, 64], "stage0w_budget": [0, 4, 32], "stage0w_budget_auto": [0, 1],
         "heavy_mode": [0, 1, 2],
         "split_budget": [1, 16, 64, 1024], "memo_lane_entries": [2, 256], "wave_grid": [0, 5],
         "wave_min_rem": [0, 4, 64], "split_xmemo": [0, 1], "memo_lds": [0, 1, 2], "dag_states": [0, 6, 128, 1024],
         "stage0_budget_auto": [0, 1], "memo_after": [1, 32, 100], "timing_events": [0, 1],
         "fold": [0, 1], "resume_cap": [0, 1, 7, 64],
         "tail_cap": [0, 3, 40, 256], "tail_min": [0, 65536], "heavy_buckets": [0, 1],
         "early": [0, 0, 0, 1]}   # (early: QSMD_FLAG_EARLY_EXIT_BATCH for the batch, not a context knob)
DEFAULT_KNOBS = {"stage0_budget": 32, "stage0w_budget": 32, "stage0w_budget_auto": 1, "heavy_mode": 2,
                 "split_budget": 1024,
                 "memo_lane_entries": 128, "wave_grid": 0, "wave_min_rem": 4, "split_xmemo": 1,
                 "memo_lds": 1, "dag_states": 128, "stage0_budget_auto": 1, "memo_after": 32, "timing_events": 0,
                 "fold": 1, "resume_cap": 0, "tail_cap": 256, "tail_min": 65536, "heavy_buckets": 1}


def run(ctx, batches=40, seed=1, knobs=False, wide=False, only=-1, dump=None, log=None):
    """The sweep on context ctx; returns the stats dict (knobs restored)."""
    rng = random.Random(seed)
    stats = {"batches": 0, "histories": 0, "nodes": 0, "mismatch_status": 0, "mismatch_nodes": 0,
             "mismatch_witness": 0, "lin": 0, "nonlin": 0, "error": 0, "encode": 0, "timed_out_batches": 0}
    t0 = time.time()

    def compare(model_id, hdr, ev, batch, kn):
        early = bool(kn.get("early"))
        flags = device.QSMD_FLAG_EXHAUSTIVE | (device.QSMD_FLAG_EARLY_EXIT_BATCH if early else 0)
        st_d, nd_d, w_d, _ = ctx.check_arrays(model_id, hdr, ev, None, max_nodes=200_000, witness=True, flags=flags)
        st_o, nd_o, w_o = oracle_c.check_batch(model_id, hdr, ev, None, 200_000, 16, witness=True)
        if early:                                    # everything after the first failure: SKIPPED, 0 nodes
            fails = np.nonzero((st_o == 0) | (st_o == 2))[0]
            if len(fails):
                st_o, nd_o = st_o.copy(), nd_o.copy()
                st_o[fails[0] + 1:] = codec.STATUS_SKIPPED
                nd_o[fails[0] + 1:] = 0
        # the safety net fired: its BUDGET results are not the reference's, but
        # every other result of the batch still must be (recorded and compared)
        cmp = np.ones(len(hdr), dtype=bool)
        if ctx.timed_out():
            stats["timed_out_batches"] += 1
            cmp = st_d != codec.STATUS_BUDGET
            if log:
                log(json.dumps({"batch": batch, "knobs": kn, "timed_out": True,
                                "budget": int((~cmp).sum())}))
        bad = np.nonzero(cmp & ((st_d != st_o) | (nd_d != nd_o)))[0]
        if len(bad) and dump:
            os.makedirs(os.path.dirname(dump) or ".", exist_ok=True)
            np.savez(f"{dump}_{batch}.npz", hdr=hdr, ev=ev, bad=bad, model_id=model_id, knobs=json.dumps(kn),
                     st_d=st_d[bad], nd_d=nd_d[bad], st_o=st_o[bad], nd_o=nd_o[bad])
        if len(bad) and log:
            log(json.dumps({"batch": batch, "knobs": kn, "bad": bad[:8].tolist(),
                            "dev": [st_d[bad[:8]].tolist(), nd_d[bad[:8]].tolist()],
                            "oracle": [st_o[bad[:8]].tolist(), nd_o[bad[:8]].tolist()]}))
        stats["batches"] += 1
        stats["histories"] += len(hdr)
        stats["nodes"] += int(nd_o.sum())
        stats["mismatch_status"] += int((cmp & (st_d != st_o)).sum())
        stats["mismatch_nodes"] += int((cmp & (nd_d != nd_o)).sum())
        for i in np.nonzero(st_d == codec.STATUS_LIN)[0]:
            a, b = int(hdr[i]["ev_off"]), int(hdr[i]["ev_off"]) + int(hdr[i]["n_ev"])
            stats["mismatch_witness"] += int(not np.array_equal(w_d[a:b], w_o[a:b]))
        for k, s_ in (("lin", 1), ("nonlin", 0), ("error", 2), ("encode", 3)):
            stats[k] += int((st_o == s_).sum())

    try:
        for b in range(batches):
            kn = {}
            if knobs:
                for k, vals in KNOBS.items():
                    kn[k] = rng.choice(vals)
                    if k != "early":
                        ctx.set_param(k, kn[k])
            check = only < 0 or only == b
            if b % 2 == 0:                               # generator with random parameters
                name = rng.choice(list(gen.CONFIGS))
                kw = dict(gen.CONFIGS[name])
                ticket = kw["model_id"] == models.MODEL_TICKET
                kw["n_clients"] = rng.randint(1, 8)
                kw["n_ops"] = rng.randint(max(kw["n_clients"], 2), 32 if rng.random() < 0.7 else 64)
                kw["prefix_ops"] = rng.randint(0 if ticket else kw["n_clients"], kw["n_ops"])
                kw["overlap"] = rng.randint(0, kw["n_clients"])
                kw["p_bug"] = rng.choice([0.0, 0.2, 0.6, 1.0])
                kw["lin_policy"] = rng.randint(0, 1)
                kw["money_max"] = rng.choice([3, 10, 100])
                kw["seed"] = rng.getrandbits(48)
                first = rng.randint(0, 10**6)
                if check:
                    hdr, ev, _ = gen.generate(gen.params(**kw), first, 20000 if kw["n_ops"] <= 32 else 4000)
                    compare(kw["model_id"], hdr, ev, b, kn)
            else:                                        # any shape (ill-formed, shared pids, pending, errors)
                model = rng.choice(["ticket", "bank"])
                hs = []
                w = wide and rng.random() < 0.3          # beyond the compact stages: the giant stage
                for _ in range(1000 if w else 3000):
                    if rng.random() < 0.5:
                        hs.append(histgen.random_history(rng, model, rng.randint(0, 100 if w else 40),
                                                         rng.randint(1, 12 if w else 8)))
                    else:
                        hs.append(histgen.wellformed_history(rng, model, rng.randint(1, 50 if w else 24),
                                                             rng.randint(1, 12 if w else 8)))
                m = models.BY_NAME[model]
                if check:
                    bt = codec.encode(m, hs)
                    compare(m.model_id, bt.hdr, bt.events, b, kn)
            if check and log:
                log(json.dumps({"batch": b, **{k: stats[k] for k in ("histories", "mismatch_status",
                                                                     "mismatch_nodes", "mismatch_witness")},
                                "t": round(time.time() - t0, 1)}))
    finally:
        if knobs:
            for k, v in DEFAULT_KNOBS.items():
                if k != "early":
                    ctx.set_param(k, v)
    stats["seconds"] = round(time.time() - t0, 1)
    return stats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=40)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--knobs", action="store_true", help="random stage budgets / heavy mode per batch")
    ap.add_argument("--wide", action="store_true", help="also any-shape histories up to 100 events / 12 pids")
    ap.add_argument("--only", type=int, default=-1, help="check only this batch (the others only draw their randoms)")
    ap.add_argument("--dump", default="gpurun_out/stress_mismatch", help="mismatching batches: <dump>_<batch>.npz")
    args = ap.parse_args()
    ctx = device.Context(0, time_limit_ms=60000)
    stats = run(ctx, args.batches, args.seed, args.knobs, args.wide, args.only, args.dump,
                log=lambda line: print(line, file=sys.stderr, flush=True))
    ctx.close()
    print(json.dumps(stats), flush=True)
    sys.exit(0 if stats["mismatch_status"] + stats["mismatch_nodes"] + stats["mismatch_witness"] == 0 else 1)


if __name__ == "__main__":
    main()
