"""Randomised parity sweep (test infrastructure): generated batches with
random generator parameters and random any-shape histories, through the
default cascade (adaptive probe, memo stage, witnesses), against the C
oracle.  Prints one JSON summary line; exits 1 on any mismatch.
    python tools/stress_parity.py [--batches 40] [--seed 1]"""

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

ap = argparse.ArgumentParser()
ap.add_argument("--batches", type=int, default=40)
ap.add_argument("--seed", type=int, default=1)
args = ap.parse_args()
rng = random.Random(args.seed)
ctx = device.Context(0, time_limit_ms=60000)
t0 = time.time()
stats = {"batches": 0, "histories": 0, "nodes": 0, "mismatch_status": 0, "mismatch_nodes": 0,
         "mismatch_witness": 0, "lin": 0, "nonlin": 0, "error": 0, "encode": 0}


def compare(model_id, hdr, ev, model0=None):
    st_d, nd_d, w_d, _ = ctx.check_arrays(model_id, hdr, ev, model0, max_nodes=200_000, witness=True)
    st_o, nd_o, w_o = oracle_c.check_batch(model_id, hdr, ev, model0, 200_000, 16, witness=True)
    stats["batches"] += 1
    stats["histories"] += len(hdr)
    stats["nodes"] += int(nd_o.sum())
    stats["mismatch_status"] += int((st_d != st_o).sum())
    stats["mismatch_nodes"] += int((nd_d != nd_o).sum())
    for i in np.nonzero(st_d == codec.STATUS_LIN)[0]:
        a, b = int(hdr[i]["ev_off"]), int(hdr[i]["ev_off"]) + int(hdr[i]["n_ev"])
        stats["mismatch_witness"] += int(not np.array_equal(w_d[a:b], w_o[a:b]))
    for k, s in (("lin", 1), ("nonlin", 0), ("error", 2), ("encode", 3)):
        stats[k] += int((st_o == s).sum())


for b in range(args.batches):
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
        hdr, ev, _ = gen.generate(gen.params(**kw), rng.randint(0, 10**6), 20000 if kw["n_ops"] <= 32 else 4000)
        compare(kw["model_id"], hdr, ev)
    else:                                        # any shape (ill-formed, shared pids, pending, errors)
        model = rng.choice(["ticket", "bank"])
        hs = []
        for _ in range(3000):
            if rng.random() < 0.5:
                hs.append(histgen.random_history(rng, model, rng.randint(0, 40), rng.randint(1, 8)))
            else:
                hs.append(histgen.wellformed_history(rng, model, rng.randint(1, 24), rng.randint(1, 8)))
        m = models.BY_NAME[model]
        bt = codec.encode(m, hs)
        compare(m.model_id, bt.hdr, bt.events)
    print(json.dumps({"batch": b, **{k: stats[k] for k in ("histories", "mismatch_status", "mismatch_nodes",
                                                           "mismatch_witness")},
                      "t": round(time.time() - t0, 1)}), file=sys.stderr, flush=True)
stats["seconds"] = round(time.time() - t0, 1)
print(json.dumps(stats), flush=True)
sys.exit(0 if stats["mismatch_status"] + stats["mismatch_nodes"] + stats["mismatch_witness"] == 0 else 1)
