"""Adversarial TicketDispenser history (BASELINE config 4 shape) in
exhaustive mode through the split stage's exact-count memo."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"), os.path.join(ROOT, "oracle")]
import torch  # noqa: E402,F401

from qsmd import device, gen, models  # noqa: E402

ctx = device.Context(0, time_limit_ms=20000)
for nc, no in ((4, 17), (6, 30), (8, 40), (8, 64)):
    for bug in (False, True):
        h, e, _ = gen.adversarial_ticket(nc, no, bug=bug)
        t = time.time()
        st, nd, _, tot = ctx.check_arrays(models.MODEL_TICKET, h, e)
        print(json.dumps({"clients": nc, "ops": no, "bug": bug, "status": int(st[0]), "nodes": int(nd[0]),
                          "s": round(time.time() - t, 3), "timed_out": tot.get("timed_out")}), flush=True)
