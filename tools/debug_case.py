"""Run one parity case outside pytest with stage-by-stage timing
(QSMD_SYNC_STAGES=1) and a short time limit (diagnostic)."""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("quickcheck-state-machine-distributed_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))

import numpy as np  # noqa: E402

import histgen  # noqa: E402
import oracle_c  # noqa: E402
from qsmd import codec, device, models  # noqa: E402


def main():
    n_ev, n_pid = int(sys.argv[1]), int(sys.argv[2])
    ctx = device.Context(0, time_limit_ms=int(os.environ.get("QSMD_TL", "10000")))
    rng = random.Random(n_ev * 1000 + n_pid)
    for model in ("ticket", "bank"):
        hs = [histgen.wellformed_history(rng, model, n_ev // 2, n_pid, p_pending=0.0)[:n_ev] for _ in range(300)]
        hs += [histgen.random_history(rng, model, n_ev, n_pid) for _ in range(300)]
        m = models.BY_NAME[model]
        b = codec.encode(m, hs)
        t = time.time()
        st, nd, _, tot = ctx.check_arrays(m.model_id, b.hdr, b.events, max_nodes=200000)
        print(model, "device", time.time() - t, tot, ctx.probe(), flush=True)
        st_o, nd_o, _ = oracle_c.check_batch(m.model_id, b.hdr, b.events, None, 200000, 8)
        bad = np.nonzero((st != st_o) | (nd != nd_o))[0]
        print(model, "mismatches", len(bad), bad[:5], st[bad[:5]], st_o[bad[:5]], nd[bad[:5]], nd_o[bad[:5]], flush=True)


if __name__ == "__main__":
    main()
