"""Dump the state-DAG arrays of one history of a test batch (diagnostic; the
dag_debug_ptr / dag_debug_hist knobs).
    python tools/dag_debug.py n_ev n_pid model hist"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("quickcheck-state-machine-distributed_amd", "tests", "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import histgen  # noqa: E402
import oracle_c  # noqa: E402
from qsmd import codec, device, models  # noqa: E402


def main():
    n_ev, n_pid, model, hi = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4])
    rng = random.Random(n_ev * 1000 + n_pid)
    hs = {}
    for mname in ("ticket", "bank"):
        h = [histgen.wellformed_history(rng, mname, n_ev // 2, n_pid, p_pending=0.0)[:n_ev] for _ in range(300)]
        h += [histgen.random_history(rng, mname, n_ev, n_pid) for _ in range(300)]
        hs[mname] = h
    m = models.BY_NAME[model]
    b = codec.encode(m, hs[model])
    ctx = device.Context(0)
    ctx.set_param("heavy_mode", 0)
    buf = torch.zeros(1 << 16, dtype=torch.int32, device="cuda:0")
    ctx.set_param("dag_debug_ptr", buf.data_ptr())
    ctx.set_param("dag_debug_hist", hi)
    st, nd, _, _ = ctx.check_arrays(m.model_id, b.hdr, b.events, max_nodes=200000)
    st_o, nd_o, _ = oracle_c.check_batch(m.model_id, b.hdr, b.events, max_nodes=200000)
    q = buf.cpu().numpy().view(np.uint32)
    print("device", st[hi], nd[hi], "oracle", st_o[hi], nd_o[hi], "dbg", q[:4])
    SC, IC = int(q[2]), int(q[3])
    base = 16
    sitem, glo, ghi, gfl = (q[base + k * SC: base + (k + 1) * SC] for k in range(4))
    item = q[base + 4 * SC: base + 4 * SC + IC]
    for s_ in range(min(SC, 40)):
        off, deg = int(sitem[s_]) & 0xFFFF, int(sitem[s_]) >> 16
        its = [(int(x) & 0xFFF, (int(x) >> 12) & 3, (int(x) >> 14) & 127) for x in item[off:off + deg]]
        print(s_, "off", off, "deg", deg, "g", int(glo[s_]) | int(ghi[s_]) << 32, int(gfl[s_]), its)
    ctx.close()


if __name__ == "__main__":
    main()
