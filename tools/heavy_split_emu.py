"""Design study (CPU, no GPU): how long is the longest lane's DFS chain in the
heavy stage if each heavy history is cut at depth D into subtree tasks dealt
round-robin to S lanes (each lane with its own exact-count memo), against one
lane per history?  Emulates the heavy stage's per-lane DFS over the Lemma L1
event bitset for the paired Bank histories of a config, counting iterations
(tries + backtracks) per lane.
    python tools/heavy_split_emu.py [config] [n_hist] [budget]
"""
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import oracle_c  # noqa: E402
from qsmd import gen  # noqa: E402

OPEN, DEP, WD, CHK, TR = range(5)
CREATED, DEPMADE, WDMADE, TRMADE, EXISTS, NOEX, INSUF, BAL = range(8)


def post_next(m, inv, resp):
    """Bank post on the pre-state and next'; returns (ok, err, model')."""
    ex, bal = m
    if any(v < 0 for v in bal.values()):
        return False, False, None
    code, a, b, v = inv
    rc, rv = resp
    if code == OPEN:
        ok = rc == (EXISTS if a in bal else CREATED)
    elif code == DEP:
        ok = rc == DEPMADE
    elif code == WD:
        ok = rc == (WDMADE if a in bal and bal[a] >= v else INSUF)
    elif code == CHK:
        if rc != BAL:
            ok = False
        elif a not in bal:
            return False, True, None
        else:
            ok = rv == bal[a]
    else:
        ok = rc == (TRMADE if a in bal and bal[a] >= v else INSUF)
    if not ok:
        return False, False, None
    nb = dict(bal)
    if code == OPEN:
        nb.setdefault(a, 0)
    elif code == DEP:
        nb[a] = nb.get(a, 0) + v if a in nb else v
    elif code == WD:
        nb[a] = nb[a] - v if a in nb else v
    elif code == TR:
        nb[a] = nb[a] - v if a in nb else v
        nb[b] = nb[b] + v if b in nb else v
    return True, False, (None, nb)


class Lane:
    def __init__(self):
        self.memo = {}
        self.iters = 0


def search(hist, D, S):
    """hist: list of events (resp, pid, code, a, b, val); returns per-lane iterations
    and the total node count (checked against the oracle)."""
    n = len(hist)
    pair = {}
    openi = {}
    for i, (r, p, *_rest) in enumerate(hist):
        if not r:
            openi[p] = i
        else:
            pair[openi.pop(p)] = i
    INV = [i for i in range(n) if not hist[i][0]]

    def cands(rem):
        out = []
        for i in range(n):
            if not (rem >> i) & 1:
                continue
            if hist[i][0]:
                break
            out.append(i)
        return out

    lanes = [Lane() for _ in range(S)]
    task = [0]

    def key(rem, m):
        return rem, tuple(sorted(m[1].items()))

    # returns (result, nodes): result True / False / 'err'
    def sub(lane, rem, m, depth, is_root):
        cs = cands(rem)
        if not cs:
            return (False if is_root else True), 0
        nodes = 0
        for j in cs:
            lane.iters += 1
            if j not in pair:
                continue
            r = pair[j]
            nodes += 1
            _, p, code, a, b, v = hist[j]
            ok, err, m2 = post_next(m, (code, a, b, v), (hist[r][2], hist[r][5]))
            if err:
                return "err", nodes
            if not ok:
                continue
            rem2 = rem & ~((1 << j) | (1 << r))
            k = key(rem2, m2)
            if k in lane.memo:
                nodes += lane.memo[k]
                continue
            res, c = sub(lane, rem2, m2, depth + 1, False)
            nodes += c
            lane.iters += 1          # the backtrack
            if res is True or res == "err":
                return res, nodes
            lane.memo[k] = c
        return False, nodes

    # top: DFS to depth D, tasks round-robin; every lane walks the top
    results = {}

    def top(rem, m, depth, is_root, lanes_all):
        cs = cands(rem)
        if not cs:
            return (False if is_root else True), 0
        nodes = 0
        for j in cs:
            for ln in lanes_all:
                ln.iters += 1
            if j not in pair:
                continue
            r = pair[j]
            nodes += 1
            _, p, code, a, b, v = hist[j]
            ok, err, m2 = post_next(m, (code, a, b, v), (hist[r][2], hist[r][5]))
            if err:
                return "err", nodes
            if not ok:
                continue
            rem2 = rem & ~((1 << j) | (1 << r))
            if depth + 1 == D:
                t = task[0]
                task[0] += 1
                ln = lanes_all[t % S]
                res, c = sub(ln, rem2, m2, depth + 1, False)
                results[t] = (res, c)
            else:
                res, c = top(rem2, m2, depth + 1, False, lanes_all)
            nodes += c
            if res is True or res == "err":
                return res, nodes
        return False, nodes

    m0 = (None, {})
    full = (1 << n) - 1
    if D == 0:
        res, nodes = sub(lanes[0], full, m0, 0, True)
    else:
        res, nodes = top(full, m0, 0, True, lanes)
    return [ln.iters for ln in lanes], nodes, res


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "bank_4x16"
    nh = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
    budget = int(sys.argv[3]) if len(sys.argv) > 3 else 26
    h, e, _ = gen.generate_config(cfg, 0, nh)
    st, nd, _ = oracle_c.check_batch(int(h[0]["model_id"]), h, e, threads=8)
    heavy = np.nonzero(nd > budget)[0]
    print(f"{cfg}: {len(heavy)} of {nh} over {budget} nodes, max {nd.max()}")
    for D, S in [(0, 1), (1, 4), (2, 16), (2, 8), (3, 16), (3, 64)]:
        worst = []
        for i in heavy:
            off, ne = int(h[i]["ev_off"]), int(h[i]["n_ev"])
            ev = e[off:off + ne]
            hist = [(int(x["kp"]) >> 7, int(x["kp"]) & 0x7F, int(x["code"]), int(x["a"]), int(x["b"]), int(x["val"]))
                    for x in ev]
            its, nodes, res = search(hist, D, S)
            if D == 0:
                assert nodes == nd[i], (i, nodes, nd[i])
            worst.append(max(its))
        w = np.array(worst)
        print(f"D={D} S={S}: longest lane iterations max {w.max()}  p99 {np.percentile(w, 99):.0f}  "
              f"mean {w.mean():.1f}", flush=True)


if __name__ == "__main__":
    main()
