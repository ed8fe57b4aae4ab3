"""CPU emulation of the lane-mode heavy stage's work per history (csrc/memo.hip
memo_step over LaneDFS, lane.h): for the histories stage 0 stops at its node
budget, the DFS iterations the heavy stage runs after resuming stage 0's saved
state, with the exact-count memo joining after `memo_after` nodes in a
direct-mapped table of `entries` slots (the kernel's hash) or a perfect one.

One iteration = LaneDFS's step: an optional backtrack, then one candidate
try.  The reference semantics are oracle/ref_cpu.c's (bank_post / bank_next,
src/Linearisability.hs:25-69); verdict and node count are checked against the
C oracle for every emulated history.

    python tools/heavy_emu.py [n_hist] [budget] [memo_after] [entries|0=perfect]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quickcheck-state-machine-distributed_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from qsmd import gen  # noqa: E402

OPEN, DEPOSIT, WITHDRAW, CHECK, TRANSFER = range(5)
# response codes (include/qsmd.h)
CREATED, DEPOSIT_MADE, WITHDRAWAL_MADE, TRANSFER_MADE, EXISTS, INSUFFICIENT, BALANCE = 0, 1, 2, 3, 4, 6, 7
NOENTRY = None
M32 = 0xFFFFFFFF


def bank_post(ex, bal, inv, resp):
    """test/Bank.hs:118-131 (ref_cpu.c bank_post): 1 True, 0 False, 2 error."""
    code, a, _, m = inv
    rc, rv = resp
    if any(((ex >> q) & 1) and bal[q] < 0 for q in range(8)):
        return 0
    exa = (ex >> a) & 1
    if code == OPEN:
        return int(rc == (EXISTS if exa else CREATED))
    if code == DEPOSIT:
        return int(rc == DEPOSIT_MADE)
    if code == WITHDRAW:
        return int(rc == (WITHDRAWAL_MADE if exa and bal[a] >= m else INSUFFICIENT))
    if code == CHECK:
        if rc != BALANCE:
            return 0
        if not exa:
            return 2
        return int(rv == bal[a])
    return int(rc == (TRANSFER_MADE if exa and bal[a] >= m else INSUFFICIENT))


def bank_next(ex, bal, inv):
    code, a, b, m = inv
    bal = list(bal)
    if code == OPEN:
        if not (ex >> a) & 1:
            bal[a] = 0
        ex |= 1 << a
    elif code in (DEPOSIT, WITHDRAW, TRANSFER):
        s = 1 if code == DEPOSIT else -1
        bal[a] = bal[a] + s * m if (ex >> a) & 1 else m
        ex |= 1 << a
        if code == TRANSFER:
            bal[b] = bal[b] + m if (ex >> b) & 1 else m
            ex |= 1 << b
    return ex, tuple(bal)


def rotr(x, k):
    return ((x >> k) | (x << (32 - k))) & M32


def slot_of(rem, ex, bal, mask):
    """memo.hip memo_key: the slot hash (the top bits of one multiplicative
    hash), or None when a balance is beyond i16."""
    if any(not (-32768 <= v <= 32767) for v in bal):
        return None
    m = [((bal[2 * q] & 0xFFFF) | ((bal[2 * q + 1] & 0xFFFF) << 16)) & M32 for q in range(4)]
    v = m[0] ^ ex ^ rotr(m[1], 8) ^ rotr(m[2], 16) ^ rotr(m[3], 24)
    t = (rem & M32) ^ rotr(v, 13)
    return ((t * 0x9E3779B1) & M32) >> (32 - (mask + 1).bit_length() + 1)


class Hist:
    def __init__(self, evs):
        self.n = len(evs)
        self.pid = [e["kp"] & 0x7F for e in evs]
        self.resp = [(e["kp"] >> 7) & 1 for e in evs]
        self.code = [int(e["code"]) for e in evs]
        self.a = [int(e["a"]) for e in evs]
        self.b = [int(e["b"]) for e in evs]
        self.val = [int(e["val"]) for e in evs]
        self.INV = sum(1 << i for i in range(self.n) if not self.resp[i])
        self.RESP = sum(1 << i for i in range(self.n) if self.resp[i])
        self.PM = {}
        for i in range(self.n):
            self.PM[self.pid[i]] = self.PM.get(self.pid[i], 0) | (1 << i)


def cands(rem, h):
    rr = rem & h.RESP
    low = (rr & -rr) - 1 if rr else -1
    return rem & h.INV & low


def lowbit(x):
    return (x & -x).bit_length() - 1


def run(h, budget, memo_after, entries, policy="backtrack", alias=64, record_early=False):
    """Returns (status, nodes, iterations after the resume, stage-0 iterations, descents, hits)."""
    ALL = h.INV | h.RESP
    rem, ex, bal = ALL, 0, (0,) * 8
    stack = []              # (rem, ex, bal, j) of the parent per level
    entry = []              # node count at entry per level (None: entered in stage 0)
    cand = cands(rem, h)
    found, nodes, depth = 0, 0, 0
    table = {}
    mask = entries - 1 if entries else 0
    own = set()             # policy 'entry': alias classes of the path's pending slots
    pslot = []              # policy 'entry': the level's pending slot (None: none)
    limit = budget
    phase0 = True
    it0 = it1 = desc = hits = 0
    skip = False
    info = {}
    run.info = info
    while True:
        if phase0:
            it0 += 1
        else:
            it1 += 1
        memo = (not phase0) and nodes >= memo_after
        empty = cand == 0
        term = empty and (found == 0 or depth == 0)
        if term:
            return (1 if (not found and depth > 0) else 0), nodes, it1, it0, desc, hits
        if empty:
            ps = pslot.pop()
            if ps is not None:                  # policy 'entry': the pending entry gets its count
                own.discard(ps % alias)
                table[ps] = (table[ps][0], nodes - entry[depth - 1])
            if policy == "backtrack" and (memo or (record_early and not phase0)) and not skip and entry[depth - 1] is not None:
                cnt = nodes - entry[depth - 1]
                key = (rem, ex, bal)
                if entries:
                    s = slot_of(rem, ex, bal, mask)
                    if s is not None:
                        table[s] = (key, cnt)
                else:
                    table[key] = cnt
            skip = False
            prem, pex, pbal, j = stack.pop()
            entry.pop()
            rem, ex, bal = prem, pex, pbal
            depth -= 1
            cand = cands(rem, h) & ~((2 << j) - 1)
            found = 1
        if cand:
            j = lowbit(cand)
            cand &= cand - 1
            p = h.PM[h.pid[j]]
            rr = rem & p & h.RESP
            has = rr != 0
            over = has and nodes >= limit
            if over:
                # stage 0 stops here: the saved state puts j back (LaneDFS::save)
                cand |= 1 << j
                phase0 = False
                limit = 1 << 62
                entry = [None] * len(entry)
                pslot = [None] * len(pslot)
                info["depth"] = depth
                info["cand"] = bin(cand).count("1")
                info["stack_untried"] = sum(bin(cands(pr, h) & ~((2 << pj) - 1)).count("1") for pr, _, _, pj in stack)
                info["fails"] = nodes - depth
                continue
            if not has:
                continue
            r = lowbit(rr)
            nodes += 1
            found = 1
            post = bank_post(ex, bal, (h.code[j], h.a[j], h.b[j], h.val[j]), (h.code[r], h.val[r]))
            if post == 2:
                return 2, nodes, it1, it0, desc, hits
            if post == 1:
                fi = rem & p & h.INV
                stack.append((rem, ex, bal, j))
                entry.append(nodes)
                pslot.append(None)
                ex, bal = bank_next(ex, bal, (h.code[j], h.a[j], h.b[j], h.val[j]))
                rem = rem & ~((fi & -fi) | (1 << r))
                depth += 1
                desc += 1
                cand = cands(rem, h)
                found = 0
                if memo or (policy in ("entry", "noevict") and not phase0 and record_early):
                    key = (rem, ex, bal)
                    cnt = None
                    if entries:
                        s = slot_of(rem, ex, bal, mask)
                        free = s is not None and (policy == "backtrack" or s % alias not in own)
                        if memo and free and s in table and table[s][0] == key:
                            cnt = table[s][1]
                            assert cnt is not None
                        if policy == "noevict" and free and cnt is None and s not in table:
                            table[s] = (key, None)
                            own.add(s % alias)
                            pslot[-1] = s
                        if policy == "entry" and free and cnt is None:
                            table[s] = (key, None)
                            own.add(s % alias)
                            pslot[-1] = s
                    else:
                        cnt = table.get(key)
                    if cnt is not None:
                        nodes += cnt
                        cand = 0
                        found = 1
                        skip = True
                        hits += 1


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    budget = int(sys.argv[2]) if len(sys.argv) > 2 else 18
    memo_after = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    entries = int(sys.argv[4]) if len(sys.argv) > 4 else 128
    policy = sys.argv[5] if len(sys.argv) > 5 else "backtrack"
    alias = int(sys.argv[6]) if len(sys.argv) > 6 else 64
    config = sys.argv[7] if len(sys.argv) > 7 else "bank_4x16"
    import oracle_c
    hdr, ev, _ = gen.generate_config(config, 0, n, threads=8)
    st_o, nd_o, _ = oracle_c.check_batch(2, hdr, ev, threads=8)
    heavy = np.nonzero(nd_o > budget)[0]
    its, its0, descs = [], [], []
    bad = 0
    for i in heavy:
        hd = hdr[i]
        h = Hist(ev[int(hd["ev_off"]): int(hd["ev_off"]) + int(hd["n_ev"])])
        s, nd, it1, it0, desc, hits = run(h, budget, memo_after, entries, policy, alias, os.environ.get("EARLY") == "1")
        if s != int(st_o[i]) or nd != int(nd_o[i]):
            bad += 1
        its.append(it1)
        its0.append(it0)
        descs.append(desc)
    its = np.array(its)
    print(f"n={n} budget={budget} memo_after={memo_after} entries={entries} policy={policy} alias={alias}: heavy {len(heavy)} "
          f"({len(heavy) / n:.4f}), mismatches {bad}")
    q = np.percentile(its, [50, 90, 99, 99.9, 100])
    print("iterations after resume: mean %.1f p50 %d p90 %d p99 %d p99.9 %d max %d" % (its.mean(), *q))
    g = len(its) // 64
    if g:
        gm = its[: g * 64].reshape(g, 64).max(axis=1)
        print("group of 64 (list order): max-iterations median %d p90 %d max %d; lane utilisation %.3f"
              % (np.median(gm), np.percentile(gm, 90), gm.max(), its[: g * 64].sum() / (gm.sum() * 64)))
        srt = np.sort(its)[::-1][: g * 64].reshape(g, 64)
        print("sorted groups: utilisation %.3f, sum of group maxima %d vs %d unsorted"
              % (srt.sum() / (srt.max(axis=1).sum() * 64), srt.max(axis=1).sum(), gm.sum()))
    top = np.argsort(its)[::-1][:10]
    print("longest:", [(int(heavy[k]), int(its[k]), int(nd_o[heavy[k]])) for k in top])


if __name__ == "__main__":
    main()
