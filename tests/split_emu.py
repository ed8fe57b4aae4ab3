"""CPU emulation of the split-search entry points (split_frontier /
check_tasks) -- TEST INFRASTRUCTURE for the multi-rank orchestration in
qsmd.dist (gloo, no GPU).  A direct counter-state restatement of the
reference DFS (src/Linearisability.hs:52-69, SURVEY.md §8a Lemma L1) with a
depth cut and subtree search; pinned to oracle/ref_cpu.c in test_distributed.
"""

import numpy as np

from qsmd import device

FALSE, TRUE, ERR, BUDGET = 0, 1, 2, 4


class _Hist:
    def __init__(self, model_id, hdr, events):
        h = hdr[0]
        ev = events[int(h["ev_off"]): int(h["ev_off"]) + int(h["n_ev"])]
        self.model_id = model_id
        self.ev = [(int(x["kp"]) & 0x7F, int(x["kp"]) >> 7, int(x["code"]), int(x["a"]), int(x["b"]),
                    int(x["val"])) for x in ev]
        self.n_pid = int(h["n_pid"])
        self.ord, cnt = [], {}
        self.resp_pos = {p: [] for p in range(self.n_pid)}
        for i, (p, r, *_rest) in enumerate(self.ev):
            self.ord.append(cnt.get((p, r), 0))
            cnt[(p, r)] = cnt.get((p, r), 0) + 1
            if r:
                self.resp_pos[p].append(i)

    def model0(self):
        return (0, 0) if self.model_id == 1 else {}

    def post(self, m, inv, resp):
        code, a, money = inv[2], inv[3], inv[5]
        rc, rv = resp[2], resp[5]
        if self.model_id == 1:                                       # TicketDispenser.hs:99-102
            if code == 0:
                return TRUE if rc == 0 and m[0] and rv == m[1] + 1 else FALSE
            return TRUE if rc == 1 else FALSE
        if any(v < 0 for v in m.values()):                           # Bank.hs:103-104,118
            return FALSE
        ge = a in m and m[a] >= money
        exp = {0: 4 if a in m else 0, 1: 1, 2: 2 if ge else 6, 3: 7, 4: 3 if ge else 6}[code]
        if rc != exp:
            return FALSE
        if code == 3:
            if a not in m:
                return ERR                                           # Map.!
            return TRUE if rv == m[a] else FALSE
        return TRUE

    def next(self, m, inv):
        code, a, b, money = inv[2], inv[3], inv[4], inv[5]
        if self.model_id == 1:
            return (m[0], m[1] + 1 if m[0] else 0) if code == 0 else (1, 0)
        m = dict(m)
        if code == 0:
            m.setdefault(a, 0)
        elif code == 1:
            m[a] = m[a] + money if a in m else money
        elif code in (2, 4):
            m[a] = m[a] - money if a in m else money
            if code == 4:
                m[b] = m[b] + money if b in m else money
        return m


class _Search:
    def __init__(self, H, limit):
        self.H, self.limit, self.nodes, self.path = H, limit, 0, []
        self.cut, self.tasks = None, []

    def expand(self, k, m, is_root):
        H = self.H
        R = min([H.resp_pos[p][k[p]] for p in range(H.n_pid) if k[p] < len(H.resp_pos[p])],
                default=len(H.ev))
        any_child = False
        for e in range(R):
            p, r = H.ev[e][0], H.ev[e][1]
            if r or H.ord[e] < k[p] or k[p] >= len(H.resp_pos[p]):
                continue
            any_child = True
            res = self.step(k, m, p, e, H.resp_pos[p][k[p]])
            if res != FALSE:
                return res
        return (FALSE if is_root else TRUE) if not any_child else FALSE

    def step(self, k, m, p, e, r):
        if self.limit and self.nodes >= self.limit:
            return BUDGET
        self.nodes += 1
        ok = self.H.post(m, self.H.ev[e], self.H.ev[r])
        if ok != TRUE:
            return ok
        m2 = self.H.next(m, self.H.ev[e])
        self.path.append(e)
        k[p] += 1
        if self.cut is not None and len(self.path) == self.cut:
            self.tasks.append((list(self.path), self.nodes))
            res = FALSE
        else:
            res = self.expand(k, m2, False)
        k[p] -= 1
        if res != TRUE:
            self.path.pop()
        return res


class EmuChecker:
    """split_frontier / check_tasks with the signatures of qsmd.device.Context."""

    def split_frontier(self, model_id, hdr, events, model0=None, flags=1, max_nodes=0, min_tasks=64,
                       max_tasks=4096, witness=False):
        H = _Hist(model_id, hdr, events)
        if not H.ev:
            fr = device.Frontier(status=TRUE, depth=0, top_nodes=0, n_tasks=0)
            return fr, np.zeros(0, dtype=device.TASK_DTYPE), np.zeros(0, np.uint8)

        def top(cut):
            s = _Search(H, max_nodes)
            s.cut = cut
            res = s.expand([0] * H.n_pid, H.model0(), True)
            return s, res

        dmax = min(16, len(H.ev) // 2)
        cut = 1
        while True:
            s, res = top(cut)
            if len(s.tasks) > max_tasks and cut > 1:
                cut -= 1
                break
            if len(s.tasks) >= min_tasks or cut >= dmax:
                break
            cut += 1
        s, res = top(cut)
        tasks = np.zeros(len(s.tasks), dtype=device.TASK_DTYPE)
        for i, (path, before) in enumerate(s.tasks):
            tasks[i]["depth"] = cut
            tasks[i]["top_before"] = before
            tasks[i]["path"][:cut] = path
        w = np.full(max(len(H.ev), 1), 0xFF, np.uint8)
        if res == TRUE:
            w[: len(s.path)] = s.path
        fr = device.Frontier(status=res, depth=cut, top_nodes=s.nodes, n_tasks=len(tasks))
        return fr, tasks, w[: len(H.ev)]

    def check_tasks(self, model_id, hdr, events, tasks, model0=None, flags=1, max_nodes=0, witness=False):
        H = _Hist(model_id, hdr, events)
        st = np.zeros(len(tasks), np.uint8)
        nd = np.zeros(len(tasks), np.uint64)
        wit = np.full((len(tasks), 64), 0xFF, np.uint8)
        decided = False
        for i, t in enumerate(tasks):
            if decided:
                st[i] = 5
                continue
            k, m = [0] * H.n_pid, H.model0()
            path = [int(x) for x in t["path"][: int(t["depth"])]]
            for e in path:
                p = H.ev[e][0]
                m = H.next(m, H.ev[e])
                k[p] += 1
            s = _Search(H, max_nodes)
            s.path = list(path)
            res = s.expand(k, m, False)
            st[i], nd[i] = res, s.nodes
            if res == TRUE:
                wit[i, : len(s.path)] = s.path
            decided = res in (TRUE, ERR)
        return st, nd, wit
