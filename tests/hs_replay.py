"""A line-by-line Python mirror of `replay` in hs/Linearisability/Device.hs
(no GHC in this image, so the Haskell itself cannot run): the test suite
checks that it accepts exactly the successful root-to-leaf paths of the
reference's tree (src/Linearisability.hs:25-69) and rejects truncated and
out-of-prefix witnesses.  Keep it in step with the Haskell text."""


def hs_replay(transition, postcondition, model0, hist, ws):
    # replay _ _ _ hist [] = null hist
    if not ws:
        return len(hist) == 0
    rest0 = list(enumerate(hist))            # zip [0 ..] hist

    def is_inv(ev):                          # isInv (_, Left _) = True
        return ev[1][0] == "L"

    def prefix(rest):                        # takeWhile (isInv . snd)
        out = []
        for i, ev in rest:
            if not is_inv(ev):
                break
            out.append((i, ev))
        return out

    def first_resp(pid, rest):               # [ (k, r) | (k, (q, Right r)) <- rest, q == pid ]
        for k, (q, (kind, r)) in rest:
            if kind == "R" and q == pid:
                return (k, r)
        return None

    def roots(rest):
        return [i for i, (pid, _) in prefix(rest) if first_resp(pid, rest) is not None]

    def drop_first_inv(pid, evs):            # break isInvOf evs
        for n, (_, (q, (kind, _))) in enumerate(evs):
            if kind == "L" and q == pid:
                return evs[:n] + evs[n + 1:]
        return evs

    def go(m, rest, ws):
        if not ws:                           # go _ rest [] = null (roots rest)
            return not roots(rest)
        j, js = ws[0], ws[1:]
        hit = dict(prefix(rest)).get(j)      # lookup j (prefix rest)
        if hit is None:
            return False
        pid, (_, inv) = hit
        kr = first_resp(pid, rest)
        if kr is None:
            return False
        k, resp = kr
        return (postcondition(m, inv, resp)
                and go(transition(transition(m, ("L", inv)), ("R", resp)),
                       drop_first_inv(pid, [e for e in rest if e[0] != k]), js))

    return go(model0, rest0, list(ws))


def successful_paths(transition, postcondition, model0, hist, limit=10000):
    """Every root-to-leaf path of the reference's tree whose postconditions
    all hold, as invocation-event indices (the nodes are `interleavings`,
    src/Linearisability.hs:36-42, over index-tagged events)."""
    out = []

    def children(rest):
        for n, (i, (pid, ev)) in enumerate(rest):
            if ev[0] != "L":
                break                        # takeInvocations
            # filter1 (not . matchInvocation pid): the first invocation of pid
            es1 = list(rest)
            for t, (_, (q, e2)) in enumerate(es1):
                if q == pid and e2[0] == "L":
                    es1 = es1[:t] + es1[t + 1:]
                    break
            # findResponse pid
            for t, (_, (q, e2)) in enumerate(es1):
                if q == pid and e2[0] == "R":
                    yield i, ev[1], e2[1], es1[:t] + es1[t + 1:]
                    break

    def walk(m, rest, path):
        if len(out) >= limit:
            return
        kids = list(children(rest))
        if not kids:
            if path:
                out.append(list(path))
            return
        for i, inv, resp, rest2 in kids:
            try:
                if not postcondition(m, inv, resp):
                    continue
            except Exception:
                continue
            walk(transition(transition(m, ("L", inv)), ("R", resp)), rest2, path + [i])

    walk(model0, list(enumerate(hist)), [])
    return out
