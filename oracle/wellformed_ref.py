"""TEST INFRASTRUCTURE (oracle): a literal restatement of the reference's
`isSequential` / `wellformed` (src/Linearisability.hs:97-135), the checker for
the batched device kernel (csrc/wellformed.hip).  Never imported by the
product path.

A history is a list of (pid, (kind, payload)) with kind "L" (Left inv) or
"R" (Right resp).  Returns None (Right ()) or (constructor, args)."""


def process_subhistory(pid, history):            # :106-107
    return [e for e in history if e[0] == pid]


def is_sequential(history):                      # :109-128
    if history and history[0][1][0] == "R":
        pid, (_, resp) = history[0]
        return ("FirstEventIsntInvocation", (pid, resp))
    return _go(history)


def _go(h):
    while True:
        if not h:
            return None
        if len(h) == 1:
            pid, (k, x) = h[0]
            return ("LoneResponse", (pid, x)) if k == "R" else None
        (p0, (k0, x0)), (p1, (k1, x1)) = h[0], h[1]
        if k0 == "L" and k1 == "R":
            if p0 == p1:
                h = h[2:]
                continue
            return ("InvocationFollowedByNonMatchingResponse", (p0, x0, p1, x1))
        if k0 == "L" and k1 == "L":
            return ("InvocationFollowedByInvocation", (p0, x0, p1, x1))
        if k0 == "R" and k1 == "R":
            return ("ResponseFollowedByResponse", (p0, x0, p1, x1))
        return ("ResponseFollowedByInvocation", (p0, x0, p1, x1))


def wellformed(pids, history):                   # :130-135, allRight = foldr (>>) (Right ())
    for pid in pids:
        err = is_sequential(process_subhistory(pid, history))
        if err is not None:
            return err
    return None
