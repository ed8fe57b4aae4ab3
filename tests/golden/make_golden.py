"""Generate tests/golden/histories.json from the literal list transliteration
of src/Linearisability.hs:25-69 (oracle/linearise_lists.py).

The reference itself (Haskell) cannot run in this pipeline (no GHC, SURVEY.md
§8c), so these vectors are produced by the transliteration and pinned by the
reference's own known answer (test/TicketDispenser.hs:326-347).  They contain
only data: histories in the Haskell value shapes, the verdict and the node
count.  Re-run:  python tests/golden/make_golden.py
"""

import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "..", "oracle")]

import histgen  # noqa: E402
import linearise_lists as LL  # noqa: E402
from kats import KATS  # noqa: E402


def _json(x):
    return list(_json(y) for y in x) if isinstance(x, tuple) else x


def main():
    rng = random.Random(20181030)
    cases = []
    for name, (model, hist, _, _) in sorted(KATS.items()):
        cases.append((name, model, hist, None, 0))
    for i in range(700):
        model = rng.choice(["ticket", "bank"])
        kind = rng.random()
        if kind < 0.4:
            hist = histgen.random_history(rng, model, rng.randint(0, 14), rng.randint(1, 4))
        else:
            hist = histgen.wellformed_history(rng, model, rng.randint(0, 8), rng.randint(1, 4))
        model0 = None
        if rng.random() < 0.15:
            model0 = rng.randint(0, 4) if model == "ticket" else {"p0": rng.randint(0, 30)}
        cases.append((f"rand{i:04d}", model, hist, model0, 50000))
    out = []
    for cid, model, hist, model0, max_nodes in cases:
        status, nodes, _ = LL.check(model, hist, model0=model0, max_nodes=max_nodes)
        out.append({"id": cid, "model": model, "model0": model0, "max_nodes": max_nodes,
                    "history": [[p, k, _json(x)] for p, (k, x) in hist],
                    "status": status, "nodes": nodes})
    with open(os.path.join(HERE, "histories.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "semantics": "src/Linearisability.hs:25-69 literal transliteration",
                   "cases": out}, f, separators=(",", ":"))
    print(len(out), "cases")


if __name__ == "__main__":
    main()
