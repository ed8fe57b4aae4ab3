#!/bin/bash
# Round 6: the GPU suite and smoke() on the current tree.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_tests
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
