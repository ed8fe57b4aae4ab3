#!/bin/bash
# Round 6: the wave stage's chain paths (wave.hip ticket_shared_chain /
# ticket_chain): the GPU suite, then config 4 through the host entry.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${TAG:-r06_chain}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q -k "chain or adversarial" --timeout 240 --timeout-method thread > $O/pytest_chain.log 2>&1 || { tail -30 $O/pytest_chain.log; exit 1; }
tail -1 $O/pytest_chain.log
timeout -k 10 120 python3 tools/config4.py --reps 200 "" > $O/c4.log 2>&1 || { tail $O/c4.log; exit 1; }
timeout -k 10 120 python3 tools/config4.py --bug 0 --reps 200 "" >> $O/c4.log 2>&1 || { tail $O/c4.log; exit 1; }
cat $O/c4.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
