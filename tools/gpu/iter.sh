#!/bin/bash
# Iteration check on the GPU: smoke, the -m gpu suite (stop at the first
# failure), wave-mode stats on config 2, a short bench.  Each GPU step has its
# own time limit; the chain stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} \
    > gpurun_out/pytest.log 2>&1 &&
timeout -k 10 120 python -u tools/wave_stats.py bank_4x16 1000000 > gpurun_out/wave_stats.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
tail -3 gpurun_out/smoke.log; tail -5 gpurun_out/pytest.log; cat gpurun_out/wave_stats.log 2>/dev/null | grep -v amdgpu.ids
cat gpurun_out/bench.json 2>/dev/null | head -c 1500
exit $rc
