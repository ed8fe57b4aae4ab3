# memo defaults: full suite, first-call and steady-state timing of every config
set -e
O=gpurun_out/memo2; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python tools/first_call.py > $O/first_call.json 2> $O/first_call.err
cat $O/first_call.json
