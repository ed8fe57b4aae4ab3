O=gpurun_out/wf1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_wellformed.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1; tail -4 $O/tests.log
timeout -k 10 120 python tools/bench_wellformed.py > $O/bench.json 2> $O/bench.err; cat $O/bench.json
