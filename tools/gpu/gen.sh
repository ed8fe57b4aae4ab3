set -e
O=gpurun_out/gen; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gen.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python bench.py --device-gen --steps 10 --warmup 3 --cpu-seconds 3 > $O/bench.json 2> $O/bench.err
tail -3 $O/bench.err; cat $O/bench.json
