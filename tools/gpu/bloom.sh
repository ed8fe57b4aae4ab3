set -e
O=gpurun_out/bloom; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "memo or straggler" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python tools/memo_stats.py 2>/dev/null
timeout -k 10 120 python tools/memo_stats.py --config bank_6x24 --n 100000 2>/dev/null
timeout -k 10 200 python bench.py --config bank_4x16_bugs --inflight 1 --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bugs inflight1', d['ms_per_step'], d['value'])"
timeout -k 10 200 python bench.py --config bank_4x16_bugs --inflight 2 --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bugs inflight2', d['ms_per_step'], d['value'])"
