#!/bin/bash
# Paired state DAG: the wave-mode parity tests, DAG timings (pairs on / off),
# then one rank with and without RCCL (dedicated all-reduce stream).
set -o pipefail
mkdir -p gpurun_out/rccl
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py -x -q --timeout 120 \
    --timeout-method thread -k "wave_mode or heavy_any_shape or generated_configs or memo or stage_cascade or adversarial or dag or model_error or budget" \
    > gpurun_out/pair_pytest.log 2>&1 || { tail -30 gpurun_out/pair_pytest.log; exit 1; }
tail -2 gpurun_out/pair_pytest.log
rm -f gpurun_out/paircmp.log
for cfg in "bank_4x16 1000000" "bank_4x16_bugs 200000 wave_max=10000000" "bank_6x24 100000" "ticket_2x10 1000000"; do
  for kn in "dag_pair=1" "dag_pair=0"; do
    echo "== $cfg $kn" >> gpurun_out/paircmp.log
    timeout -k 10 120 python -u tools/wave_stats.py $cfg $kn --nostats 2>&1 | grep -v amdgpu.ids | tail -2 >> gpurun_out/paircmp.log || exit 1
  done
done
cat gpurun_out/paircmp.log
timeout -k 10 200 python bench.py --inflight 1 --steps 100 --no-extra --no-cpu-baseline > gpurun_out/pair_infl1.json 2> gpurun_out/pair_infl1.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/pair_infl1.json')); print('inflight1', d['value'], d['device_ms'])"
bash tools/gpu/rccl_sweep.sh 2 "none||" "dist|QSMD_BENCH_DIST=1|" "dist_noar|QSMD_BENCH_DIST=1 QSMD_BENCH_NOAR=1|" > gpurun_out/rccl/sweep2.log 2>&1
rc=$?
cat gpurun_out/rccl/sweep2.log
exit $rc
