# GPU tests, then config-2 timing (sweep tool) and the bench line.
# usage: bash tools/gpu/test_and_bench.sh <outdir> [extra sweep variants]
set -e
O=${1:-gpurun_out/tb}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python tools/sweep_params.py --config bank_4x16 --variants "${2:-stage0_grid=65536}" > $O/sweep.json 2> $O/sweep.err
cat $O/sweep.json
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
cat $O/bench.json
