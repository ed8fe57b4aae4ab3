# Round profile of the bench command (config 2): kernel trace + stats, then
# separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ instruction mix, LDS),
# summarised into profiles/<tag>/ and profiles/pmc_traffic.json.
# usage: bash tools/gpu/profile_round.sh <tag>
set -e
TAG=${1:-r01/v5}
O=gpurun_out/prof_$(echo $TAG | tr / _); mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CMD="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $CMD > $O/bench_under_rocprof.json 2> $O/trace.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $CMD > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $CMD > $O/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS -d $O/sq -o run --output-format csv -- $CMD > $O/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY -d $O/lds -o run --output-format csv -- $CMD > $O/lds.log 2>&1
python3 tools/profile_summary.py $O profiles/$TAG
