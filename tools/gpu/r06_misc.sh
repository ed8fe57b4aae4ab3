#!/bin/bash
# Round 6 measurements:
#  1. the early-exit leg: config 3 (its first failure is its second history)
#     and config 2's stream with one failure planted at 60 % (the geometric
#     rounds, a MIN per round);
#  2. config 3's exhaustive call: a kernel trace of its in-flight steps and
#     the heavy stage's anatomy (tools/memo_stats.py) at 1.25M histories;
#  3. the one-rank RCCL loss: per-thread CPU time inside the window and the
#     main thread pinned, without a process group and with a live
#     communicator (3 interleaved rounds).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_misc
mkdir -p $O/config3
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 python bench.py --early-exit --steps 20 --warmup 3 > $O/bench_early.json 2> $O/bench_early.err || { tail $O/bench_early.err; exit 1; }
timeout -k 10 200 python bench.py --early-exit --plant 0.6 --steps 20 --warmup 3 > $O/bench_early_planted.json 2> $O/bench_early_planted.err || { tail $O/bench_early_planted.err; exit 1; }
python3 -c "
import json
for f in ('bench_early', 'bench_early_planted'):
    d = json.load(open('$O/%s.json' % f)); e = d['early_exit']
    print(f, 'ms_to_decision %.3f' % e['ms_to_decision'], 'searched/s %.3e' % e['histories_searched_per_sec'], 'searched', e['searched'], 'rounds', e['rounds'], 'first_fail', e['first_fail'], 'mism', e.get('mismatches_vs_oracle'))
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/config3/trace -o c3 -- python3 bench.py --config bank_4x16_bugs --n-hist 1250000 --steps 10 --warmup 3 --inflight 3 --stage0-budget -1 --rotate 1 --no-extra --no-cpu-baseline --roof-calls 10 > $O/config3/bench.json 2> $O/config3/bench.err || { tail $O/config3/bench.err; exit 1; }
find $O/config3/trace -name "*_trace.csv" -size +4M -delete
timeout -k 10 120 python tools/memo_stats.py bank_4x16_bugs 1250000 heavy_mode=1 memo_lds=0 > $O/config3/memo_stats.json 2> $O/config3/memo_stats.err || { tail $O/config3/memo_stats.err; exit 1; }
cat $O/config3/memo_stats.json
cat $(find $O/config3/trace -name "*kernel_stats.csv") | head -12
for r in 1 2 3; do
  for v in none rccl rccl_pin none_pin; do
    case $v in
      none) E="";; none_pin) E="QSMD_BENCH_PIN=1";;
      rccl) E="QSMD_BENCH_DIST=1 QSMD_BENCH_COUNTERS=rccl";; rccl_pin) E="QSMD_BENCH_DIST=1 QSMD_BENCH_COUNTERS=rccl QSMD_BENCH_PIN=1";;
    esac
    env $E QSMD_BENCH_THREADS=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $O/rccl_$v$r.json 2> $O/rccl_$v$r.err || { tail $O/rccl_$v$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/rccl_$v$r.json'))
th = [json.loads(l) for l in open('$O/rccl_$v$r.err') if l.startswith('{\"window_ms')]
print('$v round $r', '%.3e' % d['value'], th[-1] if th else '')
"
  done
done
