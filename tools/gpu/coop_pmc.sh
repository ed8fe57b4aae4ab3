export TMPDIR=/tmp
O=gpurun_out/cp; mkdir -p $O
CMD="python3 tools/spread_diag.py --config bank_4x16 --reps 1 --variants stage0_budget=64"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $CMD > $O/trace.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $O/p1 -o run --output-format csv -- $CMD > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT -d $O/p2 -o run --output-format csv -- $CMD > $O/p2.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
O='gpurun_out/cp'
for f in glob.glob(O+'/trace/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print('STAT', r['Name'][:60], r['Calls'], r['AverageNs'])
for d in ('p1','p2'):
    for f in glob.glob(O+'/'+d+'/**/*counter_collection.csv', recursive=True):
        agg = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if 'coop' in r.get('Kernel_Name',''):
                agg[r['Counter_Name']] += float(r['Counter_Value'])
        print(d, dict(agg))
PY
