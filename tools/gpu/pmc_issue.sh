set -e
O=gpurun_out/pmc_issue; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CMD="python3 bench.py --inflight 1 --steps 6 --warmup 2 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VALU -d $O/p1 -o run --output-format csv -- $CMD > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH -d $O/p2 -o run --output-format csv -- $CMD > $O/p2.log 2>&1
python3 - <<'PY'
import csv, glob, collections
KEY = "compact_search<2u, false, qsmd::(anonymous namespace)::G32>"
for d in ("p1", "p2"):
    for f in glob.glob(f"gpurun_out/pmc_issue/{d}/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if KEY in r.get("Kernel_Name", ""):
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        agg = collections.defaultdict(list)
        for disp in per.values():
            for k, v in disp.items():
                agg[k].append(v)
        print(d, {k: "%.4g" % (sum(v) / len(v)) for k, v in agg.items()})
PY
