# repeat of inflight_budget.sh: auto vs fixed 32 alternated, 3 reps, plus the
# bug batch and the 6x24 sweep config
set -e
O=gpurun_out/inflight_budget2; mkdir -p $O
for r in 1 2 3; do
  for c in bank_4x16 ticket_2x10 bank_4x16_bugs bank_6x24; do
    N=1000000; [ $c = bank_6x24 ] && N=100000
    for b in auto 32; do
      if [ $b = auto ]; then A=""; else A="--stage0-budget $b"; fi
      timeout -k 10 200 python bench.py --config $c --n-hist $N $A --steps 40 --warmup 6 --no-cpu-baseline > $O/${c}_${b}_$r.json 2> $O/${c}_${b}_$r.err || { tail -5 $O/${c}_${b}_$r.err; exit 1; }
    done
  done
done
python - <<'PY'
import json, glob, collections
v = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/inflight_budget2/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    c, b, r = f.split("/")[-1][:-5].rsplit("_", 2)
    v[(c, b)].append(d["value"])
for k in sorted(v):
    print(k, ["%.4g" % x for x in v[k]])
PY
