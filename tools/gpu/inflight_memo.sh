# bench default (3 in flight, stage-0 budget 32) vs memo-stage grid and
# nearby budgets, alternated, 2 reps
set -e
O=gpurun_out/inflight_memo; mkdir -p $O
declare -A V=([base]="" [mg256]="--param memo_grid=256" [mg512]="--param memo_grid=512" [b24]="--stage0-budget 24" [b40]="--stage0-budget 40")
for r in 1 2; do
  for c in bank_4x16 ticket_2x10 bank_4x16_bugs; do
    for v in base mg256 mg512 b24 b40; do
      timeout -k 10 200 python bench.py --config $c ${V[$v]} --steps 40 --warmup 6 --no-cpu-baseline > $O/${c}_${v}_$r.json 2> $O/${c}_${v}_$r.err || { tail -5 $O/${c}_${v}_$r.err; exit 1; }
    done
  done
done
python - <<'PY'
import json, glob, collections
v = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/inflight_memo/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    c, b, r = f.split("/")[-1][:-5].rsplit("_", 2)
    v[(c, b)].append(d["value"])
for k in sorted(v):
    print(k, ["%.4g" % x for x in v[k]])
PY
