# finer stage-0 budget sweep under 3 calls in flight: the bug batch and
# TicketDispenser 2x10, alternated, 2 reps
set -e
O=gpurun_out/inflight_budget3; mkdir -p $O
for r in 1 2; do
  for cb in bank_4x16_bugs:32 bank_4x16_bugs:40 bank_4x16_bugs:48 bank_4x16_bugs:64 bank_4x16_bugs:96 ticket_2x10:16 ticket_2x10:20 ticket_2x10:24 ticket_2x10:28 bank_4x16:20 bank_4x16:28; do
    c=${cb%:*}; b=${cb#*:}
    timeout -k 10 200 python bench.py --config $c --stage0-budget $b --steps 40 --warmup 6 --no-cpu-baseline > $O/${c}_${b}_$r.json 2> $O/${c}_${b}_$r.err || { tail -5 $O/${c}_${b}_$r.err; exit 1; }
  done
done
python - <<'PY'
import json, glob, collections
v = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/inflight_budget3/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    c, b, r = f.split("/")[-1][:-5].rsplit("_", 2)
    v[(c, int(b))].append(d["value"])
for k in sorted(v):
    print(k, ["%.4g" % x for x in v[k]])
PY
