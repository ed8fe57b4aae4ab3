set -e
for v in "" "stage0_budget=512" "stage0_budget=128" "stage0_budget=64" "stage0_budget=128,memo_stage=0,heavy_stage=0" "stage0_budget=64,memo_stage=0,heavy_stage=0" "stage0_budget=32,memo_stage=0,heavy_stage=0"; do
  timeout -k 10 120 python tools/memo_stats.py --config bank_4x16 --set "$v" 2>/dev/null
done
