#!/bin/bash
# Round 6: BASELINE config 4 through the host entry -- 100 calls of the one
# adversarial 8 x 64 TicketDispenser history (QSMD_FLAG_MEMO) under a kernel
# + HIP API trace (tools/config4.py), then untraced.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r06_config4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $O/trace -o c4 -- python3 tools/config4.py --reps 100 > $O/traced.log 2>&1 || { tail -20 $O/traced.log; exit 1; }
tail -3 $O/traced.log
# keep the summaries and the config-4 calls' records (the traces of torch's start-up are large)
python3 tools/trace_c4.py $O/trace > $O/c4_summary.txt 2>&1 || { tail $O/c4_summary.txt; exit 1; }
find $O/trace -name "*_trace.csv" -size +2M -delete
cat $O/c4_summary.txt
timeout -k 10 100 python3 tools/config4.py --reps 200 > $O/untraced.log 2>&1 || { tail -20 $O/untraced.log; exit 1; }
cat $O/untraced.log
find $O/trace -name "*stats*" | head
