#!/bin/bash
# A/B of bench.py settings on one box, alternated (diagnostic):
#   tools/gpu/archive/ab_params.sh ROUNDS "TAG|ENV|ARGS" ...
# ENV: space-separated VAR=VALUE (e.g. QSMD_LIB_PATH=ablib/x.so), may be empty.
# Each run: bench.py --no-cpu-baseline --no-extra ARGS; prints TAG value stage0/call means.
R=$1; shift
mkdir -p gpurun_out/abp
for r in $(seq 1 "$R"); do
  for spec in "$@"; do
    tag=${spec%%|*}; rest=${spec#*|}; envs=${rest%%|*}; args=${rest#*|}
    env $envs timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extra $args > gpurun_out/abp/$tag.$r.json 2> gpurun_out/abp/$tag.$r.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "$tag rc=$rc"; exit $rc; fi
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/abp/$tag.$r.json') if l.startswith('{')][-1]); f=d['device_ms']['in_flight']; a=d['device_ms']['alone']; print('$tag', '%.4g' % d['value'], 'in flight %.1f %.1f alone %.1f %.1f' % (1e3*f['stage0_mean'], 1e3*f['call_mean'], 1e3*a['stage0_mean'], 1e3*a['call_mean']))"
  done
done
