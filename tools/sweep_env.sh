#!/bin/bash
# one bench per setting in VALS of the environment variable VAR (C3, no CPU baseline):
# prints value, median superstep, supersteps 2/3 and the standalone k_lpa_units time
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in $(seq 1 ${REPS:-1}); do
for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python3 -u bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/sw_$v.json 2> gpurun_out/sw_$v.err || { tail -5 gpurun_out/sw_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sw_$v.json'));r=d['iteration_roofline'];print('$VAR=$v', d['value'], r['median_iter_ms'], r['iter_ms'][0], r['iter_ms'][1], d['kernel_ms_per_step'].get('k_lpa_units'))"
done
done
