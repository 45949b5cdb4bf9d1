#!/bin/bash
# Repeated C3 bench runs (no CPU baseline) to separate signal from run-to-run noise.
# Prints: value, median superstep, superstep 2, superstep 3 per run.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-rep}; REPS=${REPS:-3}
for i in $(seq 1 $REPS); do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/${TAG}_$i.json'));r=d['iteration_roofline'];print('run $i', d['value'], r['median_iter_ms'], r['iter_ms'][0], r['iter_ms'][1])"
done
