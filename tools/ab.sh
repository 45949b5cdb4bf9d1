#!/bin/bash
# A/B of two builds of liblpa_hip.so on the C3 bench, interleaved runs:
#   LIB_B=<path to the alternative .so>  (A = the in-tree build)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-ab}; REPS=${REPS:-3}
for i in $(seq 1 $REPS); do
  for v in A B; do
    if [ $v = B ]; then export LPA_LIB_PATH=$LIB_B; else unset LPA_LIB_PATH; fi
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_${v}$i.json 2> gpurun_out/${TAG}_${v}$i.err || { tail -5 gpurun_out/${TAG}_${v}$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_${v}$i.json'));r=d['iteration_roofline'];print('$v$i', d['value'], r['median_iter_ms'], r['iter_ms'][0], r['iter_ms'][1])"
  done
done
