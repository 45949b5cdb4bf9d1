#!/bin/bash
# A/B of one in-tree build under two environment settings on the C3 bench,
# interleaved runs:  ENV_A="X=1" ENV_B="X=0" TAG=... REPS=3 tools/ab_env.sh
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-abe}; REPS=${REPS:-3}
for i in $(seq 1 $REPS); do
  for v in A B; do
    if [ $v = A ]; then E=$ENV_A; else E=$ENV_B; fi
    env $E timeout -k 10 200 python3 -u bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_${v}$i.json 2> gpurun_out/${TAG}_${v}$i.err || { tail -5 gpurun_out/${TAG}_${v}$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_${v}$i.json'));r=d['iteration_roofline'];print('$v$i', d['value'], r['median_iter_ms'], r['iter_ms'][0], r['iter_ms'][1])"
  done
done
