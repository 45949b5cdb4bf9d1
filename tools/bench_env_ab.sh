#!/bin/bash
# A/B of bench.py under environment knobs: ENVS="A=1 B=2;C=3" (';' separates
# variants), BENCH_ARGS for the bench; one JSON per variant in gpurun_out/${TAG}_v<k>.json
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-ab}
IFS=';' read -ra VARS <<< "${ENVS}"
k=0
for v in "${VARS[@]}"; do
  echo "== variant $k: $v"
  env $v timeout -k 10 ${LIMIT:-300} python3 -u bench.py --no-cpu-baseline --no-outlier ${BENCH_ARGS} > gpurun_out/${TAG}_v$k.json 2> gpurun_out/${TAG}_v$k.err || { tail -5 gpurun_out/${TAG}_v$k.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/${TAG}_v$k.json'))
print(d['value'], d['ms_per_superstep'], d['baseline_method']['median_ms_per_superstep_2_to_10'], d['run_maxiter10_ms'])"
  k=$((k+1))
done
