#!/bin/bash
# C5 (Chung-Lu 40 M / 1.4 B, one GPU) under environment variants: ENVS="A=1;B=2"
# (';' separates variants); prints value, per-superstep medians and lpa_run(10) ms.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-c5ab}
IFS=';' read -ra VARS <<< "${ENVS}"
k=0
for v in "${VARS[@]}"; do
  echo "== variant $k: $v"
  env $v timeout -k 10 ${LIMIT:-400} python3 -u bench.py --config C5 --no-cpu-baseline --no-outlier --steps 2 --warmup 1 > gpurun_out/${TAG}_v$k.json 2> gpurun_out/${TAG}_v$k.err || { tail -5 gpurun_out/${TAG}_v$k.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_v$k.json'))
print(d['value'], d['ms_per_superstep'], d['baseline_method']['median_ms_per_superstep_2_to_10'], d['run_maxiter10_ms'], d['roofline']['avg_launch_ms'])"
  k=$((k+1))
done
