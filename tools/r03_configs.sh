#!/bin/bash
# Round 3: bench on C2, C5 and C4 (one GPU), no CPU baseline / outlier / quality legs.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-cf}
for C in ${CONFIGS:-C2 C5 C4}; do
  timeout -k 10 400 python3 -u bench.py --config $C --steps 5 --warmup 1 --no-cpu-baseline --no-outlier --no-quality > gpurun_out/${TAG}_$C.json 2> gpurun_out/${TAG}_$C.err || { tail -20 gpurun_out/${TAG}_$C.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$C.json'));print('$C', d['value'], d['ms_per_step'], d['baseline_method']['median_ms_per_superstep_2_to_10'], d['run_maxiter10_ms'])"
done
