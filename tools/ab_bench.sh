#!/bin/bash
# Same-box A/B of the in-tree library (new) against tools/ab_lib/liblpa_hip.so (base):
# bench.py ${CFG:-C3} without the CPU baseline / outlier / quality, alternating, N rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in $(seq 1 ${N:-2}); do
  for v in new base; do
    if [ $v = base ]; then export LPA_LIB_PATH=$PWD/tools/ab_lib/liblpa_hip.so; else unset LPA_LIB_PATH; fi
    timeout -k 10 300 python3 -u bench.py --config ${CFG:-C3} --no-cpu-baseline --no-outlier --no-quality ${ARGS} \
      > gpurun_out/ab_${CFG:-C3}_${v}_$r.json 2> gpurun_out/ab_${CFG:-C3}_${v}_$r.err || { tail -5 gpurun_out/ab_${CFG:-C3}_${v}_$r.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab_${CFG:-C3}_${v}_$r.json'))
print('$v', d['value'], d['ms_per_step'], d['baseline_method']['median_ms_per_superstep_2_to_10'][:4])"
  done
done
