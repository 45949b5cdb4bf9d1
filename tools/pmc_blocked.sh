#!/bin/bash
# L2 behaviour of the superstep-1 labels-mode rebuild, class-blocked (LPA_BLOCK_DEG=64)
# against the plain stream (LPA_BLOCK_DEG=0): TCC hits / misses and FETCH_SIZE of
# k_al_rebuild_hot over tools/pmc_workload3.py (C3), one counter group per rocprofv3
# pass (kernel trace only).  Output: gpurun_out/${TAG}_b{0,64}_{hit,fetch}/
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-pmcb}
for B in 0 64; do
  for P in "hit:TCC_HIT_sum TCC_MISS_sum" "fetch:FETCH_SIZE"; do
    n=${P%%:*}; c=${P#*:}
    LPA_BLOCK_DEG=$B timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "k_al_rebuild_hot" \
      -d gpurun_out/${TAG}_b${B}_$n -o run --output-format csv -- python3 tools/pmc_workload3.py \
      gpurun_out/${TAG}_info.json > gpurun_out/${TAG}_b${B}_$n.log 2>&1 || { echo "pass $B $n failed"; tail -5 gpurun_out/${TAG}_b${B}_$n.log; exit 1; }
  done
done
echo done
