#!/bin/bash
# Round 3: serialized per-superstep kernel times (C3) and the per-kernel PMC table of
# supersteps 1..5 (SQ occupancy/issue/LDS, HBM bytes, L2 hits), one pass per counter set.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-p1}
timeout -k 10 200 python3 -u tools/superstep_breakdown.py C3 > gpurun_out/${TAG}_breakdown.txt 2>&1 || { tail -20 gpurun_out/${TAG}_breakdown.txt; exit 1; }
cat gpurun_out/${TAG}_breakdown.txt | tail -40
TAG=${TAG}_dense N=5 bash tools/pmc_dense.sh
