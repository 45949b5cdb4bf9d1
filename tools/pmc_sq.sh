#!/bin/bash
# SQ counters of k_al_rebuild_hot (superstep-1 rebuild), class-blocked vs plain, C5.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for B in 512 0; do
  LPA_BLOCK_DEG=$B timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
    --kernel-include-regex "k_al_rebuild_hot" -d gpurun_out/sq_b$B -o run --output-format csv \
    -- python3 tools/pmc_sq_rebuild.py ${CFG:-C5} > gpurun_out/sq_b$B.log 2>&1 || { echo "pass $B failed"; tail -5 gpurun_out/sq_b$B.log; exit 1; }
done
echo done
