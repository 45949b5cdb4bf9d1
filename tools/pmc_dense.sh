#!/bin/bash
# SQ / GRBM / TCC counters of every kernel of supersteps 1..N (serialized schedule, C3):
# occupancy, issue and LDS behaviour of the label-dense tallies, HBM bytes and L2 hits.  One rocprofv3
# --pmc pass per counter set (guide: at most 8 SQ + 2 GRBM per pass).
# Output: gpurun_out/${TAG}_pmc<k>/ (csv) and gpurun_out/${TAG}_dense.txt
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-dense}
CFG=${CFG:-C3}
N=${N:-4}
SETS=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum"
)
k=0
for S in "${SETS[@]}"; do
  timeout -s KILL 240 rocprofv3 --pmc $S -d gpurun_out/${TAG}_pmc$k -o run --output-format csv -- python3 tools/pmc_dense_workload.py $CFG $N > gpurun_out/${TAG}_pmc$k.log 2>&1 || { echo "pass $k failed"; tail -5 gpurun_out/${TAG}_pmc$k.log; exit 1; }
  k=$((k+1))
done
python3 tools/pmc_dense.py gpurun_out/${TAG} $N > gpurun_out/${TAG}_dense.txt && cat gpurun_out/${TAG}_dense.txt
