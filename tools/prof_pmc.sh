#!/bin/bash
# PMC passes over the LPA kernels of the C3 bench, one counter group per run
# (rocprofv3 does not split counters over passes).  Output: gpurun_out/pmc_<i>/
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS="${BENCH_ARGS:---no-cpu-baseline --steps 9 --warmup 1}"
i=0
while read -r COUNTERS; do
  [ -z "$COUNTERS" ] && continue
  i=$((i+1))
  echo "pass $i: $COUNTERS"
  timeout -s KILL 180 rocprofv3 --pmc $COUNTERS --kernel-include-regex "k_lpa" -d gpurun_out/pmc_$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_${i}_bench.json 2> gpurun_out/pmc_${i}.err || { echo "pass $i failed rc=$?"; tail -5 gpurun_out/pmc_${i}.err; exit 1; }
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS_ATOMIC SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS
FETCH_SIZE TCC_HIT_sum
TCC_MISS_sum WRITE_SIZE
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT
LIST
