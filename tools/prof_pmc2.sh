#!/bin/bash
# instruction-mix PMC passes for the LPA kernels (steady state read from the last dispatches)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS="${BENCH_ARGS:---no-cpu-baseline --steps 9 --warmup 1}"
i=0
while read -r COUNTERS; do
  [ -z "$COUNTERS" ] && continue
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $COUNTERS --kernel-include-regex "k_lpa|k_hub|k_diff|k_al" -d gpurun_out/pmc_$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_${i}_bench.json 2> gpurun_out/pmc_${i}.err || { echo "pass $i failed"; tail -5 gpurun_out/pmc_${i}.err; exit 1; }
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA
FETCH_SIZE TCC_HIT_sum
TCC_MISS_sum WRITE_SIZE
LIST
python3 tools/pmc_summary.py gpurun_out 4 | grep -A30 -E "== (k_lpa_wave|k_lpa_seg)" | grep -v GRBM
