#!/bin/bash
# SQ / LDS counter passes (one group per run) over chosen kernels of the C3 bench.
#   KREGEX="k_lpa_units|k_hub_small" TAG=x bash tools/pmc_sq.sh
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-sq}; KREGEX=${KREGEX:-k_lpa_units}
i=0
while read -r COUNTERS; do
  [ -z "$COUNTERS" ] && continue
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $COUNTERS --kernel-include-regex "$KREGEX" -d gpurun_out/${TAG}_$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { echo "pass $i failed"; tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS_ATOMIC SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS
LIST
python3 tools/pmc_dispatch.py "gpurun_out/${TAG}_*" > gpurun_out/${TAG}_table.txt
cat gpurun_out/${TAG}_table.txt
