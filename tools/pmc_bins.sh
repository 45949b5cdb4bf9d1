#!/bin/bash
# Per-bin counter evidence (north_star: achieved HBM GB/s, LDS bank conflicts, wave
# occupancy per degree bin).  Three --pmc passes over the C3 bench, one counter group
# each (SQ / GRBM, FETCH_SIZE, WRITE_SIZE + L2 hit/miss), superstep kernels only.
#   TAG=bins bash tools/pmc_bins.sh   -> gpurun_out/${TAG}_table.txt
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-bins}
KREGEX=${KREGEX:-"k_lpa_|k_hub_|k_al_|k_diff"}
i=0
while read -r COUNTERS; do
  [ -z "$COUNTERS" ] && continue
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $COUNTERS --kernel-include-regex "$KREGEX" -d gpurun_out/${TAG}_$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { echo "pass $i failed"; tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
  echo "pass $i done"
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
LIST
python3 tools/pmc_bins.py "gpurun_out/${TAG}_[0-9]*" > gpurun_out/${TAG}_table.txt
cat gpurun_out/${TAG}_table.txt
