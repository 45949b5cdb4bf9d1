#!/bin/bash
# HBM traffic per launch (MI355X guide, HBM section): FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 --pmc passes, no trace domains.
#   1. calibration: mb_rebuild's stream kernel (4 B/lane non-temporal col reads and
#      al writes, exact byte counts known) and its rebuild variants
#   2. the library: tools/pmc_workload.py (C3, labelPropagation(10), frontier off)
# Output: gpurun_out/${TAG}_pmc_*/ and gpurun_out/${TAG}_traffic.json
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-pmc}
timeout -k 10 200 python3 tools/microbench/dump_deg.py C3 /tmp/deg_c3.bin > /dev/null || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  c=$(echo $C | cut -d_ -f1 | tr A-Z a-z)
  MB_BASIC=1 timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "k_floor|k_hot" -d gpurun_out/${TAG}_pmc_mb_$c -o run --output-format csv -- ./tools/microbench/mb_rebuild /tmp/deg_c3.bin 2 > gpurun_out/${TAG}_pmc_mb_$c.log 2>&1 || { echo "mb pass $C failed"; tail -5 gpurun_out/${TAG}_pmc_mb_$c.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "k_lpa_units|k_al_rebuild_hot|k_diff|k_lpa_wave|k_lpa_rows" -d gpurun_out/${TAG}_pmc_lib_$c -o run --output-format csv -- python3 tools/pmc_workload.py gpurun_out/${TAG}_info.json > gpurun_out/${TAG}_pmc_lib_$c.log 2>&1 || { echo "lib pass $C failed"; tail -5 gpurun_out/${TAG}_pmc_lib_$c.log; exit 1; }
done
python3 tools/pmc_r02.py gpurun_out/${TAG} > gpurun_out/${TAG}_traffic.json && cat gpurun_out/${TAG}_traffic.json
