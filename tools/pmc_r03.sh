#!/bin/bash
# Round-3 HBM traffic per launch (MI355X guide, HBM section): FETCH_SIZE and WRITE_SIZE
# in separate rocprofv3 --pmc passes (kernel trace only) over tools/pmc_workload3.py;
# the read factor (2.0 for 4 B/lane streams) is the round-2 calibration
# (profiles/r02/traffic/pmc_traffic.json).  Output: gpurun_out/${TAG}_traffic.json
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-pmc3}
for C in FETCH_SIZE WRITE_SIZE; do
  c=$(echo $C | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_lpa_units|k_al_rebuild_hot|k_abits_pass|k_first_runs" -d gpurun_out/${TAG}_pmc_lib_$c -o run --output-format csv -- python3 tools/pmc_workload3.py gpurun_out/${TAG}_info.json > gpurun_out/${TAG}_pmc_lib_$c.log 2>&1 || { echo "lib pass $C failed"; tail -5 gpurun_out/${TAG}_pmc_lib_$c.log; exit 1; }
done
python3 tools/pmc_r03.py gpurun_out/${TAG} > gpurun_out/${TAG}_traffic.json && cat gpurun_out/${TAG}_traffic.json
