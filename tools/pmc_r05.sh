#!/bin/bash
# Round-5 HBM traffic per launch (MI355X guide, HBM section) of one bench config (CFG,
# default C3): FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes (kernel
# trace only) over tools/pmc_workload5.py; the read factor is the round-2 calibration
# (profiles/r02/traffic/pmc_traffic.json), applied here by tools/pmc_r05.py after the merge.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-pmc5}
CFG=${CFG:-C3}
RX="k_first_runs|k_al_rebuild_hot|k_code_rebuild|k_code_build|k_code_settle|k_lpa_units|k_hub_bucket|k_hub_scatter|k_lpa_block|k_lpa_wave|k_abits_pass|k_giant_pick"
for C in FETCH_SIZE WRITE_SIZE; do
  c=$(echo $C | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL ${LIMIT:-400} rocprofv3 --pmc $C --kernel-include-regex "$RX" -d gpurun_out/${TAG}_$c -o run --output-format csv -- python3 tools/pmc_workload5.py $CFG gpurun_out/${TAG}_info.json > gpurun_out/${TAG}_$c.log 2>&1 || { echo "pass $C failed"; tail -5 gpurun_out/${TAG}_$c.log; exit 1; }
done
# the byte model runs where the round-2 calibration lives (it does not travel):
#   python3 tools/pmc_r05.py gpurun_out/${TAG} $CFG > profiles/r05/traffic/pmc_traffic_$CFG.json
exit 0
