cd "$GRAFT_REPO_ROOT" || exit 1
TAG=c2 CFG=C2 N=5 bash tools/pmc_dense.sh > /dev/null; rc=$?; grep -E "superstep|k_lpa_rows|k_al_rebuild|k_diff" gpurun_out/c2_dense.txt | head -40; exit $rc
