#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "quality or rmat_bit_exact or degree_mix or chunglu_heavy or sbm_bit" > gpurun_out/b2_tests.log 2>&1
rc=$?; tail -5 gpurun_out/b2_tests.log; [ $rc -ne 0 ] && exit $rc
TAG=b2 bash tools/r03_bench.sh
