#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-b3}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/${TAG}_tests.log | head -20; exit $rc; }
TAG=$TAG bash tools/r03_bench.sh
