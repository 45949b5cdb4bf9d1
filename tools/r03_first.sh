#!/bin/bash
# Round 3 first GPU call: the full -m gpu suite, then the outlier-L2 probe.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=r03a LIMIT=600 PER_TEST=300 bash tools/gpu_tests.sh || exit 1
bash tools/r03_l2probe.sh
