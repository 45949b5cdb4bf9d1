#!/bin/bash
# Round 3: the driver's exact bench command, then the same under a kernel + copy trace
# (outlier L2 leg investigation).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/l2_driver.json 2> gpurun_out/l2_driver.err || { tail -20 gpurun_out/l2_driver.err; exit 1; }
cat gpurun_out/l2_driver.json
timeout -k 10 300 python3 -u tools/outlier_prof.py C3 > gpurun_out/l2_outlier_prof.txt 2>&1 || { tail -20 gpurun_out/l2_outlier_prof.txt; exit 1; }
cat gpurun_out/l2_outlier_prof.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/l2_prof -o run --output-format csv -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/l2_prof.json 2> gpurun_out/l2_prof.err || { tail -20 gpurun_out/l2_prof.err; exit 1; }
cat gpurun_out/l2_prof.json
