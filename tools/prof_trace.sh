#!/bin/bash
# kernel-trace + stats pass over the C3 bench (no CPU baseline); writes gpurun_out/prof_kt
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 9 --warmup 1 > gpurun_out/prof_kt_bench.json
