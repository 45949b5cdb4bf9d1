#!/bin/bash
# rocprofv3 kernel trace + stats of the C3 bench (no CPU baseline / outlier), then
# the per-superstep dispatch table; outputs under gpurun_out/${TAG}_prof*.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-prof}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-outlier ${BENCH_ARGS} > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err
rc=$?
[ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_prof.err; exit $rc; }
cat gpurun_out/${TAG}_prof.json
exit 0
