#!/bin/bash
# Round 3: the driver's bench command with per-phase progress on stderr (file under
# gpurun_out/), then a kernel trace of the default bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-b}
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err
rc=$?
cat gpurun_out/${TAG}_c3.json; tail -25 gpurun_out/${TAG}_c3.err
[ $rc -ne 0 ] && exit $rc
[ -n "$NO_PROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 -u bench.py --no-cpu-baseline --no-quality > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err
rc=$?
cat gpurun_out/${TAG}_prof.json; tail -5 gpurun_out/${TAG}_prof.err
exit $rc
