#!/bin/bash
# Bench sweep on one GPU: default bench (C3, N = 1, CPU baseline + outlier), then
# --config C2 / C5, then a rocprofv3 kernel-trace + stats pass of the default bench.
# Each GPU step has its own limit; the chain stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-bench}
run() {  # name limit args...
  local n=$1 l=$2; shift 2
  timeout -k 10 $l python3 -u bench.py "$@" > gpurun_out/${TAG}_$n.json 2> gpurun_out/${TAG}_$n.err
  local rc=$?
  cat gpurun_out/${TAG}_$n.json
  [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_$n.err; exit $rc; }
  return 0
}
run c3 400 ${BENCH_ARGS}
[ -n "$ONLY_C3" ] && exit 0
run c2 200 --config C2 --no-cpu-baseline
run c5 400 --config C5 --no-cpu-baseline --no-outlier --steps 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-outlier > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err
rc=$?
[ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_prof.err; exit $rc; }
cat gpurun_out/${TAG}_prof.json
exit 0
