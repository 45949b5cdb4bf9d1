#!/bin/bash
# One GPU call: parity tests -> kernel-trace+stats profile of the C3 bench ->
# plain C3 bench with the CPU baseline.  Every GPU step has its own time limit
# and the chain stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-run}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_tests.log | head -20; exit $rc; }
[ -n "$TESTS_ONLY" ] && exit 0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_bench_prof.json 2> gpurun_out/${TAG}_bench_prof.err
rc=$?
[ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_bench_prof.err; exit $rc; }
cat gpurun_out/${TAG}_bench_prof.json
python3 tools/dispatch_table.py gpurun_out/${TAG}_prof/run_kernel_trace.csv > gpurun_out/${TAG}_dispatch.txt
cat gpurun_out/${TAG}_dispatch.txt
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python3 -u bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?
cat gpurun_out/${TAG}_bench.json
[ $rc -ne 0 ] && tail -20 gpurun_out/${TAG}_bench.err
exit $rc
