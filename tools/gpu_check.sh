#!/bin/bash
# parity tests, then a kernel-traced C3 bench; prints the per-dispatch table
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit $rc; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 150 rocprofv3 --kernel-trace -d gpurun_out/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_kt.json 2> gpurun_out/bench_kt.err
rc=$?
[ $rc -ne 0 ] && { tail -20 gpurun_out/bench_kt.err; exit $rc; }
cat gpurun_out/bench_kt.json
python3 tools/dispatch_table.py gpurun_out/kt/run_kernel_trace.csv
