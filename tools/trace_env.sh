#!/bin/bash
# kernel trace of the C3 bench under the environment in ENVS (e.g. "X=1"), then the
# timeline of superstep STEP (index of the k_lpa_units dispatch, default 2 = timed superstep 2)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
[ -n "$ENVS" ] && export $ENVS
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tenv -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/tenv.json 2> gpurun_out/tenv.err || { tail -5 gpurun_out/tenv.err; exit 1; }
python3 tools/timeline.py gpurun_out/tenv/run_kernel_trace.csv ${STEP:-2}
