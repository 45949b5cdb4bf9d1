#!/bin/bash
# kernel-traced C3 bench for the product build and each diagnostic ablation build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 2 3}; do
  if [ "$v" = 0 ]; then unset LPA_LIB_PATH; else export LPA_LIB_PATH=$GRAFT_REPO_ROOT/build/lpa_hip/diag$v/liblpa_hip.so; fi
  echo "=== variant $v"
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/diag_kt$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/diag$v.json 2> gpurun_out/diag$v.err || { tail -5 gpurun_out/diag$v.err; exit 1; }
  python3 tools/dispatch_table.py gpurun_out/diag_kt$v/run_kernel_trace.csv
done
