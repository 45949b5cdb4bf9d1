#!/bin/bash
# kernel trace of the C3 bench for each library in LIBS (paths; "A" = in-tree);
# prints the rows matching ROWS of the per-superstep dispatch table
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for L in $LIBS; do
  i=$((i+1))
  if [ "$L" = A ]; then unset LPA_LIB_PATH; else export LPA_LIB_PATH=$L; fi
  echo "== $L"
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/plib$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/plib$i.json 2> gpurun_out/plib$i.err || { tail -5 gpurun_out/plib$i.err; exit 1; }
  python3 tools/dispatch_table.py gpurun_out/plib$i/run_kernel_trace.csv | grep -E "${ROWS:-rebuild|^sum}" | cut -c1-110
done
