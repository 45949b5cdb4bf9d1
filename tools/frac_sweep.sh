#!/bin/bash
# kernel-traced C3 bench at several al-rebuild thresholds (LPA_REBUILD_FRAC)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for f in ${FRACS:-0.25 0.7}; do
  LPA_REBUILD_FRAC=$f timeout -k 10 150 rocprofv3 --kernel-trace -d gpurun_out/frac_$f -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/frac_$f.json 2> gpurun_out/frac_$f.err || { tail -5 gpurun_out/frac_$f.err; exit 1; }
  echo "frac $f"; grep -o '"value": [0-9.]*' gpurun_out/frac_$f.json
  python3 tools/dispatch_table.py gpurun_out/frac_$f/run_kernel_trace.csv | grep "k_al\|k_diff\|sum"
done
