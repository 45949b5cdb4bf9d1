#!/bin/bash
# kernel trace + L2 counters of the al rebuild kernels under $CMD
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-rb}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_tr -o run --output-format csv -- $CMD > gpurun_out/${TAG}_tr.json 2> gpurun_out/${TAG}_tr.err || { tail -5 gpurun_out/${TAG}_tr.err; exit 1; }
grep -E "rebuild" gpurun_out/${TAG}_tr/run_kernel_stats.csv | cut -d, -f1-8
KREGEX=k_al_rebuild CMD="$CMD" TAG=${TAG}_pmc tools/pmc_rebuild.sh | sort | uniq -c | sort -rn | head -8
