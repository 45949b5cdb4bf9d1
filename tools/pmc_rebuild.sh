#!/bin/bash
# L2 hit rate and memory-side fetches of the al rebuild: one --pmc pass per group,
#   CMD="python3 bench.py --no-cpu-baseline" TAG=x tools/pmc_rebuild.sh
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-pr}; KREGEX=${KREGEX:-k_al_rebuild}
i=0
while read -r COUNTERS; do
  [ -z "$COUNTERS" ] && continue
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $COUNTERS --kernel-include-regex "$KREGEX" -d gpurun_out/${TAG}_$i -o run --output-format csv -- $CMD > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { echo "pass $i failed"; tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
done <<'LIST'
TCC_HIT_sum TCC_MISS_sum
FETCH_SIZE
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
LIST
python3 tools/pmc_dispatch.py "gpurun_out/${TAG}_*" > gpurun_out/${TAG}_table.txt
cat gpurun_out/${TAG}_table.txt
