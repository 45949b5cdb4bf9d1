#!/bin/bash
# PMC passes (one counter group per run) over the superstep kernels of a short C3 bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS="${BENCH_ARGS:---no-cpu-baseline --steps 3 --warmup 1}"
TAG=${TAG:-pmc}
i=0
while read -r COUNTERS; do
  [ -z "$COUNTERS" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $COUNTERS --kernel-include-regex "${KREGEX:-k_lpa|k_hub|k_diff|k_al}" -d gpurun_out/${TAG}_$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/${TAG}_${i}_bench.json 2> gpurun_out/${TAG}_${i}.err || { echo "pass $i failed"; tail -5 gpurun_out/${TAG}_${i}.err; exit 1; }
done <<'LIST'
FETCH_SIZE TCC_HIT_sum
TCC_MISS_sum WRITE_SIZE
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
LIST
echo done
