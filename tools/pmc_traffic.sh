#!/bin/bash
# HBM traffic of the bench's tally kernels (k_lpa_*) and of a known-bytes
# calibration kernel (k_diff: int4 streams of exactly 2 x 4 vpad bytes), per the
# MI355X guide's HBM/rocprofv3 recipe: FETCH_SIZE and WRITE_SIZE in separate --pmc
# passes (TCC budget), no trace domains.  Output: gpurun_out/${TAG}_pmc_{fetch,write}/
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-traffic}
for C in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/${TAG}_pmc_$(echo $C | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "k_lpa_|k_diff" -d $d -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > $d.json 2> $d.err || { echo "pass $C failed"; tail -5 $d.err; exit 1; }
done
python3 tools/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write gpurun_out/${TAG}_pmc_fetch.json > gpurun_out/${TAG}_traffic.json
cat gpurun_out/${TAG}_traffic.json
