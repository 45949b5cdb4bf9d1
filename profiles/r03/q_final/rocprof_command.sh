cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fin3p
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/fin3p -o run --output-format csv -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-outlier --no-cpu-baseline > gpurun_out/fin3p/bench_c3_under_rocprof.json 2> gpurun_out/fin3p/err.txt || { tail -5 gpurun_out/fin3p/err.txt; exit 1; }
f=$(find gpurun_out/fin3p -name '*kernel_trace.csv' | head -1); python3 tools/rebuild_launches.py "$f" > gpurun_out/fin3p/rebuild_launches.txt 2>&1; rm -f "$f"; head -5 gpurun_out/fin3p/rebuild_launches.txt
