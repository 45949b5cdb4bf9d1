cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/c2prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c2prof -o run --output-format csv -- python3 -u bench.py --config C2 --steps 2 --warmup 1 --no-quality --no-cpu-baseline --no-outlier > gpurun_out/c2prof/bench.json 2> gpurun_out/c2prof/bench.err || { tail -5 gpurun_out/c2prof/bench.err; exit 1; }
f=$(find gpurun_out/c2prof -name '*kernel_trace.csv' | head -1)
python3 tools/timeline2.py "$f" 21 22 23 24 25 26 27 > gpurun_out/c2prof/timeline.txt 2>&1
head -3 gpurun_out/c2prof/timeline.txt
