set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "frontier or rmat or c3 or schedule or hub" > gpurun_out/ab4_tests.log 2>&1 || { tail -30 gpurun_out/ab4_tests.log; exit 1; }
tail -2 gpurun_out/ab4_tests.log
TAG=ab4 ENVS="LPA_BLOCK_AT=0;LPA_BLOCK_AT=4;LPA_BLOCK_AT=0;LPA_BLOCK_AT=4" bash tools/bench_env_ab.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab4_prof -o run -- python3 bench.py --no-cpu-baseline --no-outlier --steps 2 > gpurun_out/ab4_prof.json 2> gpurun_out/ab4_prof.err
