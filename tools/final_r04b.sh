#!/bin/bash
# Round-4 late evidence (after the tally rings; the -m gpu tests ran on the same library
# in the A/B call): the driver's bench command, the C3 bench under rocprofv3 (kernel trace
# + stats), the PMC traffic passes, then C2 / C4 / C5.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r04y}
echo "== driver command"
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_driver.json 2> gpurun_out/${TAG}_driver.err || { tail -5 gpurun_out/${TAG}_driver.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_driver.json')); print(d['value'], d['run_maxiter10_ms'], d['roofline']['frac'], d['iteration_roofline']['frac'], {k: v for k, v in d.items() if k.startswith('outlier_l') and k.endswith('ms')})"
TAG=$TAG STEPS="prof" bash tools/gpu_session.sh || exit 1
TAG=${TAG}_pmc bash tools/pmc_r03.sh > gpurun_out/${TAG}_pmc.out 2>&1; echo "pmc rc $?"
TAG=$TAG STEPS="c2 c4 c5" bash tools/gpu_session.sh || exit 1
exit 0
