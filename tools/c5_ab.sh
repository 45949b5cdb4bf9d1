#!/bin/bash
# C5 runs under a list of environment settings:  SETTINGS="LPA_WARM=-1 LPA_WARM=4000000" tools/c5_ab.sh
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-c5ab}; i=0
for E in $SETTINGS; do
  i=$((i+1))
  env $E timeout -k 10 200 python3 -u tools/c5_run.py ${C5_ARGS} > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$i.json'));print('$E', d['gteps'], d['iter_ms'][:3], d['iter_ms'][-1])"
done
