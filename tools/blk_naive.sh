#!/bin/bash
# The piece machinery on a plain access pattern (LPA_BLOCK_NAIVE=1: aligned 64-arc pieces,
# contiguous per class) against the class-blocked pieces, per-block wall clock
# (tools/blk_times.py, diagnostic build tools/diag_lib/).
cd "$GRAFT_REPO_ROOT" || exit 1
for cfg in C3 C5; do
  for mode in blocked naive; do
    env LPA_BLOCK_MIN_SLOTS=0 $( [ $mode = naive ] && echo LPA_BLOCK_NAIVE=1 ) LPA_LIB_PATH=tools/diag_lib/liblpa_hip.so \
      timeout -k 10 400 python3 tools/blk_times.py $cfg > gpurun_out/naive_${cfg}_$mode.json 2> gpurun_out/naive_${cfg}_$mode.err || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/naive_${cfg}_$mode.json')); c=d['call0']; print('$cfg $mode', d['info'], c['kernel_us'], [(v['pieces_end_max'], v['end_max']) for k,v in c['groups'].items()])"
  done
done
