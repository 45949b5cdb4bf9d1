#!/bin/bash
# Ablations of the class-blocked rebuild's pieces phase (csrc/Makefile blktime blkabl):
# base, no label gathers (abl1), no stores (abl2), no column loads (abl3); per-block wall
# clock of the first call's superstep-1 rebuild (tools/blk_times.py).  CFG: C3 | C5.
cd "$GRAFT_REPO_ROOT" || exit 1
CFG=${CFG:-C3}
for v in "" abl1/ abl2/ abl3/; do
  n=${v%/}; n=${n:-base}
  LPA_LIB_PATH=tools/diag_lib/${v}liblpa_hip.so timeout -k 10 400 python3 tools/blk_times.py $CFG > gpurun_out/ablt_${CFG}_$n.json 2> gpurun_out/ablt_${CFG}_$n.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/ablt_${CFG}_$n.json')); c=d['call0']; print('$n', c['kernel_us'], [v['pieces_end_max'] for k,v in c['groups'].items()])"
done
