#!/bin/bash
# A/B of HIP runtime graph-launch settings on the timed call (tools/step_trace.py, C3),
# plus the host enqueue timing of the default.  Every run under its own time limit.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
LPA_HOST_TIMING=1 timeout -k 10 200 python3 tools/step_trace.py > gpurun_out/ht1.log 2>&1 || exit 1
tail -13 gpurun_out/ht1.log
for v in "X=0" "LPA_CONV_STREAMS=1" "LPA_GRAPHS=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" \
         "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "X=1"; do
  echo "== $v"
  env $v timeout -k 10 200 python3 tools/step_trace.py > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  grep "step(9)" gpurun_out/ab.log | tr '\n' ' '; echo
done
