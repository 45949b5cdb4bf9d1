#!/bin/bash
# SQ counters of the tally kernels (supersteps 1-2 of CFG, default C3; RX overrides the kernel
# filter), two passes + a kernel trace; outputs under gpurun_out/${TAG:-sqt}*.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
RX="${RX:-k_lpa_wave|k_lpa_rows|k_lpa_group|k_hub|k_units|k_first_runs}"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
  --kernel-include-regex "$RX" -d gpurun_out/${TAG:-sqt}1 -o run --output-format csv \
  -- python3 tools/pmc_sq_tally.py ${CFG:-C3} > gpurun_out/${TAG:-sqt}1.log 2>&1 || { echo "pass 1 failed"; tail -5 gpurun_out/${TAG:-sqt}1.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE \
  --kernel-include-regex "$RX" -d gpurun_out/${TAG:-sqt}2 -o run --output-format csv \
  -- python3 tools/pmc_sq_tally.py ${CFG:-C3} > gpurun_out/${TAG:-sqt}2.log 2>&1 || { echo "pass 2 failed"; tail -5 gpurun_out/${TAG:-sqt}2.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "$RX" -d gpurun_out/${TAG:-sqt}0 -o run --output-format csv \
  -- python3 tools/pmc_sq_tally.py ${CFG:-C3} > gpurun_out/${TAG:-sqt}0.log 2>&1 || { echo "trace failed"; exit 1; }
echo done
