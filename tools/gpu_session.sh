#!/bin/bash
# One GPU session: the -m gpu tests, then the bench configs and profiles named in
# STEPS (space-separated, in order; default "tests c3"):
#   tests     pytest -m gpu (FILES, PER_TEST as tools/gpu_tests.sh)
#   c3        bench.py default (C3, CPU baseline, outlier, quality)
#   drv       the driver's command (bench.py --gpus 1 --steps 20 --warmup 5)
#   c3q       bench.py C3 without the CPU baseline, outlier and quality
#   c2 / c4 / c5   bench.py --config C2 / C4 / C5 (no CPU baseline, outlier or quality)
#   prof      rocprofv3 kernel trace + stats of the C3 bench (no CPU baseline)
#   prof5     the same for C5 (2 timed calls)
#   outprof   rocprofv3 kernel trace + stats of tools/outlier_prof.py C3
#   tally     tools/rank_tally.py C4 8 (per-rank tally time, caller-driven ranks)
# Outputs land in gpurun_out/${TAG}_*; every GPU step has its own time limit and the
# chain stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-s}
STEPS=${STEPS:-"tests c3"}
bench() {  # name limit args...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" python3 -u bench.py "$@" > "gpurun_out/${TAG}_$n.json" 2> "gpurun_out/${TAG}_$n.err"
  local rc=$?
  [ $rc -ne 0 ] && { tail -20 "gpurun_out/${TAG}_$n.err"; exit $rc; }
  python3 - "gpurun_out/${TAG}_$n.json" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
ir = d.get("iteration_roofline", {})
print(sys.argv[1], "value", d["value"], "ms/step", d["ms_per_step"], "per-superstep",
      d["baseline_method"]["median_ms_per_superstep_2_to_10"], "run10", d["run_maxiter10_ms"],
      "ss1", ir.get("whole_call", {}).get("superstep1_ms"), "full-work frac", ir.get("frac"),
      "outlier", {k: v for k, v in d.items() if k.startswith("outlier_l") and k.endswith("ms")})
EOF
}
for st in $STEPS; do
  echo "== $st"
  case $st in
    tests) TAG=$TAG LIMIT=${LIMIT:-600} PER_TEST=${PER_TEST:-300} bash tools/gpu_tests.sh || exit 1 ;;
    c3) bench c3 400 ;;
    drv) bench drv 500 --gpus 1 --steps 20 --warmup 5 ;;   # the driver's command
    c3q) bench c3q 300 --no-cpu-baseline --no-outlier --no-quality ;;
    c2) bench c2 300 --config C2 --no-cpu-baseline --no-outlier --no-quality ;;
    c4) bench c4 400 --config C4 --no-cpu-baseline --no-outlier --no-quality --steps 3 ;;
    c5) bench c5 400 --config C5 --no-cpu-baseline --no-outlier --no-quality --steps 3 ;;
    prof5)
      cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
      timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "gpurun_out/${TAG}_prof5" -o run --output-format csv \
        -- python3 bench.py --config C5 --no-cpu-baseline --no-outlier --no-quality --steps 2 --warmup 1 \
        > "gpurun_out/${TAG}_prof5.json" 2> "gpurun_out/${TAG}_prof5.err" || exit 1 ;;
    prof|outprof)
      cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
      if [ $st = prof ]; then
        timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "gpurun_out/${TAG}_prof" -o run --output-format csv \
          -- python3 bench.py --no-cpu-baseline --no-quality > "gpurun_out/${TAG}_prof.json" 2> "gpurun_out/${TAG}_prof.err" || exit 1
      else
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/${TAG}_outprof" -o run --output-format csv \
          -- python3 tools/outlier_prof.py C3 > "gpurun_out/${TAG}_outprof.txt" 2>&1 || exit 1
        grep -E "^L[12] " "gpurun_out/${TAG}_outprof.txt"
      fi ;;
    tally) timeout -k 10 400 python3 -u tools/rank_tally.py C4 8 > "gpurun_out/${TAG}_tally.json" 2> "gpurun_out/${TAG}_tally.err" || exit 1
           cat "gpurun_out/${TAG}_tally.json" ;;
    refresh)   # per-rank superstep-1 refresh at C4 / P = 8 against the single GPU (kernel trace)
      cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
      timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/${TAG}_rr" -o run \
        -- python3 tools/rank_refresh.py C4 8 > "gpurun_out/${TAG}_rr_run.json" 2> "gpurun_out/${TAG}_rr.err" || exit 1
      python3 tools/refresh_trace.py "gpurun_out/${TAG}_rr" 8 3 > "gpurun_out/${TAG}_rr.json" || exit 1
      cat "gpurun_out/${TAG}_rr_run.json" "gpurun_out/${TAG}_rr.json" ;;
    conv)   # kernel trace of C3's timed calls (tools/step_trace.py): converged-superstep timelines
      cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/${TAG}_conv" -o run \
        -- python3 tools/step_trace.py ${CONV_CFG:-C3} > "gpurun_out/${TAG}_conv.txt" 2>&1 || exit 1
      f=$(ls gpurun_out/${TAG}_conv/*/*kernel_trace.csv gpurun_out/${TAG}_conv/*kernel_trace.csv 2>/dev/null | head -1)
      python3 tools/timeline2.py "$f" > "gpurun_out/${TAG}_conv_timeline.txt" || exit 1
      head -3 "gpurun_out/${TAG}_conv_timeline.txt" ;;
    ab)   # bench A/B of the default library against VLIB (LPA_LIB_PATH) on CONFIGS (default "C3 C5")
      for c in ${CONFIGS:-C3 C5}; do
        for v in default variant; do
          if [ $v = default ]; then
            timeout -k 10 400 python3 -u bench.py --config $c --no-cpu-baseline --no-outlier --no-quality --steps 5 \
              > "gpurun_out/${TAG}_ab_${c}_$v.json" 2> "gpurun_out/${TAG}_ab_${c}_$v.err" || exit 1
          else
            LPA_LIB_PATH="$VLIB" timeout -k 10 400 python3 -u bench.py --config $c --no-cpu-baseline --no-outlier \
              --no-quality --steps 5 > "gpurun_out/${TAG}_ab_${c}_$v.json" 2> "gpurun_out/${TAG}_ab_${c}_$v.err" || exit 1
          fi
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['run_maxiter10_ms'], d['baseline_method']['median_ms_per_superstep_2_to_10'])" "gpurun_out/${TAG}_ab_${c}_$v.json"
        done
      done ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
exit 0
