#!/bin/bash
# Same-box A/B of whole labelPropagation(10) calls (tools/run_ab.py: per-superstep
# medians, lpa_run(10) wall time, a label checksum that must match across variants).
#   CFGS="C3 C5"            configs, in order
#   ENVS="A=1;A=2 B=3"      variants (';' separates; an entry may set LPA_LIB_PATH=...)
#   K=7                     calls per variant
#   ROUNDS=1                alternate the variants this many times
# One JSON line per (config, variant, round) in gpurun_out/${TAG}_runab.jsonl.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-runab}
OUT=gpurun_out/${TAG}_runab.jsonl
IFS=';' read -ra VARS <<< "${ENVS:-LPA_NONE=0}"
for cfg in ${CFGS:-C3}; do
  for r in $(seq 1 ${ROUNDS:-1}); do
    for v in "${VARS[@]}"; do
      echo "== $cfg round $r: $v"
      env $v timeout -k 10 ${LIMIT:-300} python3 -u tools/run_ab.py "$cfg" "${K:-7}" "$v" >> "$OUT" 2> "gpurun_out/${TAG}_err.txt" \
        || { tail -20 "gpurun_out/${TAG}_err.txt"; exit 1; }
      tail -1 "$OUT"
    done
  done
done
exit 0
