for o in 0 1 2 3; do
  echo "== order $o"
  ENVS="LPA_STREAM_ORDER=$o" bash tools/trace_env.sh > gpurun_out/so$o.txt || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/tenv.json'));print('value',d['value'],d['iteration_roofline']['iter_ms'][:3])"
  grep -E "hub_count|k_diff|rebuild|hub_final|group<1>" gpurun_out/so$o.txt
done
