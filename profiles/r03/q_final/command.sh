cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fin3
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/fin3/bench_c3_driver_cmd.json 2> gpurun_out/fin3/bench_c3_driver_cmd.progress.txt || { tail -5 gpurun_out/fin3/bench_c3_driver_cmd.progress.txt; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/fin3/bench_c3_driver_cmd.json'));print('C3', d['value'], d['call_ms_min_median_max'], d['baseline_method']['median_ms_per_superstep_2_to_10'], d['run_maxiter10_ms'], d['roofline']['frac'], d['outlier_l1_ms'], d['outlier_l2_ms'], d['cpu_baseline']['value'])"
