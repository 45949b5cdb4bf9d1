for v in "" abl1/ abl2/ abl3/; do
  n=${v%/}; n=${n:-base}
  LPA_LIB_PATH=tools/diag_lib/${v}liblpa_hip.so timeout -k 10 200 python3 tools/blk_times.py C3 > gpurun_out/ablt_$n.json 2> gpurun_out/ablt_$n.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/ablt_$n.json')); print('$n', d['call1']['kernel_us'], [v['pieces_end_max'] for k,v in d['call1']['groups'].items()])"
done
