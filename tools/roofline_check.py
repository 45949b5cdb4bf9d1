"""Cross-check of bench.py's roofline leg against the rocprofv3 kernel trace of the
same command: the dominant kernel's average duration over the dispatches of the
breakdown pass (standalone, serialized) -- dispatch order per superstep-launched
kernel: prime (1), warmup (W), timed (K), warmup (W), breakdown (K), warmup (W),
concurrent stats (K).   python tools/roofline_check.py trace.csv bench.json"""
import csv
import json
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
b = json.load(open(sys.argv[2]))
k = b["roofline"]["kernel"]
W, K = b["warmup"], b["steps"]
pat = re.compile(r'(k_[A-Za-z0-9_]+(<[^>]*>)?)')
durs = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in rows
        if (m := pat.search(r['Kernel_Name'])) and m.group(1) == k]
lo = 1 + W + K + W
sel = durs[lo:lo + K]
avg = sum(sel) / len(sel)
print(f"kernel {k}: {len(durs)} dispatches in the trace; breakdown-pass dispatches {lo}..{lo + K - 1}")
print(f"  trace average {avg:.4f} ms vs bench avg_launch_ms {b['roofline']['avg_launch_ms']:.4f} ms "
      f"(ratio {avg / b['roofline']['avg_launch_ms']:.3f}); per dispatch: " + " ".join(f"{d:.3f}" for d in sel))
print(f"  achieved from the trace: {b['roofline']['bytes_per_launch'] / (avg * 1e-3) / 1e9:.1f} GB/s "
      f"(bench: {b['roofline']['achieved']} GB/s, peak {b['roofline']['peak']})")
