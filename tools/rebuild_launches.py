"""Durations of the al[] rebuild launches in a rocprofv3 kernel trace of bench.py: the
kernel is launched in every superstep's refresh but returns at once unless it rebuilds,
so the --stats average mixes no-op launches with real ones.  Classified by duration:
rebuilding launches of superstep 2 (bits mode) vs superstep 1 (labels mode, untimed).

    python tools/rebuild_launches.py run_kernel_trace.csv
"""
import csv
import statistics
import sys

d = []
for r in csv.DictReader(open(sys.argv[1])):
    if "k_al_rebuild_hot" in r["Kernel_Name"]:
        d.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
noop = [x for x in d if x < 0.1]
work = sorted(x for x in d if x >= 0.1)
# the two rebuilding launches of a call: superstep 1 (labels mode) is the longer one
split = (work[0] + work[-1]) / 2 if work else 0.0
ss2 = [x for x in work if x < split]
ss1 = [x for x in work if x >= split]
print(f"k_al_rebuild_hot launches: {len(d)} total, {len(noop)} no-op (< 0.1 ms, mean {statistics.mean(noop) if noop else 0:.4f} ms)")
if ss2:
    print(f"superstep-2 (bits mode, timed window): {len(ss2)} launches, mean {statistics.mean(ss2):.4f} ms, "
          f"median {statistics.median(ss2):.4f} ms")
if ss1:
    print(f"superstep-1 (labels mode, untimed): {len(ss1)} launches, mean {statistics.mean(ss1):.4f} ms")
