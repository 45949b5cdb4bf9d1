"""Reads the rocprofv3 kernel trace of tools/rank_refresh.py: the refresh groups (from
k_giant_pick through the rebuild / code kernels that follow it) in trace order, their
summed kernel durations, and the single-GPU vs per-rank figures.  One JSON line.

    python tools/refresh_trace.py DIR P REPS
"""
import csv
import glob
import json
import statistics
import sys

d, P, REPS = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
GROUP = ("k_giant_pick", "k_giant_bits", "k_code_mode", "k_al_rebuild_hot", "k_code_build", "k_code_rebuild",
         "k_al_rebuild")
groups, cur = [], None
for s, e, n in rows:
    base = n.replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].replace("void ", "").strip()
    base = base.split("::")[-1]
    if base == "k_giant_pick":
        cur = {"total_ms": 0.0, "kernels": {}}
        groups.append(cur)
    if cur is not None and base in GROUP:
        ms = (e - s) / 1e6
        cur["total_ms"] += ms
        cur["kernels"][base] = round(cur["kernels"].get(base, 0.0) + ms, 4)
    elif cur is not None and base not in GROUP:
        cur = None
# layout (tools/rank_refresh.py): the single handle's build refresh, REPS superstep-1
# refreshes, one superstep-2 refresh; the P rank handles' build refreshes, REPS x P
# superstep-1 refreshes (rank order), P superstep-2 refreshes
single = groups[1:1 + REPS]
r0 = 1 + REPS + 1 + P
ranks = groups[r0:r0 + REPS * P]
assert len(groups) == r0 + REPS * P + P, (len(groups), r0 + REPS * P + P)
per_rank = [statistics.median(ranks[k * P + r]["total_ms"] for k in range(REPS)) for r in range(P)]
one = statistics.median(g["total_ms"] for g in single)
print(json.dumps(dict(
    groups_found=len(groups), single_gpu_refresh_ms=round(one, 4), single_gpu_kernels=single[-1]["kernels"],
    per_rank_refresh_ms=[round(x, 4) for x in per_rank], rank_max_refresh_ms=round(max(per_rank), 4),
    single_over_P_ms=round(one / P, 4), ratio_rank_max_over_single_div_P=round(max(per_rank) / (one / P), 3),
    rank_kernels_last_rep=[ranks[(REPS - 1) * P + r]["kernels"] for r in range(P)])))
