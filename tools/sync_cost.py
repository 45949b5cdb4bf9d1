"""Workload + analysis for the cost of the per-superstep host read in the P > 1 exchange
(lpa_exchange.hip exchange_collective: the (delta, giant) count pairs are read on the
host to size the allgather).  Runs labelPropagation(10) calls of a ONE-RANK RCCL job
(the distributed path with its ncclAllGather and host read; the one-GPU box allows no
second rank) on a bench config; under rocprofv3 --kernel-trace the analysis step then
measures, per superstep, the GPU idle gap between k_split_counts (the last kernel before
the read) and the next kernel, against the superstep's span.

    python tools/sync_cost.py run C3          (the workload)
    python tools/sync_cost.py analyze <kernel_trace.csv>
"""
import csv
import json
import re
import statistics
import sys

if sys.argv[1] == "run":
    sys.path.insert(0, ".")
    import bench  # noqa: E402
    import graphframes_amd as gfa  # noqa: E402
    import torch  # noqa: E402

    cfg = bench.CONFIGS[sys.argv[2]]
    src, dst, V = bench.make_edges(gfa, cfg, 0)
    g = gfa.Graph(src, dst, V, rank=0, nranks=1, comm_id=gfa.comm_unique_id())
    del src, dst
    torch.cuda.empty_cache()
    for _ in range(4):
        g.run(10)
    torch.cuda.synchronize()
    g.close()
    sys.exit(0)

rows = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    m = re.search(r"(k_[A-Za-z0-9_]+)", n)
    return m.group(1) if m else n[:24]


gaps, spans, starts = [], [], []
last_split_end = None
ss_start = None
calls = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == "k_first_runs"]
seg = rows[calls[-2]:calls[-1]] if len(calls) > 1 else rows
for i, r in enumerate(seg):
    k = short(r["Kernel_Name"])
    if last_split_end is not None:
        gaps.append((int(r["Start_Timestamp"]) - last_split_end) / 1e3)
        last_split_end = None
    if k == "k_split_counts":
        last_split_end = int(r["End_Timestamp"])
    if k == "k_frontier_lists":
        if ss_start is not None:
            spans.append((int(r["Start_Timestamp"]) - ss_start) / 1e3)
        ss_start = int(r["Start_Timestamp"])
        starts.append(ss_start)


def idle_us(t0, t1):
    """time in [t0, t1) with no kernel of the trace running (copies count as idle)"""
    iv = sorted((max(int(r["Start_Timestamp"]), t0), min(int(r["End_Timestamp"]), t1)) for r in seg
                if int(r["End_Timestamp"]) > t0 and int(r["Start_Timestamp"]) < t1)
    busy, cur_s, cur_e = 0, None, None
    for a, b in iv:
        if cur_e is None or a > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    if cur_e is not None:
        busy += cur_e - cur_s
    return (t1 - t0 - busy) / 1e3


idles = [idle_us(a, b) for a, b in zip(starts, starts[1:])]
conv = spans[4:] if len(spans) > 4 else spans
conv_idle = idles[4:] if len(idles) > 4 else idles
print(json.dumps({
    "what": "one-rank RCCL job, the last full labelPropagation(10) call of the trace: GPU idle gap between "
            "k_split_counts and the next kernel (the host read of the count pairs) per superstep, and the "
            "superstep spans (k_frontier_lists to k_frontier_lists)",
    "gaps_us": [round(x, 1) for x in gaps],
    "superstep_spans_us": [round(x, 1) for x in spans],
    "median_gap_us": round(statistics.median(gaps), 1) if gaps else None,
    "median_converged_span_us": round(statistics.median(conv), 1) if conv else None,
    "gap_over_converged_span": round(statistics.median(gaps) / statistics.median(conv), 3) if gaps and conv else None,
    "superstep_idle_us": [round(x, 1) for x in idles],
    "median_converged_idle_us": round(statistics.median(conv_idle), 1) if conv_idle else None,
    "converged_idle_fraction": round(statistics.median(conv_idle) / statistics.median(conv), 3)
    if conv_idle and conv else None,
}, indent=1))
