"""Per-rank tally time of the partitioned path against the single-GPU handle
("per-rank tally time at P = 8 within 1.3x of single-GPU / 8").

Every kernel of the tally runs standalone: each handle is in the serialized profiling
schedule (lpa_set_serial, HIP events around every tally kernel) and the P ranks are
caller-driven handles stepped ONE AFTER ANOTHER from this thread (lpa_step needs no
collective there), the label exchange done by this script between supersteps with the
library's own delta / full protocol (lpa_exchange_get_delta / put_delta, or get / put
when a rank's changes exceed the delta capacity, as exchange_collective decides).
Frontier on (the shipped schedule).  Prints one JSON line.

    python tools/rank_tally.py [C3|C4|C5] [P]
"""
import json
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
import graphframes_amd as gfa  # noqa: E402
import torch  # noqa: E402

TALLY = ("k_lpa_units", "hub", "k_lpa_wave<16>", "k_lpa_wave<8>", "k_lpa_wave<4>", "k_lpa_wave<2>",
         "k_lpa_rows<64>", "k_lpa_rows<32>", "k_lpa_rows<16>", "k_lpa_rows<8>", "k_lpa_group<4>",
         "k_lpa_group<2>", "k_lpa_group<1>", "k_frontier_lists", "k_lpa_block")
MAX_ITER = 10

name = sys.argv[1] if len(sys.argv) > 1 else "C4"
P = int(sys.argv[2]) if len(sys.argv) > 2 else 8
src, dst, V = bench.make_edges(gfa, bench.CONFIGS[name], 0)


def tally_ms(st):
    return sum(st["kernel_ms"][k] for k in TALLY)


# ---- single GPU: supersteps 2..10, serialized after the column-run superstep 1 ----
with gfa.Graph(src, dst, V) as g:
    g.step(1)
    g.reset()
    g.step(1)
    g.set_serial(True)
    one = [g.step(1, stats=True) for _ in range(MAX_ITER - 1)]
    ref = g.labels()
torch.cuda.synchronize()
torch.cuda.empty_cache()
one_tally = [tally_ms(st) for st in one]

# ---- P caller-driven ranks, stepped in turn ----
ranks = [gfa.Graph(src, dst, V, rank=r, nranks=P) for r in range(P)]
del src, dst
torch.cuda.empty_cache()
dcap = max(1, ranks[0].info()["slice"] // 4)


def exchange():
    deltas = [g.exchange_get_delta() for g in ranks]
    if max(e.size for e in deltas) <= dcap:
        for g in ranks:
            g.exchange_put_delta(deltas)
        return "delta"
    # full: the deltas were only read; the slices are unchanged by get_delta
    full = np.concatenate([g.exchange_get() for g in ranks])
    for g in ranks:
        g.exchange_put(full)
    return "full"


per_rank = [[0.0] * (MAX_ITER - 1) for _ in range(P)]
conv_k = [dict() for _ in range(P)]   # per-kernel ms summed over the converged supersteps 5..10
modes = []
for g in ranks:
    g.step(1)   # superstep 1 (column runs; not serialized)
modes.append(exchange())
for g in ranks:
    g.set_serial(True)
for t in range(MAX_ITER - 1):
    for r, g in enumerate(ranks):
        st = g.step(1, stats=True)
        per_rank[r][t] = tally_ms(st)
        if t >= 3:
            for k in TALLY:
                conv_k[r][k] = conv_k[r].get(k, 0.0) + st["kernel_ms"][k]
    modes.append(exchange())
# every rank's replica equals the single-GPU labels after superstep 10
ok = all(np.array_equal(g.labels(), ref) for g in ranks)
for g in ranks:
    g.close()

one_sum = sum(one_tally)
rank_max = [max(per_rank[r][t] for r in range(P)) for t in range(MAX_ITER - 1)]
print(json.dumps(dict(
    config=name, P=P, labels_equal_single_gpu=ok, exchange_modes=modes,
    single_tally_ms_per_superstep=[round(x, 4) for x in one_tally],
    rank_max_tally_ms_per_superstep=[round(x, 4) for x in rank_max],
    single_tally_ms=round(one_sum, 4), single_over_P_ms=round(one_sum / P, 4),
    rank_max_tally_ms=round(sum(rank_max), 4),
    ratio_rank_max_over_single_div_P=round(sum(rank_max) / (one_sum / P), 3),
    per_rank_tally_ms=[round(sum(x), 4) for x in per_rank],
    # converged supersteps 5..10, per kernel: the single GPU and the slowest rank
    single_converged_kernel_ms={k: round(sum(st["kernel_ms"][k] for st in one[3:]), 4) for k in TALLY},
    rank_converged_kernel_ms={k: round(v, 4) for k, v in conv_k[max(range(P), key=lambda r: sum(per_rank[r][3:]))].items()})))
