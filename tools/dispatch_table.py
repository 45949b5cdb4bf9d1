"""Per-dispatch durations (ms) of the LPA kernels from a rocprofv3 kernel trace."""
import csv
import collections
import sys

path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
d = collections.defaultdict(list)
keys = ('k_lpa_seg', 'k_hub_small', 'k_hub_merge', 'k_lpa_hub_final', 'k_lpa_hub_write',
        'k_lpa_wave<8>', 'k_lpa_wave<4>', 'k_lpa_wave<2>', 'k_lpa_group<64>', 'k_lpa_group<32>',
        'k_lpa_group<16>', 'k_lpa_group<8>', 'k_lpa_group<4>', 'k_lpa_group<2>', 'k_lpa_group<1>',
        'k_diff', 'k_al_scatter', 'k_al_rebuild', 'k_lpa_iter1')
for r in rows:
    name = r['Kernel_Name']
    for k in keys:
        if k + '(' in name or (k in name and '<' not in k):
            d[k].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
            break
tot = None
for k in keys:
    if k in d:
        v = d[k]
        print(f"{k:18s}", ' '.join(f"{x:6.3f}" for x in v))
        tot = v if tot is None else [a + b for a, b in zip(tot, v)]
if tot:
    print(f"{'sum':18s}", ' '.join(f"{x:6.3f}" for x in tot))
