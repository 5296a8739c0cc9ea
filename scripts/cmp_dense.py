"""Dense-conv-path breakdown (level, conv, phase) of one or two per-layer reports
(bench.py --layer-report ..._per_layer.json): us per step and TB/s, side by side."""
import collections
import json
import re
import sys


def agg(path):
    a = collections.defaultdict(lambda: [0.0, 0.0])
    for r in json.load(open(path)):
        m = re.match(r"block_(\d)_\d\.(conv_[\d-]+)$", r["layer"])
        if m and int(m.group(1)) in (0, 1) and r["phase"] != "prelu":
            k = (m.group(1), m.group(2), r["phase"])
            a[k][0] += r["us"]
            a[k][1] += r["gbs"] * r["us"] * 1e-6
    return a


runs = [agg(p) for p in sys.argv[1:]]
keys = sorted(set().union(*[r.keys() for r in runs]))
tot = [[0.0, 0.0] for _ in runs]
for k in keys:
    cells = []
    for i, r in enumerate(runs):
        us, gb = r.get(k, (0.0, 0.0))
        tot[i][0] += us
        tot[i][1] += gb
        cells.append(f"{us:8.1f} us {gb / (us * 1e-6) / 1e3 if us else 0:5.2f} TB/s")
    print(f"L{k[0]} {k[1]:9s} {k[2]:7s} " + " | ".join(cells))
print("total          " + " | ".join(f"{u:8.1f} us {g / (u * 1e-6) / 8e3:.4f} of 8 TB/s" for u, g in tot))
