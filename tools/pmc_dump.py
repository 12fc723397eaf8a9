"""Per-kernel totals of every counter in a rocprofv3 --pmc counter_collection.csv
(flash-attention kernels by default), one line per kernel."""
import collections
import csv
import sys

path = sys.argv[1]
keys = sys.argv[2:] or ["fa_fwd", "fa_bwd_dkdv", "fa_bwd_dq", "fa_bwd_pre"]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(path)):
    for k in keys:
        if k in r["Kernel_Name"]:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, " ".join(f"{c}={val:.4g}" for c, val in sorted(v.items())))
