"""Per-kernel totals of every counter in a rocprofv3 --pmc counter_collection.csv,
one line per kernel: `pmc_dump.py file.csv [name-substring ...]` (no substrings:
every kernel, by the first 60 characters of its name)."""
import collections
import csv
import sys

path = sys.argv[1]
keys = sys.argv[2:]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if keys:
        for k in keys:
            if k in name:
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    else:
        agg[name[:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, " ".join(f"{c}={val:.4g}" for c, val in sorted(v.items())))
