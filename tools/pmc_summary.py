"""Aggregate rocprofv3 --pmc counter_collection.csv per kernel (substring match)."""
import collections, csv, sys
path = sys.argv[1]
keys = sys.argv[2:] or ["fa_fwd", "fa_bwd_dkdv", "fa_bwd_dq"]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(path)):
    for k in keys:
        if k in r["Kernel_Name"]:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    wc = v.get("SQ_WAVE_CYCLES", 0) or 1
    extra = ""
    if "SQ_WAIT_ANY" in v:
        extra = (f" wait={v['SQ_WAIT_ANY'] / wc:.0%} stall={v.get('SQ_WAIT_INST_ANY', 0) / wc:.0%} "
                 f"active={v.get('SQ_ACTIVE_INST_ANY', 0) / wc:.0%}")
    if v.get("SQ_LDS_IDX_ACTIVE"):
        extra += f" lds_conflict={v.get('SQ_LDS_BANK_CONFLICT', 0) / v['SQ_LDS_IDX_ACTIVE']:.0%}"
    print(k + extra)
