"""Counter validation of the HIP bandwidth probes (BASELINE.json: "hand-written
HIP bandwidth-probe kernel tuned for gfx950 (LDS-staged, validated with
rocprof counters)").

Driver mode (run under rocprofv3 --pmc):
    python tools/probe_pmc.py run [--mib 1024] [--iters 4]
runs kgwe_probe_hbm once: each of copy / read / write / LDS-staged pull is
dispatched 2 (warm-up) + iters times over a buffer of --mib MiB (4x the
256 MiB Infinity Cache, so L2/MALL misses reach HBM).

Summary mode:
    python tools/probe_pmc.py summarize <fetch.csv> <write.csv> <sq.csv> [--mib 1024]
compares the bytes each kernel dispatch SHOULD move (read n*16 B, write n*16 B
per element pass) with TCC FETCH_SIZE / WRITE_SIZE (KiB, L2 <-> memory fabric)
and reports LDS instruction / bank-conflict counts of the LDS-staged kernel.
"""
from __future__ import annotations

import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

KERNELS = {"copy_kernel": (1, 1), "read_kernel": (1, 0), "write_kernel": (0, 1),
           "lds_pull_kernel": (1, 1)}  # (read passes, write passes) over the buffer


def run(mib: int, iters: int) -> None:
    from kgwe.agent import probes

    r = probes.probe_hbm(0, mib << 20, iters)
    print(json.dumps({"mib": mib, "iters": iters, "copy_gbps": r.copy_gbps, "read_gbps": r.read_gbps,
                      "write_gbps": r.write_gbps, "lds_copy_gbps": r.lds_copy_gbps}), flush=True)


def per_dispatch(path: str) -> dict:
    """kernel -> counter -> list of per-dispatch values."""
    vals = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"]
        k = next((k for k in KERNELS if k in name), None)
        if k is None:
            continue
        disp = row.get("Dispatch_Id") or row.get("Correlation_Id") or "0"
        vals[k][row["Counter_Name"]][disp] += float(row["Counter_Value"])
    return {k: {c: list(d.values()) for c, d in cs.items()} for k, cs in vals.items()}


def summarize(fetch_csv: str, write_csv: str, sq_csv: str, raw_csv: str | None, mib: int) -> str:
    f, w, s = per_dispatch(fetch_csv), per_dispatch(write_csv), per_dispatch(sq_csv)
    raw = per_dispatch(raw_csv) if raw_csv else {}
    buf = mib * 2**20
    lines = ["| kernel | dispatches | expected read MiB | FETCH_SIZE MiB | ratio | expected write MiB | "
             "WRITE_SIZE MiB | ratio |", "|---|---:|---:|---:|---:|---:|---:|---:|"]
    for k, (rp, wp) in KERNELS.items():
        fe = f.get(k, {}).get("FETCH_SIZE", [])
        wr = w.get(k, {}).get("WRITE_SIZE", [])
        if not fe and not wr:
            continue
        mf = sum(fe) / len(fe) / 1024 if fe else float("nan")  # KiB -> MiB, mean per dispatch
        mw = sum(wr) / len(wr) / 1024 if wr else float("nan")
        er, ew = rp * buf / 2**20, wp * buf / 2**20
        rr = f"{mf / er:.3f}" if er else "-"
        rw = f"{mw / ew:.3f}" if ew else "-"
        lines.append(f"| `{k}` | {len(fe) or len(wr)} | {er:.0f} | {mf:.1f} | {rr} | {ew:.0f} | {mw:.1f} | {rw} |")
    if raw:
        # gfx950: the FETCH_SIZE expression counts 128-B reads through
        # TCC_BUBBLE; the 128-B EA read request counter is TCC_EA0_RDREQ_128B.
        lines += ["", "Read bytes from the raw TCC->EA request counts (128 B x RDREQ_128B + 32 B x "
                  "RDREQ_32B + 64 B x the rest):", "",
                  "| kernel | RDREQ | RDREQ_32B | RDREQ_128B | TCC_BUBBLE | read MiB | expected MiB | ratio |",
                  "|---|---:|---:|---:|---:|---:|---:|---:|"]
        for k, (rp, _) in KERNELS.items():
            c = raw.get(k, {})
            if not c:
                continue
            m = {n: sum(v) / len(v) for n, v in c.items()}
            req, r32, r128 = m.get("TCC_EA0_RDREQ_sum", 0), m.get("TCC_EA0_RDREQ_32B_sum", 0), \
                m.get("TCC_EA0_RDREQ_128B_sum", 0)
            mib_rd = (128 * r128 + 32 * r32 + 64 * (req - r128 - r32)) / 2**20
            er = rp * buf / 2**20
            lines.append(f"| `{k}` | {req:.4g} | {r32:.4g} | {r128:.4g} | {m.get('TCC_BUBBLE_sum', 0):.4g} | "
                         f"{mib_rd:.1f} | {er:.0f} | {mib_rd / er if er else float('nan'):.3f} |")
    lines.append("")
    lines.append("| kernel | SQ counter | per dispatch |")
    lines.append("|---|---|---:|")
    for k in KERNELS:
        for c, v in sorted(s.get(k, {}).items()):
            lines.append(f"| `{k}` | {c} | {sum(v) / len(v):.4g} |")
    return "\n".join(lines)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        import argparse

        ap = argparse.ArgumentParser()
        ap.add_argument("mode")
        ap.add_argument("--mib", type=int, default=1024)
        ap.add_argument("--iters", type=int, default=4)
        a = ap.parse_args()
        run(a.mib, a.iters)
    else:
        raw = sys.argv[5] if len(sys.argv) > 5 else None
        print(summarize(sys.argv[2], sys.argv[3], sys.argv[4], raw, 1024))
