"""Turn a rocprofv3 --stats kernel_stats.csv into a committed profile summary.

    python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv \
        profiles/<name> --title "..." [--bench gpurun_out/bench_full.log] [--top 25]

Writes <dir>/kernel_stats.csv (copy), <dir>/SUMMARY.md (top kernels + kgwe
HIP kernel share) and, if --bench is given, <dir>/bench.json (the JSON line).
"""
from __future__ import annotations

import argparse
import csv
import json
import shutil
from pathlib import Path


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("out")
    ap.add_argument("--title", default="rocprofv3 kernel stats")
    ap.add_argument("--bench")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--steps", type=int, default=0, help="training steps in the profiled run")
    a = ap.parse_args(argv)
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    shutil.copy(a.stats, out / "kernel_stats.csv")
    rows = list(csv.DictReader(open(a.stats)))
    total = sum(int(r["TotalDurationNs"]) for r in rows)
    lines = [f"# {a.title}", "", f"Total kernel time {total / 1e6:.1f} ms"
             + (f" ({a.steps} steps, {total / 1e6 / a.steps:.1f} ms/step)" if a.steps else "") + ".", ""]
    kg = sum(int(r["TotalDurationNs"]) for r in rows
             if "(anonymous namespace)::" in r["Name"] and "at::" not in r["Name"])
    lines += [f"kgwe hand-written HIP kernels: {kg / 1e6:.1f} ms ({100 * kg / max(total, 1):.1f} %).", "",
              "| ms total | % | calls | avg us | kernel |", "|---:|---:|---:|---:|---|"]
    for r in rows[:a.top]:
        t = int(r["TotalDurationNs"])
        lines.append(f"| {t / 1e6:.2f} | {100 * t / total:.2f} | {r['Calls']} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | `{r['Name'][:90]}` |")
    if a.bench:
        for ln in open(a.bench):
            if ln.startswith("{") and '"metric"' in ln:
                (out / "bench.json").write_text(json.dumps(json.loads(ln), indent=1) + "\n")
    (out / "SUMMARY.md").write_text("\n".join(lines) + "\n")
    print("\n".join(lines[:8]))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
