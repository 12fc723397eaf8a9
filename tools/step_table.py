"""One training step cut out of a rocprofv3 kernel trace of bench.py.

The window runs from one cross-entropy forward to the next (backward of step
k, its AdamW, forward of step k + 1: one step's worth of every kernel); with
--step N the N-th such window (default: the last).  Prints a markdown table
of kernel classes: ms per step, share, launches.

  python tools/step_table.py gpurun_out/prof/run_kernel_trace.csv
"""
import argparse
import collections
import csv
import re

CLASSES = [  # (regex on the kernel name, label)
    (r"^Custom_Cijk_Alik_Bljk_BBS_BH_MT", 'hipBLASLt LM head GEMMs `Custom_Cijk_Alik_Bljk_BBS_BH_MT256x256x64…`'),
    (r"^Custom_Cijk_Alik_Bljk", 'hipBLASLt "nt" GEMM (forward, dX, dW from transposed gradients) `Custom_Cijk_Alik_Bljk…MT256x256x64`'),
    (r"^Cijk_Alik_Bjlk.*MT256x256", 'hipBLASLt "tt" GEMM `Cijk_Alik_Bjlk…MT256x256x64`'),
    (r"^Cijk_Alik_Bjlk", 'hipBLASLt "tt" GEMM, other tile `Cijk_Alik_Bjlk…`'),
    (r"^Cijk_", "hipBLASLt GEMM, other layout"),
    (r"wgrad_kernel", "kgwe `wgrad_kernel`"),
    (r"wgrad_reduce_kernel", "kgwe `wgrad_reduce_kernel`"),
    (r"adamw_kernel", "kgwe `adamw_kernel`"),
    (r"fa_bwd_dkdv_kernel", "kgwe `fa_bwd_dkdv_kernel`"),
    (r"fa_bwd_dkdv_finalize", "kgwe `fa_bwd_dkdv_finalize`"),
    (r"fa_bwd_dq_kernel", "kgwe `fa_bwd_dq_kernel`"),
    (r"fa_fwd_kernel", "kgwe `fa_fwd_kernel`"),
    (r"swiglu_bwd_t_kernel", "kgwe `swiglu_bwd_t_kernel` (gradient in both layouts)"),
    (r"swiglu_bwd_kernel", "kgwe `swiglu_bwd_kernel`"),
    (r"swiglu_fwd_kernel", "kgwe `swiglu_fwd_kernel`"),
    (r"transpose_bf16_kernel", "kgwe `transpose_bf16_kernel`"),
    (r"rmsnorm_bwd_kernel", "kgwe `rmsnorm_bwd_kernel`"),
    (r"rmsnorm_fwd_kernel", "kgwe `rmsnorm_fwd_kernel`"),
    (r"rope_kernel", "kgwe `rope_kernel`"),
    (r"ce_bwd_kernel", "kgwe `ce_bwd_kernel`"),
    (r"ce_fwd_kernel", "kgwe `ce_fwd_kernel`"),
    (r"dw_cast_kernel", "kgwe `dw_cast_kernel`"),
    (r"zero_f32_kernel", "kgwe `zero_f32_kernel`"),
    (r"copyBuffer|fillBuffer", "runtime copy / fill"),
]


def label(name: str) -> str:
    for pat, lab in CLASSES:
        if re.search(pat, name):
            return lab
    return "other (PyTorch elementwise, embedding, sort)"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-1)
    a = ap.parse_args()
    rows = []
    with open(a.trace, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [s for s, _, n in rows if "ce_fwd_kernel" in n]
    if len(marks) < 2:
        raise SystemExit("need at least two cross-entropy forwards in the trace")
    windows = list(zip(marks[:-1], marks[1:]))
    t0, t1 = windows[a.step]
    ms = collections.Counter()
    calls = collections.Counter()
    for s, e, n in rows:
        if t0 <= s < t1:
            lab = label(n)
            ms[lab] += (e - s) / 1e6
            calls[lab] += 1
    total = sum(ms.values())
    print(f"window {(t1 - t0) / 1e6:.1f} ms wall, kernel time {total:.1f} ms, {sum(calls.values())} launches\n")
    print("| ms / step | % | launches | kernel |")
    print("|---:|---:|---:|---|")
    for lab, v in ms.most_common():
        print(f"| {v:.2f} | {100 * v / total:.1f} | {calls[lab]} | {lab} |")
    hand = sum(v for lab, v in ms.items() if lab.startswith("kgwe"))
    gemm = sum(v for lab, v in ms.items() if "GEMM" in lab or "wgrad_kernel" in lab)
    print(f"\nhand-written kgwe kernels {hand:.1f} ms ({100 * hand / total:.1f} %), GEMMs (library + wgrad) "
          f"{gemm:.1f} ms ({100 * gemm / total:.1f} %)")


if __name__ == "__main__":
    main()
