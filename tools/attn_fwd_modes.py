"""Time the flash-attention forward at the training shapes (B = 2 / 4, causal
and full) and compare it with PyTorch SDPA.  With the variant kernel of
profiles/r03_attn/skew_kernel.patch applied, KGWE_FA_FWD (read once per process
by the launcher) selects it: 0 shipped kernel, 1 / 2 phase-skewed halves, 3 the
variant's code with nobody late; without the patch the variable does nothing."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from kgwe.ops import attn

H, HKV, D, S = 32, 8, 128, 4096
mode = os.environ.get("KGWE_FA_FWD", "0")


def bench(fn, n=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


for B, causal in ((2, True), (4, True), (4, False)):
    g = torch.Generator(device="cuda").manual_seed(B)
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g)
    k = torch.randn(B, S, HKV, D, device="cuda", dtype=torch.bfloat16, generator=g)
    v = torch.randn(B, S, HKV, D, device="cuda", dtype=torch.bfloat16, generator=g)
    fl = 4 * B * H * S * S * D / (2 if causal else 1)
    ts = sorted(bench(lambda: attn.flash_fwd(q, k, v, causal)) for _ in range(3))
    o1, _ = attn.flash_fwd(q, k, v, causal)
    o2 = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                        is_causal=causal, enable_gqa=True).transpose(1, 2)
    err = (o1.float() - o2.float()).abs().max().item()
    print(f"mode {mode} B={B} causal={int(causal)}: {ts[0]*1e3:.3f} / {ts[1]*1e3:.3f} / {ts[2]*1e3:.3f} ms "
          f"(best {fl/ts[0]/1e12:.0f} TF/s)  max|o - sdpa| {err:.4f}", flush=True)
