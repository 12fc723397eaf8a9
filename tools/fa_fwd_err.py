"""Max |O - O_ref| of the flash-attention forward on the numerics-test inputs
(tests/test_flash_attn_gpu.py), printed per case, to see the margin under the
test's 2e-2 bound.  GPU only."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from kgwe.ops import attn
from kgwe.ops import reference as ref

for (B, S, Hq, Hkv, causal) in [(1, 128, 4, 4, True), (2, 256, 8, 2, True), (1, 1024, 8, 2, True),
                                (2, 384, 4, 1, False), (1, 200, 4, 2, True), (1, 600, 4, 2, False),
                                (1, 1000, 8, 8, True), (1, 4096, 8, 1, True)]:
    for mode in ("randn", "growing-max", "max-jump"):
        g = torch.Generator(device="cuda").manual_seed(0)
        q, k, v = (torch.randn(B, S, h, 128, device="cuda", dtype=torch.bfloat16, generator=g) for h in (Hq, Hkv, Hkv))
        if mode == "growing-max":
            k = (k.float() * torch.linspace(0.5, 4.0, S, device="cuda")[None, :, None, None]).to(k.dtype)
        elif mode == "max-jump":
            k = k.clone(); k[:, S // 2:] *= 6
        o, _ = attn.flash_fwd(q, k, v, causal)
        e = (o.float() - ref.attention(q, k, v, causal).float()).abs().max().item()
        print(f"B{B} S{S} {Hq}/{Hkv} causal={int(causal)} {mode:12s} max err {e:.2e}", flush=True)
