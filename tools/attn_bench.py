"""Time kgwe flash attention vs PyTorch SDPA at the Llama-3-8B shape."""
import math, sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from kgwe.ops import attn

B, S, H, HKV, D = 2, 4096, 32, 8, 128
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g)
k = torch.randn(B, S, HKV, D, device="cuda", dtype=torch.bfloat16, generator=g)
v = torch.randn(B, S, HKV, D, device="cuda", dtype=torch.bfloat16, generator=g)
fl = 4 * B * H * S * S * D / 2  # causal fwd FLOPs

def bench(fn, n=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / n

t_k = bench(lambda: attn.flash_fwd(q, k, v, True))
qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
t_s = bench(lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=True, enable_gqa=True))
print(f"fwd kgwe {t_k*1e3:.3f} ms ({fl/t_k/1e12:.0f} TF/s)  sdpa {t_s*1e3:.3f} ms ({fl/t_s/1e12:.0f} TF/s)", flush=True)
o1, _ = attn.flash_fwd(q, k, v, True)
o2 = F.scaled_dot_product_attention(qt, kt, vt, is_causal=True, enable_gqa=True).transpose(1, 2)
print("max |kgwe - sdpa|", (o1.float() - o2.float()).abs().max().item(), flush=True)
if attn.hip_flash_available():
    qg, kg, vg = (x.detach().clone().requires_grad_(True) for x in (q, k, v))
    def fb():
        o = attn.attention(qg, kg, vg, True); o.backward(torch.ones_like(o))
    t_kb = bench(fb, 10)
    qs_, ks_, vs_ = (x.detach().clone().transpose(1, 2).requires_grad_(True) for x in (q, k, v))
    def sb():
        o = F.scaled_dot_product_attention(qs_, ks_, vs_, is_causal=True, enable_gqa=True); o.backward(torch.ones_like(o))
    t_sb = bench(sb, 10)
    print(f"fwd+bwd kgwe {t_kb*1e3:.3f} ms ({3.5*fl/t_kb/1e12:.0f} TF/s)  sdpa {t_sb*1e3:.3f} ms ({3.5*fl/t_sb/1e12:.0f} TF/s)", flush=True)
