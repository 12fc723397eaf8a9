"""Run only the flash-attention forward + backward a few times (for rocprofv3 --pmc)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from kgwe.ops import attn

B = int(os.environ.get("FA_B", "2"))
S, H, HKV, D = 4096, 32, 8, 128
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn(B, S, h, D, device="cuda", dtype=torch.bfloat16, generator=g).requires_grad_(True)
           for h in (H, HKV, HKV))
for _ in range(int(os.environ.get("ITERS", "3"))):
    o = attn.attention(q, k, v, True)
    o.backward(torch.ones_like(o))
torch.cuda.synchronize()
print("ok", flush=True)
