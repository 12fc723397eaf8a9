"""Time PyTorch SDPA (GQA expanded) fwd+bwd at the Llama-3-8B attention shape."""
import time
import torch
import torch.nn.functional as F

B, S, H, HKV, D = 2, 4096, 32, 8, 128
q = torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(B, HKV, S, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(B, HKV, S, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
for name, kw in [("expand", {}), ("enable_gqa", {"enable_gqa": True})]:
    try:
        for it in range(4):
            torch.cuda.synchronize(); t = time.perf_counter()
            if kw:
                o = F.scaled_dot_product_attention(q, k, v, is_causal=True, **kw)
            else:
                o = F.scaled_dot_product_attention(q, k.repeat_interleave(4, 1), v.repeat_interleave(4, 1), is_causal=True)
            torch.cuda.synchronize(); t1 = time.perf_counter()
            o.backward(torch.ones_like(o))
            torch.cuda.synchronize(); t2 = time.perf_counter()
        fl = 4 * B * H * S * S * D / 2
        print(f"{name}: fwd {1e3*(t1-t):.2f} ms ({fl/(t1-t)/1e12:.0f} TF/s) bwd {1e3*(t2-t1):.2f} ms ({2.5*fl/(t2-t1)/1e12:.0f} TF/s)", flush=True)
    except Exception as e:
        print(name, "failed", e)
for be in ["FLASH_ATTENTION", "EFFICIENT_ATTENTION", "MATH"]:
    print(be, getattr(torch.backends.cuda, "is_flash_attention_available", lambda: None)() if be=="FLASH_ATTENTION" else "")
x = torch.randn(8192, 4096, device="cuda", dtype=torch.bfloat16)
w = torch.randn(14336*2, 4096, device="cuda", dtype=torch.bfloat16)
for it in range(3):
    torch.cuda.synchronize(); t = time.perf_counter()
    y = F.linear(x, w)
    torch.cuda.synchronize(); t1 = time.perf_counter()
print(f"gemm 8192x28672x4096: {1e3*(t1-t):.2f} ms {2*8192*28672*4096/(t1-t)/1e12:.0f} TF/s")
