"""Time the bf16 transpose at the training step's shapes (GB/s of read + write)."""
import time

import torch

from kgwe.ops import functional as K

for rows, cols in [(16384, 4096), (16384, 14336), (16384, 6144), (4096, 16384)]:
    x = torch.randn(rows, cols, device="cuda").bfloat16()
    out = torch.empty(cols, rows, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        K.transpose(x, out)
    torch.cuda.synchronize()
    t = time.perf_counter()
    n = 20
    for _ in range(n):
        K.transpose(x, out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / n
    assert torch.equal(out, x.t().contiguous())
    print(f"{rows}x{cols}: {dt * 1e6:.1f} us, {2 * x.numel() * 2 / dt / 1e12:.2f} TB/s", flush=True)
