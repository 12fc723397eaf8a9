"""Time the decode projections of a serving batch (M = 32 rows by default):
the matrix-core skinny GEMM of kgwe.ops.decode.gemv with its fused RMSNorm /
SwiGLU / argmax against the library GEMM alone (torch F.linear: no norm, no
SwiGLU, no argmax — a floor for the unfused path)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from kgwe.ops import decode as dec

M = int(sys.argv[1]) if len(sys.argv) > 1 else 32
SHAPES = [  # name, N (SWIGLU: F), K, mode
    ("1b wqkv", 3072, 2048, dec.GEMV_PLAIN), ("1b wqkv  norm fused", 3072, 2048, dec.GEMV_NORM),
    ("1b wo", 2048, 2048, dec.GEMV_PLAIN),
    ("1b w13   swiglu", 8192, 2048, dec.GEMV_SWIGLU), ("1b w2", 2048, 8192, dec.GEMV_PLAIN),
    ("1b head  argmax", 128256, 2048, dec.GEMV_ARGMAX),
    ("8b wqkv", 6144, 4096, dec.GEMV_PLAIN), ("8b wo", 4096, 4096, dec.GEMV_PLAIN),
    ("8b w13   swiglu", 14336, 4096, dec.GEMV_SWIGLU), ("8b w2", 4096, 14336, dec.GEMV_PLAIN),
]
COPIES_MB = 1200  # distinct weight copies per shape: past the 256 MB of last-level cache


def bench(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


g = torch.Generator(device="cuda").manual_seed(0)
for name, N, K, mode in (SHAPES if M <= 32 else []):  # past 32 rows only the attention sweep
    if M <= 8 and mode == dec.GEMV_ARGMAX:
        mode = dec.GEMV_NORM_ARGMAX  # M <= 8: the argmax kernel always carries the fused norm
    rows = 2 * N if mode & dec.GEMV_SWIGLU else N
    x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).bfloat16()
    res = torch.randn_like(x) if mode & dec.GEMV_NORM else None
    n_copies = max(1, min(10, int(COPIES_MB * 1e6 // (rows * K * 2))))
    ws = [(torch.randn(rows, K, device="cuda", generator=g) / K ** 0.5).bfloat16() for _ in range(n_copies)]
    gw = torch.ones(K, device="cuda", dtype=torch.bfloat16)
    h = torch.empty_like(x) if res is not None else None
    best = (torch.zeros(M, dec.argmax_slots(N, M), dtype=torch.long, device="cuda")
            if mode & dec.GEMV_ARGMAX else None)
    graph = torch.cuda.CUDAGraph()

    def run(i=0):
        return dec.gemv(x, ws[i % n_copies], mode, res=res, g=gw if mode & dec.GEMV_NORM else None, h_out=h,
                        best=best)

    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        run()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(graph):
        for i in range(10):
            run(i)
    t_k = bench(graph.replay, 50) / 10
    glib = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        F.linear(x, ws[0])
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(glib):
        for i in range(10):
            F.linear(x, ws[i % n_copies])
    t_l = bench(glib.replay, 50) / 10
    mb = rows * K * 2 / 1e6
    print(f"M={M} {name:24s} [{rows:6d} x {K:5d}] {mb:7.1f} MB  kgwe {t_k*1e6:7.1f} us ({mb/1e6/t_k:5.2f} TB/s)   "
          f"library GEMM alone {t_l*1e6:7.1f} us ({mb/1e6/t_l:5.2f} TB/s)", flush=True)


# ---- decode attention at this batch: split-count sweep (KGWE_DECODE_SPLITS) ----
hq, hkv, d, smax, filled = 32, 8, 64, 1024, 640
cos = torch.randn(smax, d // 2, device="cuda")
sin = torch.randn(smax, d // 2, device="cuda")
kc = torch.randn(M, hkv, smax, d, device="cuda").bfloat16()
vc = torch.randn(M, hkv, smax, d, device="cuda").bfloat16()
qkv = torch.randn(M, (hq + 2 * hkv) * d, device="cuda").bfloat16()
lens = torch.full((M,), filled, dtype=torch.int32, device="cuda")
layers = 16  # distinct caches, as the layers of a model (no cache reuse between calls)
kcs = [kc.clone() for _ in range(layers)]
vcs = [vc.clone() for _ in range(layers)]
for sp in (0, 1, 2, 4, 8, 16):
    if sp:
        os.environ["KGWE_DECODE_SPLITS"] = str(sp)
    att = dec.DecodeAttention(M, hq, hkv, d, smax, "cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        att.rope_attend(qkv, cos, sin, kcs[0], vcs[0], lens)
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for i in range(layers):
            att.rope_attend(qkv, cos, sin, kcs[i], vcs[i], lens)
    t = bench(gr.replay, 50) / layers
    mb = M * hkv * filled * d * 2 * 2 / 1e6
    print(f"M={M} decode attention, {filled} of {smax} cached, splits {att.splits:2d}{' (default)' if not sp else ''}: "
          f"{t*1e6:6.1f} us ({mb/1e6/t:4.2f} TB/s of KV)", flush=True)
