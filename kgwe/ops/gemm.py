"""Hand-written MFMA GEMMs (native/ops/wgrad_gemm.hip).

``wgrad(dy, x)`` is the weight gradient of a linear layer, dW[N, K] =
dY[T, N]^T X[T, K], computed from both operands exactly as autograd stores
them (token-major): no transposed copy of either is made.  fp32 accumulation,
bf16 result — the contract of ``torch.mm`` on bf16 operands.
"""
from __future__ import annotations

import torch

from ._lib import check, lib, ptr, stream, use_hip

_ws: dict = {}  # (device, bytes) -> fp32 split-K workspace, reused across calls


def wgrad_supported(dy: torch.Tensor, x: torch.Tensor) -> bool:
    """Shapes the kernel takes: bf16, 2-D, unit inner stride, N and K multiples
    of 256, T a multiple of 64, rows 16-byte aligned."""
    if not (use_hip(x) and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16):
        return False
    if dy.dim() != 2 or x.dim() != 2 or dy.shape[0] != x.shape[0]:
        return False
    T, N = dy.shape
    K = x.shape[1]
    if T % 64 or N % 256 or K % 256 or T == 0:
        return False
    if dy.stride(1) != 1 or x.stride(1) != 1 or dy.stride(0) % 8 or x.stride(0) % 8:
        return False
    if dy.stride(0) < N or x.stride(0) < K or (dy.data_ptr() | x.data_ptr()) & 15:
        return False
    return T * max(dy.stride(0), x.stride(0)) < 2**31


def wgrad(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor | None = None, splits: int = 0) -> torch.Tensor:
    """dW[N, K] = dy[T, N]^T @ x[T, K] (bf16 in, fp32 accumulate, bf16 out)."""
    if not wgrad_supported(dy, x):
        raise ValueError(f"wgrad: unsupported operands {tuple(dy.shape)} x {tuple(x.shape)}")
    T, N = dy.shape
    K = x.shape[1]
    if out is None:
        out = torch.empty(N, K, device=x.device, dtype=torch.bfloat16)
    elif out.shape != (N, K) or out.dtype != torch.bfloat16 or not out.is_contiguous() or out.device != x.device:
        raise ValueError("wgrad: out must be a contiguous bf16 [N, K] tensor on the operands' device")
    L = lib()
    s = splits or L.kgwe_wgrad_splits(N, K, T)
    ws = None
    if s > 1:
        need = s * N * K * 4
        key = (x.device, torch.cuda.current_stream(x.device).cuda_stream)
        ws = _ws.get(key)
        if ws is None or ws.numel() * 4 < need:
            ws = _ws[key] = torch.empty(need // 4, device=x.device, dtype=torch.float32)
    check(L.kgwe_wgrad_bf16(ptr(dy), ptr(x), ptr(out), ptr(ws), N, K, T, dy.stride(0), x.stride(0), K, s,
                            stream(x)), "wgrad_bf16")
    return out
