"""Autograd wrappers around the gfx950 HIP kernels.

Each op has a HIP path (GPU tensors, mandatory on a GPU host) and the fp32
PyTorch reference path (CPU tensors only).  Shapes follow the Llama block in
``kgwe.models.llama``.
"""
from __future__ import annotations

import os

import torch

from . import reference as ref
from ._lib import check, lib, ptr, stream, use_hip
from .gemm import wgrad, wgrad_supported


def _require(cond: bool, msg: str) -> None:
    """Shape/dtype contract of a HIP kernel, checked on the host before launch
    (an out-of-contract launch would read or write out of bounds)."""
    if not cond:
        raise ValueError(msg)


# --------------------------------------------------------------------------
# Transposed gradients handed from a producer's backward to the consuming
# linear layer's backward
# --------------------------------------------------------------------------
# A weight gradient dW = dY^T X reduces over tokens; the library's fastest GEMM
# layout wants dY^T and X^T (token dimension contiguous).  Transposing dY in
# a pass of its own costs what the layout gains, so the kernel that PRODUCES
# dY (SwiGLU backward for the gate|up projection; the same in the RoPE
# backward for the QKV projection measured no gain and was dropped) writes dY^T
# next to it and offers it here, keyed by dY's storage; the linear layer's backward, the next
# autograd node to run, takes it.  One entry: an offer nobody took is dropped
# by the next one.
_offered: dict = {}


def _dual_grads() -> bool:
    return os.environ.get("KGWE_DUAL_GRADS", "1") != "0"


def _offer_transposed(dy: torch.Tensor, dy_t: torch.Tensor) -> None:
    _offered.clear()
    # dy itself is held too: while the offer stands its storage cannot be
    # reused for another tensor that would then match the key
    _offered[(dy.data_ptr(), dy.shape[0], dy.shape[1], dy.device)] = (dy_t, dy)


def _take_transposed(dy2: torch.Tensor) -> torch.Tensor | None:
    hit = _offered.pop((dy2.data_ptr(), dy2.shape[0], dy2.shape[1], dy2.device), None)
    return None if hit is None else hit[0]


# --------------------------------------------------------------------------
# RMSNorm (+ fused residual add)
# --------------------------------------------------------------------------
class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps, residual):
        H = x.shape[-1]
        x2 = x.reshape(-1, H)
        T = x2.shape[0]
        y = torch.empty_like(x2)
        rstd = torch.empty(T, device=x.device, dtype=torch.float32)
        h = torch.empty_like(x2) if residual is not None else x2
        r2 = residual.reshape(-1, H) if residual is not None else None
        check(lib().kgwe_rmsnorm_fwd(ptr(x2), ptr(r2), ptr(w), ptr(y),
                                     ptr(h) if residual is not None else None, ptr(rstd),
                                     T, H, eps, stream(x)), "rmsnorm_fwd")
        ctx.save_for_backward(h, w, rstd)
        ctx.has_res = residual is not None
        ctx.shape = x.shape
        if residual is None:
            return y.view(x.shape)
        return y.view(x.shape), h.view(x.shape)

    @staticmethod
    def backward(ctx, dy, dh=None):
        h, w, rstd = ctx.saved_tensors
        H = h.shape[-1]
        T = h.shape[0]
        dy2 = dy.reshape(-1, H).contiguous()
        dadd = dh.reshape(-1, H).contiguous() if dh is not None else None
        dx = torch.empty_like(dy2)
        partial = torch.empty(H, device=h.device, dtype=torch.float32)  # dw accumulator
        dw = torch.empty(H, device=h.device, dtype=w.dtype)
        dw_bf = dw if w.dtype == torch.bfloat16 else None
        dw_f = dw if w.dtype == torch.float32 else None
        check(lib().kgwe_rmsnorm_bwd(ptr(dy2), ptr(h), ptr(w), ptr(rstd), ptr(dadd), ptr(dx),
                                     ptr(partial), ptr(dw_bf), ptr(dw_f), T, H, stream(h)),
              "rmsnorm_bwd")
        dx = dx.view(ctx.shape)
        return dx, dw, None, (dx if ctx.has_res else None)


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5,
            residual: torch.Tensor | None = None):
    """Returns (normed, h) where h = x + residual (the new residual stream)."""
    if use_hip(x):
        H = x.shape[-1]
        _require(x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16,
                 "rmsnorm: x and w must be bf16")
        _require(H in (512, 1024, 2048, 4096, 8192) and w.numel() == H,
                 "rmsnorm: hidden size must be 512*2^k <= 8192 and w [H]")
        _require(residual is None or (residual.shape == x.shape and residual.dtype == x.dtype),
                 "rmsnorm: residual must match x")
        if residual is None:
            return _RMSNorm.apply(x.contiguous(), w.contiguous(), eps, None), x
        return _RMSNorm.apply(x.contiguous(), w.contiguous(), eps, residual.contiguous())
    return ref.rmsnorm(x, w, eps, residual)


# --------------------------------------------------------------------------
# SwiGLU on the fused [T, 2F] gate|up projection
# --------------------------------------------------------------------------
class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        F2 = gu.shape[-1]
        Fh = F2 // 2
        gu2 = gu.reshape(-1, F2)
        T = gu2.shape[0]
        out = torch.empty(T, Fh, device=gu.device, dtype=gu.dtype)
        check(lib().kgwe_swiglu_fwd(ptr(gu2), gu2.data_ptr() + Fh * gu2.element_size(), F2,
                                    ptr(out), T, Fh, stream(gu)), "swiglu_fwd")
        ctx.save_for_backward(gu2)
        ctx.shape = gu.shape
        return out.view(*gu.shape[:-1], Fh)

    @staticmethod
    def backward(ctx, dout):
        (gu2,) = ctx.saved_tensors
        T, F2 = gu2.shape
        Fh = F2 // 2
        d2 = dout.reshape(-1, Fh).contiguous()
        dgu = torch.empty_like(gu2)
        es = gu2.element_size()
        if _dual_grads() and T % 64 == 0 and Fh % 64 == 0:
            # also the transposed gradient, for the producing projection's dW GEMM
            dgu_t = torch.empty(F2, T, device=gu2.device, dtype=gu2.dtype)
            check(lib().kgwe_swiglu_bwd_t(ptr(gu2), gu2.data_ptr() + Fh * es, F2, ptr(d2),
                                          ptr(dgu), dgu.data_ptr() + Fh * es, F2, ptr(dgu_t), T, Fh,
                                          stream(gu2)), "swiglu_bwd_t")
            _offer_transposed(dgu, dgu_t)
        else:
            check(lib().kgwe_swiglu_bwd(ptr(gu2), gu2.data_ptr() + Fh * es, F2, ptr(d2),
                                        ptr(dgu), dgu.data_ptr() + Fh * es, F2, T, Fh,
                                        stream(gu2)), "swiglu_bwd")
        return dgu.view(ctx.shape)


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    """silu(gu[..., :F]) * gu[..., F:]"""
    if use_hip(gu):
        _require(gu.dtype == torch.bfloat16 and gu.shape[-1] % 16 == 0,
                 "swiglu: gu must be bf16 [..., 2F] with F % 8 == 0")
        return _SwiGLU.apply(gu.contiguous())
    Fh = gu.shape[-1] // 2
    return ref.swiglu(gu[..., :Fh], gu[..., Fh:])


# --------------------------------------------------------------------------
# Fused QKV split + RoPE
# --------------------------------------------------------------------------
class _RopeQKV(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, seq_len, hq, hkv, d):
        T = qkv.shape[0]
        q = torch.empty(T, hq, d, device=qkv.device, dtype=qkv.dtype)
        k = torch.empty(T, hkv, d, device=qkv.device, dtype=qkv.dtype)
        v = torch.empty(T, hkv, d, device=qkv.device, dtype=qkv.dtype)
        check(lib().kgwe_rope_qkv_fwd(ptr(qkv), ptr(q), ptr(k), ptr(v), ptr(cos), ptr(sin), T,
                                      seq_len, hq, hkv, d, stream(qkv)), "rope_fwd")
        ctx.save_for_backward(cos, sin)
        ctx.meta = (T, seq_len, hq, hkv, d)
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        cos, sin = ctx.saved_tensors
        T, S, hq, hkv, d = ctx.meta
        dev = cos.device
        dt = next(t.dtype for t in (dq, dk, dv) if t is not None)
        z = lambda h: torch.zeros(T, h, d, device=dev, dtype=dt)  # noqa: E731
        dq = dq.contiguous() if dq is not None else z(hq)
        dk = dk.contiguous() if dk is not None else z(hkv)
        dv = dv.contiguous() if dv is not None else z(hkv)
        dqkv = torch.empty(T, (hq + 2 * hkv) * d, device=dev, dtype=dt)
        check(lib().kgwe_rope_qkv_bwd(ptr(dq), ptr(dk), ptr(dv), ptr(dqkv), ptr(cos), ptr(sin),
                                      T, S, hq, hkv, d, stream(dqkv)), "rope_bwd")
        return dqkv, None, None, None, None, None, None


def rope_qkv(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, seq_len: int,
             hq: int, hkv: int, d: int):
    """qkv [T, (hq+2hkv)d] -> q [T,hq,d], k [T,hkv,d], v [T,hkv,d] (rotated q, k)."""
    if use_hip(qkv):
        # Host-side operand checks: the kernel indexes cos/sin as fp32 [S, d/2]
        # rows by (row % S) and reads qkv rows of (hq+2hkv)*d bf16.
        _require(qkv.dtype == torch.bfloat16 and qkv.dim() == 2
                 and qkv.shape[1] == (hq + 2 * hkv) * d, "rope: qkv must be bf16 [T, (hq+2hkv)*d]")
        _require(d % 16 == 0, "rope: head_dim must be a multiple of 16")
        _require(qkv.shape[0] % seq_len == 0, "rope: T must be a multiple of seq_len")
        cos = cos.to(torch.float32).contiguous()
        sin = sin.to(torch.float32).contiguous()
        _require(cos.shape == sin.shape and cos.dim() == 2 and cos.shape[0] >= seq_len
                 and cos.shape[1] == d // 2 and cos.device == qkv.device,
                 "rope: cos/sin must be fp32 [>=S, d/2] on the qkv device")
        return _RopeQKV.apply(qkv.contiguous(), cos, sin, seq_len, hq, hkv, d)
    return ref.rope_qkv(qkv, cos, sin, seq_len, hq, hkv, d)


# --------------------------------------------------------------------------
# Cross-entropy over the vocabulary (mean over non-ignored rows)
# --------------------------------------------------------------------------
class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        T, V = logits.shape
        loss = torch.empty(T, device=logits.device, dtype=torch.float32)
        lse = torch.empty(T, device=logits.device, dtype=torch.float32)
        check(lib().kgwe_cross_entropy_fwd(ptr(logits), ptr(labels), ptr(loss), ptr(lse), T, V,
                                           ignore_index, stream(logits)), "ce_fwd")
        n = (labels != ignore_index).sum().clamp_min(1).to(torch.float32)
        ctx.save_for_backward(logits, labels, lse, n)
        ctx.ignore_index = ignore_index
        return loss.sum() / n

    @staticmethod
    def backward(ctx, g):
        logits, labels, lse, n = ctx.saved_tensors
        T, V = logits.shape
        scale = (g.to(torch.float32) / n).reshape(1).contiguous()
        dlogits = torch.empty_like(logits)
        check(lib().kgwe_cross_entropy_bwd(ptr(logits), ptr(labels), ptr(lse), ptr(scale),
                                           ptr(dlogits), T, V, ctx.ignore_index,
                                           stream(logits)), "ce_bwd")
        return dlogits, None, None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100):
    logits = logits.reshape(-1, logits.shape[-1])
    labels = labels.reshape(-1)
    if use_hip(logits):
        _require(logits.dtype == torch.bfloat16 and logits.shape[-1] % 8 == 0,
                 "cross_entropy: logits must be bf16 with vocab % 8 == 0 (16-B rows)")
        _require(labels.numel() == logits.shape[0] and labels.device == logits.device,
                 "cross_entropy: one label per logits row, same device")
        return _CrossEntropy.apply(logits.contiguous(), labels.to(torch.int64).contiguous(),
                                   ignore_index)
    return ref.cross_entropy(logits, labels, ignore_index)


# --------------------------------------------------------------------------
# Linear layer with layout-aware weight-gradient GEMMs
# --------------------------------------------------------------------------
def transpose(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """[R, C] bf16 -> contiguous [C, R] (LDS-tiled HIP transpose; fp32-free
    copy on CPU)."""
    if not use_hip(x):
        t = x.t().contiguous()
        return t if out is None else out.copy_(t)
    _require(x.dim() == 2 and x.dtype == torch.bfloat16 and x.is_contiguous()
             and x.shape[0] % 8 == 0 and x.shape[1] % 8 == 0,
             "transpose: contiguous bf16 [R, C] with R % 8 == 0 and C % 8 == 0")
    if out is None:
        out = torch.empty(x.shape[1], x.shape[0], device=x.device, dtype=x.dtype)
    _require(out.shape == (x.shape[1], x.shape[0]) and out.dtype == x.dtype and out.is_contiguous()
             and out.device == x.device, "transpose: out must be a contiguous [C, R] bf16 tensor")
    check(lib().kgwe_transpose_bf16(ptr(x), ptr(out), x.shape[0], x.shape[1], stream(x)),
          "transpose_bf16")
    return out


def _wgrad_mode() -> str:
    mode = os.environ.get("KGWE_WGRAD", "auto")
    _require(mode in ("auto", "kernel", "library"), "KGWE_WGRAD must be auto, kernel or library")
    return mode


def weight_grad(dy2: torch.Tensor, x2: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """dW[N, K] = dY[T, N]^T X[T, K] by the fastest route for the shape; with
    ``out`` (contiguous, dY's dtype) the GEMM writes there — the data-parallel
    wrapper passes the parameter's slice of its gradient bucket, so no copy of
    the gradient is ever made."""
    N, K = dy2.shape[1], x2.shape[1]
    mode = _wgrad_mode()
    dy_t = _take_transposed(dy2)
    if dy_t is not None and mode != "kernel" and x2.is_contiguous() and x2.shape[0] % 8 == 0 and K % 8 == 0:
        # both operands token-contiguous: the library's "nt" layout
        return torch.mm(dy_t, transpose(x2).t(), out=out)
    if (mode != "library" and (N < K or mode == "kernel") and wgrad_supported(dy2, x2)
            and (out is None or out.data_ptr() % 8 == 0)):
        return wgrad(dy2, x2, out=out)
    if x2.shape[0] % 8 or N % 8 or K % 8 or not x2.is_contiguous():
        return torch.mm(dy2.t(), x2, out=out)
    if N >= K:
        return torch.mm(dy2.t(), transpose(x2).t(), out=out)   # "tt"
    return torch.mm(transpose(dy2), x2, out=out)               # "nn"


class _Linear(torch.autograd.Function):
    """y = x W^T.  Forward is the plain library GEMM ("nt"); the input
    gradient uses the weight's persistent transposed copy when one exists
    (``w._kgwe_wt``, kept by kgwe.parallel.zero) so it runs "nt" as well; the
    weight gradient dW = dY^T X — a reduction over the leading (token)
    dimension of both stored operands, the slowest hipBLASLt layout on MI355X
    — is issued after transposing the SMALLER of X / dY, which moves it to
    the "tt" / "nn" kernels (tools/gemm_layouts.py: ~1.35 vs ~1.1 PF/s for
    the Llama-3-8B shapes; the transpose of a [T, 4096] operand costs ~25 us).

    Where the library would need dY itself transposed (N < K, the MLP down
    projection) the hand-written MFMA kernel of kgwe.ops.gemm takes both
    operands as stored and is the faster of the two (1.70 vs 1.82 ms at
    [4096, 14336] over 16,384 tokens); ``KGWE_WGRAD=kernel`` uses it for every
    shape it supports, ``KGWE_WGRAD=library`` never.

    A weight with a gradient sink (``w._kgwe_grad_sink``, set by
    kgwe.parallel.zero at world > 1) gets its dW written by the GEMM straight
    into the reduce-scatter bucket; autograd then sees no gradient for it."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        # Persistent W^T copy kept by the data-parallel wrapper, if any
        # (kgwe.parallel.zero): makes dX = dY W an "nt" GEMM.
        ctx.wt = getattr(w, "_kgwe_wt", None)
        ctx.sink = getattr(w, "_kgwe_grad_sink", None)
        return torch.nn.functional.linear(x, w)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        N, K = w.shape
        x2 = x.reshape(-1, K)
        dy2 = dy.reshape(-1, N)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = dw = None
        if ctx.needs_input_grad[0]:
            wt = ctx.wt
            dx = (torch.mm(dy2, wt.t()) if wt is not None else torch.mm(dy2, w)).view(x.shape)
        if ctx.needs_input_grad[1]:
            if ctx.sink is None or not ctx.sink(dy2, x2):
                dw = weight_grad(dy2, x2)
        return dx, dw


def linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    if use_hip(x) and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16:
        return _Linear.apply(x, w)
    return torch.nn.functional.linear(x, w)
