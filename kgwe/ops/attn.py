"""Causal GQA attention for the Llama block.

Dispatch order on a GPU:
  1. ``kgwe_flash_attn_*`` — the hand-written gfx950 MFMA flash-attention
     kernels in ``native/ops/flash_attn.hip`` (when built into the library);
  2. otherwise (head_dim != 128, or forced) PyTorch SDPA (ROCm flash
     backend) with the GQA heads expanded.
On CPU the fp32 reference is used.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import reference as ref
from ._lib import check, has_symbol, lib, ptr, stream, use_hip


class _FlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal):
        B, S, Hq, D = q.shape
        Hkv = k.shape[2]
        o = torch.empty_like(q)
        lse = torch.empty(B, Hq, S, device=q.device, dtype=torch.float32)
        scale = 1.0 / math.sqrt(D)
        check(lib().kgwe_flash_attn_fwd(ptr(q), ptr(k), ptr(v), ptr(o), ptr(lse), B, S, Hq, Hkv,
                                        D, scale, int(causal), stream(q)), "flash_attn_fwd")
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal = causal
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        B, S, Hq, D = q.shape
        Hkv = k.shape[2]
        do = do.contiguous()
        dq = torch.empty_like(q)
        dk = torch.empty_like(k)
        dv = torch.empty_like(v)
        ws = lib().kgwe_flash_attn_bwd_workspace(B, S, Hq, Hkv, D)
        work = torch.empty(max(ws, 4) // 4, device=q.device, dtype=torch.float32)
        check(lib().kgwe_flash_attn_bwd(ptr(q), ptr(k), ptr(v), ptr(o), ptr(lse), ptr(do),
                                        ptr(dq), ptr(dk), ptr(dv), ptr(work), None, B, S, Hq,
                                        Hkv, D, 1.0 / math.sqrt(D), int(ctx.causal),
                                        stream(q)), "flash_attn_bwd")
        return dq, dk, dv, None


_FORCE_SDPA = False


def set_force_sdpa(flag: bool) -> None:
    global _FORCE_SDPA
    _FORCE_SDPA = flag


def hip_flash_available() -> bool:
    return has_symbol("kgwe_flash_attn_fwd") and has_symbol("kgwe_flash_attn_bwd")


def flash_fwd(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True):
    """Forward only (inference / tests): returns (o, lse2) with lse2 in log2 units."""
    B, S, Hq, D = q.shape
    if not (q.is_contiguous() and k.is_contiguous() and v.is_contiguous()
            and q.dtype == k.dtype == v.dtype == torch.bfloat16 and D == 128
            and k.shape == v.shape == (B, S, k.shape[2], D) and Hq % k.shape[2] == 0):
        raise ValueError("flash_fwd: contiguous bf16 [B,S,H,128] q/k/v with Hq % Hkv == 0")
    o = torch.empty_like(q)
    lse = torch.empty(B, Hq, S, device=q.device, dtype=torch.float32)
    check(lib().kgwe_flash_attn_fwd(ptr(q), ptr(k), ptr(v), ptr(o), ptr(lse), B, S, Hq, k.shape[2],
                                    D, 1.0 / math.sqrt(D), int(causal), stream(q)), "flash_attn_fwd")
    return o, lse


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True):
    """q [B,S,Hq,D], k/v [B,S,Hkv,D] -> o [B,S,Hq,D]."""
    if not use_hip(q):
        return ref.attention(q, k, v, causal)
    if not _FORCE_SDPA and q.shape[-1] == 128 and hip_flash_available():
        return _FlashAttn.apply(q.contiguous(), k.contiguous(), v.contiguous(), causal)
    hq, hkv = q.shape[2], k.shape[2]
    qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
    if hq != hkv:
        kt = kt.repeat_interleave(hq // hkv, dim=1)
        vt = vt.repeat_interleave(hq // hkv, dim=1)
    o = F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal)
    return o.transpose(1, 2)
