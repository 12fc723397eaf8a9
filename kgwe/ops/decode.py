"""Decode-step ops for the bf16 inference harness (``native/ops/decode.hip``).

* ``rope_append``   — RoPE of the new token's q / k at its position and the
  append of k / v to the head-major KV cache, one kernel;
* ``decode_attention`` — split-K GQA attention of one query token per
  sequence over the cache (HBM-bound; one workgroup per (sequence, kv head,
  key chunk) serves all query heads of the group).

On a GPU the HIP kernels are mandatory; on CPU the fp32 references below run
(also the numerics oracle of the GPU tests).
"""
from __future__ import annotations

import math

import torch

from ._lib import check, lib, ptr, stream, use_hip


def _require(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(msg)


# ------------------------------------------------------------------ references
def rope_append_reference(qkv, pos, cos, sin, kc, vc, hq, hkv, d):
    B = qkv.shape[0]
    x = qkv.float().view(B, hq + 2 * hkv, d)
    c = cos[pos.long()].float()[:, None, :]  # [B, 1, d/2]
    s = sin[pos.long()].float()[:, None, :]
    h = d // 2

    def rot(t):
        a, b = t[..., :h], t[..., h:]
        return torch.cat([a * c - b * s, b * c + a * s], dim=-1)

    q = rot(x[:, :hq]).to(qkv.dtype)
    k = rot(x[:, hq:hq + hkv]).to(kc.dtype)
    v = x[:, hq + hkv:].to(vc.dtype)
    for b in range(B):
        p = int(pos[b])
        kc[b, :, p] = k[b]
        vc[b, :, p] = v[b]
    return q


def decode_attention_reference(q, kc, vc, lens):
    """q [B,Hq,D], caches [B,Hkv,Smax,D], lens [B] -> [B,Hq,D] (fp32 math)."""
    B, hq, d = q.shape
    hkv = kc.shape[1]
    out = torch.empty_like(q)
    for b in range(B):
        n = int(lens[b])
        k = kc[b, :, :n].float().repeat_interleave(hq // hkv, dim=0)  # [Hq, n, D]
        v = vc[b, :, :n].float().repeat_interleave(hq // hkv, dim=0)
        sc = torch.einsum("hd,hnd->hn", q[b].float(), k) / math.sqrt(d)
        out[b] = torch.einsum("hn,hnd->hd", sc.softmax(-1), v).to(q.dtype)
    return out


# ------------------------------------------------------------------ ops
def rope_append(qkv: torch.Tensor, pos: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor,
                kc: torch.Tensor, vc: torch.Tensor, hq: int, hkv: int, d: int) -> torch.Tensor:
    """qkv [B,(hq+2hkv)d] bf16, pos [B] int32 -> q [B,hq,d]; writes k/v into
    kc/vc [B,hkv,Smax,d] at pos."""
    if not use_hip(qkv):
        return rope_append_reference(qkv, pos, cos, sin, kc, vc, hq, hkv, d)
    B = qkv.shape[0]
    _require(qkv.dtype == torch.bfloat16 and qkv.is_contiguous() and qkv.shape == (B, (hq + 2 * hkv) * d),
             "rope_append: qkv must be contiguous bf16 [B, (hq+2hkv)*d]")
    _require(pos.dtype == torch.int32 and pos.shape == (B,) and pos.is_cuda, "rope_append: pos int32 [B]")
    _require(kc.shape == vc.shape and kc.dim() == 4 and kc.shape[:2] == (B, hkv) and kc.shape[3] == d
             and kc.dtype == vc.dtype == torch.bfloat16 and kc.is_contiguous() and vc.is_contiguous(),
             "rope_append: caches must be contiguous bf16 [B, hkv, Smax, d]")
    _require(cos.dtype == sin.dtype == torch.float32 and cos.shape == sin.shape
             and cos.shape[0] >= kc.shape[2] and cos.shape[1] == d // 2,
             "rope_append: cos/sin fp32 [>=Smax, d/2]")
    q = torch.empty(B, hq, d, device=qkv.device, dtype=qkv.dtype)
    check(lib().kgwe_decode_rope_append(ptr(qkv), ptr(pos), ptr(cos), ptr(sin), ptr(q), ptr(kc), ptr(vc),
                                        B, hq, hkv, d, kc.shape[2], stream(qkv)), "decode_rope_append")
    return q


class DecodeAttention:
    """Split count + workspace sized once for a cache (hipGraph-safe)."""

    def __init__(self, B: int, hq: int, hkv: int, d: int, smax: int, device):
        self.B, self.hq, self.hkv, self.d, self.smax = B, hq, hkv, d, smax
        self.hip = torch.device(device).type == "cuda"
        if self.hip:
            _require(hq % hkv == 0 and hq // hkv in (1, 2, 4, 8) and d in (64, 128),
                     "decode_attention: head_dim 64/128 and Hq/Hkv in {1,2,4,8}")
            self.splits = int(lib().kgwe_decode_attn_splits(B, hkv, smax))
            n = int(lib().kgwe_decode_attn_workspace(B, hq, d, self.splits))
            self.work = torch.empty(n, device=device, dtype=torch.float32)

    def __call__(self, q: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, lens: torch.Tensor):
        if not self.hip:
            return decode_attention_reference(q, kc, vc, lens)
        _require(q.shape == (self.B, self.hq, self.d) and q.dtype == torch.bfloat16 and q.is_contiguous(),
                 "decode_attention: q must be contiguous bf16 [B, Hq, D]")
        _require(kc.shape == vc.shape == (self.B, self.hkv, self.smax, self.d), "decode_attention: cache shape")
        _require(lens.dtype == torch.int32 and lens.shape == (self.B,), "decode_attention: lens int32 [B]")
        out = torch.empty_like(q)
        check(lib().kgwe_decode_attn(ptr(q), ptr(kc), ptr(vc), ptr(lens), ptr(self.work), ptr(out),
                                     self.B, self.hq, self.hkv, self.d, self.smax, self.splits,
                                     1.0 / math.sqrt(self.d), stream(q)), "decode_attn")
        return out
