"""Plain PyTorch fp32 references of every hand-written kernel.

These define the semantics the HIP kernels are tested against (numerics tests
compare kernel output with these) and provide the CPU execution path used by
the control-plane test-suite, which has no GPU.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float,
            residual: torch.Tensor | None = None):
    """Returns (y, h) with h = x + residual (or x)."""
    h = x if residual is None else (x.float() + residual.float()).to(x.dtype)
    hf = h.float()
    rstd = torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + eps)
    y = (hf * rstd * w.float()).to(x.dtype)
    return y, h


def swiglu(g: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    return (F.silu(g.float()) * u.float()).to(g.dtype)


def rope_tables(seq_len: int, head_dim: int, theta: float = 500000.0,
                device=None) -> tuple[torch.Tensor, torch.Tensor]:
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    t = torch.arange(seq_len, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def rope_qkv(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, seq_len: int,
             hq: int, hkv: int, d: int):
    """qkv: [T, (hq+2hkv)*d] -> q [T,hq,d], k [T,hkv,d], v [T,hkv,d]."""
    T = qkv.shape[0]
    x = qkv.view(T, hq + 2 * hkv, d).float()
    q, k, v = x[:, :hq], x[:, hq:hq + hkv], x[:, hq + hkv:]
    pos = torch.arange(T, device=qkv.device) % seq_len
    c = cos[pos].unsqueeze(1)
    s = sin[pos].unsqueeze(1)

    def rot(t):
        t1, t2 = t[..., : d // 2], t[..., d // 2:]
        return torch.cat([t1 * c - t2 * s, t2 * c + t1 * s], dim=-1)

    dt = qkv.dtype
    return rot(q).to(dt), rot(k).to(dt), v.to(dt).contiguous()


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor,
                  ignore_index: int = -100) -> torch.Tensor:
    return F.cross_entropy(logits.float(), labels, ignore_index=ignore_index)


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True):
    """q: [B, S, Hq, D], k/v: [B, S, Hkv, D] -> [B, S, Hq, D] (GQA)."""
    hq, hkv = q.shape[2], k.shape[2]
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    if hq != hkv:
        kf = kf.repeat_interleave(hq // hkv, dim=1)
        vf = vf.repeat_interleave(hq // hkv, dim=1)
    o = F.scaled_dot_product_attention(qf, kf, vf, is_causal=causal)
    return o.transpose(1, 2).to(q.dtype)


def adamw_(p, g, m, v, lr, b1, b2, eps, wd, step):
    m.mul_(b1).add_(g, alpha=1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = (v.sqrt() / (bc2 ** 0.5)).add_(eps)
    p.sub_(lr * (m / bc1 / denom + wd * p))
