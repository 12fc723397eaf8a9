"""Llama-3 family decoder (random init) built on the kgwe gfx950 kernels.

This is the FSDP workload the platform schedules and benchmarks
(BASELINE.json config 3: "8-GPU Llama-3-8B FSDP torchrun pod, backend=RCCL").
The reference has no model code at all — it only carries the workload as
metadata (reference: src/scheduler/types.go:92-110 WorkloadSpec,
src/optimizer/workload_optimizer.py:275-285 MODEL_RESOURCE_MAP keyed by
parameter count) — so this module is new, written MI355X-first:

* fused QKV projection -> one HIP kernel does the q/k/v split + RoPE;
* fused gate|up (w13) projection -> one HIP SwiGLU kernel reading it in place;
* residual add fused into RMSNorm (one HBM pass instead of two);
* fused vocabulary cross-entropy (no fp32 logits copy);
* GEMMs are hipBLASLt GEMMs; the weight-gradient GEMMs get their operands
  transposed into the library's fast layouts (``K.linear``).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass

import torch
import torch.nn as nn

from ..ops import attn as attn_ops
from ..ops import functional as K
from ..ops import reference as ref


@dataclass(frozen=True)
class LlamaConfig:
    name: str = "llama3-8b"
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    ffn_dim: int = 14336
    vocab_size: int = 128256
    norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    max_seq_len: int = 8192

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    def num_params(self) -> int:
        d, f, v = self.dim, self.ffn_dim, self.vocab_size
        hd = self.head_dim
        attn = d * (self.n_heads + 2 * self.n_kv_heads) * hd + self.n_heads * hd * d
        mlp = 3 * d * f
        per_layer = attn + mlp + 2 * d
        return self.n_layers * per_layer + 2 * v * d + d

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs per token (fwd+bwd = 3x fwd), incl. causal attention."""
        dense = 6.0 * (self.num_params() - self.vocab_size * self.dim)  # no embedding gather
        attn = 6.0 * self.n_layers * self.dim * seq_len  # 2*2*S*d fwd, halved by causality, x3
        return dense + attn

    def to_dict(self) -> dict:
        return asdict(self)


PRESETS = {
    "llama3-8b": LlamaConfig(),
    "llama3-70b": LlamaConfig(name="llama3-70b", dim=8192, n_layers=80, n_heads=64,
                              n_kv_heads=8, ffn_dim=28672),
    "llama3.2-1b": LlamaConfig(name="llama3.2-1b", dim=2048, n_layers=16, n_heads=32,
                               n_kv_heads=8, ffn_dim=8192),
    # Test-sized model: same code paths, kernels' shape constraints respected
    # (dim multiple of 512, head_dim 64/128, ffn multiple of 8, vocab % 8 == 0).
    "tiny": LlamaConfig(name="tiny", dim=512, n_layers=2, n_heads=4, n_kv_heads=2,
                        ffn_dim=1024, vocab_size=1024, max_seq_len=512),
}


class RopeCache:
    """fp32 cos/sin tables [S, head_dim/2] per (S, device); a plain object (not
    an nn.Module / buffer) so FSDP neither shards nor casts it."""

    _tables: dict = {}

    def __init__(self, cfg: "LlamaConfig"):
        self.head_dim = cfg.head_dim
        self.theta = cfg.rope_theta

    def __call__(self, seq_len: int, device) -> tuple[torch.Tensor, torch.Tensor]:
        key = (seq_len, self.head_dim, self.theta, str(device))
        t = RopeCache._tables.get(key)
        if t is None:
            t = ref.rope_tables(seq_len, self.head_dim, self.theta, device)
            RopeCache._tables[key] = t
        return t


class Attention(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        hd = cfg.head_dim
        self.wqkv = nn.Parameter(torch.empty((cfg.n_heads + 2 * cfg.n_kv_heads) * hd, cfg.dim))
        self.wo = nn.Parameter(torch.empty(cfg.dim, cfg.n_heads * hd))

    def forward(self, x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
        B, S, _ = x.shape
        c = self.cfg
        qkv = K.linear(x, self.wqkv).view(B * S, -1)
        q, k, v = K.rope_qkv(qkv, cos, sin, S, c.n_heads, c.n_kv_heads, c.head_dim)
        o = attn_ops.attention(q.view(B, S, c.n_heads, c.head_dim),
                               k.view(B, S, c.n_kv_heads, c.head_dim),
                               v.view(B, S, c.n_kv_heads, c.head_dim), causal=True)
        return K.linear(o.reshape(B, S, -1), self.wo)


class FeedForward(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.w13 = nn.Parameter(torch.empty(2 * cfg.ffn_dim, cfg.dim))
        self.w2 = nn.Parameter(torch.empty(cfg.dim, cfg.ffn_dim))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return K.linear(K.swiglu(K.linear(x, self.w13)), self.w2)


class TransformerBlock(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        self.attention = Attention(cfg)
        self.feed_forward = FeedForward(cfg)
        self.attention_norm = nn.Parameter(torch.ones(cfg.dim))
        self.ffn_norm = nn.Parameter(torch.ones(cfg.dim))
        self.rope_tables = RopeCache(cfg)

    def forward(self, x, residual):
        """(x, residual) -> (mlp_out, residual'); the residual add happens inside
        the next RMSNorm kernel.  RoPE tables come from the shared cache, NOT
        from forward args: FSDP2's MixedPrecisionPolicy casts floating-point
        forward inputs to bf16, which would corrupt the fp32 cos/sin tables."""
        eps = self.cfg.norm_eps
        cos, sin = self.rope_tables(x.shape[1], x.device)
        if residual is None:
            xn, residual = K.rmsnorm(x, self.attention_norm, eps)
        else:
            xn, residual = K.rmsnorm(x, self.attention_norm, eps, residual=residual)
        a = self.attention(xn, cos, sin)
        xn, residual = K.rmsnorm(a, self.ffn_norm, eps, residual=residual)
        return self.feed_forward(xn), residual


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        self.tok_embeddings = nn.Embedding(cfg.vocab_size, cfg.dim)
        self.layers = nn.ModuleList(TransformerBlock(cfg) for _ in range(cfg.n_layers))
        self.norm = nn.Parameter(torch.ones(cfg.dim))
        self.output = nn.Parameter(torch.empty(cfg.vocab_size, cfg.dim))
        self.activation_checkpointing = False

    @torch.no_grad()
    def init_weights(self, std: float = 0.02, seed: int = 0) -> None:
        g = torch.Generator(device=self.output.device).manual_seed(seed)
        for name, p in self.named_parameters():
            if name.endswith("norm") or name == "norm":
                p.fill_(1.0)
            else:
                p.normal_(0.0, std, generator=g)

    def forward_hidden(self, tokens: torch.Tensor) -> torch.Tensor:
        h = self.tok_embeddings(tokens)
        residual = None
        for layer in self.layers:
            if self.activation_checkpointing and torch.is_grad_enabled():
                h, residual = torch.utils.checkpoint.checkpoint(
                    layer, h, residual, use_reentrant=False)
            else:
                h, residual = layer(h, residual)
        h, _ = K.rmsnorm(h, self.norm, self.cfg.norm_eps, residual=residual)
        return h

    def forward(self, tokens: torch.Tensor, labels: torch.Tensor | None = None):
        h = self.forward_hidden(tokens)
        logits = K.linear(h, self.output)
        if labels is None:
            return logits
        return K.cross_entropy(logits, labels)


def build(cfg: LlamaConfig | str, device="cpu", dtype=torch.float32) -> Llama:
    if isinstance(cfg, str):
        cfg = PRESETS[cfg]
    with torch.device(device):
        m = Llama(cfg)
    m.to(dtype)
    m.init_weights()
    return m
