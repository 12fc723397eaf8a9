"""bf16 Llama decoding on the kgwe HIP kernels (the inference pods the
platform co-locates / partitions: BASELINE.json config 4, "8 bf16 inference
pods"; reference README.md:31 "7x GPU density").

* prefill: the training forward's kernels (fused QKV split + RoPE, flash
  attention at head_dim 128, SDPA otherwise) and a copy of K/V into the
  cache;
* decode step: RMSNorm (+residual) -> QKV GEMM -> fused RoPE + KV-cache
  append (``kgwe_decode_rope_append``) -> split-K GQA decode attention
  (``kgwe_decode_attn``) -> o-proj -> RMSNorm -> w13 GEMM -> SwiGLU -> w2,
  greedy argmax; positions advance INSIDE the step, so the whole step is
  captured once in a hipGraph (``torch.cuda.CUDAGraph`` is hipGraph on ROCm)
  and replayed — a 1B-parameter decode step is ~200 kernels, launch-bound
  without a graph.

KV cache: one bf16 tensor [L, B, Hkv, Smax, D] (head-major, so one
(sequence, kv head) is a contiguous slab the decode kernel streams).
"""
from __future__ import annotations

import torch

from ..ops import attn as attn_ops
from ..ops import decode as dec
from ..ops import functional as K
from ..ops import reference as ref
from .llama import Llama


class Generator:
    def __init__(self, model: Llama, batch: int, max_seq: int, keep_logits: bool = False):
        self.m = model
        self.keep_logits = keep_logits
        self.logits = None
        c = model.cfg
        self.cfg = c
        p = next(model.parameters())
        self.dev = p.device
        self.B, self.smax = batch, max_seq
        hq, hkv, d = c.n_heads, c.n_kv_heads, c.head_dim
        self.kv = torch.zeros(2, c.n_layers, batch, hkv, max_seq, d, device=self.dev, dtype=p.dtype)
        self.cos, self.sin = ref.rope_tables(max_seq, d, c.rope_theta, self.dev)
        self.cos, self.sin = self.cos.float().contiguous(), self.sin.float().contiguous()
        self.attn = dec.DecodeAttention(batch, hq, hkv, d, max_seq, self.dev)
        self.tok = torch.zeros(batch, dtype=torch.long, device=self.dev)
        self.pos = torch.zeros(batch, dtype=torch.int32, device=self.dev)
        self.lens = torch.zeros(batch, dtype=torch.int32, device=self.dev)
        # 1 = the row decodes; 0 = the row is idle (its position does not
        # advance, so an unused slot of a serving batch never runs off the cache)
        self.active = torch.ones(batch, dtype=torch.int32, device=self.dev)
        self.graph = None
        self.filled = 0  # host-side count of cached positions (no device sync)
        # Fused decode projections (native/ops/gemv.hip): RMSNorm + residual,
        # SwiGLU and the greedy argmax ride inside the weight-streaming GEMVs.
        import os  # noqa: PLC0415

        self.fused = (self.dev.type == "cuda" and os.environ.get("KGWE_DECODE_FUSED", "1") != "0"
                      and dec.gemv_supported(batch, c.dim) and dec.gemv_supported(batch, hq * d))
        if self.fused:
            self.hbuf = torch.empty(2, batch, c.dim, device=self.dev, dtype=p.dtype)
            self.best = torch.zeros(batch, dec.argmax_slots(c.vocab_size, batch), dtype=torch.long, device=self.dev)
            self.w2_fused = dec.gemv_supported(batch, c.ffn_dim)
            self.split_norm = batch > 8

    # ------------------------------------------------------------ prefill
    @torch.no_grad()
    def prefill(self, tokens: torch.Tensor, rows: tuple[int, int] | None = None) -> torch.Tensor:
        """tokens [B, P] -> next token [B]; fills cache positions [0, P).
        With rows=(r0, r1) only batch rows [r0, r1) are prefilled (tokens
        [r1 - r0, P]); the other rows' cache, tokens and positions are left as
        they are, so a serving loop admits a request between two decode steps."""
        c, m = self.cfg, self.m
        B, P = tokens.shape
        r0, r1 = rows if rows is not None else (0, self.B)
        if not (0 <= r0 < r1 <= self.B) or B != r1 - r0 or P >= self.smax:
            raise ValueError(f"prefill: expected [B={r1 - r0}, P<{self.smax}] for rows {r0}:{r1} of {self.B}, "
                             f"got {tuple(tokens.shape)}")
        hq, hkv, d = c.n_heads, c.n_kv_heads, c.head_dim
        cos, sin = self.cos[:P], self.sin[:P]
        h = m.tok_embeddings(tokens)
        residual = None
        for i, layer in enumerate(m.layers):
            if residual is None:
                xn, residual = K.rmsnorm(h, layer.attention_norm, c.norm_eps)
            else:
                xn, residual = K.rmsnorm(h, layer.attention_norm, c.norm_eps, residual=residual)
            qkv = K.linear(xn, layer.attention.wqkv).view(B * P, -1)
            q, k, v = K.rope_qkv(qkv, cos, sin, P, hq, hkv, d)
            k4, v4 = k.view(B, P, hkv, d), v.view(B, P, hkv, d)
            self.kv[0, i, r0:r1, :, :P].copy_(k4.transpose(1, 2))
            self.kv[1, i, r0:r1, :, :P].copy_(v4.transpose(1, 2))
            o = attn_ops.attention(q.view(B, P, hq, d), k4, v4, causal=True)
            a = K.linear(o.reshape(B, P, -1), layer.attention.wo)
            xn, residual = K.rmsnorm(a, layer.ffn_norm, c.norm_eps, residual=residual)
            h = layer.feed_forward(xn)
        h, _ = K.rmsnorm(h, m.norm, c.norm_eps, residual=residual)
        logits = K.linear(h[:, -1], m.output)
        if self.keep_logits and rows is None:
            self.logits = logits.clone()
        nxt = logits.argmax(-1)
        self.tok[r0:r1].copy_(nxt)
        self.pos[r0:r1].fill_(P)
        self.lens[r0:r1].fill_(P + 1)
        self.filled = max(P, self.filled) if rows is not None else P
        return nxt

    # ------------------------------------------------------------ decode
    @torch.no_grad()
    def _step_fused(self) -> None:
        """One decode step in 5 kernels per layer (7 for a serving batch, whose
        two RMSNorms are kernels of their own): [RMSNorm(+res) -> wqkv],
        [RoPE + KV append + split-K attention + merge], wo,
        [RMSNorm(+res) -> w13 -> SwiGLU], w2; and [RMSNorm(+res) -> LM head ->
        argmax] at the end."""
        c, m = self.cfg, self.m
        hq, hkv, d = c.n_heads, c.n_kv_heads, c.head_dim
        B, eps = self.B, c.norm_eps
        x = m.tok_embeddings(self.tok)  # [B, dim]
        res = None
        if self.split_norm:
            # A serving batch (8 < B <= 32): the projections run on the matrix-core
            # kernel, whose every workgroup stages x.  Fused, each of them would redo
            # the RMSNorm of all B rows; one small kernel does it once instead, and
            # the projections stage a plain copy.  SwiGLU and argmax stay fused.
            for i, layer in enumerate(m.layers):
                at, ff = layer.attention, layer.feed_forward
                xn, h = K.rmsnorm(x, layer.attention_norm, eps, residual=res)
                qkv = dec.gemv(xn, at.wqkv)
                o = self.attn.rope_attend(qkv, self.cos, self.sin, self.kv[0, i], self.kv[1, i], self.lens)
                a = dec.gemv(o.view(B, -1), at.wo)
                xn, res = K.rmsnorm(a, layer.ffn_norm, eps, residual=h)
                f = dec.gemv(xn, ff.w13, dec.GEMV_SWIGLU)
                x = dec.gemv(f, ff.w2) if self.w2_fused else K.linear(f, ff.w2)
            xn, _ = K.rmsnorm(x, m.norm, eps, residual=res)
            if self.keep_logits and self.logits is None:
                self.logits = torch.empty(B, c.vocab_size, device=self.dev, dtype=x.dtype)
            dec.gemv(xn, m.output, dec.GEMV_ARGMAX, y=self.logits if self.keep_logits else None, best=self.best)
            dec.argmax_finish(self.best, self.tok)
            self.pos.add_(self.active)
            self.lens.add_(self.active)
            return
        hA, hB = self.hbuf[0], self.hbuf[1]
        for i, layer in enumerate(m.layers):
            at, ff = layer.attention, layer.feed_forward
            if res is None:
                qkv = dec.gemv(x, at.wqkv, dec.GEMV_NORM, g=layer.attention_norm, eps=eps)
                h = x
            else:
                qkv = dec.gemv(x, at.wqkv, dec.GEMV_NORM, res=res, g=layer.attention_norm, eps=eps, h_out=hA)
                h = hA
            o = self.attn.rope_attend(qkv, self.cos, self.sin, self.kv[0, i], self.kv[1, i], self.lens)
            a = dec.gemv(o.view(B, -1), at.wo)
            f = dec.gemv(a, ff.w13, dec.GEMV_NORM_SWIGLU, res=h, g=layer.ffn_norm, eps=eps, h_out=hB)
            x = dec.gemv(f, ff.w2) if self.w2_fused else K.linear(f, ff.w2)
            res = hB
        if self.keep_logits and self.logits is None:
            self.logits = torch.empty(B, c.vocab_size, device=self.dev, dtype=x.dtype)
        dec.gemv(x, m.output, dec.GEMV_NORM_ARGMAX, res=res, g=m.norm, eps=eps,
                 y=self.logits if self.keep_logits else None, best=self.best)
        dec.argmax_finish(self.best, self.tok)
        self.pos.add_(self.active)
        self.lens.add_(self.active)

    @torch.no_grad()
    def _step(self) -> None:
        if self.fused:
            return self._step_fused()
        c, m = self.cfg, self.m
        hq, hkv, d = c.n_heads, c.n_kv_heads, c.head_dim
        h = m.tok_embeddings(self.tok)  # [B, dim]
        residual = None
        for i, layer in enumerate(m.layers):
            if residual is None:
                xn, residual = K.rmsnorm(h, layer.attention_norm, c.norm_eps)
            else:
                xn, residual = K.rmsnorm(h, layer.attention_norm, c.norm_eps, residual=residual)
            qkv = K.linear(xn, layer.attention.wqkv)
            if self.dev.type == "cuda":  # RoPE + cache append inside the attention launch
                o = self.attn.rope_attend(qkv, self.cos, self.sin, self.kv[0, i], self.kv[1, i], self.lens)
            else:
                q = dec.rope_append(qkv, self.pos, self.cos, self.sin, self.kv[0, i], self.kv[1, i], hq, hkv, d)
                o = self.attn(q, self.kv[0, i], self.kv[1, i], self.lens)
            a = K.linear(o.view(self.B, -1), layer.attention.wo)
            xn, residual = K.rmsnorm(a, layer.ffn_norm, c.norm_eps, residual=residual)
            h = layer.feed_forward(xn)
        h, _ = K.rmsnorm(h, m.norm, c.norm_eps, residual=residual)
        logits = K.linear(h, m.output)
        if self.keep_logits:  # tests: a static buffer the graph writes every replay
            if self.logits is None:
                self.logits = torch.empty_like(logits)
            self.logits.copy_(logits)
        self.tok.copy_(logits.argmax(-1))
        self.pos.add_(self.active)
        self.lens.add_(self.active)

    def capture(self) -> None:
        """Record one decode step in a hipGraph (warm-up on a side stream, as
        graph capture requires).  Positions advance inside the graph."""
        if self.dev.type != "cuda":
            return
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        saved = (self.tok.clone(), self.pos.clone(), self.lens.clone())
        with torch.cuda.stream(s):
            self._step()  # allocator warm-up, lazy library handles
        torch.cuda.current_stream(self.dev).wait_stream(s)
        self.tok.copy_(saved[0])
        self.pos.copy_(saved[1])
        self.lens.copy_(saved[2])
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._step()
        self.graph = g
        # capture does not execute the work: state is unchanged

    def idle_rows(self, r0: int, r1: int, idle: bool = True) -> None:
        """Park batch rows [r0, r1) (or wake them): a parked row keeps decoding
        position 0 of its own cache slab and is ignored by the caller."""
        self.active[r0:r1].fill_(0 if idle else 1)
        if idle:
            self.pos[r0:r1].zero_()
            self.lens[r0:r1].fill_(1)

    def step(self, check: bool = True) -> torch.Tensor:
        """One decode step for every row.  check=False: the caller tracks each
        row group's length itself (a serving loop whose rows start at different
        times)."""
        if check and self.filled + 1 >= self.smax:
            raise RuntimeError("KV cache full")
        if self.graph is not None:
            self.graph.replay()
        else:
            self._step()
        self.filled += 1
        return self.tok

    @torch.no_grad()
    def generate(self, prompt: torch.Tensor, new_tokens: int, graph: bool = True) -> torch.Tensor:
        self.prefill(prompt)
        if graph and self.graph is None:
            self.capture()
        out = [self.tok.clone()]
        for _ in range(new_tokens - 1):
            out.append(self.step().clone())
        return torch.stack(out, 1)
