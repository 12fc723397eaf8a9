"""Decode-step ops for the bf16 inference harness (``native/ops/decode.hip``).

* ``rope_append``   — RoPE of the new token's q / k at its position and the
  append of k / v to the head-major KV cache, one kernel;
* ``decode_attention`` — split-K GQA attention of one query token per
  sequence over the cache (HBM-bound; one workgroup per (sequence, kv head,
  key chunk) serves all query heads of the group);
* ``gemv`` — the decode step's projections as weight-streaming skinny GEMMs
  with the layer's RMSNorm (+ residual add), SwiGLU and greedy argmax fused
  in: M <= 8 rows on the vector ALU (``native/ops/gemv.hip``), 8 < M <= 32 —
  the batch of a shared-model server — on the matrix cores
  (``native/ops/skinny_gemm.hip``).

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
            import os  # noqa: PLC0415

            forced = int(os.environ.get("KGWE_DECODE_SPLITS", "0"))  # tuning knob: 1..64
            if forced > 0:
                self.splits = max(1, min(64, forced, (smax + 63) // 64))
            n = int(lib().kgwe_decode_attn_workspace(B, hq, d, self.splits))
            # zeroed once: the tail holds the split tickets, which every call
            # returns to zero
            self.work = torch.zeros(n, device=device, dtype=torch.float32)

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


    def rope_attend(self, qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, kc: torch.Tensor,
                    vc: torch.Tensor, lens: torch.Tensor) -> torch.Tensor:
        """``rope_append`` + ``__call__`` in one launch: qkv [B, (hq+2hkv)d] of
        the new token at position lens - 1; RoPE'd k and v are appended to the
        caches there.  Returns [B, hq, d]."""
        if not self.hip:
            q = rope_append_reference(qkv, lens - 1, cos, sin, kc, vc, self.hq, self.hkv, self.d)
            return decode_attention_reference(q, kc, vc, lens)
        B, hq, hkv, d = self.B, self.hq, self.hkv, self.d
        _require(qkv.dtype == torch.bfloat16 and qkv.is_contiguous() and qkv.shape == (B, (hq + 2 * hkv) * d),
                 "decode_attention: qkv must be contiguous bf16 [B, (hq+2hkv)*d]")
        _require(kc.shape == vc.shape == (B, hkv, self.smax, d) and kc.is_contiguous() and vc.is_contiguous(),
                 "decode_attention: cache shape")
        _require(lens.dtype == torch.int32 and lens.shape == (B,), "decode_attention: lens int32 [B]")
        _require(cos.dtype == sin.dtype == torch.float32 and cos.shape == sin.shape
                 and cos.shape[0] >= self.smax and cos.shape[1] == d // 2 and cos.is_contiguous()
                 and sin.is_contiguous(), "decode_attention: cos/sin fp32 [>=Smax, d/2]")
        out = torch.empty(B, hq, d, device=qkv.device, dtype=qkv.dtype)
        check(lib().kgwe_decode_attn_rope(ptr(qkv), ptr(cos), ptr(sin), ptr(kc), ptr(vc), ptr(lens),
                                          ptr(self.work), ptr(out), B, hq, hkv, d, self.smax, self.splits,
                                          1.0 / math.sqrt(d), stream(qkv)), "decode_attn_rope")
        return out


# ------------------------------------------------------------------ projections
GEMV_PLAIN, GEMV_NORM, GEMV_SWIGLU, GEMV_NORM_SWIGLU, GEMV_NORM_ARGMAX = 0, 1, 2, 3, 5
GEMV_ARGMAX = 4  # argmax of a projection whose input is already normalised (8 < M <= 32 only)
GEMV_M = (1, 2, 4, 8)
SKINNY_MAX_M = 32


def _skinny(M: int) -> bool:
    """Batches past the vector-ALU kernels' 8 rows go to the MFMA kernel."""
    return 8 < M <= SKINNY_MAX_M


def gemv_supported(M: int, K: int) -> bool:
    if _skinny(M):
        return K % 64 == 0
    return M in GEMV_M and K % 8 == 0 and M * K * 2 <= 96 * 1024


def _rows_per_wave(N: int) -> int:
    # fill >= ~512 workgroups of 4 waves before packing several rows per wave
    return 1 if N <= 4096 else (2 if N <= 16384 else 4)


def gemv_reference(x, w, mode=GEMV_PLAIN, res=None, g=None, eps=1e-5):
    """fp32 oracle of ``gemv``: returns (y, h) with the same roundings as the
    unfused path (bf16 h = x + res, bf16 normalised x)."""
    h = x
    xin = x.float()
    if mode & GEMV_NORM:
        if res is not None:
            h = (x.float() + res.float()).to(x.dtype)
        hf = h.float()
        rstd = torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + eps)
        xin = (hf * rstd * g.float()).to(x.dtype).float()
    if mode & GEMV_SWIGLU:
        F = w.shape[0] // 2
        gt = xin @ w[:F].float().t()
        up = xin @ w[F:].float().t()
        y = (gt / (1 + torch.exp(-gt)) * up).to(x.dtype)
    else:
        y = (xin @ w.float().t()).to(x.dtype)
    return y, h


_MAX_WGS = None


def max_wgs() -> int:
    """Grid cap of the decode GEMVs: 8 workgroups per CU this process may use
    (a CoLocate share's ``KGWE_CU_RANGE`` = "begin-end", else the device)."""
    global _MAX_WGS
    if _MAX_WGS is None:
        import os  # noqa: PLC0415

        cus = 0
        rng = os.environ.get("KGWE_CU_RANGE", "")
        if "-" in rng:
            try:
                b, e = (int(v) for v in rng.split("-"))
                cus = max(0, e - b)
            except ValueError:
                cus = 0
        if cus <= 0:
            cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count \
                if torch.cuda.is_available() else 256
        _MAX_WGS = 8 * cus
    return _MAX_WGS


def argmax_slots(N: int, M: int = 1) -> int:
    """Entries per row of the ARGMAX partial-maximum buffer for an [N, K] head
    at batch M (one per workgroup of the capped grid; one per block of 32
    weight rows for 8 < M <= 32)."""
    if _skinny(M):
        return (N + 31) // 32
    R = _rows_per_wave(N)
    return min((N + 4 * R - 1) // (4 * R), max_wgs())


_SKINNY_WS: dict = {}


def _skinny_workspace(x: torch.Tensor, N: int, K: int, swiglu: bool) -> torch.Tensor:
    """Split-K partials + tickets of the MFMA kernel for this shape, zeroed
    once (every launch leaves the tickets at zero).  One per device and shape:
    launches that share it must be ordered by their stream, as the layers of
    one decode step are.  (Not per stream: a hipGraph capture runs on a stream
    of its own, and a workspace first created there would be allocated — and
    zero-filled again on every replay — inside the graph.)"""
    cus = max_wgs() // 8
    key = (x.device, N, K, swiglu, cus)
    ws = _SKINNY_WS.get(key)
    if ws is None:
        nbytes = lib().kgwe_decode_skinny_workspace(N, K, int(swiglu), cus)
        _require(nbytes > 0, "gemv: unsupported [N, K] for the batched decode kernel")
        ws = _SKINNY_WS[key] = torch.zeros((nbytes + 3) // 4, dtype=torch.int32, device=x.device)
    return ws


def gemv(x: torch.Tensor, w: torch.Tensor, mode: int = GEMV_PLAIN, res=None, g=None, eps: float = 1e-5,
         h_out=None, y=None, best=None):
    """x [M, K] bf16, w [N, K] (SWIGLU: [2F, K]) -> y [M, N] (SWIGLU: [M, F]).
    NORM modes: h_out (written: the new residual stream x + res) must not
    alias x / res.  ARGMAX: ``best`` int64 [M, argmax_slots(N)] receives one
    packed (value, index) maximum per workgroup; ``argmax_finish`` reduces it."""
    if not use_hip(x):
        yy, h = gemv_reference(x, w, mode, res, g, eps)
        if h_out is not None and res is not None and mode & GEMV_NORM:
            h_out.copy_(h)
        if mode & GEMV_ARGMAX and best is not None:
            best.zero_()
            best[:, 0] = yy.float().argmax(-1)  # CPU: the token itself in slot 0
        if y is not None:
            y.copy_(yy)
            return y
        return yy
    M, K = x.shape
    N = w.shape[0] // 2 if mode & GEMV_SWIGLU else w.shape[0]
    _require(x.dtype == w.dtype == torch.bfloat16 and x.is_contiguous() and w.is_contiguous()
             and w.shape[1] == K and gemv_supported(M, K), "gemv: bf16 contiguous x [M in 1,2,4,8 (K%8==0) or 9..32 (K%64==0)], w [N, K]")
    _require(not (mode & GEMV_NORM) or (g is not None and g.numel() == K), "gemv: NORM needs g [K]")
    _require(res is None or (res.shape == x.shape and res.is_contiguous()), "gemv: res must match x")
    _require(h_out is None or (h_out.shape == x.shape and h_out.data_ptr() not in (
        x.data_ptr(), res.data_ptr() if res is not None else -1)), "gemv: h_out must not alias x / res")
    _require(mode != GEMV_ARGMAX or _skinny(M), "gemv: ARGMAX without NORM needs 8 < M <= 32")
    _require(not mode & GEMV_ARGMAX or (best is not None and best.dtype == torch.long
                                          and best.numel() == M * argmax_slots(N, M)),
             "gemv: ARGMAX needs best int64 [M, argmax_slots(N, M)]")
    if y is None and not mode & GEMV_ARGMAX:
        y = torch.empty(M, N, device=x.device, dtype=x.dtype)
    if _skinny(M):
        ws = _skinny_workspace(x, N, K, bool(mode & GEMV_SWIGLU))
        check(lib().kgwe_decode_skinny(ptr(x), ptr(res) if res is not None else None,
                                       ptr(g) if g is not None else None,
                                       ptr(h_out) if h_out is not None else None, float(eps), ptr(w),
                                       ptr(y) if y is not None else None,
                                       ptr(best) if best is not None else None, ptr(ws), M, N, K, mode,
                                       max_wgs() // 8, stream(x)), "decode_skinny")
        return y
    check(lib().kgwe_decode_gemv(ptr(x), ptr(res) if res is not None else None,
                                 ptr(g) if g is not None else None,
                                 ptr(h_out) if h_out is not None else None, float(eps), ptr(w),
                                 ptr(y) if y is not None else None,
                                 ptr(best) if best is not None else None, M, N, K, mode,
                                 _rows_per_wave(N), max_wgs(), stream(x)), "decode_gemv")
    return y


def argmax_finish(best: torch.Tensor, tok: torch.Tensor) -> None:
    """best [M, slots] (GEMV_NORM_ARGMAX partial maxima) -> tok [M] int64."""
    if not use_hip(best):
        tok.copy_(best[:, 0])
        return
    M, slots = best.shape
    check(lib().kgwe_decode_argmax_finish(ptr(best), ptr(tok), M, slots, stream(best)), "decode_argmax_finish")
