"""Hand-written gfx950 MFMA flash attention vs the fp32 PyTorch reference."""
import math

import pytest
import torch

from kgwe.ops import attn
from kgwe.ops import reference as ref

pytestmark = pytest.mark.gpu


def _inputs(B, S, Hq, Hkv, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    mk = lambda h: torch.randn(B, S, h, 128, device="cuda", dtype=torch.bfloat16, generator=g)  # noqa: E731
    return mk(Hq), mk(Hkv), mk(Hkv)


@pytest.mark.parametrize("B,S,Hq,Hkv,causal", [
    (1, 128, 4, 4, True), (2, 256, 8, 2, True), (1, 1024, 8, 2, True),
    (2, 384, 4, 1, False), (1, 200, 4, 2, True), (1, 600, 4, 2, False), (1, 1000, 8, 8, True)])
@pytest.mark.parametrize("growing_max", ["randn", "growing-max", "max-jump"])
def test_flash_fwd_matches_reference(B, S, Hq, Hkv, causal, growing_max):
    q, k, v = _inputs(B, S, Hq, Hkv)
    if growing_max == "growing-max":
        # keys get larger along the sequence, so the running row max moves on
        # late tiles and the conditional O rescale must fire mid-sweep
        k = (k.float() * torch.linspace(0.5, 4.0, S, device="cuda")[None, :, None, None]).to(k.dtype)
    elif growing_max == "max-jump":
        # the second half's scores are ~6x the first half's: the deferred
        # running max (raised only past 2^8 growth) must be raised mid-sweep,
        # rescaling O and l computed against the stale max
        k = k.clone()
        k[:, S // 2:] *= 6
    o, lse2 = attn.flash_fwd(q, k, v, causal)
    o_ref = ref.attention(q, k, v, causal)
    err = (o.float() - o_ref.float()).abs()
    assert err.max().item() < 2e-2, err.max().item()
    # lse2 (log2 units) vs reference logsumexp of the scaled scores
    kf = k.float().repeat_interleave(Hq // Hkv, dim=2)
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), kf) / math.sqrt(128)
    if causal:
        s = s.masked_fill(torch.ones(S, S, device="cuda", dtype=torch.bool).triu(1), float("-inf"))
    lse_ref = torch.logsumexp(s, dim=-1) / math.log(2)
    assert (lse2 - lse_ref).abs().max().item() < 1e-2


@pytest.mark.parametrize("B,S,Hq,Hkv,causal", [
    (1, 128, 4, 4, True), (2, 256, 8, 2, True), (1, 512, 8, 2, True), (1, 256, 4, 1, False),
    (1, 200, 4, 2, True), (1, 384, 8, 2, True)])
def test_flash_bwd_matches_reference(B, S, Hq, Hkv, causal):
    q, k, v = _inputs(B, S, Hq, Hkv, seed=1)
    qh, kh, vh = (t.clone().requires_grad_(True) for t in (q, k, v))
    o = attn._FlashAttn.apply(qh, kh, vh, causal)
    do = torch.randn_like(o)
    o.backward(do)
    qr, kr, vr = (t.float().clone().requires_grad_(True) for t in (q, k, v))
    o_ref = ref.attention(qr, kr, vr, causal)
    o_ref.backward(do.float())
    for name, a, b in (("dq", qh.grad, qr.grad), ("dk", kh.grad, kr.grad), ("dv", vh.grad, vr.grad)):
        rel = ((a.float() - b).norm() / b.norm()).item()
        assert rel < 2e-2, (name, rel)


def test_model_uses_hip_flash_attention():
    assert attn.hip_flash_available()
