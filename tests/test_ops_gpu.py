"""Numerics of the hand-written gfx950 kernels vs plain PyTorch fp32 references.

All tests here run on a real MI355X (``pytest -m gpu`` via gpurun) and exercise
the HIP path only: the library must be loaded (no silent fallback).
"""
import numpy as np
import pytest
import torch

from kgwe.ops import _lib
from kgwe.ops import functional as K
from kgwe.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _close(a, b, rtol, atol):
    a, b = a.float(), b.float()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).float().mean().item()
    assert bad < 1e-3, f"{bad*100:.3f}% elements out of tolerance; max err {err.max().item():.4g}"


def test_library_loaded():
    L = _lib.lib()
    assert L is not None
    import os
    maps = open(f"/proc/{os.getpid()}/maps").read()
    assert "libkgwe_ops.so" in maps


@pytest.mark.parametrize("H", [512, 2048, 4096, 8192])
@pytest.mark.parametrize("with_res", [False, True])
def test_rmsnorm_fwd_bwd(H, with_res):
    torch.manual_seed(0)
    T = 1000
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    r = torch.randn(T, H, device=DEV, dtype=torch.bfloat16, requires_grad=True) if with_res else None
    y, h = K.rmsnorm(x, w, 1e-5, residual=r)
    # reference in fp32 on leaf copies
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True) if with_res else None
    hr = xr + rr if with_res else xr
    yr = hr * torch.rsqrt(hr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    _close(y, yr, 2e-2, 2e-2)
    if with_res:
        _close(h, hr, 1e-2, 1e-2)
    dy = torch.randn_like(y)
    dh = torch.randn_like(y) if with_res else None
    if with_res:
        torch.autograd.backward([y, h], [dy, dh])
        torch.autograd.backward([yr, hr], [dy.float(), dh.float()])
    else:
        y.backward(dy)
        yr.backward(dy.float())
    _close(x.grad, xr.grad, 3e-2, 3e-2)
    rel = (w.grad.float() - wr.grad).norm() / wr.grad.norm()
    assert rel.item() < 2e-2
    if with_res:
        _close(r.grad, rr.grad, 3e-2, 3e-2)


def test_swiglu_fwd_bwd():
    torch.manual_seed(1)
    T, F = 777, 1792
    gu = torch.randn(T, 2 * F, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    out = K.swiglu(gu)
    gr = gu.detach().float().requires_grad_(True)
    outr = torch.nn.functional.silu(gr[:, :F]) * gr[:, F:]
    _close(out, outr, 2e-2, 2e-2)
    d = torch.randn_like(out)
    out.backward(d)
    outr.backward(d.float())
    _close(gu.grad, gr.grad, 3e-2, 3e-2)


@pytest.mark.parametrize("D", [64, 128])
def test_rope_qkv_fwd_bwd(D):
    torch.manual_seed(2)
    B, S, hq, hkv = 2, 96, 8, 2
    T = B * S
    qkv = torch.randn(T, (hq + 2 * hkv) * D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    cos, sin = ref.rope_tables(S, D, 500000.0, DEV)
    q, k, v = K.rope_qkv(qkv, cos, sin, S, hq, hkv, D)
    qr_in = qkv.detach().float().requires_grad_(True)
    qr, kr, vr = ref.rope_qkv(qr_in, cos, sin, S, hq, hkv, D)
    _close(q, qr, 2e-2, 2e-2)
    _close(k, kr, 2e-2, 2e-2)
    assert torch.equal(v.float(), vr.float())
    dq, dk, dv = torch.randn_like(q), torch.randn_like(k), torch.randn_like(v)
    torch.autograd.backward([q, k, v], [dq, dk, dv])
    torch.autograd.backward([qr, kr, vr], [dq.float(), dk.float(), dv.float()])
    _close(qkv.grad, qr_in.grad, 2e-2, 2e-2)


@pytest.mark.parametrize("V", [1024, 128256])
def test_cross_entropy_fwd_bwd(V):
    torch.manual_seed(3)
    T = 257
    logits = (3 * torch.randn(T, V, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    labels = torch.randint(0, V, (T,), device=DEV)
    labels[5] = -100
    loss = K.cross_entropy(logits, labels)
    lr_ = logits.detach().float().requires_grad_(True)
    lref = torch.nn.functional.cross_entropy(lr_, labels, ignore_index=-100)
    assert abs(loss.item() - lref.item()) < 1e-3 * max(1.0, abs(lref.item()))
    loss.backward()
    lref.backward()
    _close(logits.grad, lr_.grad, 2e-2, 1e-5)
    assert logits.grad[5].abs().max().item() == 0.0


def test_fused_adamw_matches_reference():
    from kgwe.ops import FusedAdamW

    torch.manual_seed(4)
    shapes = [(1000,), (333, 77), (4096, 17), (5,)]
    ps = [torch.randn(s, device=DEV, requires_grad=True) for s in shapes]
    pr = [p.detach().clone() for p in ps]
    ms = [torch.zeros_like(p) for p in pr]
    vs = [torch.zeros_like(p) for p in pr]
    opt = FusedAdamW(ps, lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    for step in range(1, 4):
        gs = [torch.randn_like(p) for p in ps]
        for p, g in zip(ps, gs):
            p.grad = g.clone()
        opt.step()
        for p, g, m, v in zip(pr, gs, ms, vs):
            ref.adamw_(p, g, m, v, 1e-2, 0.9, 0.95, 1e-8, 0.1, step)
    for p, r in zip(ps, pr):
        assert torch.allclose(p.detach(), r, rtol=1e-5, atol=1e-6)


def test_fused_adamw_bf16_master_weights():
    """bf16 params: fp32 master kept by the optimizer, bf16 grads read directly,
    rounded result written back into the bf16 parameter (odd sizes and an
    unaligned view exercise the scalar tail path)."""
    from kgwe.ops import FusedAdamW

    torch.manual_seed(6)
    shapes = [(1000,), (333, 77), (4096, 17), (5,)]
    base = torch.randn(sum(int(np.prod(s)) for s in shapes) + 3, device=DEV)
    ps, off = [], 3  # offset 3 elements: 6-byte misaligned bf16 storage
    flat = base.to(torch.bfloat16)
    for s in shapes:
        n = int(np.prod(s))
        ps.append(torch.nn.Parameter(flat[off:off + n].view(s)))
        off += n
    master = [p.detach().float().clone() for p in ps]
    ms = [torch.zeros_like(p) for p in master]
    vs = [torch.zeros_like(p) for p in master]
    opt = FusedAdamW(ps, lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    for step in range(1, 4):
        gs = [torch.randn(p.shape, device=DEV).to(torch.bfloat16) for p in ps]
        for p, g in zip(ps, gs):
            p.grad = g.clone()
        opt.step()
        for p, g, m, v in zip(master, gs, ms, vs):
            ref.adamw_(p, g.float(), m, v, 1e-2, 0.9, 0.95, 1e-8, 0.1, step)
    for p, r in zip(ps, master):
        assert p.dtype == torch.bfloat16
        assert torch.allclose(opt.state[p]["master"], r, rtol=1e-5, atol=1e-6)
        assert torch.equal(p.detach(), r.to(torch.bfloat16))


def test_llama_tiny_train_step_hip():
    """End-to-end forward/backward/optimizer of the tiny Llama on the HIP path,
    checked against the same model on the fp32 CPU reference path."""
    from kgwe.models import llama

    torch.manual_seed(5)
    m_gpu = llama.build("tiny", device=DEV, dtype=torch.bfloat16)
    m_cpu = llama.build("tiny", device="cpu", dtype=torch.float32)
    m_cpu.load_state_dict({k: v.float().cpu() for k, v in m_gpu.state_dict().items()})
    tok = torch.randint(0, 1024, (2, 129))
    l_gpu = m_gpu(tok[:, :-1].to(DEV), tok[:, 1:].to(DEV))
    l_cpu = m_cpu(tok[:, :-1], tok[:, 1:])
    assert abs(l_gpu.item() - l_cpu.item()) < 0.05
    l_gpu.backward()
    for n, p in m_gpu.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad.float()).all(), n


def test_rope_rejects_out_of_contract_tables():
    """bf16 tables (e.g. cast by an FSDP MixedPrecisionPolicy) are converted,
    too-short tables are rejected on the host before any launch."""
    qkv = torch.randn(2 * 64, 8 * 128, device=DEV, dtype=torch.bfloat16)
    cos, sin = ref.rope_tables(64, 128, 500000.0, DEV)
    q1, _, _ = K.rope_qkv(qkv, cos.bfloat16(), sin.bfloat16(), 64, 4, 2, 128)
    q2, _, _ = K.rope_qkv(qkv, cos, sin, 64, 4, 2, 128)
    assert (q1.float() - q2.float()).abs().max().item() < 0.1
    with pytest.raises(ValueError):
        K.rope_qkv(qkv, cos[:10], sin[:10], 64, 4, 2, 128)


@pytest.mark.parametrize("parallel", ["zero", "fsdp"])
def test_single_rank_train_step(parallel):
    """The exact paths bench.py runs (1 rank, RCCL process group): sharded DP
    (default) and FSDP2, bf16 mixed precision + HIP ops + fused AdamW."""
    import torch.distributed as dist

    from kgwe.bench.train import TrainConfig, Trainer
    from kgwe.parallel import dist as kd

    info = kd.init(force_group=True)
    try:
        tr = Trainer(TrainConfig(model="tiny", seq_len=256, micro_batch=2, parallel=parallel,
                                 data="fixed"), info)
        losses = [tr.step().item() for _ in range(3)]
        assert all(torch.isfinite(torch.tensor(losses)))
        assert losses[-1] < losses[0]
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_fused_adamw_more_than_one_launch_batch():
    """37 tensors -> three launches of <= 16 by-value pointer records."""
    from kgwe.ops import FusedAdamW

    torch.manual_seed(8)
    shapes = [(17 * (i + 1) + (i % 3),) for i in range(37)] + [(70000,)]
    ps = [torch.randn(s, device=DEV, requires_grad=True) for s in shapes]
    pr = [p.detach().clone() for p in ps]
    ms = [torch.zeros_like(p) for p in pr]
    vs = [torch.zeros_like(p) for p in pr]
    opt = FusedAdamW(ps, lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    for step in range(1, 3):
        gs = [torch.randn_like(p) for p in ps]
        for p, g in zip(ps, gs):
            p.grad = g.clone()
        opt.step()
        for p, g, m, v in zip(pr, gs, ms, vs):
            ref.adamw_(p, g, m, v, 1e-2, 0.9, 0.95, 1e-8, 0.1, step)
    for p, r in zip(ps, pr):
        assert torch.allclose(p.detach(), r, rtol=1e-5, atol=1e-6)


def test_sharded_dp_overlapped_update_on_side_stream_matches_step_time_update():
    """AdamW issued per bucket from backward hooks on a side HIP stream gives
    the weights / optimizer state of the update run after backward.  Not
    bit-exact: the RMSNorm weight gradient is accumulated with fp32 atomics,
    so gradients differ in the last bits run to run; a race (weights read
    while being updated, a missed wait) moves whole tensors by ~lr instead."""
    from kgwe.models import llama
    from kgwe.parallel.zero import ShardedDataParallel

    tok = torch.randint(0, 1024, (2, 257), generator=torch.Generator().manual_seed(3)).to(DEV)
    runs = []
    for overlap in (True, False):
        torch.manual_seed(5)
        m = llama.build("tiny", device=DEV, dtype=torch.float32)
        dp = ShardedDataParallel(m, lr=1e-3, bucket_elems=1 << 19, overlap_step=overlap)
        assert len(dp.buckets) > 2
        for _ in range(3):
            loss = m(tok[:, :-1], tok[:, 1:])
            loss.backward()
            dp.step()
        dp.wait_params()
        torch.cuda.synchronize()
        # the persistent W^T copies (dgrad "nt" layout) track the updated weights
        assert sum(len(b.tparams) for b in dp.buckets) == 1 + 4 * 2  # output + 4 per block
        for b in dp.buckets:
            for p in b.tparams:
                assert torch.equal(p._kgwe_wt, p.detach().t()), p.shape
        runs.append([(b.master.clone(), b.m.clone(), b.v.clone(), b.flat.clone())
                     for b in dp.buckets])
    lr = 1e-3
    for i, (a, b) in enumerate(zip(*runs)):
        d = (a[0] - b[0]).abs()  # fp32 master
        assert d.mean().item() < 0.01 * lr, (i, d.mean().item())
        assert (d > 0.5 * lr).float().mean().item() < 0.01, i
        assert torch.allclose(a[1], b[1], rtol=1e-2, atol=1e-6)  # m
        fd = (a[3].float() - b[3].float()).abs()  # bf16 weights
        assert (fd > 0.5 * lr).float().mean().item() < 0.01, i


@pytest.mark.parametrize("shape", [(8192, 4096), (136, 72), (64, 8)])
def test_transpose_bf16(shape):
    x = torch.randn(*shape, device=DEV).to(torch.bfloat16)
    assert torch.equal(K.transpose(x), x.t().contiguous())


@pytest.mark.parametrize("N,Kd", [(6144, 512), (512, 1536), (1000, 64)])
def test_linear_layout_aware_backward_matches_fp32(N, Kd):
    """Weight gradient through the transposed-operand GEMMs ("tt" for N >= K,
    "nn" otherwise; odd sizes fall back to the plain layout) vs fp32."""
    torch.manual_seed(9)
    x = torch.randn(2, 256, Kd, device=DEV).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(N, Kd, device=DEV) * 0.05).to(torch.bfloat16).requires_grad_()
    y = K.linear(x, w)
    g = torch.randn_like(y)
    y.backward(g)
    xf, wf = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    yf = xf @ wf.t()
    yf.backward(g.float())
    assert torch.allclose(y.float(), yf, rtol=2e-2, atol=2e-2)
    for got, want in ((x.grad, xf.grad), (w.grad, wf.grad)):
        err = (got.float() - want).abs().max().item()
        assert err <= 2e-2 * want.abs().max().item() + 1e-2, err


@pytest.mark.parametrize("T,F,Kd", [(256, 512, 384), (128, 64, 64), (320, 1792, 256)])
def test_swiglu_backward_hands_its_transposed_gradient_to_the_projection(T, F, Kd, monkeypatch):
    """FFN up path x -> linear(w13) -> swiglu: the SwiGLU backward writes
    d(gate|up) and its transpose in one pass and the w13 weight gradient is
    computed from the transposed copy.  Gradients against an fp32 reference,
    bit-identical d(gate|up) with the plain backward, transposed copy exact,
    and nothing left on offer afterwards."""
    from kgwe.ops import functional as Fn

    torch.manual_seed(11)
    x = (torch.randn(T, Kd, device=DEV) * 0.5).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(2 * F, Kd, device=DEV) * 0.05).to(torch.bfloat16).requires_grad_()
    d = torch.randn(T, F, device=DEV).to(torch.bfloat16)

    def run(dual):
        monkeypatch.setenv("KGWE_DUAL_GRADS", "1" if dual else "0")
        x.grad = w.grad = None
        taken = []
        real = Fn._take_transposed

        def spy(dy2):
            t = real(dy2)
            if t is not None:
                taken.append((t.clone(), dy2.clone()))
            return t
        monkeypatch.setattr(Fn, "_take_transposed", spy)
        K.swiglu(K.linear(x, w)).backward(d)
        monkeypatch.setattr(Fn, "_take_transposed", real)
        return x.grad.clone(), w.grad.clone(), taken

    gx1, gw1, taken = run(True)
    assert len(taken) == 1 and not Fn._offered
    dy_t, dy = taken[0]
    assert dy_t.shape == (2 * F, T) and torch.equal(dy_t, dy.t().contiguous())
    gx0, gw0, none = run(False)
    assert not none
    assert torch.equal(gx1, gx0)                      # same d(gate|up), same dX GEMM
    xf, wf = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    gu = xf @ wf.t()
    (torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]).backward(d.float())
    for got in (gw1, gw0):
        err = (got.float() - wf.grad).abs().max().item()
        assert err <= 2e-2 * wf.grad.abs().max().item() + 1e-2, err
    # a shape the tiled kernel does not take falls back to the plain backward
    x2 = torch.randn(72, 64, device=DEV).to(torch.bfloat16).requires_grad_()
    w2 = (torch.randn(2 * 40, 64, device=DEV) * 0.05).to(torch.bfloat16).requires_grad_()
    monkeypatch.setenv("KGWE_DUAL_GRADS", "1")
    K.swiglu(K.linear(x2, w2)).sum().backward()
    assert not Fn._offered and torch.isfinite(w2.grad.float()).all()

