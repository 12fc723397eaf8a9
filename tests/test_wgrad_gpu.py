"""Hand-written weight-gradient GEMM (native/ops/wgrad_gemm.hip) against an
fp32 PyTorch reference of the same product."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(dy, x):
    return dy.float().t() @ x.float()


@pytest.mark.parametrize("T,N,K,splits", [
    (320, 256, 256, 1), (448, 512, 256, 1),                      # 5 and 7 K-tiles
    (64, 256, 256, 1), (128, 256, 512, 1), (192, 512, 256, 1),   # odd K-tile count, both tile grids
    (1024, 768, 1280, 1), (1024, 768, 1280, 2), (1024, 768, 1280, 4),
    (4096, 1024, 512, 0),                                         # launcher-chosen split
])
def test_wgrad_matches_fp32_reference(T, N, K, splits):
    from kgwe.ops.gemm import wgrad

    g = torch.Generator(device="cuda").manual_seed(T + N + K)
    dy = torch.randn(T, N, device="cuda", generator=g).to(torch.bfloat16)
    x = torch.randn(T, K, device="cuda", generator=g).to(torch.bfloat16)
    got = wgrad(dy, x, splits=splits).float()
    ref = _ref(dy, x)
    # bf16 output rounding (2^-8 relative) on top of fp32 accumulation
    err = (got - ref).abs().max().item()
    assert err <= 2.0 ** -7 * ref.abs().max().item() + 1e-3, err
    assert torch.allclose(got, ref, rtol=2.0 ** -7, atol=0.02 * ref.abs().max().item())


def test_wgrad_exact_on_integers_and_asymmetric_operands():
    """A = identity-like selector with an asymmetric B: a swapped row / column
    map or a wrong token order inside a fragment shows up as wrong entries,
    which random data within tolerance could hide."""
    from kgwe.ops.gemm import wgrad

    T, N, K = 256, 256, 512
    dy = torch.zeros(T, N, device="cuda")
    dy[torch.arange(T), torch.arange(T)] = 1.0          # dW[n, :] = x[n, :] for n < T
    x = (torch.arange(T, device="cuda")[:, None] * 3 + torch.arange(K, device="cuda")[None, :] * 5) % 127
    got = wgrad(dy.to(torch.bfloat16), x.to(torch.bfloat16)).float()
    assert torch.equal(got, x.float())
    # every token weighted differently: the reduction over tokens is complete and in range
    w = (torch.arange(T, device="cuda") % 7 + 1).float()
    dy2 = w[:, None].expand(T, N).contiguous()
    x2 = ((torch.arange(T, device="cuda")[:, None] + torch.arange(K, device="cuda")[None, :]) % 5).float()
    got2 = wgrad(dy2.to(torch.bfloat16), x2.to(torch.bfloat16)).float()
    ref2 = (dy2.t() @ x2)
    assert torch.equal(got2, ref2.to(torch.bfloat16).float())


def test_wgrad_strided_rows_and_contract():
    from kgwe.ops.gemm import wgrad, wgrad_supported

    T, N, K = 512, 256, 256
    big = torch.randn(T, N + K + 64, device="cuda").to(torch.bfloat16)
    dy, x = big[:, :N], big[:, N:N + K]      # row stride 576: views of a fused activation
    assert wgrad_supported(dy, x)
    got = wgrad(dy, x).float()
    assert torch.allclose(got, _ref(dy, x), rtol=2.0 ** -7, atol=0.5)
    assert not wgrad_supported(dy[:, :200], x)                  # N % 256
    assert not wgrad_supported(dy[:100], x[:100])               # T % 64
    assert not wgrad_supported(dy.float(), x)                   # dtype
    with pytest.raises(ValueError):
        wgrad(dy[:, :200], x)


def test_linear_backward_uses_the_kernel_and_matches_autograd_reference():
    from kgwe.ops import functional as F

    torch.manual_seed(0)
    x = torch.randn(2, 256, 512, device="cuda").to(torch.bfloat16).requires_grad_()
    w = (torch.randn(768, 512, device="cuda") * 0.05).to(torch.bfloat16).requires_grad_()
    y = F.linear(x, w)
    gy = torch.randn_like(y)
    y.backward(gy)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().float().requires_grad_()
    (torch.nn.functional.linear(xr, wr) * gy.float()).sum().backward()
    assert torch.allclose(w.grad.float(), wr.grad, rtol=2.0 ** -6, atol=0.05 * wr.grad.abs().max().item())
    assert torch.allclose(x.grad.float(), xr.grad, rtol=2.0 ** -6, atol=0.05 * xr.grad.abs().max().item())
