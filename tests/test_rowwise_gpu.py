"""Fused decoder-head kernel (l2norm + reconstruction loss, fwd + bwd) vs the plain PyTorch fp32
composite of the reference's ops (modules/normalize.py:7-8 + modules/loss.py:5-10).
Tolerance: rtol 1e-5 / atol 1e-6 on recon, rtol 1e-4 / atol 1e-7 on the gradient."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,C", [(65536, 768), (7, 96), (3, 4), (1000, 1024), (33, 4096)])
def test_l2norm_recon_vs_torch(device, B, C):
    from rqvae_hip import ops
    g = torch.Generator(device=device).manual_seed(B + C)
    pre = torch.randn(B, C, generator=g, device=device)
    pre[0] = 0.0                                   # clamped row (|pre| < eps)
    x = F.normalize(torch.randn(B, C, generator=g, device=device), dim=-1)
    gr = torch.rand(B, generator=g, device=device)
    a = pre.clone().requires_grad_(True)
    r = ops.l2norm_recon_loss(a, x)
    (r * gr).sum().backward()
    b = pre.clone().requires_grad_(True)
    rr = ((F.normalize(b, p=2, dim=-1, eps=1e-12) - x) ** 2).sum(-1)
    (rr * gr).sum().backward()
    assert torch.allclose(r, rr, rtol=1e-5, atol=1e-6)
    assert torch.allclose(a.grad, b.grad, rtol=1e-4, atol=1e-7)
    assert torch.isfinite(a.grad).all()


@pytest.mark.parametrize("B,C", [(65537, 768), (5, 96), (3, 4), (1001, 1024), (9, 1000)])
def test_l2norm_recon_ragged_vs_fp64(device, B, C):
    """Ragged row counts (a partly filled last workgroup) and widths (a partial float4 vector per lane) with a
    zero row (the F.normalize eps path): reconstruction loss and input gradient vs the fp64 composition
    (modules/rqvae.py:145-150 with modules/loss.py:5-10), and bitwise repeatable."""
    from rqvae_hip import ops
    g = torch.Generator(device=device).manual_seed(B * 3 + C)
    pre = torch.randn(B, C, generator=g, device=device)
    pre[-1] = 0.0
    x = F.normalize(torch.randn(B, C, generator=g, device=device), dim=-1)
    gr = torch.rand(B, generator=g, device=device)
    outs = []
    for _ in range(2):
        a = pre.clone().requires_grad_(True)
        r = ops.l2norm_recon_loss(a, x)
        (r * gr).sum().backward()
        outs.append((r.detach(), a.grad))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    p64 = pre.double().requires_grad_(True)
    r64 = ((F.normalize(p64, dim=-1, eps=1e-12) - x.double()) ** 2).sum(-1)
    (r64 * gr.double()).sum().backward()
    assert torch.allclose(outs[0][0].double(), r64.detach(), rtol=1e-5, atol=1e-6)
    assert torch.allclose(outs[0][1].double(), p64.grad, rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("shape", [(11000, 512), (7, 128), (3, 5, 4096), (1, 4), (0, 64)])
def test_rmsnorm_fused_matches_fp64(device, shape):
    """Fused RMSNorm vs the reference formula (modules/normalize.py:22-32) in fp64.
    Tolerance: y, gx 2e-5 * max|ref|; gw 2e-5 * sum_b |gy x rstd| (fp32 row sums)."""
    from modules.normalize import RMSNorm
    from rqvae_hip import ops
    D = shape[-1]
    gen = torch.Generator(device=device).manual_seed(D + len(shape))
    x = torch.randn(*shape, generator=gen, device=device) * 3
    m = RMSNorm(D).to(device)
    with torch.no_grad():
        m.weight.copy_(1 + 0.1 * torch.randn(D, generator=gen, device=device))
    assert ops.rmsnorm_supported(x, m.weight)
    xr = x.clone().requires_grad_(True)
    y = m(xr)
    gy = torch.randn(*shape, generator=gen, device=device)
    (y * gy).sum().backward()
    x64 = x.double().requires_grad_(True)
    w64 = m.weight.detach().double().requires_grad_(True)
    y64 = x64 * torch.rsqrt(x64.pow(2).mean(-1, keepdim=True) + m.eps) * w64
    (y64 * gy.double()).sum().backward()
    if x.numel() == 0:
        assert y.shape == x.shape and not m.weight.grad.any()
        return
    def ok(a, b, scale):
        return ((a.double() - b).abs() <= 2e-5 * scale + 1e-7).all()
    assert ok(y, y64, y64.abs().max())
    assert ok(xr.grad, x64.grad, x64.grad.abs().max())
    r = torch.rsqrt(x.double().pow(2).mean(-1, keepdim=True) + m.eps)
    assert ok(m.weight.grad, w64.grad, (gy.double() * x.double() * r).abs().reshape(-1, D).sum(0))
