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
