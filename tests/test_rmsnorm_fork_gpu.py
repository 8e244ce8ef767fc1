"""RMSNorm fan-out node (ops.rmsnorm_fork: x -> norm_1(x) [dropout], [norm_2(x) [dropout]], x) and the
RMSNorm backward's fusions (rq_rmsnorm_dropout_bwd: residual gradient added in-kernel, weight grad
accumulated into a flat gradient bucket). Reference: modules/normalize.py:22-32 and the pre-norm block
of modules/transformer/model.py:75-82 (x feeds attn_norm, cross_attn_norm and the residual add).

Checks: the fork equals the composition of two ops.rmsnorm calls and the identity under the same
dropout keys — outputs bitwise, the input gradient within fp32 summation order of the three branch
gradients, weight gradients bitwise; direct accumulation into dp.GradBuckets flat views equals
plain autograd; rq_rmsnorm_dropout_bwd with gres == bwd + gres.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("two,p", [(True, 0.0), (True, 0.3), (False, 0.3)])
def test_rmsnorm_fork_equals_composition(device, two, p):
    from rqvae_hip import ops
    B, D = 3001, 512
    gen = torch.Generator(device=device).manual_seed(4)
    x = torch.randn(B, D, generator=gen, device=device)
    w1 = torch.randn(D, generator=gen, device=device).requires_grad_(True)
    w2 = torch.randn(D, generator=gen, device=device).requires_grad_(True)
    gs = [torch.randn(B, D, generator=gen, device=device) for _ in range(3)]

    def run(fork):
        for t in (w1, w2):
            t.grad = None
        xx = x.clone().requires_grad_(True)
        ops._SEED["n"] = 0
        if fork:
            outs = ops.rmsnorm_fork(xx, 1e-6, w1, p, w2 if two else None, p)
        else:
            outs = [ops.rmsnorm(xx, w1, 1e-6, p)] + ([ops.rmsnorm(xx, w2, 1e-6, p)] if two else []) + [xx]
        loss = sum((o * g).sum() for o, g in zip(outs, gs if two else [gs[0], gs[2]]))
        loss.backward()
        return [o.detach().clone() for o in outs], xx.grad.clone(), w1.grad.clone(), (w2.grad.clone() if two else None)

    of, gxf, g1f, g2f = run(True)
    oc, gxc, g1c, g2c = run(False)
    for a, b in zip(of, oc):
        assert torch.equal(a, b)
    assert torch.allclose(gxf, gxc, rtol=1e-6, atol=1e-6)
    assert torch.equal(g1f, g1c)
    if two:
        assert torch.equal(g2f, g2c)


def test_rmsnorm_bwd_gres_and_accumulate(device):
    from rqvae_hip import ops
    from rqvae_hip._lib import ptr, stream_handle
    B, D = 1000, 384
    gen = torch.Generator(device=device).manual_seed(6)
    x, gy, gres = (torch.randn(B, D, generator=gen, device=device) for _ in range(3))
    w = torch.randn(D, generator=gen, device=device)
    y = torch.empty_like(x)
    rstd = torch.empty(B, device=device)
    ops.call("rq_rmsnorm_dropout_fwd", ptr(x), ptr(w), B, D, 1e-6, 0.0, 0, ptr(y), ptr(rstd), stream_handle(device))
    nb = ops._lib.load().rq_rmsnorm_bwd_workspace(B, D)
    ws = torch.empty(nb, device=device, dtype=torch.uint8)
    gx0, gw0 = torch.empty_like(x), torch.empty(D, device=device)
    ops.call("rq_rmsnorm_dropout_bwd", ptr(x), ptr(w), ptr(rstd), ptr(gy), None, B, D, 0.0, 0, ptr(gx0), ptr(gw0), 0, 0,
             None, ptr(ws), nb, stream_handle(device))
    gx1 = torch.empty_like(x)
    gw1 = torch.randn(D, generator=gen, device=device)
    base = gw1.clone()
    ops.call("rq_rmsnorm_dropout_bwd", ptr(x), ptr(w), ptr(rstd), ptr(gy), ptr(gres), B, D, 0.0, 0, ptr(gx1), ptr(gw1), 1,
             0, None, ptr(ws), nb, stream_handle(device))
    assert torch.equal(gx1, gx0 + gres)
    assert torch.equal(gw1, base + gw0)


def test_fork_direct_grad_equals_autograd(device):
    from modules.transformer.model import TransformerBlock
    from ops.jagged import Jagged
    from rqvae_hip import dp, ops
    torch.set_float32_matmul_precision("high")
    try:
        torch.manual_seed(1)
        a = TransformerBlock(128, 128, 0.2, 4, False, [256], do_cross_attn=True, enable_kv_cache=False).to(device).train()
        b = copy.deepcopy(a)
        buckets = dp.GradBuckets(b.parameters(), overlap=False, flat_views=True)
        gen = torch.Generator(device=device).manual_seed(2)
        lens = torch.tensor([5, 1, 7, 3], device=device)
        klens = torch.tensor([9, 4, 2, 12], device=device)
        off = torch.cat([torch.zeros(1, dtype=torch.int64, device=device), lens.cumsum(0)])
        koff = torch.cat([torch.zeros(1, dtype=torch.int64, device=device), klens.cumsum(0)])
        xv = torch.randn(int(lens.sum()), 128, generator=gen, device=device)
        kv = torch.randn(int(klens.sum()), 128, generator=gen, device=device)
        g = torch.randn_like(xv)
        res = []
        for m in (a, b):
            if m is b:
                buckets.zero_grad()
            ops._SEED["n"] = 0
            jx = Jagged(xv.clone(), off, int(lens.max()))
            jk = Jagged(kv.clone(), koff, int(klens.max()))
            out = m._forward_jagged(jx, jk, True).values()
            out.backward(g)
            res.append(out.detach())
        buckets.synchronize()
        assert torch.equal(res[0], res[1])
        for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
            if pa.grad is None:
                assert pb.grad is None, n
            else:
                assert torch.equal(pa.grad, pb.grad), n
    finally:
        torch.set_float32_matmul_precision("highest")


@pytest.mark.parametrize("p1,p2,B,D", [(0.0, 0.0, 3001, 512), (0.3, 0.3, 2049, 384), (0.1, 0.5, 40, 384)])
@pytest.mark.parametrize("buckets", [False, True])
def test_rmsnorm_fork_dual_kernel_bitwise(device, monkeypatch, p1, p2, B, D, buckets):
    """The fork's two norms in one launch each way (rq_rmsnorm2_dropout_fwd / _bwd) vs the chained single-norm
    launches: outputs, the input gradient (norm2'(g2) + (norm1'(g1) + g_pass)) and both weight gradients
    bitwise — returned to autograd, or added into flat gradient-bucket views through the deferred reduction."""
    from rqvae_hip import dp, ops
    gen = torch.Generator(device=device).manual_seed(11)
    x = torch.randn(B, D, generator=gen, device=device)
    w1 = torch.nn.Parameter(torch.randn(D, generator=gen, device=device))
    w2 = torch.nn.Parameter(torch.randn(D, generator=gen, device=device))
    gs = [torch.randn(B, D, generator=gen, device=device) for _ in range(3)]
    gb = dp.GradBuckets([w1, w2], flat_views=True) if buckets else None
    res = {}
    for dual in (True, False):
        monkeypatch.setattr(ops, "_RMS_DUAL", dual)
        if gb is not None:
            gb.zero_grad()
        else:
            w1.grad = w2.grad = None
        xx = x.clone().requires_grad_(True)
        ops._SEED["n"] = 0
        outs = ops.rmsnorm_fork(xx, 1e-6, w1, p1, w2, p2)
        sum((o * g).sum() for o, g in zip(outs, gs)).backward()
        if gb is not None:
            ops.flush_reductions()
        res[dual] = [o.detach().clone() for o in outs] + [xx.grad.clone(), w1.grad.clone(), w2.grad.clone()]
    for a, b in zip(res[True], res[False]):
        assert torch.equal(a, b)
