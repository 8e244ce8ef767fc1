"""Row-norm and loss-mean kernels of RqVae.forward's statistics (rq_row_norms, rq_loss_means) on
every lane grouping (D/4 lanes per row) and ragged lengths (vector body + scalar tail)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,D", [(196608, 64), (1000, 32), (7, 4), (513, 96), (300, 768), (5, 1028)])
def test_row_norms(device, rows, D):
    from rqvae_hip import ops
    x = torch.randn(rows, D, device=device, generator=torch.Generator(device=device).manual_seed(rows + D))
    got = ops.row_norms(x)
    ref = x.double().norm(dim=1)
    assert ((got.double() - ref).abs() <= 2e-6 * ref + 1e-7).all()


@pytest.mark.parametrize("B", [65536, 65537, 3, 1, 4097])
def test_loss_means(device, B):
    from rqvae_hip import ops
    g = torch.Generator(device=device).manual_seed(B)
    r = torch.rand(B, device=device, generator=g)
    q = torch.rand(B, device=device, generator=g)
    loss, rm, qm = ops.loss_means(r, q)
    for got, ref in ((loss, (r.double() + q.double()).mean()), (rm, r.double().mean()), (qm, q.double().mean())):
        assert abs(float(got) - float(ref)) <= 1e-6 * abs(float(ref)) + 1e-7
    again = ops.loss_means(r, q)
    assert all(torch.equal(a, b) for a, b in zip((loss, rm, qm), again)), "fixed-order reduction"


def _loss_means_order(r, q):
    """numpy fp32 restatement of loss_means_kernel's fixed order: thread t of 1024 sums float4 groups t, t + 1024, ...
    (each group ((r.x + q.x) + (r.y + q.y)) + ...), then element 4 (B // 4) + t of the tail, then the pairwise
    tree red[t] += red[t + o], o = 512 .. 1; each mean = total / B."""
    B = r.size
    n4 = B // 4
    acc = np.zeros((3, 1024), np.float32)
    rg, qg = r[:4 * n4].reshape(n4, 4), q[:4 * n4].reshape(n4, 4)
    for k in range(0, n4, 1024):
        m = min(1024, n4 - k)
        R, Q = rg[k:k + m], qg[k:k + m]
        s = R[:, 0] + Q[:, 0]
        for j in range(1, 4):
            s = s + (R[:, j] + Q[:, j])
        sr = R[:, 0] + R[:, 1] + R[:, 2] + R[:, 3]
        sq = Q[:, 0] + Q[:, 1] + Q[:, 2] + Q[:, 3]
        acc[0, :m] += s
        acc[1, :m] += sr
        acc[2, :m] += sq
    tail = B - 4 * n4
    for t in range(tail):
        rv, qv = r[4 * n4 + t], q[4 * n4 + t]
        acc[0, t] += rv + qv
        acc[1, t] += rv
        acc[2, t] += qv
    o = 512
    while o > 0:
        acc[:, :o] = acc[:, :o] + acc[:, o:2 * o]
        o //= 2
    return acc[:, 0] / np.float32(B)


@pytest.mark.parametrize("B", [65536, 65537, 4097, 40960, 3])
def test_loss_means_order(device, B):
    """rq_loss_means against a numpy restatement of its summation order: bitwise."""
    from rqvae_hip import ops
    g = torch.Generator(device=device).manual_seed(7 * B)
    r = torch.rand(B, device=device, generator=g)
    q = torch.rand(B, device=device, generator=g)
    got = torch.stack(ops.loss_means(r, q)).cpu().numpy()
    ref = _loss_means_order(r.cpu().numpy(), q.cpu().numpy())
    assert np.array_equal(got.view(np.uint32), ref.astype(np.float32).view(np.uint32)), (got, ref)


@pytest.mark.parametrize("B", [65536, 65537, 3, 1])
def test_loss_means_backward(device, B):
    """LossMeansFunction.backward when only the total loss has a gradient (rq_loss_means_bwd, one launch):
    bitwise torch's (g / B).expand(B) for both inputs; with the logged means also differentiated, the torch
    composite."""
    from rqvae_hip import ops
    gen = torch.Generator(device=device).manual_seed(B + 1)
    for scale in (1.0, 0.37, 3.0):
        r = torch.rand(B, device=device, generator=gen).requires_grad_(True)
        q = torch.rand(B, device=device, generator=gen).requires_grad_(True)
        loss, rm, qm = ops.loss_means(r, q)
        g = torch.tensor(scale, device=device)
        loss.backward(g)
        want = (g / B).expand(B)
        assert torch.equal(r.grad, want) and torch.equal(q.grad, want)
        r.grad = q.grad = None
        loss, rm, qm = ops.loss_means(r, q)
        (loss * scale + rm).backward()
        torch.testing.assert_close(r.grad, torch.full((B,), (scale + 1.0) / B, device=device), rtol=1e-6, atol=0)
        torch.testing.assert_close(q.grad, torch.full((B,), scale / B, device=device), rtol=1e-6, atol=0)
