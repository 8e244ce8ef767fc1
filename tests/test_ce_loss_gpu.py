"""Fused decoder loss head (rq_ce_loss_fwd / rq_ce_loss_bwd, ops.CrossEntropyLossFunction) against the
reference's torch composition (modules/model.py:137-143): logits = X.view(B, npos + 1, K)[:, :-1].flatten(0, 1),
unred = cross_entropy(logits, tgt, reduction='none', ignore_index=-1), loss = unred.sum(1).mean(),
loss_d = unred.mean(0) — values and the gradient of X through all three outputs, with ignored targets;
bitwise repeatable."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,npos,K", [(256, 5, 256), (8, 5, 256), (3, 2, 1000), (1, 1, 64)])
def test_ce_loss_matches_torch(device, B, npos, K):
    from rqvae_hip import ops
    g = torch.Generator(device=device).manual_seed(B * 7 + K)
    X0 = torch.randn(B * (npos + 1), K, generator=g, device=device) * 3
    tgt = torch.randint(0, K, (B, npos), generator=g, device=device)
    tgt[0, -1] = -1                      # ignore_index
    if B > 2:
        tgt[2, 0] = -1
    w_d = torch.randn(npos, generator=g, device=device)
    w_l = torch.randn(B * npos, K, generator=g, device=device) * 0.01

    def run(fused):
        X = X0.clone().requires_grad_(True)
        if fused:
            loss, loss_d, logits = ops.cross_entropy_loss(X, tgt, B)
        else:
            logits = X.view(B, -1, K)[:, :-1, :].flatten(end_dim=1)
            unred = F.cross_entropy(logits, tgt.flatten(), reduction="none", ignore_index=-1).view(B, -1)
            loss, loss_d = unred.sum(axis=1).mean(), unred.mean(axis=0)
        (loss + (loss_d * w_d).sum() + (logits * w_l).sum()).backward()
        return loss.detach(), loss_d.detach(), logits.detach(), X.grad
    f, r = run(True), run(False)
    torch.testing.assert_close(f[0], r[0], rtol=2e-6, atol=1e-6)
    torch.testing.assert_close(f[1], r[1], rtol=2e-6, atol=1e-6)
    assert torch.equal(f[2], r[2])
    torch.testing.assert_close(f[3], r[3], rtol=1e-5, atol=1e-7)
    f2 = run(True)
    assert all(torch.equal(a, b) for a, b in zip(f, f2))
