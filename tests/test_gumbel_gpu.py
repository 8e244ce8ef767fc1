"""Training-mode GUMBEL_SOFTMAX + L2 quantize on rq_gumbel_softmax_fwd / _bwd (modules/quantize.py:107-129,
distributions/gumbel.py:14-18) against the torch composite of the reference math (RQ_GUMBEL_HIP=0 path),
with the same injected noise: ids exact on margin-safe rows, emb / loss / grads within fp32 tolerance. The
reference fixtures (tests/test_reference_fixtures_gpu.py::test_quantize_variant_vs_reference[gumbel*])
pin the same path against the reference itself."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,D,K,T,sim", [(1000, 32, 256, 0.5, False), (777, 64, 256, 0.2, False),
                                         (300, 16, 1000, 1.0, True), (65, 100, 64, 0.7, False)])
def test_gumbel_hip_vs_composite(device, monkeypatch, B, D, K, T, sim):
    import distributions.gumbel as gumbel
    import modules.quantize as mq
    from modules.quantize import Quantize, QuantizeForwardMode
    gen = torch.Generator().manual_seed(B + K)
    x0 = torch.randn(B, D, generator=gen)
    cb0 = torch.randn(K, D, generator=gen) * 0.7
    u = torch.rand(B, K, generator=gen)
    noise = (-torch.log(-torch.log(u + 1e-20) + 1e-20)).to(device)
    monkeypatch.setattr(gumbel, "sample_gumbel", lambda shape, device, eps=1e-20: noise.reshape(shape))
    g_emb = torch.randn(B, D, generator=gen).to(device)
    out = {}
    for hip in (True, False):
        monkeypatch.setattr(mq, "GUMBEL_HIP", hip)
        q = Quantize(D, K, do_kmeans_init=False, sim_vq=sim, forward_mode=QuantizeForwardMode.GUMBEL_SOFTMAX).to(device)
        with torch.no_grad():
            q.embedding.weight.copy_(cb0)
            if sim:
                q.out_proj[0].weight.copy_(torch.eye(D) * 0.9)
        q.train(True)
        x = x0.clone().to(device).requires_grad_(True)
        o = q(x, temperature=T)
        ((o.embeddings * g_emb).sum() + o.loss.sum()).backward()
        out[hip] = (o.ids.cpu(), o.embeddings.detach().cpu(), o.loss.detach().cpu(), x.grad.cpu(),
                    q.embedding.weight.grad.cpu())
    a, b = out[True], out[False]
    # fp64 truth of the forward from the same inputs and noise
    cb = (cb0 @ (torch.eye(D) * 0.9).t() if sim else cb0).double()
    xd = x0.double()
    dist = (xd ** 2).sum(1, keepdim=True) + (cb ** 2).sum(1)[None] - 2 * xd @ cb.t()
    w = torch.softmax((noise.cpu().double() - dist) / T, dim=1)
    emb64 = w @ cb
    # ids: exact where the two smallest distances are apart (fp32 dot orders differ between the paths)
    top2 = dist.topk(2, dim=1, largest=False).values
    safe = (top2[:, 1] - top2[:, 0]) > 1e-4 * top2[:, 0].abs().clamp_min(1.0)
    assert safe.float().mean() > 0.9
    assert torch.equal(a[0][safe], b[0][safe])
    assert torch.equal(a[0][safe], dist.argmin(1)[safe])
    # the HIP path is no further from fp64 than the torch composite (plus fp32 slack), and both agree
    e_hip = (a[1].double() - emb64).abs().max().item()
    e_ref = (b[1].double() - emb64).abs().max().item()
    print(f"emb max |err| vs fp64: hip {e_hip:.3e}, composite {e_ref:.3e}")
    assert e_hip <= 2 * e_ref + 1e-5, (e_hip, e_ref)
    for i, name in ((2, "loss"), (3, "grad_x"), (4, "grad_codebook")):
        d = (a[i] - b[i]).abs().max().item()
        m = b[i].abs().max().item()
        print(f"{name}: max |hip - composite| {d:.3e} (max |composite| {m:.3e})")
        assert d <= 1e-2 * m + 1e-6, (name, d, m)   # the reference fixtures pin these tighter
