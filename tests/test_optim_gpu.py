"""rq_adamw_step (rqvae_hip.optim.AdamW) against torch.optim.AdamW, the optimizer the reference's loops
step (train_rqvae.py:96-100, train_decoder.py:151-160): ragged tensor sizes (chunk tails, 1-element
and exactly-one-chunk tensors), two parameter groups, several steps, state-dict layout."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SIZES = [(1,), (4096,), (4097,), (768, 512), (3, 256, 64), (129, 7)]


def _params(device, seed):
    g = torch.Generator(device=device).manual_seed(seed)
    return [torch.randn(s, device=device, generator=g) for s in SIZES]


@pytest.mark.parametrize("wd", [0.01, 0.0])
def test_adamw_matches_torch(device, wd):
    from rqvae_hip.optim import AdamW
    ref = [torch.nn.Parameter(t.clone()) for t in _params(device, 1)]
    got = [torch.nn.Parameter(t.clone()) for t in _params(device, 1)]
    groups = lambda ps, lr: [{"params": ps[:3], "lr": lr}, {"params": ps[3:], "lr": 3 * lr}]  # noqa: E731
    o_ref = torch.optim.AdamW(groups(ref, 1e-3), betas=(0.9, 0.995), eps=1e-8, weight_decay=wd, foreach=False)
    o_got = AdamW(groups(got, 1e-3), betas=(0.9, 0.995), eps=1e-8, weight_decay=wd)
    gen = torch.Generator(device=device).manual_seed(7)
    for _ in range(6):
        for a, b in zip(ref, got):
            gr = torch.randn(a.shape, device=device, generator=gen)
            a.grad = gr.clone()
            b.grad = gr.clone()
        o_ref.step()
        o_got.step()
    torch.cuda.synchronize()
    for a, b in zip(ref, got):
        torch.testing.assert_close(b.detach(), a.detach(), rtol=2e-6, atol=1e-7)
        sa, sb = o_ref.state[a], o_got.state[b]
        assert set(sb) == {"step", "exp_avg", "exp_avg_sq"} and float(sb["step"]) == float(sa["step"]) == 6
        # torch's single-tensor AdamW updates exp_avg with lerp, the kernel (like torch's fused AdamW) with
        # b1*m + (1-b1)*g: the two differ by ~1 ulp of the O(1) gradient scale, so the moment tolerances
        # are absolute at that scale
        torch.testing.assert_close(sb["exp_avg"], sa["exp_avg"], rtol=1e-6, atol=2e-7)
        torch.testing.assert_close(sb["exp_avg_sq"], sa["exp_avg_sq"], rtol=1e-6, atol=2e-7)


def test_adamw_skips_params_without_grad_and_rejects_cpu(device):
    from rqvae_hip import RqHipError
    from rqvae_hip.optim import AdamW
    a = torch.nn.Parameter(torch.ones(10, device=device))
    b = torch.nn.Parameter(torch.ones(5000, device=device))
    opt = AdamW([a, b], lr=0.1)
    b.grad = torch.ones_like(b)
    opt.step()
    torch.cuda.synchronize()
    assert torch.equal(a.detach(), torch.ones_like(a)) and len(opt.state[a]) == 0
    assert (b.detach() < 1).all()
    c = torch.nn.Parameter(torch.ones(3))
    c.grad = torch.ones(3)
    with pytest.raises(RqHipError):
        AdamW([c]).step()


def test_adamw_more_tensors_than_one_launch(device):
    """> 64 tensors (the per-launch segment table) plus re-allocated grads every step (set_to_none)."""
    from rqvae_hip.optim import AdamW
    g = torch.Generator(device=device).manual_seed(3)
    init = [torch.randn(int(n), device=device, generator=g) for n in torch.randint(1, 9000, (150,), generator=None)]
    ref = [torch.nn.Parameter(t.clone()) for t in init]
    got = [torch.nn.Parameter(t.clone()) for t in init]
    o_ref = torch.optim.AdamW(ref, lr=1e-2, weight_decay=0.01, foreach=False)
    o_got = AdamW(got, lr=1e-2, weight_decay=0.01)
    for _ in range(3):
        o_ref.zero_grad(set_to_none=True)
        o_got.zero_grad(set_to_none=True)
        for a, b in zip(ref, got):
            gr = torch.randn(a.shape, device=device, generator=g)
            a.grad = gr.clone()
            b.grad = gr.clone()
        o_ref.step()
        o_got.step()
    torch.cuda.synchronize()
    for a, b in zip(ref, got):
        # lr 1e-2: torch decays with p*(1 - lr*wd) (factor rounded in double), the kernel with p - (lr*wd)*p;
        # the two differ by a few ulp of |p| ~ 1
        torch.testing.assert_close(b.detach(), a.detach(), rtol=2e-6, atol=4e-7)
