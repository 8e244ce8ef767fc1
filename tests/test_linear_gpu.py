"""Split-K weight-gradient kernel (rq_linear_wgrad) vs an fp64 torch reference, and the
modules.linear.Linear drop-in vs torch.nn.Linear (same parameters, same gradients within fp32
tolerance). Tolerance: |err| <= 1e-5 * sum_b |g_b||x_b| per element (fp32 accumulation of up to
65,536 products)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(g, x):
    return (g.double().t() @ x.double()), g.double().sum(0)


def _bound(g, x):
    return g.double().abs().t() @ x.double().abs()


@pytest.mark.parametrize("N,O,I", [(65536, 512, 768), (65536, 64, 128), (4097, 256, 132), (37, 8, 12), (1, 4, 4),
                                   (3000, 768, 512)])
def test_wgrad_matches_fp64(device, N, O, I):
    from rqvae_hip import ops
    gen = torch.Generator(device=device).manual_seed(N + O + I)
    g = torch.randn(N, O, generator=gen, device=device)
    x = torch.randn(N, I, generator=gen, device=device)
    dW, db = ops.linear_wgrad(g, x, True)
    rW, rb = _ref(g, x)
    tol = 1e-5 * _bound(g, x) + 1e-6
    assert ((dW.double() - rW).abs() <= tol).all()
    assert ((db.double() - rb).abs() <= 1e-5 * g.double().abs().sum(0) + 1e-6).all()
    dW2, db2 = ops.linear_wgrad(g, x, True)
    assert torch.equal(dW, dW2) and torch.equal(db, db2), "fixed-order reduction must be bitwise repeatable"


def test_wgrad_empty_batch(device):
    from rqvae_hip import ops
    g = torch.empty(0, 8, device=device)
    x = torch.empty(0, 12, device=device)
    dW, db = ops.linear_wgrad(g, x, True)
    assert dW.shape == (8, 12) and not dW.any() and not db.any()


@pytest.mark.parametrize("bias", [False, True])
def test_linear_module_matches_nn_linear(device, bias):
    """Same gradients as torch.nn.Linear in fp64 (scale-aware fp32 tolerance: 1e-5 * max |ref|)."""
    from modules.linear import Linear
    torch.manual_seed(0)
    ref = torch.nn.Linear(96, 64, bias=bias).to(device).double()
    mine = Linear(96, 64, bias=bias).to(device)
    mine.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    x = torch.randn(5, 700, 96, device=device)   # >= WGRAD_MIN_ROWS rows
    x64 = x.double().requires_grad_(True)
    x32 = x.clone().requires_grad_(True)
    (ref(x64).sin().sum()).backward()
    (mine(x32).sin().sum()).backward()

    def close(a, b):
        return (a.double() - b).abs().max() <= 1e-5 * b.abs().max() + 1e-6
    assert close(x32.grad, x64.grad)
    assert close(mine.weight.grad, ref.weight.grad)
    if bias:
        assert close(mine.bias.grad, ref.bias.grad)


def test_mlp_uses_wgrad_kernel(device):
    """The RQ-VAE encoder MLP routes its weight gradients through the HIP kernel."""
    from modules.encoder import MLP
    from rqvae_hip import ops
    calls = []
    orig = ops.linear_wgrad

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)
    ops.linear_wgrad = spy
    try:
        m = MLP(768, [512, 256, 128], 64).to(device)
        m(torch.randn(2048, 768, device=device)).square().sum().backward()
    finally:
        ops.linear_wgrad = orig
    assert len(calls) == 4
