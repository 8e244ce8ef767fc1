"""Split-bf16 GEMM (rq_gemm_bf16x3): the fp32 matmul at PyTorch's 'high' precision, which the
reference selects at import (modules/rqvae.py:19, modules/model.py:27).

Checks, for every operand layout the Linear layers use (forward x W^T, data grad g W, weight grad
g^T x) and ragged / split-K shapes:
  * small-integer operands (exact in bf16, so lo = 0 and every fp32 partial sum is exact) must give
    the fp64 result bit for bit — catches any fragment / swizzle / C-map error exactly;
  * random operands within |err| <= 3e-5 * sum_k |A(m,k)| |B(n,k)| + 1e-6 of fp64 (per-product
    relative error of the split is <= ~2^-17 ~ 7.6e-6; TF32, the other 'high' form, is 2^-11);
  * bitwise repeatability (fixed-order split-K reduction).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(256, 256, 64), (65536, 512, 768), (300, 132, 200), (4, 4, 4), (12, 8, 36), (768, 512, 65536),
          (132, 260, 4100), (64, 128, 65536), (768, 512, 4099)]


def _operands(M, N, K, a_kc, b_kc, gen, device, integer):
    def make(r, c):
        if integer:
            return torch.randint(-8, 9, (r, c), generator=gen, device=device).float()
        return torch.randn(r, c, generator=gen, device=device)
    a = make(M, K) if a_kc else make(K, M)
    b = make(N, K) if b_kc else make(K, N)
    A = a if a_kc else a.t()
    B = b if b_kc else b.t()
    return a, b, A.double(), B.double()


@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, False), (False, True)])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_bf16x3_exact_on_integers(device, a_kc, b_kc, M, N, K):
    if (a_kc or b_kc) and K % 4:
        pytest.skip("k-contiguous operands need K % 4 == 0")
    from rqvae_hip import ops
    if M * N * K > 2 ** 33:
        pytest.skip("large shape: random-data test covers it")
    gen = torch.Generator(device=device).manual_seed(M * 7 + N * 3 + K)
    a, b, A, B = _operands(M, N, K, a_kc, b_kc, gen, device, True)
    C = ops.gemm_bf16x3(a, a_kc, b, b_kc, M, N, K)
    ref = A @ B.t()
    assert torch.equal(C.double(), ref), (C.double() - ref).abs().max()


@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, False)])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_bf16x3_random_within_bound(device, a_kc, b_kc, M, N, K):
    from rqvae_hip import ops
    if (a_kc or b_kc) and K % 4:
        pytest.skip("k-contiguous operands need K % 4 == 0")
    gen = torch.Generator(device=device).manual_seed(M + N + K)
    a, b, A, B = _operands(M, N, K, a_kc, b_kc, gen, device, False)
    C = ops.gemm_bf16x3(a, a_kc, b, b_kc, M, N, K)
    ref = A @ B.t()
    bound = 3e-5 * (A.abs() @ B.abs().t()) + 1e-6
    err = (C.double() - ref).abs()
    assert (err <= bound).all(), float((err / bound).max())
    C2 = ops.gemm_bf16x3(a, a_kc, b, b_kc, M, N, K)
    assert torch.equal(C, C2)


def test_gemm_bf16x3_zero_k(device):
    from rqvae_hip import ops
    a = torch.empty(8, 0, device=device)
    b = torch.empty(12, 0, device=device)
    C = ops.gemm_bf16x3(a, True, b, True, 8, 12, 0)
    assert C.shape == (8, 12) and not C.any()


@pytest.mark.parametrize("rows", [1, 37, 1237, 65535])
def test_gemm_bf16x3_ragged_rows(device, rows):
    """Row counts of any size (the batch axis): forward / data grad have M = rows (k-contiguous A),
    the weight grad K = rows (row-major operands) — exact on small integers."""
    from rqvae_hip import ops
    gen = torch.Generator(device=device).manual_seed(rows)
    x = torch.randint(-8, 9, (rows, 132), generator=gen, device=device).float()
    W = torch.randint(-8, 9, (68, 132), generator=gen, device=device).float()
    g = torch.randint(-8, 9, (rows, 68), generator=gen, device=device).float()
    assert torch.equal(ops.linear_fwd_high(x, W).double(), x.double() @ W.double().t())
    assert torch.equal(ops.linear_dgrad_high(g, W).double(), g.double() @ W.double())
    assert torch.equal(ops.linear_wgrad_high(g, x).double(), g.double().t() @ x.double())


def test_gemm_bf16x3_rejects_bad_shapes(device):
    from rqvae_hip import ops
    from rqvae_hip._lib import RqHipError
    a = torch.randn(6, 10, device=device)
    b = torch.randn(8, 10, device=device)
    with pytest.raises(RqHipError):
        ops.gemm_bf16x3(a, True, b, True, 6, 8, 10)


@pytest.mark.parametrize("bias", [False, True])
def test_linear_high_precision_matches_fp64(device, bias):
    """modules.linear.Linear under 'high': forward, input grad and weight grad within the split-bf16
    bound of an fp64 nn.Linear."""
    from modules.linear import Linear
    torch.manual_seed(0)
    ref = torch.nn.Linear(96, 64, bias=bias).to(device).double()
    mine = Linear(96, 64, bias=bias).to(device)
    mine.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    x = torch.randn(5, 700, 96, device=device)
    x64 = x.double().requires_grad_(True)
    x32 = x.clone().requires_grad_(True)
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("high")
    try:
        y32 = mine(x32)
        (y32.sin().sum()).backward()
    finally:
        torch.set_float32_matmul_precision(prev)
    y64 = ref(x64)
    (y64.sin().sum()).backward()

    def close(a, b, tol):
        return (a.double() - b).abs().max() <= tol * b.abs().max() + 1e-6
    assert close(y32, y64, 1e-4)
    assert close(x32.grad, x64.grad, 1e-4)
    assert close(mine.weight.grad, ref.weight.grad, 1e-4)
    if bias:
        assert close(mine.bias.grad, ref.bias.grad, 1e-5)


def test_rqvae_step_high_vs_highest(device):
    """The RQ-VAE train step (ML-32M dims) at 'high' (split-bf16 MLP matmuls) against the same step
    at 'highest': loss within 1e-4 relative, MLP gradients within 3 % in norm (dominated by the items whose ids flip), codebook
    gradients within 5 % in norm, and the semantic ids of >= 99 % of the items identical (near-ties may flip under a 2^-17 perturbation,
    as they do between TF32 and fp32 in the reference)."""
    import bench
    from data.schemas import SeqBatch
    m = bench.build_model(device)
    x = bench.make_items(4096, 768, torch.Generator(device=device).manual_seed(4), device)
    res = {}
    for prec in ("highest", "high"):
        torch.set_float32_matmul_precision(prec)
        m.zero_grad(set_to_none=True)
        out = m(SeqBatch(None, None, None, x, None, None), gumbel_t=0.2)
        out.loss.backward()
        with torch.no_grad():
            ids = m.get_semantic_ids(x).sem_ids
        res[prec] = (float(out.loss), {k: p.grad.clone() for k, p in m.named_parameters()}, ids)
    torch.set_float32_matmul_precision("highest")
    (l0, g0, i0), (l1, g1, i1) = res["highest"], res["high"]
    assert abs(l1 - l0) <= 1e-4 * abs(l0), (l0, l1)
    agree = float((i0 == i1).all(1).float().mean())
    assert agree >= 0.99, agree
    for k in g0:
        if k.startswith("layers."):
            # a codeword's gradient sums its assigned items: an id flip moves an item's whole
            # contribution, so compare in norm (the flips are <= 1 % of the items)
            assert (g1[k] - g0[k]).norm() <= 0.05 * g0[k].norm(), k
        else:   # flipped items also change their encoder / decoder gradient paths
            assert (g1[k] - g0[k]).norm() <= 3e-2 * g0[k].norm(), k
