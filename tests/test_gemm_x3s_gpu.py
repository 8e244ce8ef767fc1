"""64 x 64-tile form of the split-bf16 GEMM (gemm_bf16x3_kernel<..., TS = 64>), the kernel the planner
picks where 128-tiles cannot fill the chip (the decoder's 1,280 future-token rows, their weight grads).

* small-integer operands (exact in bf16, every fp32 partial sum exact) give the fp64 product bit for
  bit for all four layouts, fp32 and pre-split operands, partial tiles and split-K;
* with the same split the 64- and 128-tile kernels run the same 32-deep k steps in the same product
  order, so they agree BITWISE — including the fused epilogues (SiLU fwd / bwd with dropout,
  residual add) and accumulation into an existing output;
* the planner selects it for the decoder's 1,280-row shapes.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

LAYOUTS = [(True, True), (True, False), (False, True), (False, False)]
# (M, N, K): decoder future rows (fwd / dgrad), their weight grads (split-K over 1,280 rows),
# ragged partial tiles, a deep-K single tile
SHAPES = [(1280, 512, 512), (512, 512, 1280), (1288, 520, 96), (200, 136, 3000), (64, 64, 64)]


def _ops():
    from rqvae_hip import ops
    return ops


@pytest.fixture
def small_on():
    ops = _ops()
    with ops.gemm_policy(ops.GEMM_ONLY_64):   # forced (and never the wide kernel) for every call inside
        yield ops


def _mk(M, N, K, a_kc, b_kc, gen, device, integer):
    def make(r, c):
        if integer:
            return torch.randint(-8, 9, (r, c), generator=gen, device=device).float()
        return torch.randn(r, c, generator=gen, device=device)
    a = make(M, K) if a_kc else make(K, M)
    b = make(N, K) if b_kc else make(K, N)
    return a, b


# operand formats the plain-store dispatch builds (rq_gemm_bf16x3_run): every fp32 layout, and the
# split / mixed layouts the fused chains use
BUILT = {(ak, bk, False, False) for ak in (True, False) for bk in (True, False)} | {
    (True, True, True, True), (True, True, False, True), (True, False, True, True), (True, False, False, True),
    (False, False, True, True), (False, False, True, False), (False, False, False, True)}


@pytest.mark.parametrize("split", [(False, False), (True, True), (False, True)])
@pytest.mark.parametrize("a_kc,b_kc", LAYOUTS)
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_x3s_exact_on_integers(device, small_on, a_kc, b_kc, M, N, K, split):
    ops = small_on
    asp, bsp = split
    if (a_kc, b_kc, asp, bsp) not in BUILT:
        pytest.skip("operand combination not instantiated")
    kern, S = ops.gemm_x3_choice(M, N, K, asp, bsp, a_kc, b_kc)
    assert kern == "x3s", (M, N, K)
    gen = torch.Generator(device=device).manual_seed(M + 5 * N + 11 * K + 2 * a_kc + b_kc)
    a, b = _mk(M, N, K, a_kc, b_kc, gen, device, True)
    C = ops.gemm_x3(ops.split_bf16x3(a) if asp else a, a_kc, ops.split_bf16x3(b) if bsp else b, b_kc, M, N, K)
    A = (a if a_kc else a.t()).double()
    B = (b if b_kc else b.t()).double()
    bad = C.double() != A @ B.t()
    assert not bad.any(), (int(bad.sum()), bad.nonzero()[:8].tolist(), S)


def _both(ops, fn):
    """fn() under the 64-tile kernel and under the 128-tile kernel."""
    with ops.gemm_policy(ops.GEMM_ONLY_64):
        s = fn()
    with ops.gemm_policy(ops.GEMM_ONLY_128):
        o = fn()
    return s, o


@pytest.mark.parametrize("a_kc,b_kc", LAYOUTS)
def test_x3s_random_bitwise_equal_x3(device, small_on, a_kc, b_kc):
    """No split-K in either kernel at 4,096 rows: identical k order, identical bits; plus the
    split-bf16 bound against fp64."""
    ops = small_on
    M, N, K = 4096, 512, 256
    assert ops.gemm_x3_choice(M, N, K, False, False, a_kc, b_kc)[1] == 1
    with ops.gemm_policy(ops.GEMM_ONLY_128):
        assert ops.gemm_x3_choice(M, N, K, False, False, a_kc, b_kc)[1] == 1
    gen = torch.Generator(device=device).manual_seed(7 + 2 * a_kc + b_kc)
    a, b = _mk(M, N, K, a_kc, b_kc, gen, device, False)
    cs, co = _both(ops, lambda: ops.gemm_x3(a, a_kc, b, b_kc, M, N, K))
    assert torch.equal(cs, co)
    A = (a if a_kc else a.t()).double()
    B = (b if b_kc else b.t()).double()
    err = (cs.double() - A @ B.t()).abs()
    assert (err <= 3e-5 * (A.abs() @ B.abs().t()) + 1e-6).all()


@pytest.mark.parametrize("p", [0.0, 0.3])
def test_x3s_fused_epilogues_equal_x3(device, small_on, p):
    ops = small_on
    M, K, N = 16384, 512, 512   # neither kernel splits K here
    gen = torch.Generator(device=device).manual_seed(11)
    x32 = torch.randn(M, K, generator=gen, device=device)
    W = ops.split_bf16x3(torch.randn(N, K, generator=gen, device=device) * 0.05)
    (zs, hs), (zo, ho) = _both(ops, lambda: ops.gemm_x3(x32, True, W, True, M, N, K, ops.EPI_SILU_FWD, p=p, seed=5))
    assert torch.equal(zs, zo) and torch.equal(hs.hi, ho.hi) and torch.equal(hs.lo, ho.lo)
    g = ops.split_bf16x3(torch.randn(M, N, generator=gen, device=device))
    Z = torch.randn(M, K, generator=gen, device=device)
    bs, bo = _both(ops, lambda: ops.gemm_x3(g, True, W, False, M, K, N, ops.EPI_SILU_BWD, Z=Z, p=p, seed=6))
    assert torch.equal(bs.hi, bo.hi) and torch.equal(bs.lo, bo.lo)
    r = torch.randn(M, N, generator=gen, device=device)
    as_, ao = _both(ops, lambda: ops.gemm_x3(x32, True, W, True, M, N, K, ops.EPI_ADD, Z=r))
    assert torch.equal(as_, ao)


def test_x3s_split_k_epilogue_and_accumulate(device, small_on):
    """Split-K through the slab reduction with the SiLU epilogue and with accumulation (weight grads
    added into a flat gradient bucket): against the same call computed unsplit in fp64-exact integers."""
    ops = small_on
    gen = torch.Generator(device=device).manual_seed(12)
    M, N, K = 512, 512, 1280
    a, b = _mk(M, N, K, False, False, gen, device, True)
    kern, S = ops.gemm_x3_choice(M, N, K, False, False, False, False)
    assert kern == "x3s" and S > 1
    base = torch.randint(-8, 9, (M, N), generator=gen, device=device).float()
    out = base.clone()
    ops.gemm_x3(a, False, b, False, M, N, K, out=out, accumulate=True)
    ref = base.double() + a.t().double() @ b.double()
    assert torch.equal(out.double(), ref)


def test_x3s_planner_picks_small_for_decoder_future_rows():
    ops = _ops()   # the default policy: the time model chooses
    for (M, N, K, akc, bkc, asp, bsp) in [(1280, 512, 512, True, True, False, True),
                                          (512, 512, 1280, False, False, False, False)]:
        assert ops.gemm_x3_choice(M, N, K, asp, bsp, akc, bkc)[0] == "x3s", (M, N, K)
    assert ops.gemm_x3_choice(65536, 512, 768, False, True, True, True)[0] == "x3"


def test_x3s_split_k_accumulate_many_launches(device, small_on):
    """Weight-grad accumulation through split-K slabs, launched many times back to back: every launch
    adds exactly A B^T (integers: exact)."""
    ops = small_on
    gen = torch.Generator(device=device).manual_seed(22)
    M, N, K = 256, 512, 1280
    a, b = _mk(M, N, K, False, False, gen, device, True)
    assert ops.gemm_x3_choice(M, N, K, False, False, False, False)[1] > 1
    prod = a.t().double() @ b.double()
    out = torch.zeros(M, N, device=device)
    for _ in range(100):
        ops.gemm_x3(a, False, b, False, M, N, K, out=out, accumulate=True)
    assert torch.equal(out.double(), 100 * prod)
