"""Wide split-bf16 GEMM kernel (gemm_x3w_kernel: 256 x 256 tiles, LDS-DMA staging, 8 waves in two
staggered groups) against fp64 and against the 128-tile kernel it replaces for large shapes.

* small-integer operands (exact in bf16: lo = 0, every fp32 partial sum exact) give the fp64
  product bit for bit, for all four operand layouts, full and partial tiles, split-K — any
  fragment / swizzle / DMA-slot / stagger-ordering error shows up exactly;
* random operands: the two kernels agree BITWISE whenever they use the same split (same 32-deep k
  steps, same product order) — the fused epilogues (SiLU fwd / bwd with dropout, residual add)
  never split; the split-K store within the split-bf16 bound of fp64;
* rq_gemm_bf16x3_plan really selects the wide kernel for the shapes tested here (RQ_GEMM_FORCE_WIDE /
  RQ_GEMM_NO_WIDE descriptor flags pick the kernel per call: the library keeps no switch).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

LAYOUTS = [(True, True), (True, False), (False, True), (False, False)]
# (M, N, K): full tiles, split-K weight grads, ragged >= 2048 rows (partial tiles), deep K
SHAPES = [(4096, 1024, 256), (65536, 512, 768), (768, 512, 65536), (2304, 2056, 96), (2600, 256, 4096),
          (256, 768, 8192)]


def _ops():
    from rqvae_hip import ops
    return ops


def _mk(M, N, K, a_kc, b_kc, gen, device, integer):
    def make(r, c):
        if integer:
            return torch.randint(-8, 9, (r, c), generator=gen, device=device).float()
        return torch.randn(r, c, generator=gen, device=device)
    a = make(M, K) if a_kc else make(K, M)
    b = make(N, K) if b_kc else make(K, N)
    return a, b


@pytest.fixture
def wide_on():
    ops = _ops()
    with ops.gemm_policy(ops.GEMM_FORCE_WIDE):   # forced: these tests are about the wide kernel itself
        yield ops


@pytest.mark.parametrize("a_kc,b_kc", LAYOUTS)
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_x3w_exact_on_integers(device, wide_on, a_kc, b_kc, M, N, K):
    ops = wide_on
    kern, S = ops.gemm_x3_choice(M, N, K, True, True, a_kc, b_kc)
    assert kern == "wide", (M, N, K, a_kc, b_kc)
    gen = torch.Generator(device=device).manual_seed(M + 5 * N + 11 * K + 2 * a_kc + b_kc)
    a, b = _mk(M, N, K, a_kc, b_kc, gen, device, True)
    C = ops.gemm_x3(ops.split_bf16x3(a), a_kc, ops.split_bf16x3(b), b_kc, M, N, K)
    A = (a if a_kc else a.t()).double()
    B = (b if b_kc else b.t()).double()
    ref = A @ B.t()
    bad = (C.double() != ref)
    assert not bad.any(), (int(bad.sum()), bad.nonzero()[:8].tolist(), S)


@pytest.mark.parametrize("a_kc,b_kc", LAYOUTS)
@pytest.mark.parametrize("M,N,K", [(65536, 512, 768), (768, 512, 65536), (2304, 2056, 96)])
def test_x3w_random_within_bound_and_repeatable(device, wide_on, a_kc, b_kc, M, N, K):
    ops = wide_on
    gen = torch.Generator(device=device).manual_seed(M * 3 + N + K)
    a, b = _mk(M, N, K, a_kc, b_kc, gen, device, False)
    sa, sb = ops.split_bf16x3(a), ops.split_bf16x3(b)
    C = ops.gemm_x3(sa, a_kc, sb, b_kc, M, N, K)
    A = (a if a_kc else a.t()).double()
    B = (b if b_kc else b.t()).double()
    err = (C.double() - A @ B.t()).abs()
    bound = 3e-5 * (A.abs() @ B.abs().t()) + 1e-6
    assert (err <= bound).all(), float((err / bound).max())
    assert torch.equal(C, ops.gemm_x3(sa, a_kc, sb, b_kc, M, N, K))


def _both(ops, fn):
    """fn() under the wide kernel and under the 128-tile kernel."""
    with ops.gemm_policy(ops.GEMM_FORCE_WIDE):
        w = fn()
    with ops.gemm_policy(ops.GEMM_NO_WIDE):
        o = fn()
    return w, o


@pytest.mark.parametrize("p", [0.0, 0.3])
def test_x3w_fused_epilogues_equal_x3_kernel(device, wide_on, p):
    """SiLU forward (C = z, H = split(Dropout(SiLU(z)))), SiLU backward and the residual add: no
    split-K in either kernel, so wide and 128-tile results must be identical bit for bit."""
    ops = wide_on
    M, K, N = 16384, 768, 512   # enough tiles that neither kernel splits K (split-K reduces in another order)
    assert all(ops.gemm_x3_choice(16384, n, k, True, True, True, True)[1] == 1 for n, k in ((512, 768), (768, 512)))
    gen = torch.Generator(device=device).manual_seed(3)
    x32 = torch.randn(M, K, generator=gen, device=device)
    x = ops.split_bf16x3(x32)
    W = ops.split_bf16x3(torch.randn(N, K, generator=gen, device=device) * 0.05)
    assert ops.gemm_x3_choice(M, N, K, True, True, True, True, ops.EPI_SILU_FWD)[0] == "wide"
    (zw, hw), (zo, ho) = _both(ops, lambda: ops.gemm_x3(x, True, W, True, M, N, K, ops.EPI_SILU_FWD, p=p, seed=77))
    assert torch.equal(zw, zo)
    assert torch.equal(hw.hi, ho.hi) and torch.equal(hw.lo, ho.lo)
    g = ops.split_bf16x3(torch.randn(M, N, generator=gen, device=device))
    Z = torch.randn(M, K, generator=gen, device=device)
    assert ops.gemm_x3_choice(M, K, N, True, True, True, False, ops.EPI_SILU_BWD)[0] == "wide"
    bw, bo = _both(ops, lambda: ops.gemm_x3(g, True, W, False, M, K, N, ops.EPI_SILU_BWD, Z=Z, p=p, seed=78))
    assert torch.equal(bw.hi, bo.hi) and torch.equal(bw.lo, bo.lo)
    # residual add: the 128-tile kernel takes this layer's input in fp32 (split while staged: the
    # same RNE planes), the wide one pre-split
    r = torch.randn(M, N, generator=gen, device=device)
    assert ops.gemm_x3_choice(M, N, K, True, True, True, True, ops.EPI_ADD)[0] == "wide"
    aw = ops.gemm_x3(x, True, W, True, M, N, K, ops.EPI_ADD, Z=r)
    with ops.gemm_policy(ops.GEMM_NO_WIDE):
        ao = ops.gemm_x3(x32, True, W, True, M, N, K, ops.EPI_ADD, Z=r)
    assert torch.equal(aw, ao)


def test_x3w_not_chosen_for_fp32_or_small(device, wide_on):
    ops = wide_on
    assert ops.gemm_x3_choice(65536, 512, 768, False, True, True, True)[0] != "wide"      # fp32 operand
    assert ops.gemm_x3_choice(65536, 128, 256, True, True, True, True)[0] != "wide"       # N = 128: half tile
    assert ops.gemm_x3_choice(64, 64, 64, True, True, True, True)[0] != "wide"
    assert ops.gemm_x3_choice(65536, 512, 100, True, True, True, True)[0] != "wide"       # K % 32
    with ops.gemm_policy(ops.GEMM_NO_WIDE):
        assert ops.gemm_x3_choice(65536, 512, 768, True, True, True, True)[0] != "wide"
