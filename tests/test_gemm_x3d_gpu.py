"""LDS-DMA form of the 128-tile split-bf16 GEMM (gemm_x3d_kernel: fp32 k-contiguous A by LDS-DMA into an
fp32 row image, split while its fragments are read; split B by LDS-DMA into the wide kernel's half-plane
images) against fp64 and against the register-staged 128-tile kernel it replaces.

* small-integer operands (exact in bf16, every fp32 partial sum exact) give the fp64 product bit for bit
  for both B layouts, full and partial tiles, split-K — any fragment / swizzle / DMA-slot / ring-order
  error shows up exactly;
* random operands: the two kernels agree BITWISE (same split of A, same 16x16x32 product order, same k
  steps) for every epilogue (store, split-K store, SiLU fwd / bwd with dropout, residual add with dropout);
* rq_gemm_bf16x3_choice reports 'x3d' for these shapes and 'x3' with the switch off.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (M, N, K): decoder context rows (11,264), partial row / column tiles, split-K (few tiles, deep K)
SHAPES = [(11264, 1536, 512), (11332, 512, 1536), (300, 264, 96), (1000, 512, 4096), (128, 128, 32)]


def _ops():
    from rqvae_hip import ops
    return ops


@pytest.fixture
def x3d_on():
    ops = _ops()
    prev = ops.gemm_x3d_enable(2)   # forced for both B layouts: these tests are about the kernel itself
    prev_w = ops.gemm_x3w_enable(False)   # keep the wide kernel out of the comparison
    prev_s = ops.gemm_x3s_enable(0)       # and the 64-tile form
    yield ops
    ops.gemm_x3d_enable(prev)
    ops.gemm_x3w_enable(prev_w)
    ops.gemm_x3s_enable(prev_s)


def _both(ops, fn):
    ops.gemm_x3d_enable(2)
    d = fn()
    ops.gemm_x3d_enable(False)
    try:
        o = fn()
    finally:
        ops.gemm_x3d_enable(2)
    return d, o


@pytest.mark.parametrize("b_kc", [True, False])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_x3d_exact_on_integers(device, x3d_on, b_kc, M, N, K):
    ops = x3d_on
    kern, S = ops.gemm_x3_choice(M, N, K, False, True, True, b_kc)
    assert kern == "x3d", (M, N, K, b_kc)
    gen = torch.Generator(device=device).manual_seed(M + 5 * N + 11 * K + b_kc)
    a = torch.randint(-8, 9, (M, K), generator=gen, device=device).float()
    b = torch.randint(-8, 9, (N, K) if b_kc else (K, N), generator=gen, device=device).float()
    C = ops.gemm_x3(a, True, ops.split_bf16x3(b), b_kc, M, N, K)
    ref = a.double() @ (b if b_kc else b.t()).double().t()
    bad = C.double() != ref
    assert not bad.any(), (int(bad.sum()), bad.nonzero()[:8].tolist(), S)


@pytest.mark.parametrize("b_kc", [True, False])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_x3d_store_bitwise_and_bounded(device, x3d_on, b_kc, M, N, K):
    ops = x3d_on
    gen = torch.Generator(device=device).manual_seed(3 * M + N + K)
    a = torch.randn(M, K, generator=gen, device=device)
    b = torch.randn((N, K) if b_kc else (K, N), generator=gen, device=device)
    sb = ops.split_bf16x3(b)
    d, o = _both(ops, lambda: ops.gemm_x3(a, True, sb, b_kc, M, N, K))
    assert torch.equal(d, o)
    B = (b if b_kc else b.t()).double()
    err = (d.double() - a.double() @ B.t()).abs()
    assert (err <= 3e-5 * (a.double().abs() @ B.abs().t()) + 1e-6).all()
    assert torch.equal(d, ops.gemm_x3(a, True, sb, b_kc, M, N, K))   # repeatable


@pytest.mark.parametrize("p", [0.0, 0.3])
def test_x3d_fused_epilogues_bitwise(device, x3d_on, p):
    """SiLU forward (C = z, H = split(Dropout(SiLU(z)))), SiLU backward and the residual add (the decoder's
    fp32-input forms) — unsplit, so both kernels must agree bit for bit."""
    ops = x3d_on
    M, K, N = 11264, 512, 1024
    gen = torch.Generator(device=device).manual_seed(5)
    x = torch.randn(M, K, generator=gen, device=device)
    W = ops.split_bf16x3(torch.randn(N, K, generator=gen, device=device) * 0.05)
    assert ops.gemm_x3_choice(M, N, K, False, True, True, True, ops.EPI_SILU_FWD)[0] == "x3d"
    (zd, hd), (zo, ho) = _both(ops, lambda: ops.gemm_x3(x, True, W, True, M, N, K, ops.EPI_SILU_FWD, p=p, seed=91))
    assert torch.equal(zd, zo) and torch.equal(hd.hi, ho.hi) and torch.equal(hd.lo, ho.lo)
    g = torch.randn(M, N, generator=gen, device=device)
    Z = torch.randn(M, K, generator=gen, device=device)
    bd, bo = _both(ops, lambda: ops.gemm_x3(g, True, W, False, M, K, N, ops.EPI_SILU_BWD, Z=Z, p=p, seed=92))
    assert torch.equal(bd.hi, bo.hi) and torch.equal(bd.lo, bo.lo)
    r = torch.randn(M, N, generator=gen, device=device)
    ad, ao = _both(ops, lambda: ops.gemm_x3(x, True, W, True, M, N, K, ops.EPI_ADD, Z=r, p=p, seed=93))
    assert torch.equal(ad, ao)


def test_x3d_choice(device, x3d_on):
    ops = x3d_on
    assert ops.gemm_x3_choice(11264, 1536, 512, True, True, True, True)[0] != "x3d"    # split A: not this form
    assert ops.gemm_x3_choice(11264, 1536, 512, False, True, False, True)[0] != "x3d"  # m-contiguous A
    assert ops.gemm_x3_choice(11264, 1536, 500, False, True, True, True)[0] != "x3d"   # K % 32
    ops.gemm_x3d_enable(True)   # mode 1: n-contiguous B only
    assert ops.gemm_x3_choice(11264, 1536, 512, False, True, True, True)[0] == "x3"
    assert ops.gemm_x3_choice(11264, 512, 1536, False, True, True, False)[0] == "x3d"
    ops.gemm_x3d_enable(False)
    assert ops.gemm_x3_choice(11264, 512, 1536, False, True, True, False)[0] == "x3"
