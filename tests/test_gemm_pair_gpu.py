"""Paired data-/weight-gradient launch (rq_gemm_bf16x3_pair / ops.gemm_x3_pair: both problems' workgroups in
one gemm_x3_pair_kernel grid) against the same two problems as separate rq_gemm_bf16x3 calls — bitwise
(each workgroup runs the unchanged kernel body), for every paired operand form (fp32 / split A, plain and
SiLU'-with-dropout data gradient; fp32 / split operands of the weight gradient), both tile sizes (the
decoder's 1,280 future-token rows -> 64-tile form, 11,264 context rows -> 128-tile form), split-K slabs,
accumulation into an existing gradient and the deferred slab reduction. Each problem keeps the plan it has
alone (a split-K data gradient stays split in the pair), so every result is bitwise the separate call's."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from rqvae_hip import ops
    return ops


@pytest.mark.parametrize("rows,I,O", [(1280, 512, 512), (1280, 512, 1536), (11264, 512, 512), (40, 384, 1152)])
@pytest.mark.parametrize("a_split", [False, True])
@pytest.mark.parametrize("x_split", [False, True])
@pytest.mark.parametrize("silu", [False, True])
def test_pair_bitwise_equals_two_launches(device, rows, I, O, a_split, x_split, silu):
    ops = _ops()
    if silu and a_split:
        pytest.skip("the SiLU' data gradient takes an fp32 output gradient (MLP chain backward)")
    gen = torch.Generator(device=device).manual_seed(rows + I + 3 * O + 7 * a_split + 11 * x_split + silu)
    g32 = torch.randn(rows, O, generator=gen, device=device)
    g = ops.split_bf16x3(g32) if a_split else g32
    x32 = torch.randn(rows, I, generator=gen, device=device)
    x = ops.split_bf16x3(x32) if x_split else x32
    W = ops.split_bf16x3(torch.randn(O, I, generator=gen, device=device) * 0.05)
    Z = torch.randn(rows, I, generator=gen, device=device)
    dspec = dict(a=g, a_kcontig=True, b=W, b_kcontig=False, M=rows, N=I, K=O)
    if silu:
        dspec.update(epilogue=ops.EPI_SILU_BWD, Z=Z, p=0.3, seed=17)
    dW0 = torch.randn(O, I, generator=gen, device=device)
    for accumulate in (False, True):
        out1, out2 = dW0.clone(), dW0.clone()
        wkw = dict(out=out1, accumulate=True) if accumulate else {}
        wspec = dict(a=g, a_kcontig=False, b=x, b_kcontig=False, M=O, N=I, K=rows, **wkw)
        r_d, r_w = ops.gemm_x3_pair(dspec, wspec)
        wspec2 = dict(wspec, **(dict(out=out2) if accumulate else {}))
        s_d = ops.gemm_x3(**dspec)
        s_w = ops.gemm_x3(**wspec2)
        assert torch.equal(r_w, s_w)
        # the same plan paired or alone (split-K included): bitwise
        if silu:
            assert torch.equal(r_d.hi, s_d.hi) and torch.equal(r_d.lo, s_d.lo)
        else:
            assert torch.equal(r_d, s_d)


def test_pair_plan_and_no_pair_flag(device):
    ops = _ops()
    from rqvae_hip import _lib
    lib = _lib.load()
    with ops.gemm_policy(ops.GEMM_NO_PAIR):   # the descriptors ask for two launches
        gen = torch.Generator(device=device).manual_seed(1)
        g = torch.randn(1280, 512, generator=gen, device=device)
        x = torch.randn(1280, 512, generator=gen, device=device)
        W = ops.split_bf16x3(torch.randn(512, 512, generator=gen, device=device))
        a, b = ops.gemm_x3_pair(dict(a=g, a_kcontig=True, b=W, b_kcontig=False, M=1280, N=512, K=512),
                                dict(a=g, a_kcontig=False, b=x, b_kcontig=False, M=512, N=512, K=1280))
        assert torch.equal(a, ops.gemm_x3(g, True, W, False, 1280, 512, 512))
        assert torch.equal(b, ops.gemm_x3(g, False, x, False, 512, 512, 1280))
    assert lib.rq_gemm_bf16x3_pair_plan(None) == 0


def test_pair_deferred_reduction(device):
    """A split-K weight gradient accumulated with the deferred slab reduction through the pair: after
    flush_reductions the bucket equals the immediate accumulation."""
    ops = _ops()
    gen = torch.Generator(device=device).manual_seed(2)
    rows, I, O = 11264, 512, 512
    g = torch.randn(rows, O, generator=gen, device=device)
    x = torch.randn(rows, I, generator=gen, device=device)
    W = ops.split_bf16x3(torch.randn(O, I, generator=gen, device=device))
    assert ops.gemm_x3_choice(O, I, rows, False, False, False, False)[1] > 1   # split-K weight gradient
    base = torch.randn(O, I, generator=gen, device=device)
    b1, b2 = base.clone(), base.clone()
    ops.gemm_x3_pair(dict(a=g, a_kcontig=True, b=W, b_kcontig=False, M=rows, N=I, K=O),
                     dict(a=g, a_kcontig=False, b=x, b_kcontig=False, M=O, N=I, K=rows, out=b1, accumulate=True,
                          defer=True))
    assert ops.pending_reductions() > 0
    ops.flush_reductions()
    ops.gemm_x3(g, False, x, False, O, I, rows, out=b2, accumulate=True)
    assert torch.equal(b1, b2)
