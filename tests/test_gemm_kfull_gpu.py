"""Unmasked staging of the 128-/64-tile split-bf16 GEMM (the default; RQ_GEMM_MASKED keeps the masked path: launches whose K and split-K
chunk are whole 32-deep stages drop the k masks, masked addresses and zeroing selects) against the masked
path — bitwise, for every operand layout / split form, both tile sizes, split-K slabs, fused epilogues and
the paired launch; shapes whose K is not a whole number of stages keep the masked path either way."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from rqvae_hip import ops
    return ops


def _both(fn):
    ops = _ops()
    a = fn()
    with ops.gemm_policy(ops.GEMM_MASKED):
        b = fn()
    return a, b


@pytest.mark.parametrize("M,N,K", [(11264, 512, 512), (11264, 1536, 512), (1280, 512, 1024), (512, 512, 11264),
                                   (40, 384, 1152), (304, 208, 96), (264, 136, 104)])
@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, False)])
@pytest.mark.parametrize("a_split,b_split", [(False, True), (False, False), (True, True)])
def test_kfull_bitwise(device, M, N, K, a_kc, b_kc, a_split, b_split):
    ops = _ops()
    gen = torch.Generator(device=device).manual_seed(M + 3 * N + 7 * K + 11 * a_kc + 13 * b_kc + 17 * a_split)
    A = torch.randn(*((M, K) if a_kc else (K, M)), generator=gen, device=device)
    B = torch.randn(*((N, K) if b_kc else (K, N)), generator=gen, device=device)
    a = ops.split_bf16x3(A) if a_split else A
    b = ops.split_bf16x3(B) if b_split else B
    r1, r2 = _both(lambda: ops.gemm_x3(a, a_kc, b, b_kc, M, N, K))
    assert torch.equal(r1, r2)


@pytest.mark.parametrize("rows,I,O", [(1280, 512, 512), (11264, 512, 1024)])
def test_kfull_pair_and_epilogues_bitwise(device, rows, I, O):
    ops = _ops()
    gen = torch.Generator(device=device).manual_seed(rows + I + O)
    g = torch.randn(rows, O, generator=gen, device=device)
    x = torch.randn(rows, I, generator=gen, device=device)
    W = ops.split_bf16x3(torch.randn(O, I, generator=gen, device=device) * 0.05)
    Z = torch.randn(rows, I, generator=gen, device=device)
    dW0 = torch.randn(O, I, generator=gen, device=device)

    def run():
        out = dW0.clone()
        dspec = dict(a=g, a_kcontig=True, b=W, b_kcontig=False, M=rows, N=I, K=O, epilogue=ops.EPI_SILU_BWD, Z=Z,
                     p=0.3, seed=5)
        wspec = dict(a=g, a_kcontig=False, b=x, b_kcontig=False, M=O, N=I, K=rows, out=out, accumulate=True)
        d, w = ops.gemm_x3_pair(dspec, wspec)
        return d.hi.clone(), d.lo.clone(), w.clone()

    r1, r2 = _both(run)
    for u, v in zip(r1, r2):
        assert torch.equal(u, v)
