"""Split-K for every epilogue of the split-bf16 GEMM (rq_gemm_bf16x3_run): when the output tiles cannot
fill the chip (the decoder's 1,280 future-token rows: 40 tiles of 128 x 128) the partial products go
to slabs and a fixed-order reduction applies the epilogue (SiLU fwd / bwd with dropout, residual add)
— and accumulation into an existing buffer (C += A B^T, the weight gradient added into a flat
gradient bucket). Reference ops: nn.Linear / SiLU / Dropout of modules/encoder.py:7-36 and the
residual adds of modules/transformer/model.py:75-82.

Checks: the split path (M = 320) equals the first 320 rows of the same product at M = 16,384 (no
split; the dropout mask key m N + n is the same for those rows) up to fp32 reassociation; both
within the split-bf16 bound of an fp64 reference; the reduction is deterministic (bitwise repeat);
accumulate == C0 + product, split and unsplit.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from rqvae_hip import ops
    return ops


@pytest.fixture(autouse=True)
def _x3_tiles_only():
    """These tests are about the 128-tile kernel's split-K path: keep the 64-tile form (which serves
    1,280-row launches unsplit) out of the way."""
    ops = _ops()
    with ops.gemm_policy(ops.GEMM_ONLY_128):
        yield


def _close(a, b, tol):
    return float((a - b).abs().max()) <= tol * max(1e-30, float(b.abs().max()))


def _merge(h):
    return h.hi.float() + h.lo.float()


@pytest.mark.parametrize("p", [0.0, 0.3])
def test_fused_epilogues_split_equal_unsplit_rows(device, p):
    ops = _ops()
    Mbig, M, N, K = 16384, 320, 512, 512
    gen = torch.Generator(device=device).manual_seed(11)
    a_big = torch.randn(Mbig, K, generator=gen, device=device)
    W = ops.split_bf16x3(torch.randn(N, K, generator=gen, device=device) * 0.05)
    a = a_big[:M].contiguous()
    assert ops.gemm_x3_choice(M, N, K, False, True, True, True, ops.EPI_SILU_FWD)[1] > 1
    assert ops.gemm_x3_choice(Mbig, N, K, False, True, True, True, ops.EPI_SILU_FWD)[1] == 1
    # SiLU forward (+ dropout): z and H
    z, h = ops.gemm_x3(a, True, W, True, M, N, K, ops.EPI_SILU_FWD, p=p, seed=5)
    zb, hb = ops.gemm_x3(a_big, True, W, True, Mbig, N, K, ops.EPI_SILU_FWD, p=p, seed=5)
    assert _close(z, zb[:M], 1e-6)
    assert _close(_merge(h), _merge(hb)[:M], 1e-5)
    z2, h2 = ops.gemm_x3(a, True, W, True, M, N, K, ops.EPI_SILU_FWD, p=p, seed=5)
    assert torch.equal(z, z2) and torch.equal(h.hi, h2.hi) and torch.equal(h.lo, h2.lo)
    ref = a.double() @ (W.hi.double() + W.lo.double()).t()
    assert _close(z.double(), ref, 3e-5)
    if p == 0.0:
        assert _close(_merge(h).double(), torch.nn.functional.silu(ref), 3e-5)
    else:   # the same kept set as the unsplit launch, scaled by 1 / (1 - p)
        assert torch.equal(_merge(h) == 0, _merge(hb)[:M] == 0)
    # SiLU backward (+ dropout): H = split(SiLU'(Z) * Dropout(g W))
    g_big = torch.randn(Mbig, N, generator=gen, device=device)
    Wt = ops.split_bf16x3(torch.randn(N, K, generator=gen, device=device) * 0.05)   # (N=out, K=in)
    Zb = torch.randn(Mbig, K, generator=gen, device=device)
    g, Zs = g_big[:M].contiguous(), Zb[:M].contiguous()
    assert ops.gemm_x3_choice(M, K, N, False, True, True, False, ops.EPI_SILU_BWD)[1] > 1
    hs = ops.gemm_x3(g, True, Wt, False, M, K, N, ops.EPI_SILU_BWD, Z=Zs, p=p, seed=6)
    hsb = ops.gemm_x3(g_big, True, Wt, False, Mbig, K, N, ops.EPI_SILU_BWD, Z=Zb, p=p, seed=6)
    assert _close(_merge(hs), _merge(hsb)[:M], 1e-5)
    # residual add: C = A B^T + Z
    r_big = torch.randn(Mbig, N, generator=gen, device=device)
    ca = ops.gemm_x3(a, True, W, True, M, N, K, ops.EPI_ADD, Z=r_big[:M].contiguous())
    cab = ops.gemm_x3(a_big, True, W, True, Mbig, N, K, ops.EPI_ADD, Z=r_big)
    assert _close(ca, cab[:M], 1e-6)


@pytest.mark.parametrize("M,N,K", [(512, 512, 11332), (1536, 512, 1280), (65536, 512, 768), (128, 64, 65536)])
def test_accumulate_into_existing(device, M, N, K):
    """C += g^T x (weight-grad layout) and C += x W^T: the product lands on top of C's contents, split
    or not, and an accumulating call equals store + add up to the one extra rounding."""
    ops = _ops()
    gen = torch.Generator(device=device).manual_seed(M + N + K)
    if M < N * 4 or K > 4096:   # weight-grad layout: A(m, k) = g[k, m], B(n, k) = x[k, n]
        a = torch.randn(K, M, generator=gen, device=device)
        b = torch.randn(K, N, generator=gen, device=device)
        akc = bkc = False
        A, B = a.t().double(), b.t().double()
    else:
        a = torch.randn(M, K, generator=gen, device=device)
        b = torch.randn(N, K, generator=gen, device=device)
        akc = bkc = True
        A, B = a.double(), b.double()
    c0 = torch.randn(M, N, generator=gen, device=device)
    c = c0.clone()
    out = ops.gemm_x3(a, akc, b, bkc, M, N, K, out=c, accumulate=True)
    assert out.data_ptr() == c.data_ptr()
    prod = ops.gemm_x3(a, akc, b, bkc, M, N, K)
    assert _close(c, c0 + prod, 1e-6)
    ref = c0.double() + A @ B.t()
    bound = 3e-5 * (A.abs() @ B.abs().t()) + 1e-5
    assert ((c.double() - ref).abs() <= bound).all()


def _emulated_slab_sum(P, S):
    """The split-K reductions' defined order on torch fp32 adds: p_w = 0 + P[w] + P[w + 4] + ..., then
    ((p0 + p1) + p2) + p3."""
    p = [torch.zeros_like(P[0]) for _ in range(4)]
    for s in range(S):
        p[s % 4] = p[s % 4] + P[s]
    return ((p[0] + p[1]) + p[2]) + p[3]


@pytest.mark.parametrize("S,n", [(1, 64), (3, 4096), (4, 1000), (7, 4100), (16, 2048), (21, 6000), (40, 512)])
def test_reduce_partials_order(device, S, n):
    """rq_reduce_partials layout 0 (and with accumulate) is bitwise the defined four-way order, for S below,
    at and past one 16-load round and n not a multiple of a workgroup's columns."""
    import ctypes
    from rqvae_hip import ops
    g = torch.Generator(device=device).manual_seed(S * 131 + n)
    P = torch.randn(S, n, generator=g, device=device) * torch.logspace(-3, 3, n, device=device)
    for acc in (0, 1):
        out = torch.randn(n, generator=g, device=device)
        ref = _emulated_slab_sum(P, S)
        ref = out + ref if acc else ref
        Pp = (ctypes.c_void_p * 1)(P.data_ptr())
        Op = (ctypes.c_void_p * 1)(out.data_ptr())
        ops.call("rq_reduce_partials", 1, Pp, Op, (ctypes.c_int64 * 1)(n), (ctypes.c_int * 1)(S), (ctypes.c_int * 1)(0),
                 (ctypes.c_int * 1)(acc), ops.stream_handle(device))
        torch.cuda.synchronize()
        assert torch.equal(out, ref), (S, n, acc)


@pytest.mark.parametrize("M,N,K,S", [(40, 512, 512, 8), (40, 1536, 384, 12), (1280, 512, 1024, 4), (96, 256, 2048, 21)])
def test_splitk_reduction_order(device, M, N, K, S):
    """A forced-split GEMM's immediate slab reduction (x3_reduce_kernel, accumulate) equals its deferred slabs
    summed in the defined order, and the deferred batched reduction gives the same bits."""
    from rqvae_hip import ops
    g = torch.Generator(device=device).manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g, device=device)
    b = ops.split_bf16x3(torch.randn(N, K, generator=g, device=device) * 0.05)
    base = torch.randn(M, N, generator=g, device=device)
    f = ops.gemm_split(S)
    out_imm = base.clone()
    with ops.gemm_policy(f):
        ops.gemm_x3(a, True, b, True, M, N, K, out=out_imm, accumulate=True)
        out_def = base.clone()
        ops.flush_reductions()
        ops.gemm_x3(a, True, b, True, M, N, K, out=out_def, accumulate=True, defer=True)
        pend = list(ops._DEFER["pending"])
        assert len(pend) == 1 and pend[0][3] > 1   # the forced count, rounded to whole 32-deep chunks
        ws, _, n, S_, _, _ = pend[0]
        slabs = ws.view(torch.float32)[:S_ * n].view(S_, n).clone()
        ops.flush_reductions()
    torch.cuda.synchronize()
    ref = base.reshape(-1) + _emulated_slab_sum(slabs, S_)
    assert torch.equal(out_imm.reshape(-1), ref)
    assert torch.equal(out_def, out_imm)
