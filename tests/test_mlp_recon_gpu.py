"""RqVae MLP chains at matmul precision 'high' with split operands handed straight to the wide GEMM
kernel (reference: modules/encoder.py:7-36, modules/rqvae.py:145-148, modules/loss.py:5-10):

* MLPL2ReconFunction (decoder chain + l2norm + ReconstructionLoss, whose backward emits the output
  gradient split) against the unfused composition MLPFunction -> L2NormReconFunction (fp32
  gradient, split while staged by the 128-tile kernel): the split planes are the same RNE planes and
  the wide kernel accumulates in the 128-tile kernel's order, so the loss, the input gradient and
  every weight gradient computed without split-K agree BITWISE; split-K weight grads (different
  slab counts) within fp32 reassociation; everything against an fp64 torch reference;
* MLPFunction with a pre-split input (the encoder's first layer on the wide kernel) against the
  same chain with the wide kernel off (fp32 input split while staged): within fp32 reassociation
  (split-K slab counts differ between the kernels);
* rq_l2norm_recon_bwd_split planes == rq_split_bf16x3 of rq_l2norm_recon_bwd's fp32 output.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from rqvae_hip import ops
    return ops


def _weights(dims, gen, device):
    return [torch.nn.Parameter(torch.randn(dims[i + 1], dims[i], generator=gen, device=device) / dims[i] ** 0.5)
            for i in range(len(dims) - 1)]


def _reset_seeds(ops):
    ops._SEED["n"] = 0


def _ref64(e, x, ws):
    h = e.double()
    for i, w in enumerate(ws):
        h = h @ w.double().t()
        if i < len(ws) - 1:
            h = torch.nn.functional.silu(h)
    y = h / h.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    return ((y - x.double()) ** 2).sum(-1)


@pytest.mark.parametrize("p", [0.0, 0.3])
def test_mlp_l2norm_recon_equals_composition(device, p):
    ops = _ops()
    with ops.gemm_policy(ops.GEMM_FORCE_WIDE):   # forced: the split gradient's path onto the wide kernel
        B, dims = 16384, [64, 128, 256, 512, 768]   # no split-K on the last data grad for either kernel
        gen = torch.Generator(device=device).manual_seed(21)
        ws = _weights(dims, gen, device)
        e = torch.randn(B, dims[0], generator=gen, device=device).requires_grad_(True)
        x = torch.nn.functional.normalize(torch.randn(B, dims[-1], generator=gen, device=device), dim=-1)
        gr = torch.rand(B, generator=gen, device=device)
        # the last data grad takes the split gradient on the wide kernel (the composition: fp32 on x3)
        assert ops.gemm_x3_choice(B, 512, 768, True, True, True, False, ops.EPI_SILU_BWD)[0] == "wide"
        assert ops.gemm_x3_choice(B, 512, 768, False, True, True, False, ops.EPI_SILU_BWD)[0] == "x3"

        def run(fused):
            _reset_seeds(ops)
            for w in ws:
                w.grad = None
            e.grad = None
            if fused:
                r = ops.mlp_l2norm_recon(e, x, ws, p)
            else:
                r = ops.l2norm_recon_loss(ops.mlp_chain(e, ws, p), x)
            r.backward(gr)
            return r.detach().clone(), e.grad.clone(), [w.grad.clone() for w in ws]

        rf, ef, wf = run(True)
        rc, ec, wc = run(False)
        assert torch.equal(rf, rc)
        assert torch.equal(ef, ec)
        for i, (a, b) in enumerate(zip(wf, wc)):   # split-K reassociation: fp32 rounding of the slab sums
            assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max()), i
        for i in range(len(ws) - 1):   # every layer but the last: same kernels on identical operands
            if ops.gemm_x3_choice(dims[i + 1], dims[i], B, True, True, False, False)[1] == 1:
                assert torch.equal(wf[i], wc[i]), i
        if p == 0.0:
            ref = _ref64(e.detach(), x, [w.detach() for w in ws])
            assert torch.allclose(rf.double(), ref, rtol=2e-4, atol=1e-6)


@pytest.mark.parametrize("mode", ["mean", "mixed", "sum", "no_grad"])
def test_mlp_l2norm_recon_speculative_gradient(device, mode):
    """The fused node writes the split output gradient in its forward for g_recon = 1 / B (the batch-mean
    loss) and its backward only checks g_recon: mean (one expanded value: every row speculated), mixed
    (a per-row gradient, half the rows 1 / B: the others recomputed), sum (g_recon = 1: all recomputed) —
    each bitwise the composition's gradients; under no_grad the forward writes no planes (same loss)."""
    ops = _ops()
    with ops.gemm_policy(ops.GEMM_FORCE_WIDE):
        B, dims = 16384, [64, 128, 256, 512, 768]   # as above: no split-K on the last data grad
        gen = torch.Generator(device=device).manual_seed(23)
        ws = _weights(dims, gen, device)
        e = torch.randn(B, dims[0], generator=gen, device=device).requires_grad_(True)
        x = torch.nn.functional.normalize(torch.randn(B, dims[-1], generator=gen, device=device), dim=-1)
        mixed = torch.where(torch.arange(B, device=device) % 2 == 0, torch.full((B,), 1.0 / B, device=device),
                            torch.rand(B, generator=gen, device=device))

        def run(fused):
            _reset_seeds(ops)
            for w in ws:
                w.grad = None
            e.grad = None
            if mode == "no_grad":
                with torch.no_grad():
                    r = ops.mlp_l2norm_recon(e, x, ws) if fused else ops.l2norm_recon_loss(ops.mlp_chain(e, ws), x)
                return r.clone(), None, []
            r = ops.mlp_l2norm_recon(e, x, ws) if fused else ops.l2norm_recon_loss(ops.mlp_chain(e, ws), x)
            if mode == "mean":
                r.mean().backward()
            elif mode == "mixed":
                r.backward(mixed)
            else:
                r.sum().backward()
            return r.detach().clone(), e.grad.clone(), [w.grad.clone() for w in ws]

        rf, ef, wf = run(True)
        rc, ec, wc = run(False)
        assert torch.equal(rf, rc)
        if mode != "no_grad":
            assert torch.equal(ef, ec)
            for i, (a, b) in enumerate(zip(wf, wc)):
                assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max()), i


def test_mlp_presplit_input_equals_fp32_input(device):
    ops = _ops()
    B, dims = 8192, [768, 512, 256]
    gen = torch.Generator(device=device).manual_seed(5)
    ws = _weights(dims, gen, device)
    x = torch.randn(B, dims[0], generator=gen, device=device).requires_grad_(True)
    g = torch.randn(B, dims[-1], generator=gen, device=device)
    with ops.gemm_policy(ops.GEMM_FORCE_WIDE):
        assert ops._presplit_input(B, ws, len(ws))
    with ops.gemm_policy(ops.GEMM_NO_WIDE):
        assert not ops._presplit_input(B, ws, len(ws))

    def run(wide):
        with ops.gemm_policy(ops.GEMM_FORCE_WIDE if wide else ops.GEMM_NO_WIDE):
            for w in ws:
                w.grad = None
            x.grad = None
            y = ops.mlp_chain(x, ws, 0.0)
            y.backward(g)
            return y.detach().clone(), x.grad.clone(), [w.grad.clone() for w in ws]

    yw, xw, gw = run(True)
    yo, xo, go = run(False)
    # the plain-store launches (last forward layer, input grad, weight grads) may split K into a
    # different slab count on the two kernels: fp32 reassociation only
    for a, b in [(yw, yo), (xw, xo), *zip(gw, go)]:
        assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max())


def test_l2norm_recon_bwd_split_planes(device):
    from rqvae_hip._lib import ptr, stream_handle
    ops = _ops()
    B, C = 1000, 768
    gen = torch.Generator(device=device).manual_seed(9)
    pre = torch.randn(B, C, generator=gen, device=device)
    pre[3] = 0.0                                    # a clamped row (|pre| < eps)
    x = torch.nn.functional.normalize(torch.randn(B, C, generator=gen, device=device), dim=-1)
    g = torch.rand(B, generator=gen, device=device)
    recon = torch.empty(B, device=device)
    norms = torch.empty(B, device=device)
    ops.call("rq_l2norm_recon_fwd", ptr(pre), ptr(x), B, C, ptr(recon), ptr(norms), stream_handle(device))
    g32 = torch.empty_like(pre)
    ops.call("rq_l2norm_recon_bwd", ptr(pre), ptr(x), ptr(norms), ptr(g), B, C, ptr(g32), stream_handle(device))
    hi = torch.empty(B, C, device=device, dtype=torch.bfloat16)
    lo = torch.empty_like(hi)
    ops.call("rq_l2norm_recon_bwd_split", ptr(pre), ptr(x), ptr(norms), ptr(g), B, C, ptr(hi), ptr(lo),
             stream_handle(device))
    ref = ops.split_bf16x3(g32)
    assert torch.equal(hi, ref.hi) and torch.equal(lo, ref.lo)
