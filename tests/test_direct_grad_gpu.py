"""Weight gradients added straight into data-parallel flat gradient buckets (rqvae_hip.dp.direct_grad):
with dp.GradBuckets owning flat buffers, the split-bf16 weight-grad GEMMs of LinearFunction,
LinearAddFunction and the fused MLP chain accumulate into the bucket view in their slab reduction
(C += g^T x) and hand autograd None, replacing the AccumulateGrad add kernel per parameter per step
(reference semantics: torch autograd's .grad accumulation, modules/encoder.py / transformer Linears).

Checks, at matmul precision 'high': gradients (one backward, and two accumulated micro-batches)
bitwise equal to plain autograd on an identical model; the buckets' usage tracking still sees the
parameters (no grad reset to None after synchronize); the decoder model's gradients match too; the
weight-split scope (one multi-tensor split per forward) gives bitwise the same forward.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        from modules.encoder import MLP
        from modules.linear import Linear
        self.mlp = MLP(64, [128, 96], 64)
        self.lin = Linear(64, 64, bias=False)
        self.proj = Linear(64, 64, bias=False)

    def forward(self, x):
        from rqvae_hip import ops
        h = self.mlp(x)
        y = self.lin(h)
        return ops.linear_add(y, self.proj.weight, h)


def _grads(m):
    return {n: p.grad.clone() for n, p in m.named_parameters()}


@pytest.mark.parametrize("micro", [1, 2])
def test_direct_grad_equals_autograd(device, micro):
    from rqvae_hip import dp
    torch.set_float32_matmul_precision("high")
    try:
        torch.manual_seed(0)
        a = _Net().to(device)
        b = copy.deepcopy(a)
        buckets = dp.GradBuckets(b.parameters(), overlap=False, flat_views=True)
        gen = torch.Generator(device=device).manual_seed(1)
        xs = [torch.randn(4096, 64, generator=gen, device=device) for _ in range(micro)]
        gs = [torch.randn(4096, 64, generator=gen, device=device) for _ in range(micro)]
        for x, g in zip(xs, gs):
            a(x).backward(g)
        buckets.zero_grad()
        calls = []
        orig = dp.direct_grad_done
        dp.direct_grad_done = lambda p: (calls.append(id(p)), orig(p))
        try:
            for x, g in zip(xs, gs):
                b(x).backward(g)
        finally:
            dp.direct_grad_done = orig
        # the direct path really ran for every GEMM weight, once per micro-batch
        assert sorted(calls) == sorted([id(p) for p in b.parameters()] * micro)
        with torch.no_grad():
            assert all(dp.direct_grad(p) is not None for p in b.parameters())
        buckets.synchronize()
        ga, gb = _grads(a), _grads(b)
        for n in ga:
            assert torch.equal(ga[n], gb[n]), n
    finally:
        torch.set_float32_matmul_precision("highest")


def test_direct_grad_decoder_model(device):
    """The decoder (EncoderDecoderRetrievalModel, dropout 0) with flat buckets vs plain autograd."""
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    from rqvae_hip import dp
    torch.set_float32_matmul_precision("high")
    try:
        torch.manual_seed(3)
        a = EncoderDecoderRetrievalModel(embedding_dim=64, attn_dim=128, dropout=0.0, num_heads=4, n_layers=4,
                                         num_embeddings=64, sem_id_dim=4, inference_verifier_fn=None,
                                         max_pos=80).to(device).train()
        b = copy.deepcopy(a)
        buckets = dp.GradBuckets(b.parameters(), overlap=False, flat_views=True)
        batch = synthetic_tokenized_batch(32, 20, 4, 64, 7, device)
        from rqvae_hip import ops
        ops._SEED["n"] = 0            # same dropout keys for both models (the norm dropouts, p = 0.5)
        la = a(batch).loss
        la.backward()
        buckets.zero_grad()
        ops._SEED["n"] = 0
        lb = b(batch).loss
        lb.backward()
        buckets.synchronize()
        assert torch.equal(la.detach(), lb.detach())
        for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
            if pa.grad is None:
                assert pb.grad is None, n
                continue
            assert torch.equal(pa.grad, pb.grad), n
    finally:
        torch.set_float32_matmul_precision("highest")


@pytest.mark.parametrize("buckets_on", [False, True])
def test_hoisted_kv_matches_per_layer(device, buckets_on):
    """The decoder's cross-attention K/V projections of the shared context as one hoisted GEMM
    (HoistedProjectionFunction; its backward reads the attention kernels' gradient blocks in place)
    vs one Linear per layer: same loss and gradients (split-K orders may differ: fp32 tolerances)."""
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    from modules.transformer import model as tm
    from rqvae_hip import dp, ops
    torch.set_float32_matmul_precision("high")
    prev = tm._HOIST_KV
    try:
        torch.manual_seed(5)
        a = EncoderDecoderRetrievalModel(embedding_dim=64, attn_dim=128, dropout=0.0, num_heads=4, n_layers=4,
                                         num_embeddings=64, sem_id_dim=4, inference_verifier_fn=None,
                                         max_pos=80).to(device).train()
        b = copy.deepcopy(a)
        if buckets_on:
            buckets = dp.GradBuckets(b.parameters(), overlap=False, flat_views=True)
            buckets.zero_grad()
        batch = synthetic_tokenized_batch(48, 20, 4, 64, 11, device)
        tm._HOIST_KV = False
        ops._SEED["n"] = 0
        la = a(batch).loss
        la.backward()
        calls = []
        orig = ops.HoistedProjectionFunction.forward

        def counted(ctx, x, *ws):
            calls.append(len(ws))
            return orig(ctx, x, *ws)
        ops.HoistedProjectionFunction.forward = staticmethod(counted)
        tm._HOIST_KV = True
        ops._SEED["n"] = 0
        try:
            lb = b(batch).loss
            lb.backward()
        finally:
            ops.HoistedProjectionFunction.forward = staticmethod(orig)
        if buckets_on:
            buckets.synchronize()
        assert calls == [2]   # n_layers=4: two decoder layers, one hoisted launch for both
        torch.testing.assert_close(lb.detach(), la.detach(), rtol=1e-6, atol=0)
        for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
            if pa.grad is None:
                assert pb.grad is None, n
                continue
            # split-K orders differ between the hoisted (M = 2 x 2A) and per-layer GEMMs: fp32 rounding only
            scale = float(pa.grad.abs().max())
            err = float((pb.grad - pa.grad).abs().max())
            assert err <= 1e-4 * scale + 1e-7, (n, err, scale)
    finally:
        tm._HOIST_KV = prev
        torch.set_float32_matmul_precision("highest")


@pytest.mark.parametrize("model_kind", ["mlp", "decoder"])
def test_deferred_reductions_bitwise(device, model_kind):
    """Deferred weight-gradient reductions (split-K slabs and RMSNorm partials batched into
    rq_reduce_partials launches at GradBuckets' flush points) give bitwise the gradients of the
    immediate reductions; they are pending after backward and flushed by synchronize()."""
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    from rqvae_hip import dp, ops
    torch.set_float32_matmul_precision("high")
    try:
        torch.manual_seed(7)
        if model_kind == "mlp":
            a = _Net().to(device)
            gen = torch.Generator(device=device).manual_seed(3)
            x = torch.randn(8192, 64, generator=gen, device=device)
            g = torch.randn(8192, 64, generator=gen, device=device)

            def run(m):
                m(x).backward(g)
        else:
            a = EncoderDecoderRetrievalModel(embedding_dim=64, attn_dim=128, dropout=0.0, num_heads=4, n_layers=4,
                                             num_embeddings=64, sem_id_dim=4, inference_verifier_fn=None,
                                             max_pos=80).to(device).train()
            batch = synthetic_tokenized_batch(64, 20, 4, 64, 9, device)

            def run(m):
                ops._SEED["n"] = 0
                m(batch).loss.backward()
        b = copy.deepcopy(a)
        res = {}
        for m, defer in ((a, False), (b, True)):
            buckets = dp.GradBuckets(m.parameters(), overlap=False, flat_views=True, defer_reductions=defer)
            buckets.zero_grad()
            run(m)
            if defer:
                assert ops.pending_reductions() > 0
            buckets.synchronize()
            assert ops.pending_reductions() == 0
            res[defer] = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
        assert res[True].keys() == res[False].keys()
        for n in res[False]:
            assert torch.equal(res[True][n], res[False][n]), n
    finally:
        torch.set_float32_matmul_precision("highest")


def test_segment_sum_multi_matches_per_table(device):
    """rq_segment_sum_multi over several sources (padding keys, out-of-range keys, an empty source) is
    bitwise the per-source rq_segment_sum into the stacked output."""
    import ctypes
    from rqvae_hip import _lib, ops
    gen = torch.Generator(device=device).manual_seed(11)
    spec = [(700, 257, 256), (0, 33, None), (1500, 1025, 1024), (90, 7, -1), (333, 64, 5)]
    E = 64
    rows, keys, pads = [], [], []
    for n, K, pad in spec:
        rows.append(torch.randn(n, E, generator=gen, device=device))
        keys.append(torch.randint(-2, K + 3, (n,), generator=gen, device=device))
        pads.append(-2 if pad is None else pad % K)
    n = len(spec)
    I64, P = ctypes.c_int64 * n, ctypes.c_void_p * n
    rn, Ks = I64(*[r.shape[0] for r in rows]), I64(*[s[1] for s in spec])
    L = _lib.load()
    nbytes = L.rq_segment_sum_multi_workspace(n, rn, Ks, E)
    ws = torch.empty(nbytes, device=device, dtype=torch.uint8)
    out = torch.full((sum(s[1] for s in spec), E), float("nan"), device=device)
    _lib.call("rq_segment_sum_multi", n, P(*[r.data_ptr() for r in rows]), P(*[k.data_ptr() for k in keys]), rn, Ks,
              I64(*pads), E, out.data_ptr(), ws.data_ptr(), nbytes, _lib.stream_handle(out.device))
    base = 0
    for (nr, K, _), r, k, pad in zip(spec, rows, keys, pads):
        kk = torch.where(k == pad, -1, k)
        want = ops.segment_sum(r, kk, K, with_counts=False)[0] if nr else torch.zeros(K, E, device=device)
        assert torch.equal(out[base:base + K], want)
        base += K


def test_deferred_embedding_grads_bitwise(device):
    """Embedding-table gradients batched at the flush (one rq_segment_sum_multi + the batched reduction)
    equal the per-table segmented sums bit for bit, and are pending until synchronize()."""
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    from rqvae_hip import dp, ops
    torch.set_float32_matmul_precision("high")
    try:
        torch.manual_seed(9)
        a = EncoderDecoderRetrievalModel(embedding_dim=64, attn_dim=128, dropout=0.0, num_heads=4, n_layers=2,
                                         num_embeddings=64, sem_id_dim=4, inference_verifier_fn=None,
                                         max_pos=80).to(device).train()
        b = copy.deepcopy(a)
        batch = synthetic_tokenized_batch(64, 20, 4, 64, 9, device)
        res = {}
        for m, on in ((a, False), (b, True)):
            prev = ops.emb_defer_enable(on)
            try:
                buckets = dp.GradBuckets(m.parameters(), overlap=False, flat_views=True, defer_reductions=True)
                buckets.zero_grad()
                ops._SEED["n"] = 0
                m(batch).loss.backward()
                if on:
                    assert len(ops._EMB["pending"]) > 0
                buckets.synchronize()
                assert ops.pending_reductions() == 0
            finally:
                ops.emb_defer_enable(prev)
            res[on] = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
        assert res[True].keys() == res[False].keys()
        for n in res[False]:
            assert torch.equal(res[True][n], res[False][n]), n
    finally:
        torch.set_float32_matmul_precision("highest")
