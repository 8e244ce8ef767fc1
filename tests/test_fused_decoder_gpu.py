"""Decoder-side fusions against plain PyTorch fp32 references of the same ops:
RMSNorm + Dropout, SiLU + Dropout, residual + Dropout (counter-based masks regenerated in the
backward), the segmented-sum embedding backward, and packed-projection attention (no chunk cat).

Dropout masks are random by design, so the reference recovers the kernel's mask from its output
(kept elements are exactly value * 1/(1-p), dropped ones exactly 0) and checks the rest of the op
and its gradient against torch with that mask; the keep rate is checked statistically."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rms_ref(x, w, eps):
    return (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps)) * w


def _kernel_scale(p, device):
    """The kernels' 1/(1-p) (fp32, computed by the library) for bitwise comparisons."""
    import ctypes
    from rqvae_hip import _lib
    thr, scale = ctypes.c_uint32(), ctypes.c_float()
    assert _lib.load().rq_dropout_params(ctypes.c_float(p), ctypes.byref(thr), ctypes.byref(scale)) == 0
    return torch.tensor(scale.value, dtype=torch.float32, device=device)


def _check_rate(mask, p):
    n = mask.numel()
    rate = 1.0 - mask.float().mean().item()
    assert abs(rate - p) < 6 * np.sqrt(p * (1 - p) / n) + 1e-6, (rate, p)


@pytest.mark.parametrize("T,D,p", [(1000, 512, 0.3), (257, 128, 0.5), (64, 1024, 0.1)])
def test_rmsnorm_dropout(device, T, D, p):
    from rqvae_hip import ops
    g = torch.Generator(device=device).manual_seed(T + D)
    x = torch.randn(T, D, device=device, generator=g)
    w = torch.rand(D, device=device, generator=g) + 0.5
    gy = torch.randn(T, D, device=device, generator=g)
    plain = ops.rmsnorm(x, w, 1e-6)
    seed = 1234567
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    y = ops.RMSNormFunction.apply(xr, wr, 1e-6, p, seed)
    y.backward(gy)
    scale = _kernel_scale(p, device)
    mask = y != 0
    _check_rate(mask, p)
    assert torch.equal(y[mask], plain[mask] * scale), "kept values = rmsnorm * 1/(1-p), bitwise"
    y2 = ops.RMSNormFunction.apply(x, w, 1e-6, p, seed)
    assert torch.equal(y, y2), "same seed -> same mask"
    assert not torch.equal(y != 0, ops.RMSNormFunction.apply(x, w, 1e-6, p, seed + 1) != 0)
    xt, wt = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    ref = _rms_ref(xt, wt, 1e-6) * mask * scale
    ref.backward(gy)
    torch.testing.assert_close(xr.grad, xt.grad, rtol=2e-5, atol=2e-6)
    torch.testing.assert_close(wr.grad, wt.grad, rtol=2e-5, atol=2e-5)


def test_rmsnorm_dropout_p0_is_rmsnorm(device):
    from rqvae_hip import ops
    x = torch.randn(300, 512, device=device)
    w = torch.rand(512, device=device)
    assert torch.equal(ops.RMSNormFunction.apply(x, w, 1e-6, 0.0, 99), ops.rmsnorm(x, w, 1e-6))


@pytest.mark.parametrize("n,p", [(11600 * 1024, 0.3), (4096, 0.5)])
def test_silu_dropout(device, n, p):
    from rqvae_hip import ops
    g = torch.Generator(device=device).manual_seed(n)
    z = torch.randn(n, device=device, generator=g) * 3
    z[z == 0] = 1.0   # silu(0) == 0 would read as a dropped element below
    gh = torch.randn(n, device=device, generator=g)
    zr = z.clone().requires_grad_(True)
    h = ops.SiluDropoutFunction.apply(zr, p, 42)
    h.backward(gh)
    mask = h != 0
    _check_rate(mask, p)
    zt = z.clone().requires_grad_(True)
    ref = torch.nn.functional.silu(zt) * mask * _kernel_scale(p, device)
    ref.backward(gh)
    torch.testing.assert_close(h, ref, rtol=2e-6, atol=1e-7)
    torch.testing.assert_close(zr.grad, zt.grad, rtol=2e-6, atol=1e-7)
    # p = 0: plain SiLU
    torch.testing.assert_close(ops.SiluDropoutFunction.apply(z, 0.0, 1), torch.nn.functional.silu(z), rtol=2e-6, atol=0)


def test_dropout_add(device):
    from rqvae_hip import ops
    T, D, p = 5000, 512, 0.3
    g = torch.Generator(device=device).manual_seed(21)
    hh = torch.randn(T, D, device=device, generator=g)
    y = torch.randn(T, D, device=device, generator=g)
    go = torch.randn(T, D, device=device, generator=g)
    go[go == 0] = 1.0   # a zero gradient would read as a dropped element below
    hr, yr = hh.clone().requires_grad_(True), y.clone().requires_grad_(True)
    out = ops.DropoutAddFunction.apply(hr, yr, p, 7)
    out.backward(go)
    scale = _kernel_scale(p, device)
    mask = yr.grad != 0   # gradient of y carries the mask
    _check_rate(mask, p)
    assert torch.equal(out, hh + torch.where(mask, y * scale, torch.zeros_like(y)))
    assert torch.equal(hr.grad, go)
    assert torch.equal(yr.grad, torch.where(mask, go * scale, torch.zeros_like(go)))


def test_embedding_segment_sum_backward(device):
    from rqvae_hip import ops
    K, E = 1025, 128
    g = torch.Generator(device=device).manual_seed(5)
    w = torch.randn(K, E, device=device, generator=g)
    idx = torch.randint(0, K, (256, 80), device=device, generator=g)
    idx[:, 40:] = K - 1   # padding rows
    idx[:, 3:40:4] = 768  # a heavy key (the dedup-column token): 2,560 rows, split across workgroups
    go = torch.randn(256, 80, E, device=device, generator=g)
    wr = w.clone().requires_grad_(True)
    out = ops.embedding(idx, wr, K - 1)
    out.backward(go)
    wt = w.clone().requires_grad_(True)
    ref = torch.nn.functional.embedding(idx, wt, padding_idx=K - 1)
    ref.backward(go)
    assert torch.equal(out, ref)
    torch.testing.assert_close(wr.grad, wt.grad, rtol=1e-5, atol=1e-4)   # 2,560-row sums, other order
    assert torch.all(wr.grad[K - 1] == 0)
    # bitwise deterministic
    wr2 = w.clone().requires_grad_(True)
    ops.embedding(idx, wr2, K - 1).backward(go)
    assert torch.equal(wr.grad, wr2.grad)


def test_embedding_pair_equals_concatenated_gather(device):
    """embedding_pair(ia, ib): outputs and table gradient bitwise equal to gathering cat([ia, ib], 1)
    and slicing (the SemIdEmbedder's context + future tokens), a missing output gradient included."""
    from rqvae_hip import ops
    K, E = 1025, 128
    g = torch.Generator(device=device).manual_seed(9)
    w = torch.randn(K, E, device=device, generator=g)
    ia = torch.randint(0, K, (256, 80), device=device, generator=g)
    ia[:, 50:] = K - 1
    ib = torch.randint(0, 1024, (256, 5), device=device, generator=g)
    ga = torch.randn(256, 80, E, device=device, generator=g)
    gb = torch.randn(256, 5, E, device=device, generator=g)
    for use_b in (True, False):
        w1 = w.clone().requires_grad_(True)
        a, b = ops.embedding_pair(ia, ib, w1, K - 1)
        ((a * ga).sum() + ((b * gb).sum() if use_b else 0)).backward()
        w2 = w.clone().requires_grad_(True)
        both = ops.embedding(torch.cat([ia, ib], 1), w2, K - 1)
        ((both[:, :80] * ga).sum() + ((both[:, 80:] * gb).sum() if use_b else 0)).backward()
        assert torch.equal(a, both[:, :80]) and torch.equal(b, both[:, 80:])
        assert torch.equal(w1.grad, w2.grad)


@pytest.mark.parametrize("B,rest", [(256, (80, 128)), (3, (1, 4)), (1000, (7, 12))])
def test_batch_add_and_repeat(device, B, rest):
    """batch_add / batch_repeat (modules/model.py:92-93): forward bitwise equal to torch's broadcast
    add / repeat; the parameter gradient (fixed-order batch sum) within fp32 summation-order tolerance
    of torch's and bitwise reproducible; col_sum of an empty batch is zero."""
    from rqvae_hip import ops
    g = torch.Generator(device=device).manual_seed(B)
    x = torch.randn((B,) + rest, device=device, generator=g)
    p = torch.randn((1,) + rest, device=device, generator=g)
    go = torch.randn((B,) + rest, device=device, generator=g)
    grads = []
    for _ in range(2):
        xa, pa = x.clone().requires_grad_(True), p.clone().requires_grad_(True)
        y = ops.batch_add(xa, pa)
        y.backward(go)
        grads.append(pa.grad)
    xb, pb = x.clone().requires_grad_(True), p.clone().requires_grad_(True)
    yb = pb + xb
    yb.backward(go)
    assert torch.equal(y, yb) and torch.equal(xa.grad, xb.grad)
    torch.testing.assert_close(grads[0], pb.grad, rtol=1e-5, atol=1e-5)
    assert torch.equal(grads[0], grads[1])
    q = p[0].clone().requires_grad_(True)
    r = ops.batch_repeat(q, B)
    r.backward(go)
    qt = p[0].clone().requires_grad_(True)
    rt = qt.unsqueeze(0).repeat((B,) + (1,) * qt.dim())
    rt.backward(go)
    assert torch.equal(r, rt)
    torch.testing.assert_close(q.grad, qt.grad, rtol=1e-5, atol=1e-5)
    assert torch.all(ops.col_sum(torch.empty((0,) + rest, device=device)) == 0)


@pytest.mark.parametrize("N,D,K", [(20000, 128, 1025), (5000, 64, 7), (3, 8, 4096), (65536, 1024, 300)])
def test_segment_sum_vs_index_add(device, N, D, K):
    """Deterministic segmented sum (light segments in one workgroup, heavy ones split and finalized)
    against torch index_add_ in fp64; out-of-range keys are skipped."""
    from rqvae_hip import ops
    g = torch.Generator(device=device).manual_seed(N + K)
    rows = torch.randn(N, D, device=device, generator=g)
    keys = torch.randint(0, K, (N,), device=device, generator=g)
    keys[: N // 3] = min(5, K - 1)    # heavy segment
    keys[N // 3: N // 3 + 7] = -1     # skipped
    sums, counts = ops.segment_sum(rows, keys, K)
    ok = keys >= 0
    ref = torch.zeros(K, D, device=device, dtype=torch.float64).index_add_(0, keys[ok], rows[ok].double())
    torch.testing.assert_close(sums.double(), ref, rtol=1e-5, atol=max(1e-4, 5e-8 * N))   # fp32 sums of N/3 rows
    assert torch.equal(counts, torch.bincount(keys[ok], minlength=K))
    sums2, _ = ops.segment_sum(rows, keys, K)
    assert torch.equal(sums, sums2)


@pytest.mark.parametrize("cross", [False, True])
def test_packed_attention_matches_unpacked(device, cross):
    from rqvae_hip import ops
    H, A = 8, 512
    g = torch.Generator(device=device).manual_seed(11)
    lens_q = torch.tensor([5, 5, 5, 5], device=device) if cross else torch.tensor([45, 1, 81, 17], device=device)
    lens_k = torch.tensor([45, 1, 81, 17], device=device)
    cu_q = torch.cat([torch.zeros(1, device=device, dtype=torch.int64), lens_q.cumsum(0)])
    cu_k = torch.cat([torch.zeros(1, device=device, dtype=torch.int64), lens_k.cumsum(0)])
    Tq, Tk = int(cu_q[-1]), int(cu_k[-1])
    if cross:
        qs = torch.randn(Tq, A, device=device, generator=g).requires_grad_(True)
        kvs = torch.randn(Tk, 2 * A, device=device, generator=g).requires_grad_(True)
        out = ops.varlen_attention_packed(qs, kvs, cu_q, cu_k, H, False, 5, 81)
        q2, kv2 = qs.detach().clone().requires_grad_(True), kvs.detach().clone().requires_grad_(True)
        k, v = kv2.chunk(2, dim=-1)
        ref = ops.varlen_attention(q2, k, v, cu_q, cu_k, H, False, 5, 81)
    else:
        qs = torch.randn(Tq, 3 * A, device=device, generator=g).requires_grad_(True)
        kvs = None
        out = ops.varlen_attention_packed(qs, None, cu_q, cu_q, H, True, 81, 81)
        q2 = qs.detach().clone().requires_grad_(True)
        q, k, v = q2.chunk(3, dim=-1)
        ref = ops.varlen_attention(q, k, v, cu_q, cu_q, H, True, 81, 81)
    go = torch.randn_like(out)
    out.backward(go)
    ref.backward(go)
    assert torch.equal(out, ref)
    assert torch.equal(qs.grad, q2.grad)
    if cross:
        assert torch.equal(kvs.grad, kv2.grad)


@pytest.mark.parametrize("rows", [1280, 11332])
def test_mlp_residual_dropout_equals_composition(device, rows):
    """h + Dropout(MLP(x)) with the residual and the output dropout in the chain's last GEMM epilogue
    (ops.mlp_chain_residual) equals mlp_chain followed by dropout_add under the same dropout keys:
    bitwise output and gradients (x, h, weights)."""
    from rqvae_hip import ops
    torch.set_float32_matmul_precision("high")
    g = torch.Generator(device=device).manual_seed(rows)
    A, F = 512, 1024
    x0 = torch.randn(rows, A, generator=g, device=device)
    h0 = torch.randn(rows, A, generator=g, device=device)
    w0 = [torch.randn(F, A, generator=g, device=device) * 0.04, torch.randn(A, F, generator=g, device=device) * 0.03]
    go = torch.randn(rows, A, generator=g, device=device)
    res = []
    for fused in (True, False):
        x, h = x0.clone().requires_grad_(True), h0.clone().requires_grad_(True)
        ws = [w.clone().requires_grad_(True) for w in w0]
        ops._SEED["n"] = 0
        if fused:
            out = ops.mlp_chain_residual(x, ws, 0.3, h, 0.3)
        else:
            out = ops.dropout_add(h, ops.mlp_chain(x, ws, 0.3), 0.3)
        out.backward(go)
        res.append((out.detach(), x.grad, h.grad, *[w.grad for w in ws]))
    for a, b, what in zip(res[0], res[1], ("out", "dx", "dh", "dw0", "dw1")):
        assert torch.equal(a, b), f"{what}: max abs diff {(a - b).abs().max().item():.3e}"


@pytest.mark.parametrize("buckets", [False, True])
@pytest.mark.parametrize("B,max_items,sem_id_dim", [(16, 20, 4), (3, 7, 3), (40, 200, 4)])
def test_decoder_prologue_equals_composition(device, monkeypatch, buckets, B, max_items, sem_id_dim):
    """The fused input embeddings (rq_dec_prologue_fwd: user / sem-ID / position / token-type gathers, the
    adds, bos, the +1-1 jagged gather, both offsets) vs the model's composition of the same ops: loss and
    every parameter gradient bitwise equal, with plain .grad accumulation and with the flat-bucket
    (deferred segmented sum) path; the context's allocation tail zero."""
    from data.processed import synthetic_tokenized_batch
    from modules import model as model_mod
    from ops.jagged import row_counts
    from rqvae_hip import dp, ops
    torch.manual_seed(0)
    m = model_mod.EncoderDecoderRetrievalModel(embedding_dim=64, attn_dim=128, dropout=0.0, num_heads=4, n_layers=2,
                                               num_embeddings=64, sem_id_dim=sem_id_dim, inference_verifier_fn=None,
                                               max_pos=max_items * sem_id_dim).to(device)
    m.do.p = 0.0
    batch = synthetic_tokenized_batch(B, max_items, sem_id_dim, 64, 7, device)
    batch = batch._replace(user_ids=batch.user_ids - 500_000)   # negative ids: remainder's sign convention
    from ops.jagged import register_row_counts
    register_row_counts(batch.seq_mask, batch.seq_mask.sum(1).tolist())
    gb = dp.GradBuckets(m.parameters(), flat_views=True) if buckets else None
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(model_mod, "_FUSED_PROLOGUE", fused)
        if gb is not None:
            gb.zero_grad()
        else:
            m.zero_grad(set_to_none=True)
        loss = m(batch).loss
        loss.backward()
        if gb is not None:
            ops.flush_reductions()
        res[fused] = (loss.detach().clone(), {n: (None if p.grad is None else p.grad.detach().clone())
                                              for n, p in m.named_parameters()})
    assert torch.equal(res[True][0], res[False][0])
    for n in res[False][1]:
        a, b = res[True][1][n], res[False][1][n]
        assert (a is None) == (b is None), n
        if a is not None:
            assert torch.equal(a, b), (n, float((a - b).abs().max()))
    # the op alone: values of the allocation tail are zero, offsets as the composition's
    se, ue = m.sem_id_embedder, m.user_id_embedder
    alloc = m.context_rows(batch, 64)
    cv, co, fv, fo = ops.decoder_prologue(ue.emb.weight, se.emb.weight, m.wpe.weight, m.tte.weight, m.bos_emb,
                                          batch.user_ids, batch.sem_ids, batch.token_type_ids, batch.seq_mask,
                                          batch.sem_ids_fut, batch.token_type_ids_fut, ue.num_buckets,
                                          se.num_embeddings, se.padding_idx, alloc)
    lens = batch.seq_mask.sum(1) + 1
    assert torch.equal(co, torch.cat([lens.new_zeros(1), lens.cumsum(0)]))
    assert torch.equal(fo, torch.arange(B + 1, device=device) * (batch.sem_ids_fut.shape[1] + 1))
    assert torch.count_nonzero(cv[int(co[-1]):]) == 0
    assert row_counts(batch.seq_mask)[0] + B == int(co[-1])
    # the longest-first order handed to the attention launches: length descending, ties by index
    ln = lens.tolist()
    want = sorted(range(B), key=lambda b: (-ln[b], b))
    assert co._rq_lpt_order[:B].tolist() == want


@pytest.mark.parametrize("M,I,O1,O2", [(40, 384, 1152, 384), (1280, 512, 1536, 512), (300, 64, 192, 64)])
def test_linear_pair_equals_two_linears(device, M, I, O1, O2):
    """linear_pair (the block's self-attention qkv + cross-attention q projections of two inputs in one
    rq_gemm_bf16x3_pair launch, slab reductions batched) vs two LinearFunction calls: outputs and all four
    gradients bitwise, at split-K row counts (40: the C4 future tokens) and unsplit ones."""
    from rqvae_hip import ops
    g = torch.Generator(device=device).manual_seed(M + I)
    x1, x2 = (torch.randn(M, I, device=device, generator=g) for _ in range(2))
    w1 = torch.randn(O1, I, device=device, generator=g) * 0.05
    w2 = torch.randn(O2, I, device=device, generator=g) * 0.05
    gy1 = torch.randn(M, O1, device=device, generator=g)
    gy2 = torch.randn(M, O2, device=device, generator=g)
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("high")
    try:
        res = []
        for paired in (True, False):
            ts = [t.clone().requires_grad_(True) for t in (x1, w1, x2, w2)]
            if paired:
                assert ops.linear_pair_supported(*ts)
                y1, y2 = ops.linear_pair(*ts)
            else:
                y1 = ops.LinearFunction.apply(ts[0], ts[1], None)
                y2 = ops.LinearFunction.apply(ts[2], ts[3], None)
            torch.autograd.backward([y1, y2], [gy1, gy2])
            res.append((y1.detach(), y2.detach(), *[t.grad for t in ts]))
    finally:
        torch.set_float32_matmul_precision(prev)
    for a, b, what in zip(res[0], res[1], ("y1", "y2", "dx1", "dw1", "dx2", "dw2")):
        assert torch.equal(a, b), f"{what}: max abs diff {(a - b).abs().max().item():.3e}"
    ref = x1 @ w1.t()
    torch.testing.assert_close(res[0][0], ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("buckets", [False, True])
def test_decoder_pair_proj_equals_separate(device, monkeypatch, buckets):
    """The decoder with the block's qkv / cross-q projections paired (_PAIR_PROJ) vs two launches: loss and
    every parameter gradient bitwise, with and without flat gradient buckets."""
    from data.processed import synthetic_tokenized_batch
    from modules import model as model_mod
    from modules.transformer import model as tmodel
    from rqvae_hip import dp, ops
    torch.manual_seed(0)
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("high")
    try:
        m = model_mod.EncoderDecoderRetrievalModel(embedding_dim=64, attn_dim=128, dropout=0.1, num_heads=4,
                                                   n_layers=2, num_embeddings=64, sem_id_dim=4,
                                                   inference_verifier_fn=None, max_pos=80).to(device)
        batch = synthetic_tokenized_batch(24, 20, 4, 64, 7, device)
        gb = dp.GradBuckets(m.parameters(), flat_views=True) if buckets else None
        res = {}
        for paired in (True, False):
            monkeypatch.setattr(tmodel, "_PAIR_PROJ", paired)
            if gb is not None:
                gb.zero_grad()
            else:
                m.zero_grad(set_to_none=True)
            torch.manual_seed(5)
            ops._SEED["base"] = None   # restart the dropout-key counter: both passes draw the same masks
            loss = m(batch).loss
            loss.backward()
            if gb is not None:
                ops.flush_reductions()
            res[paired] = (loss.detach().clone(), {n: (None if p.grad is None else p.grad.detach().clone())
                                                   for n, p in m.named_parameters()})
    finally:
        torch.set_float32_matmul_precision(prev)
    assert torch.equal(res[True][0], res[False][0])
    for n in res[False][1]:
        a, b = res[True][1][n], res[False][1][n]
        assert (a is None) == (b is None), n
        if a is not None:
            assert torch.equal(a, b), (n, float((a - b).abs().max()))


@pytest.mark.parametrize("B,max_items", [(256, 20), (16, 20), (5, 7)])
def test_decoder_prologue_noncanonical_mask_and_short_alloc(device, B, max_items):
    """a bool mask whose bytes are any nonzero value (a uint8 tensor viewed as bool) counts as the
    canonical 0 / 1 mask (the staged many-sequence path sums bytes); an allocation below the valid total
    clamps the context offsets to it, so no consumer reads past the values."""
    from data.processed import synthetic_tokenized_batch
    from modules import model as model_mod
    from rqvae_hip import ops
    torch.manual_seed(0)
    m = model_mod.EncoderDecoderRetrievalModel(embedding_dim=64, attn_dim=128, dropout=0.0, num_heads=4, n_layers=2,
                                               num_embeddings=64, sem_id_dim=4, inference_verifier_fn=None,
                                               max_pos=max_items * 4).to(device)
    batch = synthetic_tokenized_batch(B, max_items, 4, 64, 11, device)
    se, ue = m.sem_id_embedder, m.user_id_embedder

    def run(mask, alloc):
        return ops.decoder_prologue(ue.emb.weight, se.emb.weight, m.wpe.weight, m.tte.weight, m.bos_emb,
                                    batch.user_ids, batch.sem_ids, batch.token_type_ids, mask, batch.sem_ids_fut,
                                    batch.token_type_ids_fut, ue.num_buckets, se.num_embeddings, se.padding_idx, alloc)
    total = int(batch.seq_mask.sum()) + B
    ref = run(batch.seq_mask, total)
    raw = batch.seq_mask.to(torch.uint8) * torch.tensor([2, 255, 17, 128], dtype=torch.uint8, device=device).repeat(
        batch.seq_mask.shape[1] // 4 + 1)[:batch.seq_mask.shape[1]]
    odd = raw.view(torch.bool)
    got = run(odd, total)
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
    short = total - max(1, total // 3)
    cv, co, _, _ = run(batch.seq_mask, short)
    assert int(co.max()) <= short and bool((co[1:] >= co[:-1]).all())
    assert torch.equal(co, ref[1].clamp(max=short))
    assert torch.equal(cv[:short], ref[0][:short])
