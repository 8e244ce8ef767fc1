"""Parity of the HIP jagged conversion and varlen attention (and the decoder model built on them)
with the reference's golden vectors and the pinned oracle.

Jagged values / offsets / grads: bit-exact (byte-moving kernels; `+1-1` rounding reproduced).
Attention: fp32 MFMA vs float64 oracle, |err| <= 2e-5 + 2e-4 |ref| (fwd) and 1e-4 + 1e-3 |ref| (bwd).
Decoder model (reference fixture, dropout 0): loss rel 1e-5, logits |err| <= 2e-4 max|logit|, grads rtol 2e-3.
"""
import numpy as np
import pytest
import torch

import gen_inputs as gi
from oracle import attention as A
from oracle import jagged as J

pytestmark = pytest.mark.gpu


def test_jagged_vs_reference(golden, device):
    from ops.jagged import padded_to_jagged_tensor, jagged_to_flattened_tensor
    z = golden("jagged")
    for case in ("ragged", "full", "ctx"):
        x = torch.from_numpy(z[f"{case}_x"]).to(device).requires_grad_(True)
        lengths = torch.from_numpy(z[f"{case}_lengths"]).to(device)
        nt = padded_to_jagged_tensor(x, lengths, x.shape[1])
        vals = jagged_to_flattened_tensor(nt)
        assert np.array_equal(nt.offsets().cpu().numpy(), z[f"{case}_offsets"])
        assert np.array_equal(vals.detach().cpu().numpy().view(np.uint32), z[f"{case}_values"].view(np.uint32))
        (vals * torch.from_numpy(z[f"{case}_gv"]).to(device)).sum().backward()
        assert np.array_equal(x.grad.cpu().numpy(), z[f"{case}_grad_x"])


@pytest.mark.parametrize("B,N,D,dtype", [(256, 81, 128, torch.float32), (64, 801, 128, torch.float32),
                                         (3, 7, 6, torch.float32), (37, 20, 128, torch.bfloat16),
                                         (5, 1, 8, torch.float32)])
def test_jagged_roundtrip_sizes(device, B, N, D, dtype):
    """padded -> jagged -> padded reproduces x on valid rows and zeros elsewhere (incl. empty rows)."""
    from rqvae_hip import ops
    g = gi.rng(B * N + D)
    lengths = torch.from_numpy(g.integers(0, N + 1, size=B)).to(device)
    x = torch.from_numpy(g.standard_normal((B, N, D), dtype=np.float32)).to(device=device, dtype=dtype)
    off = ops.jagged_offsets(lengths, N)
    total = int(off[-1])
    vals = ops.PaddedToJaggedValues.apply(x, off, total, False)
    back = ops.JaggedToPaddedValues.apply(vals, off, N)
    mask = torch.arange(N, device=device)[None, :] < lengths[:, None]
    assert torch.equal(back[mask], x[mask])
    assert torch.count_nonzero(back[~mask]) == 0
    v_np, o_np = J.padded_to_jagged(x.float().cpu().numpy(), lengths.cpu().numpy())
    if dtype == torch.float32:
        p1 = ops.PaddedToJaggedValues.apply(x, off, total, True)
        assert np.array_equal(p1.cpu().numpy().view(np.uint32), v_np.view(np.uint32))
    assert np.array_equal(off.cpu().numpy(), o_np)


def _varlen_case(g, B, max_q, max_k, H, hd, same):
    lq = g.integers(1, max_q + 1, size=B)
    lk = lq.copy() if same else g.integers(1, max_k + 1, size=B)
    cq = np.concatenate([[0], np.cumsum(lq)]).astype(np.int64)
    ck = np.concatenate([[0], np.cumsum(lk)]).astype(np.int64)
    q = g.standard_normal((cq[-1], H, hd), dtype=np.float32)
    k = g.standard_normal((ck[-1], H, hd), dtype=np.float32)
    v = g.standard_normal((ck[-1], H, hd), dtype=np.float32)
    do = g.standard_normal((cq[-1], H, hd), dtype=np.float32)
    return q, k, v, do, cq, ck


@pytest.mark.parametrize("B,max_q,max_k,H,hd,causal,same", [
    (7, 81, 81, 8, 64, False, True),     # encoder self-attention (DA)
    (9, 5, 5, 8, 64, True, True),        # decoder causal self-attention (DA)
    (6, 5, 81, 8, 64, False, False),     # cross-attention (DA)
    (3, 300, 300, 6, 64, False, True),   # long context (DM-like)
    (2, 801, 801, 6, 64, False, True),   # DM longest context (200 items x 4 + 1)
    (2, 1281, 1281, 8, 64, False, True), # C5 longest context (256 items x 5 + 1)
    (3, 6, 1281, 8, 64, False, False),   # C5 cross-attention: L+2 future queries x 1281 keys
    (2, 6, 6, 8, 64, True, True),        # C5 decoder causal self-attention
    (5, 128, 128, 8, 64, True, True),    # short forms: longest staged range (128 rows), causal
    (4, 64, 100, 8, 64, False, False),   # short forms: 64 queries x 100 keys (dQ stages 112 keys)
    (3, 17, 17, 8, 64, True, True),      # short forms: two query tiles per sequence, causal diagonal
    (5, 16, 128, 8, 64, False, False),   # few-query fused backward: a full query tile, 2 key tiles per wave
    (4, 16, 16, 8, 64, True, True),      # few-query fused backward: one wave, causal
    (3, 12, 40, 8, 64, False, False),    # few-query fused backward: two waves
    (4, 70, 70, 4, 32, True, True),
    (2, 40, 90, 2, 128, False, False),
    (5, 30, 30, 4, 16, True, True),      # small head dim (decoder fixtures: A=64, H=4)
    (4, 20, 33, 4, 16, False, False),
    (3, 200, 200, 6, 64, True, True),    # causal over several 64-key blocks (fused dQ partials, causal reduce)
    (4, 150, 260, 6, 64, False, False),  # long ragged q x k, lq != lk
])
@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("dma", [True, False])
def test_varlen_attention_vs_oracle(device, B, max_q, max_k, H, hd, causal, same, fused, dma):
    """One-pass (fused) and two-pass backwards, and the LDS-DMA short forms (key ranges <= 128, hd 64) on
    and off: the per-call RQ_ATTN_* policy flags."""
    from rqvae_hip import ops
    flags = (0 if fused else ops.ATTN_TWO_PASS) | (0 if dma else ops.ATTN_NO_DMA)
    with ops.attn_policy(flags):
        _attention_vs_oracle(device, B, max_q, max_k, H, hd, causal, same)


def _attention_vs_oracle(device, B, max_q, max_k, H, hd, causal, same):
    from rqvae_hip import ops
    g = gi.rng(B * 131 + max_q + hd)
    q, k, v, do, cq, ck = _varlen_case(g, B, max_q, max_k, H, hd, same)
    A_ = H * hd
    # strided inputs like the fused qkv projection output: (T, 3A) buffer
    qkv = np.concatenate([q.reshape(-1, A_), np.zeros_like(q.reshape(-1, A_)), np.zeros_like(q.reshape(-1, A_))], 1)
    qb = torch.from_numpy(qkv).to(device)[:, :A_].requires_grad_(True)
    kt = torch.from_numpy(k.reshape(-1, A_)).to(device).requires_grad_(True)
    vt = torch.from_numpy(v.reshape(-1, A_)).to(device).requires_grad_(True)
    cqt, ckt = torch.from_numpy(cq).to(device), torch.from_numpy(ck).to(device)
    out = ops.varlen_attention(qb, kt, vt, cqt, ckt, H, causal, int(np.diff(cq).max()), int(np.diff(ck).max()))
    out.backward(torch.from_numpy(do.reshape(-1, A_)).to(device))
    ref, _ = A.attn_fwd(q, k, v, cq, ck, causal)
    dq, dk, dv = A.attn_bwd(q, k, v, do, cq, ck, causal)
    def chk(a, b, atol, rtol, what):
        a = a.detach().cpu().double().numpy().reshape(b.shape)
        err = np.abs(a - b) - (atol + rtol * np.abs(b))
        assert err.max() <= 0, f"{what}: max abs err {np.abs(a - b).max():.3e}"
    chk(out, ref, 2e-5, 2e-4, "out")
    chk(qb.grad, dq, 1e-4, 1e-3, "dq")
    chk(kt.grad, dk, 1e-4, 1e-3, "dk")
    chk(vt.grad, dv, 1e-4, 1e-3, "dv")


@pytest.mark.parametrize("n", [81, 400])
def test_varlen_attention_deterministic(device, n):
    from rqvae_hip import ops
    g = gi.rng(11)
    q, k, v, do, cq, ck = _varlen_case(g, 16, n, n, 8, 64, True)
    mx = int(np.diff(cq).max())
    outs = []
    for _ in range(2):
        qt, kt, vt = (torch.from_numpy(a.reshape(a.shape[0], -1)).to(device).requires_grad_(True) for a in (q, k, v))
        o = ops.varlen_attention(qt, kt, vt, torch.from_numpy(cq).to(device), torch.from_numpy(ck).to(device), 8, False, mx, mx)
        o.backward(torch.from_numpy(do.reshape(do.shape[0], -1)).to(device))
        outs.append((o.detach(), qt.grad, kt.grad, vt.grad))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_varlen_attention_split_keys_cross(device):
    """Split-key forward (<= 16 queries over > 128 keys: the decoder's cross-attention) vs the fp64 oracle
    on ragged contexts incl. one shorter than a key block and an empty one, with zero-padded tail rows."""
    from rqvae_hip import ops
    g = gi.rng(2024)
    H, hd, nq = 6, 64, 6
    lk = [801, 0, 100, 300, 129]
    A_ = H * hd
    B = len(lk)
    cq = np.arange(B + 1, dtype=np.int64) * nq
    ck = np.concatenate([[0], np.cumsum(lk)]).astype(np.int64)
    Tq = int(cq[-1]) + 5
    q = g.standard_normal((Tq, H, hd), dtype=np.float32)
    k = g.standard_normal((ck[-1], H, hd), dtype=np.float32)
    v = g.standard_normal((ck[-1], H, hd), dtype=np.float32)
    do = g.standard_normal((Tq, H, hd), dtype=np.float32)
    qt = torch.from_numpy(q.reshape(Tq, A_)).to(device).requires_grad_(True)
    kt = torch.from_numpy(k.reshape(-1, A_)).to(device).requires_grad_(True)
    vt = torch.from_numpy(v.reshape(-1, A_)).to(device).requires_grad_(True)
    out = ops.varlen_attention(qt, kt, vt, torch.from_numpy(cq).to(device), torch.from_numpy(ck).to(device), H, False,
                               nq, max(lk))
    out.backward(torch.from_numpy(do.reshape(Tq, A_)).to(device))
    o = out.detach().cpu().double().numpy().reshape(Tq, H, hd)
    dq = qt.grad.cpu().double().numpy().reshape(Tq, H, hd)
    assert np.count_nonzero(o[cq[-1]:]) == 0 and np.count_nonzero(dq[cq[-1]:]) == 0
    for b in range(B):
        s0, s1 = cq[b], cq[b + 1]
        if lk[b] == 0:
            assert np.count_nonzero(o[s0:s1]) == 0 and np.count_nonzero(dq[s0:s1]) == 0
            continue
        cqb = np.array([0, nq], np.int64)
        ckb = np.array([0, lk[b]], np.int64)
        kb_, vb_ = k[ck[b]:ck[b + 1]], v[ck[b]:ck[b + 1]]
        ref, _ = A.attn_fwd(q[s0:s1], kb_, vb_, cqb, ckb, False)
        rdq, rdk, rdv = A.attn_bwd(q[s0:s1], kb_, vb_, do[s0:s1], cqb, ckb, False)
        assert np.all(np.abs(o[s0:s1] - ref) <= 2e-5 + 2e-4 * np.abs(ref)), b
        assert np.all(np.abs(dq[s0:s1] - rdq) <= 1e-4 + 1e-3 * np.abs(rdq)), b
        gk = kt.grad.cpu().double().numpy().reshape(-1, H, hd)[ck[b]:ck[b + 1]]
        assert np.all(np.abs(gk - rdk) <= 1e-4 + 1e-3 * np.abs(rdk)), b


@pytest.mark.parametrize("lq,lk", [([40, 50, 33], [200, 0, 140]), ([170, 0, 150], [170, 0, 150])])
def test_varlen_attention_fused_empty_and_tail(device, lq, lk):
    """Fused backward vs the two-pass form on ragged ranges with an empty segment and zero-padded tail
    rows (row bucketing): empty-key / empty-query segments and tail rows get zero gradients."""
    from rqvae_hip import ops
    g = gi.rng(sum(lq) + sum(lk))
    H, hd = 6, 64
    A_ = H * hd
    cq = torch.tensor(np.concatenate([[0], np.cumsum(lq)]), device=device)
    ck = torch.tensor(np.concatenate([[0], np.cumsum(lk)]), device=device)
    Tq, Tk = int(cq[-1]) + 7, int(ck[-1]) + 5   # allocated rows past the last segment
    q0 = torch.from_numpy(g.standard_normal((Tq, A_), dtype=np.float32)).to(device)
    k0 = torch.from_numpy(g.standard_normal((Tk, A_), dtype=np.float32)).to(device)
    v0 = torch.from_numpy(g.standard_normal((Tk, A_), dtype=np.float32)).to(device)
    do = torch.from_numpy(g.standard_normal((Tq, A_), dtype=np.float32)).to(device)
    res = {}
    for fused in (True, False):
        with ops.attn_policy(0 if fused else ops.ATTN_TWO_PASS):
            qt, kt, vt = (t.clone().requires_grad_(True) for t in (q0, k0, v0))
            o = ops.varlen_attention(qt, kt, vt, cq, ck, H, False, max(lq), max(lk))
            o.backward(do)
        res[fused] = (o.detach(), qt.grad, kt.grad, vt.grad)
    for a, b, what in zip(res[True], res[False], ("out", "dq", "dk", "dv")):
        assert torch.isfinite(a).all(), what
        torch.testing.assert_close(a, b, rtol=2e-5, atol=2e-5, msg=what)
    _, dq, dk, dv = res[True]
    assert torch.count_nonzero(dq[int(cq[-1]):]) == 0 and torch.count_nonzero(dk[int(ck[-1]):]) == 0
    assert torch.count_nonzero(dv[int(ck[-1]):]) == 0
    for b in range(len(lq)):
        if lk[b] == 0:
            assert torch.count_nonzero(dq[int(cq[b]):int(cq[b + 1])]) == 0


@pytest.mark.parametrize("lq,lk,causal", [
    ([5, 3, 0, 16], [81, 0, 40, 128], False),    # few queries (cross-attention)
    ([5, 1, 16, 7], [5, 1, 16, 7], True),        # few queries, causal
    ([81, 9, 0, 45, 17], [81, 9, 0, 45, 17], False),   # short self-attention (the Amazon encoder)
    ([81, 33, 70, 1, 17], [81, 33, 70, 1, 17], True),
    ([40, 0, 128, 20], [100, 30, 128, 0], False),      # 128 staged rows
])
def test_varlen_attention_fewq_fused_vs_two_pass(device, lq, lk, causal):
    """One-pass backwards (attn_bwd_fewq_fused_kernel: <= 16 queries; attn_bwd_short_fused_kernel: short
    self-attention) vs the two-pass kernels on ragged ranges with empty-query / empty-key segments and
    zero-padded tail rows; each run bitwise deterministic."""
    from rqvae_hip import ops
    g = gi.rng(sum(lq) * 7 + sum(lk))
    H, hd = 8, 64
    A_ = H * hd
    cq = torch.tensor(np.concatenate([[0], np.cumsum(lq)]), device=device)
    ck = torch.tensor(np.concatenate([[0], np.cumsum(lk)]), device=device)
    Tq, Tk = int(cq[-1]) + 3, int(ck[-1]) + 5
    q0 = torch.from_numpy(g.standard_normal((Tq, A_), dtype=np.float32)).to(device)
    k0 = torch.from_numpy(g.standard_normal((Tk, A_), dtype=np.float32)).to(device)
    v0 = torch.from_numpy(g.standard_normal((Tk, A_), dtype=np.float32)).to(device)
    do = torch.from_numpy(g.standard_normal((Tq, A_), dtype=np.float32)).to(device)
    res = {}
    for fused in (True, True, False):
        with ops.attn_policy(0 if fused else ops.ATTN_TWO_PASS):
            qt, kt, vt = (t.clone().requires_grad_(True) for t in (q0, k0, v0))
            o = ops.varlen_attention(qt, kt, vt, cq, ck, H, causal, max(lq), max(lk))
            o.backward(do)
        r = (qt.grad, kt.grad, vt.grad)
        if fused in res:
            for a, b in zip(res[fused], r):
                assert torch.equal(a, b)
        res[fused] = r
    for a, b, what in zip(res[True], res[False], ("dq", "dk", "dv")):
        assert torch.isfinite(a).all(), what
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5, msg=what)
    dq, dk, dv = res[True]
    assert torch.count_nonzero(dq[int(cq[-1]):]) == 0 and torch.count_nonzero(dk[int(ck[-1]):]) == 0
    assert torch.count_nonzero(dv[int(ck[-1]):]) == 0
    for b in range(len(lq)):
        if lk[b] == 0:
            assert torch.count_nonzero(dq[int(cq[b]):int(cq[b + 1])]) == 0
        if lq[b] == 0:
            assert torch.count_nonzero(dk[int(ck[b]):int(ck[b + 1])]) == 0


@pytest.mark.parametrize("bucket", [False, True])
def test_decoder_model_vs_reference(golden, device, monkeypatch, bucket):
    """Decoder fixture; `bucket` runs the context with its row count padded to the GEMM row bucket
    (zero tail rows carried through every row-wise op, ignored by attention): same results."""
    from data.schemas import TokenizedSeqBatch
    from modules.model import EncoderDecoderRetrievalModel
    from rqvae_hip import gemm_tuning
    monkeypatch.setattr(gemm_tuning, "is_enabled", lambda: bucket)
    z = golden("decoder_small")
    E, A_, H, nl, K, L1, n_max, seed = (int(z[k]) for k in ("E", "A", "H", "n_layers", "K", "L1", "n_max", "seed"))
    model = EncoderDecoderRetrievalModel(embedding_dim=E, attn_dim=A_, dropout=0.0, num_heads=H, n_layers=nl,
                                         num_embeddings=K, sem_id_dim=L1, inference_verifier_fn=None,
                                         max_pos=n_max * L1, jagged_mode=True)
    for m in model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    with torch.no_grad():
        for name, p in model.named_parameters():
            p.copy_(torch.from_numpy(gi.named_param(name, p.shape, seed)))
    model = model.to(device).train()
    keys = ("user_ids", "sem_ids", "sem_ids_fut", "seq_mask", "token_type_ids", "token_type_ids_fut")
    batch = TokenizedSeqBatch(**{k: torch.from_numpy(z[k]).to(device) for k in keys})
    out = model(batch)
    out.loss.backward()
    assert float(out.loss) == pytest.approx(float(z["loss"]), rel=1e-5)
    # fixture logits reach |400|: fp32 summation-order noise through 4 blocks scales with them
    scale = np.abs(z["logits"]).max()
    assert np.abs(out.logits.detach().cpu().numpy() - z["logits"]).max() <= 2e-4 * scale
    assert np.allclose(out.loss_d.detach().cpu().numpy(), z["loss_d"], rtol=2e-5, atol=0)
    for name, p in model.named_parameters():
        assert p.grad is None or bool(torch.isfinite(p.grad).all()), name
        key = "grad__" + name
        if key in z:
            ref = z[key]
            got = p.grad.cpu().numpy()
            assert np.all(np.abs(got - ref) <= 1e-5 + 2e-3 * np.abs(ref)), f"{name}: {np.abs(got - ref).max():.3e}"
        elif key + "__norm" in z:
            assert p.grad.double().norm().item() == pytest.approx(float(z[key + "__norm"]), rel=1e-4)
            assert np.all(np.abs(p.grad[0].cpu().numpy() - z[key + "__row0"]) <= 1e-5 + 2e-3 * np.abs(z[key + "__row0"]))


@pytest.mark.parametrize("B,max_q,max_k,H,causal,same", [
    (7, 81, 81, 8, False, True),      # encoder self-attention (DA)
    (9, 5, 5, 8, True, True),         # decoder causal self-attention
    (6, 5, 81, 8, False, False),      # cross-attention (DA)
    (2, 300, 300, 6, False, True),    # long context (DM-like)
    (3, 6, 400, 8, False, False),     # few queries over a long key range
])
def test_c_abi_entry_points_vs_oracle(device, B, max_q, max_k, H, causal, same):
    """The SURVEY §8(b)-named entries varlen_attn_fwd / varlen_attn_bwd (no scratch: no longest-first
    order, no split-key partials, the two-pass backward) called directly through the C ABI — the
    binding a reference-side maintainer would use — against the fp64 oracle."""
    from rqvae_hip._lib import call, ptr, stream_handle
    hd = 64
    g = gi.rng(B * 7 + max_q + max_k)
    q, k, v, do, cq, ck = _varlen_case(g, B, max_q, max_k, H, hd, same)
    A_ = H * hd
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a.reshape(a.shape[0], -1))).to(device)  # noqa: E731
    qt, kt, vt, dot = t(q), t(k), t(v), t(do)
    cqt, ckt = torch.from_numpy(cq).to(device), torch.from_numpy(ck).to(device)
    Tq, Tk = qt.shape[0], kt.shape[0]
    mq, mk = int(np.diff(cq).max()), int(np.diff(ck).max())
    scale = 1.0 / np.sqrt(hd)
    out = torch.empty((Tq, A_), device=device)
    lse = torch.empty((H, Tq), device=device)
    st = stream_handle(device)
    call("varlen_attn_fwd", ptr(qt), A_, ptr(kt), A_, ptr(vt), A_, ptr(cqt), ptr(ckt), B, H, hd, mq, mk, int(causal),
         float(scale), ptr(out), A_, ptr(lse), Tq, None, 0, 0, st)
    dq, dk, dv = (torch.empty((n, A_), device=device) for n in (Tq, Tk, Tk))
    delta = torch.empty((H, Tq), device=device)
    call("varlen_attn_bwd", ptr(qt), A_, ptr(kt), A_, ptr(vt), A_, ptr(out), A_, ptr(dot), A_, ptr(lse), Tq, ptr(cqt),
         ptr(ckt), B, H, hd, mq, mk, int(causal), float(scale), ptr(dq), A_, ptr(dk), A_, ptr(dv), A_, Tk, ptr(delta),
         None, 0, 0, st)
    torch.cuda.synchronize()
    ref, _ = A.attn_fwd(q, k, v, cq, ck, causal)
    rdq, rdk, rdv = A.attn_bwd(q, k, v, do, cq, ck, causal)

    def chk(a, b, atol, rtol, what):
        a = a.cpu().double().numpy().reshape(b.shape)
        err = np.abs(a - b) - (atol + rtol * np.abs(b))
        assert err.max() <= 0, f"{what}: max abs err {np.abs(a - b).max():.3e}"
    chk(out, ref, 2e-5, 2e-4, "out")
    chk(dq, rdq, 1e-4, 1e-3, "dq")
    chk(dk, rdk, 1e-4, 1e-3, "dk")
    chk(dv, rdv, 1e-4, 1e-3, "dv")


@pytest.mark.parametrize("qsplit", [1, 2, 3, 4])
def test_fused_backward_query_splits(device, qsplit):
    """The fused backward with each key block's query range split over `qsplit` workgroups (dK / dV
    partials summed in split order by attn_kv_reduce_kernel; the RQ_ATTN_QSPLIT(n) flag forces the count) vs
    the fp64 oracle on ragged long sequences (ML-32M lengths, causal and not) incl. an empty one and
    zero-padded tail rows; bitwise deterministic run to run."""
    from rqvae_hip import ops
    with ops.attn_policy(ops.ATTN_QSPLIT(qsplit)):
        for causal in (False, True):
            g = gi.rng(77 + qsplit + 5 * causal)
            H, hd = 6, 64
            A_ = H * hd
            ls = [801, 0, 333, 64, 517]
            cq = np.concatenate([[0], np.cumsum(ls)]).astype(np.int64)
            T = int(cq[-1]) + 9
            q = g.standard_normal((T, H, hd), dtype=np.float32)
            k = g.standard_normal((T, H, hd), dtype=np.float32)
            v = g.standard_normal((T, H, hd), dtype=np.float32)
            do = g.standard_normal((T, H, hd), dtype=np.float32)
            cqt = torch.from_numpy(cq).to(device)
            runs = []
            for _ in range(2):
                qt, kt, vt = (torch.from_numpy(a.reshape(T, A_)).to(device).requires_grad_(True) for a in (q, k, v))
                o = ops.varlen_attention(qt, kt, vt, cqt, cqt, H, causal, max(ls), max(ls))
                o.backward(torch.from_numpy(do.reshape(T, A_)).to(device))
                runs.append((o.detach(), qt.grad, kt.grad, vt.grad))
            for a, b in zip(*runs):
                assert torch.equal(a, b)
            _, dq, dk, dv = runs[0]
            n = int(cq[-1])
            for t in (dq, dk, dv):
                assert torch.count_nonzero(t[n:]) == 0
            rdq, rdk, rdv = A.attn_bwd(q[:n], k[:n], v[:n], do[:n], cq, cq, causal)
            for got, ref, what in ((dq, rdq, "dq"), (dk, rdk, "dk"), (dv, rdv, "dv")):
                a = got[:n].cpu().double().numpy().reshape(ref.shape)
                assert np.all(np.abs(a - ref) <= 1e-4 + 1e-3 * np.abs(ref)), (what, causal)



@pytest.mark.parametrize("B,max_q,max_k,H,hd,causal,same", [
    (3, 200, 200, 6, 64, True, True),     # chunked forward, causal
    (4, 150, 260, 6, 64, False, False),   # ragged q x k (key-split forward at few workgroups)
    (2, 801, 801, 6, 64, False, True),    # ML-32M context length (fused backward with query splits)
    (2, 700, 700, 4, 64, True, True),     # causal, several key blocks (dQ partials)
    (8, 81, 81, 8, 64, False, True),      # Amazon encoder contexts: short fused backward, 96 staged rows
    (5, 60, 60, 4, 64, True, True),       # short causal, 64 staged rows
    (4, 120, 100, 4, 64, False, False),   # short ragged q x k, 128 staged rows
    (5, 6, 801, 6, 64, False, False),     # cross-attention: few queries over long keys (key-split form)
])
def test_varlen_attention_split_bf16_vs_oracle(device, B, max_q, max_k, H, hd, causal, same):
    """At matmul precision 'high' the long-range forwards and the fused backward multiply in split-bf16
    (RQ_ATTN_SPLIT_BF16; per-product relative error <= ~2^-16, fp32 softmax / P / dS): the same oracle
    tolerances as the exact-fp32 forms, and within 1e-4 (forward) / 2e-4 (gradients) of them, relative to
    the largest magnitude."""
    from rqvae_hip import ops
    prev = torch.get_float32_matmul_precision()
    try:
        torch.set_float32_matmul_precision("high")
        _attention_vs_oracle(device, B, max_q, max_k, H, hd, causal, same)
        g = gi.rng(B * 7 + max_k)
        q, k, v, do, cq, ck = _varlen_case(g, B, max_q, max_k, H, hd, same)
        A_ = H * hd
        args = [torch.from_numpy(a.reshape(-1, A_)).to(device) for a in (q, k, v)]
        cqt, ckt = torch.from_numpy(cq).to(device), torch.from_numpy(ck).to(device)
        mq, mk = int(np.diff(cq).max()), int(np.diff(ck).max())
        dot = torch.from_numpy(do.reshape(-1, A_)).to(device)
        res = []
        for prec in ("high", "highest"):
            torch.set_float32_matmul_precision(prec)
            xs = [a.clone().requires_grad_(True) for a in args]
            o = ops.varlen_attention(*xs, cqt, ckt, H, causal, mq, mk)
            o.backward(dot)
            res.append([o.detach()] + [x.grad for x in xs])
        for i, (a, b) in enumerate(zip(*res)):
            tol = 1e-4 if i == 0 else 2e-4
            assert float((a - b).abs().max()) <= tol * float(b.abs().max()), ("out", "dq", "dk", "dv")[i]
    finally:
        torch.set_float32_matmul_precision(prev)


@pytest.mark.parametrize("fwd_prec,bwd_prec", [("highest", "high"), ("high", "highest")])
@pytest.mark.parametrize("B,max_q,max_k,H,hd,causal,same", [
    (2, 700, 700, 4, 64, True, True),     # chunked fwd / fused bwd (both split-bf16 at 'high')
    (8, 81, 81, 8, 64, False, True),      # short split-bf16 fwd at 'high' / short fp32 bwd always
    (6, 5, 81, 8, 64, False, False),      # few-query fp32 fwd always / few-query fp32 bwd
    (5, 6, 801, 6, 64, False, False),     # key-split fwd (split at 'high') / fused bwd (split at 'high')
    (5, 20, 20, 4, 64, True, True),       # max_k <= 32: fp32 fwd always / short bwd
])
def test_varlen_attention_precision_pairings_vs_oracle(device, fwd_prec, bwd_prec, B, max_q, max_k, H, hd, causal,
                                                       same):
    """lse (and O) may come from a forward at one product precision while the backward recomputes P from S at
    the other: the kernel a launch picks decides whether its products are split-bf16 or exact fp32 at 'high'
    (forwards: key-split, short_x3 (> 32 keys), chunked NW=4 split; fewq, NW 1/2 and <= 32 keys fp32;
    backward: only the fused long-range kernel is split). Every pairing — including the matmul precision
    changed between forward and backward — stays within the oracle tolerances of the exact forms."""
    from rqvae_hip import ops
    prev = torch.get_float32_matmul_precision()
    try:
        g = gi.rng(B * 977 + max_k)
        q, k, v, do, cq, ck = _varlen_case(g, B, max_q, max_k, H, hd, same)
        A_ = H * hd
        xs = [torch.from_numpy(a.reshape(-1, A_)).to(device).requires_grad_(True) for a in (q, k, v)]
        cqt, ckt = torch.from_numpy(cq).to(device), torch.from_numpy(ck).to(device)
        torch.set_float32_matmul_precision(fwd_prec)
        out = ops.varlen_attention(*xs, cqt, ckt, H, causal, int(np.diff(cq).max()), int(np.diff(ck).max()))
        torch.set_float32_matmul_precision(bwd_prec)
        out.backward(torch.from_numpy(do.reshape(-1, A_)).to(device))
        ref, _ = A.attn_fwd(q, k, v, cq, ck, causal)
        rg = A.attn_bwd(q, k, v, do, cq, ck, causal)
        for got, want, atol, rtol, what in ((out, ref, 2e-5, 2e-4, "out"), (xs[0].grad, rg[0], 1e-4, 1e-3, "dq"),
                                            (xs[1].grad, rg[1], 1e-4, 1e-3, "dk"), (xs[2].grad, rg[2], 1e-4, 1e-3, "dv")):
            a = got.detach().cpu().double().numpy().reshape(want.shape)
            assert np.all(np.abs(a - want) <= atol + rtol * np.abs(want)), (what, float(np.abs(a - want).max()))
    finally:
        torch.set_float32_matmul_precision(prev)



@pytest.mark.parametrize("lq,lk,causal", [
    ([81, 9, 45, 0, 17, 64, 33, 81], None, False),    # Amazon encoder self-attention (short one-pass forms)
    ([5, 1, 16, 7, 3], None, True),                    # few-query causal self-attention
    ([300, 12, 801, 45], None, False),                 # long ranges (LPT forward; fused backward)
])
def test_varlen_attention_lpt_order_bitwise(device, lq, lk, causal):
    """Longest-first dispatch of the short / few-query forms (RQ_ATTN_LPT_SHORT, computed by an order launch or
    taken from the offsets' attached order: RQ_ATTN_ORDER_GIVEN, as the decoder prologue provides it) only
    reorders independent (sequence, head) workgroups: out and gradients bitwise the default order's."""
    from rqvae_hip import ops
    g = gi.rng(sum(lq) * 5 + 3)
    H, hd = 8, 64
    A_ = H * hd
    lens = np.array(lq, dtype=np.int64)
    cu_np = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    Tq = int(cu_np[-1]) + 2
    q0, k0, v0, do = (torch.from_numpy(g.standard_normal((Tq, A_), dtype=np.float32)).to(device) for _ in range(4))
    order_np = sorted(range(len(lq)), key=lambda b: (-lq[b], b))
    res = {}
    for mode in ("default", "lpt", "given"):
        cu = torch.from_numpy(cu_np).to(device)
        if mode == "given":
            o = np.zeros(((len(lq) + 3) & ~3,), dtype=np.int32)
            o[:len(lq)] = order_np
            cu._rq_lpt_order = torch.from_numpy(o).to(device)
        with ops.attn_policy(ops.ATTN_LPT_SHORT if mode == "lpt" else 0):
            qt, kt, vt = (t.clone().requires_grad_(True) for t in (q0, k0, v0))
            out = ops.varlen_attention(qt, kt, vt, cu, cu, H, causal, max(lq), max(lq))
            out.backward(do)
        res[mode] = (out.detach(), qt.grad, kt.grad, vt.grad)
    for mode in ("lpt", "given"):
        for a, b, what in zip(res[mode], res["default"], ("out", "dq", "dk", "dv")):
            assert torch.equal(a, b), (mode, what)


@pytest.mark.parametrize("B,max_k,lpt", [
    (96, 81, False),    # the Amazon cross-attention shape: 96 x 8 units > 512 slots (workgroups walk twice)
    (96, 81, True),     # ... dispatched longest-first
    (40, 64, False),    # 64 staged key rows (phase-A DMA only)
    (70, 96, False),    # 96 rows
    (40, 128, False),   # 128 staged key rows (one slot per CU)
])
def test_varlen_attention_fewq_stream_bitwise(device, B, max_k, lpt):
    """The persistent few-query backward (attn_bwd_fewq_stream_kernel: each workgroup walks units, the next
    unit's K / V / Q / dO / O / lse staged by LDS-DMA while this one multiplies) against the workgroup-per-unit
    kernel (RQ_ATTN_FEWQ_WG): dQ, dK, dV bitwise, over ragged ranges with empty segments, rows past the last
    segment and more units than resident workgroups."""
    from rqvae_hip import ops
    g = gi.rng(B * 131 + max_k)
    H, hd = 8, 64
    A_ = H * hd
    lq = g.integers(0, 17, size=B)
    lk = g.integers(0, max_k + 1, size=B)
    lq[0], lk[0], lk[1], lk[2], lq[3] = 16, 1, max_k, 0, 0
    cq = torch.tensor(np.concatenate([[0], np.cumsum(lq)]), device=device)
    ck = torch.tensor(np.concatenate([[0], np.cumsum(lk)]), device=device)
    Tq, Tk = int(cq[-1]) + 3, int(ck[-1]) + 5
    q0 = torch.from_numpy(g.standard_normal((Tq, A_), dtype=np.float32)).to(device)
    k0 = torch.from_numpy(g.standard_normal((Tk, A_), dtype=np.float32)).to(device)
    v0 = torch.from_numpy(g.standard_normal((Tk, A_), dtype=np.float32)).to(device)
    do = torch.from_numpy(g.standard_normal((Tq, A_), dtype=np.float32)).to(device)
    res = {}
    for mode in ("stream", "wg", "stream2"):
        flags = (ops.ATTN_FEWQ_WG if mode == "wg" else 0) | (ops.ATTN_LPT_SHORT if lpt else 0)
        with ops.attn_policy(flags):
            qt, kt, vt = (t.clone().requires_grad_(True) for t in (q0, k0, v0))
            out = ops.varlen_attention(qt, kt, vt, cq, ck, H, False, 16, max_k)
            out.backward(do)
        res[mode] = (qt.grad, kt.grad, vt.grad)
    for mode in ("wg", "stream2"):
        for a, b, what in zip(res[mode], res["stream"], ("dq", "dk", "dv")):
            assert torch.equal(a, b), (mode, what)
    dq, dk, dv = res["stream"]
    assert torch.isfinite(dq).all() and torch.isfinite(dk).all() and torch.isfinite(dv).all()
    assert torch.count_nonzero(dq[int(cq[-1]):]) == 0 and torch.count_nonzero(dk[int(ck[-1]):]) == 0
    assert torch.count_nonzero(dv[int(ck[-1]):]) == 0
    for b in range(B):
        if lq[b] == 0:
            assert torch.count_nonzero(dk[int(ck[b]):int(ck[b + 1])]) == 0
