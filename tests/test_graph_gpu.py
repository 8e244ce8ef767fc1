"""hipGraph capture of the decoder train step (rqvae_hip.graph.GraphedSteps) and the device-side
pieces it relies on:
* the jagged gather and the varlen attention kernels keep a row-bucketed buffer's tail rows zero
  on the device (outputs and gradients), whatever the allocation held;
* the dropout epoch (csrc/common.h) changes every mask key and is restored by setting it back;
* replaying a captured step equals the eager step (dropout 0: bitwise) for several batches of the
  same bucket with different exact row totals, and for a second bucket; with dropout on, every
  replay draws fresh masks (the epoch advances inside the graph).
"""
import numpy as np
import pytest
import torch

import gen_inputs as gi

pytestmark = pytest.mark.gpu


def test_gather_zero_fills_tail(device):
    from rqvae_hip import ops
    g = gi.rng(5)
    B, N, D = 7, 9, 16
    lengths = torch.from_numpy(g.integers(0, N + 1, size=B)).to(device)
    x = torch.from_numpy(g.standard_normal((B, N, D), dtype=np.float32)).to(device)
    off = ops.jagged_offsets(lengths, N)
    total = int(off[-1])
    for alloc in (total, total + 1, total + 37):
        torch.cuda.synchronize()
        junk = torch.full((alloc + 5, D), float("nan"), device=device)   # the allocator may hand back this memory
        del junk
        vals = ops.PaddedToJaggedValues.apply(x, off, alloc, False)
        assert vals.shape == (alloc, D)
        assert torch.equal(vals[total:], torch.zeros_like(vals[total:]))
        ref = ops.PaddedToJaggedValues.apply(x, off, total, False)
        assert torch.equal(vals[:total], ref)


@pytest.mark.parametrize("self_attn", [True, False])
def test_attention_zero_tails(device, self_attn):
    from rqvae_hip import ops
    g = gi.rng(9 + self_attn)
    H, hd, B = 4, 64, 5
    A = H * hd
    lq = g.integers(1, 40, size=B)
    lk = lq if self_attn else g.integers(1, 60, size=B)
    cq = torch.from_numpy(np.concatenate([[0], np.cumsum(lq)])).to(device)
    ck = torch.from_numpy(np.concatenate([[0], np.cumsum(lk)])).to(device)
    Tq, Tk = int(lq.sum()) + 29, int(lk.sum()) + 11
    if self_attn:
        qsrc = torch.randn(Tq, 3 * A, device=device)
        qsrc[int(lq.sum()):] = float("nan")           # tail rows: garbage must not leak anywhere
        kvsrc = None
    else:
        qsrc = torch.randn(Tq, A, device=device)
        kvsrc = torch.randn(Tk, 2 * A, device=device)
        qsrc[int(lq.sum()):] = float("nan")
        kvsrc[int(lk.sum()):] = float("nan")
    qsrc.requires_grad_(True)
    if kvsrc is not None:
        kvsrc.requires_grad_(True)
    out = ops.varlen_attention_packed(qsrc, kvsrc, cq, ck, H, False, int(lq.max()), int(lk.max()))
    assert torch.equal(out[int(lq.sum()):], torch.zeros_like(out[int(lq.sum()):]))
    assert bool(torch.isfinite(out).all())
    go = torch.randn_like(out)
    go[int(lq.sum()):] = 0
    out.backward(go)
    assert bool(torch.isfinite(qsrc.grad).all())
    assert torch.equal(qsrc.grad[int(lq.sum()):], torch.zeros_like(qsrc.grad[int(lq.sum()):]))
    if kvsrc is not None:
        assert torch.equal(kvsrc.grad[int(lk.sum()):], torch.zeros_like(kvsrc.grad[int(lk.sum()):]))


def test_seed_epoch_changes_masks(device):
    from rqvae_hip import ops
    h = torch.zeros(1 << 14, device=device)
    y = torch.ones(1 << 14, device=device)
    outs = []
    for epoch in (0, 3, 0):
        ops.seed_epoch_set(epoch)
        outs.append(ops.DropoutAddFunction.apply(h, y, 0.3, 1234).clone())
    ops.seed_epoch_set(0)
    assert torch.equal(outs[0], outs[2])
    assert not torch.equal(outs[0], outs[1])
    keep = [float((o != 0).float().mean()) for o in outs]
    assert all(abs(k - 0.7) < 0.02 for k in keep)


def _decoder(device, dropout):
    from modules.model import EncoderDecoderRetrievalModel
    torch.manual_seed(0)
    m = EncoderDecoderRetrievalModel(embedding_dim=32, attn_dim=64, dropout=dropout, num_heads=4, n_layers=4,
                                     num_embeddings=64, sem_id_dim=4, inference_verifier_fn=None, max_pos=40).to(device)
    if dropout == 0:
        for mod in m.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.0
    return m.train()


def _graphed(m, bucket=64):
    from ops.jagged import copy_row_counts
    from rqvae_hip import dp
    from rqvae_hip.graph import GraphedSteps
    buckets = dp.GradBuckets(m.parameters(), overlap=False, flat_views=True)
    gs = GraphedSteps(lambda b: m(b).loss, lambda b: m.context_rows(b, bucket), buckets,
                      prepare=lambda s, b: copy_row_counts(s.seq_mask, b.seq_mask))
    return gs, buckets


def test_graph_replay_equals_eager(device, monkeypatch):
    from data.processed import synthetic_tokenized_batch
    from rqvae_hip import gemm_tuning
    monkeypatch.setattr(gemm_tuning, "is_enabled", lambda: True)
    monkeypatch.setattr(gemm_tuning, "ROW_BUCKET", 64)
    torch.set_float32_matmul_precision("high")
    m = _decoder(device, 0.0)
    gs, buckets = _graphed(m)
    batches = [synthetic_tokenized_batch(12, 10, 4, 64, 100 + i, device) for i in range(24)]
    keys = [m.context_rows(b, 64) for b in batches]
    # three batches sharing a bucket (different exact totals) and one from another bucket
    same = [b for b, k in zip(batches, keys) if k == keys[0]][:3]
    other = next(b for b, k in zip(batches, keys) if k != keys[0])
    assert len(same) >= 2
    for b in same + [other] + same[:1]:
        loss_g = gs(b).clone()
        buckets.synchronize()
        grads_g = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
        buckets.zero_grad()
        loss_e = m(b).loss
        loss_e.backward()
        buckets.synchronize()
        loss_e = loss_e.detach()   # drop the eager autograd graph: its AccumulateGrad nodes (default
        #                            stream) must not be alive when the next bucket is captured
        assert torch.equal(loss_g, loss_e), (float(loss_g), float(loss_e))
        for n, p in m.named_parameters():
            if p.grad is not None:
                assert torch.equal(grads_g[n], p.grad), n
    assert len(gs.graphs) == 2
    unused = {n for n, p in m.named_parameters() if p.grad is None}
    assert unused and all("tte_fut" in n or "ffn_norm" in n for n in unused), unused


def test_graph_dropout_fresh_masks(device, monkeypatch):
    from data.processed import synthetic_tokenized_batch
    from rqvae_hip import gemm_tuning
    monkeypatch.setattr(gemm_tuning, "is_enabled", lambda: True)
    monkeypatch.setattr(gemm_tuning, "ROW_BUCKET", 64)
    m = _decoder(device, 0.3)
    gs, buckets = _graphed(m)
    b = synthetic_tokenized_batch(12, 10, 4, 64, 7, device)
    losses = [float(gs(b)) for _ in range(4)]
    assert len(set(losses)) == 4, losses     # same batch, same weights: only the masks differ
    assert len(gs.graphs) == 1
