#!/usr/bin/env python3
"""Bisect hipGraph capture of the decoder step: python3 tools/graph_debug.py <stage> (one stage per
process; a crash in capture ends the process)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
import torch  # noqa: E402


def graphed(stage):
    """GraphedSteps over batches of two buckets, interleaved with eager steps (the GPU test's flow)."""
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    from ops.jagged import copy_row_counts
    from rqvae_hip import dp, gemm_tuning
    from rqvae_hip.graph import GraphedSteps
    if "bucket" in stage:
        gemm_tuning.is_enabled = lambda: True
        gemm_tuning.ROW_BUCKET = 64
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = EncoderDecoderRetrievalModel(embedding_dim=32, attn_dim=64, dropout=0.0, num_heads=4, n_layers=4,
                                     num_embeddings=64, sem_id_dim=4, inference_verifier_fn=None, max_pos=40).to(dev)
    if "p0" in stage:
        for mod in m.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.0
    if "highest" in stage:
        torch.set_float32_matmul_precision("highest")
    buckets = dp.GradBuckets(m.parameters(), overlap=False, flat_views=True)
    bk = 64 if "bucket" in stage else None
    gs = GraphedSteps(lambda b: m(b).loss, lambda b: m.context_rows(b, bk), buckets,
                      prepare=lambda s, b: copy_row_counts(s.seq_mask, b.seq_mask))
    batches = [synthetic_tokenized_batch(12, 10, 4, 64, 100 + i, dev) for i in range(24)]
    keys = [m.context_rows(b, bk) for b in batches]
    print("keys", keys[:8], flush=True)
    order = [0, 1, next(i for i, k in enumerate(keys) if k != keys[0]), 0]
    for i in order:
        print("step", i, "key", keys[i], "captured", list(gs.graphs), flush=True)
        loss = gs(batches[i])
        torch.cuda.synchronize()
        print(" graph loss", float(loss), flush=True)
        if "eager" in stage:
            buckets.zero_grad()
            m(batches[i]).loss.backward()
            torch.cuda.synchronize()
            print(" eager ok", flush=True)


def main(stage):
    if stage.startswith("graphed"):
        return graphed(stage)
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    from ops.jagged import copy_row_counts
    from rqvae_hip import dp, ops
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = EncoderDecoderRetrievalModel(embedding_dim=32, attn_dim=64, dropout=0.0, num_heads=4, n_layers=4,
                                     num_embeddings=64, sem_id_dim=4, inference_verifier_fn=None, max_pos=40).to(dev)
    if "p0" in stage:
        for mod in m.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.0
    b = synthetic_tokenized_batch(12, 10, 4, 64, 7, dev)
    static = type(b)(*[t.clone() for t in b])
    copy_row_counts(static.seq_mask, b.seq_mask)
    buckets = dp.GradBuckets(m.parameters(), overlap=False, flat_views=True) if "buckets" in stage else None

    def body():
        if buckets is not None:
            buckets.zero_grad()
        loss = m(static).loss
        if "bwd" in stage:
            loss.backward()
        if "epoch" in stage:
            ops.seed_epoch_advance()
        return loss.detach()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            body()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    if buckets is None:
        m.zero_grad(set_to_none=True)
    g = torch.cuda.CUDAGraph()
    print("capturing", stage, flush=True)
    with torch.cuda.graph(g):
        loss = body()
    print("captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print("replayed", float(loss), flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
