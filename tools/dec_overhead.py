#!/usr/bin/env python3
"""Where the decoder step's wall time goes beyond its kernels: times the bench decoder step
(a) as is, (b) with the context jagged totals taken from a per-batch host cache (no device ->
host sync inside the step), and reports the host-side enqueue time of one step (no sync).

  python tools/dec_overhead.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import ops.jagged as J  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    from rqvae_hip import gemm_tuning
    gemm_tuning.enable()
    D = bench.DEC
    torch.manual_seed(3)
    m = EncoderDecoderRetrievalModel(embedding_dim=D["E"], attn_dim=D["A"], dropout=D["dropout"], num_heads=D["H"],
                                     n_layers=D["layers"], num_embeddings=D["K"], sem_id_dim=D["sem_id_dim"],
                                     inference_verifier_fn=None, max_pos=D["max_items"] * D["sem_id_dim"]).to(dev)
    opt = torch.optim.AdamW(m.parameters(), lr=D["lr"], weight_decay=D["wd"], fused=True)
    batches = [synthetic_tokenized_batch(D["B"], D["max_items"], D["sem_id_dim"], D["K"], 50 + i, dev) for i in range(4)]
    it = [0]

    def step():
        b = batches[it[0] % 4]
        it[0] += 1
        opt.zero_grad(set_to_none=True)
        m(b).loss.backward()
        opt.step()

    def timed(n=20):
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    res = {"eager_ms": timed()}
    # host-side enqueue time of one step (GPU left to run behind)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step()
    res["enqueue_ms_one_step_incl_sync"] = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    # cached totals: no device->host sync in the step
    orig = J.padded_to_jagged
    cache = {}

    def cached(x, lengths, max_len, total=None, add_one_sub_one=True, known_max=None, row_bucket=None, known_min=None):
        if total is None:
            key = ((it[0] - 1) % 4, lengths.shape[0], int(max_len))   # the batch being stepped
            if key not in cache:
                n = min(int(max_len), x.shape[1])
                cache[key] = (int(lengths.clamp(0, n).sum()), int(lengths.clamp(0, n).max()))
            total, known_max = cache[key]
        return orig(x, lengths, max_len, total=total, add_one_sub_one=add_one_sub_one, known_max=known_max,
                    row_bucket=row_bucket, known_min=known_min)
    import modules.model as MM
    J.padded_to_jagged = cached
    MM.padded_to_jagged = cached
    res["no_sync_ms"] = timed()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step()
    res["enqueue_ms_one_step_no_sync"] = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    print(json.dumps({k: round(v, 3) for k, v in res.items()}))


if __name__ == "__main__":
    main()
