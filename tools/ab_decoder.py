#!/usr/bin/env python3
"""In-process A/B of the bench decoder step under a switch (interleaved rounds):

  python tools/ab_decoder.py presplit     # batched weight splits per forward vs one split per Linear call
"""
import contextlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "presplit"
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
    orig = type(m)._split_scope
    arms = {"on": lambda: setattr(type(m), "_split_scope", orig),
            "off": lambda: setattr(type(m), "_split_scope", lambda self: contextlib.nullcontext())}
    if what != "presplit":
        raise SystemExit(what)
    res = {a: [] for a in arms}
    for a, f in arms.items():
        f()
        for _ in range(5):
            step()
    for _ in range(5):
        for a, f in arms.items():
            f()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                step()
            torch.cuda.synchronize()
            res[a].append((time.perf_counter() - t0) / 10 * 1e3)
    print(json.dumps({a: round(sorted(v)[2], 3) for a, v in res.items()}))


if __name__ == "__main__":
    main()
