#!/usr/bin/env python3
"""cProfile of the host side of the bench decoder step (which is enqueue-bound): top functions by
own time and by cumulative time over 10 steps."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


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

    def step(i):
        opt.zero_grad(set_to_none=True)
        m(batches[i % 4]).loss.backward()
        opt.step()
    torch.autograd.set_multithreading_enabled(False)   # backward on this thread: visible to cProfile
    for i in range(5):
        step(i)
    torch.cuda.synchronize()
    import time
    t0 = time.perf_counter()
    for i in range(10):
        step(i)
    torch.cuda.synchronize()
    print("ms/step (single-threaded autograd, no profiler):", (time.perf_counter() - t0) * 100)
    pr = cProfile.Profile()
    pr.enable()
    for i in range(10):
        step(i)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumulative").print_stats(45)


if __name__ == "__main__":
    main()
