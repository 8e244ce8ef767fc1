#!/usr/bin/env python3
"""In-process A/B of step-level options (rounds interleaved, one box, one process: guide §5.4
rule 24). Options toggle module-level switches between rounds.

  python tools/ab_steps.py wgrad      # split-K kernel vs tuned library GEMM for weight grads
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from rqvae_hip import gemm_tuning, ops  # noqa: E402


def decoder_step_fn(device):
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    D = bench.DEC
    torch.manual_seed(3)
    m = EncoderDecoderRetrievalModel(embedding_dim=D["E"], attn_dim=D["A"], dropout=D["dropout"], num_heads=D["H"],
                                     n_layers=D["layers"], num_embeddings=D["K"], sem_id_dim=D["sem_id_dim"],
                                     inference_verifier_fn=None, max_pos=D["max_items"] * D["sem_id_dim"]).to(device)
    opt = torch.optim.AdamW(m.parameters(), lr=D["lr"], weight_decay=D["wd"], fused=True)
    batches = [synthetic_tokenized_batch(D["B"], D["max_items"], D["sem_id_dim"], D["K"], 50 + i, device)
               for i in range(4)]
    it = [0]

    def step():
        b = batches[it[0] % 4]
        it[0] += 1
        opt.zero_grad(set_to_none=True)
        m(b).loss.backward()
        opt.step()
    return step


def rqvae_step_fn(device):
    from data.schemas import SeqBatch
    m = bench.build_model(device)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=0.01, fused=True)
    x = bench.make_items(65536, 768, torch.Generator(device=device).manual_seed(0), device)

    def step():
        opt.zero_grad(set_to_none=True)
        m(SeqBatch(None, None, None, x, None, None), gumbel_t=0.2).loss.backward()
        opt.step()
    return step


def timed(step, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "wgrad"
    dev = torch.device("cuda", 0)
    gemm_tuning.enable()
    if what == "wgrad":
        arms = {"hip": lambda: setattr(ops, "WGRAD_TUNED_LIB_MAX_ROWS", 0),
                "lib": lambda: setattr(ops, "WGRAD_TUNED_LIB_MAX_ROWS", 1 << 30)}
    else:
        raise SystemExit(f"unknown A/B {what}")
    for name, make in (("decoder", decoder_step_fn), ("rqvae", rqvae_step_fn)):
        step = make(dev)
        res = {a: [] for a in arms}
        for a, setup in arms.items():   # warm both arms (tuning of new shapes happens here)
            setup()
            timed(step, 6)
        for _ in range(4):
            for a, setup in arms.items():
                setup()
                res[a].append(timed(step, 8))
        print(name, {a: round(sorted(v)[len(v) // 2], 3) for a, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()
