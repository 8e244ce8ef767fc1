#!/usr/bin/env python3
"""Per-launch-shape device times (HIP events via ops.TIMER) of every timed C-ABI call in one eager
decoder train step at the bench's Amazon config (or ML-32M with `dm`): GEMM keys
gemm_bf16x3:MxNxK:<a_kc><b_kc><a_split><b_split><epi>, attention, jagged.

  python tools/dec_gemm_keys.py [steps] [dm]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from rqvae_hip import dp, ops  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    cfg = dict(bench.DEC_DM if any(a.startswith("dm") for a in sys.argv[2:]) else bench.DEC)
    for a in sys.argv[2:]:   # dm8: the ML-32M config at 8 sequences
        if a.startswith("dm") and a[2:].isdigit():
            cfg["B"] = int(a[2:])
    dev = torch.device("cuda", 0)
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    torch.manual_seed(3)
    m = EncoderDecoderRetrievalModel(embedding_dim=cfg["E"], attn_dim=cfg["A"], dropout=cfg["dropout"],
                                     num_heads=cfg["H"], n_layers=cfg["layers"], num_embeddings=cfg["K"],
                                     sem_id_dim=cfg["sem_id_dim"], inference_verifier_fn=None,
                                     max_pos=cfg["max_items"] * cfg["sem_id_dim"]).to(dev).train()
    buckets = dp.GradBuckets(m.parameters(), overlap=False, flat_views=True)
    opt = bench.make_adamw(m.parameters(), cfg["lr"], cfg["wd"])
    b = synthetic_tokenized_batch(cfg["B"], cfg["max_items"], cfg["sem_id_dim"], cfg["K"], 50, dev)

    def step():
        buckets.zero_grad()
        m(b).loss.backward()
        buckets.synchronize()
        opt.step()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ops.TIMER.reset()
    ops.TIMER.enabled = True
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ops.TIMER.enabled = False
    tot = 0.0
    rows = []
    for k in sorted(ops.TIMER.events):
        ms, n = ops.TIMER.mean_ms(k)
        tot += ms * n / steps
        r = dict(key=k, us=round(ms * 1e3, 1), per_step=n // steps, us_per_step=round(ms * 1e3 * n / steps, 1))
        if k.startswith("gemm_bf16x3:"):
            M, N, K = (int(v) for v in k.split(":")[1].split("x"))
            r["tflops"] = round(2.0 * M * N * K / (ms * 1e-3) / 1e12, 1)
            f = [int(c) for c in k.split(":")[2]] + [0, 0, 0]
            r["plan"] = ops.gemm_x3_choice(M, N, K, bool(f[2]), bool(f[3]), bool(f[0]), bool(f[1]), f[4])
        rows.append(r)
    for r in sorted(rows, key=lambda r: -r["us_per_step"]):
        print(json.dumps(r))
    print(json.dumps({"timed_ms_per_step": round(tot, 3)}))


if __name__ == "__main__":
    main()
