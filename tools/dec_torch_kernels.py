#!/usr/bin/env python3
"""Which Python call sites launch the torch (non-rqhip) GPU kernels of one eager decoder train step
at the bench's Amazon config (same model, GradBuckets with flat views, HIP AdamW): torch.profiler
with stacks, device time per (kernel, top user frame).   python tools/dec_torch_kernels.py [dm B]
(`dm 8`: the ML-32M config at 8 sequences, the C4 per-rank shape)."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from rqvae_hip import dp, gemm_tuning
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    cfg = dict(bench.DEC)
    if len(sys.argv) > 2 and sys.argv[1] == "dm":
        cfg = dict(bench.DEC_DM, B=int(sys.argv[2]))
    dev = torch.device("cuda", 0)
    gemm_tuning.enable()
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
    torch.autograd.set_multithreading_enabled(False)
    for _ in range(4):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_stack_n=12)
    rows = []
    for e in ka:
        dt = getattr(e, "self_device_time_total", 0.0)
        if dt <= 0 or not e.key.startswith("aten::"):
            continue
        st = [f.split("rq-vae-recommender_amd/")[-1] for f in (e.stack or [])
              if "rq-vae-recommender_amd" in f or "bench.py" in f]
        rows.append((dt, e.count, e.key, " <- ".join(st[:4])))
    tot = 0.0
    for dt, n, k, st in sorted(rows, reverse=True):
        tot += dt
        print(f"{dt:8.1f} us {n:3d}  {k:32s} {st}")
    print(f"total aten self device time {tot:.1f} us")


if __name__ == "__main__":
    main()
