"""The deferred partial reductions of one decoder train step (ops.flush_reductions -> rq_reduce_partials):
entries (n, S, layout), slab bytes, and the launch's time and effective bandwidth (eager step, HIP events
around the flush). One JSON line per flush.

  python tools/defer_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    import bench
    from rqvae_hip import dp, gemm_tuning, ops
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    gemm_tuning.enable()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    orig = ops.flush_reductions
    rec = []

    def flush():
        pend = list(ops._DEFER["pending"])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        orig()
        e1.record()
        torch.cuda.synchronize()
        if pend:
            ents = [(int(e[2]), int(e[3]), int(e[4])) for e in pend]
            rd = sum(4 * n * S for n, S, _ in ents)
            rec.append({"entries": len(ents), "slab_MB": round(rd / 1e6, 2), "out_M": round(sum(n for n, _, _ in ents) / 1e6, 3),
                        "us": round(e0.elapsed_time(e1) * 1e3, 1),
                        "TBps": round((rd + 8 * sum(n for n, _, _ in ents)) / (e0.elapsed_time(e1) * 1e-3) / 1e12, 2),
                        "top": sorted(ents, key=lambda x: -x[0] * x[1])[:12]})
    ops.flush_reductions = flush
    for cfg, B in ((bench.DEC, None), (bench.DEC_DM, 8)):
        B = B or cfg["B"]
        torch.manual_seed(3)
        m = EncoderDecoderRetrievalModel(embedding_dim=cfg["E"], attn_dim=cfg["A"], dropout=cfg["dropout"],
                                         num_heads=cfg["H"], n_layers=cfg["layers"], num_embeddings=cfg["K"],
                                         sem_id_dim=cfg["sem_id_dim"], inference_verifier_fn=None,
                                         max_pos=cfg["max_items"] * cfg["sem_id_dim"]).to(dev).train()
        buckets = dp.GradBuckets(m.parameters(), overlap=True, flat_views=True)
        b = synthetic_tokenized_batch(B, cfg["max_items"], cfg["sem_id_dim"], cfg["K"], 50, dev)
        for it in range(3):
            rec.clear()
            buckets.zero_grad()
            m(b).loss.backward()
            buckets.synchronize()
            torch.cuda.synchronize()
        for r in rec:
            print(json.dumps(dict(config=cfg["name"], B=B, **r)), flush=True)
        del m, buckets


if __name__ == "__main__":
    main()
