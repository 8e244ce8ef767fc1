"""Device time of the decoder prologue's two launches (rq_dec_prologue_fwd: offsets / order kernel + gather
kernel) at the bench's Amazon and C4 batch shapes, as a hipGraph of 20 calls. One JSON line per config.

  RQVAE_HIP_LIB=... python tools/prologue_probe.py [tag]
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
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    from rqvae_hip import ops
    dev = torch.device("cuda", 0)
    tag = sys.argv[1] if len(sys.argv) > 1 else "default"
    for cfg, B in ((bench.DEC, bench.DEC["B"]), (bench.DEC_DM, 8)):
        torch.manual_seed(3)
        m = EncoderDecoderRetrievalModel(embedding_dim=cfg["E"], attn_dim=cfg["A"], dropout=cfg["dropout"],
                                         num_heads=cfg["H"], n_layers=1, num_embeddings=cfg["K"],
                                         sem_id_dim=cfg["sem_id_dim"], inference_verifier_fn=None,
                                         max_pos=cfg["max_items"] * cfg["sem_id_dim"]).to(dev)
        b = synthetic_tokenized_batch(B, cfg["max_items"], cfg["sem_id_dim"], cfg["K"], 50, dev)
        se, ue = m.sem_id_embedder, m.user_id_embedder
        alloc = m.context_rows(b, 256)

        def fn():
            with torch.no_grad():
                ops.decoder_prologue(ue.emb.weight, se.emb.weight, m.wpe.weight, m.tte.weight, m.bos_emb, b.user_ids,
                                     b.sem_ids, b.token_type_ids, b.seq_mask, b.sem_ids_fut, b.token_type_ids_fut,
                                     ue.num_buckets, se.num_embeddings, se.padding_idx, alloc)
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                fn()
        best = None
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) * 1000.0 / 20
            best = t if best is None else min(best, t)
        print(json.dumps({"tag": tag, "config": cfg["name"], "B": B, "N": b.sem_ids.shape[1], "us_per_call": round(best, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
