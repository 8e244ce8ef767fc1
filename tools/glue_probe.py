"""Which torch-side kernels (fills, adds, copies, reductions) one eager Amazon decoder train step launches,
grouped by Python call site (torch.profiler, stack depth 6). python tools/glue_probe.py"""
import os
import sys

import torch

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "rq-vae-recommender_amd"))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    from rqvae_hip import dp
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    cfg = bench.DEC
    torch.manual_seed(3)
    m = EncoderDecoderRetrievalModel(embedding_dim=cfg["E"], attn_dim=cfg["A"], dropout=cfg["dropout"],
                                     num_heads=cfg["H"], n_layers=cfg["layers"], num_embeddings=cfg["K"],
                                     sem_id_dim=cfg["sem_id_dim"], inference_verifier_fn=None,
                                     max_pos=cfg["max_items"] * cfg["sem_id_dim"]).to(dev).train()
    buckets = dp.GradBuckets(m.parameters(), overlap=False, flat_views=True)
    b = synthetic_tokenized_batch(cfg["B"], cfg["max_items"], cfg["sem_id_dim"], cfg["K"], 50, dev)
    for _ in range(3):
        buckets.zero_grad()
        m(b).loss.backward()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        buckets.zero_grad()
        m(b).loss.backward()
        torch.cuda.synchronize()
    import collections
    keys = ("fill", "add", "copy", "sum", "cat", "gather", "mul", "where", "zero", "index")
    agg = collections.defaultdict(lambda: [0, 0.0])
    for e in prof.events():
        if e.device_type.name != "CPU" or not e.name.startswith("aten::") or not any(k in e.name for k in keys):
            continue
        if e.cpu_parent is not None and e.cpu_parent.name.startswith("aten::") and any(
                k in e.cpu_parent.name for k in keys):
            continue   # counted at the outermost glue op
        chain, p = [], e.cpu_parent
        while p is not None and len(chain) < 4:
            chain.append(p.name[:70])
            p = p.cpu_parent
        a = agg[(e.name, " <- ".join(chain))]
        a[0] += 1
        a[1] += e.device_time_total
    for (name, chain), (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        if us > 0:
            print(f"{us:8.1f} us {n:3d}x {name:24s} <- {chain}")
    print(prof.key_averages().table(sort_by="device_time_total", row_limit=40, max_name_column_width=60))


if __name__ == "__main__":
    main()
