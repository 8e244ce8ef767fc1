"""Host time of one captured decoder train step's replay (GraphedSteps, the bench's Amazon config) vs its
GPU time, and the node types of the captured graph (hipGraphDebugDotPrint through torch's debug dump):
which nodes make hipGraphLaunch wait for the graph to run?"""
import collections
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    import bench
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    from ops.jagged import copy_row_counts
    from rqvae_hip import dp, gemm_tuning
    from rqvae_hip.graph import GraphedSteps
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    gemm_tuning.enable()
    base = torch.cuda.CUDAGraph

    class DbgGraph(base):   # debug mode on every captured graph (node dump)
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            self.enable_debug_mode()
    torch.cuda.CUDAGraph = DbgGraph
    cfg = bench.DEC
    torch.manual_seed(0)
    m = EncoderDecoderRetrievalModel(embedding_dim=cfg["E"], attn_dim=cfg["A"], dropout=cfg["dropout"],
                                     num_heads=cfg["H"], n_layers=cfg["layers"], num_embeddings=cfg["K"],
                                     sem_id_dim=cfg["sem_id_dim"], inference_verifier_fn=None,
                                     max_pos=cfg["max_items"] * cfg["sem_id_dim"]).to(dev)
    buckets = dp.GradBuckets(m.parameters(), flat_views=True)
    opt = bench.make_adamw(m.parameters(), cfg["lr"], cfg["wd"])
    bucket = gemm_tuning.ROW_BUCKET if gemm_tuning.is_enabled() else None
    gs = GraphedSteps(lambda b: m(b).loss, lambda b: m.context_rows(b, bucket), buckets,
                      prepare=lambda static, b: copy_row_counts(static.seq_mask, b.seq_mask))
    batch = synthetic_tokenized_batch(cfg["B"], cfg["max_items"], cfg["sem_id_dim"], cfg["K"], 3, dev)
    for _ in range(2):
        gs(batch)
        buckets.synchronize()
        opt.step()
    torch.cuda.synchronize()
    res = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        gs(batch)
        t1 = time.perf_counter()
        e1.record()
        buckets.synchronize()
        opt.step()
        torch.cuda.synchronize()
        res.append({"call_host_ms": round((t1 - t0) * 1e3, 3), "gpu_ms": round(e0.elapsed_time(e1), 3)})
    print(json.dumps({"replays": res}), flush=True)
    # node types of the captured graph
    g = next(iter(gs.graphs.values()))[0]
    path = "/tmp/step_graph.dot"
    try:
        g.debug_dump(path)
        txt = open(path).read()
        kinds = collections.Counter(re.findall(r'label="\{?\s*([A-Za-z_]+)', txt))
        names = collections.Counter(re.findall(r'\\n([A-Za-z_:<>0-9, ]{3,60})', txt))
        print(json.dumps({"node_kinds": kinds.most_common(20), "dot_bytes": len(txt)}), flush=True)
        lines = [l for l in txt.splitlines() if "label" in l]
        print("\n".join(l[:300] for l in lines[:12]))
        kinds2 = collections.Counter()
        for l in lines:
            m_ = re.search(r'label="([^"\\|{]{1,40})', l)
            if m_:
                kinds2[m_.group(1).strip()] += 1
        print(json.dumps({"label_heads": kinds2.most_common(30)}))
    except Exception as e:   # debug mode must be enabled before capture on some builds
        print(json.dumps({"debug_dump_error": repr(e)[:300]}))


if __name__ == "__main__":
    main()
