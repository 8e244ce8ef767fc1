"""Which framework (non-HIP-library) device kernels one eager decoder train step launches, and from where:
torch.profiler with Python stacks over one step; prints each aten-level op that launched a device kernel
with its innermost frames under rq-vae-recommender_amd/ (so the launch can be traced to the model code).

  python tools/torch_ops_probe.py [amazon|c4|rqvae]
"""
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
    from rqvae_hip import dp, gemm_tuning
    gemm_tuning.enable()
    dev = torch.device("cuda", 0)
    which = sys.argv[1] if len(sys.argv) > 1 else "c4"
    if which == "rqvae":   # the RQ-VAE bench step (bench.build_model, 65,536 items, both buckets)
        from data.schemas import SeqBatch
        model = bench.build_model(dev)
        buckets = dp.GradBuckets([list(model.decoder.parameters()) + list(model.layers.parameters()),
                                  list(model.encoder.parameters())], flat_views=True)
        xb = bench.make_items(65536, bench.CFG["input_dim"], torch.Generator(device=dev).manual_seed(1), dev)

        def step():
            buckets.zero_grad()
            model(SeqBatch(None, None, None, xb, None, None), gumbel_t=0.2).loss.backward()
            buckets.synchronize()
    else:
        cfg, B = (bench.DEC, bench.DEC["B"]) if which == "amazon" else (bench.DEC_DM, 8)
        torch.manual_seed(3)
        m = EncoderDecoderRetrievalModel(embedding_dim=cfg["E"], attn_dim=cfg["A"], dropout=cfg["dropout"],
                                         num_heads=cfg["H"], n_layers=cfg["layers"], num_embeddings=cfg["K"],
                                         sem_id_dim=cfg["sem_id_dim"], inference_verifier_fn=None,
                                         max_pos=cfg["max_items"] * cfg["sem_id_dim"]).to(dev).train()
        buckets = dp.GradBuckets(m.parameters(), overlap=True, flat_views=True)
        batch = synthetic_tokenized_batch(B, cfg["max_items"], cfg["sem_id_dim"], cfg["K"], 50, dev)

        def step():
            buckets.zero_grad()
            m(batch).loss.backward()
            buckets.synchronize()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    # device kernels that are not the library's, with the CPU op that launched them (in launch order), its
    # input shapes, the enclosing autograd node / Python frames when recorded
    evs = sorted(prof.events(), key=lambda e: e.time_range.start)
    for ev in evs:
        if ev.device_type != torch.autograd.DeviceType.CPU or not ev.name.startswith("aten::"):
            continue
        kids = list(getattr(ev, "kernels", []) or [])
        if not kids:
            continue
        par = ev.cpu_parent
        chain = []
        while par is not None and len(chain) < 3:
            chain.append(par.name[:50])
            par = par.cpu_parent
        frames = [f for f in (ev.stack or []) if "rq-vae-recommender_amd" in f or "/tools/" in f]
        print(f"{ev.name:26s} k={len(kids)} shapes={str(ev.input_shapes)[:70]} <- {' / '.join(chain)}")
        for f in frames[:3]:
            print("      ", f)


if __name__ == "__main__":
    main()
