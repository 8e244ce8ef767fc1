#!/usr/bin/env python3
"""Op-level device-time attribution (torch.profiler) for the RQ-VAE and decoder train steps."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402
from data.schemas import SeqBatch  # noqa: E402


def decoder():
    """Decoder train step (bench.measure_decoder config) with input shapes recorded."""
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    D = bench.DEC
    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    m = EncoderDecoderRetrievalModel(embedding_dim=D["E"], attn_dim=D["A"], dropout=D["dropout"], num_heads=D["H"],
                                     n_layers=D["layers"], num_embeddings=D["K"], sem_id_dim=D["sem_id_dim"],
                                     inference_verifier_fn=None, max_pos=D["max_items"] * D["sem_id_dim"]).to(dev).train()
    opt = torch.optim.AdamW(m.parameters(), lr=D["lr"], weight_decay=D["wd"], foreach=True)
    b = synthetic_tokenized_batch(D["B"], D["max_items"], D["sem_id_dim"], D["K"], 50, dev)

    def step():
        opt.zero_grad(set_to_none=True)
        m(b).loss.backward()
        opt.step()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(3):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=45,
                                                             max_name_column_width=40, max_shapes_column_width=70))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "decoder":
        return decoder()
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01, fused=True)
    x = bench.make_items(65536, 768, torch.Generator(device=dev).manual_seed(0), dev)

    def step():
        opt.zero_grad(set_to_none=False)
        out = model(SeqBatch(None, None, None, x, None, None), gumbel_t=0.2)
        out.loss.backward()
        opt.step()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(5):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=35, max_name_column_width=60))


if __name__ == "__main__":
    main()
