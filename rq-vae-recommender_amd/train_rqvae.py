"""RQ-VAE training entry point — drop-in for reference train_rqvae.py (same gin-configurable
`train(...)` signature, `python train_rqvae.py configs/rqvae_ml32m.gin`).

Differences from the reference loop (train_rqvae.py:24-250), all on the MI355X path:
  * one process per GPU (torchrun env) with rqvae_hip.dp instead of accelerate/DDP: each rank
    draws a DISJOINT shard of every global batch (`split_batches` semantics), k-means init runs
    on rank 0 and is broadcast, gradients are all-reduced over RCCL;
  * no per-step `.item()` host syncs — losses are read back every `log_every` iterations;
  * `cuda_graphs=True` (default; the reference compiles RqVae.forward with
    torch.compile(mode="reduce-overhead"), modules/rqvae.py:140): after one eager probe step the
    forward + backward (all micro-batches) is captured once and replayed every iteration
    (rqvae_hip.graph.GraphedSteps) — the batch indices are drawn eagerly and copied into the graph's
    static index buffer, the gradient exchange is captured inside the graph with RCCL, and the HIP
    AdamW step (host-side bias corrections) runs after the replay;
  * checkpoints are plain state dicts {"iter", "model", "model_config", "optimizer"} (loadable with
    weights_only=True); swanlab logging is replaced by printed JSON lines (out of scope);
  * the loop runs `iterations + 1` times like the reference (SURVEY A-4).
Data: `data.processed.ItemData` (seeded synthetic corpus unless `data_path` names a feature file).
"""
import contextlib
import json
import os
import time
import warnings
from enum import Enum

import numpy as np
import torch

from data.processed import ItemData, RecDataset
from data.schemas import SeqBatch
from modules.ginlite import gin
from modules.quantize import QuantizeForwardMode
from modules.rqvae import RqVae
from modules.tokenizer.semids import SemanticIdTokenizer
from modules.utils import parse_config
from rqvae_hip import dp, gemm_tuning
from rqvae_hip import optim as hip_optim
from rqvae_hip.graph import GraphedSteps


def sample_batch_indices(gen: torch.Generator, n_items: int, global_batch: int, device) -> torch.Tensor:
    """Item indices of one GLOBAL batch (every rank draws the same stream and keeps its own slice).
    The reference samples without replacement per epoch (BatchSampler(RandomSampler), train_rqvae.py:68);
    here i.i.d. draws on the device (no host round trip per step). Module-level so a test can
    substitute the reference's recorded batch order."""
    return torch.randint(0, n_items, (global_batch,), generator=gen, device=device)



# Last train() call: steady-state time per iteration (CUDA-synchronised once at the start and once at
# the end of the measured span, nothing inside it), the step mode and the captured graphs — for the
# bench's trainer line and the tests.
LAST_RUN = {}


@gin.configurable
def train(iterations=50000, batch_size=64, learning_rate=0.0001, weight_decay=0.01, dataset_folder="dataset/ml-1m",
          dataset=RecDataset.ML_1M, pretrained_rqvae_path=None, save_dir_root="out/", use_kmeans_init=True,
          split_batches=True, amp=False, swanlab_logging=False, do_eval=True, force_dataset_process=False,
          mixed_precision_type="fp16", gradient_accumulate_every=1, save_model_every=1000000, eval_every=50000,
          commitment_weight=0.25, vae_n_cat_feats=18, vae_input_dim=18, vae_embed_dim=16, vae_hidden_dims=[18, 18],
          vae_codebook_size=32, vae_codebook_normalize=False, vae_codebook_mode=QuantizeForwardMode.GUMBEL_SOFTMAX,
          vae_sim_vq=False, vae_n_layers=3, dataset_split="beauty", data_path=None, log_every=100, seed=0,
          cuda_graphs=True):
    if amp:
        # The reference's amp=True wraps the step in accelerate's fp16 autocast. This build does not enable
        # autocast: the flag is accepted and the step runs in fp32 — the RQ-VAE hot path's matmul-shaped ops are
        # HIP kernels at the 'high' split-bf16 precision (finer than fp16); any remaining torch ops (e.g. the
        # Gumbel-softmax composite) also stay fp32, where the reference would cast them to fp16. No
        # GradScaler is needed (gradients are fp32); mixed_precision_type is recorded for the log only.
        warnings.warn(f"amp=True ({mixed_precision_type}): accepted, but the step runs in fp32 with no autocast "
                      "(the RQ-VAE hot path is split-bf16 'high' MFMA GEMMs + fp32 kernels)", stacklevel=2)
    LAST_RUN.clear()
    rank, world, local_rank = dp.init_from_env()
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    gemm_tuning.enable()   # fastest measured library GEMM per shape (RQVAE_TUNABLE_GEMM=0: heuristic)

    train_ds = ItemData(root=dataset_folder, dataset=dataset, train_test_split="train" if do_eval else "all",
                        data_path=data_path, seed=seed)
    eval_ds = ItemData(root=dataset_folder, dataset=dataset, train_test_split="eval", data_path=data_path,
                       seed=seed) if do_eval else None
    index_ds = ItemData(root=dataset_folder, dataset=dataset, train_test_split="all", data_path=data_path,
                        seed=seed) if do_eval else train_ds
    items = train_ds.item_data[:, :vae_input_dim].to(device)      # resident corpus
    n_items = items.shape[0]
    global_batch = batch_size if split_batches else batch_size * world
    lo, hi = dp.shard_range(global_batch, rank, world)
    w_shard = dp.shard_weight(hi - lo, global_batch)

    torch.manual_seed(seed)
    model = RqVae(input_dim=vae_input_dim, embed_dim=vae_embed_dim, hidden_dims=vae_hidden_dims,
                  codebook_size=vae_codebook_size, codebook_kmeans_init=use_kmeans_init and pretrained_rqvae_path is None,
                  codebook_normalize=vae_codebook_normalize, codebook_sim_vq=vae_sim_vq, codebook_mode=vae_codebook_mode,
                  n_layers=vae_n_layers, n_cat_features=vae_n_cat_feats, commitment_weight=commitment_weight).to(device)
    opt = hip_optim.AdamW(model.parameters(), lr=learning_rate, weight_decay=weight_decay)
    start_iter = 0
    if pretrained_rqvae_path is not None:
        state = torch.load(pretrained_rqvae_path, map_location=device, weights_only=True)
        model.load_state_dict(state["model"])
        opt.load_state_dict(state["optimizer"])
        start_iter = state["iter"] + 1

    tokenizer = SemanticIdTokenizer(input_dim=vae_input_dim, hidden_dims=vae_hidden_dims, output_dim=vae_embed_dim,
                                    codebook_size=vae_codebook_size, n_layers=vae_n_layers, n_cat_feats=vae_n_cat_feats,
                                    rqvae_codebook_normalize=vae_codebook_normalize, rqvae_sim_vq=vae_sim_vq).to(device)
    tokenizer.rq_vae = model

    # k-means init on rank 0 over the first min(20000, N) items (reference :139-141), then broadcast
    if start_iter == 0 and use_kmeans_init and pretrained_rqvae_path is None:
        if rank == 0:
            with torch.no_grad():
                model(SeqBatch(None, None, None, items[: min(20000, n_items)], None, None), 0.2)
        for layer in model.layers:
            layer.kmeans_initted = True
    # grads become ready decoder -> codebooks -> encoder: the first bucket's all-reduce overlaps the
    # encoder backward
    buckets = dp.GradBuckets([list(model.decoder.parameters()) + list(model.layers.parameters()),
                              list(model.encoder.parameters())], flat_views=cuda_graphs)
    buckets.broadcast_params()
    acc = gradient_accumulate_every

    def step_body(idx):
        """Forward + backward of one iteration's micro-batches (idx: (acc, local batch) item indices);
        the per-step statistics as one device tensor."""
        total = 0.0
        for micro in range(acc):
            out = model(SeqBatch(None, None, None, items[idx[micro]], None, None), gumbel_t=0.2)
            # shard mean -> global-batch mean under unequal shards (dp.shard_weight), / micro-batches
            loss = out.loss * (w_shard / acc)
            with (contextlib.nullcontext() if micro == acc - 1 else buckets.no_sync()):
                loss.backward()
            total = total + out.loss.detach() / acc
        return torch.stack([total, out.reconstruction_loss.detach(), out.rqvae_loss.detach(),
                            out.p_unique_ids.detach()])

    graphed = GraphedSteps(step_body, lambda idx: 0, buckets, run_backward=False) if cuda_graphs else None
    gen = torch.Generator(device=device).manual_seed(seed + 17)   # same stream on every rank
    hist = []
    t0 = time.time()
    last_it = start_iter + iterations
    t_from = start_iter + min(5, iterations // 2)   # measured span: [t_from, last_it) (warm-up / captures before)
    t_mark = None
    for it in range(start_iter, start_iter + 1 + iterations):
        if it == t_from:
            torch.cuda.synchronize()
            t_mark = time.perf_counter()
        model.train()
        idx = torch.stack([sample_batch_indices(gen, n_items, global_batch, device)[lo:hi] for _ in range(acc)])
        if graphed is not None:
            stats = graphed(idx).clone()   # the graph's output buffer is rewritten by the next replay
        else:
            buckets.zero_grad()
            stats = step_body(idx)
        buckets.synchronize()
        opt.step()
        hist.append(stats)
        if it == last_it - 1 and t_mark is not None:
            torch.cuda.synchronize()
            LAST_RUN.update(iter_ms=(time.perf_counter() - t_mark) * 1e3 / max(1, last_it - t_from),
                            timed_iters=last_it - t_from, batch_per_rank=hi - lo, world=world,
                            step_mode="hipgraph" if graphed is not None else "eager",
                            graphs=len(graphed.graphs) if graphed is not None else 0,
                            eager_steps=graphed.eager_steps if graphed is not None else iterations + 1,
                            exchange="in-graph" if graphed is not None and graphed.in_graph else "hooks + synchronize")
        if it % log_every == 0 or it == start_iter + iterations:
            vals = torch.stack(hist).mean(0)
            hist = []
            if world > 1:
                # global-batch means, as the reference logs them (its ranks all see the whole batch, SURVEY A-5):
                # each rank's shard means weighted by its share; p_unique_ids stays this rank's shard value
                g = vals[:3] * ((hi - lo) / global_batch)
                torch.distributed.all_reduce(g)
                vals = torch.cat([g, vals[3:]])
            vals = vals.tolist()
        if rank == 0 and (it % log_every == 0 or it == start_iter + iterations):
            print(json.dumps({"iter": it, "loss": vals[0], "rl": vals[1], "vl": vals[2], "p_unique_ids": vals[3],
                              "elapsed_s": round(time.time() - t0, 2)}), flush=True)
        if do_eval and ((it + 1) % eval_every == 0 or it + 1 == iterations) and rank == 0:
            model.eval()
            with torch.no_grad():
                ev = [model(SeqBatch(None, None, None, eval_ds.item_data[a:a + 4096, :vae_input_dim].to(device), None,
                                     None), gumbel_t=0.2).loss for a in range(0, len(eval_ds), 4096)]
            print(json.dumps({"iter": it, "eval_total_loss": float(torch.stack(ev).mean())}), flush=True)
        if rank == 0 and ((it + 1) % save_model_every == 0 or it + 1 == iterations):
            os.makedirs(save_dir_root, exist_ok=True)
            config = {k: (v.name if isinstance(v, Enum) else v) for k, v in model.config.items()}   # tensors/plain only
            torch.save({"iter": it, "model": model.state_dict(), "model_config": config,
                        "optimizer": opt.state_dict()}, os.path.join(save_dir_root, f"checkpoint_{it}.pt"))
            tokenizer.reset()
            model.eval()
            corpus_ids = tokenizer.precompute_corpus_ids(index_ds)
            _, counts = torch.unique(corpus_ids[:, :-1], dim=0, return_counts=True)
            p = counts / corpus_ids.shape[0]
            stats = {"iter": it, "rqvae_entropy": float(-(p * torch.log(p)).sum()),
                     "max_id_duplicates": float(corpus_ids[:, -1].max() / corpus_ids.shape[0])}
            for cid in range(vae_n_layers):
                stats[f"codebook_usage_{cid}"] = len(torch.unique(corpus_ids[:, cid])) / vae_codebook_size
            print(json.dumps(stats), flush=True)
    return model


if __name__ == "__main__":
    parse_config()
    train()
