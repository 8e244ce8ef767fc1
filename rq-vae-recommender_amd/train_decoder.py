"""Decoder (generative retrieval) training entry point — drop-in for reference train_decoder.py
(same gin-configurable `train(...)` signature; `python train_decoder.py configs/decoder_amazon.gin`).

MI355X path: frozen RQ-VAE tokenizer (fused eval quantize + device dedup; corpus quantization
sharded over the ranks and all-gathered), decoder on the HIP jagged conversion + varlen attention
kernels, one process per GPU with rqvae_hip.dp: each global batch is split into TOKEN-BALANCED
shards (dp.balanced_partition over context lengths, so ranks finish together), each rank scales its
shard-mean loss by n_local * world / n_global (dp.shard_weight) so the averaged gradient is the
gradient of the reference's global-batch mean (model.py:261), bucketed RCCL all-reduce overlapped
with backward, no_sync() for all but the last micro-batch of an accumulation step.
`cuda_graphs=True` (default; the reference compiles the model's forward with
torch.compile(mode="reduce-overhead"), modules/model.py:247): forward + backward replayed from one
hipGraph per (input shapes, context row bucket) (rqvae_hip.graph.GraphedSteps, the gradient exchange
captured inside the graph with RCCL); the loss weight rides in as a device scalar. Gradient
accumulation (> 1 micro-batch) runs eagerly. A rank whose token-balanced shard is empty (a short last
batch with fewer sequences than ranks) runs no backward and joins the exchange from synchronize();
buckets launch in index order on every rank, so the collective sequence still matches.
The reference rejects non-AMAZON datasets and its ML-32M gin binds a non-existent parameter
(SURVEY A-8); this entry accepts every RecDataset (the ML-32M config still fails on
`train.attn_dropout`, exactly like gin). Checkpoints: plain state dicts with "scheduler".
"""
import contextlib
import json
import os
import time
import warnings

import torch

from data.processed import ItemData, RecDataset, SeqData, batch_loader
from data.utils import batch_to, cycle
from modules.ginlite import gin
from modules.model import EncoderDecoderRetrievalModel
from modules.scheduler.inv_sqrt import InverseSquareRootScheduler
from modules.tokenizer.semids import SemanticIdTokenizer
from modules.utils import parse_config
from rqvae_hip import dp, gemm_tuning
from rqvae_hip import optim as hip_optim
from rqvae_hip.graph import GraphedSteps
from ops.jagged import copy_row_counts, register_row_counts, row_counts


def token_balanced_shard(seq_mask: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    """Indices (host int64) of this rank's sequences of a host-side global batch: the batch is split
    into `world` bins of near-equal context-token counts (dp.balanced_partition over
    seq_mask.sum(1)); every rank computes the same partition, no communication."""
    if world == 1:
        return torch.arange(seq_mask.shape[0])
    costs = seq_mask.sum(1).tolist()
    return torch.tensor(dp.balanced_partition(costs, world)[rank], dtype=torch.int64)



class _Prefetch:
    """The host side of the next iterations on a background thread while the GPU runs the current one:
    the loader's next global batch (the reference's DataLoader, same order), this rank's token-balanced
    shard, its host-side context row counts and largest item id, pinned for a non-blocking copy. Yields
    (shard or None, counts, n_glob, ids_max) in loader order; `depth` batches ahead."""

    def __init__(self, loader, rank: int, world: int, sem_ids_dim: int, depth: int = 2):
        import queue
        import threading
        self.q = queue.Queue(maxsize=depth)
        self.stop = False
        pin = torch.cuda.is_available()

        def work():
            try:
                while not self.stop:
                    data = next(loader)
                    n_glob = data.seq_mask.shape[0]
                    if world > 1:
                        mine = token_balanced_shard(data.seq_mask, rank, world)
                        if len(mine) == 0:
                            self.q.put((None, None, n_glob, None))
                            continue
                        data = type(data)(*[v[mine] for v in data])
                    counts = (data.seq_mask.sum(1) * sem_ids_dim).tolist()
                    ids_max = int(max(int(data.ids.max()), int(data.ids_fut.max())))
                    if pin:
                        data = type(data)(*[v.pin_memory() if hasattr(v, "pin_memory") else v for v in data])
                    self.q.put((data, counts, n_glob, ids_max))
            except BaseException as e:   # surfaced on the consumer side
                self.q.put(e)
        self.thread = threading.Thread(target=work, daemon=True)
        self.thread.start()

    def next(self):
        item = self.q.get()
        if isinstance(item, BaseException):
            raise item
        return item

    def close(self):
        """Stop the feed thread and join it (it may be blocked on a full queue: keep draining)."""
        import queue
        self.stop = True
        while self.thread.is_alive():
            try:
                while True:
                    self.q.get_nowait()
            except queue.Empty:
                pass
            self.thread.join(timeout=0.01)


# Last train() call: steady-state time per iteration (CUDA-synchronised once at the start and once at
# the end of the measured span, nothing inside it), the step mode and the captured graphs — for the
# bench's trainer line and the tests.
LAST_RUN = {}


@gin.configurable
def train(iterations=500000, batch_size=64, learning_rate=0.001, weight_decay=0.01, dataset_folder="dataset/ml-1m",
          save_dir_root="out/", dataset=RecDataset.ML_1M, pretrained_rqvae_path=None, pretrained_decoder_path=None,
          split_batches=True, amp=False, swanlab_logging=False, force_dataset_process=False,
          mixed_precision_type="fp16", gradient_accumulate_every=1, save_model_every=1000000,
          partial_eval_every=1000, full_eval_every=10000, vae_input_dim=18, vae_embed_dim=16,
          vae_hidden_dims=[18, 18], vae_codebook_size=32, vae_codebook_normalize=False, vae_sim_vq=False,
          vae_n_cat_feats=18, vae_n_layers=3, decoder_embed_dim=64, dropout_p=0.1, attn_heads=8,
          attn_embed_dim=64, attn_layers=4, dataset_split="beauty", push_vae_to_hf=False,
          train_data_subsample=True, model_jagged_mode=True, vae_hf_model_name="edobotta/rqvae-amazon-beauty",
          data_path=None, log_every=100, seed=0, cuda_graphs=True):
    if amp:
        # The reference's amp=True wraps the step in accelerate's fp16 autocast. This build does not enable
        # autocast: the flag is accepted and the step runs in fp32 — the decoder hot path's matmul-shaped ops are
        # HIP kernels at the 'high' split-bf16 precision (finer than fp16); any remaining torch ops (e.g. the
        # Gumbel-softmax composite) also stay fp32, where the reference would cast them to fp16. No
        # GradScaler is needed (gradients are fp32); mixed_precision_type is recorded for the log only.
        warnings.warn(f"amp=True ({mixed_precision_type}): accepted, but the step runs in fp32 with no autocast "
                      "(the decoder hot path is split-bf16 'high' MFMA GEMMs + fp32 kernels)", stacklevel=2)
    if push_vae_to_hf:
        raise NotImplementedError("HF hub upload is out of scope (network)")
    LAST_RUN.clear()
    rank, world, local_rank = dp.init_from_env()
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    gemm_tuning.enable()   # fastest measured library GEMM per shape (RQVAE_TUNABLE_GEMM=0: heuristic)
    item_ds = ItemData(root=dataset_folder, dataset=dataset, data_path=data_path, seed=seed)
    # the decoder reads item ids only (the tokenizer maps them to cached semantic ids): no feature gather
    train_ds = SeqData(root=dataset_folder, dataset=dataset, is_train=True, subsample=train_data_subsample,
                       data_path=data_path, seed=seed, with_features=False)
    global_batch = batch_size if split_batches else batch_size * world
    g = torch.Generator().manual_seed(seed + 5)
    # the reference DataLoader's shuffled order, batches fetched whole (SeqData list indexing)
    loader = cycle(batch_loader(train_ds, global_batch, g))

    tokenizer = SemanticIdTokenizer(input_dim=vae_input_dim, hidden_dims=vae_hidden_dims, output_dim=vae_embed_dim,
                                    codebook_size=vae_codebook_size, n_layers=vae_n_layers, n_cat_feats=vae_n_cat_feats,
                                    rqvae_weights_path=pretrained_rqvae_path,
                                    rqvae_codebook_normalize=vae_codebook_normalize, rqvae_sim_vq=vae_sim_vq).to(device)
    corpus_ids = tokenizer.precompute_corpus_ids(item_ds, shard=True)   # not DDP-wrapped (reference A-7)
    top = int(corpus_ids.max())
    if top >= vae_codebook_size:   # would index past the SemIdEmbedder table on the device
        raise ValueError(f"semantic id / dedup value {top} >= codebook size {vae_codebook_size}: the tokenizer's "
                         "RQ-VAE maps too many items to one tuple (pass a trained pretrained_rqvae_path)")
    torch.manual_seed(seed)
    model = EncoderDecoderRetrievalModel(embedding_dim=decoder_embed_dim, attn_dim=attn_embed_dim, dropout=dropout_p,
                                         num_heads=attn_heads, n_layers=attn_layers, num_embeddings=vae_codebook_size,
                                         inference_verifier_fn=lambda x: tokenizer.exists_prefix(x),
                                         sem_id_dim=tokenizer.sem_ids_dim,
                                         max_pos=train_ds.max_seq_len * tokenizer.sem_ids_dim,
                                         jagged_mode=model_jagged_mode).to(device)
    opt = hip_optim.AdamW(model.parameters(), lr=learning_rate, weight_decay=weight_decay)
    sched = InverseSquareRootScheduler(optimizer=opt, warmup_steps=10000)
    start_iter = 0
    if pretrained_decoder_path is not None:
        ck = torch.load(pretrained_decoder_path, map_location=device, weights_only=True)
        model.load_state_dict(ck["model"])
        opt.load_state_dict(ck["optimizer"])
        if "scheduler" in ck:
            sched.load_state_dict(ck["scheduler"])
        start_iter = ck["iter"] + 1
    use_graphs = cuda_graphs and gradient_accumulate_every == 1
    buckets = dp.GradBuckets(model.parameters(), flat_views=use_graphs)
    buckets.broadcast_params()
    bucket = gemm_tuning.ROW_BUCKET if gemm_tuning.is_enabled() else None

    def graph_body(inp):
        # the raw (device) SeqBatch goes into the graph and is tokenized there: the tokenizer's cache lookups,
        # mask expansion and token types are ~10 small launches whose host cost (~2 ms per iteration) the
        # replay removes. The caller checked on the host that every id hits the cache (ids_max); the raw
        # mask carries the TOKENIZED row counts (register_row_counts in the loop), handed to the tokenized
        # mask so the jagged conversions size their buffers without a device read.
        data, w = inp
        tok = tokenizer(data, ids_max=0)
        copy_row_counts(tok.seq_mask, data.seq_mask)
        out = model(tok)
        (out.loss * w).backward()
        return out.loss.detach()

    def graph_key(inp):
        c = row_counts(inp[0].seq_mask)   # (sum, min, max, rows) of the tokenized context counts
        total = c[0] + c[3]               # + the user token per sequence (model.context_rows)
        return total if not bucket else (total + bucket - 1) // bucket * bucket

    graphed = GraphedSteps(graph_body, graph_key, buckets, run_backward=False,
                           prepare=lambda static, inp: copy_row_counts(static[0].seq_mask, inp[0].seq_mask)
                           ) if use_graphs else None
    feed = _Prefetch(loader, rank, world, tokenizer.sem_ids_dim)
    try:
        _train_loop(feed, model, tokenizer, graphed, buckets, opt, sched, device, rank, world, start_iter, iterations,
                    gradient_accumulate_every, log_every, save_model_every, save_dir_root)
    finally:
        feed.close()
    return model


_PHASES = ("feed_wait", "tokenize", "step", "exchange", "optimizer", "log_save")


def _train_loop(feed, model, tokenizer, graphed, buckets, opt, sched, device, rank, world, start_iter, iterations,
                gradient_accumulate_every, log_every, save_model_every, save_dir_root):
    """The reference's loop (train_decoder.py:180-204) over the prefetched batches. Host time per phase
    is accumulated over the steady span (LAST_RUN["host_ms_per_iter"]): the loop must stay ahead of the
    GPU, so these are the numbers to read when the trainer is slower than its bench step."""
    w_dev = {}
    t0, hist = time.time(), []
    t_from = start_iter + min(5, (iterations - start_iter) // 2)   # measured span: [t_from, iterations)
    t_mark, toks = None, 0
    # steady state: the iterations after the last graph capture (a new row bucket's capture costs two
    # eager warm-up passes + the capture; a long run amortises the few buckets a dataset has)
    s_mark, s_from, s_toks = None, None, 0
    phase = dict.fromkeys(_PHASES, 0.0)
    clock = time.perf_counter
    for it in range(start_iter, iterations):
        if it == t_from:
            torch.cuda.synchronize()
            t_mark = clock()
        if t_mark is not None and s_mark is None:
            torch.cuda.synchronize()
            s_mark, s_from, s_toks = clock(), it, 0
            phase = dict.fromkeys(_PHASES, 0.0)
        n_graphs = len(graphed.graphs) if graphed is not None else 0
        model.train()
        if graphed is None:
            buckets.zero_grad()
        total = None
        for micro in range(gradient_accumulate_every):
            # the loader's next global batch, this rank's token-balanced shard (n_glob: the loader's last
            # batch of an epoch may be short) and its host-side context row counts — no device sync for
            # the jagged total, and a captured step is keyed by its row bucket — prepared on the feed thread
            c0 = clock()
            data, counts, n_glob, ids_max = feed.next()
            c1 = clock()
            phase["feed_wait"] += c1 - c0
            if data is None:   # fewer sequences than ranks: zero gradient, exchange in synchronize()
                if graphed is not None:
                    buckets.zero_grad()
                continue
            if t_mark is not None:
                toks += sum(counts) + len(counts)   # context tokens (+ the user token per sequence)
                s_toks += sum(counts) + len(counts)
            # this rank's shard mean -> share of the GLOBAL-batch mean (unequal, token-balanced shards)
            w = dp.shard_weight(len(counts), n_glob) / gradient_accumulate_every
            data = batch_to(data, device)
            if graphed is not None and tokenizer.cache_hit(ids_max):   # tokenized inside the replayed graph
                register_row_counts(data.seq_mask, counts)
                c2 = clock()
                phase["tokenize"] += c2 - c1
                wt = w_dev.get(w)
                if wt is None:   # a few distinct weights over a run: one device scalar each, no per-step copy
                    wt = w_dev[w] = torch.tensor(w, device=device)
                loss = graphed((data, wt)).clone()   # the graph's output buffer is overwritten by the next replay
            else:
                if graphed is not None:   # an id past the cache (never with a precomputed corpus): eager step
                    buckets.zero_grad()
                tok = tokenizer(data, ids_max=ids_max)
                register_row_counts(tok.seq_mask, counts)
                c2 = clock()
                phase["tokenize"] += c2 - c1
                out = model(tok)
                last = micro == gradient_accumulate_every - 1
                with (contextlib.nullcontext() if last else buckets.no_sync()):
                    (out.loss * w).backward()
                loss = out.loss.detach() / gradient_accumulate_every
            if world > 1:   # the global-batch mean is the shard means weighted by their shares (logged below)
                loss = loss * (len(counts) / n_glob)
            total = loss if total is None else total + loss
            phase["step"] += clock() - c2
        c3 = clock()
        buckets.synchronize()
        c4 = clock()
        opt.step()
        sched.step()
        c5 = clock()
        phase["exchange"] += c4 - c3
        phase["optimizer"] += c5 - c4
        hist.append(total if total is not None else torch.zeros((), device=device))
        if graphed is not None and len(graphed.graphs) != n_graphs:
            s_mark = None   # this iteration captured: the steady span restarts after it
        if it == iterations - 1 and t_mark is not None:
            torch.cuda.synchronize()
            t_end = clock()
            dt = t_end - t_mark
            steady = {}
            if s_mark is not None and iterations - s_from >= 3:
                ds = t_end - s_mark
                n_s = iterations - s_from
                steady = dict(steady_iter_ms=ds * 1e3 / n_s, steady_iters=n_s,
                              steady_ctx_tokens_per_s_rank=s_toks / ds, ctx_tokens_per_iter_rank=s_toks / n_s,
                              host_ms_per_iter={k: round(v * 1e3 / n_s, 4) for k, v in phase.items()})
            LAST_RUN.update(iter_ms=dt * 1e3 / max(1, iterations - t_from), timed_iters=iterations - t_from,
                            ctx_tokens_per_s_rank=toks / dt, world=world, **steady,
                            step_mode="hipgraph" if graphed is not None else "eager",
                            graphs=len(graphed.graphs) if graphed is not None else 0,
                            eager_steps=graphed.eager_steps if graphed is not None else iterations - start_iter,
                            exchange="in-graph" if graphed is not None and graphed.in_graph else "hooks + synchronize")
        c6 = clock()
        if it % log_every == 0 or it + 1 == iterations:
            mean = torch.stack(hist).mean()
            hist = []
            if world > 1:   # global-batch loss, as the reference logs it (its ranks all see the whole batch, A-5)
                torch.distributed.all_reduce(mean)
            if rank == 0:
                print(json.dumps({"iter": it, "loss": float(mean), "lr": opt.param_groups[0]["lr"],
                                  "elapsed_s": round(time.time() - t0, 2)}), flush=True)
        if rank == 0 and ((it + 1) % save_model_every == 0 or it + 1 == iterations):
            os.makedirs(save_dir_root, exist_ok=True)
            torch.save({"iter": it, "model": model.state_dict(), "optimizer": opt.state_dict(),
                        "scheduler": sched.state_dict()}, os.path.join(save_dir_root, f"checkpoint_{it}.pt"))
        phase["log_save"] += clock() - c6



if __name__ == "__main__":
    parse_config()
    train()
