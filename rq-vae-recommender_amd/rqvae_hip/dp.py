"""Data-parallel engine: one process per GPU, RCCL (torch "nccl" backend on ROCm) over xGMI.

Replaces the reference's implicit DDP via HF accelerate (train_rqvae.py:60-63,115-117,153;
train_decoder.py:171-173,196) and fixes its defects:
  * every rank draws a DISJOINT shard of each global batch (`shard_range`), instead of all
    ranks iterating the same un-sharded generator;
  * parameters (incl. k-means-initialised codebooks) are broadcast from rank 0 once, after init;
  * gradients live in ONE flat fp32 buffer per dtype ("gradient-as-bucket-view"), so the
    exchange is a few large all-reduces with no pack/unpack copies;
  * parameters that receive no gradient on ANY rank in the first step (the decoder's `tte_fut`
    and `ffn_norm`, SURVEY A-7) are found once (one small all-reduce of a usage mask at the first
    `synchronize`) and from then on keep `grad = None` after every exchange, exactly as with one
    process (AdamW skips them; 1-rank and N-rank checkpoints stay identical);
  * buckets are all-reduced asynchronously as soon as backward has produced all their grads
    (post-accumulate-grad hooks), overlapping the RCCL ring with the rest of backward; the
    optimizer step waits on the handles. Average = sum / world. Buckets are LAUNCHED IN INDEX
    ORDER on every rank (a ready bucket waits for its predecessors), so the collective sequence is
    the same on every rank whatever order backward finishes them in — including a rank whose shard
    is empty and that launches everything from `synchronize()`;
  * a parameter may receive its gradient once per backward (as with DDP): a second contribution —
    a HIP op accumulating into the flat bucket after the bucket's exchange may have started — raises;
  * inside a captured hipGraph (rqvae_hip.graph.GraphedSteps, RCCL backend) the hooks' all-reduces
    and the final wait / average are captured too (`finish()`), so the exchange of the replayed
    step overlaps its backward; the caller's `synchronize()` after such a replay is a no-op;
  * gradient accumulation: backward passes run inside `no_sync()` except the last micro-batch
    (like DDP), so the exchange starts once, on the accumulated gradients.
Loss normalisation for unequal shards (`shard_range` with a remainder, token-balanced decoder
shards from `balanced_partition`): each rank scales its shard-mean loss by
`shard_weight(n_local, n_global)` = n_local * world / n_global, so the averaged gradient is the
gradient of the GLOBAL-batch mean (the reference's mean over B, model.py:261, rqvae.py:150).
Bucket size: 32 MiB by default — large enough that each ring step is link-bandwidth-bound on
the 7 point-to-point xGMI links, small enough to start overlapping early in backward.
Works with the gloo backend on CPU for tests.
"""
import contextlib
import os
from typing import Iterable, List, Optional, Sequence

import torch
import torch.distributed as dist


def world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


_FR_ENV = ("TORCH_FR_BUFFER_SIZE", "TORCH_NCCL_TRACE_BUFFER_SIZE")


def watchdog_record_enabled() -> bool:
    """True when torch's flight recorder records RCCL collectives (read once by torch, when the first
    process group is created): GraphedSteps then checks that the watchdog has retired every eager
    collective before it captures the exchange (graph.watchdog_retired)."""
    for k in _FR_ENV:
        try:
            if int(os.environ.get(k, "0") or 0) > 0:
                return True
        except ValueError:
            pass
    return False


def enable_watchdog_record(entries: int = 256):
    """Turn on torch's flight recorder (a ring of the last `entries` collectives and their state)
    unless the environment already configures it. Must run before the first RCCL process group is
    created; init_from_env does."""
    if not watchdog_record_enabled():
        os.environ["TORCH_FR_BUFFER_SIZE"] = str(int(entries))


def init_from_env(backend: Optional[str] = None):
    """Initialise torch.distributed from RANK / WORLD_SIZE / MASTER_* (torchrun env). Returns
    (rank, world, local_rank). No-op for WORLD_SIZE=1.

    Rehearsal switches (one-GPU box): RQVAE_DIST_BACKEND=gloo selects the backend, and
    RQVAE_SHARE_DEVICE=1 maps every rank to device 0 (RCCL refuses two ranks on one GPU, gloo
    moves the CUDA tensors through the host), so the multi-rank code paths run end to end."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rk = int(os.environ.get("RANK", "0"))
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("RQVAE_SHARE_DEVICE", "0") == "1":
        lr = 0
    if ws > 1 and not dist.is_initialized():
        backend = backend or os.environ.get("RQVAE_DIST_BACKEND")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            enable_watchdog_record()
            torch.cuda.set_device(lr)
            dist.init_process_group(backend, device_id=torch.device("cuda", lr))
        else:
            dist.init_process_group(backend)
    return rk, ws, lr


def shard_range(global_batch: int, rank_: int, world_: int):
    """Contiguous [start, stop) slice of a global batch owned by `rank_` (split_batches=True
    semantics: the global batch is split, per-rank batch = global / world; remainder rows go to
    the first ranks)."""
    base, rem = divmod(global_batch, world_)
    start = rank_ * base + min(rank_, rem)
    return start, start + base + (1 if rank_ < rem else 0)


def shard_weight(n_local: int, n_global: int) -> float:
    """Factor on a rank's shard-MEAN loss that makes the world-averaged gradient equal the gradient
    of the global-batch mean: n_local * world / n_global (1.0 for equal shards)."""
    return float(n_local) * world() / float(n_global) if n_global > 0 else 0.0


def balanced_partition(costs: Sequence[int], world_: int) -> List[List[int]]:
    """Split items with the given costs (e.g. context tokens per sequence) into `world_` bins of
    near-equal total cost (longest-first greedy: each item goes to the currently lightest bin; ties
    to the lower rank). Deterministic, host-only; every rank computes the same partition. Bins keep
    their items in ascending index order. Used for token-balanced decoder shards."""
    order = sorted(range(len(costs)), key=lambda i: (-int(costs[i]), i))
    load = [0] * world_
    bins: List[List[int]] = [[] for _ in range(world_)]
    for i in order:
        r = min(range(world_), key=lambda k: (load[k], k))
        bins[r].append(i)
        load[r] += int(costs[i])
    return [sorted(b) for b in bins]


def all_gather_rows(local: torch.Tensor, n_total: int) -> torch.Tensor:
    """Concatenate the per-rank row blocks of a tensor sharded by `shard_range(n_total, r, world)`
    (rank order) on every rank: one all_gather of equal-size padded blocks, no host sync beyond
    the collective."""
    ws = world()
    if ws == 1:
        return local
    spans = [shard_range(n_total, r, ws) for r in range(ws)]
    width = max(b - a for a, b in spans)
    pad = torch.zeros((width,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    parts = [torch.empty_like(pad) for _ in range(ws)]
    dist.all_gather(parts, pad)
    return torch.cat([p[:b - a] for p, (a, b) in zip(parts, spans)], 0)


# Parameters whose weight gradient a HIP op may add straight into the flat bucket (C += g^T x in the
# GEMM's slab reduction) instead of returning it to autograd, which would run an AccumulateGrad add
# kernel per parameter per step into the flat view. id(param) -> (flat view, hook).
_DIRECT = {}
_OWNER = {}   # id(param) -> (GradBuckets, bucket index)


def direct_grad(p) -> Optional[torch.Tensor]:
    """The flat-bucket view p's gradient may be accumulated into in place (GradBuckets with flat
    buffers, p.grad currently that view), else None. The caller adds its gradient into the view,
    returns None to autograd for p and calls direct_grad_done(p)."""
    e = _DIRECT.get(id(p))
    if e is None or torch.is_grad_enabled():
        return None
    g = p.grad
    if g is None or g.data_ptr() != e[0].data_ptr():
        return None
    owner = _OWNER.get(id(p))
    if owner is not None:
        owner[0]._check_first(owner[1], p)   # a second contribution would race the bucket's exchange
    return e[0]


def defer_ok(p) -> bool:
    """True when p's owner GradBuckets batches the split-K / RMSNorm weight-gradient reductions into its
    flat views (ops.flush_reductions at its flush points) instead of reducing per op."""
    owner = _OWNER.get(id(p))
    return owner is not None and owner[0].defer


def direct_grad_done(p) -> None:
    """The caller has added its contribution into p's flat-bucket view. Nothing to do: the op returns
    None for p to autograd, and the engine still runs p's AccumulateGrad node (with an undefined
    gradient) once ALL of p's contributions of this backward are in — its post-accumulate hook is the
    single point where GradBuckets marks p ready (firing here as well would count p twice, and could
    start the bucket's exchange before a second op has added its share)."""
    return None


class GradBuckets:
    """Flat gradient buffers + bucketed async all-reduce for a module's parameters."""

    def __init__(self, params, bucket_bytes: int = 32 << 20, average: bool = True, overlap: bool = True,
                 flat_views: bool = False, force_exchange: bool = False, defer_reductions: bool = True):
        """`params`: an iterable of parameters (buckets follow reverse registration order, ~ the order
        grads become ready), or a list of parameter groups given in the order their grads become
        ready (each group gets its own buckets, so an early group's all-reduce overlaps the rest of
        the backward — e.g. [decoder + codebooks, encoder] for the RQ-VAE).
        `overlap=False`: the exchange starts in `synchronize()` only (hooks just record which
        parameters took part).
        `flat_views=True`: gradients live in the flat buffers even with one process, so they sit
        at fixed addresses that several captured graphs can share.
        `overlap=True` is also right for captured steps: GraphedSteps suspends the hooks where the
        backend cannot be captured (gloo) and exchanges after the replay instead.
        `defer_reductions=True`: weight-gradient partial reductions into the flat views (split-K slabs,
        RMSNorm partials) are batched (ops.flush_reductions) and run before a bucket's exchange and in
        finish / synchronize / zero_grad — so gradients are complete only after synchronize()."""
        params = list(params)
        grouped = bool(params) and isinstance(params[0], (list, tuple))
        groups = [list(g) for g in params] if grouped else [list(reversed(params))]
        seen = set()
        groups = [[p for p in g if p.requires_grad and not (id(p) in seen or seen.add(id(p)))] for g in groups]
        self.params: List[torch.nn.Parameter] = [p for g in groups for p in g]
        self.average = average
        # `force_exchange` (tests): run the collectives even with one process (a world-1 RCCL group
        # exercises the captured exchange on a one-GPU box)
        self.exchange = world() > 1 or force_exchange
        # single process without flat_views: no flat views (AccumulateGrad steals, no add_)
        self.active = self.exchange or flat_views
        self.overlap = overlap and self.exchange
        self.defer = bool(defer_reductions) and self.active
        self.buckets = []
        self._pending = {}
        self._next = 0             # buckets [0, _next) are launched this pass (launch order = index order)
        self._sync = True          # False inside no_sync(): hooks record usage but launch nothing
        self._unused = None        # ids of params unused on every rank (decided at the first sync)
        self._graph_done = False   # a captured replay already ran this step's exchange
        for g in (groups if self.active else []):
            by_dtype = {}
            for p in g:
                by_dtype.setdefault((p.dtype, p.device), []).append(p)
            for (dt, dev), ps in by_dtype.items():
                cur, cur_bytes = [], 0
                for p in ps:
                    cur.append(p)
                    cur_bytes += p.numel() * p.element_size()
                    if cur_bytes >= bucket_bytes:
                        self._make_bucket(cur, dt, dev)
                        cur, cur_bytes = [], 0
                if cur:
                    self._make_bucket(cur, dt, dev)
        for bi, b in enumerate(self.buckets):   # usage tracking (+ overlapped launches when overlap)
            for p, v in zip(b["params"], b["views"]):
                hook = self._make_hook(bi)
                p.register_post_accumulate_grad_hook(hook)
                _DIRECT[id(p)] = (v, hook)
                _OWNER[id(p)] = (self, bi)

    def _make_bucket(self, ps, dt, dev):
        n = sum(p.numel() for p in ps)
        flat = torch.zeros(n, dtype=dt, device=dev)
        off = 0
        views = []
        for p in ps:
            v = flat[off:off + p.numel()].view_as(p)
            p.grad = v          # grads accumulate in place into the flat buffer
            views.append(v)
            off += p.numel()
        self.buckets.append(dict(params=ps, flat=flat, views=views, used=set(), fired=set(), expect=len(ps),
                                 ready=False))

    def _make_hook(self, bi):
        def hook(p):
            b = self.buckets[bi]
            if self._unused is not None and id(p) in self._unused:
                raise RuntimeError("GradBuckets: a parameter that received no gradient on any rank in the first "
                                   "step got one later; its gradient would not be exchanged (build the buckets "
                                   "without it, or make it take part in the first step)")
            b["used"].add(id(p))
            if not self._sync:
                return
            # count this pass's grads only: after no_sync micro-batches `used` is already full, and a
            # launch on the first hook of the last micro-batch would reduce partial gradients
            self._check_first(bi, p)
            b["fired"].add(id(p))
            if self.overlap and len(b["fired"]) == b["expect"]:
                b["ready"] = True
                self._launch_ready()
        return hook

    def _check_first(self, bi, p):
        """With the exchange started from the hooks (overlap), a bucket may be all-reducing as soon as
        its last parameter has fired: a second contribution to a fired parameter would race it."""
        if self.overlap and self._sync and id(p) in self.buckets[bi]["fired"]:
            raise RuntimeError("GradBuckets: a parameter received a second gradient contribution in one backward "
                               "(used by two ops that accumulate into its flat bucket); its bucket's exchange may "
                               "already be running. Use each parameter once per backward, or run the extra "
                               "backward passes inside no_sync().")

    def _launch_ready(self):
        """Launch, in index order, every bucket whose predecessors are all launched and that is ready
        (all its used parameters' grads produced, or nothing in it is used on any rank)."""
        while self._next < len(self.buckets):
            b = self.buckets[self._next]
            if not (b["ready"] or b["expect"] == 0):
                return
            self._launch(self._next)
            self._next += 1

    @contextlib.contextmanager
    def no_sync(self):
        """Backward passes inside accumulate into the flat buffers without starting the exchange
        (all micro-batches but the last of a gradient-accumulation step)."""
        prev, self._sync = self._sync, False
        try:
            yield
        finally:
            self._sync = prev
            for b in self.buckets:
                b["fired"].clear()
                b["ready"] = False

    def _launch(self, bi):
        if bi in self._pending:
            return
        b = self.buckets[bi]
        if b["expect"] == 0:   # every parameter of the bucket is unused on every rank
            return
        from . import ops
        ops.flush_reductions()    # every deferred reduction into the flat views lands before the exchange
        self._pending[bi] = dist.all_reduce(b["flat"], op=dist.ReduceOp.SUM, async_op=True)

    def zero_grad(self):
        if not self.active:
            for p in self.params:
                p.grad = None
            return
        if self.defer:   # a step left unsynchronised: its deferred reductions must not land after the zeroing
            from . import ops
            ops.flush_reductions()
        unused = self._unused or ()
        flats = [b["flat"] for b in self.buckets]
        if len(flats) > 1 and all(f.is_cuda for f in flats):
            torch._foreach_zero_(flats)   # every bucket in one multi-tensor launch
        else:
            for f in flats:
                f.zero_()
        for b in self.buckets:
            b["used"].clear()
            b["fired"].clear()
            b["ready"] = False
            for p, v in zip(b["params"], b["views"]):
                if id(p) in unused:
                    continue
                if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                    p.grad = v
        self._pending = {}
        self._next = 0

    def synchronize(self):
        """Finish the exchange (launch buckets whose hooks did not all fire — params unused this
        step contribute zeros — then wait) and average."""
        if not self.active:
            return
        if self._graph_done:   # the captured replay ran the exchange (GraphedSteps, in-graph mode)
            self._graph_done = False
        else:
            self.finish()
        if self._unused is None:
            self._find_unused()
        for p in self._unused_params:
            p.grad = None

    def finish(self):
        """Launch what is left (in index order) and wait for every bucket, then average. Pure stream
        work (no host sync): GraphedSteps captures it at the end of the replayed backward."""
        from . import ops
        ops.flush_reductions()
        if self.exchange:
            while self._next < len(self.buckets):
                self._launch(self._next)
                self._next += 1
            ws = world()
            for bi, h in sorted(self._pending.items()):
                h.wait()
                if self.average and ws > 1:
                    self.buckets[bi]["flat"].div_(ws)
        self._pending = {}
        self._next = 0

    def mark_graph_exchanged(self):
        """The step's exchange ran inside a replayed graph: the next synchronize() only finalises."""
        self._graph_done = True

    @contextlib.contextmanager
    def suspended(self):
        """Hooks record usage but launch nothing (graph warm-up passes: every rank must run exactly
        one exchange per step, so warm-ups of a newly captured key must not communicate)."""
        prev, self._sync = self._sync, False
        try:
            yield
        finally:
            self._sync = prev
            for b in self.buckets:
                b["fired"].clear()
                b["ready"] = False
            self._pending = {}
            self._next = 0

    def _find_unused(self):
        """Once, at the first exchange: parameters whose grad hook fired on no rank. They are
        structurally unused (the decoder's tte_fut / ffn_norm): from now on their grad stays None,
        and a bucket launches as soon as its USED parameters are ready."""
        flags = [float(id(p) in b["used"]) for b in self.buckets for p in b["params"]]
        if world() > 1:
            dev = self.buckets[0]["flat"].device if self.buckets else torch.device("cpu")
            used = torch.tensor(flags, device=dev)
            dist.all_reduce(used, op=dist.ReduceOp.MAX)
            flags = used.cpu().tolist()
        self._unused, self._unused_params, k = set(), [], 0
        for b in self.buckets:
            for p in b["params"]:
                if flags[k] == 0.0:
                    self._unused.add(id(p))
                    self._unused_params.append(p)
                k += 1
            b["expect"] = sum(1 for p in b["params"] if id(p) not in self._unused)

    def broadcast_params(self, src: int = 0):
        if world() == 1:
            return
        with torch.no_grad():
            for p in self.params:
                dist.broadcast(p.data, src=src)


def broadcast_module(module: torch.nn.Module, src: int = 0):
    """Broadcast all parameters and buffers of `module` from rank `src`."""
    if world() == 1:
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src=src)


def all_reduce_mean_(t: torch.Tensor) -> torch.Tensor:
    if world() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t.div_(world())
    return t
