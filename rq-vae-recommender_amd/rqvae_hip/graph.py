"""Whole-step hipGraph capture (torch.cuda.CUDAGraph on ROCm = hipGraph).

The reference relies on torch.compile(mode="reduce-overhead") (CUDA graphs via inductor,
modules/rqvae.py:140) to amortise launch cost at its B=64 config; inductor emits Triton on
ROCm, so this build captures the eager step instead. Every HIP kernel of the path is launched
on torch's current stream with caller-owned workspaces and no host synchronisation, so the
full forward + backward (+ optimizer) records into one graph.

    step = CapturedStep(lambda: train_step(static_x), warmup=3)
    static_x.copy_(next_batch); out = step()      # replays the recorded kernels

Requirements: static shapes, inputs copied into the captured tensors before replay,
optimizer constructed with capturable=True, grads zeroed in place (set_to_none=False) inside
the step, and no data-dependent host syncs (the RQ-VAE step has none; the decoder step's
jagged total is data-dependent and is not captured).
"""
import torch


class CapturedStep:
    def __init__(self, step_fn, warmup: int = 3):
        self.step_fn = step_fn
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                step_fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = step_fn()

    def __call__(self):
        self.graph.replay()
        return self.out


def _in_graph_default(buckets) -> bool:
    """Capture the exchange inside the step graph where the backend can be captured (RCCL; gloo
    cannot: it moves tensors through the host)."""
    import torch.distributed as dist
    if buckets is None or not buckets.exchange:
        return False
    if not dist.is_initialized():
        return False
    return dist.get_backend() == "nccl"


WATCHDOG_RETIRE_S = 5.0
WATCHDOG_RETIRE_AGREED_S = 60.0   # world > 1 without the local fallback: wait longer, then fail loudly


def _local_fallback_default() -> bool:
    """RQVAE_LOCAL_EXCHANGE_FALLBACK=1 lets one rank of a world > 1 job move its exchange out of the graph
    on its own (the round-5 behaviour). Off by default: RCCL with captured collectives on some ranks and
    eager ones on others has never run on hardware, so a rank that cannot capture fails loudly instead."""
    import os
    return os.environ.get("RQVAE_LOCAL_EXCHANGE_FALLBACK", "0") == "1"


def watchdog_retired(timeout_s: float = None):
    """Before an in-graph capture: wait until the RCCL process groups' watchdogs have RETIRED every
    eager collective of this process. On ROCm a watchdog query of such a collective's event while the
    exchange is being captured fails the capture even in thread-local mode ("dependency created on
    uncaptured work in another stream", tools/graph_exchange_probe.py race_forever); the watchdog stops
    querying a Work when it retires it. The flight recorder (dp.enable_watchdog_record, on by default in
    dp.init_from_env) marks each recorded collective `retired` exactly then, and captured collectives
    are never recorded (tools/fr_probe.py), so "every entry retired" is the watchdog's list being empty.
    Returns True once it is (device work synchronised first: the watchdog retires completed work only),
    False if it is not within the bound, None when the flight recorder is off (nothing to check)."""
    import json
    import threading
    import time
    from .dp import watchdog_record_enabled
    if not watchdog_record_enabled():
        return None
    import torch._C._distributed_c10d as c10d
    torch.cuda.synchronize()
    deadline = time.monotonic() + (WATCHDOG_RETIRE_S if timeout_s is None else timeout_s)
    poll = threading.Event()
    while True:
        d = json.loads(c10d._dump_nccl_trace_json(includeCollectives=True, onlyActive=False))
        if all(e.get("retired", False) for e in d.get("entries", [])):
            return True
        if time.monotonic() > deadline:
            return False
        poll.wait(0.002)   # poll interval: the watchdog wakes every ~100 ms (retired ~40 ms after completion)


class GraphedSteps:
    """One captured forward + backward per input "key" for steps whose shapes depend on the data
    only through a small set of host-known keys — the decoder train step: its context rows are
    allocated at the valid total rounded up to the GEMM row bucket, and nothing else in the step
    depends on the batch on the host (the jagged gather and the attention kernels keep the tail rows
    zero on the device; attention runs over the padded width). Replaces the reference's
    torch.compile(mode="reduce-overhead") on EncoderDecoderRetrievalModel.forward
    (modules/model.py:247) and RqVae.forward (modules/rqvae.py:140) without inductor: ~140 host
    launches per step become one graph launch.

        gs = GraphedSteps(loss_fn, key_fn, buckets)
        loss = gs(batch)              # copy batch -> static inputs, replay the key's graph
        buckets.synchronize(); opt.step()

    * `loss_fn(static_batch) -> loss` runs forward + the loss; `gs` calls backward inside the
      capture. With `run_backward=False`, `loss_fn` runs its own backward pass(es) (e.g. micro-batches
      under `buckets.no_sync()`) and returns the detached tensor(s) to keep. Gradients accumulate
      into `buckets`' flat buffers (dp.GradBuckets with flat_views=True), zeroed inside the graph, so
      every key's graph writes the same gradient storage the optimizer reads.
    * Gradient exchange (N > 1): with an RCCL process group the buckets' all-reduces are captured
      where their hooks fire (in bucket order, overlapping the rest of the backward) together with
      the final wait / average (`in_graph_exchange`, the default there); `buckets.synchronize()` after
      the replay then only finalises. With gloo (rehearsals, CPU tests) the hooks are suspended in the
      graph and the exchange runs after the replay. The placement is one decision shared by every rank:
      the job's first capture (the same step on every rank) settles it with one MIN all-reduce of the
      ranks' capture outcomes; a later capture that cannot hold the collectives raises at world > 1
      (falls back at world 1, or with `local_fallback`).
      Every rank runs exactly one exchange per step: the very first step is an eager probe (it also
      settles which parameters are unused on every rank), and a new key's warm-up passes do not
      communicate.
    * Dropout: each dropout site's key is fixed at capture; the device-side epoch
      (ops.seed_epoch_advance, captured last) changes every replay, so masks are fresh per step.
    * `key_fn(batch) -> hashable` (host only, no sync); a batch (a tensor, or a nested tuple /
      NamedTuple of tensors) is copied into static inputs of identical shapes (one set per shape
      signature, shared by all keys of that signature; a graph is keyed by (signature, key)).
      `prepare(static, batch)` may re-attach host-side metadata (e.g. registered row counts) to the
      static inputs before a capture. Beyond `max_graphs` distinct graphs, new (signature, key)
      pairs run eagerly (e.g. token-balanced shards whose sequence count changes every step).
    * All graphs share one memory pool (they never run concurrently).
    * `capture=False` runs the same bodies eagerly (the exchange inside the body, as captured): the
      CPU / gloo tests exercise the in-graph exchange logic this way.
    * A capture must not overlap a live eager autograd graph of the same parameters (e.g. a kept
      `loss` of an eager step): its AccumulateGrad nodes belong to the default stream and would
      break the capture. Drop such references (or `.detach()` them) before a new key's first call."""

    def __init__(self, loss_fn, key_fn, buckets, prepare=None, warmup: int = 2, run_backward: bool = True,
                 in_graph_exchange=None, capture: bool = True, max_graphs: int = 16, local_fallback=None):
        self.loss_fn, self.key_fn, self.buckets, self.prepare, self.warmup = loss_fn, key_fn, buckets, prepare, warmup
        self.run_backward = run_backward
        self.in_graph = _in_graph_default(buckets) if in_graph_exchange is None else bool(in_graph_exchange)
        self.local_fallback = _local_fallback_default() if local_fallback is None else bool(local_fallback)
        self.capture = capture
        self.capture_error = None
        self.max_graphs = max_graphs
        self.graphs = {}
        self.statics = {}
        self.static = None
        self.pool = None
        self._probed = False
        self._settled = False   # the job's first capture (and with it the exchange placement) is done
        self.eager_steps = 0

    @staticmethod
    def _signature(batch):
        """Shapes / dtypes of every tensor of a (nested tuple / NamedTuple of) batch: batches with
        the same signature share one set of static input tensors."""
        if isinstance(batch, torch.Tensor):
            return (tuple(batch.shape), batch.dtype)
        if batch is None:
            return None
        return tuple(GraphedSteps._signature(t) for t in batch)

    @staticmethod
    def _clone(batch):
        if isinstance(batch, torch.Tensor):
            return batch.clone()
        if batch is None:
            return None
        items = [GraphedSteps._clone(t) for t in batch]
        return type(batch)(*items) if hasattr(batch, "_fields") else type(batch)(items)

    @staticmethod
    def _pairs(dst, src, out):
        if isinstance(dst, torch.Tensor):
            out.append((dst, src))
        elif dst is not None:
            for d, s_ in zip(dst, src):
                GraphedSteps._pairs(d, s_, out)
        return out

    @staticmethod
    def _copy(dst, src):
        """The batch into the static inputs: one multi-tensor copy launch per dtype (torch's foreach copy
        takes its single-launch route only for lists of one dtype) instead of one copy per field."""
        groups = {}
        for d, s_ in GraphedSteps._pairs(dst, src, []):
            groups.setdefault((d.dtype, s_.dtype, d.device), []).append((d, s_))
        for pairs in groups.values():
            if len(pairs) == 1:
                pairs[0][0].copy_(pairs[0][1], non_blocking=True)
            else:
                torch._foreach_copy_([d for d, _ in pairs], [s_ for _, s_ in pairs], non_blocking=True)

    def _copy_in(self, batch, sig):
        st = self.statics.get(sig)
        if st is None:
            st = self.statics[sig] = self._clone(batch)
        else:
            self._copy(st, batch)
        self.static = st

    def _body(self, exchange: bool):
        from . import ops
        b = self.buckets
        if b is not None:
            b.zero_grad()
        out = self.loss_fn(self.static)
        if self.run_backward:
            out.backward(self._seed_grad(out))
            out = out.detach()
        ops.flush_reductions()    # deferred weight-grad reductions (their list lives only at capture)
        if exchange and b is not None:
            b.finish()
        if self.capture:   # eager bodies draw their dropout keys from the host counter
            ops.seed_epoch_advance()
        return out

    def _warm(self):
        import contextlib
        side = torch.cuda.Stream() if self.capture else None
        if side is not None:
            side.wait_stream(torch.cuda.current_stream())
        ctx = torch.cuda.stream(side) if side is not None else contextlib.nullcontext()
        susp = self.buckets.suspended() if self.buckets is not None else contextlib.nullcontext()
        with ctx, susp:   # first launches (library init, GEMM tuning) stay out of the graph; no exchange
            for _ in range(self.warmup):
                self._body(exchange=False)
        if side is not None:
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()

    def _agreed(self) -> bool:
        """True when every rank must keep the same exchange placement: world > 1 without the opt-in
        local fallback (RQVAE_LOCAL_EXCHANGE_FALLBACK=1 / local_fallback=True)."""
        return self._world() > 1 and not self.local_fallback

    def _deviate(self, why: str):
        """This rank cannot capture the exchange. World 1 (or the opt-in local fallback): record why and
        exchange after the replay. World > 1 by default: raise — a rank replaying RCCL collectives from a
        graph while a peer issues the same all-reduces eagerly has never been run on hardware, and a
        mismatch would hang the whole job; an error on one rank ends it (torchrun tears the others down)."""
        self.capture_error = why[:300]
        if self._agreed():
            raise RuntimeError(
                "GraphedSteps: rank %d cannot capture the gradient exchange (%s); its peers capture it, and "
                "mixing captured and eager RCCL collectives across ranks is unverified. Set "
                "RQVAE_LOCAL_EXCHANGE_FALLBACK=1 to let this rank exchange after its replay, or build the "
                "GraphedSteps with in_graph_exchange=False on every rank." % (self._rank(), why))

    def _agree_all(self, ok: bool) -> bool:
        """MIN over the ranks of this rank's outcome (one small eager all-reduce on the default group); the
        local outcome when no process group is up."""
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            return ok
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self._device())
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    def _capture(self, key, batch):
        """Warm up and capture a new key's step. Whether a graph holds the exchange is decided ONCE for
        the job, the same on every rank: at the job's FIRST capture — every rank's second call (the first
        is the eager probe), so the same step everywhere whatever the keys — each rank tries to capture the
        collectives and one MIN all-reduce of the outcomes settles it; if any rank failed, every rank
        records its graphs without them and exchanges after the replay from then on. A later capture (a new
        key) that cannot hold the collectives after the job agreed on in-graph exchange raises at world > 1
        (`_deviate`) unless the local fallback is enabled; at world 1 it falls back to a graph without them.
        With the local fallback, every rank still issues the same all-reduces in bucket order once per step,
        in the graph or after it, so ranks that decide differently — or that capture different keys in the
        same step (the decoder's keys come from each rank's own shard), or replay while another rank
        captures or runs eagerly past `max_graphs` — issue matching sequences."""
        if self.prepare is not None:
            self.prepare(self.static, batch)
        self._warm()
        exchanged = self.in_graph
        agree = exchanged and not self._settled and self._agreed()   # the job's first capture, world > 1
        # thread_local capture mode everywhere: other threads of the process keep making HIP calls while
        # the step is captured — the process group's watchdog polls the events of earlier (eager)
        # collectives, a trainer's feed thread pins host memory (the caching host allocator queries and
        # records events) — and under the default global mode any such call fails the capture ("operation
        # not permitted when stream is capturing", seen on MI355X with the watchdog)
        if exchanged and self.capture:
            bound = WATCHDOG_RETIRE_AGREED_S if self._agreed() else WATCHDOG_RETIRE_S
            idle = watchdog_retired(bound)
            if not idle:
                exchanged = False
                why = ("flight recorder off: the watchdog's work list cannot be checked" if idle is None else
                       f"watchdog kept an eager collective past {bound} s")
                if agree:
                    self.capture_error = why
                else:
                    self._deviate(why)
                    if idle is None:   # cannot be checked in this process: never capture the exchange
                        self.in_graph = False
        g, out, err = self._try_capture(exchanged)
        if err is not None:
            if not exchanged:
                raise err if isinstance(err, BaseException) else RuntimeError(err)
            if self.capture:
                torch.cuda.synchronize()
            if agree:
                self.capture_error = repr(err)[:300]
            else:
                self._deviate(repr(err))
                self.in_graph = False   # this rank exchanges after the replay from now on
            exchanged = False
            g, out, err2 = self._try_capture(False)
            if err2 is not None:
                raise err2
        if agree:
            if not self._agree_all(exchanged):   # some rank could not: nobody holds the exchange in a graph
                self.in_graph = False
                self.capture_error = self.capture_error or "a peer rank could not capture the exchange"
                if exchanged:
                    exchanged = False
                    if self.capture:
                        torch.cuda.synchronize()
                    g, out, err2 = self._try_capture(False)   # the graph with the collectives is dropped unreplayed
                    if err2 is not None:
                        raise err2
        self._settled = True
        if g is not None and self.pool is None:
            self.pool = g.pool()
        self.graphs[key] = (g, out, exchanged)
        return self.graphs[key]

    def _try_capture(self, in_graph: bool):
        """Capture one step body: (graph, its output, None) or (None, None, the exception).
        capture=False: (None, None, None) — the body runs eagerly at every call."""
        import contextlib
        if not self.capture:
            return None, None, None
        g = torch.cuda.CUDAGraph()
        susp = contextlib.nullcontext() if in_graph else self.buckets.suspended()
        try:
            with torch.cuda.graph(g, pool=self.pool, capture_error_mode="thread_local"), susp:
                out = self._body(exchange=in_graph)
        except Exception as e:
            return None, None, e
        return g, out, None

    @staticmethod
    def _world() -> int:
        import torch.distributed as dist
        return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1

    @staticmethod
    def _rank() -> int:
        import torch.distributed as dist
        return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0

    def _device(self):
        b = self.buckets
        if b is not None and b.buckets:
            return b.buckets[0]["flat"].device
        return torch.device("cuda", torch.cuda.current_device())

    def _eager(self, batch):
        """One ordinary eager step on the batch itself (the exchange from the hooks; the caller's
        synchronize() finishes it)."""
        self.eager_steps += 1
        b = self.buckets
        if b is not None:
            b.zero_grad()
        out = self.loss_fn(batch)
        if self.run_backward:
            out.backward(self._seed_grad(out))
            out = out.detach()
        return out

    def _seed_grad(self, out):
        """d out / d out = 1 for a scalar loss, kept across steps (backward() would fill a fresh one: a
        launch per step); None (autograd's own seed) for anything else."""
        if out.dim() != 0:
            return None
        one = getattr(self, "_one", None)
        if one is None or one.device != out.device or one.dtype != out.dtype:
            one = self._one = torch.ones((), device=out.device, dtype=out.dtype)
        return one

    def __call__(self, batch):
        sig = self._signature(batch)
        key = (sig, self.key_fn(batch))
        entry = self.graphs.get(key)
        if not self._probed or (entry is None and len(self.graphs) >= self.max_graphs):
            # first step: eager on every rank (settles the unused parameters before anything is
            # captured); past max_graphs: eager. Neither touches the static inputs.
            self._probed = True
            return self._eager(batch)
        self._copy_in(batch, sig)
        if entry is None:
            entry = self._capture(key, batch)
        g, out, exchanged = entry
        if g is None:   # capture=False: the body runs eagerly, with the captured form's exchange
            import contextlib
            if self.prepare is not None:
                self.prepare(self.static, batch)
            susp = self.buckets.suspended() if (self.buckets is not None and not exchanged) else contextlib.nullcontext()
            with susp:
                out = self._body(exchange=exchanged)
        else:
            g.replay()
        if exchanged and self.buckets is not None:
            self.buckets.mark_graph_exchanged()
        return out
