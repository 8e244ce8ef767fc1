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
      the replay then only finalises. With gloo (rehearsals, CPU tests) or when capturing the
      collectives fails, the hooks are suspended in the graph and the exchange runs after the replay.
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
                 in_graph_exchange=None, capture: bool = True, max_graphs: int = 16):
        self.loss_fn, self.key_fn, self.buckets, self.prepare, self.warmup = loss_fn, key_fn, buckets, prepare, warmup
        self.run_backward = run_backward
        self.in_graph = _in_graph_default(buckets) if in_graph_exchange is None else bool(in_graph_exchange)
        self.capture = capture
        self.capture_error = None
        self.max_graphs = max_graphs
        self.graphs = {}
        self.statics = {}
        self.static = None
        self.pool = None
        self._probed = False
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
    def _copy(dst, src):
        if isinstance(dst, torch.Tensor):
            dst.copy_(src, non_blocking=True)
        elif dst is not None:
            for d, s_ in zip(dst, src):
                GraphedSteps._copy(d, s_)

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
            out.backward()
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

    def _capture(self, key, batch):
        if self.prepare is not None:
            self.prepare(self.static, batch)
        self._warm()
        if not self.capture:
            self.graphs[key] = (None, None)
            return self.graphs[key]
        # thread_local capture mode everywhere: other threads of the process keep making HIP calls while
        # the step is captured — the process group's watchdog polls the events of earlier (eager)
        # collectives, a trainer's feed thread pins host memory (the caching host allocator queries and
        # records events) — and under the default global mode any such call fails the capture ("operation
        # not permitted when stream is capturing", seen on MI355X with the watchdog)
        if self.in_graph:
            self._quiesce()
        g, out, err = self._try_capture(self.in_graph)
        if self.in_graph and self._world() > 1:
            # one decision for all ranks: if any rank failed to capture its collectives, every rank
            # exchanges after the replay (a mixed in-graph / post-replay world would still issue the same
            # all-reduces, but nothing would test it)
            ok = torch.tensor([0.0 if err is not None else 1.0], device=self._device())
            import torch.distributed as dist
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if float(ok.item()) == 0.0:
                err = err or "capture of the exchange failed on another rank"
        if err is not None:
            if not self.in_graph:
                raise err if isinstance(err, BaseException) else RuntimeError(err)
            self.capture_error = repr(err)[:300]
            self.in_graph = False
            torch.cuda.synchronize()
            g, out, err2 = self._try_capture(False)
            if err2 is not None:
                raise err2
        if self.pool is None:
            self.pool = g.pool()
        self.graphs[key] = (g, out)
        return self.graphs[key]

    # ProcessGroupNCCL's watchdog thread wakes every 100 ms and queries the end events of the collectives
    # it tracks until it sees them complete. On ROCm a query of such an event from another thread while
    # the exchange is being captured fails the capture even in thread-local mode ("dependency created on
    # uncaptured work in another stream", tools/graph_exchange_probe.py race_forever), so before an
    # in-graph capture every earlier collective is completed on the device and the watchdog is given
    # more than two of its polling periods to retire them.
    QUIESCE_S = 0.3

    def _quiesce(self):
        import time
        torch.cuda.synchronize()
        time.sleep(self.QUIESCE_S)

    def _try_capture(self, in_graph: bool):
        """Capture one step body: (graph, its output, None) or (None, None, the exception)."""
        import contextlib
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
            out.backward()
            out = out.detach()
        return out

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
        g, out = entry
        if g is None:   # capture=False: the body runs eagerly, with the captured form's exchange
            if self.prepare is not None:
                self.prepare(self.static, batch)
            out = self._body(exchange=self.in_graph)
        else:
            g.replay()
        if self.in_graph and self.buckets is not None:
            self.buckets.mark_graph_exchanged()
        return out
