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


class GraphedSteps:
    """One captured forward + backward per input "key" for steps whose shapes depend on the data
    only through a small set of host-known keys — the decoder train step: its context rows are
    allocated at the valid total rounded up to the GEMM row bucket, and nothing else in the step
    depends on the batch on the host (the jagged gather and the attention kernels keep the tail rows
    zero on the device; attention runs over the padded width). Replaces the reference's
    torch.compile(mode="reduce-overhead") on EncoderDecoderRetrievalModel.forward
    (modules/model.py:247) without inductor: ~140 host launches per step become one graph launch.

        gs = GraphedSteps(loss_fn, key_fn, buckets)
        loss = gs(batch)              # copy batch -> static inputs, replay the key's graph
        buckets.synchronize(); opt.step()

    * `loss_fn(static_batch) -> loss` runs forward + the loss; `gs` calls backward inside the
      capture. Gradients accumulate into `buckets`' flat buffers (dp.GradBuckets with
      flat_views=True, overlap=False), zeroed inside the graph, so every key's graph writes the
      same gradient storage the optimizer reads. The exchange (N > 1) and the optimizer step run
      after the replay, outside the graph.
    * Dropout: each dropout site's key is fixed at capture; the device-side epoch
      (ops.seed_epoch_advance, captured last) changes every replay, so masks are fresh per step.
    * `key_fn(batch) -> hashable` (host only, no sync); a batch's tensors are copied into static
      inputs of identical shapes (shared by all keys). `prepare(static, batch)` may re-attach
      host-side metadata (e.g. registered row counts) to the static inputs before a capture.
    * All graphs share one memory pool (they never run concurrently).
    * A capture must not overlap a live eager autograd graph of the same parameters (e.g. a kept
      `loss` of an eager step): its AccumulateGrad nodes belong to the default stream and would
      break the capture. Drop such references (or `.detach()` them) before a new key's first call."""

    def __init__(self, loss_fn, key_fn, buckets, prepare=None, warmup: int = 2):
        self.loss_fn, self.key_fn, self.buckets, self.prepare, self.warmup = loss_fn, key_fn, buckets, prepare, warmup
        self.graphs = {}
        self.static = None
        self.pool = None

    def _copy_in(self, batch):
        if self.static is None:
            self.static = type(batch)(*[None if t is None else t.clone() for t in batch])
        else:
            for dst, src in zip(self.static, batch):
                if dst is not None:
                    dst.copy_(src, non_blocking=True)

    def _body(self):
        from . import ops
        self.buckets.zero_grad()
        loss = self.loss_fn(self.static)
        loss.backward()
        ops.join_wgrad_stream()   # side-stream weight grads rejoin inside the capture
        ops.seed_epoch_advance()
        return loss.detach()

    def _capture(self, key, batch):
        if self.prepare is not None:
            self.prepare(self.static, batch)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):   # first launches (library init, GEMM tuning) stay out of the graph
            for _ in range(self.warmup):
                self._body()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self.pool):
            loss = self._body()
        if self.pool is None:
            self.pool = g.pool()
        self.graphs[key] = (g, loss)
        return self.graphs[key]

    def __call__(self, batch):
        key = self.key_fn(batch)
        self._copy_in(batch)
        entry = self.graphs.get(key)
        if entry is None:
            entry = self._capture(key, batch)
        entry[0].replay()
        return entry[1]
