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
