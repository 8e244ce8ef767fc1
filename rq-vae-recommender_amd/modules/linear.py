"""nn.Linear with the MI355X weight-gradient path.

Same parameters, init and state-dict keys as torch.nn.Linear (the reference builds its MLPs from
nn.Linear, modules/encoder.py:20-31), so checkpoints are interchangeable. Device fp32 inputs run
rqvae_hip.ops.LinearFunction: at matmul precision 'high' (the reference's setting) forward, data and
weight gradients on the split-bf16 MFMA GEMM; at 'highest' forward / data gradient on hipBLASLt and
grad_weight / grad_bias on rq_linear_wgrad. Module-level CPU use (building a model, loading a
checkpoint, the reference's own CPU runs) keeps nn.Linear's torch path — that is the module's
contract, not a fallback of a HIP op: every rqvae_hip op raises RqHipError on CPU tensors.
"""
import torch
from torch import nn
from torch.nn import functional as F

from rqvae_hip import ops


class Linear(nn.Linear):
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda and x.dtype == torch.float32 and ops.wgrad_supported(self.weight):
            return ops.LinearFunction.apply(x, self.weight, self.bias)
        return F.linear(x, self.weight, self.bias)
