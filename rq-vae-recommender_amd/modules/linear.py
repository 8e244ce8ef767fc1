"""nn.Linear with the MI355X weight-gradient path.

Same parameters, init and state-dict keys as torch.nn.Linear (the reference builds its MLPs from
nn.Linear, modules/encoder.py:20-31), so checkpoints are interchangeable. On the device the forward
and data gradient stay on hipBLASLt while grad_weight / grad_bias — a reduction over the whole
batch — run on rq_linear_wgrad (rqvae_hip.ops.LinearFunction). CPU tensors take torch's path.
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
