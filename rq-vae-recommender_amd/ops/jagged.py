"""Padded <-> jagged (NJT) conversion — drop-in for reference ops/triton/jagged.py.

API kept: ``padded_to_jagged_tensor(x, lengths, max_len) -> NestedTensor`` (:80-85) and
``jagged_to_flattened_tensor(nt) -> Tensor`` (:88-89); backward returns (grad_x, None, None)
semantics (:69-77): grad_x = zeros(B, N, D) with grad_x[mask] = grad_values.

MI355X path: offsets come from a one-block scan kernel, the values from the HIP gather kernel
(jagged_from_padded, one 16-B-per-lane pass over the valid rows, reproducing the reference's
``target + 1 - 1`` rounding bit-exactly), the backward from jagged_to_padded (writes every
padded element once: copy or zero). Offsets are int64 (the reference stores them in x.dtype,
SURVEY A-1), and the NJT carries exact min/max sequence lengths, so downstream varlen
attention never recomputes them.
"""
import torch
from torch import Tensor

from rqvae_hip import ops as hip_ops

__all__ = ["padded_to_jagged_tensor", "jagged_to_flattened_tensor", "jagged_to_padded_tensor"]


def padded_to_jagged_tensor(x: Tensor, lengths: Tensor, max_len: int):
    assert x.dim() == 3
    assert lengths.shape[0] == x.shape[0]
    assert x.is_contiguous()
    hip_ops.require_gpu(x, lengths, what="padded_to_jagged_tensor")
    B, N, _ = x.shape
    n = min(int(max_len), N)
    offsets = hip_ops.jagged_offsets(lengths, n)
    # one host sync (the reference's torch.empty(lengths.sum()) has the same one)
    total, lmin, lmax = torch.stack([offsets[-1], lengths.clamp(0, n).min(), lengths.clamp(0, n).max()]).tolist()
    values = hip_ops.PaddedToJaggedValues.apply(x, offsets, int(total), True)
    return torch.nested.nested_tensor_from_jagged(values, offsets, min_seqlen=int(lmin), max_seqlen=int(lmax))


def jagged_to_flattened_tensor(x) -> Tensor:
    return x.values()


def jagged_to_padded_tensor(x, max_len: int) -> Tensor:
    """NJT (B, j, D) -> zero-padded (B, max_len, D) via the HIP scatter kernel (differentiable)."""
    return hip_ops.JaggedToPaddedValues.apply(x.values(), x.offsets(), int(max_len))
