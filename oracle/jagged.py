"""Padded <-> jagged conversion — numpy restatement. Test infrastructure only.

Reference: ops/triton/jagged.py (PaddedToJaggedTensor forward :11-66 incl. the Triton
kernel :92-125, backward :69-77).
"""
import numpy as np


def offsets_from_lengths(lengths):
    """offsets = [0, cumsum(lengths)] (ops/triton/jagged.py:30-33)."""
    return np.concatenate([[0], np.cumsum(np.asarray(lengths, np.int64))]).astype(np.int64)


def padded_to_jagged(x, lengths, add_one_sub_one=True):
    """values[offsets[b] + t] = x[b, t] for t < len_b (kernel :112-124), then `target + 1 - 1`
    (:65), which rounds each value through (v + 1) in x.dtype before subtracting 1."""
    off = offsets_from_lengths(lengths)
    vals = np.concatenate([x[b, : int(lengths[b])] for b in range(x.shape[0])], 0).astype(x.dtype)
    if add_one_sub_one:
        one = x.dtype.type(1)
        vals = ((vals + one).astype(x.dtype) - one).astype(x.dtype)
    return vals, off


def jagged_to_padded_grad(grad_values, lengths, N):
    """grad_x = zeros(B,N,D); grad_x[mask] = grad_values  (backward :69-77)."""
    lengths = np.asarray(lengths, np.int64)
    B, D = lengths.shape[0], grad_values.shape[1]
    out = np.zeros((B, N, D), grad_values.dtype)
    off = offsets_from_lengths(lengths)
    for b in range(B):
        out[b, : lengths[b]] = grad_values[off[b]: off[b + 1]]
    return out
