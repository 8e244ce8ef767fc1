"""Alias of ops.jagged (reference import path ops/triton/jagged.py); HIP kernels, no Triton."""
from ops.jagged import jagged_to_flattened_tensor, jagged_to_padded_tensor, padded_to_jagged_tensor  # noqa: F401
