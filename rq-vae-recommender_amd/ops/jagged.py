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
import weakref

import torch
from torch import Tensor

from rqvae_hip import ops as hip_ops

__all__ = ["padded_to_jagged_tensor", "jagged_to_flattened_tensor", "jagged_to_padded_tensor", "Jagged",
           "padded_to_jagged", "as_jagged"]


class Jagged:
    """Dense view of a jagged batch: values (T, C) + int64 offsets (B+1) + length bounds.

    The model internals run on this (every op on the jagged axis is row-wise, so it applies to
    ``values`` directly) instead of torch NJT, whose per-op Python dispatch dominated the decoder
    step on the host. Exposes ``values()`` / ``offsets()`` like an NJT; ``to_nested()`` converts.
    """

    __slots__ = ("_values", "_offsets", "max_len", "min_len", "rows")

    def __init__(self, values: Tensor, offsets: Tensor, max_len: int, min_len: int = 0, rows: int = None):
        self._values, self._offsets, self.max_len, self.min_len = values, offsets, int(max_len), int(min_len)
        # valid rows (= offsets[-1]) when known on the host, else None; values may carry zero tail
        # rows past it (row bucketing, see rqvae_hip.gemm_tuning), which every row-wise op carries
        # along and the attention / gather kernels keep zero on the device
        self.rows = None if rows is None else int(rows)

    def values(self) -> Tensor:
        return self._values

    def offsets(self) -> Tensor:
        return self._offsets

    def with_values(self, values: Tensor) -> "Jagged":
        return Jagged(values, self._offsets, self.max_len, self.min_len, self.rows)

    def valid_rows(self) -> int:
        """offsets[-1] (a device -> host sync when the caller did not know it)."""
        return self.rows if self.rows is not None else int(self._offsets[-1])

    def to_nested(self):
        return torch.nested.nested_tensor_from_jagged(self._values[:self.valid_rows()], self._offsets,
                                                      min_seqlen=self.min_len, max_seqlen=self.max_len)

    @property
    def shape(self):
        return (self._offsets.shape[0] - 1, None, self._values.shape[-1])


def as_jagged(x) -> Jagged:
    """NJT or Jagged -> Jagged (no copy)."""
    if isinstance(x, Jagged):
        return x
    mx = getattr(x, "_maybe_max_seqlen", None)  # NJT: values rows == offsets[-1]
    mn = getattr(x, "_maybe_min_seqlen", None)
    if mx is None:
        mx = x._get_max_seqlen()
    return Jagged(x.values(), x.offsets(), int(mx), int(mn or 0), int(x.values().shape[0]))


_HOST_ROWS = {}


def register_row_counts(mask: Tensor, counts) -> None:
    """Attach host-side per-row valid counts to a device mask tensor (a data loader that builds its
    batches on the CPU knows them for free), so the jagged conversions of that batch need no
    device -> host sync: the entry lives as long as the tensor."""
    c = [int(v) for v in counts]
    key = id(mask)
    _HOST_ROWS[key] = (weakref.ref(mask), (sum(c), min(c), max(c), len(c)))
    weakref.finalize(mask, _HOST_ROWS.pop, key, None)


def copy_row_counts(dst: Tensor, src: Tensor) -> None:
    """Give `dst` the host-side row counts registered for `src` (e.g. a captured step's static
    input mask takes over the counts of the batch it is captured with)."""
    e = _HOST_ROWS.get(id(src))
    if e is not None and e[0]() is src:
        key = id(dst)
        d = _HOST_ROWS.get(key)
        if d is not None and d[0]() is dst:   # dst already tracked (a static input): update, no new finalizer
            _HOST_ROWS[key] = (d[0], e[1])
            return
        _HOST_ROWS[key] = (weakref.ref(dst), e[1])
        weakref.finalize(dst, _HOST_ROWS.pop, key, None)


def row_counts(mask: Tensor):
    """(sum, min, max, rows) of the counts registered for `mask`, or None."""
    e = _HOST_ROWS.get(id(mask))
    return e[1] if e is not None and e[0]() is mask else None


def padded_to_jagged(x: Tensor, lengths: Tensor, max_len: int, total: int = None, add_one_sub_one: bool = True,
                     known_max: int = None, row_bucket: int = None, known_min: int = None,
                     alloc_rows: int = None) -> Jagged:
    """HIP padded -> jagged gather. `total` / `known_max` (host ints) skip the host sync when the
    caller already knows them (e.g. fixed-length decoder inputs). `row_bucket`: allocate the values
    with their row count rounded up to this multiple (bounded set of GEMM shapes). `alloc_rows`: the
    allocation itself (>= the valid total; graph-captured steps pass the bucket and never the exact
    total). Rows past the valid total are zero-filled by the kernel on the device."""
    assert x.dim() == 3 and x.is_contiguous()
    hip_ops.require_gpu(x, lengths, what="padded_to_jagged")
    B, N, _ = x.shape
    n = min(int(max_len), N)
    offsets = hip_ops.jagged_offsets(lengths, n)
    if alloc_rows is not None:
        lmax = known_max if known_max is not None else n
        lmin = known_min if known_min is not None else 0
        alloc = int(alloc_rows)
    else:
        if total is None:
            total, lmin, lmax = torch.stack([offsets[-1], lengths.clamp(0, n).min(), lengths.clamp(0, n).max()]).tolist()
        else:
            lmax = known_max if known_max is not None else n
            lmin = known_min if known_min is not None else lmax
        alloc = int(total) if not row_bucket else (int(total) + row_bucket - 1) // row_bucket * row_bucket
    values = hip_ops.PaddedToJaggedValues.apply(x, offsets, alloc, add_one_sub_one, total)
    return Jagged(values, offsets, int(lmax), int(lmin), None if total is None else int(total))


def padded_to_jagged_tensor(x: Tensor, lengths: Tensor, max_len: int):
    assert x.dim() == 3
    assert lengths.shape[0] == x.shape[0]
    assert x.is_contiguous()
    # one host sync (the reference's torch.empty(lengths.sum()) has the same one)
    return padded_to_jagged(x, lengths, max_len).to_nested()


def jagged_to_flattened_tensor(x) -> Tensor:
    return x.values()


def jagged_to_padded_tensor(x, max_len: int) -> Tensor:
    # accepts an NJT or a Jagged
    """NJT (B, j, D) -> zero-padded (B, max_len, D) via the HIP scatter kernel (differentiable)."""
    return hip_ops.JaggedToPaddedValues.apply(x.values(), x.offsets(), int(max_len))
