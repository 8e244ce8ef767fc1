"""Torch-facing ops over the HIP C ABI: autograd Functions for the RQ-VAE hot path.

  rq_quantize(x, codebooks, mode, beta)      fused L-level residual quantization (fwd + VJP)
  unique_count(ids, K)                       #distinct semantic-ID tuples (device scalar)
  unique_fraction(ids, K)                    p_unique_ids = that count / B (fp32 device scalar, 2 launches)
  padded_to_jagged_values(x, lengths, N)     jagged gather (+1-1 rounding) + offsets (fwd + VJP)
  varlen_attention(q, k, v, cu_q, cu_k, ...) jagged SDPA (fwd + deterministic VJP)
  gemm_bf16x3 / gemm_x3 / mlp_chain          fp32 matmuls at 'high' precision (split-bf16 MFMA)

All kernels run on torch's current HIP stream; tensors must be on the GPU (no CPU path).
"""
import contextlib
import math
from typing import NamedTuple

import torch
import torch.distributed as _dist

from . import _lib
from ._lib import RqHipError, call, ptr, stream_handle, require_gpu

MODE_EVAL, MODE_GUMBEL, MODE_STE, MODE_ROTATION = 0, 1, 2, 3


class KernelTimer:
    """Opt-in measurement hook: when ``ops.TIMER.enabled`` is set, HIP events are recorded on the
    launching stream around each named C-ABI call, so a benchmark can report per-kernel device
    time for the exact launches inside its timed region (no extra synchronisation)."""

    def __init__(self):
        self.enabled = False
        self.only = None      # optional set of name prefixes to record (others run untimed)
        self.events = {}
        self.bytes = {}

    def wants(self, name: str) -> bool:
        return self.enabled and (self.only is None or any(name.startswith(p) for p in self.only))

    def around(self, name, fn, *args):
        if not self.wants(name):
            return fn(*args)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn(*args)
        b.record()
        self.events.setdefault(name, []).append((a, b))

    def reset(self):
        self.events = {}
        self.bytes = {}

    def gbps(self, name):
        """Algorithmic bytes / device time over all recorded launches of `name`."""
        ev = self.events.get(name, [])
        t = sum(a.elapsed_time(b) for a, b in ev) * 1e-3
        return (sum(self.bytes.get(name, [])) / t / 1e9) if t > 0 else 0.0

    def mean_ms(self, name):
        ev = self.events.get(name, [])
        return sum(a.elapsed_time(b) for a, b in ev) / max(1, len(ev)), len(ev)


TIMER = KernelTimer()
_DTYPES = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def _c(t):
    return None if t is None else t.contiguous()


# ------------------------------------------------------------------------------- quantize
class RqQuantizeFunction(torch.autograd.Function):
    """Fused RqVae level loop (modules/rqvae.py:114-138 over modules/quantize.py:99-156).

    forward(x (B,D), codebooks (L,K,D)) -> emb_out (L,B,D), residuals (L,B,D), ids (B,L),
    qloss (B,), emb_sum (B,D) [, emb_norms (L,B) = |emb_out[l][b]| (no grad) when with_norms].
    """

    @staticmethod
    def forward(ctx, x, codebooks, mode: int, beta: float, with_norms: bool = False):
        require_gpu(x, codebooks, what="rq_quantize")
        assert x.dim() == 2 and codebooks.dim() == 3 and x.shape[1] == codebooks.shape[2]
        assert x.dtype == torch.float32 and codebooks.dtype == torch.float32, "fp32 path (reference default)"
        x = x.contiguous()
        cbs = codebooks.contiguous()
        B, D = x.shape
        L, K, _ = cbs.shape
        dev = x.device
        csq = torch.empty((L, K), device=dev, dtype=torch.float32)
        ids = torch.empty((B, L), device=dev, dtype=torch.int64)
        emb = torch.empty((L, B, D), device=dev, dtype=torch.float32)
        res = torch.empty((L, B, D), device=dev, dtype=torch.float32)
        ql = torch.empty((B,), device=dev, dtype=torch.float32)
        es = torch.empty((B, D), device=dev, dtype=torch.float32)
        s = stream_handle(dev)
        call("rq_codebook_sqnorm", ptr(cbs), L * K, D, ptr(csq), s)
        norms = torch.empty((L, B), device=dev, dtype=torch.float32) if with_norms else None
        TIMER.around("rq_quantize_fwd", call, "rq_quantize_fwd", ptr(x), B, D, ptr(cbs), ptr(csq), K, L,
                     int(mode), float(beta), ptr(ids), ptr(emb), ptr(res), ptr(ql), ptr(es), ptr(norms), 0, s)
        ctx.save_for_backward(res, ids, cbs)
        ctx.mode, ctx.beta = int(mode), float(beta)
        ctx.mark_non_differentiable(ids)
        ctx.set_materialize_grads(False)   # unused outputs arrive as None = NULL (no (L,B,D) zero fills)
        if with_norms:
            ctx.mark_non_differentiable(ids, norms)
            return emb, res, ids, ql, es, norms
        return emb, res, ids, ql, es

    @staticmethod
    def backward(ctx, g_emb, g_res, g_ids, g_ql, g_es, *g_norms):
        res, ids, cbs = ctx.saved_tensors
        L, B, D = res.shape
        K = cbs.shape[1]
        dev = res.device
        gx = torch.empty((B, D), device=dev, dtype=torch.float32)
        gcb = torch.empty_like(cbs)
        nbytes = _lib.load().rq_quantize_bwd_workspace(B, D, K, L)
        ws = torch.empty((nbytes,), device=dev, dtype=torch.uint8)
        TIMER.around("rq_quantize_bwd", call, "rq_quantize_bwd", ptr(res), ptr(ids), ptr(cbs), B, D, K, L, ctx.mode,
                     ctx.beta, ptr(_c(g_emb)), ptr(_c(g_es)), ptr(_c(g_res)), ptr(_c(g_ql)), ptr(gx), ptr(gcb), ptr(ws),
                     nbytes, stream_handle(dev))
        return gx, gcb, None, None, None


def rq_quantize(x, codebooks, mode=MODE_ROTATION, beta=0.25, with_norms=False):
    """(emb_out, residuals, ids, qloss, emb_sum[, emb_norms]) — see RqQuantizeFunction."""
    return RqQuantizeFunction.apply(x, codebooks, mode, beta, with_norms)


class StackParamsFunction(torch.autograd.Function):
    """torch.stack(params) whose backward adds each slice of the gradient straight into the parameter's
    flat-bucket view through the step's batched reduction (rq_reduce_partials, like the split-K weight
    gradients) when its GradBuckets defers reductions — instead of autograd's stack backward plus one
    AccumulateGrad add kernel per parameter (the RQ-VAE's per-level codebooks: 3 launches a step). Same
    values: the view receives view + g[i] either way."""

    @staticmethod
    def forward(ctx, *ps):
        ctx.ps = ps
        return torch.stack(ps)

    @staticmethod
    def backward(ctx, g):
        from . import dp
        ps, ctx.ps = ctx.ps, None
        out = []
        for i, p in enumerate(ps):
            gi = g[i]
            sink = dp.direct_grad(p) if isinstance(p, torch.nn.Parameter) and dp.defer_ok(p) else None
            if (sink is not None and sink.is_contiguous() and gi.is_contiguous() and gi.numel() % 4 == 0 and
                    (sink.data_ptr() | gi.data_ptr()) % 16 == 0 and sink.data_ptr() not in _DEFER["outs"]):
                _defer_push(gi, sink, gi.numel(), 1, 0)
                dp.direct_grad_done(p)
                out.append(None)
            else:
                out.append(gi)
        return tuple(out)


def stack_params(ps) -> torch.Tensor:
    """torch.stack of parameters with the deferred-gradient backward (StackParamsFunction) on the device."""
    if all(p.is_cuda and p.dtype == torch.float32 for p in ps):
        return StackParamsFunction.apply(*ps)
    return torch.stack(list(ps))


def segment_sum(rows: torch.Tensor, keys: torch.Tensor, K: int, with_counts: bool = True, out: torch.Tensor = None):
    """(sums (K, D), counts (K,) or None) of `rows` grouped by `keys` — deterministic (no float
    atomics). Rows whose key is outside [0, K) are skipped. `out`: a contiguous fp32 (K, D) destination."""
    require_gpu(rows, keys, what="segment_sum")
    rows = rows.contiguous().float()
    keys = keys.contiguous().to(torch.int64)
    B, D = rows.shape
    if out is None:
        out = torch.empty((K, D), device=rows.device, dtype=torch.float32)
    elif not (out.is_contiguous() and out.dtype == torch.float32 and tuple(out.shape) == (K, D)):
        raise RqHipError(f"segment_sum: out must be a contiguous fp32 ({K}, {D}) tensor")
    counts = torch.empty((K,), device=rows.device, dtype=torch.int64) if with_counts else None
    nbytes = _lib.load().rq_segment_sum_workspace(B, K)
    ws = torch.empty((nbytes,), device=rows.device, dtype=torch.uint8)
    call("rq_segment_sum", ptr(rows), ptr(keys), B, D, int(K), ptr(out), ptr(counts), ptr(ws), nbytes,
         stream_handle(rows.device))
    return out, counts


def linear_wgrad(g: torch.Tensor, x: torch.Tensor, with_bias: bool):
    """(dW = g^T x (O, I), db = g.sum(0) (O,) or None) for g (N, O), x (N, I) fp32 — split-K MFMA
    kernel with a fixed-order reduction (rq_linear_wgrad)."""
    require_gpu(g, x, what="linear_wgrad")
    g = g.contiguous()
    x = x.contiguous()
    N, O = g.shape
    I = x.shape[1]
    dW = torch.empty((O, I), device=g.device, dtype=torch.float32)
    db = torch.empty((O,), device=g.device, dtype=torch.float32) if with_bias else None
    nbytes = _lib.load().rq_linear_wgrad_workspace(N, O, I)
    ws = torch.empty((nbytes,), device=g.device, dtype=torch.uint8)
    call("rq_linear_wgrad", ptr(g), O, ptr(x), I, N, O, I, ptr(dW), ptr(db), ptr(ws), nbytes,
         stream_handle(g.device))
    return dW, db



# weight grads over fewer rows than this go to the library GEMM (one launch beats split-K + reduce)
WGRAD_MIN_ROWS = 1024


def wgrad_supported(weight: torch.Tensor) -> bool:
    O, I = weight.shape
    return weight.dtype == torch.float32 and O % 4 == 0 and I % 4 == 0


# With tuned library GEMMs (rqvae_hip.gemm_tuning) the library's g^T x beats the split-K kernel
# up to this many rows (measured: decoder weight grads over ~11k rows 2.8 -> ~2.0 ms/step on the
# tuned library path, RQ-VAE grads over 65,536 rows 1.29 ms on the split-K kernel vs 1.45 ms).
WGRAD_TUNED_LIB_MAX_ROWS = 32768


def _wgrad_choice(g2: torch.Tensor, x2: torch.Tensor, with_bias: bool) -> str:
    """'hip' (split-K MFMA kernel, rq_linear_wgrad) or 'lib' (library GEMM g^T x)."""
    from . import gemm_tuning
    N = g2.shape[0]
    if N < WGRAD_MIN_ROWS or (N <= WGRAD_TUNED_LIB_MAX_ROWS and gemm_tuning.is_enabled()):
        return "lib"
    return "hip"


def matmul_high() -> bool:
    """True when fp32 matmuls may run at PyTorch's 'high' precision (split-bf16), which the
    reference selects at import (modules/rqvae.py:19, modules/model.py:27); 'highest' keeps the
    exact-fp32 path."""
    return torch.get_float32_matmul_precision() != "highest"


def gemm_bf16x3(a: torch.Tensor, a_kcontig: bool, b: torch.Tensor, b_kcontig: bool, M: int, N: int, K: int,
                out: torch.Tensor = None) -> torch.Tensor:
    """C (M, N) = sum_k A(m, k) B(n, k) in split-bf16 ('high' fp32 matmul precision, rq_gemm_bf16x3).
    A(m, k) is a[m, k] for a k-contiguous a (M, K), else a[k, m] for a (K, M); B likewise."""
    require_gpu(a, b, what="gemm_bf16x3")
    a = a.contiguous()
    b = b.contiguous()
    lda, ldb = a.shape[1], b.shape[1]
    C = out if out is not None else torch.empty((M, N), device=a.device, dtype=torch.float32)
    nbytes = _x3_workspace(M, N, K)
    ws = torch.empty((nbytes,), device=a.device, dtype=torch.uint8) if nbytes else None
    args = ("rq_gemm_bf16x3", ptr(a), lda, int(a_kcontig), ptr(b), ldb, int(b_kcontig), M, N, K, ptr(C), N, ptr(ws),
            nbytes, stream_handle(a.device))
    if TIMER.wants("gemm_bf16x3"):
        TIMER.around(f"gemm_bf16x3:{M}x{N}x{K}:{int(a_kcontig)}{int(b_kcontig)}", call, *args)
    else:
        call(*args)
    return C


def linear_fwd_high(x2: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """y = x2 W^T (rows, O) at 'high' precision."""
    O, I = weight.shape
    return gemm_bf16x3(x2, True, weight, True, x2.shape[0], O, I)


def linear_dgrad_high(g2: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """gx = g2 W (rows, I) at 'high' precision."""
    O, I = weight.shape
    return gemm_bf16x3(g2, True, weight, False, g2.shape[0], I, O)


def linear_wgrad_high(g2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    """dW = g2^T x2 (O, I) at 'high' precision (split-K over the rows, fixed-order reduction)."""
    return gemm_bf16x3(g2, False, x2, False, g2.shape[1], x2.shape[1], g2.shape[0])


class Split(NamedTuple):
    """x = hi + lo: two bf16 planes of x's shape, the operand form the split-bf16 GEMM consumes
    without converting (rq_split_bf16x3, or a GEMM epilogue that emits it)."""
    hi: torch.Tensor
    lo: torch.Tensor


def split_bf16x3(x: torch.Tensor) -> Split:
    require_gpu(x, what="split_bf16x3")
    x = x.contiguous()
    hi = torch.empty(x.shape, device=x.device, dtype=torch.bfloat16)
    lo = torch.empty(x.shape, device=x.device, dtype=torch.bfloat16)
    call("rq_split_bf16x3", ptr(x), x.numel(), ptr(hi), ptr(lo), stream_handle(x.device))
    return Split(hi, lo)


_SPLIT_MULTI_MAX = 48   # rq_split_bf16x3_multi's tensor table


def split_bf16x3_many(xs, outs=None) -> list:
    """split_bf16x3 of up to 48 tensors in one launch (rq_split_bf16x3_multi); `outs`: per tensor a
    contiguous Split of its shape to write (e.g. row blocks of one stacked pair of planes), or None."""
    import ctypes
    xs = [x.contiguous() for x in xs]
    if not xs:
        return []
    require_gpu(*xs, what="split_bf16x3_many")
    assert len(xs) <= _SPLIT_MULTI_MAX
    outs = outs or [None] * len(xs)
    out = [o if o is not None else Split(torch.empty(x.shape, device=x.device, dtype=torch.bfloat16),
                                         torch.empty(x.shape, device=x.device, dtype=torch.bfloat16))
           for x, o in zip(xs, outs)]
    assert all(o.hi.shape == x.shape and o.hi.is_contiguous() and o.lo.is_contiguous() for x, o in zip(xs, out))
    n = len(xs)
    P = ctypes.c_void_p * n
    call("rq_split_bf16x3_multi", n, P(*[x.data_ptr() for x in xs]), (ctypes.c_int64 * n)(*[x.numel() for x in xs]),
         P(*[o.hi.data_ptr() for o in out]), P(*[o.lo.data_ptr() for o in out]), stream_handle(xs[0].device))
    return out


_WSPLIT = {}   # id(weight) -> (Split, weight): the current forward's pre-split weights (weight_split_scope)
_WSTACK = {}   # ids of a weight stack -> (stacked Split, weights): their planes as row blocks of one pair


def _splittable(p) -> bool:
    return p.is_cuda and p.dtype == torch.float32 and p.dim() == 2 and p.shape[0] % 8 == 0 and p.shape[1] % 8 == 0


@contextlib.contextmanager
def weight_split_scope(params, stacks=()):
    """Split every GEMM weight among `params` (2-D fp32 device tensors, both dims % 8) once, in a few
    multi-tensor launches (rq_split_bf16x3_multi, 48 per launch), for the forward run inside the
    scope: the Linear / MLP ops take their split operand from here instead of one split launch per
    weight per call (the decoder: ~32 -> 3 launches per step). `stacks`: lists of equal-shape weights
    whose planes are written as row blocks of one stacked pair (stacked_split: the hoisted cross-attention
    K/V projection's concatenated weight, without a cat and a split launch of its own). Only at matmul
    precision 'high'."""
    ws = [p for p in params if _splittable(p)] if matmul_high() else []
    prev, prev_st = dict(_WSPLIT), dict(_WSTACK)
    dst = {}
    with torch.no_grad():
        for st in (stacks if ws else ()):
            st = list(st)
            if not st or not all(_splittable(w) and w.shape == st[0].shape for w in st):
                continue
            O, I = st[0].shape
            big = Split(torch.empty((len(st) * O, I), device=st[0].device, dtype=torch.bfloat16),
                        torch.empty((len(st) * O, I), device=st[0].device, dtype=torch.bfloat16))
            for j, w in enumerate(st):
                dst[id(w)] = Split(big.hi[j * O:(j + 1) * O], big.lo[j * O:(j + 1) * O])
            _WSTACK[tuple(id(w) for w in st)] = (big, st)
        ids = {id(w) for w in ws}
        ws = ws + [w for w in (w for st in stacks for w in st) if id(w) in dst and id(w) not in ids]
        for i in range(0, len(ws), _SPLIT_MULTI_MAX):
            chunk = ws[i:i + _SPLIT_MULTI_MAX]
            for w, sp in zip(chunk, split_bf16x3_many([w.detach() for w in chunk], [dst.get(id(w)) for w in chunk])):
                _WSPLIT[id(w)] = (sp, w)
    try:
        yield
    finally:
        _WSPLIT.clear()
        _WSPLIT.update(prev)
        _WSTACK.clear()
        _WSTACK.update(prev_st)


def stacked_split(weights) -> Split:
    """The split planes of cat(weights, 0): the weight_split_scope's stacked pair when it registered this
    stack, else a cat and one split launch."""
    e = _WSTACK.get(tuple(id(w) for w in weights))
    if e is not None and all(a is b for a, b in zip(e[1], weights)):
        return e[0]
    return split_bf16x3(torch.cat([w.detach() for w in weights], 0))


def split_weight(w: torch.Tensor) -> Split:
    """w's split planes: from the enclosing weight_split_scope, else one split launch."""
    e = _WSPLIT.get(id(w))
    return e[0] if e is not None and e[1] is w else split_bf16x3(w)


def split_weights(weights) -> list:
    """split_weight of each, with the uncached ones split in one multi-tensor launch."""
    out = [(_WSPLIT.get(id(w)) or (None, None)) for w in weights]
    miss = [i for i, (sp, w) in enumerate(out) if sp is None or w is not weights[i]]
    res = [sp for sp, _ in out]
    for j in range(0, len(miss), _SPLIT_MULTI_MAX):
        idx = miss[j:j + _SPLIT_MULTI_MAX]
        for i, sp in zip(idx, split_bf16x3_many([weights[i] for i in idx])):
            res[i] = sp
    return res


def _operand_tensors(t):
    return [t.hi, t.lo] if isinstance(t, Split) else [t]


def _wgrad_into(weight, g, g_kc: bool, inp, inp_kc: bool, O: int, I: int, rows: int):
    """dW = g^T inp for `weight` (split-bf16 GEMM): added straight into weight's flat gradient bucket
    when dp.GradBuckets owns one (returns None: autograd must not accumulate it again), else a new
    (O, I) tensor for autograd. (A side stream for these was measured slower inside the captured steps:
    Amazon 6.16 -> 6.38-6.43 ms, profiles/r03 — one stream it is.)"""
    from . import dp
    sink = dp.direct_grad(weight)
    if sink is None:
        return gemm_x3(g, g_kc, inp, inp_kc, O, I, rows)
    gemm_x3(g, g_kc, inp, inp_kc, O, I, rows, out=sink, accumulate=True, defer=dp.defer_ok(weight))
    dp.direct_grad_done(weight)
    return None


def _wgrad_spec(weight, g, g_kc: bool, inp, inp_kc: bool, O: int, I: int, rows: int):
    """gemm_x3 keywords of dW = g^T inp for a paired launch with the data gradient (gemm_x3_pair), added
    straight into weight's flat gradient bucket when dp.GradBuckets owns one — or None when the GEMM
    policy asks for separate launches (GEMM_NO_PAIR: _wgrad_into)."""
    from . import dp
    if not _pairing():
        return None
    sink = dp.direct_grad(weight)
    spec = dict(a=g, a_kcontig=g_kc, b=inp, b_kcontig=inp_kc, M=O, N=I, K=rows)
    if sink is not None:
        spec.update(out=sink, accumulate=True, defer=dp.defer_ok(weight))
    return spec


def _wgrad_result(weight, spec, result):
    """What autograd gets for weight after a paired launch: None when the gradient went into its bucket."""
    if spec.get("accumulate"):
        from . import dp
        dp.direct_grad_done(weight)
        return None
    return result


# Kernel policy of the split-bf16 GEMM calls (rq_gemm_desc.flags, RQ_GEMM_* in include/rqvae_hip.h; 0 = the
# time model's choice): set only by kernel-vs-kernel tests and A/B probes through gemm_policy(); the library
# itself keeps no state — the flags travel in every descriptor.
GEMM_ONLY_128, GEMM_ONLY_64, GEMM_FORCE_WIDE, GEMM_NO_WIDE, GEMM_MASKED, GEMM_NO_PAIR = 1, 2, 4, 8, 16, 32
GEMM_SPLIT_SHIFT, GEMM_SPLIT_MASK = 16, 0xFFF


def gemm_split(S: int) -> int:
    """RQ_GEMM_SPLIT(S): policy bits forcing S split-K chunks on the kernel the other bits / the planner pick."""
    return (int(S) & GEMM_SPLIT_MASK) << GEMM_SPLIT_SHIFT
_GEMM_POLICY = {"flags": 0}


class _Policy:
    def __init__(self, store, flags):
        self.store, self.flags = store, int(flags)

    def __enter__(self):
        self.prev = self.store["flags"]
        self.store["flags"] = self.flags
        return self

    def __exit__(self, *exc):
        self.store["flags"] = self.prev
        return False


def gemm_policy(flags: int) -> _Policy:
    """`with ops.gemm_policy(ops.GEMM_ONLY_64): ...` — every split-bf16 GEMM launched inside (forward and
    the backward run inside the block) carries these RQ_GEMM_* flags."""
    return _Policy(_GEMM_POLICY, flags)


def _pairing() -> bool:
    return not (_GEMM_POLICY["flags"] & GEMM_NO_PAIR)


EPI_STORE, EPI_SILU_FWD, EPI_SILU_BWD, EPI_ADD = 0, 1, 2, 3
_X3_WS = {}


def _x3_workspace(M: int, N: int, K: int) -> int:
    """Split-K slab bytes of rq_gemm_bf16x3_run for a shape (host-only plan, memoised per shape)."""
    key = (M, N, K)
    nb = _X3_WS.get(key)
    if nb is None:
        nb = _X3_WS[key] = int(_lib.load().rq_gemm_bf16x3_workspace(M, N, K))
    return nb


class _X3Call(NamedTuple):
    """One prepared rq_gemm_bf16x3 call: its rq_gemm_desc field values, outputs and what to do after it."""
    fields: tuple
    C: torch.Tensor
    H: "Split"
    ws: torch.Tensor
    defer: bool
    key: str
    epilogue: int
    M: int
    N: int
    dev: torch.device


def _x3_setup(a, a_kcontig: bool, b, b_kcontig: bool, M: int, N: int, K: int, epilogue: int = EPI_STORE,
              Z: torch.Tensor = None, p: float = 0.0, seed: int = 0, out: torch.Tensor = None,
              accumulate: bool = False, defer: bool = False, flags: int = None) -> _X3Call:
    def desc(t):
        if isinstance(t, Split):
            return t.hi, t.lo, t.hi.shape[-1], 1
        if not (t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.shape[1] and t.stride(0) % 4 == 0 and
                t.data_ptr() % 16 == 0):
            t = t.contiguous()   # row-strided 2-D views (column blocks of a wider buffer) are read in place
        return t, None, t.stride(0) if t.dim() == 2 else t.shape[-1], 0
    ah, al, lda, asp = desc(a)
    bh, bl, ldb, bsp = desc(b)
    dev = ah.device
    if accumulate and (epilogue != EPI_STORE or out is None):
        raise RqHipError("gemm_x3: accumulate needs the plain epilogue and an output tensor")
    if out is not None and not (out.is_contiguous() and out.dtype == torch.float32 and out.shape == (M, N)):
        raise RqHipError(f"gemm_x3: out must be a contiguous fp32 ({M}, {N}) tensor")
    C = None if epilogue == EPI_SILU_BWD else (out if out is not None else
                                                torch.empty((M, N), device=dev, dtype=torch.float32))
    H = None
    if epilogue in (EPI_SILU_FWD, EPI_SILU_BWD):
        H = Split(torch.empty((M, N), device=dev, dtype=torch.bfloat16),
                  torch.empty((M, N), device=dev, dtype=torch.bfloat16))
    flags = _GEMM_POLICY["flags"] if flags is None else int(flags)   # per-call override (probes)
    nbytes = _x3_workspace(M, N, K)
    forced = (flags >> GEMM_SPLIT_SHIFT) & GEMM_SPLIT_MASK
    if forced > 1:   # a forced split count: its slabs (the library sizes only the planner's)
        nbytes = max(nbytes, forced * M * N * 4)
    ws = torch.empty((nbytes,), device=dev, dtype=torch.uint8) if nbytes else None
    defer = bool(defer and accumulate and nbytes)
    if defer and C.data_ptr() in _DEFER["outs"]:
        flush_reductions()   # a pending reduction into the same output must land first
    fields = (ptr(ah), ptr(al), lda, int(a_kcontig), ptr(bh), ptr(bl), ldb, int(b_kcontig), M, N, K, ptr(C), N,
              int(epilogue), ptr(Z), ptr(H.hi if H else None), ptr(H.lo if H else None), N, float(p), int(seed),
              int(accumulate), int(defer), ptr(ws), nbytes, flags, 0)
    key = f"gemm_bf16x3:{M}x{N}x{K}:{int(a_kcontig)}{int(b_kcontig)}{asp}{bsp}{epilogue}{int(accumulate)}"
    return _X3Call(fields, C, H, ws, defer, key, epilogue, M, N, dev)


def _x3_result(c: _X3Call, splits: int):
    if c.defer and splits > 0:
        _defer_push(c.ws, c.C, c.M * c.N, splits, 0)
    if c.epilogue in (EPI_STORE, EPI_ADD):
        return c.C
    return (c.C, c.H) if c.epilogue == EPI_SILU_FWD else c.H


def gemm_x3(a, a_kcontig: bool, b, b_kcontig: bool, M: int, N: int, K: int, epilogue: int = EPI_STORE,
            Z: torch.Tensor = None, p: float = 0.0, seed: int = 0, out: torch.Tensor = None,
            accumulate: bool = False, defer: bool = False):
    """Split-bf16 GEMM with pre-split operands and fused epilogues (rq_gemm_bf16x3_run). a / b: fp32
    tensors or Split. Returns C (EPI_STORE; EPI_ADD: A B^T + Z), (C, H) (EPI_SILU_FWD: C = z,
    H = split(Dropout(SiLU(z)))) or H (EPI_SILU_BWD: split(SiLU'(Z) * Dropout(A B^T))); H is a Split
    of shape (M, N). `out`: the (M, N) contiguous fp32 destination of C; `accumulate` (EPI_STORE
    only): out += A B^T; with `defer` a split call's slab reduction joins the pending batch
    (flush_reductions) instead of running now."""
    import ctypes
    c = _x3_setup(a, a_kcontig, b, b_kcontig, M, N, K, epilogue, Z, p, seed, out, accumulate, defer)
    splits = ctypes.c_int(0)
    d = _desc_type()(*c.fields)
    args = ("rq_gemm_bf16x3_run", ctypes.byref(d), ctypes.byref(splits), stream_handle(c.dev))
    if TIMER.wants("gemm_bf16x3"):
        TIMER.around(c.key, call, *args)
    else:
        call(*args)
    return _x3_result(c, splits.value)


_DESC = {}


def _desc_type():
    import ctypes
    t = _DESC.get("t")
    if t is None:
        P, I64, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int

        class Desc(ctypes.Structure):   # rq_gemm_desc (include/rqvae_hip.h)
            _fields_ = [("A", P), ("A_lo", P), ("lda", I64), ("a_kcontig", I), ("B", P), ("B_lo", P), ("ldb", I64),
                        ("b_kcontig", I), ("M", I64), ("N", I64), ("K", I64), ("C", P), ("ldc", I64),
                        ("epilogue", I), ("Z", P), ("H_hi", P), ("H_lo", P), ("ldh", I64), ("p", ctypes.c_float),
                        ("seed", ctypes.c_uint64), ("accumulate", I), ("defer", I), ("workspace", P),
                        ("ws_bytes", ctypes.c_size_t), ("flags", I), ("reserved", I)]
        t = _DESC["t"] = Desc
    return t


def gemm_x3_pair(spec1: dict, spec2: dict):
    """Two independent gemm_x3 calls (keyword dicts of gemm_x3's arguments: a, a_kcontig, b, b_kcontig, M,
    N, K, ...) through rq_gemm_bf16x3_pair — one launch where a paired instantiation exists (a Linear's data
    and weight gradients), results identical to two gemm_x3 calls. Returns (result1, result2)."""
    import ctypes
    c1 = _x3_setup(**spec1)
    c2 = _x3_setup(**spec2)
    D = _desc_type()
    arr = (D * 2)(D(*c1.fields), D(*c2.fields))
    splits = (ctypes.c_int * 2)(0, 0)
    if TIMER.wants("gemm_bf16x3"):
        TIMER.around(f"gemm_pair:{c1.key}+{c2.key}", call, "rq_gemm_bf16x3_pair", arr, splits, stream_handle(c1.dev))
    else:
        call("rq_gemm_bf16x3_pair", arr, splits, stream_handle(c1.dev))
    return _x3_result(c1, splits[0]), _x3_result(c2, splits[1])


_PAIR_RESPLIT = True   # False: a paired weight gradient keeps the split count it is planned with alone (A/B)
_RESPLIT_CACHE = {}


def _spec_key(sp: dict):
    a, b = sp["a"], sp["b"]
    return (int(sp["M"]), int(sp["N"]), int(sp["K"]), bool(sp["a_kcontig"]), bool(sp["b_kcontig"]),
            isinstance(a, Split), isinstance(b, Split), int(sp.get("epilogue", EPI_STORE)))


def _bwd_pair(dspec: dict, wspec: dict):
    """gemm_x3_pair of a Linear's data gradient (dspec) and weight gradient (wspec) with the weight gradient's
    split count chosen for the PAIR: where the data gradient alone leaves resident slots idle (128-tile
    kernel, unsplit), the weight gradient's k chunks are sized like the data gradient's K (S = ceil(rows / K_d))
    when that is fewer slabs than its own plan and the pair still spans more than one round of workgroups —
    equal-length workgroups instead of a tail of short ones, and fewer slabs (measured on the paired launches of
    the decoder's 11k-row qkv / MLP-up layers: 152 -> 127 and 93 -> 85 us, tools/pair_split_probe.py)."""
    if _PAIR_RESPLIT and _GEMM_POLICY["flags"] == 0 and wspec.get("flags") is None and \
            int(wspec.get("epilogue", EPI_STORE)) == EPI_STORE:
        key = (_spec_key(dspec), _spec_key(wspec))
        S = _RESPLIT_CACHE.get(key)
        if S is None:
            S = 0
            kd, sd = gemm_x3_choice(*key[0][:3], key[0][5], key[0][6], key[0][3], key[0][4], key[0][7])
            kw, sw = gemm_x3_choice(*key[1][:3], key[1][5], key[1][6], key[1][3], key[1][4], EPI_STORE)
            if kd == "x3" and kw == "x3" and sd == 1 and sw > 1:
                slots = 2 * torch.cuda.get_device_properties(dspec["a"].hi.device if isinstance(dspec["a"], Split)
                                                             else dspec["a"].device).multi_processor_count
                w1 = -(-int(dspec["M"]) // 128) * -(-int(dspec["N"]) // 128)
                t2 = -(-int(wspec["M"]) // 128) * -(-int(wspec["N"]) // 128)
                s_bal = -(-int(wspec["K"]) // int(dspec["K"]))
                if w1 < slots and 1 < s_bal < sw and w1 + t2 * s_bal > slots:
                    S = s_bal
            _RESPLIT_CACHE[key] = S
        if S:
            wspec = dict(wspec, flags=gemm_split(S))
    return gemm_x3_pair(dspec, wspec)


# Deferred partial reductions (rq_reduce_partials): split-K weight-gradient slabs and RMSNorm weight-
# gradient partials that accumulate into flat gradient buckets wait here and run as ONE launch (per 48)
# at the next flush — before a bucket's exchange, in GradBuckets.finish / synchronize / zero_grad, and at
# the end of a captured step — instead of one reduction launch each (~40 per decoder step).
_DEFER = {"pending": [], "outs": set()}


def _defer_push(ws: torch.Tensor, out: torch.Tensor, n: int, S: int, layout: int):
    _DEFER["pending"].append((ws, out, int(n), int(S), int(layout), torch.cuda.current_stream(out.device)))
    _DEFER["outs"].add(out.data_ptr())


# Deferred embedding-table gradients: each table's (rows, keys) waits here when its weight's gradient lives
# in a flat bucket; the flush sums every waiting table in ONE segmented-sum chain (rq_segment_sum_multi) and
# adds each table's slice into its bucket view through the batched reduction above — instead of one
# 6-launch chain plus an accumulate per table (the decoder's 4-6 tables: ~30 launches a step).
_EMB = {"pending": [], "on": True}
_EMB_KMAX = 4096          # rq_segment_sum's key limit, per batch
_EMB_SRC_MAX = 16         # sources per rq_segment_sum_multi call


def emb_defer_enable(enable) -> bool:
    """Batched (deferred) embedding-table gradients on/off (A/B); returns the previous setting."""
    prev = _EMB["on"]
    _EMB["on"] = bool(enable)
    return prev


def _emb_grad(weight, g: torch.Tensor, keys: torch.Tensor, K: int, padding_idx):
    """An embedding table's gradient: deferred into its flat bucket view (returns None) when the owner
    GradBuckets batches reductions, else the (K, E) tensor from _table_grad."""
    from . import dp
    E = g.shape[-1]
    if _EMB["on"] and E % 4 == 0 and 4 <= E <= 1024 and K <= _EMB_KMAX and weight is not None \
            and dp.defer_ok(weight):
        sink = dp.direct_grad(weight)
        if sink is not None and sink.is_contiguous() and sink.data_ptr() % 16 == 0 \
                and sink.dtype == torch.float32 and sink.data_ptr() not in _DEFER["outs"]:
            pad = -2 if padding_idx is None else int(padding_idx) % K
            _EMB["pending"].append((g.contiguous().float(), keys.contiguous().to(torch.int64), int(K), pad, sink,
                                    torch.cuda.current_stream(g.device)))
            _DEFER["outs"].add(sink.data_ptr())
            dp.direct_grad_done(weight)
            return None
    return _table_grad(g, keys, K, padding_idx)


def _rows_grad(weight, rows: torch.Tensor, K: int):
    """The gradient of a table whose first rows.shape[0] rows were each gathered once (keys 0..n-1): `rows`
    itself — deferred as an add into the table's flat bucket prefix when its owner batches reductions
    (returns None), else the (K, E) tensor. The segmented sum of such keys is each row alone, so this is
    _emb_grad's result without the sort and sum."""
    from . import dp
    n, E = rows.shape
    if weight is not None and dp.defer_ok(weight):
        sink = dp.direct_grad(weight)
        if sink is not None and sink.is_contiguous() and sink.data_ptr() % 16 == 0 and rows.is_contiguous() \
                and rows.data_ptr() % 16 == 0 and (n * E) % 4 == 0 and sink.data_ptr() not in _DEFER["outs"]:
            _defer_push(rows, sink, n * E, 1, 0)
            dp.direct_grad_done(weight)
            return None
    out = rows.new_zeros((K, E))
    out[:n] = rows
    return out


def _flush_embeddings() -> None:
    """Sum the waiting tables (grouped by row width, <= 16 sources and <= 4096 keys a call) and queue each
    table's slice as an accumulate-into-sink entry of the batched reduction."""
    import ctypes
    pend, _EMB["pending"] = _EMB["pending"], []
    groups, cur_key = [], None
    for e in sorted(pend, key=lambda e: e[0].shape[-1]):
        E = e[0].shape[-1]
        if not groups or cur_key != E or len(groups[-1]) == _EMB_SRC_MAX or \
                sum(x[2] for x in groups[-1]) + e[2] > _EMB_KMAX:
            groups.append([])
            cur_key = E
        groups[-1].append(e)
    L = _lib.load()
    for grp in groups:
        dev = grp[0][0].device
        cs = torch.cuda.current_stream(dev)
        for e in grp:
            if e[5] != cs:
                cs.wait_stream(e[5])
        n, E = len(grp), grp[0][0].shape[-1]
        I64, P = ctypes.c_int64 * n, ctypes.c_void_p * n
        rows_n = I64(*[e[0].shape[0] for e in grp])
        Ks = I64(*[e[2] for e in grp])
        nbytes = L.rq_segment_sum_multi_workspace(n, rows_n, Ks, E)
        ws = torch.empty((nbytes,), device=dev, dtype=torch.uint8)
        out = torch.empty((sum(e[2] for e in grp), E), device=dev, dtype=torch.float32)
        TIMER.around("emb_segsum", call, "rq_segment_sum_multi", n, P(*[e[0].data_ptr() for e in grp]),
                     P(*[e[1].data_ptr() for e in grp]), rows_n, Ks, I64(*[e[3] for e in grp]), E, ptr(out),
                     ptr(ws), nbytes, stream_handle(dev))
        base = 0
        for e in grp:
            _defer_push(out[base:base + e[2]], e[4], e[2] * E, 1, 0)
            base += e[2]


def flush_reductions() -> None:
    """Run every pending deferred reduction (stream-ordered after their producers: side-stream weight
    grads are joined first) and release their partial buffers."""
    if _EMB["pending"]:
        _flush_embeddings()
    pend = _DEFER["pending"]
    if not pend:
        return
    import ctypes
    dev = pend[0][1].device
    cur = torch.cuda.current_stream(dev)
    for ws, out, _, _, _, st in pend:
        if st != cur:
            cur.wait_stream(st)
            ws.record_stream(cur)
    n = len(pend)
    P = ctypes.c_void_p * n
    TIMER.around("reduce_partials", call, "rq_reduce_partials", n, P(*[e[0].data_ptr() for e in pend]),
                 P(*[e[1].data_ptr() for e in pend]), (ctypes.c_int64 * n)(*[e[2] for e in pend]),
                 (ctypes.c_int * n)(*[e[3] for e in pend]), (ctypes.c_int * n)(*[e[4] for e in pend]),
                 (ctypes.c_int * n)(*([1] * n)), stream_handle(dev))
    _DEFER["pending"] = []
    _DEFER["outs"] = set()


def pending_reductions() -> int:
    return len(_DEFER["pending"]) + len(_EMB["pending"])


def gemm_x3_choice(M: int, N: int, K: int, a_split: bool, b_split: bool, a_kcontig: bool, b_kcontig: bool,
                   epilogue: int = EPI_STORE):
    """(kernel, splits) rq_gemm_bf16x3_run picks for a call under the current gemm_policy: kernel 'wide'
    (256 x 256 tiles, LDS-DMA, both operands split), 'x3' (128 x 128 tiles) or 'x3s' (its 64 x 64-tile
    form); 'none' for an empty or invalid shape. Host-only (rq_gemm_bf16x3_plan)."""
    import ctypes
    d = _desc_type()(A_lo=16 if a_split else None, lda=K if a_kcontig else M, a_kcontig=int(a_kcontig),
                     B_lo=16 if b_split else None, ldb=K if b_kcontig else N, b_kcontig=int(b_kcontig), M=M, N=N, K=K,
                     ldc=N, epilogue=int(epilogue), ldh=N, flags=_GEMM_POLICY["flags"])
    s_ = ctypes.c_int(0)
    k = _lib.load().rq_gemm_bf16x3_plan(ctypes.byref(d), ctypes.byref(s_))
    return {1: "wide", 2: "x3s", 0: "x3"}.get(k, "none"), int(s_.value)


def mlp_fusable(x: torch.Tensor, weights) -> bool:
    """The fused chain needs fp32 device tensors, split-operand widths (every dim % 8) and rows."""
    return (x.is_cuda and x.dtype == torch.float32 and x.numel() > 0 and
            all(w.dtype == torch.float32 and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0 for w in weights))


def _presplit_input(rows: int, weights, n_layers: int) -> bool:
    """Split the fp32 chain input once up front when that moves the first layer's forward (and its
    weight grad, which reads the same operand) onto the wide LDS-DMA kernel, which takes split
    operands only: at the RQ-VAE batch the split (one HBM pass) costs less than the 128-tile kernel's
    on-the-fly conversion loses (ML-32M encoder layer 0: 235 -> ~150 us forward, 178 -> ~145 us wgrad)."""
    O, I = weights[0].shape
    epi = EPI_SILU_FWD if n_layers > 1 else EPI_STORE
    return gemm_x3_choice(rows, O, I, True, True, True, True, epi)[0] == "wide"


def _mlp_forward(a, wsp, rows: int, p: float, seeds, residual=None, p_out: float = 0.0, seed_out: int = 0):
    """The chain's forward GEMMs from input a (fp32 or Split): (out fp32, zs, hs). With `residual`
    (rows, O) the last GEMM's epilogue returns residual + Dropout_{p_out}(out) instead."""
    n = len(wsp)
    zs, hs = [], []
    out = None
    for i, w in enumerate(wsp):
        O, I = w.hi.shape
        if i < n - 1:
            z, h = gemm_x3(a, True, w, True, rows, O, I, EPI_SILU_FWD, p=p, seed=seeds[i])
            zs.append(z)
            hs.append(h)
            a = h
        elif residual is not None:
            out = gemm_x3(a, True, w, True, rows, O, I, EPI_ADD, Z=residual, p=p_out, seed=seed_out)
        else:
            out = gemm_x3(a, True, w, True, rows, O, I)
    return out, zs, hs


def _mlp_backward(gcur, x_in, wsp, zs, hs, rows: int, p: float, seeds, need_w, need_x: bool, weights):
    """The chain's backward from the output grad gcur (fp32 or Split): (dx fp32 or None, [dW]); a
    weight grad added straight into its flat gradient bucket comes back as None (_wgrad_into)."""
    n = len(wsp)
    dws = [None] * n
    dx = None
    for i in reversed(range(n)):
        O, I = wsp[i].hi.shape
        inp = x_in if i == 0 else hs[i - 1]
        if i > 0:
            dspec = dict(a=gcur, a_kcontig=True, b=wsp[i], b_kcontig=False, M=rows, N=I, K=O, epilogue=EPI_SILU_BWD,
                         Z=zs[i - 1], p=p, seed=seeds[i - 1])
        elif need_x:
            dspec = dict(a=gcur, a_kcontig=True, b=wsp[0], b_kcontig=False, M=rows, N=I, K=O)
        else:
            dspec = None
        wspec = _wgrad_spec(weights[i], gcur, False, inp, False, O, I, rows) if need_w[i] else None
        if dspec is not None and wspec is not None:   # dW = g^T h_{i-1} and the data grad in one launch
            gnext, wres = _bwd_pair(dspec, wspec)
            dws[i] = _wgrad_result(weights[i], wspec, wres)
        else:
            if need_w[i]:
                dws[i] = _wgrad_into(weights[i], gcur, False, inp, False, O, I, rows)   # dW = g^T h_{i-1}
            gnext = gemm_x3(**dspec) if dspec is not None else None
        if i > 0:
            gcur = gnext
        elif need_x:
            dx = gnext
    return dx, dws


def _mlp_save(ctx, x_in, wsp, zs, hs):
    xs = list(x_in) if isinstance(x_in, Split) else [x_in]
    ctx.x_split = isinstance(x_in, Split)
    return [*xs, *[t for s_ in wsp for t in s_], *zs, *[t for h in hs for t in h]]


def _mlp_load(ctx, n: int, saved):
    k = 2 if ctx.x_split else 1
    x_in = Split(saved[0], saved[1]) if ctx.x_split else saved[0]
    wsp = [Split(saved[k + 2 * i], saved[k + 1 + 2 * i]) for i in range(n)]
    zs = list(saved[k + 2 * n:k + 2 * n + (n - 1)])
    hb = k + 2 * n + (n - 1)
    hs = [Split(saved[hb + 2 * i], saved[hb + 2 * i + 1]) for i in range(n - 1)]
    return x_in, wsp, zs, hs, hb + 2 * (n - 1)


def _mlp_prologue(x, p: float, weights):
    n = len(weights)
    x2 = x.reshape(-1, weights[0].shape[1]).contiguous()
    rows = x2.shape[0]
    wsp = split_weights(weights)
    seeds = [next_seed() if p > 0 else 0 for _ in range(n - 1)]
    x_in = split_bf16x3(x2) if _presplit_input(rows, weights, n) else x2
    return x_in, rows, wsp, seeds


class MLPFunction(torch.autograd.Function):
    """The whole bias-free Linear -> SiLU -> [Dropout] -> ... -> Linear chain of modules/encoder.py:7-36
    at 'high' matmul precision, as one autograd node. Each hidden layer is ONE GEMM launch whose
    epilogue keeps z (for SiLU') and emits h = Dropout(SiLU(z)) already split into bf16 planes, so
    the next layer's forward and this layer's weight grad read it without converting; backward
    mirrors it (the data-grad GEMM's epilogue applies SiLU' and the dropout mask and emits the
    split pre-activation grad). Weights are split once per call; a large fp32 input is split once
    too (_presplit_input). Replaces eager torch's Linear + SiLU + Dropout + mask kernels (forward)
    and their backward passes."""

    @staticmethod
    def forward(ctx, x, p: float, *weights):
        x_in, rows, wsp, seeds = _mlp_prologue(x, p, weights)
        out, zs, hs = _mlp_forward(x_in, wsp, rows, p, seeds)
        ctx.n, ctx.p, ctx.seeds, ctx.xshape, ctx.weights = len(weights), float(p), seeds, x.shape, weights
        ctx.save_for_backward(*_mlp_save(ctx, x_in, wsp, zs, hs))
        return out.view(*x.shape[:-1], weights[-1].shape[0])

    @staticmethod
    def backward(ctx, g):
        x_in, wsp, zs, hs, _ = _mlp_load(ctx, ctx.n, ctx.saved_tensors)
        rows = (x_in.hi if ctx.x_split else x_in).shape[0]
        gcur = g.reshape(rows, -1).contiguous()
        dx, dws = _mlp_backward(gcur, x_in, wsp, zs, hs, rows, ctx.p, ctx.seeds, ctx.needs_input_grad[2:],
                                ctx.needs_input_grad[0], ctx.weights)
        ctx.weights = None
        return (None if dx is None else dx.view(ctx.xshape), None, *dws)


def mlp_chain(x: torch.Tensor, weights, p: float = 0.0) -> torch.Tensor:
    """Fused Linear-SiLU-[Dropout]-...-Linear at 'high' precision (MLPFunction)."""
    return MLPFunction.apply(x, float(p), *weights)


class MLPResidualFunction(torch.autograd.Function):
    """h + Dropout_{p_out}(MLP(x)): the transformer block's feed-forward output (modules/transformer/
    model.py:76-82, `x + Dropout(MLP(RMSNorm(x)))`) as MLPFunction whose last GEMM epilogue adds the
    residual and applies the output dropout (the mask of the standalone dropout_add kernel, so the
    backward regenerates it with rq_dropout_bwd): one launch fewer per block than MLP + dropout_add."""

    @staticmethod
    def forward(ctx, x, h, p: float, p_out: float, *weights):
        x_in, rows, wsp, seeds = _mlp_prologue(x, p, weights)
        seed_out = next_seed()
        out, zs, hs = _mlp_forward(x_in, wsp, rows, p, seeds, residual=h.reshape(rows, -1).contiguous(),
                                   p_out=p_out, seed_out=seed_out)
        ctx.n, ctx.p, ctx.seeds, ctx.xshape, ctx.weights = len(weights), float(p), seeds, x.shape, weights
        ctx.p_out, ctx.seed_out = float(p_out), seed_out
        ctx.save_for_backward(*_mlp_save(ctx, x_in, wsp, zs, hs))
        return out.view(*x.shape[:-1], weights[-1].shape[0])

    @staticmethod
    def backward(ctx, g):
        x_in, wsp, zs, hs, _ = _mlp_load(ctx, ctx.n, ctx.saved_tensors)
        rows = (x_in.hi if ctx.x_split else x_in).shape[0]
        g2 = g.reshape(rows, -1).contiguous()
        gy = torch.empty_like(g2)
        call("rq_dropout_bwd", ptr(g2), g2.numel(), ctx.p_out, ctx.seed_out, ptr(gy), stream_handle(g2.device))
        dx, dws = _mlp_backward(gy, x_in, wsp, zs, hs, rows, ctx.p, ctx.seeds, ctx.needs_input_grad[4:],
                                ctx.needs_input_grad[0], ctx.weights)
        ctx.weights = None
        gh = g if ctx.needs_input_grad[1] else None
        return (None if dx is None else dx.view(ctx.xshape), gh, None, None, *dws)


def mlp_chain_residual(x: torch.Tensor, weights, p: float, h: torch.Tensor, p_out: float) -> torch.Tensor:
    """h + Dropout_{p_out}(MLP(x)) at 'high' precision in the chain's launches (MLPResidualFunction)."""
    return MLPResidualFunction.apply(x, h, float(p), float(p_out), *weights)


class MLPL2ReconFunction(torch.autograd.Function):
    """The RqVae decoder (modules/rqvae.py:145-148: MLP chain ending in l2norm, modules/encoder.py:34)
    fused with ReconstructionLoss (modules/loss.py:5-10): recon_b = |l2norm(MLP(e)_b) - x_b|^2 at
    'high' matmul precision. Same as MLPFunction followed by L2NormReconFunction, except that the
    output gradient comes already split, so the chain's last data-grad and weight-grad GEMMs take split
    operands (the wide kernel) without a conversion pass — and it is written by the forward's row pass
    for the batch-mean loss's g_recon = 1 / B (rq_l2norm_recon_fwd_grad; the backward's
    rq_l2norm_recon_bwd_fix recomputes any row whose g_recon differs, bitwise the unspeculated result).
    Gradients w.r.t. e and the weights (x is data)."""

    @staticmethod
    def forward(ctx, e, x, p: float, grad_mode: bool, *weights):
        x_in, rows, wsp, seeds = _mlp_prologue(e, p, weights)
        pre, zs, hs = _mlp_forward(x_in, wsp, rows, p, seeds)
        x2 = x.reshape(rows, -1).contiguous()
        C = pre.shape[1]
        recon = torch.empty((rows,), device=pre.device, dtype=torch.float32)
        norms = torch.empty((rows,), device=pre.device, dtype=torch.float32)
        ctx.g, ctx.gs = None, 0.0
        if grad_mode and any(ctx.needs_input_grad):
            # the batch-mean loss (loss_means) hands every row g_recon = 1 / B: its split gradient is written
            # in this pass over pre and x, and the backward only checks g_recon (rq_l2norm_recon_bwd_fix)
            ctx.gs = float(torch.tensor(1.0, dtype=torch.float32) / rows)
            ctx.g = Split(torch.empty((rows, C), device=pre.device, dtype=torch.bfloat16),
                          torch.empty((rows, C), device=pre.device, dtype=torch.bfloat16))
            call("rq_l2norm_recon_fwd_grad", ptr(pre), ptr(x2), rows, C, ptr(recon), ptr(norms), ctx.gs,
                 ptr(ctx.g.hi), ptr(ctx.g.lo), stream_handle(pre.device))
        else:
            call("rq_l2norm_recon_fwd", ptr(pre), ptr(x2), rows, C, ptr(recon), ptr(norms), stream_handle(pre.device))
        ctx.n, ctx.p, ctx.seeds, ctx.eshape, ctx.weights = len(weights), float(p), seeds, e.shape, weights
        ctx.save_for_backward(*_mlp_save(ctx, x_in, wsp, zs, hs), pre, x2, norms)
        return recon.view(e.shape[:-1])

    @staticmethod
    def backward(ctx, g_recon):
        x_in, wsp, zs, hs, k = _mlp_load(ctx, ctx.n, ctx.saved_tensors)
        pre, x2, norms = ctx.saved_tensors[k:k + 3]
        rows, C = pre.shape
        g_recon = g_recon.reshape(rows)
        if ctx.g is not None:   # the forward's planes, rows with another g_recon recomputed
            g, ctx.g = ctx.g, None
            uniform = g_recon.stride(0) == 0   # the mean's expand: one value for every row
            gr = g_recon if uniform else g_recon.contiguous()
            call("rq_l2norm_recon_bwd_fix", ptr(pre), ptr(x2), ptr(norms), ptr(gr), 0 if uniform else 1, rows, C,
                 ctx.gs, ptr(g.hi), ptr(g.lo), stream_handle(pre.device))
        else:   # a second backward through the same graph: the planes were handed out already
            g = Split(torch.empty((rows, C), device=pre.device, dtype=torch.bfloat16),
                      torch.empty((rows, C), device=pre.device, dtype=torch.bfloat16))
            call("rq_l2norm_recon_bwd_split", ptr(pre), ptr(x2), ptr(norms), ptr(g_recon.contiguous()), rows, C,
                 ptr(g.hi), ptr(g.lo), stream_handle(pre.device))
        de, dws = _mlp_backward(g, x_in, wsp, zs, hs, rows, ctx.p, ctx.seeds, ctx.needs_input_grad[4:],
                                ctx.needs_input_grad[0], ctx.weights)
        ctx.weights = None
        return (None if de is None else de.view(ctx.eshape), None, None, None, *dws)


def mlp_l2norm_recon(e: torch.Tensor, x: torch.Tensor, weights, p: float = 0.0) -> torch.Tensor:
    """recon_b = |l2norm(MLP(e)_b) - x_b|^2 (MLPL2ReconFunction); fp32 device tensors, split-operand
    widths (mlp_fusable), x of the chain's output width."""
    require_gpu(e, x, what="mlp_l2norm_recon")
    return MLPL2ReconFunction.apply(e, x, float(p), torch.is_grad_enabled(), *weights)


class LinearFunction(torch.autograd.Function):
    """y = x W^T + b. At matmul precision 'high' (the reference's setting) the forward, data and
    weight gradients all run on the split-bf16 MFMA GEMM (rq_gemm_bf16x3). At 'highest': the
    forward and data gradient on the fp32 library GEMM (hipBLASLt) and the weight / bias gradient
    on rq_linear_wgrad (a reduction over the whole batch, where the library leaves CUs idle)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.weight = weight
        ctx.has_bias = bias is not None
        ctx.high = matmul_high()
        O, I = weight.shape
        ctx.wsp = None
        if ctx.high and x.numel() > 0:
            x2 = x.reshape(-1, I)
            if I % 8 == 0:   # split the weight once: forward and data grad read it without converting
                ctx.wsp = split_weight(weight)
                y = gemm_x3(x2, True, ctx.wsp, True, x2.shape[0], O, I)
            else:
                y = linear_fwd_high(x2, weight)
            if bias is not None:
                y += bias
            return y.view(*x.shape[:-1], O)
        return torch.nn.functional.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        O, I = weight.shape
        g2 = g.reshape(-1, O)
        gx = dW = db = None
        high = ctx.high and g2.shape[0] > 0
        if (high and ctx.wsp is not None and ctx.needs_input_grad[0] and ctx.needs_input_grad[1] and
                not ctx.has_bias):
            wspec = _wgrad_spec(ctx.weight, g2.contiguous(), False, x.reshape(-1, I).contiguous(), False, O, I,
                                g2.shape[0])
            if wspec is not None:   # data and weight gradient in one launch
                gx, wres = _bwd_pair(dict(a=g2, a_kcontig=True, b=ctx.wsp, b_kcontig=False, M=g2.shape[0], N=I,
                                             K=O), wspec)
                dW = _wgrad_result(ctx.weight, wspec, wres)
                ctx.wsp = ctx.weight = None
                return gx.view(x.shape), dW, None
        if ctx.needs_input_grad[0]:
            if high and ctx.wsp is not None:
                gx = gemm_x3(g2, True, ctx.wsp, False, g2.shape[0], I, O).view(x.shape)
            else:
                gx = (linear_dgrad_high(g2, weight) if high else g2 @ weight).view(x.shape)
        ctx.wsp = None
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            x2 = x.reshape(-1, I)
            if high:
                if ctx.needs_input_grad[1]:
                    dW = _wgrad_into(ctx.weight, g2.contiguous(), False, x2.contiguous(), False, O, I, g2.shape[0])
                db = g2.sum(0) if ctx.has_bias else None
            elif _wgrad_choice(g2, x2, ctx.has_bias) == "hip":
                dW, db = linear_wgrad(g2, x2, ctx.has_bias)
            else:   # library GEMM: small row counts, or measured faster for this shape
                dW = g2.t() @ x2
                db = g2.sum(0) if ctx.has_bias else None
        ctx.weight = None
        return gx, dW, db if ctx.has_bias else None


def _linear_bwd_high(x, g, weight, wsp, need_x: bool, need_w: bool):
    """(gx, dW) of y = x W^T at 'high' with W's split planes wsp: data and weight gradient in one paired launch
    where both are needed (the weight gradient straight into its bucket: dW None), else one each."""
    O, I = weight.shape
    g2 = g.reshape(-1, O)
    x2 = x.reshape(-1, I)
    if g2.shape[0] == 0:
        return (torch.zeros_like(x) if need_x else None), (torch.zeros_like(weight) if need_w else None)
    if need_x and need_w:
        wspec = _wgrad_spec(weight, g2.contiguous(), False, x2.contiguous(), False, O, I, g2.shape[0])
        if wspec is not None:
            gx, wres = _bwd_pair(dict(a=g2, a_kcontig=True, b=wsp, b_kcontig=False, M=g2.shape[0], N=I, K=O), wspec)
            return gx.view(x.shape), _wgrad_result(weight, wspec, wres)
    gx = gemm_x3(g2, True, wsp, False, g2.shape[0], I, O).view(x.shape) if need_x else None
    dW = _wgrad_into(weight, g2.contiguous(), False, x2.contiguous(), False, O, I, g2.shape[0]) if need_w else None
    return gx, dW


class LinearPairFunction(torch.autograd.Function):
    """(x1 W1^T, x2 W2^T): two bias-free projections of different inputs in ONE launch (rq_gemm_bf16x3_pair's
    forward pairing; split-K slabs of both reduced in one batched launch) — the decoder block's self-attention
    qkv of attn_norm(x) and cross-attention q of cross_attn_norm(x) (modules/transformer/model.py:68-82,
    modules/transformer/attention.py:96-104). Backward: each projection's paired data + weight gradient, as
    LinearFunction's. Results bitwise two LinearFunction calls (same plans per problem)."""

    @staticmethod
    def forward(ctx, x1, w1, x2, w2):
        (O1, I1), (O2, I2) = w1.shape, w2.shape
        a1, a2 = x1.reshape(-1, I1), x2.reshape(-1, I2)
        s1, s2 = split_weight(w1), split_weight(w2)
        y1, y2 = gemm_x3_pair(dict(a=a1, a_kcontig=True, b=s1, b_kcontig=True, M=a1.shape[0], N=O1, K=I1),
                              dict(a=a2, a_kcontig=True, b=s2, b_kcontig=True, M=a2.shape[0], N=O2, K=I2))
        ctx.save_for_backward(x1, x2)
        ctx.w, ctx.wsp = (w1, w2), (s1, s2)
        return y1.view(*x1.shape[:-1], O1), y2.view(*x2.shape[:-1], O2)

    @staticmethod
    def backward(ctx, g1, g2):
        x1, x2 = ctx.saved_tensors
        (w1, w2), (s1, s2) = ctx.w, ctx.wsp
        ni = ctx.needs_input_grad
        gx1 = dW1 = gx2 = dW2 = None
        if g1 is not None:
            gx1, dW1 = _linear_bwd_high(x1, g1, w1, s1, ni[0], ni[1])
        if g2 is not None:
            gx2, dW2 = _linear_bwd_high(x2, g2, w2, s2, ni[2], ni[3])
        ctx.w = ctx.wsp = None
        return gx1, dW1, gx2, dW2


def linear_pair_supported(x1: torch.Tensor, w1: torch.Tensor, x2: torch.Tensor, w2: torch.Tensor) -> bool:
    """LinearPairFunction applies: 'high' precision, fp32 device tensors, split-operand widths, rows."""
    return (matmul_high() and all(t.is_cuda and t.dtype == torch.float32 for t in (x1, w1, x2, w2)) and
            w1.shape[1] % 8 == 0 and w2.shape[1] % 8 == 0 and x1.shape[-1] == w1.shape[1] and
            x2.shape[-1] == w2.shape[1] and x1.numel() > 0 and x2.numel() > 0)


def linear_pair(x1, w1, x2, w2):
    return LinearPairFunction.apply(x1, w1, x2, w2)


class LinearAddFunction(torch.autograd.Function):
    """y = x W^T + r (bias-free Linear followed by a residual add, e.g. the attention output
    projection plus the block input, modules/transformer/model.py:75-78) as ONE split-bf16 GEMM
    launch at 'high' precision (residual added in the epilogue); backward: dx = g W, dW = g^T x,
    dr = g."""

    @staticmethod
    def forward(ctx, x, weight, r):
        O, I = weight.shape
        x2 = x.reshape(-1, I)
        wsp = split_weight(weight)
        y = gemm_x3(x2, True, wsp, True, x2.shape[0], O, I, EPI_ADD, Z=r.reshape(-1, O).contiguous())
        ctx.save_for_backward(x, weight)
        ctx.wsp, ctx.weight = wsp, weight
        return y.view(*x.shape[:-1], O)

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        O, I = weight.shape
        g2 = g.reshape(-1, O)
        gx = dW = None
        wspec = None
        if ctx.needs_input_grad[0] and ctx.needs_input_grad[1]:
            wspec = _wgrad_spec(ctx.weight, g2.contiguous(), False, x.reshape(-1, I).contiguous(), False, O, I,
                                g2.shape[0])
        if wspec is not None:   # data and weight gradient in one launch
            gx, wres = _bwd_pair(dict(a=g2, a_kcontig=True, b=ctx.wsp, b_kcontig=False, M=g2.shape[0], N=I, K=O),
                                    wspec)
            gx = gx.view(x.shape)
            dW = _wgrad_result(ctx.weight, wspec, wres)
            ctx.wsp = ctx.weight = None
            return gx, dW, g if ctx.needs_input_grad[2] else None
        if ctx.needs_input_grad[0]:
            gx = gemm_x3(g2, True, ctx.wsp, False, g2.shape[0], I, O).view(x.shape)
        ctx.wsp = None
        if ctx.needs_input_grad[1]:
            dW = _wgrad_into(ctx.weight, g2.contiguous(), False, x.reshape(-1, I).contiguous(), False, O, I,
                             g2.shape[0])
        ctx.weight = None
        return gx, dW, g if ctx.needs_input_grad[2] else None


def linear_add(x: torch.Tensor, weight: torch.Tensor, r: torch.Tensor) -> torch.Tensor:
    """x W^T + r: one fused launch at 'high' precision for fp32 device tensors with I % 8 == 0 and
    O % 4 == 0 (else the Linear and the add run separately)."""
    O, I = weight.shape
    if (matmul_high() and x.is_cuda and x.dtype == torch.float32 and r.dtype == torch.float32 and
            weight.dtype == torch.float32 and I % 8 == 0 and O % 4 == 0 and x.numel() > 0 and
            r.shape == (*x.shape[:-1], O)):
        return LinearAddFunction.apply(x, weight, r)
    return LinearFunction.apply(x, weight, None) + r if wgrad_supported(weight) else \
        torch.nn.functional.linear(x, weight) + r


def linear(x: torch.Tensor, weight: torch.Tensor, bias=None) -> torch.Tensor:
    """Drop-in for F.linear on the device path (fp32, O and I multiples of 4)."""
    require_gpu(x, weight, bias, what="linear")
    if not wgrad_supported(weight) or x.dtype != torch.float32:
        raise RqHipError(f"linear: fp32 weights with both dims % 4 == 0 required, got {tuple(weight.shape)} "
                         f"{weight.dtype}")
    return LinearFunction.apply(x, weight, bias)


class RMSNormFunction(torch.autograd.Function):
    """y = Dropout_p((x * rsqrt(mean(x^2, -1) + eps)) * w) over the last axis (modules/normalize.py:22-32,
    followed by the nn.Dropout the decoder applies to every norm output it feeds to attention), one HBM
    pass forward (rq_rmsnorm_dropout_fwd) and one backward (gx and a deterministic gw); the dropout
    mask is regenerated from `seed` in the backward, never stored. p = 0: plain RMSNorm."""

    @staticmethod
    def forward(ctx, x, weight, eps: float, p: float = 0.0, seed: int = 0):
        require_gpu(x, weight, what="rmsnorm")
        D = x.shape[-1]
        x2 = x.contiguous().view(-1, D)
        B = x2.shape[0]
        y = torch.empty_like(x2)
        rstd = torch.empty((B,), device=x.device, dtype=torch.float32)
        call("rq_rmsnorm_dropout_fwd", ptr(x2), ptr(weight), B, D, float(eps), float(p), int(seed), ptr(y), ptr(rstd),
             stream_handle(x.device))
        ctx.save_for_backward(x2, weight, rstd)
        ctx.shape, ctx.p, ctx.seed, ctx.weight = x.shape, float(p), int(seed), weight
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, gy):
        x2, weight, rstd = ctx.saved_tensors
        gx, gw = _rmsnorm_bwd(x2, ctx.weight, rstd, gy, None, ctx.p, ctx.seed, ctx.needs_input_grad[1])
        ctx.weight = None
        return gx.view(ctx.shape), gw, None, None, None


def _rmsnorm_bwd(x2, weight, rstd, gy, gres, p: float, seed: int, need_w: bool):
    """(gx [+ gres], gw) of one RMSNorm(+dropout) — gw added straight into the parameter's flat
    gradient bucket when dp.GradBuckets owns one (then returned as None), rq_rmsnorm_dropout_bwd."""
    from . import dp
    B, D = x2.shape
    gy2 = gy.contiguous().view(B, D)
    gx = torch.empty_like(x2)
    sink = dp.direct_grad(weight) if need_w else None
    gw = sink if sink is not None else torch.empty((D,), device=x2.device, dtype=torch.float32)
    nbytes = _lib.load().rq_rmsnorm_bwd_workspace(B, D)
    ws = torch.empty((nbytes,), device=x2.device, dtype=torch.uint8)
    defer = sink is not None and dp.defer_ok(weight)
    if defer and sink.data_ptr() in _DEFER["outs"]:
        flush_reductions()
    import ctypes
    parts = ctypes.c_int(0)
    call("rq_rmsnorm_dropout_bwd", ptr(x2), ptr(weight), ptr(rstd), ptr(gy2),
         ptr(None if gres is None else gres.contiguous().view(B, D)), B, D, float(p), int(seed), ptr(gx), ptr(gw),
         int(sink is not None), int(defer), ctypes.byref(parts), ptr(ws), nbytes, stream_handle(x2.device))
    if defer and parts.value > 0:
        _defer_push(ws, sink, D, parts.value, 1)
    if sink is not None:
        dp.direct_grad_done(weight)
        return gx, None
    return gx, (gw if need_w else None)


_RMS_DUAL = True   # False: the fork's two norms as two launches each way (A/B probes set the attribute)


def _rmsnorm2_bwd(x2, ws_, rstd, g1, g2, gres, ps, seeds, need):
    """(gx, gw1, gw2) of the fork's two norms in one rq_rmsnorm2_dropout_bwd launch — gx = norm2'(g2) +
    (norm1'(g1) + gres), the chained calls' order; weight gradients into their flat-bucket views (deferred
    like _rmsnorm_bwd's) or returned. None when the two weights' gradient destinations differ in kind
    (one bucket view, one returned tensor): the caller chains two single-norm backwards then."""
    from . import dp
    w1, w2 = ws_
    B, D = x2.shape
    s1 = dp.direct_grad(w1) if need[0] else None
    s2 = dp.direct_grad(w2) if need[1] else None
    if (s1 is None) != (s2 is None) or not (need[0] and need[1]):
        return None
    sinks = s1 is not None
    defer = sinks and dp.defer_ok(w1) and dp.defer_ok(w2)
    if defer and (s1.data_ptr() in _DEFER["outs"] or s2.data_ptr() in _DEFER["outs"]):
        flush_reductions()
    half = _lib.load().rq_rmsnorm_bwd_workspace(B, D)
    ws = torch.empty((2 * half,), device=x2.device, dtype=torch.uint8)
    gw1 = s1 if sinks else torch.empty((D,), device=x2.device, dtype=torch.float32)
    gw2 = s2 if sinks else torch.empty((D,), device=x2.device, dtype=torch.float32)
    gx = torch.empty_like(x2)
    import ctypes
    parts = ctypes.c_int(0)
    g1c, g2c = g1.contiguous().view(B, D), g2.contiguous().view(B, D)
    call("rq_rmsnorm2_dropout_bwd", ptr(x2), ptr(w1), ptr(w2), ptr(rstd), ptr(g1c), ptr(g2c),
         ptr(None if gres is None else gres.contiguous().view(B, D)), B, D, float(ps[0]), int(seeds[0]), float(ps[1]),
         int(seeds[1]), ptr(gx), ptr(gw1), ptr(gw2), int(sinks), int(defer), ctypes.byref(parts), ptr(ws), 2 * half,
         stream_handle(x2.device))
    if defer and parts.value > 0:
        _defer_push(ws[:half], s1, D, parts.value, 1)
        _defer_push(ws[half:], s2, D, parts.value, 1)
    if sinks:
        dp.direct_grad_done(w1)
        dp.direct_grad_done(w2)
        return gx, None, None
    return gx, gw1, gw2


class RMSNormForkFunction(torch.autograd.Function):
    """x -> (RMSNorm_1(x) [dropout], [RMSNorm_2(x) [dropout]], x): the pre-norm block's fan-out of x to
    its norm branches and to the residual stream (modules/transformer/model.py:75-82: h = x +
    SelfAttn(Dropout(attn_norm(x))) [+ CrossAttn(Dropout(cross_attn_norm(x)))]; out = h +
    Dropout(MLP(RMSNorm(h)))) as one node, so the backward adds the residual gradient inside the norm
    backward kernels (rq_rmsnorm_dropout_bwd gres) instead of autograd summing the three branch
    gradients with separate add kernels. Forward = the RMSNormFunction kernels."""

    @staticmethod
    def forward(ctx, x, eps: float, p1: float, seed1: int, p2: float, seed2: int, w1, w2):
        require_gpu(x, w1, what="rmsnorm_fork")
        D = x.shape[-1]
        x2 = x.contiguous().view(-1, D)
        B = x2.shape[0]
        outs, saved = [], [x2]
        if w2 is not None and _RMS_DUAL:   # both norms in one launch (one rstd, shared by both backward halves)
            y1, y2 = torch.empty_like(x2), torch.empty_like(x2)
            rstd = torch.empty((B,), device=x.device, dtype=torch.float32)
            call("rq_rmsnorm2_dropout_fwd", ptr(x2), ptr(w1), ptr(w2), B, D, float(eps), float(p1), int(seed1),
                 float(p2), int(seed2), ptr(y1), ptr(y2), ptr(rstd), stream_handle(x.device))
            outs = [y1.view(x.shape), y2.view(x.shape)]
            saved += [w1, rstd, w2, rstd]
        for w, p, sd in (((w1, p1, seed1), (w2, p2, seed2)) if not outs else ()):
            if w is None:
                continue
            y = torch.empty_like(x2)
            rstd = torch.empty((B,), device=x.device, dtype=torch.float32)
            call("rq_rmsnorm_dropout_fwd", ptr(x2), ptr(w), B, D, float(eps), float(p), int(sd), ptr(y), ptr(rstd),
                 stream_handle(x.device))
            outs.append(y.view(x.shape))
            saved += [w, rstd]
        ctx.save_for_backward(*saved)
        ctx.shape, ctx.ps, ctx.seeds, ctx.ws = x.shape, (float(p1), float(p2)), (int(seed1), int(seed2)), (w1, w2)
        return (*outs, x.view_as(x))

    @staticmethod
    def backward(ctx, *grads):
        saved = ctx.saved_tensors
        x2 = saved[0]
        n = (len(saved) - 1) // 2
        g_pass = grads[n]
        gres, gws = g_pass, [None, None]
        if n == 2 and _RMS_DUAL:
            r = _rmsnorm2_bwd(x2, ctx.ws, saved[2], grads[0], grads[1], g_pass, ctx.ps, ctx.seeds,
                              (ctx.needs_input_grad[6], ctx.needs_input_grad[7]))
            if r is not None:
                gx, gw1, gw2 = r
                ctx.ws = None
                return gx.view(ctx.shape), None, None, None, None, None, gw1, gw2
        for i in range(n):   # gx = norm_1' g_1 + norm_2' g_2 + g_pass, each norm backward adding the previous sum
            w, rstd = saved[1 + 2 * i], saved[2 + 2 * i]
            gres, gws[i] = _rmsnorm_bwd(x2, ctx.ws[i], rstd, grads[i], gres, ctx.ps[i], ctx.seeds[i],
                                        ctx.needs_input_grad[6 + i])
        ctx.ws = None
        return gres.view(ctx.shape), None, None, None, None, None, gws[0], gws[1]


def rmsnorm_fork(x: torch.Tensor, eps: float, w1: torch.Tensor, p1: float = 0.0, w2: torch.Tensor = None,
                 p2: float = 0.0):
    """(RMSNorm_w1(x) [dropout p1], [RMSNorm_w2(x) [dropout p2]], x) as one autograd node
    (RMSNormForkFunction); the norms' dropout keys are drawn in argument order."""
    s1 = next_seed() if p1 > 0 else 0
    s2 = next_seed() if (w2 is not None and p2 > 0) else 0
    return RMSNormForkFunction.apply(x, float(eps), float(p1), s1, float(p2), s2, w1, w2)


def rmsnorm_supported(x: torch.Tensor, weight: torch.Tensor) -> bool:
    D = x.shape[-1]
    return (x.is_cuda and not x.is_nested and x.dtype == torch.float32 and weight.dtype == torch.float32
            and D % 4 == 0 and D <= 4096)


def rmsnorm(x: torch.Tensor, weight: torch.Tensor, eps: float, p: float = 0.0) -> torch.Tensor:
    return RMSNormFunction.apply(x, weight, eps, float(p), next_seed() if p > 0 else 0)


# ------------------------------------------------------------------------------- dropout
_SEED = {"base": None, "n": 0}


def next_seed() -> int:
    """Key of the next dropout mask: a counter under torch.initial_seed(), mixed with the
    data-parallel rank so ranks that share a seed draw independent masks on their different shards
    (torch.manual_seed still makes every rank's masks reproducible; the generator is counter-based
    and masks are never stored). Host-only: no device sync. A hipGraph capture freezes the key of
    each captured call."""
    base = torch.initial_seed()
    if _SEED["base"] != base:
        _SEED["base"], _SEED["n"] = base, 0
    _SEED["n"] += 1
    rank = _dist.get_rank() if _dist.is_available() and _dist.is_initialized() else 0
    return (base * 0x9E3779B97F4A7C15 + _SEED["n"] * 0xD1B54A32D192ED03 +
            rank * 0x94D049BB133111EB) & 0x7FFFFFFFFFFFFFFF   # fits int64


def seed_epoch_advance(device=None) -> None:
    """Advance the device-side dropout epoch (mixed into every mask key, csrc/common.h) on the current
    stream: a captured train step ends with this call, so every replay draws fresh masks."""
    call("rq_seed_epoch_advance", stream_handle(device))


def seed_epoch_set(value: int, device=None) -> None:
    """Set the device-side dropout epoch (0 = eager keys)."""
    call("rq_seed_epoch_set", int(value), stream_handle(device))


def dropout_fusable(t: torch.Tensor) -> bool:
    return t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.numel() % 4 == 0


class SiluDropoutFunction(torch.autograd.Function):
    """h = Dropout_p(SiLU(z)) in one pass (the MLP hidden layer, modules/encoder.py:20-28)."""

    @staticmethod
    def forward(ctx, z, p: float, seed: int):
        require_gpu(z, what="silu_dropout")
        h = torch.empty_like(z)
        call("rq_silu_dropout_fwd", ptr(z), z.numel(), float(p), int(seed), ptr(h), stream_handle(z.device))
        ctx.save_for_backward(z)
        ctx.p, ctx.seed = float(p), int(seed)
        return h

    @staticmethod
    def backward(ctx, g):
        (z,) = ctx.saved_tensors
        g = g.contiguous()
        gz = torch.empty_like(z)
        call("rq_silu_dropout_bwd", ptr(g), ptr(z), z.numel(), ctx.p, ctx.seed, ptr(gz), stream_handle(z.device))
        return gz, None, None


def silu_dropout(z: torch.Tensor, p: float) -> torch.Tensor:
    return SiluDropoutFunction.apply(z.contiguous(), float(p), next_seed())


class DropoutAddFunction(torch.autograd.Function):
    """out = h + Dropout_p(y) in one pass (the block output, modules/transformer/model.py:76/82)."""

    @staticmethod
    def forward(ctx, h, y, p: float, seed: int):
        require_gpu(h, y, what="dropout_add")
        out = torch.empty_like(h)
        call("rq_dropout_add_fwd", ptr(h), ptr(y), h.numel(), float(p), int(seed), ptr(out), stream_handle(h.device))
        ctx.p, ctx.seed = float(p), int(seed)
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        gy = torch.empty_like(g)
        call("rq_dropout_bwd", ptr(g), g.numel(), ctx.p, ctx.seed, ptr(gy), stream_handle(g.device))
        return g, gy, None, None


def dropout_add(h: torch.Tensor, y: torch.Tensor, p: float) -> torch.Tensor:
    return DropoutAddFunction.apply(h.contiguous(), y.contiguous(), float(p), next_seed())


# ------------------------------------------------------------------------------ embedding
def _table_grad(g: torch.Tensor, keys: torch.Tensor, K: int, padding_idx) -> torch.Tensor:
    """(K, E) embedding-table gradient: segmented sum of the rows g (n, E) by keys (n,), the padding
    row's gradient zero (nn.Embedding(padding_idx)). Padding at the last row (the SemIdEmbedder
    table): sum over the first K - 1 keys (the padding key falls outside and is skipped) into a
    buffer whose last row is zeroed — no key rewrite pass."""
    E = g.shape[-1]
    if padding_idx is not None and padding_idx in (K - 1, -1) and K > 1:
        out = torch.empty((K, E), device=g.device, dtype=torch.float32)
        out[K - 1].zero_()
        segment_sum(g, keys, K - 1, with_counts=False, out=out[:K - 1])
        return out
    if padding_idx is not None:   # padding rows are skipped (key -1): their row's grad is 0
        keys = torch.where(keys == padding_idx, -1, keys)
    return segment_sum(g, keys, K, with_counts=False)[0]


class EmbeddingFunction(torch.autograd.Function):
    """F.embedding forward (a row gather); backward = deterministic segmented sum of the output
    gradient rows by index (rq_segment_sum: stable counting sort + fixed-order per-row sums), with the
    padding row's gradient zero as in nn.Embedding(padding_idx). Replaces torch's sort + scatter
    embedding backward (~4 launches and a data-dependent atomic reduction per table)."""

    @staticmethod
    def forward(ctx, weight, idx, padding_idx):
        require_gpu(weight, idx, what="embedding")
        ctx.save_for_backward(idx)
        ctx.K, ctx.padding_idx = weight.shape[0], padding_idx
        ctx.weight = weight if isinstance(weight, torch.nn.Parameter) else None
        return torch.nn.functional.embedding(idx, weight, padding_idx)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        return _emb_grad(ctx.weight, g.reshape(-1, g.shape[-1]), idx.reshape(-1), ctx.K, ctx.padding_idx), None, None


class EmbeddingPairFunction(torch.autograd.Function):
    """Two row gathers from one table, (F.embedding(ia), F.embedding(ib)) for ia (B, Na), ib (B, Nb),
    whose backward is ONE segmented sum over the (B, Na + Nb) gradient rows in the order of
    F.embedding(cat([ia, ib], 1)) — the same reduction (and bits) as gathering the concatenated
    indices and slicing the result, without the two slice-backward zero fills, copies and add."""

    @staticmethod
    def forward(ctx, weight, ia, ib, padding_idx):
        require_gpu(weight, ia, ib, what="embedding_pair")
        ctx.save_for_backward(ia, ib)
        ctx.K, ctx.padding_idx = weight.shape[0], padding_idx
        ctx.weight = weight if isinstance(weight, torch.nn.Parameter) else None
        F_ = torch.nn.functional
        return F_.embedding(ia, weight, padding_idx), F_.embedding(ib, weight, padding_idx)

    @staticmethod
    def backward(ctx, ga, gb):
        ia, ib = ctx.saved_tensors
        if not ctx.needs_input_grad[0]:
            return None, None, None, None
        E = (ga if ga is not None else gb).shape[-1]
        ga = torch.zeros(ia.shape + (E,), device=ia.device) if ga is None else ga
        gb = torch.zeros(ib.shape + (E,), device=ib.device) if gb is None else gb
        keys = torch.cat([ia, ib], dim=1).reshape(-1)
        g = torch.cat([ga, gb], dim=1).reshape(-1, E)
        return _emb_grad(ctx.weight, g, keys, ctx.K, ctx.padding_idx), None, None, None


def embedding_pair(ia: torch.Tensor, ib: torch.Tensor, weight: torch.Tensor, padding_idx=None):
    """(embedding(ia), embedding(ib)) with one backward reduction (EmbeddingPairFunction)."""
    return EmbeddingPairFunction.apply(weight, ia, ib, padding_idx)


def col_sum(x: torch.Tensor) -> torch.Tensor:
    """x (S, ...) -> sum over the leading axis, shape x.shape[1:], fixed order (rq_col_sum)."""
    require_gpu(x, what="col_sum")
    x = x.contiguous()
    S, n = x.shape[0], math.prod(x.shape[1:])
    out = torch.empty(x.shape[1:], device=x.device, dtype=torch.float32)
    call("rq_col_sum", ptr(x), S, n, ptr(out), 0, stream_handle(x.device))
    return out


def _col_sum_ok(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype == torch.float32 and x.dim() >= 2 and math.prod(x.shape[1:]) % 4 == 0


class BatchAddFunction(torch.autograd.Function):
    """x + p with p (1, *rest) broadcast over x's leading batch axis (x (B, *rest)); p's gradient is
    the batch sum of g on rq_col_sum (one fixed-order launch instead of torch's reduction)."""

    @staticmethod
    def forward(ctx, x, p):
        return x + p

    @staticmethod
    def backward(ctx, g):
        gp = col_sum(g).unsqueeze(0) if ctx.needs_input_grad[1] else None
        return (g if ctx.needs_input_grad[0] else None), gp


class BatchRepeatFunction(torch.autograd.Function):
    """p (*rest) repeated B times along a new leading axis: (B, *rest); backward = batch sum of g."""

    @staticmethod
    def forward(ctx, p, B: int):
        return p.unsqueeze(0).expand((B,) + tuple(p.shape)).contiguous()

    @staticmethod
    def backward(ctx, g):
        return col_sum(g), None


def batch_add(x: torch.Tensor, p: torch.Tensor) -> torch.Tensor:
    """x + p for p of shape (1, *x.shape[1:]) (modules/model.py:92 `pos + seq_emb`)."""
    if _col_sum_ok(x) and p.shape[0] == 1 and p.shape[1:] == x.shape[1:] and p.dtype == x.dtype:
        return BatchAddFunction.apply(x, p)
    return x + p


def batch_repeat(p: torch.Tensor, B: int) -> torch.Tensor:
    """p repeated B times on a new leading axis (modules/model.py:93 `bos_emb.repeat(B, 1, 1)` for
    p of shape (1, E): pass p.view(1, E) and get (B, 1, E))."""
    if p.is_cuda and p.dtype == torch.float32 and p.numel() % 4 == 0 and B > 0:
        return BatchRepeatFunction.apply(p, B)
    return p.unsqueeze(0).repeat((B,) + (1,) * p.dim())


class DecoderPrologueFunction(torch.autograd.Function):
    """The decoder's input embeddings (user / sem-ID / position / token-type tables, bos) written straight
    into the context and future jagged batches (rq_dec_prologue_fwd: reference modules/model.py:101-129,
    modules/embedding/id_embedder.py:28-53): two launches instead of the ~24 of the composition (gathers,
    masks, adds, cats, offsets, padded -> jagged), bitwise the same values. The backward is the
    composition's: the context's padded gradient by the jagged scatter, the position table's batch sum
    (rq_col_sum) and the four tables' deterministic segmented sums (deferred into their flat buckets when
    GradBuckets batches them), bos's batch sum — the same reductions in the same order, so the same bits."""

    @staticmethod
    def forward(ctx, user_w, sem_w, wpe_w, tte_w, bos, user_ids, sem_ids, type_ids, seq_mask, sem_fut, type_fut,
                n_buckets: int, K: int, pad: int, alloc: int):
        require_gpu(user_w, sem_w, wpe_w, tte_w, bos, user_ids, sem_ids, type_ids, seq_mask, sem_fut, type_fut,
                    what="decoder_prologue")
        B, N = sem_ids.shape
        L = sem_fut.shape[1]
        E = sem_w.shape[1]
        dev = sem_w.device
        i64 = torch.int64
        ctx_vals = torch.empty((int(alloc), E), device=dev, dtype=torch.float32)
        fut_vals = torch.empty((B * (L + 1), E), device=dev, dtype=torch.float32)
        ctx_off = torch.empty((B + 1,), device=dev, dtype=i64)
        fut_off = torch.empty((B + 1,), device=dev, dtype=i64)
        keys = torch.empty((B, N + L), device=dev, dtype=i64)
        uid_mod = torch.empty((B,), device=dev, dtype=i64)
        # the contexts' LPT order (int32, padded like the attention scratch's order slot) when B allows
        order = torch.empty(((B + 3) & ~3,), device=dev, dtype=torch.int32) if 2 <= B <= 4096 else None
        c = [t.contiguous() for t in (user_ids, sem_ids, type_ids, seq_mask, sem_fut, type_fut)]
        TIMER.around("dec_prologue", call, "rq_dec_prologue_fwd", *[ptr(t) for t in c], B, N, L, E, ptr(user_w),
                     int(n_buckets), ptr(sem_w), sem_w.shape[0], int(K), int(pad), ptr(wpe_w), wpe_w.shape[0],
                     ptr(tte_w), tte_w.shape[0], ptr(bos), ptr(ctx_vals), int(alloc), ptr(ctx_off), ptr(fut_vals),
                     ptr(fut_off), ptr(keys), ptr(uid_mod), ptr(order), stream_handle(dev))
        ctx.save_for_backward(ctx_off, keys, uid_mod, c[5])
        ctx.meta = (B, N, L, E, int(pad))
        ctx.tables = tuple(w if isinstance(w, torch.nn.Parameter) else None for w in (user_w, sem_w, wpe_w, tte_w))
        ctx.rows = (user_w.shape[0], sem_w.shape[0], wpe_w.shape[0], tte_w.shape[0])
        ctx.mark_non_differentiable(ctx_off, fut_off)
        ctx.set_materialize_grads(False)   # no zero-filled int64 "gradients" for the offsets (two launches)
        if order is not None:
            ctx_off._rq_lpt_order = order   # self-attention launches over these offsets reuse it (RQ_ATTN_ORDER_GIVEN)
        return ctx_vals, ctx_off, fut_vals, fut_off

    @staticmethod
    def backward(ctx, g_ctx, _g_off, g_fut, _g_foff):
        ctx_off, keys, uid_mod, type_fut = ctx.saved_tensors
        B, N, L, E, pad = ctx.meta
        w_user, w_sem, w_wpe, w_tte = ctx.tables
        k_user, k_sem, k_wpe, k_tte = ctx.rows
        dev = ctx_off.device
        need = ctx.needs_input_grad
        if g_ctx is None:   # no gradient reached the context rows: the padded gradient is all zeros
            g_pad = torch.zeros((B, N + 1, E), device=dev, dtype=torch.float32)
        else:
            g_ctx = g_ctx.contiguous()
            g_pad = torch.empty((B, N + 1, E), device=dev, dtype=torch.float32)
            TIMER.around("jagged_to_padded", call, "jagged_to_padded", ptr(g_ctx), ptr(ctx_off), B, N + 1, E, ptr(g_pad),
                         _DTYPES[torch.float32], stream_handle(dev))
        g_futp = (torch.zeros((B, L + 1, E), device=dev) if g_fut is None else g_fut.contiguous().view(B, L + 1, E))
        g_seq = g_pad[:, 1:]
        gu = _emb_grad(w_user, g_pad[:, :1].reshape(-1, E), uid_mod, k_user, None) if need[0] else None
        gw = None
        if need[2]:   # the position table: the batch sum of the sequence rows IS its gradient on rows 0..N-1
            # (the gather over arange(N) hits each row once); the column sums of whole padded rows, user
            # slot included, take the sequence rows' sums without a contiguous copy (same order per column)
            gw = _rows_grad(w_wpe, col_sum(g_pad.view(B, (N + 1) * E)).view(N + 1, E)[1:], k_wpe)
        gs = None
        if need[1]:   # one segmented sum over the context and future rows (EmbeddingPairFunction's order)
            g = torch.cat([g_seq, g_futp[:, 1:]], dim=1).reshape(-1, E)
            gs = _emb_grad(w_sem, g, keys.reshape(-1), k_sem, pad)
        gt = _emb_grad(w_tte, g_futp[:, 1:].reshape(-1, E), type_fut.reshape(-1), k_tte, None) if need[3] else None
        gb = col_sum(g_futp.view(B, (L + 1) * E)).view(L + 1, E)[0] if need[4] else None
        return (gu, gs, gw, gt, gb) + (None,) * 10


def decoder_prologue_supported(user_w, sem_w, wpe_w, tte_w, bos, user_ids, sem_ids, type_ids, seq_mask, sem_fut,
                               type_fut) -> bool:
    """Shapes / dtypes rq_dec_prologue_fwd serves (the training batch, future tokens present); the model keeps
    its composition otherwise."""
    if sem_fut is None or type_fut is None:
        return False
    ts = (user_w, sem_w, wpe_w, tte_w, bos)
    if not all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() for t in ts):
        return False
    E = sem_w.shape[1]
    if not (E % 4 == 0 and all(embedding_supported(w) for w in ts[:4]) and all(w.shape[1] == E for w in ts[:4]) and
            bos.shape == (E,)):
        return False
    ids = (user_ids, sem_ids, type_ids, sem_fut, type_fut)
    if not all(t.is_cuda and t.dtype == torch.int64 for t in ids) or not (seq_mask.is_cuda and seq_mask.dtype == torch.bool):
        return False
    B, N = sem_ids.shape
    return (user_ids.numel() == B and type_ids.shape == (B, N) and seq_mask.shape == (B, N) and sem_fut.dim() == 2 and
            sem_fut.shape[0] == B and type_fut.shape == sem_fut.shape and wpe_w.shape[0] >= N and 2 * B + 1 < 65535)


def decoder_prologue(user_w, sem_w, wpe_w, tte_w, bos, user_ids, sem_ids, type_ids, seq_mask, sem_fut, type_fut,
                     n_buckets: int, K: int, pad: int, alloc: int):
    """(ctx values (alloc, E), ctx offsets (B+1), fut values (B (L+1), E), fut offsets) — DecoderPrologueFunction."""
    return DecoderPrologueFunction.apply(user_w, sem_w, wpe_w, tte_w, bos, user_ids, sem_ids, type_ids, seq_mask,
                                         sem_fut, type_fut, n_buckets, K, pad, alloc)


def embedding_supported(weight: torch.Tensor) -> bool:
    """Shapes the HIP gather + segmented-sum backward (rq_segment_sum: float4 rows) serve; other tables
    take torch's embedding op."""
    K, E = weight.shape
    return (weight.is_cuda and weight.dtype == torch.float32 and K <= 4096 and 4 <= E <= 1024 and E % 4 == 0)


def embedding(idx: torch.Tensor, weight: torch.Tensor, padding_idx=None) -> torch.Tensor:
    return EmbeddingFunction.apply(weight, idx, padding_idx)


def unique_count(ids: torch.Tensor, K: int) -> torch.Tensor:
    """Number of distinct rows of ids (B, L) as a device int64 scalar (modules/rqvae.py:152-157)."""
    require_gpu(ids, what="unique_count")
    ids = ids.contiguous().to(torch.int64)
    B, L = ids.shape
    out = torch.empty((), device=ids.device, dtype=torch.int64)
    nbytes = _lib.load().rq_unique_workspace(B, L, int(K))
    ws = torch.empty((nbytes,), device=ids.device, dtype=torch.uint8)
    call("rq_unique_count", ptr(ids), B, L, int(K), ptr(out), ptr(ws), nbytes, stream_handle(ids.device))
    return out


_UNIQ_WS = {}   # (device, bytes) -> the zero-between-calls workspace of rq_unique_fraction


def unique_fraction(ids: torch.Tensor, K: int) -> torch.Tensor:
    """p_unique_ids = (number of distinct rows of ids (B, L)) / B as a device fp32 scalar, bitwise
    torch.true_divide(unique_count(ids, K), B) (modules/rqvae.py:152-157): two launches, through a workspace kept
    per device and size that rq_unique_fraction leaves zero (allocated zeroed on the first call, outside any
    graph capture that follows)."""
    require_gpu(ids, what="unique_fraction")
    ids = ids.contiguous().to(torch.int64)
    B, L = ids.shape
    if B == 0:
        return torch.full((), float("nan"), device=ids.device)
    out = torch.empty((), device=ids.device, dtype=torch.float32)
    nbytes = _lib.load().rq_unique_fraction_workspace(B, L, int(K))
    key = (ids.device, nbytes)
    ws = _UNIQ_WS.get(key)
    if ws is None:
        ws = _UNIQ_WS[key] = torch.zeros((nbytes,), device=ids.device, dtype=torch.uint8)
    call("rq_unique_fraction", ptr(ids), B, L, int(K), None, ptr(out), ptr(ws), nbytes, stream_handle(ids.device))
    return out


class CrossEntropyLossFunction(torch.autograd.Function):
    """The decoder's loss head (reference modules/model.py:137-143) on rq_ce_loss_fwd / rq_ce_loss_bwd:
    X = out_proj output (B * npos_x, K) whose last position per sequence is dropped, tgt (B, npos) int64
    with ignore_index -1 -> (loss = unred.sum(1).mean(), loss_d = unred.mean(0), logits (B * npos, K)),
    all three differentiable; 3 launches in place of the slice copy, log_softmax / nll_loss, the sums
    and their backward chain (~13 torch kernels)."""

    @staticmethod
    def forward(ctx, X, tgt, B: int):
        K = X.shape[1]
        npos = tgt.shape[-1]
        npos_x = X.shape[0] // B
        dev = X.device
        t = tgt.reshape(-1).contiguous()
        u = torch.empty(B * npos, device=dev, dtype=torch.float32)
        lse = torch.empty_like(u)
        logits = torch.empty((B * npos, K), device=dev, dtype=torch.float32)
        loss = torch.empty((), device=dev, dtype=torch.float32)
        loss_d = torch.empty(npos, device=dev, dtype=torch.float32)
        call("rq_ce_loss_fwd", ptr(X), X.stride(0), K, ptr(t), B, npos, npos_x, ptr(u), ptr(lse), ptr(logits), ptr(loss),
             ptr(loss_d), stream_handle(dev))
        ctx.save_for_backward(X, t, lse)
        ctx.dims = (B, npos, npos_x)
        ctx.set_materialize_grads(False)   # unused outputs (loss_d, logits in training) arrive as NULL: no zero fills
        return loss, loss_d, logits

    @staticmethod
    def backward(ctx, g_loss, g_loss_d, g_logits):
        X, t, lse = ctx.saved_tensors
        B, npos, npos_x = ctx.dims
        K = X.shape[1]
        dX = torch.empty((B * npos_x, K), device=X.device, dtype=torch.float32)
        gl = g_loss.contiguous() if g_loss is not None else None
        gd = g_loss_d.contiguous() if g_loss_d is not None else None
        gg = g_logits.contiguous() if g_logits is not None else None
        call("rq_ce_loss_bwd", ptr(X), X.stride(0), K, ptr(t), ptr(lse), B, npos, npos_x, ptr(gl), ptr(gd), ptr(gg),
             ptr(dX), stream_handle(X.device))
        return dX, None, None


def ce_loss_supported(X: torch.Tensor, tgt: torch.Tensor, B: int) -> bool:
    return (X.is_cuda and X.dtype == torch.float32 and X.dim() == 2 and X.stride(1) == 1 and 0 < X.shape[1] <= 1024
            and tgt.is_cuda and tgt.dtype == torch.int64 and tgt.dim() == 2 and tgt.shape[0] == B and B > 0 and
            X.shape[0] % B == 0 and X.shape[0] // B >= tgt.shape[1] > 0)


def cross_entropy_loss(X: torch.Tensor, tgt: torch.Tensor, B: int):
    """(loss, loss_d, logits) of the decoder loss head (CrossEntropyLossFunction)."""
    return CrossEntropyLossFunction.apply(X, tgt, B)


class L2NormReconFunction(torch.autograd.Function):
    """recon_b = sum_c (pre_b / max(|pre_b|, 1e-12) - x_b)^2 — the l2norm that ends the RqVae
    decoder fused with ReconstructionLoss (modules/rqvae.py:145-148). Gradient w.r.t. pre only
    (x is data)."""

    @staticmethod
    def forward(ctx, pre, x):
        require_gpu(pre, x, what="l2norm_recon")
        pre, x = pre.contiguous(), x.contiguous()
        B, C = pre.shape
        recon = torch.empty((B,), device=pre.device, dtype=torch.float32)
        norms = torch.empty((B,), device=pre.device, dtype=torch.float32)
        call("rq_l2norm_recon_fwd", ptr(pre), ptr(x), B, C, ptr(recon), ptr(norms), stream_handle(pre.device))
        ctx.save_for_backward(pre, x, norms)
        return recon

    @staticmethod
    def backward(ctx, g_recon):
        pre, x, norms = ctx.saved_tensors
        B, C = pre.shape
        g_pre = torch.empty_like(pre)
        call("rq_l2norm_recon_bwd", ptr(pre), ptr(x), ptr(norms), ptr(g_recon.contiguous()), B, C, ptr(g_pre),
             stream_handle(pre.device))
        return g_pre, None


def l2norm_recon_loss(pre, x):
    return L2NormReconFunction.apply(pre, x)


class GumbelSoftmaxQuantizeFunction(torch.autograd.Function):
    """Training-mode GUMBEL_SOFTMAX + L2 quantize (modules/quantize.py:107-129, distributions/gumbel.py:14-18):
    (x, codebook, noise, T) -> (emb = softmax((noise - dist) / T) @ codebook, ids = argmin dist) on
    rq_gumbel_softmax_fwd; backward: dx and d/d dist on rq_gumbel_softmax_bwd, the codebook gradient
    w^T g + 2 colsum(ddist) (.) c - 2 ddist^T x as three torch GEMM / reduction ops."""

    @staticmethod
    def forward(ctx, x, codebook, noise, temperature):
        require_gpu(x, codebook, noise, what="gumbel_softmax_quantize")
        x, cb, noise = x.detach().contiguous(), codebook.detach().contiguous(), noise.detach().contiguous()
        B, D = x.shape
        K = cb.shape[0]
        w = torch.empty((B, K), device=x.device, dtype=torch.float32)
        emb = torch.empty((B, D), device=x.device, dtype=torch.float32)
        ids = torch.empty((B,), device=x.device, dtype=torch.int64)
        call("rq_gumbel_softmax_fwd", ptr(x), B, D, ptr(cb), K, ptr(noise), float(temperature), ptr(w), ptr(emb),
             ptr(ids), stream_handle(x.device))
        ctx.save_for_backward(x, cb, w)
        ctx.temperature = float(temperature)
        ctx.mark_non_differentiable(ids)
        return emb, ids

    @staticmethod
    def backward(ctx, g_emb, _g_ids):
        x, cb, w = ctx.saved_tensors
        B, D = x.shape
        K = cb.shape[0]
        g = g_emb.contiguous()
        dx = torch.empty_like(x)
        ddist = torch.empty((B, K), device=x.device, dtype=torch.float32)
        call("rq_gumbel_softmax_bwd", ptr(x), ptr(cb), ptr(w), ptr(g), B, D, K, ctx.temperature, ptr(dx), ptr(ddist),
             stream_handle(x.device))
        dcb = None
        if ctx.needs_input_grad[1]:
            dcb = w.t() @ g - 2.0 * (ddist.t() @ x) + 2.0 * ddist.sum(dim=0).unsqueeze(1) * cb
        return dx, dcb, None, None


def gumbel_softmax_supported(x: torch.Tensor, codebook: torch.Tensor) -> bool:
    return (x.is_cuda and x.dtype == torch.float32 and codebook.dtype == torch.float32 and x.dim() == 2
            and 0 < x.shape[1] <= 256 and 0 < codebook.shape[0] <= 4096)


def gumbel_softmax_quantize(x, codebook, noise, temperature):
    return GumbelSoftmaxQuantizeFunction.apply(x, codebook, noise, temperature)


def row_norms(x: torch.Tensor) -> torch.Tensor:
    """|x_r|_2 over the last axis (no grad): one HBM pass (rq_row_norms)."""
    require_gpu(x, what="row_norms")
    x = x.detach().contiguous()
    D = x.shape[-1]
    out = torch.empty(x.shape[:-1], device=x.device, dtype=torch.float32)
    call("rq_row_norms", ptr(x), x.numel() // D, D, ptr(out), stream_handle(x.device))
    return out


class LossMeansFunction(torch.autograd.Function):
    """(mean(recon + qloss), mean(recon), mean(qloss)) in one deterministic pass; backward
    broadcasts (g0 + g1) / B to recon and (g0 + g2) / B to qloss."""

    @staticmethod
    def forward(ctx, recon, qloss):
        require_gpu(recon, qloss, what="loss_means")
        recon, qloss = recon.contiguous(), qloss.contiguous()
        out = torch.empty((3,), device=recon.device, dtype=torch.float32)
        call("rq_loss_means", ptr(recon), ptr(qloss), recon.numel(), ptr(out), stream_handle(recon.device))
        ctx.B = recon.numel()
        ctx.set_materialize_grads(False)   # the logged means usually get no gradient
        return out[0], out[1], out[2]

    @staticmethod
    def backward(ctx, g0, g1, g2):
        B = ctx.B

        def tot(a, b):
            if a is None:
                return b
            return a if b is None else a + b
        gr, gq = tot(g0, g1), tot(g0, g2)
        if gr is None and gq is None:
            return None, None
        if gr is gq:   # only the total loss has a gradient: one scale for both inputs, one launch
            if gr.is_cuda and gr.dtype == torch.float32 and gr.dim() == 0:
                s = torch.empty((), device=gr.device, dtype=torch.float32)
                vec = torch.empty((B,), device=gr.device, dtype=torch.float32)
                call("rq_loss_means_bwd", ptr(gr.contiguous()), B, ptr(s), ptr(vec), stream_handle(gr.device))
                return s.expand(B), vec   # bitwise (gr / B).expand(B), the qloss one materialised
            gr = gq = (gr / B).expand(B)
            return gr, gq
        return (None if gr is None else (gr / B).expand(B)), (None if gq is None else (gq / B).expand(B))


def loss_means(recon, qloss):
    return LossMeansFunction.apply(recon, qloss)


# --------------------------------------------------------------------------------- jagged
def jagged_offsets(lengths: torch.Tensor, N: int) -> torch.Tensor:
    require_gpu(lengths, what="jagged_offsets")
    lengths = lengths.contiguous().to(torch.int64)
    B = lengths.shape[0]
    off = torch.empty((B + 1,), device=lengths.device, dtype=torch.int64)
    call("jagged_offsets", ptr(lengths), B, int(N), ptr(off), stream_handle(lengths.device))
    return off


class PaddedToJaggedValues(torch.autograd.Function):
    """values (T, D) of the NJT built by ops/triton/jagged.py:11-66; backward = :69-77. `alloc` rows
    are allocated (>= the valid total offsets[B]); the kernel zero-fills the rows past offsets[B] on
    the device, so the valid total never has to be known on the host. `total` (optional, host int)
    only labels the kernel timer's algorithmic bytes."""

    @staticmethod
    def forward(ctx, x, offsets, alloc: int, add_one_sub_one: bool, total: int = None):
        require_gpu(x, offsets, what="padded_to_jagged")
        assert x.dim() == 3 and x.is_contiguous()
        B, N, D = x.shape
        vals = torch.empty((int(alloc), D), device=x.device, dtype=x.dtype)
        TIMER.around("jagged_from_padded", call, "jagged_from_padded_rows", ptr(x), B, N, D, ptr(offsets), ptr(vals),
                     int(alloc), _DTYPES[x.dtype], int(add_one_sub_one), stream_handle(x.device))
        if TIMER.wants("jagged_from_padded"):
            TIMER.bytes.setdefault("jagged_from_padded", []).append(2 * (alloc if total is None else total) * D *
                                                                    x.element_size())
        ctx.save_for_backward(offsets)
        ctx.shape = (B, N, D)
        return vals

    @staticmethod
    def backward(ctx, g_vals):
        (offsets,) = ctx.saved_tensors
        B, N, D = ctx.shape
        g_vals = g_vals.contiguous()
        gx = torch.empty((B, N, D), device=g_vals.device, dtype=g_vals.dtype)
        TIMER.around("jagged_to_padded", call, "jagged_to_padded", ptr(g_vals), ptr(offsets), B, N, D, ptr(gx),
                     _DTYPES[g_vals.dtype], stream_handle(g_vals.device))
        if TIMER.wants("jagged_to_padded"):
            TIMER.bytes.setdefault("jagged_to_padded", []).append((g_vals.numel() + gx.numel()) * gx.element_size())
        return gx, None, None, None, None


class JaggedToPaddedValues(torch.autograd.Function):
    """Inverse conversion (padded (B,N,D) with zero fill) — used for the encoder-cache repeat in
    generation (modules/model.py:222-228) and as the backward of the gather."""

    @staticmethod
    def forward(ctx, vals, offsets, N: int):
        require_gpu(vals, offsets, what="jagged_to_padded")
        vals = vals.contiguous()
        B = offsets.shape[0] - 1
        D = vals.shape[1]
        x = torch.empty((B, N, D), device=vals.device, dtype=vals.dtype)
        call("jagged_to_padded", ptr(vals), ptr(offsets), B, N, D, ptr(x), _DTYPES[vals.dtype],
             stream_handle(vals.device))
        ctx.save_for_backward(offsets)
        ctx.total = vals.shape[0]
        return x

    @staticmethod
    def backward(ctx, gx):
        (offsets,) = ctx.saved_tensors
        return PaddedToJaggedValues.apply(gx.contiguous(), offsets, ctx.total, False), None, None


# ------------------------------------------------------------------------------ attention
# Kernel policy of the attention calls (the `flags` argument, RQ_ATTN_* in include/rqvae_hip.h; 0 = the
# measured-best forms): set only by kernel-vs-kernel tests and A/B probes through attn_policy().
ATTN_NO_DMA, ATTN_TWO_PASS, ATTN_NO_SPLIT, ATTN_SPLIT_BF16, ATTN_LPT_SHORT, ATTN_ORDER_GIVEN = 1, 2, 4, 8, 32, 64
ATTN_FEWQ_WG = 16
_ATTN_POLICY = {"flags": 0}


def ATTN_QSPLIT(n: int) -> int:
    return int(n) << 8


def attn_policy(flags: int) -> _Policy:
    """`with ops.attn_policy(ops.ATTN_TWO_PASS): ...` — every varlen attention launch inside (forward and
    the backward run inside the block) carries these RQ_ATTN_* flags."""
    return _Policy(_ATTN_POLICY, flags)


# False: exact-fp32 attention products at 'high' too (A/B probes set the attributes; _ATTN_X3_BWD: the backward)
_ATTN_X3 = True
_ATTN_X3_BWD = True


_GIVEN_ORDER = True   # False: ignore the prologue's LPT order (A/B probes set the attribute)


def _given_order(cu_q, cu_k, n_needed: int):
    """The LPT order the decoder prologue attached to a context's offsets (`_rq_lpt_order`, int32), usable as
    the whole scratch of a self-attention launch over those offsets (RQ_ATTN_ORDER_GIVEN) when the launch
    needs nothing else; else None."""
    order = getattr(cu_k, "_rq_lpt_order", None) if _GIVEN_ORDER else None
    if order is None or cu_q is not cu_k or n_needed != order.numel():
        return None
    return order


def _attn_fwd(q, k, v, cu_q, cu_k, B, H, hd, max_q, max_k, causal, scale, out, lse):
    """Forward launch(es) (varlen_attn_fwd with scratch for the LPT order and split-key partials). At matmul
    precision 'high' (the reference's setting, modules/model.py:27) the long-range forms multiply in split-bf16
    like every Linear (RQ_ATTN_SPLIT_BF16); 'highest' keeps exact fp32 products. A self-attention over offsets
    that carry the prologue's LPT order dispatches its sequences longest-first without an order launch."""
    import ctypes
    Tq = q.shape[0]
    flags = _ATTN_POLICY["flags"] | (ATTN_SPLIT_BF16 if _ATTN_X3 and matmul_high() else 0)
    n = ctypes.c_int64(0)
    call("varlen_attn_fwd_ws_elems", B, H, hd, int(max_q), int(max_k), Tq, int(causal), flags, ctypes.byref(n))
    ws = _given_order(cu_q, cu_k, int(n.value))
    if ws is not None:
        flags |= ATTN_LPT_SHORT | ATTN_ORDER_GIVEN
    else:
        ws = torch.empty((max(1, int(n.value)),), device=q.device, dtype=torch.float32)
    TIMER.around("varlen_attn_fwd", call, "varlen_attn_fwd", ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v),
                 v.stride(0), ptr(cu_q), ptr(cu_k), B, H, hd, int(max_q), int(max_k), int(causal), float(scale),
                 ptr(out), out.stride(0), ptr(lse), Tq, ptr(ws), ws.numel(), flags, stream_handle(q.device))
    return ws if flags & ATTN_ORDER_GIVEN else None


def _attn_bwd(q, k, v, out, dout, lse, cu_q, cu_k, B, H, max_q, max_k, causal, scale, dq, dk, dv, order=None):
    """Backward launch(es) of varlen attention into dq / dk / dv (row-strided views); scratch sized for
    the fused form's query splits (Tk given). At 'high' the fused long-range form multiplies in split-bf16.
    `order`: the forward's given LPT order (the short one-pass forms then dispatch longest-first too)."""
    import ctypes
    Tq, A = q.shape
    flags = _ATTN_POLICY["flags"] | (ATTN_SPLIT_BF16 if _ATTN_X3 and _ATTN_X3_BWD and matmul_high() else 0)
    delta = torch.empty((H, Tq), device=q.device, dtype=torch.float32)   # scratch: rowsum(dO * O)
    n = ctypes.c_int64(0)
    ws = None
    if order is not None:
        call("varlen_attn_bwd_ws_elems", B, H, A // H, int(max_q), int(max_k), Tq, k.shape[0],
             flags | ATTN_LPT_SHORT, ctypes.byref(n))
        if n.value == order.numel():
            ws, flags = order, flags | ATTN_LPT_SHORT | ATTN_ORDER_GIVEN
    if ws is None:
        call("varlen_attn_bwd_ws_elems", B, H, A // H, int(max_q), int(max_k), Tq, k.shape[0], flags, ctypes.byref(n))
        ws = torch.empty((int(n.value),), device=q.device, dtype=torch.float32) if n.value else None
    TIMER.around("varlen_attn_bwd", call, "varlen_attn_bwd", ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v),
                 v.stride(0), ptr(out), out.stride(0), ptr(dout), dout.stride(0), ptr(lse), Tq, ptr(cu_q), ptr(cu_k), B,
                 H, A // H, int(max_q), int(max_k), int(causal), float(scale), ptr(dq), dq.stride(0), ptr(dk),
                 dk.stride(0), ptr(dv), dv.stride(0), k.shape[0], ptr(delta), ptr(ws), int(n.value), flags,
                 stream_handle(q.device))


class VarlenAttentionFunction(torch.autograd.Function):
    """softmax(q k^T * scale [causal]) v per segment; q/k/v are (T, H*hd) row views (any row stride)."""

    @staticmethod
    def forward(ctx, q, k, v, cu_q, cu_k, num_heads: int, causal: bool, max_q: int, max_k: int, scale: float):
        require_gpu(q, k, v, cu_q, cu_k, what="varlen_attention")
        for t in (q, k, v):
            assert t.dim() == 2 and t.stride(1) == 1 and t.dtype == torch.float32
        Tq, A = q.shape
        hd = A // num_heads
        B = cu_q.shape[0] - 1
        out = torch.empty((Tq, A), device=q.device, dtype=torch.float32)
        lse = torch.empty((num_heads, Tq), device=q.device, dtype=torch.float32)
        ctx.order = _attn_fwd(q, k, v, cu_q, cu_k, B, num_heads, hd, max_q, max_k, causal, scale, out, lse)
        ctx.save_for_backward(q, k, v, out, lse, cu_q, cu_k)
        ctx.cfg = (num_heads, bool(causal), int(max_q), int(max_k), float(scale))
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse, cu_q, cu_k = ctx.saved_tensors
        H, causal, max_q, max_k, scale = ctx.cfg
        dout = dout.contiguous()
        Tq, A = q.shape
        B = cu_q.shape[0] - 1
        dq = torch.empty((Tq, A), device=q.device, dtype=torch.float32)
        dk = torch.empty((k.shape[0], A), device=q.device, dtype=torch.float32)
        dv = torch.empty((v.shape[0], A), device=q.device, dtype=torch.float32)
        _attn_bwd(q, k, v, out, dout, lse, cu_q, cu_k, B, H, max_q, max_k, causal, scale, dq, dk, dv, ctx.order)
        ctx.order = None
        return dq, dk, dv, None, None, None, None, None, None, None


class PackedVarlenAttentionFunction(torch.autograd.Function):
    """Varlen attention on the packed projection outputs: self-attention reads q/k/v as the three
    column blocks of qkv (T, 3A); cross-attention reads q (Tq, A) and k/v as the two column blocks
    of kv (Tk, 2A). The backward writes dq/dk/dv straight into one gradient buffer per projection
    output (row-strided), so autograd never concatenates the three chunk gradients. Buffers may
    carry zero tail rows past the last sequence (row bucketing): the kernels write zero outputs
    and gradients there themselves."""

    @staticmethod
    def forward(ctx, qsrc, kvsrc, cu_q, cu_k, num_heads: int, causal: bool, max_q: int, max_k: int, scale: float):
        require_gpu(qsrc, cu_q, cu_k, what="varlen_attention")
        self_attn = kvsrc is None
        A = qsrc.shape[1] // 3 if self_attn else qsrc.shape[1]
        src_kv = qsrc if self_attn else kvsrc
        koff = A if self_attn else 0
        for t in (qsrc, src_kv):
            assert t.dim() == 2 and t.stride(1) == 1 and t.dtype == torch.float32
        q = qsrc[:, :A]
        k = src_kv[:, koff:koff + A]
        v = src_kv[:, koff + A:koff + 2 * A]
        Tq = q.shape[0]
        hd = A // num_heads
        B = cu_q.shape[0] - 1
        out = torch.empty((Tq, A), device=q.device, dtype=torch.float32)
        lse = torch.empty((num_heads, Tq), device=q.device, dtype=torch.float32)
        ctx.order = _attn_fwd(q, k, v, cu_q, cu_k, B, num_heads, hd, max_q, max_k, causal, scale, out, lse)
        if self_attn:
            ctx.save_for_backward(qsrc, out, lse, cu_q, cu_k)
        else:
            ctx.save_for_backward(qsrc, kvsrc, out, lse, cu_q, cu_k)
        ctx.cfg = (self_attn, A, num_heads, bool(causal), int(max_q), int(max_k), float(scale))
        ctx.kv_sink = None if self_attn else getattr(kvsrc, "_rq_grad_sink", None)
        return out

    @staticmethod
    def backward(ctx, dout):
        self_attn, A, H, causal, max_q, max_k, scale = ctx.cfg
        if self_attn:
            qsrc, out, lse, cu_q, cu_k = ctx.saved_tensors
            kvsrc = None
        else:
            qsrc, kvsrc, out, lse, cu_q, cu_k = ctx.saved_tensors
        src_kv = qsrc if self_attn else kvsrc
        koff = A if self_attn else 0
        dout = dout.contiguous()
        gq_src = torch.empty_like(qsrc)
        if self_attn:
            gkv_src = gq_src
        elif ctx.kv_sink is not None:   # a column block of the hoisted K/V projection's gradient buffer
            gkv_src = ctx.kv_sink[0].block(ctx.kv_sink[1])
        else:
            gkv_src = torch.empty_like(kvsrc)
        ctx.kv_sink = None
        q, k, v = qsrc[:, :A], src_kv[:, koff:koff + A], src_kv[:, koff + A:koff + 2 * A]
        dq, dk, dv = gq_src[:, :A], gkv_src[:, koff:koff + A], gkv_src[:, koff + A:koff + 2 * A]
        B = cu_q.shape[0] - 1
        _attn_bwd(q, k, v, out, dout, lse, cu_q, cu_k, B, H, max_q, max_k, causal, scale, dq, dk, dv, ctx.order)
        ctx.order = None
        return gq_src, (None if self_attn else gkv_src), None, None, None, None, None, None, None


def varlen_attention_packed(qsrc, kvsrc, cu_q, cu_k, num_heads, causal, max_q, max_k, scale=None):
    """qsrc = qkv (T, 3A) with kvsrc None (self-attention), or q (Tq, A) with kv (Tk, 2A) (cross).
    Rows past the last sequence (bucket tail) come out zero in the output and the gradients."""
    A = qsrc.shape[1] // 3 if kvsrc is None else qsrc.shape[1]
    if scale is None:
        scale = 1.0 / math.sqrt(A // num_heads)
    return PackedVarlenAttentionFunction.apply(qsrc, kvsrc, cu_q, cu_k, num_heads, causal, max_q, max_k, scale)


class _GradSink:
    """The (T, n * W) gradient buffer of a hoisted projection, allocated by the first consumer
    backward that writes its column block (every block is written whole: no zero fill)."""

    def __init__(self, like: torch.Tensor, width: int, n: int):
        self.like, self.width, self.n, self.buf = like, width, n, None

    def block(self, i: int) -> torch.Tensor:
        if self.buf is None:
            self.buf = torch.empty((self.like.shape[0], self.width * self.n), device=self.like.device,
                                   dtype=torch.float32)
        return self.buf[:, i * self.width:(i + 1) * self.width]

    def is_block(self, g, i: int) -> bool:
        return (self.buf is not None and g is not None and g.shape == (self.buf.shape[0], self.width) and
                g.stride() == self.buf.stride() and
                g.data_ptr() == self.buf.data_ptr() + i * self.width * self.buf.element_size())


# False: the hoisted projection reads its fp32 input directly (A/B probes set the attribute)
_HOIST_SPLIT = True


class HoistedProjectionFunction(torch.autograd.Function):
    """[x W_0^T | x W_1^T | ...] for bias-free Linears that read the SAME input — the decoder layers'
    cross-attention K/V projections of the encoder output (reference modules/transformer/
    attention.py:186-188 `self.kv(x_kv)` in every decoder layer, transformer/model.py:124-131) — as ONE
    split-bf16 GEMM over the concatenated weights (bitwise the per-layer products: same k order per
    output column). Returns one row-strided (T, O_i) column view per weight. Backward: when each
    consumer wrote its gradient into its block of one shared buffer (PackedVarlenAttentionFunction
    does for views carrying `_rq_grad_sink`), the data gradient is one GEMM with K = sum O_i (no adds of
    per-layer input gradients) and the weight gradients one GEMM over the rows."""

    @staticmethod
    def forward(ctx, x, *weights):
        O, I = weights[0].shape
        T = x.shape[0]
        wsp = stacked_split(weights)
        # the shared input split once (4 B read + 4 B written per element): both uses — this forward
        # (T x n O x I) and the weight-gradient GEMM (its n-contiguous B) — then run on the wide LDS-DMA
        # kernel instead of splitting x while staging it
        xs = split_bf16x3(x) if _HOIST_SPLIT else x
        y = gemm_x3(xs, True, wsp, True, T, O * len(weights), I)
        sink = _GradSink(x, O, len(weights))
        outs = []
        for i in range(len(weights)):
            v = y[:, i * O:(i + 1) * O]
            v._rq_grad_sink = (sink, i)
            outs.append(v)
        ctx.save_for_backward(x)
        ctx.wsp, ctx.weights, ctx.sink, ctx.xs = wsp, weights, sink, xs
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        (x,) = ctx.saved_tensors
        weights, sink, wsp, xs = ctx.weights, ctx.sink, ctx.wsp, ctx.xs
        ctx.wsp = ctx.weights = ctx.sink = ctx.xs = None
        n = len(weights)
        O, I = weights[0].shape
        T = x.shape[0]
        if all(sink.is_block(g, i) for i, g in enumerate(gs)):
            g = sink.buf
        else:
            g = torch.cat([gi if gi is not None else x.new_zeros((T, O)) for gi in gs], 1)
        sink.buf = None
        dws = [None] * n
        if ctx.needs_input_grad[0] and any(ctx.needs_input_grad[1:]) and _pairing():
            # data gradient and the concatenated weight gradient in one launch
            gx, dw = _bwd_pair(dict(a=g, a_kcontig=True, b=wsp, b_kcontig=False, M=T, N=I, K=n * O),
                                  dict(a=g, a_kcontig=False, b=xs, b_kcontig=False, M=n * O, N=I, K=T))
            dws = _wgrad_multi_into(weights, g, xs, n * O, I, T, dw=dw)
            return (gx, *dws)
        gx = gemm_x3(g, True, wsp, False, T, I, n * O) if ctx.needs_input_grad[0] else None
        if any(ctx.needs_input_grad[1:]):
            dws = _wgrad_multi_into(weights, g, xs, n * O, I, T)
        return (gx, *dws)


def _wgrad_multi_into(weights, g, x, O_all: int, I: int, rows: int, dw=None):
    """dW_cat = g^T x (O_all, I) as one GEMM (or `dw` already computed by a paired launch), then each
    weight's row block added into its flat gradient bucket view (dp.direct_grad; returns None for it) or
    returned as its gradient."""
    from . import dp
    sinks = [dp.direct_grad(w) for w in weights]
    O = weights[0].shape[0]
    dw_in = dw

    dw = dw_in if dw_in is not None else gemm_x3(g, False, x, False, O_all, I, rows)
    for i, sk in enumerate(sinks):
        if sk is not None:
            blk = dw[i * O:(i + 1) * O]
            if (dp.defer_ok(weights[i]) and sk.is_contiguous() and (sk.data_ptr() | blk.data_ptr()) % 16 == 0 and blk.numel() % 4 == 0
                    and sk.data_ptr() not in _DEFER["outs"]):
                _defer_push(blk, sk, blk.numel(), 1, 0)   # into the step's one batched reduction (sk + blk)
            else:
                sk.add_(blk)
            dp.direct_grad_done(weights[i])
    return [None if sk is not None else dw[i * O:(i + 1) * O] for i, sk in enumerate(sinks)]


def hoisted_projection(x: torch.Tensor, weights) -> list:
    """HoistedProjectionFunction where it applies (matmul precision 'high', fp32 device tensors, equal
    bias-free weight shapes, both dims % 8), else None (callers keep their per-layer Linears)."""
    if not (weights and matmul_high() and x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and
            x.shape[0] > 0 and x.is_contiguous()):
        return None
    O, I = weights[0].shape
    if not (all(w.shape == (O, I) and w.dtype == torch.float32 and w.is_cuda for w in weights) and
            O % 8 == 0 and I % 8 == 0 and x.shape[1] == I):
        return None
    return list(HoistedProjectionFunction.apply(x, *weights))


def varlen_attention(q, k, v, cu_q, cu_k, num_heads, causal, max_q, max_k, scale=None):
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[1] // num_heads)
    return VarlenAttentionFunction.apply(q, k, v, cu_q, cu_k, num_heads, causal, max_q, max_k, scale)
