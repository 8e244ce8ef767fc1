"""ctypes binding of librqvae_hip.so (C ABI declared in include/rqvae_hip.h).

The library is loaded AFTER `import torch`, so its NEEDED libamdhip64.so.7 resolves to the
HIP runtime torch already loaded (same SONAME): one runtime, one set of streams, and the
kernels are capturable in torch.cuda.CUDAGraph (= hipGraph).

There is deliberately no CPU fallback: every op raises if the library is missing or a
tensor is not resident on the GPU.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RQVAE_HIP_LIB", os.path.join(_HERE, "librqvae_hip.so"))

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I = ctypes.c_int
_F = ctypes.c_float
_SZ = ctypes.c_size_t
_U64 = ctypes.c_uint64

_SIGS = {
    "rq_abi_version": ([], _I),
    "rq_last_error": ([], ctypes.c_char_p),
    "rq_codebook_sqnorm": ([_P, _I64, _I64, _P, _P], _I),
    "rq_quantize_fwd": ([_P, _I64, _I64, _P, _P, _I64, _I64, _I, _F, _P, _P, _P, _P, _P, _P, _I, _P], _I),
    "rq_quantize_bwd_workspace": ([_I64, _I64, _I64, _I64], _SZ),
    "rq_quantize_bwd": ([_P, _P, _P, _I64, _I64, _I64, _I64, _I, _F, _P, _P, _P, _P, _P, _P, _P, _SZ, _P], _I),
    "rq_segment_sum_workspace": ([_I64, _I64], _SZ),
    "rq_segment_sum": ([_P, _P, _I64, _I64, _I64, _P, _P, _P, _SZ, _P], _I),
    "rq_rmsnorm_fwd": ([_P, _P, _I64, _I64, _F, _P, _P, _P], _I),
    "rq_rmsnorm_bwd_workspace": ([_I64, _I64], _SZ),
    "rq_rmsnorm_bwd": ([_P, _P, _P, _P, _I64, _I64, _P, _P, _P, _SZ, _P], _I),
    "rq_rmsnorm_dropout_fwd": ([_P, _P, _I64, _I64, _F, _F, _U64, _P, _P, _P], _I),
    "rq_rmsnorm_dropout_bwd": ([_P, _P, _P, _P, _P, _I64, _I64, _F, _U64, _P, _P, _I, _I, _P, _P, _SZ, _P], _I),
    "rq_rmsnorm2_dropout_fwd": ([_P, _P, _P, _I64, _I64, _F, _F, _U64, _F, _U64, _P, _P, _P, _P], _I),
    "rq_rmsnorm2_dropout_bwd": ([_P, _P, _P, _P, _P, _P, _P, _I64, _I64, _F, _U64, _F, _U64, _P, _P, _P, _I, _I, _P, _P, _SZ,
                                 _P], _I),
    "rq_dropout_params": ([_F, _P, _P], _I),
    "rq_silu_dropout_fwd": ([_P, _I64, _F, _U64, _P, _P], _I),
    "rq_silu_dropout_bwd": ([_P, _P, _I64, _F, _U64, _P, _P], _I),
    "rq_dropout_add_fwd": ([_P, _P, _I64, _F, _U64, _P, _P], _I),
    "rq_dropout_bwd": ([_P, _I64, _F, _U64, _P, _P], _I),
    "rq_linear_wgrad_workspace": ([_I64, _I64, _I64], _SZ),
    "rq_linear_wgrad": ([_P, _I64, _P, _I64, _I64, _I64, _I64, _P, _P, _P, _SZ, _P], _I),
    "rq_gemm_bf16x3_workspace": ([_I64, _I64, _I64], _SZ),
    "rq_gemm_bf16x3": ([_P, _I64, _I, _P, _I64, _I, _I64, _I64, _I64, _P, _I64, _P, _SZ, _P], _I),
    "rq_gemm_bf16x3_run": ([_P, _P, _P], _I),
    "rq_gemm_bf16x3_plan": ([_P, _P], _I),
    "rq_reduce_partials": ([_I, _P, _P, _P, _P, _P, _P, _P], _I),
    "rq_ce_loss_fwd": ([_P, _I64, _I64, _P, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P], _I),
    "rq_ce_loss_bwd": ([_P, _I64, _I64, _P, _P, _I64, _I64, _I64, _P, _P, _P, _P, _P], _I),
    "rq_gemm_bf16x3_pair": ([_P, _P, _P], _I),
    "rq_gemm_bf16x3_pair_plan": ([_P], _I),
    "rq_segment_sum_multi_workspace": ([_I, _P, _P, _I64], _SZ),
    "rq_segment_sum_multi": ([_I, _P, _P, _P, _P, _P, _I64, _P, _P, _SZ, _P], _I),
    "rq_split_bf16x3": ([_P, _I64, _P, _P, _P], _I),
    "rq_split_bf16x3_multi": ([_I, _P, _P, _P, _P, _P], _I),
    "rq_unique_workspace": ([_I64, _I64, _I64], _SZ),
    "rq_unique_count": ([_P, _I64, _I64, _I64, _P, _P, _SZ, _P], _I),
    "rq_unique_fraction_workspace": ([_I64, _I64, _I64], _SZ),
    "rq_unique_fraction": ([_P, _I64, _I64, _I64, _P, _P, _P, _SZ, _P], _I),
    "rq_l2norm_recon_fwd": ([_P, _P, _I64, _I64, _P, _P, _P], _I),
    "rq_col_sum": ([_P, _I64, _I64, _P, _I, _P], _I),
    "rq_row_norms": ([_P, _I64, _I64, _P, _P], _I),
    "rq_loss_means": ([_P, _P, _I64, _P, _P], _I),
    "rq_loss_means_bwd": ([_P, _I64, _P, _P, _P], _I),
    "rq_gumbel_softmax_fwd": ([_P, _I64, _I64, _P, _I64, _P, _F, _P, _P, _P, _P], _I),
    "rq_gumbel_softmax_bwd": ([_P, _P, _P, _P, _I64, _I64, _I64, _F, _P, _P, _P], _I),
    "rq_l2norm_recon_bwd": ([_P, _P, _P, _P, _I64, _I64, _P, _P], _I),
    "rq_l2norm_recon_bwd_split": ([_P, _P, _P, _P, _I64, _I64, _P, _P, _P], _I),
    "rq_l2norm_recon_fwd_grad": ([_P, _P, _I64, _I64, _P, _P, _F, _P, _P, _P], _I),
    "rq_l2norm_recon_bwd_fix": ([_P, _P, _P, _P, _I64, _I64, _I64, _F, _P, _P, _P], _I),
    "jagged_offsets": ([_P, _I64, _I64, _P, _P], _I),
    "jagged_from_padded": ([_P, _I64, _I64, _I64, _P, _P, _I, _I, _P], _I),
    "jagged_from_padded_rows": ([_P, _I64, _I64, _I64, _P, _P, _I64, _I, _I, _P], _I),
    "jagged_to_padded": ([_P, _P, _I64, _I64, _I64, _P, _I, _P], _I),
    "rq_dec_prologue_fwd": ([_P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _P, _I64, _P, _I64, _I64, _I64, _P, _I64, _P,
                             _I64, _P, _P, _I64, _P, _P, _P, _P, _P, _P, _P], _I),
    "varlen_attn_fwd_ws_elems": ([_I64, _I64, _I64, _I64, _I64, _I64, _I, _I, _P], _I),
    "varlen_attn_fwd": ([_P, _I64, _P, _I64, _P, _I64, _P, _P, _I64, _I64, _I64, _I64, _I64, _I, _F, _P, _I64, _P,
                         _I64, _P, _I64, _I, _P], _I),
    "varlen_attn_bwd_ws_elems": ([_I64, _I64, _I64, _I64, _I64, _I64, _I64, _I, _P], _I),
    "varlen_attn_bwd": ([_P, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _P, _I64, _I64, _I64, _I64,
                         _I64, _I, _F, _P, _I64, _P, _I64, _P, _I64, _I64, _P, _P, _I64, _I, _P], _I),
    "rq_seed_epoch_advance": ([_P], _I),
    "rq_seed_epoch_set": ([_U64, _P], _I),
    "rq_adamw_step": ([_P, _I64, _F, _F, _F, _F, _F, _F, _F, _P], _I),
    "rq_adamw_chunk_elems": ([], _SZ),
}

EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None


class RqHipError(RuntimeError):
    pass


def load(path: str = None):
    """Load (once) and type the C-ABI library. Raises RqHipError if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RqHipError(f"HIP library not built: {p} (run `make -C rq-vae-recommender_amd/csrc` "
                         f"or __graft_entry__.build())")
    lib = ctypes.CDLL(p)
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    if path is None:
        _lib = lib
    return lib


def call(name: str, *args):
    rc = getattr(_lib if _lib is not None else load(), name)(*args)
    if rc != 0:
        msg = load().rq_last_error().decode(errors="replace")
        raise RqHipError(f"{name} failed (rc={rc}): {msg}")


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_handle(device=None):
    """torch's current HIP stream of `device` (default: the current device) as a C pointer. Uses
    the raw-stream query (no Stream object, no device-index normalisation): this runs once per
    kernel launch, so the decoder step's ~140 launches make it a visible host cost."""
    if _RAW_STREAM is not None:
        if device is None:
            idx = torch.cuda.current_device()
        elif isinstance(device, int):
            idx = device
        else:
            idx = device.index if device.index is not None else torch.cuda.current_device()
        return ctypes.c_void_p(_RAW_STREAM(idx))
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_gpu(*tensors, what="op"):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RqHipError(f"{what}: tensors must live on the MI355X (ROCm) device; got {t.device}. "
                             "This build has no CPU fallback.")
