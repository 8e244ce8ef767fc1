"""Library-GEMM solution selection for the fp32 Linear layers (forward and data gradient).

The MLP / projection GEMMs that stay on the ROCm libraries (weight gradients run on the HIP
split-K kernel, rqvae_hip.ops.linear_wgrad) are dispatched by PyTorch to hipBLASLt, whose default
heuristic picks measurably slow fp32 solutions for this workload's shapes (M = 11k-65k rows,
N, K = 64-1536): 85-130 TFLOP/s where the best rocBLAS solution of the same shape reaches up to
148 (MI355X fp32 MFMA peak 157). PyTorch's TunableOp times every hipBLASLt and rocBLAS solution
for a shape once and then always dispatches the fastest; `enable()` turns it on with a results
table kept next to this module (shipped pre-tuned for gfx950 at the bench shapes; TunableOp
appends newly tuned shapes when the process exits; delete the file to re-tune). The solutions are plain library
GEMMs at fp32 — no precision change.

Variable-length decoder batches would otherwise present a new row count (= new shape) every
step; modules.model.EncoderDecoderRetrievalModel pads the jagged row count to a multiple of
ROW_BUCKET so the set of shapes (and tunings) stays small.
"""
import os

import torch

ROW_BUCKET = 256
DEFAULT_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tunableop", "results_gfx950.csv")


def enable(results_file: str = None, tune_new_shapes: bool = True, max_tuning_ms: int = 30) -> str:
    """Turn on TunableOp GEMM selection; returns the results file in use. Set RQVAE_TUNABLE_GEMM=0 to
    keep the default library heuristic."""
    if os.environ.get("RQVAE_TUNABLE_GEMM", "1") == "0":
        return ""
    import tempfile
    import torch.cuda.tunable as tunable
    path = results_file or os.environ.get("RQVAE_TUNABLEOP_FILE", DEFAULT_FILE)
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    # one writer per table: under a multi-process launch only rank 0 writes the shared table at exit; every
    # other rank reads it and keeps what it tunes itself in a file of its own outside the tree (N processes
    # rewriting one CSV at exit could leave it torn for the next run)
    rank = int(os.environ.get("RANK", "0") or 0)
    own = path if rank == 0 else os.path.join(tempfile.gettempdir(), f"rqvae_tunableop_rank{rank}.csv")
    tunable.set_filename(own, insert_device_ordinal=False)
    tunable.set_max_tuning_duration(int(max_tuning_ms))
    tunable.tuning_enable(bool(tune_new_shapes))
    tunable.enable(True)
    if os.path.exists(path):
        tunable.read_file(path)
    return own


def bucket_rows(n: int, bucket: int = ROW_BUCKET) -> int:
    return (n + bucket - 1) // bucket * bucket


def is_enabled() -> bool:
    return torch.cuda.is_available() and torch.cuda.tunable.is_enabled()
