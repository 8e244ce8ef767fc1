"""ORACLE — CPU restatement of the reference's hot path. TEST INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import
anything from this package, and there only as the checker / the timed CPU baseline.
The product (`rq-vae-recommender_amd/`) never imports it and has no CPU fallback: its
ops raise when the HIP library is missing or a tensor is not on the GPU.

Every function cites the reference file:line it restates (reference =
AdamLTy/RQ-VAE-Recommender @ 2025-07-25). Parity of this restatement is PINNED against
golden vectors produced by importing the reference itself in the build container
(`tests/golden/make_golden.py`, fixtures `tests/golden/*.npz`), see
`tests/test_oracle.py`. Floating-point math is float32 numpy unless a docstring says
otherwise; integer/index work is exact.
"""
from . import quantize, jagged, attention, unique, rqvae, kmeans  # noqa: F401
