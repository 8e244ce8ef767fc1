"""MI355X-native runtime for the RQ-VAE generative-retrieval training hot path.

`_lib`  ctypes binding of the C ABI (include/rqvae_hip.h -> librqvae_hip.so)
`ops`   autograd Functions: fused residual quantization, jagged conversion, varlen attention
`dp`    data-parallel engine (one process per GPU, RCCL all-reduce over xGMI)
"""
from ._lib import RqHipError, load  # noqa: F401
