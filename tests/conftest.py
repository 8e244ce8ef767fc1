import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "rq-vae-recommender_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG, GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)
# library-GEMM tuning (rqvae_hip.gemm_tuning) times every candidate solution per new shape: the
# suite's many tiny shapes would spend minutes tuning, so it runs on the default heuristic except
# in the test that exercises the tuning itself
os.environ.setdefault("RQVAE_TUNABLE_GEMM", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")


@pytest.fixture(autouse=True)
def exact_matmul_precision():
    """Each test starts at 'highest' (exact fp32 matmuls), whatever an earlier import set: the
    reference's modules set 'high' at import (modules/rqvae.py:19, modules/model.py:27) and so do
    ours. Tests of the 'high' (split-bf16) path set it themselves."""
    import torch
    import modules.model  # noqa: F401  (import-time precision side effect happens before the test)
    import modules.rqvae  # noqa: F401
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    yield
    torch.set_float32_matmul_precision(prev)


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
        return cache[name]

    return load


@pytest.fixture(scope="session")
def device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)
