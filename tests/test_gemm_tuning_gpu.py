"""Library-GEMM selection (rqvae_hip.gemm_tuning): TunableOp picks a solution per shape, records it
in the results table, and the Linear layers compute the same fp32 result as the default path."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_tunable_gemm_linear(device, tmp_path, monkeypatch):
    import torch.cuda.tunable as tunable
    from rqvae_hip import gemm_tuning
    from modules.linear import Linear
    monkeypatch.setenv("RQVAE_TUNABLE_GEMM", "1")
    g = torch.Generator(device=device).manual_seed(0)
    lin = Linear(512, 256, bias=False).to(device)
    x = torch.randn(4096, 512, device=device, generator=g).requires_grad_(True)
    gy = torch.randn(4096, 256, device=device, generator=g)
    y_ref = torch.nn.functional.linear(x, lin.weight)
    gx_ref = gy @ lin.weight
    path = gemm_tuning.enable(str(tmp_path / "results.csv"), max_tuning_ms=5)
    try:
        assert path and tunable.is_enabled() and gemm_tuning.is_enabled()
        y = lin(x)
        y.backward(gy)
        torch.cuda.synchronize()
        torch.testing.assert_close(y, y_ref, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(x.grad, gx_ref, rtol=1e-5, atol=1e-5)
        results = tunable.get_results()
        assert any("4096" in str(r) or "512" in str(r) for r in results), results
    finally:
        tunable.tuning_enable(False)
        tunable.enable(False)
    assert os.path.dirname(path) == str(tmp_path)
