"""Host logic of rqvae_hip.optim.AdamW (CPU-only): no CPU fallback, hyper-parameter validation, and
the torch.optim.AdamW state-dict layout (train_rqvae.py:96-100,209-221 checkpoint the optimizer)."""
import os

import pytest
import torch


@pytest.fixture
def hip_optim():
    from rqvae_hip import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    from rqvae_hip import optim
    return optim


def test_cpu_params_fail_loudly(hip_optim):
    from rqvae_hip import RqHipError
    p = torch.nn.Parameter(torch.ones(4))
    p.grad = torch.ones(4)
    opt = hip_optim.AdamW([p], lr=1e-3)
    with pytest.raises(RqHipError):
        opt.step()
    assert torch.equal(p.detach(), torch.ones(4))


@pytest.mark.parametrize("kw", [dict(lr=-1.0), dict(betas=(1.0, 0.9)), dict(amsgrad=True), dict(maximize=True)])
def test_rejects_unsupported_settings(hip_optim, kw):
    from rqvae_hip import RqHipError
    with pytest.raises((ValueError, RqHipError)):
        hip_optim.AdamW([torch.nn.Parameter(torch.ones(2))], **kw)


def test_param_group_defaults_match_torch(hip_optim):
    ps = [torch.nn.Parameter(torch.ones(2))]
    ours = hip_optim.AdamW(ps, lr=5e-4, weight_decay=0.01).state_dict()["param_groups"][0]
    ref = torch.optim.AdamW(ps, lr=5e-4, weight_decay=0.01).state_dict()["param_groups"][0]
    for k in ("lr", "betas", "eps", "weight_decay", "amsgrad", "maximize", "params"):
        assert ours[k] == ref[k], k
