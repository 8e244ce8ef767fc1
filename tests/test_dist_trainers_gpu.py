"""The drop-in trainers at world 2 on the HIP kernels (reference DDP path: train_rqvae.py:115-117,153,
train_decoder.py:171-173,196). A one-GPU box cannot host two RCCL ranks, so the two ranks share cuda:0
over gloo (RQVAE_DIST_BACKEND=gloo, RQVAE_SHARE_DEVICE=1): the real sharding (disjoint item slices,
token-balanced decoder shards and their shard weights), the bucketed exchange after every replayed step
graph and the rank-0 broadcasts all run, on the GPU kernels. The parameters after the first RQ-VAE step and
after 8 decoder steps, and both trainers' logged global-batch losses, must match a world-1 run at the same
global batch up to the summation order of the gradient (two half-batch sums + an all-reduce vs one
full-batch sum).

Both ranks start before either touches the GPU (separate processes; tools/dist_trainer_probe.py), each
under a timeout so a hung collective cannot outlive the test."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tools", "dist_trainer_probe.py")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, world, port):
    env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), RQVAE_DIST_BACKEND="gloo", RQVAE_SHARE_DEVICE="1", PYTHONUNBUFFERED="1")
    return env


def _run(world, out, tok=None, timeout=240):
    """(rank 0's loss lines, every rank's final JSON summary)."""
    port = _port()
    args = [sys.executable, PROBE, out] + ([tok] if tok else [])
    procs = [subprocess.Popen(args, env=_env(r, world, port), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for r in range(world)]
    res, lines = [], None
    try:
        for r, p in enumerate(procs):
            o, e = p.communicate(timeout=timeout)
            assert p.returncode == 0, e[-3000:]
            js = [json.loads(l) for l in o.splitlines() if l.startswith("{")]
            res.append(js[-1])
            if r == 0:
                lines = js
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return lines, res


def _params(path):
    return torch.load(path, map_location="cpu", weights_only=True)["model"]


def _rel_diff(a, b):
    """max over tensors of ||a - b|| / ||a||."""
    worst = 0.0
    for k, v in a.items():
        if not torch.is_floating_point(v):
            continue
        d = float((v.double() - b[k].double()).norm() / v.double().norm().clamp_min(1e-30))
        worst = max(worst, d)
    return worst


def test_trainers_world2_match_world1(tmp_path):
    import glob
    w1, w2 = str(tmp_path / "w1"), str(tmp_path / "w2")
    l1, r1 = _run(1, w1)
    tok = sorted(glob.glob(w1 + "/vae/checkpoint_*.pt"), key=lambda p: int(p.split("_")[-1][:-3]))[-1]
    l2, r2 = _run(2, w2, tok)
    assert r2[0]["rqvae"]["world"] == 2 and r2[0]["decoder"]["world"] == 2
    assert r2[0]["rqvae"]["step_mode"] == "hipgraph" and r2[0]["decoder"]["step_mode"] == "hipgraph"
    assert r1[0]["rqvae"]["batch_per_rank"] == 2 * r2[0]["rqvae"]["batch_per_rank"]
    # RQ-VAE: after the first step the two worlds differ only by the gradient's summation order
    d_vae0 = _rel_diff(_params(w1 + "/vae/checkpoint_0.pt"), _params(w2 + "/vae/checkpoint_0.pt"))
    dec1 = _params(sorted(glob.glob(w1 + "/dec/checkpoint_*.pt"))[-1])
    dec2 = _params(sorted(glob.glob(w2 + "/dec/checkpoint_*.pt"))[-1])
    d_dec = _rel_diff(dec1, dec2)
    rq = lambda ls: [l["loss"] for l in ls if "rl" in l]   # noqa: E731
    dc = lambda ls: [l["loss"] for l in ls if "lr" in l and "rl" not in l]   # noqa: E731
    rq1, rq2, dc1, dc2 = rq(l1), rq(l2), dc(l1), dc(l2)
    rel = lambda a, b: [abs(x - y) / abs(x) for x, y in zip(a, b)]   # noqa: E731
    print(json.dumps({"rqvae_rel_diff_step0": d_vae0, "decoder_rel_diff": d_dec, "rqvae_loss_rel": rel(rq1, rq2),
                      "decoder_loss_rel": rel(dc1, dc2)}))
    assert len(rq1) == len(rq2) == 7 and len(dc1) == len(dc2) == 8
    assert d_vae0 < 1e-4, d_vae0
    assert d_dec < 5e-5, d_dec
    assert max(rel(dc1, dc2)) < 1e-5
    # measured on MI355X: 0, 0, 6e-8, then up to 3.1e-4 (argmin near-ties flip between the worlds as the
    # summation-order differences grow); decoder losses <= 1.8e-7, parameters 9e-6 (profiles/r04)
    assert max(rel(rq1, rq2)[:3]) < 1e-6
    assert max(rel(rq1, rq2)) < 2e-3
