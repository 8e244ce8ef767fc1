"""Data-parallel engine on CPU with the gloo backend (world_size 2 and 3).

Checks: disjoint sharding of a global batch; rank-0 parameter broadcast; bucketed async
all-reduce (gradient-as-bucket-view, post-accumulate hooks) reproduces the single-process
gradient of the global-batch mean loss; parameters that receive no gradient are tolerated.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rqvae_hip import dp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        from modules.encoder import MLP
        self.mlp = MLP(24, [32, 16], 8, normalize=True)
        self.unused = torch.nn.Linear(4, 4, bias=False)   # like tte_fut / ffn_norm in the decoder

    def forward(self, x):
        return self.mlp(x)


def _loss(model, x):
    return ((model(x) - 0.1) ** 2).sum(-1).mean()


def _worker(rank, world, port, gb, bucket_bytes, q, grouped=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        r, w, _ = dp.init_from_env(backend="gloo")
        torch.manual_seed(100 + rank)          # different init per rank: broadcast must fix it
        model = _Net()
        if grouped:   # parameter groups in grad-ready order (the bench's RQ-VAE layout)
            ps = list(model.parameters())
            buckets = dp.GradBuckets([ps[len(ps) // 2:][::-1], ps[:len(ps) // 2][::-1]], bucket_bytes=bucket_bytes)
        else:
            buckets = dp.GradBuckets(model.parameters(), bucket_bytes=bucket_bytes)
        buckets.broadcast_params()
        g = torch.Generator().manual_seed(7)
        x = torch.randn(gb, 24, generator=g)
        a, b = dp.shard_range(gb, r, w)
        for _ in range(2):                     # two steps: zero_grad must reset the flat buffers
            buckets.zero_grad()
            _loss(model, x[a:b]).backward()
            buckets.synchronize()
        # numpy copies: tensors sent through a torch.multiprocessing queue are shared-memory handles
        # that die with this process (the parent may read after we exit)
        grads = {n: p.grad.detach().numpy().copy() for n, p in model.named_parameters()}
        params = {n: p.detach().numpy().copy() for n, p in model.named_parameters()}
        q.put((r, (a, b), params, grads, len(buckets.buckets)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world,gb,bucket_bytes,grouped", [(2, 64, 1 << 20, False), (3, 63, 2048, False),
                                                          (2, 64, 1 << 20, True)])
def test_bucketed_allreduce_matches_single_process(world, gb, bucket_bytes, grouped):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, gb, bucket_bytes, q, grouped)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # shards: disjoint, cover the global batch
    spans = [r[1] for r in res]
    assert spans[0][0] == 0 and spans[-1][1] == gb and all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    # params identical on all ranks (rank-0 broadcast)
    res = [(r[0], r[1], {n: torch.from_numpy(v) for n, v in r[2].items()},
            {n: torch.from_numpy(v) for n, v in r[3].items()}, r[4]) for r in res]
    for r in res[1:]:
        for n in r[2]:
            assert torch.equal(r[2][n], res[0][2][n])
    if bucket_bytes == 2048:
        assert res[0][4] > 1, "expected several buckets"
    # reference: single process, same params, mean over the shard means (equal shards when gb % world == 0)
    model = _Net()
    model.load_state_dict(res[0][2])
    g = torch.Generator().manual_seed(7)
    x = torch.randn(gb, 24, generator=g)
    total = sum(_loss(model, x[a:b]) for a, b in spans) / world
    total.backward()
    for n, p in model.named_parameters():
        got = res[0][3][n]
        ref = p.grad if p.grad is not None else torch.zeros_like(p)
        assert torch.allclose(got, ref, rtol=1e-5, atol=1e-7), n
        for r in res[1:]:
            assert torch.equal(r[3][n], got)


def test_shard_range_partitions():
    for gb in (1, 7, 64, 65536):
        for w in (1, 2, 3, 8):
            spans = [dp.shard_range(gb, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == gb
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
