"""Data-parallel engine on CPU with the gloo backend (world_size 2 and 3).

Checks: disjoint sharding of a global batch; rank-0 parameter broadcast; bucketed async
all-reduce (gradient-as-bucket-view, post-accumulate hooks) reproduces the single-process
gradient of the GLOBAL-batch mean loss — with equal shards, unequal shards (remainder rows,
dp.shard_weight), token-balanced variable-length shards (dp.balanced_partition) and gradient
accumulation (no_sync on all but the last micro-batch); parameters unused on every rank keep
grad None exactly as with one process, so AdamW steps give identical parameters at 1 and N ranks;
corpus all-gather (dp.all_gather_rows); the graphed step's in-graph exchange logic
(rqvae_hip.graph.GraphedSteps with capture=False: the bodies that a GPU run captures, run eagerly, with
the buckets' all-reduces launched from the hooks inside the body and finished at its end); a rank
whose shard is empty (global batch < world) with buckets whose grad-ready order is not their index
order (collectives must still be issued in the same order on every rank).
"""
import os
import socket

import numpy as np
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


class _DirectLinear(torch.autograd.Function):
    """y = x W^T whose weight gradient is added straight into W's flat bucket view when GradBuckets owns
    one (dp.direct_grad — what the HIP GEMMs do on the GPU) and handed to autograd as None."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x @ w.t()

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        sink = dp.direct_grad(w)
        if sink is None:
            return g @ w, g.t() @ x
        sink.add_(g.t() @ x)
        dp.direct_grad_done(w)
        return g @ w, None


class _TiedNet(torch.nn.Module):
    """One weight used by two direct-gradient ops per forward (and a plain Linear after them)."""

    def __init__(self):
        super().__init__()
        self.w = torch.nn.Parameter(torch.randn(24, 24) * 0.2)
        self.head = torch.nn.Linear(24, 8, bias=False)

    def forward(self, x):
        return self.head(torch.tanh(_DirectLinear.apply(torch.tanh(_DirectLinear.apply(x, self.w)), self.w)))


def _loss(model, x):
    """Per-row loss, mean over the rows (the reference's mean over the batch)."""
    return ((model(x) - 0.1) ** 2).sum(-1).mean()


def _seq_loss(model, x, lengths):
    """Variable-length 'sequences' (rows of x grouped by lengths): per-sequence sum over its tokens,
    mean over the sequences — the decoder's CE summed over positions and averaged over B."""
    per_tok = ((model(x) - 0.1) ** 2).sum(-1)
    off = np.concatenate([[0], np.cumsum(lengths)])
    per_seq = torch.stack([per_tok[off[i]:off[i + 1]].sum() for i in range(len(lengths))])
    return per_seq.mean()


def _data(gb):
    g = torch.Generator().manual_seed(7)
    x = torch.randn(gb, 24, generator=g)
    lengths = torch.randint(1, 9, (gb,), generator=g).tolist()
    toks = torch.randn(sum(lengths), 24, generator=g)
    return x, lengths, toks


def _seq_slice(toks, lengths, idx):
    off = np.concatenate([[0], np.cumsum(lengths)])
    rows = torch.cat([toks[off[i]:off[i + 1]] for i in idx])
    return rows, [lengths[i] for i in idx]


def _worker(rank, world, port, gb, bucket_bytes, q, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        r, w, _ = dp.init_from_env(backend="gloo")
        torch.manual_seed(100 + rank)          # different init per rank: broadcast must fix it
        model = _TiedNet() if mode == "tied" else _Net()
        if mode == "grouped":   # parameter groups in grad-ready order (the bench's RQ-VAE layout)
            ps = list(model.parameters())
            buckets = dp.GradBuckets([ps[len(ps) // 2:][::-1], ps[:len(ps) // 2][::-1]], bucket_bytes=bucket_bytes)
        elif mode == "empty":   # buckets in forward order: the last bucket's grads are ready first
            buckets = dp.GradBuckets([list(model.parameters())], bucket_bytes=bucket_bytes)
        elif mode in ("graphed", "graphed_mixed", "graphed_agree", "tied"):
            buckets = dp.GradBuckets(model.parameters(), bucket_bytes=bucket_bytes, flat_views=True)
        else:
            buckets = dp.GradBuckets(model.parameters(), bucket_bytes=bucket_bytes)
        buckets.broadcast_params()
        opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.1)
        x, lengths, toks = _data(gb)
        a, b = dp.shard_range(gb, r, w)
        mine = dp.balanced_partition(lengths, w)[r]
        gs = None
        if mode == "graphed":
            from rqvae_hip.graph import GraphedSteps
            gs = GraphedSteps(lambda xb: _loss(model, xb) * dp.shard_weight(b - a, gb), lambda xb: 0, buckets,
                              capture=False, in_graph_exchange=True)
        elif mode == "graphed_mixed":
            # ranks disagree step by step: rank 0 keeps one key (probe, capture with the
            # in-body exchange, replay); rank 1 sees a new key every step with max_graphs=1 and its
            # capture of the exchange fails (probe, graph without the exchange + post-replay exchange,
            # then an eager step past max_graphs). Every rank must still run the same collectives.
            from rqvae_hip.graph import GraphedSteps
            step = [0]
            gs = GraphedSteps(lambda xb: _loss(model, xb) * dp.shard_weight(b - a, gb),
                              lambda xb: step[0] if r == 1 else 0, buckets, capture=False, in_graph_exchange=True,
                              max_graphs=1, local_fallback=True)
            if r == 1:
                orig = gs._try_capture
                gs._try_capture = lambda in_graph: ((None, None, RuntimeError("simulated capture failure"))
                                                    if in_graph else orig(in_graph))
        elif mode == "graphed_agree":
            # rank 1's FIRST capture of the exchange fails: the MIN all-reduce at the job's first capture
            # moves every rank's exchange after the replay (no rank keeps collectives in a graph)
            from rqvae_hip.graph import GraphedSteps
            gs = GraphedSteps(lambda xb: _loss(model, xb) * dp.shard_weight(b - a, gb), lambda xb: 0, buckets,
                              capture=False, in_graph_exchange=True)
            if r == 1:
                orig = gs._try_capture
                gs._try_capture = lambda in_graph: ((None, None, RuntimeError("simulated capture failure"))
                                                    if in_graph else orig(in_graph))
        for _ in range(_steps(mode)):          # >= two steps: zero_grad must reset the flat buffers
            if gs is not None:                 # step 1: eager probe; step 2: warm-ups + the in-body exchange
                gs(x[a:b].clone())
                assert gs.graphs or _ == 0
                if mode == "graphed_mixed":
                    step[0] += 1
                buckets.synchronize()
                grads = {n: (None if p.grad is None else p.grad.detach().numpy().copy())
                         for n, p in model.named_parameters()}
                opt.step()
                continue
            buckets.zero_grad()
            if mode == "empty":
                rows, lens = _seq_slice(toks, lengths, mine) if mine else (None, [])
                if mine:
                    (_seq_loss(model, rows, lens) * dp.shard_weight(len(mine), gb)).backward()
            elif mode == "accum":                # two micro-batches: the global batch, then its reverse
                for micro, xb in enumerate((x[a:b], x.flip(0)[a:b])):
                    loss = _loss(model, xb) * dp.shard_weight(b - a, gb) / 2
                    if micro == 0:
                        with buckets.no_sync():
                            loss.backward()
                        assert not buckets._pending, "no_sync must not start the exchange"
                    else:
                        loss.backward()
            elif mode == "tokens":             # token-balanced shards of variable-length sequences
                rows, lens = _seq_slice(toks, lengths, mine)
                (_seq_loss(model, rows, lens) * dp.shard_weight(len(mine), gb)).backward()
            else:
                (_loss(model, x[a:b]) * dp.shard_weight(b - a, gb)).backward()
            buckets.synchronize()
            grads = {n: (None if p.grad is None else p.grad.detach().numpy().copy()) for n, p in model.named_parameters()}
            opt.step()
        # numpy copies: tensors sent through a torch.multiprocessing queue are shared-memory handles
        # that die with this process (the parent may read after we exit)
        params = {n: p.detach().numpy().copy() for n, p in model.named_parameters()}
        if mode == "graphed_mixed":
            assert (gs.in_graph, gs.eager_steps, len(gs.graphs)) == ((True, 1, 1) if r == 0 else (False, 2, 1))
        if mode == "graphed_agree":
            assert not gs.in_graph and [e[2] for e in gs.graphs.values()] == [False]
        q.put((r, (a, b), params, grads, len(buckets.buckets), mine))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _steps(mode):
    return 3 if mode == "graphed_mixed" else 2


def _run(world, gb, bucket_bytes, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, gb, bucket_bytes, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _single_process(state0, gb, mode, world):
    """Same two steps in one process: params after the first step + grads of the second step."""
    model = _TiedNet() if mode == "tied" else _Net()
    model.load_state_dict(state0)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.1)
    x, lengths, toks = _data(gb)
    grads = None
    for _ in range(_steps(mode)):
        opt.zero_grad(set_to_none=True)
        if mode == "accum":
            ((_loss(model, x) + _loss(model, x.flip(0))) / 2).backward()
        elif mode in ("tokens", "empty"):
            _seq_loss(model, toks, lengths).backward()
        else:
            _loss(model, x).backward()
        grads = {n: p.grad for n, p in model.named_parameters()}
        opt.step()
    return model, grads


@pytest.mark.parametrize("world,gb,bucket_bytes,mode", [
    (2, 64, 1 << 20, "plain"),      # equal shards
    (3, 64, 2048, "plain"),         # unequal shards (22/21/21), several buckets
    (2, 63, 1 << 20, "grouped"),    # unequal shards, grouped buckets
    (2, 64, 1 << 20, "accum"),      # gradient accumulation with no_sync
    (3, 61, 4096, "tokens"),        # token-balanced variable-length shards (unequal sequence counts)
    (3, 2, 2048, "empty"),          # global batch < world: rank 2 has no sequences, several buckets
    (2, 64, 2048, "graphed"),       # GraphedSteps bodies with the in-graph exchange (run eagerly)
    (2, 64, 2048, "graphed_mixed"),  # ranks with different keys / capture outcomes / eager fallbacks
    (2, 64, 2048, "graphed_agree"),  # one rank's first capture fails: every rank exchanges after the replay
    (2, 64, 1024, "tied"),          # one weight, two direct-gradient contributions per backward
])
def test_bucketed_allreduce_matches_single_process(world, gb, bucket_bytes, mode):
    res = _run(world, gb, bucket_bytes, mode)
    if mode == "empty":
        assert [len(r[5]) for r in res] == [1, 1, 0]
    if mode not in ("tokens", "empty"):   # contiguous shards: disjoint, cover the global batch
        spans = [r[1] for r in res]
        assert spans[0][0] == 0 and spans[-1][1] == gb and all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    else:                  # token-balanced shards: a partition of the sequences
        allidx = sorted(i for r in res for i in r[5])
        assert allidx == list(range(gb))
    if bucket_bytes == 2048:
        assert res[0][4] > 1, "expected several buckets"
    if mode == "empty":
        allidx = sorted(i for r in res for i in r[5])
        assert allidx == list(range(gb))
    # rank-0 broadcast + identical updates: parameters identical on all ranks after 2 AdamW steps
    for r in res[1:]:
        for n in r[2]:
            assert np.array_equal(r[2][n], res[0][2][n]), n
    # single process from the same initial parameters (rank 0's init after broadcast = seed 100)
    torch.manual_seed(100)
    state0 = (_TiedNet() if mode == "tied" else _Net()).state_dict()
    model, grads = _single_process(state0, gb, mode, world)
    for n, p in model.named_parameters():
        got = res[0][3][n]
        ref = grads[n]
        if ref is None:   # unused everywhere: grad None at N ranks as at 1 (AdamW skips it)
            assert got is None, n
            continue
        # 'empty': two 1-sequence shards summed with a zero shard and rescaled (fp32 rounding ~1e-7)
        assert torch.allclose(torch.from_numpy(got), ref, rtol=2e-5, atol=1e-6 if mode == "empty" else 1e-7), n
        for r in res[1:]:
            assert np.array_equal(r[3][n], got)
        assert np.allclose(res[0][2][n], p.detach().numpy(), rtol=1e-5, atol=1e-6), f"params {n}"
    if mode != "tied":
        assert np.array_equal(res[0][2]["unused.weight"], model.unused.weight.detach().numpy())


def test_shard_range_partitions():
    for gb in (1, 7, 64, 65536):
        for w in (1, 2, 3, 8):
            spans = [dp.shard_range(gb, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == gb
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_balanced_partition_properties():
    g = np.random.Generator(np.random.PCG64(3))
    for B, w, hi in [(256, 8, 81), (64, 8, 801), (7, 3, 10), (3, 4, 5), (1000, 2, 1281)]:
        costs = (4 * g.integers(1, hi // 4 + 1, size=B) + 1).tolist()
        bins = dp.balanced_partition(costs, w)
        assert sorted(i for b in bins for i in b) == list(range(B))
        assert all(b == sorted(b) for b in bins)
        loads = [sum(costs[i] for i in b) for b in bins]
        # longest-first greedy: the spread is at most the largest single cost
        assert max(loads) - min(loads) <= max(costs)
        assert bins == dp.balanced_partition(costs, w)   # deterministic


def _gather_worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        dp.init_from_env(backend="gloo")
        a, b = dp.shard_range(n, rank, world)
        full = torch.arange(n * 3, dtype=torch.int64).view(n, 3) * 7 % 101
        got = dp.all_gather_rows(full[a:b].clone(), n)
        q.put((rank, bool(torch.equal(got, full))))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 11), (3, 64), (3, 2)])
def test_all_gather_rows(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in res)


def test_graphed_steps_copy_in_mixed_dtypes():
    """GraphedSteps copies a nested batch into its static inputs with one foreach copy per dtype: every
    field (int64, bool, fp32, a lone tensor of its dtype, None) lands exactly, shapes / storage unchanged."""
    from collections import namedtuple
    from rqvae_hip.graph import GraphedSteps
    Batch = namedtuple("Batch", "a b mask x none nested")
    g = torch.Generator().manual_seed(0)

    def make():
        return Batch(torch.randint(0, 100, (4, 5), generator=g), torch.randint(0, 9, (3,), generator=g),
                     torch.rand(4, 5, generator=g) > 0.5, torch.randn(2, 3, generator=g), None,
                     (torch.randint(0, 7, (6,), generator=g), torch.randn(5, generator=g)))
    static, src = make(), make()
    ptrs = [t.data_ptr() for t in (static.a, static.b, static.mask, static.x, *static.nested)]
    GraphedSteps._copy(static, src)
    for d, s_ in ((static.a, src.a), (static.b, src.b), (static.mask, src.mask), (static.x, src.x),
                  (static.nested[0], src.nested[0]), (static.nested[1], src.nested[1])):
        assert torch.equal(d, s_) and d.dtype == s_.dtype
    assert ptrs == [t.data_ptr() for t in (static.a, static.b, static.mask, static.x, *static.nested)]


@pytest.mark.parametrize("world,fallback,fail_at", [(1, None, 1), (2, None, 1), (2, None, 2), (2, True, 2)])
def test_graphed_steps_capture_failure_policy(world, fallback, fail_at, monkeypatch):
    """A rank whose capture of the in-graph exchange fails. The job's first capture (call 2 on
    every rank) settles the placement for all ranks (a MIN all-reduce of the outcomes; single process here:
    the local outcome), so failing there falls back everywhere. A failure at a later capture (a new key)
    after the job agreed on in-graph exchange: world 1 or the opt-in local fallback record the graph without
    the collectives and exchange after the replay; world > 1 by default raises instead of silently replaying
    a different collective placement than its peers. Single process; the world size is what GraphedSteps sees."""
    from rqvae_hip.graph import GraphedSteps
    monkeypatch.delenv("RQVAE_LOCAL_EXCHANGE_FALLBACK", raising=False)
    torch.manual_seed(0)
    model = _Net()
    buckets = dp.GradBuckets(model.parameters(), flat_views=True)
    step = [0]
    gs = GraphedSteps(lambda xb: _loss(model, xb), lambda xb: step[0], buckets, capture=False, in_graph_exchange=True,
                      local_fallback=fallback)
    monkeypatch.setattr(GraphedSteps, "_world", staticmethod(lambda: world))
    orig = gs._try_capture
    gs._try_capture = lambda in_graph: ((None, None, RuntimeError("simulated capture failure"))
                                        if in_graph and len(gs.graphs) + 1 == fail_at else orig(in_graph))
    x = _data(16)[0]
    gs(x)                      # eager probe step
    buckets.synchronize()
    for n in range(1, 3):      # capture n (a new key each call)
        step[0] += 1
        if n == fail_at and world > 1 and not fallback and fail_at > 1:
            with pytest.raises(RuntimeError, match="cannot capture the gradient exchange"):
                gs(x)
            assert "simulated capture failure" in gs.capture_error
            return
        gs(x)
        buckets.synchronize()
        if n < fail_at:
            assert gs.in_graph and gs.capture_error is None
    assert not gs.in_graph and "simulated capture failure" in gs.capture_error and len(gs.graphs) == 2
    assert [e[2] for e in gs.graphs.values()] == [fail_at > 1, False]
