"""Host-side data path of the decoder trainer (CPU): SeqData's batched fetch against the reference's
per-item fetch + default collate (reference data/processed.py:136-166), the batch loader's order against
DataLoader(shuffle=True) with the same generator, and the trainer's prefetch thread shutting down."""
import copy

import numpy as np
import pytest
import torch
from torch.utils.data import DataLoader
from torch.utils.data._utils.collate import default_collate


@pytest.mark.parametrize("with_features", [False, True])
@pytest.mark.parametrize("subsample", [False, True])
def test_seqdata_batched_equals_collated_items(with_features, subsample):
    from data.processed import RecDataset, SeqData
    ds = SeqData(dataset=RecDataset.AMAZON, is_train=True, subsample=subsample, with_features=with_features)
    ds2 = copy.deepcopy(ds)   # same rng state
    idx = [5, 0, 17, 22362, 3, 3, 911]
    a = ds[idx]
    b = default_collate([ds2[i] for i in idx])
    for f in a._fields:
        x, y = getattr(a, f), getattr(b, f)
        assert x.shape == y.shape and x.dtype == y.dtype and torch.equal(x, y), f


def test_seqdata_windows_follow_reference_sampler():
    """Sub-windows: start in [0, len-3], end in [start+3, start+M+1] (random.randint bounds of the
    reference), history = window[:-1] padded with -1, target = window[-1]; eval = last M+1 items."""
    from data.processed import RecDataset, SeqData
    M = 20
    for subsample in (True, False):
        ds = SeqData(dataset=RecDataset.AMAZON, is_train=True, subsample=subsample, with_features=False)
        users = np.arange(0, ds.n_users, 3)
        b = ds[users]
        ids, fut, mask = b.ids.numpy(), b.ids_fut.numpy()[:, 0], b.seq_mask.numpy()
        assert ids.shape == (len(users), M) and (mask == (ids >= 0)).all()
        n_hist = mask.sum(1)
        assert (n_hist >= 2).all() and (n_hist <= M).all()
        for r, u in enumerate(users[:500]):
            h = ds.history(int(u))
            k = n_hist[r]
            if subsample:
                # the window is a contiguous run of the history ending at the target
                found = [s for s in range(0, max(0, len(h) - 3) + 1)
                         if s + k < len(h) and (h[s:s + k] == ids[r, :k]).all() and h[s + k] == fut[r]]
                assert found, (u, h, ids[r], fut[r])
            else:
                w = h[-(M + 1):]
                assert (ids[r, :k] == w[:-1]).all() and fut[r] == w[-1] and k == len(w) - 1
        assert (b.user_ids.numpy()[:, 0] == users).all()


def test_batch_loader_order_matches_dataloader():
    from data.processed import RecDataset, SeqData, batch_loader
    ds = SeqData(dataset=RecDataset.AMAZON, is_train=True, subsample=False, with_features=False)
    a = batch_loader(ds, 256, torch.Generator().manual_seed(7))
    b = DataLoader(ds, batch_size=256, shuffle=True, generator=torch.Generator().manual_seed(7))
    for _, (x, y) in zip(range(3), zip(a, b)):
        for f in x._fields:
            assert torch.equal(getattr(x, f), getattr(y, f)), f


def test_prefetch_close_joins_thread():
    import train_decoder
    from data.processed import RecDataset, SeqData, batch_loader
    from data.utils import cycle
    ds = SeqData(dataset=RecDataset.AMAZON, is_train=True, subsample=True, with_features=False)
    feed = train_decoder._Prefetch(cycle(batch_loader(ds, 64, torch.Generator().manual_seed(1))), 0, 1, 4)
    data, counts, n_glob, ids_max = feed.next()
    assert n_glob == 64 and len(counts) == 64 and sum(counts) == int(data.seq_mask.sum()) * 4
    assert ids_max == int(max(data.ids.max(), data.ids_fut.max()))
    feed.close()
    assert not feed.thread.is_alive()
