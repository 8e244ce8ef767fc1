"""Dataset surface — reference data/processed.py (RecDataset :18-22, max-seq-len table :32-36,
ItemData :39-84, SeqData :87-166).

Raw-data ingestion (Amazon / MovieLens parsing, sentence-T5 text embeddings) is OUT of scope
(network model fetch): ItemData / SeqData here serve seeded synthetic corpora with the
reference's item / sequence semantics, or a local item-feature tensor file (`data_path` pointing
to a ``.npy`` / ``.pt`` tensor of shape (n_items, >=768); loaded with allow_pickle=False /
weights_only=True). `RecDataset` keeps the gin-constant module path ``data.processed.RecDataset``.
"""
import os
from enum import Enum
from typing import Optional

import numpy as np
import torch
from torch.utils.data import Dataset

from data.schemas import SeqBatch, TokenizedSeqBatch
from ops.jagged import register_row_counts


class RecDataset(Enum):
    AMAZON = 1
    ML_1M = 2
    ML_32M = 3


from modules.ginlite import gin as _gin   # noqa: E402  (gin-config or the built-in subset)

_gin.constants_from_enum(RecDataset, module="data.processed")

DATASET_NAME_TO_MAX_SEQ_LEN = {RecDataset.AMAZON: 20, RecDataset.ML_1M: 200, RecDataset.ML_32M: 200}
# public corpus sizes used for the synthetic stand-ins
SYNTHETIC_N_ITEMS = {RecDataset.AMAZON: 12101, RecDataset.ML_1M: 3706, RecDataset.ML_32M: 87585}
SYNTHETIC_N_USERS = {RecDataset.AMAZON: 22363, RecDataset.ML_1M: 6040, RecDataset.ML_32M: 200948}
# Synthetic history lengths per dataset: U{lo..hi-1} items (None: U{4..2 max_seq_len - 1}). bench.py sets
# AMAZON to (3, 22) for its trainer line: with train_data_subsample=False every window is the whole
# history, i.e. U{2..20} context items per sequence — the length distribution of its decoder step.
SYNTHETIC_HIST_LEN = {}


def synthetic_items(n: int, dim: int = 768, seed: int = 0) -> torch.Tensor:
    """Rows ~ N(0, I) then L2-normalised (sentence-T5 embeddings are unit norm)."""
    g = np.random.Generator(np.random.PCG64(seed))
    x = g.standard_normal((n, dim), dtype=np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    return torch.from_numpy(x)


class ItemData(Dataset):
    def __init__(self, root: str = "", *args, force_process: bool = False, dataset: RecDataset = RecDataset.ML_1M,
                 train_test_split: str = "all", data_path: Optional[str] = None, seed: int = 0,
                 eval_fraction: float = 0.05, **kwargs) -> None:
        path = data_path if data_path is not None else root
        feats = None
        if path and os.path.isfile(path):
            if path.endswith(".npy"):
                feats = torch.from_numpy(np.load(path, allow_pickle=False)).float()
            else:
                feats = torch.load(path, map_location="cpu", weights_only=True).float()
        if feats is None:
            feats = synthetic_items(SYNTHETIC_N_ITEMS[dataset], 768, seed)
        n = feats.shape[0]
        is_train = torch.from_numpy(np.random.Generator(np.random.PCG64(seed + 1)).random(n) >= eval_fraction)
        keep = {"train": is_train, "eval": ~is_train}.get(train_test_split, torch.ones(n, dtype=torch.bool))
        self.item_data = feats[keep]
        self.item_text = None

    def __len__(self):
        return self.item_data.shape[0]

    def __getitem__(self, idx):
        item_ids = torch.tensor(idx).unsqueeze(0) if not isinstance(idx, torch.Tensor) else idx
        neg = -torch.ones_like(item_ids.squeeze(0))
        return SeqBatch(user_ids=neg, ids=item_ids, ids_fut=neg, x=self.item_data[idx, :768], x_fut=neg,
                        seq_mask=torch.ones_like(item_ids, dtype=torch.bool))


class SeqData(Dataset):
    """User histories. Training samples a random sub-window of 3..max_seq_len+1 items whose last
    item is the target (reference :139-146); eval uses the last max_seq_len items.

    Indexing with an int returns one sample (the reference's per-item form, collated by the
    DataLoader); indexing with a list / array of ints returns the collated SeqBatch of those samples
    in one vectorised numpy pass — the same fields, shapes and sub-window draws as collating THIS
    class's per-item samples (`__getitem__([i, j])` == default_collate([self[i], self[j]]) for the same
    rng state). The window bounds follow the reference's distribution, not its random stream; and since
    round 4 (uniform floats per sample, one flat draw of the synthetic histories) a given seed yields a
    different synthetic corpus and windows than earlier rounds, so their logged losses are not
    comparable. The reference fetches and collates per item (~12 ms per 256-sequence batch on this host,
    slower than the decoder's GPU step); `batch_loader` drives the batched form with the reference
    DataLoader's sampling order."""

    def __init__(self, root: str = "", *args, is_train: bool = True, subsample: bool = False,
                 force_process: bool = False, dataset: RecDataset = RecDataset.ML_1M, data_path: Optional[str] = None,
                 n_users: Optional[int] = None, n_items: Optional[int] = None, seed: int = 0,
                 with_features: bool = True, **kwargs) -> None:
        """`with_features=False` (this build's extension): samples carry empty (., 0) `x` / `x_fut` instead of
        the items' 768-d features — for consumers that only read ids (the decoder trainer: its tokenizer maps
        ids to cached semantic ids, reference modules/tokenizer/semids.py:137-153), which saves the per-item
        feature gather, the collate of (B, M, 768) floats and their host-to-device copy every step."""
        assert (not subsample) or is_train, "Can only subsample on training split."
        self.with_features = with_features
        self._max_seq_len = DATASET_NAME_TO_MAX_SEQ_LEN[dataset]
        self.subsample = subsample
        self.n_items = n_items or SYNTHETIC_N_ITEMS[dataset]
        self.n_users = n_users or SYNTHETIC_N_USERS[dataset]
        self.item_data = synthetic_items(self.n_items, 768, seed)
        self.rng = np.random.Generator(np.random.PCG64(seed + 2))
        g = np.random.Generator(np.random.PCG64(seed + 3))
        # histories as one flat item array + per-user offsets (user u: flat[off[u]:off[u+1]])
        lo, hi = SYNTHETIC_HIST_LEN.get(dataset) or (4, 2 * self._max_seq_len)
        self.hist_len = g.integers(lo, hi, size=self.n_users)
        self.hist_off = np.concatenate([[0], np.cumsum(self.hist_len)])
        self.hist_flat = g.integers(0, self.n_items, size=int(self.hist_off[-1]))
        self.split = "train" if is_train else "test"

    @property
    def max_seq_len(self):
        return self._max_seq_len

    def __len__(self):
        return self.n_users

    def history(self, u: int) -> np.ndarray:
        return self.hist_flat[self.hist_off[u]:self.hist_off[u + 1]]

    def _windows(self, users: np.ndarray):
        """Per sample: the window [start, stop) of the user's history (its last item is the target).
        Training sub-windows (reference :139-146): start ~ U{0..len-3}, end ~ U{start+3..start+M+1},
        stop = min(end, len) — drawn for all samples at once from two uniforms per sample."""
        n = self.hist_len[users]
        M = self._max_seq_len
        if self.subsample:
            u = self.rng.random((len(users), 2))
            start = np.minimum((u[:, 0] * (np.maximum(n - 3, 0) + 1)).astype(np.int64), np.maximum(n - 3, 0))
            end = start + 3 + np.minimum((u[:, 1] * (M - 1)).astype(np.int64), M - 2)
            stop = np.minimum(end, n)
        else:
            stop = n
            start = np.maximum(n - (M + 1), 0)
        return start, stop

    def _collate(self, users: np.ndarray) -> SeqBatch:
        M = self._max_seq_len
        B = len(users)
        start, stop = self._windows(users)
        n_hist = stop - start - 1                                     # history items before the target
        col = np.arange(M)[None, :]
        mask = col < n_hist[:, None]
        pos = self.hist_off[users][:, None] + start[:, None] + col
        ids = np.where(mask, self.hist_flat[np.where(mask, pos, 0)], -1)
        fut = self.hist_flat[self.hist_off[users] + stop - 1][:, None]
        t = torch.from_numpy
        item_ids, fut_t = t(ids.astype(np.int64)), t(fut.astype(np.int64))
        user_ids = t(users.astype(np.int64)[:, None])
        if not self.with_features:
            return SeqBatch(user_ids=user_ids, ids=item_ids, ids_fut=fut_t, x=torch.empty((B, M, 0)),
                            x_fut=torch.empty((B, 1, 0)), seq_mask=t(mask))
        x = self.item_data[item_ids.clamp_min(0), :768]
        x[item_ids == -1] = -1
        return SeqBatch(user_ids=user_ids, ids=item_ids, ids_fut=fut_t, x=x, x_fut=self.item_data[fut_t, :768],
                        seq_mask=t(mask))

    def __getitem__(self, idx):
        if isinstance(idx, (int, np.integer)) or (isinstance(idx, torch.Tensor) and idx.dim() == 0):
            b = self._collate(np.array([int(idx)], dtype=np.int64))
            return SeqBatch(*[v[0] for v in b])
        return self._collate(np.asarray(idx, dtype=np.int64).reshape(-1))


def batch_loader(ds, batch_size: int, generator: torch.Generator) -> torch.utils.data.DataLoader:
    """DataLoader(ds, batch_size, shuffle=True, generator=generator) with the batches fetched whole:
    the same RandomSampler / BatchSampler index order, one `ds[indices]` call per batch (a dataset
    whose list indexing returns the collated batch, e.g. SeqData) instead of per-item fetch + collate."""
    from torch.utils.data import BatchSampler, DataLoader, RandomSampler
    sampler = BatchSampler(RandomSampler(ds, generator=generator), batch_size, drop_last=False)
    # generator= as well: the loader iterator draws its base seed from it before the sampler's first draw
    return DataLoader(ds, batch_size=None, sampler=sampler, collate_fn=lambda b: b, generator=generator)


def synthetic_tokenized_batch(B: int, max_items: int, sem_id_dim: int, K: int, seed: int, device,
                              min_items: int = 2) -> TokenizedSeqBatch:
    """Decoder-train batch of the shape SemanticIdTokenizer.forward produces (semids.py:137-153):
    n_items ~ U{min..max}; sem ids ~ U[0, K) (dedup column 0); padded tokens -1; user ids ~ U[0, 1e6)."""
    g = np.random.Generator(np.random.PCG64(seed))
    n = g.integers(min_items, max_items + 1, size=B)
    N = max_items * sem_id_dim
    mask = np.arange(N)[None, :] < (n * sem_id_dim)[:, None]
    sem = g.integers(0, K, size=(B, N))
    sem[:, sem_id_dim - 1::sem_id_dim] = 0
    sem = np.where(mask, sem, -1)
    fut = g.integers(0, K, size=(B, sem_id_dim))
    fut[:, -1] = 0
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
    batch = TokenizedSeqBatch(user_ids=t(g.integers(0, 10 ** 6, size=(B, 1))), sem_ids=t(sem), sem_ids_fut=t(fut),
                              seq_mask=t(mask), token_type_ids=t(np.tile(np.arange(sem_id_dim), (B, max_items))),
                              token_type_ids_fut=t(np.tile(np.arange(sem_id_dim), (B, 1))))
    register_row_counts(batch.seq_mask, mask.sum(axis=1))   # built on the host: lengths known, no sync later
    return batch
