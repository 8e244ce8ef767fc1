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
    item is the target (reference :139-146); eval uses the last max_seq_len items."""

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
        lens = g.integers(4, 2 * self._max_seq_len, size=self.n_users)
        self.histories = [g.integers(0, self.n_items, size=int(l)) for l in lens]
        self.split = "train" if is_train else "test"

    @property
    def max_seq_len(self):
        return self._max_seq_len

    def __len__(self):
        return self.n_users

    def __getitem__(self, idx):
        seq = self.histories[idx]
        M = self._max_seq_len
        if self.subsample:
            start = int(self.rng.integers(0, max(0, len(seq) - 3) + 1))
            end = int(self.rng.integers(start + 3, start + M + 2))
            sample = list(seq[start:end])
        else:
            sample = list(seq[-(M + 1):])
        hist = sample[:-1]
        item_ids = torch.tensor(hist + [-1] * (M - len(hist)), dtype=torch.int64)
        fut = torch.tensor([sample[-1]], dtype=torch.int64)
        if not self.with_features:
            return SeqBatch(user_ids=torch.tensor([idx]), ids=item_ids, ids_fut=fut, x=torch.empty((M, 0)),
                            x_fut=torch.empty((1, 0)), seq_mask=item_ids >= 0)
        x = self.item_data[item_ids.clamp_min(0), :768]
        x[item_ids == -1] = -1
        return SeqBatch(user_ids=torch.tensor([idx]), ids=item_ids, ids_fut=fut, x=x,
                        x_fut=self.item_data[fut, :768], seq_mask=item_ids >= 0)


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
