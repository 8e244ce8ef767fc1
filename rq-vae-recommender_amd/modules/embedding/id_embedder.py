"""Token embedders — reference semantics: modules/embedding/id_embedder.py:14-53.

SemIdEmbedder: one table of sem_ids_dim*K + 1 rows; token (type t, id s) -> row t*K + s;
padded positions (seq_mask False) -> the padding row (index sem_ids_dim*K, padding_idx).
UserIdEmbedder: user_id mod num_buckets -> row of a num_buckets table.
"""
from typing import NamedTuple

import torch
from torch import nn
from torch import Tensor

from rqvae_hip import ops as hip_ops

# False: gather cat([seq, fut]) and slice (the unpaired form; tests / A-B probes set the attribute)
_EMB_PAIR = True


class Embedding(nn.Embedding):
    """nn.Embedding (same parameter, init and state-dict key) whose backward on the device is the
    deterministic segmented sum rqvae_hip.ops.embedding (sort by index, fixed-order row sums) instead
    of torch's sort + scatter kernels."""

    def forward(self, idx: Tensor) -> Tensor:
        if hip_ops.embedding_supported(self.weight) and idx.is_cuda and self.max_norm is None:
            return hip_ops.embedding(idx, self.weight, self.padding_idx)
        return super().forward(idx)


class SemIdEmbeddingBatch(NamedTuple):
    seq: Tensor
    fut: Tensor


class SemIdEmbedder(nn.Module):
    def __init__(self, num_embeddings, sem_ids_dim, embeddings_dim) -> None:
        super().__init__()
        self.sem_ids_dim = sem_ids_dim
        self.num_embeddings = num_embeddings
        self.padding_idx = sem_ids_dim * num_embeddings
        self.emb = Embedding(num_embeddings=self.padding_idx + 1, embedding_dim=embeddings_dim,
                             padding_idx=self.padding_idx)

    def _rows(self, type_ids, sem_ids):
        return type_ids * self.num_embeddings + sem_ids

    def forward(self, batch) -> SemIdEmbeddingBatch:
        rows = torch.where(batch.seq_mask, self._rows(batch.token_type_ids, batch.sem_ids),
                           torch.full_like(batch.sem_ids, self.padding_idx))
        if batch.sem_ids_fut is None:
            return SemIdEmbeddingBatch(seq=self.emb(rows), fut=None)
        fut_rows = self._rows(batch.token_type_ids_fut, batch.sem_ids_fut)
        w = self.emb.weight
        if _EMB_PAIR and hip_ops.embedding_supported(w) and rows.is_cuda and self.emb.max_norm is None:
            # one backward reduction for the context and future tokens of the table (no slice backward)
            seq, fut = hip_ops.embedding_pair(rows, fut_rows, w, self.padding_idx)
            return SemIdEmbeddingBatch(seq=seq, fut=fut)
        N = rows.shape[1]
        both = self.emb(torch.cat([rows, fut_rows], dim=1))
        return SemIdEmbeddingBatch(seq=both[:, :N], fut=both[:, N:])


class UserIdEmbedder(nn.Module):
    def __init__(self, num_buckets, embedding_dim) -> None:
        super().__init__()
        self.num_buckets = num_buckets
        self.emb = Embedding(num_buckets, embedding_dim)

    def forward(self, x: Tensor) -> Tensor:
        return self.emb(torch.remainder(x, self.num_buckets))
