"""Semantic-ID tokenizer — drop-in for reference modules/tokenizer/semids.py (SemanticIdTokenizer
:23-154; same constructor, `cached_ids` layout (N, L+1) with the dedup column, forward contract).

MI355X path:
  * corpus ids: the frozen RqVae's eval-mode fused quantize kernel over the whole corpus in large
    device batches (the reference walks 512-item batches); with `shard=True` under data
    parallelism each rank quantizes its contiguous slice and the ids are all-gathered,
    the dedup column is then computed on the gathered corpus (identical on every rank);
  * dedup column (`semids.py:84-99`: for each item, the number of EARLIER items with the same
    L-tuple): one stable device sort of packed tuple keys + a segmented rank, O(N log N) instead
    of the reference's O(N^2) all-pairs comparison — identical values;
  * `exists_prefix`: sorted packed-prefix keys + binary search (torch.searchsorted) instead of
    the O(P x N) broadcast compare. `reference_batching=True` (default) reproduces the reference's
    batching quirk (`math.ceil(n // 16)` skips the last partial batch of 16 prefixes, which then
    report False; SURVEY A-12) so generation matches the reference; pass False for the fixed
    behaviour.
"""
import math
from typing import List, Optional

import torch
from torch import nn
from torch import Tensor

from data.schemas import SeqBatch, TokenizedSeqBatch
from modules.rqvae import RqVae
from modules.utils import eval_mode
from rqvae_hip import dp

BATCH_SIZE = 16
CORPUS_BATCH = 65536


def _pack(cols: Tensor, base: int) -> Tensor:
    """Rows of small non-negative ints -> int64 keys (lexicographic order preserved)."""
    key = torch.zeros(cols.shape[:-1], dtype=torch.int64, device=cols.device)
    for j in range(cols.shape[-1]):
        key = key * base + cols[..., j].to(torch.int64)
    return key


def dedup_rank(ids: Tensor) -> Tensor:
    """rank[i] = #{j < i : ids[j] == ids[i]} for an (N, L) integer tensor (stable sort + segmented rank)."""
    n = ids.shape[0]
    if n == 0:
        return torch.zeros(0, dtype=torch.int64, device=ids.device)
    base = int(ids.max().item()) + 1
    key = _pack(ids, base)
    sk, order = torch.sort(key, stable=True)
    pos = torch.arange(n, device=ids.device)
    first = torch.ones(n, dtype=torch.bool, device=ids.device)
    first[1:] = sk[1:] != sk[:-1]
    start = torch.cummax(torch.where(first, pos, torch.zeros_like(pos)), dim=0).values
    rank = torch.empty(n, dtype=torch.int64, device=ids.device)
    rank[order] = pos - start
    return rank


class SemanticIdTokenizer(nn.Module):
    """Tokenizes sequences of item features into sequences of semantic ids (L codewords + dedup)."""

    def __init__(self, input_dim: int, output_dim: int, hidden_dims: List[int], codebook_size: int, n_layers: int = 3,
                 n_cat_feats: int = 18, commitment_weight: float = 0.25, rqvae_weights_path: Optional[str] = None,
                 rqvae_codebook_normalize: bool = False, rqvae_sim_vq: bool = False) -> None:
        super().__init__()
        self.rq_vae = RqVae(input_dim=input_dim, embed_dim=output_dim, hidden_dims=hidden_dims,
                            codebook_size=codebook_size, codebook_kmeans_init=False,
                            codebook_normalize=rqvae_codebook_normalize, codebook_sim_vq=rqvae_sim_vq,
                            n_layers=n_layers, n_cat_features=n_cat_feats, commitment_weight=commitment_weight)
        if rqvae_weights_path is not None:
            self.rq_vae.load_pretrained(rqvae_weights_path)
        self.rq_vae.eval()
        self.codebook_size = codebook_size
        self.n_layers = n_layers
        self.reference_batching = True
        self.reset()

    def _get_hits(self, query: Tensor, key: Tensor) -> Tensor:
        return (key.unsqueeze(0) == query.unsqueeze(1)).all(dim=-1)

    def reset(self):
        self.cached_ids = None
        self._prefix_index = {}

    @property
    def sem_ids_dim(self):
        return self.n_layers + 1

    @torch.no_grad()
    @eval_mode
    def precompute_corpus_ids(self, movie_dataset, shard: bool = False) -> Tensor:
        """(N, L+1) corpus ids (semids.py:74-101). `shard=True` (a collective: every rank must call
        it) splits the quantization over the data-parallel ranks and all-gathers the ids."""
        dev = self.rq_vae.device
        n = len(movie_dataset)
        lo, hi = dp.shard_range(n, dp.rank(), dp.world()) if shard else (0, n)
        chunks = []
        for a in range(lo, hi, CORPUS_BATCH):
            batch = movie_dataset[list(range(a, min(hi, a + CORPUS_BATCH)))]
            x = batch.x.to(dev, non_blocking=True)
            chunks.append(self.rq_vae.get_semantic_ids(x).sem_ids)
        ids = torch.cat(chunks, 0) if chunks else torch.zeros((0, self.n_layers), dtype=torch.int64, device=dev)
        if shard:
            ids = dp.all_gather_rows(ids, n)
        self.cached_ids = torch.cat([ids, dedup_rank(ids).unsqueeze(1)], 1)
        self._prefix_index = {}
        return self.cached_ids

    def _prefix_keys(self, P: int):
        if P not in self._prefix_index:
            cols = self.cached_ids[:, :P]
            base = int(self.cached_ids.max().item()) + 1
            self._prefix_index[P] = (torch.unique(_pack(cols, base)), base)
        return self._prefix_index[P]

    @torch.no_grad()
    @eval_mode
    def exists_prefix(self, sem_id_prefix: Tensor) -> Tensor:
        if self.cached_ids is None:
            raise Exception("No match can be found in empty cache.")
        P = sem_id_prefix.shape[-1]
        keys, base = self._prefix_keys(P)
        q = sem_id_prefix.to(keys.device)
        in_range = ((q >= 0) & (q < base)).all(-1)
        qk = _pack(q.clamp(0, base - 1), base)
        pos = torch.searchsorted(keys, qk).clamp_max(keys.numel() - 1)
        out = (keys[pos] == qk) & in_range
        if self.reference_batching:
            checked = math.ceil(sem_id_prefix.shape[0] // BATCH_SIZE) * BATCH_SIZE
            out[checked:] = False
        return out.to(sem_id_prefix.device)

    def _tokenize_seq_batch_from_cached(self, ids: Tensor) -> Tensor:
        # id -1 indexes the last row (then masked by the caller), exactly like the reference (A-12)
        rows = self.cached_ids[ids.flatten()]
        return rows.reshape(ids.shape[0], -1)

    def cache_hit(self, ids_max: int) -> bool:
        """True when every id up to `ids_max` (host int) maps through the precomputed corpus cache: forward
        then launches only device lookups (no RQ-VAE pass, no host read), so it can be captured."""
        return self.cached_ids is not None and int(ids_max) < self.cached_ids.shape[0]

    @torch.no_grad()
    @eval_mode
    def forward(self, batch: SeqBatch, ids_max: Optional[int] = None) -> TokenizedSeqBatch:
        """`ids_max` (this build's extension): the batch's largest item id when the caller knows it on the
        host (a CPU-side loader), so the cache check needs no device read (a sync every step)."""
        B, N = batch.ids.shape
        top = batch.ids.max() if ids_max is None else ids_max
        if self.cached_ids is None or top >= self.cached_ids.shape[0]:
            sem_ids = self.rq_vae.get_semantic_ids(batch.x).sem_ids
            D = sem_ids.shape[-1]
            seq_mask, sem_ids_fut = None, None
        else:
            D = self.cached_ids.shape[1]
            sem_ids = self._tokenize_seq_batch_from_cached(batch.ids)
            seq_mask = batch.seq_mask.repeat_interleave(D, dim=1)
            sem_ids = sem_ids.masked_fill(~seq_mask, -1)
            sem_ids_fut = self._tokenize_seq_batch_from_cached(batch.ids_fut)
        token_type_ids = torch.arange(D, device=sem_ids.device).repeat(B, N)
        token_type_ids_fut = torch.arange(D, device=sem_ids.device).repeat(B, 1)
        return TokenizedSeqBatch(user_ids=batch.user_ids, sem_ids=sem_ids, sem_ids_fut=sem_ids_fut, seq_mask=seq_mask,
                                 token_type_ids=token_type_ids, token_type_ids_fut=token_type_ids_fut)
