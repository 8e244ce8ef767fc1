"""Generative-retrieval encoder-decoder — drop-in for reference modules/model.py
(ModelOutput :30-33, GenerationOutput :36-38, EncoderDecoderRetrievalModel :41-282; same
constructor, parameter names, forward/generation contract).

Forward (training) path, jagged mode (the only working mode in the reference, SURVEY A-9):
  user token + (wpe + sem-ID embeddings) -> padded (B, 1+N, E) context, bos + (fut sem-ID +
  tte) -> (B, L+2, E) future; both converted to NJTs by the HIP gather kernel (ops.jagged);
  RMSNorm -> Dropout(0.5) -> in_proj{_context}; TransformerEncoderDecoder on NJT values with the
  HIP varlen attention kernels; out_proj -> logits (B*(L+1), K) -> CE(ignore_index=-1) summed
  over the L+1 positions and averaged over B; loss_d = per-position mean.
The module-level Dropout(p=0.5) is hard-coded as in the reference (:67).
"""
from typing import NamedTuple

import torch
from torch import nn
from torch import Tensor
from torch.nn import functional as F

from data.schemas import TokenizedSeqBatch
from modules.linear import Linear
from modules.embedding.id_embedder import Embedding, SemIdEmbedder, UserIdEmbedder
from modules.normalize import RMSNorm
from modules.transformer.model import TransformerEncoderDecoder
from modules.utils import eval_mode, maybe_repeat_interleave, reset_encoder_cache
from ops.jagged import Jagged, jagged_to_flattened_tensor, jagged_to_padded_tensor, padded_to_jagged, row_counts
from rqvae_hip import gemm_tuning
from rqvae_hip import ops as hip_ops

# The fused forms below are the product path; False selects the reference's torch composition of the same
# op (tests / A-B probes set these module attributes; nothing reads the environment):
_BATCH_SUM = True   # False: torch's broadcast add / repeat (and their reduction backward) in the prologue
_FUSED_CE = True    # False: the loss head as torch's slice + cross_entropy + means
_FUSED_PROLOGUE = True   # False: the input embeddings as gathers / adds / cats + padded -> jagged (the composition)

# As the reference (modules/model.py:27): fp32 matmuls at 'high' precision (split-bf16 GEMM on
# gfx950, rqvae_hip.ops.gemm_bf16x3); 'highest' restores the exact-fp32 library path.
torch.set_float32_matmul_precision('high')


class ModelOutput(NamedTuple):
    loss: Tensor
    logits: Tensor
    loss_d: Tensor


class GenerationOutput(NamedTuple):
    sem_ids: Tensor
    log_probas: Tensor


class EncoderDecoderRetrievalModel(nn.Module):
    def __init__(self, embedding_dim, attn_dim, dropout, num_heads, n_layers, num_embeddings, sem_id_dim,
                 inference_verifier_fn, max_pos=2048, jagged_mode: bool = True) -> None:
        super().__init__()
        if not jagged_mode:
            raise NotImplementedError("jagged_mode=False is broken in the reference (SURVEY A-9); "
                                      "only the jagged path is provided")
        self.jagged_mode = jagged_mode
        self.num_embeddings = num_embeddings
        self.sem_id_dim = sem_id_dim
        self.attn_dim = attn_dim
        self.inference_verifier_fn = inference_verifier_fn
        self.enable_generation = False

        self.bos_emb = nn.Parameter(torch.rand(embedding_dim))
        self.norm = RMSNorm(embedding_dim)
        self.norm_cxt = RMSNorm(embedding_dim)
        self.do = nn.Dropout(p=0.5)
        self.sem_id_embedder = SemIdEmbedder(num_embeddings=num_embeddings, sem_ids_dim=sem_id_dim,
                                             embeddings_dim=embedding_dim)
        self.user_id_embedder = UserIdEmbedder(2000, embedding_dim)
        self.wpe = Embedding(num_embeddings=max_pos, embedding_dim=embedding_dim)
        self.tte = Embedding(num_embeddings=sem_id_dim, embedding_dim=embedding_dim)
        self.tte_fut = Embedding(num_embeddings=sem_id_dim, embedding_dim=embedding_dim)  # unused (reference)
        self.transformer = TransformerEncoderDecoder(d_in=attn_dim, d_out=attn_dim, dropout=dropout,
                                                     num_heads=num_heads, encoder_layers=n_layers // 2,
                                                     decoder_layers=n_layers // 2)
        self.in_proj = Linear(embedding_dim, attn_dim, bias=False)
        self.in_proj_context = Linear(embedding_dim, attn_dim, bias=False)
        self.out_proj = Linear(attn_dim, num_embeddings, bias=False)

    @staticmethod
    def context_rows(batch: TokenizedSeqBatch, bucket=None) -> int:
        """Allocated rows of the jagged context: valid tokens (user token + sequence) rounded up to
        `bucket`. Host-known counts (ops.jagged.register_row_counts) avoid the device sync."""
        B = batch.seq_mask.shape[0]
        host = row_counts(batch.seq_mask)
        total = host[0] + B if host is not None and host[3] == B else int(batch.seq_mask.sum()) + B
        return total if not bucket else (total + bucket - 1) // bucket * bucket

    def _prologue_fused(self, batch: TokenizedSeqBatch, alloc: int):
        """Context / future jagged inputs in one HIP op (hip_ops.decoder_prologue), or None where it does not
        apply (generation: no future tokens)."""
        se, ue = self.sem_id_embedder, self.user_id_embedder
        args = (ue.emb.weight, se.emb.weight, self.wpe.weight, self.tte.weight, self.bos_emb, batch.user_ids,
                batch.sem_ids, batch.token_type_ids, batch.seq_mask, batch.sem_ids_fut, batch.token_type_ids_fut)
        if not (_FUSED_PROLOGUE and hip_ops.decoder_prologue_supported(*args) and
                all(e.max_norm is None for e in (se.emb, ue.emb, self.wpe, self.tte)) and
                all(e.padding_idx is None for e in (ue.emb, self.wpe, self.tte))):
            return None
        B, N = batch.sem_ids.shape
        nf = batch.sem_ids_fut.shape[1] + 1
        ctx_v, ctx_off, fut_v, fut_off = hip_ops.decoder_prologue(*args, ue.num_buckets, se.num_embeddings,
                                                                   se.padding_idx, alloc)
        return Jagged(ctx_v, ctx_off, N + 1, 0, None), Jagged(fut_v, fut_off, nf, nf, B * nf)

    def _predict(self, batch: TokenizedSeqBatch):
        bucket = gemm_tuning.ROW_BUCKET if gemm_tuning.is_enabled() else None
        fused = self._prologue_fused(batch, self.context_rows(batch, bucket))
        if fused is not None:
            ctx_j, fut_j = fused
            transformer_context = ctx_j.with_values(self.in_proj_context(self.norm.forward_dropout(ctx_j.values(),
                                                                                                   self.do)))
            transformer_input = fut_j.with_values(self.in_proj(self.norm_cxt.forward_dropout(fut_j.values(), self.do)))
            return self.transformer(x=transformer_input, context=transformer_context, padding_mask=batch.seq_mask,
                                    jagged=True)
        user_emb = self.user_id_embedder(batch.user_ids)                  # (B, 1, E)
        sem = self.sem_id_embedder(batch)
        seq_emb, fut_emb = sem.seq, sem.fut                               # (B, N, E), (B, L+1, E)
        B, N, _ = seq_emb.shape
        pos = self.wpe(torch.arange(N, device=seq_emb.device)).unsqueeze(0)
        if _BATCH_SUM:   # the broadcast parameters' batch-sum gradients on one fixed-order HIP launch each
            ctx = torch.cat([user_emb, hip_ops.batch_add(seq_emb, pos)], dim=1)          # (B, 1+N, E)
            fut = hip_ops.batch_repeat(self.bos_emb.view(1, -1), B)
        else:
            ctx = torch.cat([user_emb, pos + seq_emb], dim=1)
            fut = self.bos_emb.repeat(B, 1, 1)
        if fut_emb is not None:
            fut = torch.cat([fut, fut_emb + self.tte(batch.token_type_ids_fut)], dim=1)
        ctx_lengths = batch.seq_mask.sum(axis=1) + 1
        # the context's valid row total is data-dependent; a CPU-side loader registers it with the
        # mask (no device sync). The values buffer is allocated at the total rounded up to the GEMM
        # row bucket (bounded GEMM shapes; rqvae_hip.gemm_tuning); the gather and attention kernels
        # keep the tail rows zero on the device, and attention is launched over the padded width,
        # so nothing in the step depends on the exact total on the host: a step captured for one
        # bucket (rqvae_hip.graph.GraphedSteps) replays for every batch of that bucket.
        bucket = gemm_tuning.ROW_BUCKET if gemm_tuning.is_enabled() else None
        alloc = self.context_rows(batch, bucket)
        Nc = ctx.shape[1]
        ctx_j = padded_to_jagged(ctx.contiguous(), ctx_lengths, Nc, alloc_rows=alloc, known_max=Nc)
        nf = fut.shape[1]                                                                # fixed length: no sync
        fut_lengths = torch.full((B,), nf, device=fut.device, dtype=torch.int64)
        fut_j = padded_to_jagged(fut.contiguous(), fut_lengths, nf, total=B * nf, known_max=nf)
        transformer_context = ctx_j.with_values(self.in_proj_context(self.norm.forward_dropout(ctx_j.values(), self.do)))
        transformer_input = fut_j.with_values(self.in_proj(self.norm_cxt.forward_dropout(fut_j.values(), self.do)))
        return self.transformer(x=transformer_input, context=transformer_context, padding_mask=batch.seq_mask,
                                jagged=True)

    def _gemm_weights(self):
        return [m.weight for m in self.modules() if isinstance(m, nn.Linear)]

    def _gemm_weight_stacks(self):
        """Weights the forward multiplies as one concatenated matrix (the decoder's hoisted K/V)."""
        return [st for st in (getattr(m, "hoisted_kv_weights", lambda: None)() for m in self.modules()) if st]

    def forward(self, batch: TokenizedSeqBatch) -> ModelOutput:
        B = batch.seq_mask.shape[0]
        # every Linear weight split once per forward in a few launches (no-op at 'highest')
        with hip_ops.weight_split_scope(self._gemm_weights(), self._gemm_weight_stacks()):
            return self._forward(batch, B)

    def _forward(self, batch: TokenizedSeqBatch, B: int) -> ModelOutput:
        trnsf_out = self._predict(batch)
        if self.training or not self.enable_generation:
            predict_out = self.out_proj(jagged_to_flattened_tensor(trnsf_out))
            target = batch.sem_ids_fut
            if _FUSED_CE and hip_ops.ce_loss_supported(predict_out, target, B):
                # the whole loss head (slice, cross-entropy, both means) in three HIP launches
                loss, loss_d, logits = hip_ops.cross_entropy_loss(predict_out, target, B)
                if not self.training:
                    self.transformer.cached_enc_output = None
                return ModelOutput(loss=loss, logits=logits, loss_d=loss_d)
            # sem_ids_fut is fixed length, so the jagged values reshape to (B, L+2, K)
            logits = predict_out.view(B, -1, self.num_embeddings)[:, :-1, :].flatten(end_dim=1)
            target = batch.sem_ids_fut.flatten(end_dim=1)
            unred_loss = F.cross_entropy(logits, target, reduction="none", ignore_index=-1).view(B, -1)
            loss = unred_loss.sum(axis=1).mean()
            if not self.training:
                self.transformer.cached_enc_output = None
            return ModelOutput(loss=loss, logits=logits, loss_d=unred_loss.mean(axis=0))
        last = jagged_to_flattened_tensor(trnsf_out).contiguous().view(B, -1, self.attn_dim)[:, -1, :]
        return ModelOutput(loss=None, logits=self.out_proj(last), loss_d=None)

    @eval_mode
    @reset_encoder_cache
    @torch.no_grad()
    def generate_next_sem_id(self, batch: TokenizedSeqBatch, temperature: int = 1, top_k: bool = True) -> GenerationOutput:
        """Beam-style decoding of the next item's L+1 sem-ID tokens (reference :149-245): per step
        sample 200 candidates per beam from softmax(logits / T), drop prefixes the verifier
        rejects (-10000), keep the top 32 cumulative log-probabilities. The encoder output is
        computed once and repeated per beam with the HIP jagged kernels (jagged -> padded,
        repeat_interleave, padded -> jagged), as the reference does with torch ops."""
        assert self.enable_generation, "Model generation is not enabled"
        B = batch.sem_ids.shape[0]
        generated, log_probas = None, 0
        k = 32 if top_k else 1
        n_cand = 200 if top_k else 1
        cur = TokenizedSeqBatch(user_ids=batch.user_ids, sem_ids=batch.sem_ids, sem_ids_fut=None,
                                seq_mask=batch.seq_mask, token_type_ids=batch.token_type_ids, token_type_ids_fut=None)
        for i in range(self.sem_id_dim):
            logits = self.forward(cur).logits
            probas = F.softmax(logits / temperature, dim=-1)
            samples_b = torch.multinomial(probas, num_samples=n_cand)
            if generated is None:
                valid = self.inference_verifier_fn(samples_b.unsqueeze(-1))
            else:
                prefix = torch.cat([generated.flatten(0, 1).unsqueeze(1).repeat_interleave(n_cand, axis=1),
                                    samples_b.unsqueeze(-1)], axis=-1)
                valid = self.inference_verifier_fn(prefix).reshape(B, -1)
            sampled_lp = torch.log(torch.gather(probas, 1, samples_b)).reshape(B, -1)
            samples = samples_b.reshape(B, -1)
            sorted_lp, sorted_idx = (-10000 * (~valid) + sampled_lp +
                                     maybe_repeat_interleave(log_probas, n_cand, dim=1)).sort(-1, descending=True)
            top_lp, top_idx = sorted_lp[:, :k], sorted_idx[:, :k]
            top_samples = torch.gather(samples, 1, top_idx)
            if generated is not None:
                parent = torch.gather(generated, 1, (top_idx // n_cand).unsqueeze(2).expand(-1, -1, i))
                top_samples = torch.cat([parent, top_samples.unsqueeze(-1)], axis=-1)
                nxt = top_samples.flatten(end_dim=1)
                cur = TokenizedSeqBatch(user_ids=cur.user_ids, sem_ids=cur.sem_ids, sem_ids_fut=nxt,
                                        token_type_ids_fut=torch.arange(nxt.shape[1], device=nxt.device).repeat(nxt.shape[0], 1),
                                        seq_mask=cur.seq_mask, token_type_ids=cur.token_type_ids)
                generated = top_samples.detach().clone()
                log_probas = top_lp.detach().clone()
            else:
                nxt = top_samples.reshape(-1, 1)
                enc = self.transformer.cached_enc_output
                n_ctx = cur.sem_ids.shape[1] + 1
                padded = jagged_to_padded_tensor(enc, n_ctx).repeat_interleave(k, dim=0)
                lengths = enc.offsets().diff().repeat_interleave(k)
                self.transformer.cached_enc_output = padded_to_jagged(padded.contiguous(), lengths, n_ctx)
                cur = TokenizedSeqBatch(user_ids=cur.user_ids.repeat_interleave(k, dim=0),
                                        sem_ids=cur.sem_ids.repeat_interleave(k, dim=0), sem_ids_fut=nxt,
                                        token_type_ids_fut=torch.zeros_like(nxt),
                                        seq_mask=cur.seq_mask.repeat_interleave(k, dim=0),
                                        token_type_ids=cur.token_type_ids.repeat_interleave(k, dim=0))
                generated = top_samples.unsqueeze(-1)
                log_probas = top_lp.detach().clone()
        return GenerationOutput(sem_ids=generated.squeeze(), log_probas=log_probas.squeeze())
