"""CPU restatement of the decoder train step — TEST INFRASTRUCTURE ONLY (the parity pin for the
decoder fixtures' math and bench.py's decoder `cpu_baseline`); the product path never imports it.

Plain torch on the CPU (eager, autograd for the backward), over a state dict with the reference's
parameter names. Jagged sequences are held padded (B, N) with a validity mask: every row-wise op is
unchanged, attention masks the padded keys (and the causal triangle), and the loss only reads the
fixed-length future rows, so the math is the reference's jagged path:
  EncoderDecoderRetrievalModel._predict / forward  modules/model.py:101-147, 247-282
  SemIdEmbedder / UserIdEmbedder                    modules/embedding/id_embedder.py:28-53
  RMSNorm (eps 1e-6, fp32)                          modules/normalize.py:21-32
  TransformerBlock (A-11: cross-attn norms x)       modules/transformer/model.py:68-82
  TransformerEncoderDecoder                         modules/transformer/model.py:174-188
  MultiHeadAttention + jagged SDPA                  modules/transformer/attention.py:113-124, 185-233
  MLP (Linear-SiLU-[Dropout]-Linear)                modules/encoder.py:7-36
Pinned against tests/golden/decoder_*.npz (written by the reference) in tests/test_oracle.py.
"""
import re

import torch
import torch.nn.functional as F


def _rms(x, w, eps=1e-6):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


def _mlp(x, ws, p, training):
    for i, w in enumerate(ws):
        x = x @ w.t()
        if i < len(ws) - 1:
            x = F.silu(x)
            if p > 0:
                x = F.dropout(x, p, training)
    return x


def _mha(P, pre, x, kv, mask_q, mask_k, H, causal):
    """Multi-head attention over padded rows; mask_* (B, N) bool validity."""
    B, Nq, A = x.shape
    hd = A // H
    if kv is None:
        q, k, v = (x @ P[pre + "qkv.weight"].t()).chunk(3, dim=-1)
    else:
        q = x @ P[pre + "q.weight"].t()
        k, v = (kv @ P[pre + "kv.weight"].t()).chunk(2, dim=-1)
    Nk = k.shape[1]
    heads = lambda t, n: t.view(B, n, H, hd).transpose(1, 2)  # noqa: E731
    allow = mask_k[:, None, None, :].expand(B, 1, Nq, Nk)
    if causal:
        allow = allow & torch.ones(Nq, Nk, dtype=torch.bool).tril()[None, None]
    allow = allow | ~mask_q[:, None, :, None]          # padded query rows: any finite row, discarded later
    o = F.scaled_dot_product_attention(heads(q, Nq), heads(k, Nk), heads(v, Nk), attn_mask=allow)
    return o.transpose(1, 2).reshape(B, Nq, A) @ P[pre + "proj.weight"].t()


def _block(P, pre, x, kv, mask_x, mask_kv, H, causal, p, training):
    ffw = sorted((k for k in P if k.startswith(pre + "ff.1.mlp.") and k.endswith(".weight")),
                 key=lambda k: int(re.search(r"mlp\.(\d+)\.", k).group(1)))
    do = lambda t: F.dropout(t, p, training) if p > 0 else t  # noqa: E731
    h = x + _mha(P, pre + "attention.", do(_rms(x, P[pre + "attn_norm.weight"])), None, mask_x, mask_x, H, causal)
    if kv is not None:
        h = h + _mha(P, pre + "cross_attention.", do(_rms(x, P[pre + "cross_attn_norm.weight"])), kv, mask_x, mask_kv,
                     H, False)
    return h + do(_mlp(_rms(h, P[pre + "ff.0.weight"]), [P[k] for k in ffw], p, training))


def decoder_forward(P, batch, K, L1, H, n_layers, dropout=0.0, training=True):
    """(loss, logits (B*L1, K), loss_d (L1,)) of EncoderDecoderRetrievalModel.forward in train mode.
    P: name -> tensor (requires_grad for the backward); batch: TokenizedSeqBatch fields as tensors."""
    sem, mask = batch["sem_ids"].clone(), batch["seq_mask"]
    B, N = sem.shape
    ids = batch["token_type_ids"] * K + sem
    ids[~mask] = L1 * K                                                   # padding row
    emb = P["sem_id_embedder.emb.weight"]
    seq_emb = emb[ids]
    fut_emb = emb[batch["token_type_ids_fut"] * K + batch["sem_ids_fut"]]
    user = P["user_id_embedder.emb.weight"][batch["user_ids"] % 2000]      # (B, 1, E)
    ctx = torch.cat([user, P["wpe.weight"][:N][None] + seq_emb], 1)       # (B, 1+N, E)
    fut = torch.cat([P["bos_emb"].expand(B, 1, -1), fut_emb + P["tte.weight"][batch["token_type_ids_fut"]]], 1)
    lens = mask.sum(1) + 1
    mask_c = torch.arange(N + 1)[None] < lens[:, None]                    # jagged prefix of each row
    mask_f = torch.ones(B, fut.shape[1], dtype=torch.bool)
    p = 0.5 if (training and dropout > 0) else 0.0                        # model-level Dropout(0.5), model.py:67
    do0 = lambda t: F.dropout(t, p, training) if p > 0 else t             # noqa: E731
    c = do0(_rms(ctx, P["norm.weight"])) @ P["in_proj_context.weight"].t()
    x = do0(_rms(fut, P["norm_cxt.weight"])) @ P["in_proj.weight"].t()
    c = c * mask_c[..., None]                                            # padded rows stay zero
    for l in range(n_layers // 2):
        c = _block(P, f"transformer.encoder.layers.{l}.", c, None, mask_c, None, H, False, dropout, training)
        c = c * mask_c[..., None]
    for l in range(n_layers // 2):
        x = _block(P, f"transformer.decoder.layers.{l}.", x, c, mask_f, mask_c, H, True, dropout, training)
    logits = (x @ P["out_proj.weight"].t())[:, :-1, :].reshape(-1, K)
    target = batch["sem_ids_fut"].reshape(-1)
    unred = F.cross_entropy(logits, target, reduction="none", ignore_index=-1).view(B, -1)
    return unred.sum(1).mean(), logits, unred.mean(0)
