"""Next-rows on the GPU: corpus tokenizer + dedup, k-means codebook init, generation.

Tokenizer and k-means are pinned by reference fixtures (tokenizer.npz, kmeans.npz). Generation is
pinned against the reference in tests/test_reference_fixtures_gpu.py::test_generation_vs_reference
(generation.npz, a deterministic sampler patched into both sides); here it is additionally checked
for its structural properties with the real torch.multinomial sampler (beam shapes, sorted beams,
train mode and the encoder cache restored)."""
import numpy as np
import pytest
import torch

import gen_inputs as gi

pytestmark = pytest.mark.gpu


class _Items:
    def __init__(self, x):
        self.x = torch.from_numpy(x)

    def __len__(self):
        return self.x.shape[0]

    def __getitem__(self, idx):
        from data.schemas import SeqBatch
        ids = torch.as_tensor(idx).reshape(1, -1)
        neg = -torch.ones_like(ids[0])
        return SeqBatch(neg, ids, neg, self.x[idx], neg, torch.ones_like(ids, dtype=torch.bool))


def _tokenizer(z, device):
    from modules.tokenizer.semids import SemanticIdTokenizer
    inp, hid, D, K, L, seed = int(z["inp"]), [int(h) for h in z["hidden"]], int(z["D"]), int(z["K"]), int(z["L"]), int(z["seed"])
    tok = SemanticIdTokenizer(input_dim=inp, output_dim=D, hidden_dims=hid, codebook_size=K, n_layers=L, n_cat_feats=0)
    st = {f"encoder.mlp.{2 * j}.weight": w for j, w in enumerate(gi.mlp_weights([inp] + hid + [D], seed))}
    st.update({f"decoder.mlp.{2 * j}.weight": w for j, w in enumerate(gi.mlp_weights([D] + hid[::-1] + [inp], seed + 1))})
    st.update({f"layers.{l}.embedding.weight": z["codebooks"][l] for l in range(L)})
    tok.rq_vae.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
    return tok.to(device)


def test_tokenizer_vs_reference(golden, device):
    from data.schemas import SeqBatch
    z = golden("tokenizer")
    tok = _tokenizer(z, device)
    items = gi.items(int(z["n_items"]), int(z["inp"]), int(z["seed"]))
    ids = tok.precompute_corpus_ids(_Items(items))
    assert np.array_equal(ids.cpu().numpy(), z["corpus_ids"]), "corpus ids + dedup column"
    sb = SeqBatch(user_ids=torch.arange(6, device=device), ids=torch.from_numpy(z["seq_ids"]).to(device),
                  ids_fut=torch.from_numpy(z["fut_ids"]).to(device), x=None, x_fut=None,
                  seq_mask=torch.from_numpy(z["seq_ids"] >= 0).to(device))
    t = tok(sb)
    assert np.array_equal(t.sem_ids.cpu().numpy(), z["tok_sem_ids"])
    assert np.array_equal(t.sem_ids_fut.cpu().numpy(), z["tok_sem_ids_fut"])
    assert np.array_equal(t.seq_mask.cpu().numpy(), z["tok_seq_mask"])
    got = tok.exists_prefix(torch.from_numpy(z["prefixes"]).to(device)).cpu().numpy()
    assert np.array_equal(got, z["exists_prefix"]), "reference batching quirk reproduced"
    tok.reference_batching = False
    fixed = tok.exists_prefix(torch.from_numpy(z["prefixes"]).to(device)).cpu().numpy()
    corpus = set(map(tuple, z["corpus_ids"][:, :2]))
    assert np.array_equal(fixed, np.array([tuple(p) in corpus for p in z["prefixes"]]))


def test_dedup_rank_large(device):
    from modules.tokenizer.semids import dedup_rank
    from oracle import unique as U
    g = gi.rng(9)
    ids = g.integers(0, 6, size=(50000, 3))
    got = dedup_rank(torch.from_numpy(ids).to(device)).cpu().numpy()
    assert np.array_equal(got, U.dedup_rank(ids))


@pytest.mark.parametrize("B,D,K", [(20000, 8, 16), (65536, 64, 256), (3, 1024, 7), (1000, 16, 4096), (300000, 8, 300)])
def test_segment_sum(device, B, D, K):
    from rqvae_hip import ops
    g = gi.rng(B + D + K)
    rows = g.standard_normal((B, D), dtype=np.float32)
    keys = g.integers(0, K, size=B)
    ref = np.zeros((K, D))
    np.add.at(ref, keys, rows.astype(np.float64))
    r, k = torch.from_numpy(rows).to(device), torch.from_numpy(keys).to(device)
    s1, c1 = ops.segment_sum(r, k, K)
    s2, _ = ops.segment_sum(r, k, K)
    assert torch.equal(s1, s2), "deterministic"
    assert np.array_equal(c1.cpu().numpy(), np.bincount(keys, minlength=K))
    assert np.allclose(s1.cpu().numpy(), ref, rtol=1e-5, atol=1e-4)


def test_kmeans_vs_reference(golden, device):
    from init.kmeans import Kmeans
    z = golden("kmeans")
    np.random.seed(int(z["np_seed"]))
    out = Kmeans(k=int(z["k"]), max_iters=int(z["max_iters"])).run(torch.from_numpy(z["x"]).to(device))
    assert np.array_equal(out.assignment.cpu().numpy(), z["assignment"])
    assert np.allclose(out.centroids.cpu().numpy(), z["centroids"], rtol=1e-5, atol=1e-6)


def test_rqvae_kmeans_init_path(device):
    """First forward with codebook_kmeans_init runs the per-level init, then the fused path."""
    from data.schemas import SeqBatch
    from modules.quantize import QuantizeForwardMode
    from modules.rqvae import RqVae
    np.random.seed(0)
    m = RqVae(96, 16, [64, 32], 32, codebook_kmeans_init=True, codebook_mode=QuantizeForwardMode.ROTATION_TRICK,
              n_layers=3, n_cat_features=0).to(device)
    x = torch.from_numpy(gi.items(2000, 96, 4)).to(device)
    out = m(SeqBatch(None, None, None, x, None, None), gumbel_t=0.2)
    assert all(layer.kmeans_initted for layer in m.layers)
    assert m._fused_kernel_mode() is not None
    out2 = m(SeqBatch(None, None, None, x, None, None), gumbel_t=0.2)
    assert torch.isfinite(out.loss) and torch.isfinite(out2.loss)
    assert float(out2.p_unique_ids) > 0.3


def test_generation_properties(golden, device):
    from data.processed import synthetic_tokenized_batch
    from modules.model import EncoderDecoderRetrievalModel
    z = golden("tokenizer")
    tok = _tokenizer(z, device)
    tok.precompute_corpus_ids(_Items(gi.items(int(z["n_items"]), int(z["inp"]), int(z["seed"]))))
    K, L1 = int(z["K"]), int(z["L"]) + 1
    torch.manual_seed(0)
    model = EncoderDecoderRetrievalModel(embedding_dim=32, attn_dim=64, dropout=0.0, num_heads=4, n_layers=4,
                                         num_embeddings=max(K, 2000), sem_id_dim=L1,
                                         inference_verifier_fn=lambda x: tok.exists_prefix(x), max_pos=20 * L1).to(device)
    model.enable_generation = True
    assert model.training
    batch = synthetic_tokenized_batch(3, 5, L1, K, 7, device)
    out = model.generate_next_sem_id(batch, top_k=True, temperature=1)
    assert out.sem_ids.shape == (3, 32, L1) and out.log_probas.shape == (3, 32)
    lp = out.log_probas.cpu()
    assert torch.all(lp[:, :-1] >= lp[:, 1:]), "beams sorted by cumulative log-probability"
    assert model.training, "eval_mode restores the previous (train) mode"
    assert model.transformer.cached_enc_output is None
