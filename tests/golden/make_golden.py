#!/usr/bin/env python3
"""Generate the golden parity fixtures by importing the READ-ONLY reference.

Test infrastructure only; run in the build container (never on the GPU box, where
/root/reference does not exist):

    python tests/golden/make_golden.py [/root/reference]

The reference is imported as-is from its own tree; nothing is copied. Modules the
reference imports but this image lacks (gin, swanlab, polars, sentence_transformers,
torch_geometric) are replaced by inert stubs before import. The Triton
jagged kernel runs under TRITON_INTERPRET=1 on CPU; torch.compile is disabled
(TORCHDYNAMO_DISABLE=1) so RqVae.forward / EncoderDecoderRetrievalModel.forward run
eagerly. NJT scaled_dot_product_attention has no CPU backend, so the decoder fixtures
substitute a per-sequence dense SDPA loop over the NJT components (the reference's own
SDPA semantics; every decoder fixture records `sdpa_substitute=1`).

Outputs: small .npz files next to this script (float32 / int64 arrays; < 1 MB each).
Large inputs are regenerated from gen_inputs.py seeds and only checksummed here.
"""
import os
import sys
import types

os.environ.setdefault("TORCHDYNAMO_DISABLE", "1")
os.environ.setdefault("TRITON_INTERPRET", "1")
os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True

HERE = os.path.dirname(os.path.abspath(__file__))
REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gen_inputs as gi  # noqa: E402


# --------------------------------------------------------------------------- stubs
def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__spec__ = None
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


class _Placeholder:
    def __init__(self, *a, **k):
        raise RuntimeError("stubbed dependency; not available offline")


class _InMemoryDatasetStub:
    pass


_stub("gin", configurable=lambda f=None, **k: f if f is not None else (lambda g: g),
      constants_from_enum=lambda c=None, **k: c if c is not None else (lambda g: g),
      parse_config_file=lambda *a, **k: None)
_stub("swanlab", init=lambda *a, **k: None, log=lambda *a, **k: None, finish=lambda *a, **k: None)
_stub("polars")
_stub("sentence_transformers", SentenceTransformer=_Placeholder)
_tg = _stub("torch_geometric")
_tg.data = _stub("torch_geometric.data", HeteroData=_Placeholder, InMemoryDataset=_InMemoryDatasetStub,
                 download_url=_Placeholder, extract_zip=_Placeholder)
_tg.datasets = _stub("torch_geometric.datasets", MovieLens1M=_Placeholder)
_tg.io = _stub("torch_geometric.io", fs=None)

sys.path.insert(0, REF)

from modules.quantize import Quantize, QuantizeForwardMode  # noqa: E402
from modules.rqvae import RqVae  # noqa: E402
from modules.model import EncoderDecoderRetrievalModel  # noqa: E402
from modules.tokenizer.semids import SemanticIdTokenizer  # noqa: E402
from data.schemas import SeqBatch, TokenizedSeqBatch  # noqa: E402
from ops.triton.jagged import padded_to_jagged_tensor  # noqa: E402
from init.kmeans import Kmeans  # noqa: E402
import modules.transformer.attention as ref_attention  # noqa: E402

torch.set_num_threads(min(8, os.cpu_count() or 1))
F32 = np.float32


def npf(t):
    return t.detach().cpu().numpy().astype(F32)


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {name}: {os.path.getsize(path) / 1024:.1f} KiB")


def top2_margin(x, cb):
    """Relative gap between the two smallest reference-order distances (fp64)."""
    x64, c64 = x.astype(np.float64), cb.astype(np.float64)
    d = (x64 ** 2).sum(1, keepdims=True) + (c64 ** 2).sum(1)[None] - 2 * x64 @ c64.T
    s = np.sort(d, axis=1)
    return ((s[:, 1] - s[:, 0]) / np.maximum(np.abs(s[:, 0]), 1e-30)).astype(np.float64)


# ------------------------------------------------------------------ quantize level
MODES = {"rotation": QuantizeForwardMode.ROTATION_TRICK, "ste": QuantizeForwardMode.STE}


def quantize_fixture(tag, B, D, K, seed, store_inputs, modes=("rotation", "ste", "eval")):
    x_np, cb_np = gi.quantize_case(B, D, K, seed)
    g = gi.rng(seed + 1)
    g_emb = g.standard_normal((B, D), dtype=F32)
    g_loss = g.random(B, dtype=F32)
    out = dict(B=B, D=D, K=K, seed=seed, beta=F32(0.25),
               x_checksum=gi.checksum(x_np), cb_checksum=gi.checksum(cb_np),
               g_emb=g_emb, g_loss=g_loss, margin=top2_margin(x_np, cb_np))
    if store_inputs:
        out.update(x=x_np, codebook=cb_np)
    out["modes"] = np.array(modes)
    for mname in modes:
        q = Quantize(D, K, do_kmeans_init=False, forward_mode=MODES.get(mname, QuantizeForwardMode.ROTATION_TRICK))
        with torch.no_grad():
            q.embedding.weight.copy_(torch.from_numpy(cb_np))
        q.train(mname != "eval")
        x = torch.from_numpy(x_np.copy()).requires_grad_(True)
        o = q(x, temperature=0.2)
        ((o.embeddings * torch.from_numpy(g_emb)).sum() + (o.loss * torch.from_numpy(g_loss)).sum()).backward()
        gcb = q.embedding.weight.grad
        rows = torch.nonzero(gcb.abs().sum(1) > 0).flatten()
        out.update({
            f"{mname}_ids": o.ids.numpy().astype(np.int64),
            f"{mname}_emb": npf(o.embeddings),
            f"{mname}_loss": npf(o.loss),
            f"{mname}_grad_x": npf(x.grad),
            f"{mname}_gcb_rows": rows.numpy().astype(np.int64),
            f"{mname}_gcb": npf(gcb[rows]),
        })
    save(f"quantize_{tag}.npz", **out)


# ------------------------------------------------------------------------ RqVae
def rqvae_state(model_dims, codebooks, seed):
    """State dict with numpy-seeded MLP weights + given codebooks (reference key names)."""
    inp, hidden, emb = model_dims
    enc = gi.mlp_weights([inp] + hidden + [emb], seed)
    dec = gi.mlp_weights([emb] + hidden[::-1] + [inp], seed + 1)
    sd = {}
    for j, w in enumerate(enc):
        sd[f"encoder.mlp.{2 * j}.weight"] = torch.from_numpy(w)
    for j, w in enumerate(dec):
        sd[f"decoder.mlp.{2 * j}.weight"] = torch.from_numpy(w)
    for l, cb in enumerate(codebooks):
        sd[f"layers.{l}.embedding.weight"] = torch.from_numpy(cb)
    return sd


def make_codebooks(model, x, K, L, seed):
    """k-means-init-like codebooks: level l = K residual rows of random items."""
    with torch.no_grad():
        res = model.encode(torch.from_numpy(x))
        cbs = []
        perm = gi.rng(seed + 1).permutation(res.shape[0])    # disjoint item sets per level
        for l in range(L):
            idx = perm[l * K:(l + 1) * K]
            cb = res[idx].clone()
            cbs.append(cb.numpy().astype(F32))
            d = (res ** 2).sum(1, keepdim=True) + (cb ** 2).sum(1)[None] - 2 * res @ cb.T
            res = res - cb[d.argmin(1)]
    return cbs


def rqvae_fixture(tag, inp, hidden, D, K, L, B, seed, store_grads_full):
    model = RqVae(input_dim=inp, embed_dim=D, hidden_dims=hidden, codebook_size=K,
                  codebook_kmeans_init=False, codebook_mode=QuantizeForwardMode.ROTATION_TRICK,
                  n_layers=L, n_cat_features=0, commitment_weight=0.25)
    cb_items = gi.items(max(4 * K, 512), inp, seed + 100)
    # encoder weights first (codebooks depend on them)
    sd = rqvae_state((inp, hidden, D), [np.zeros((K, D), F32)] * L, seed)
    model.load_state_dict(sd)
    cbs = make_codebooks(model, cb_items, K, L, seed)
    model.load_state_dict(rqvae_state((inp, hidden, D), cbs, seed))
    x_np = gi.items(B, inp, seed + 200)
    out = dict(inp=inp, hidden=np.array(hidden, np.int64), D=D, K=K, L=L, B=B, seed=seed,
               x_checksum=gi.checksum(x_np), codebooks=np.stack(cbs))
    # eval-mode semantic ids (tokenizer path)
    model.eval()
    with torch.no_grad():
        ev = model.get_semantic_ids(torch.from_numpy(x_np))
    out.update(eval_sem_ids=ev.sem_ids.numpy().astype(np.int64), eval_embeddings=npf(ev.embeddings),
               eval_residuals=npf(ev.residuals), eval_quantize_loss=npf(ev.quantize_loss))
    # train-mode forward + backward
    model.train()
    batch = SeqBatch(user_ids=None, ids=None, ids_fut=None, x=torch.from_numpy(x_np.copy()),
                     x_fut=None, seq_mask=None)
    sem = model.get_semantic_ids(batch.x, 0.2)
    out.update(train_sem_ids=sem.sem_ids.numpy().astype(np.int64), train_embeddings=npf(sem.embeddings),
               train_residuals=npf(sem.residuals), train_quantize_loss=npf(sem.quantize_loss))
    model.zero_grad()
    o = model(batch, gumbel_t=0.2)
    o.loss.backward()
    out.update(loss=npf(o.loss), reconstruction_loss=npf(o.reconstruction_loss), rqvae_loss=npf(o.rqvae_loss),
               embs_norm=npf(o.embs_norm), p_unique_ids=npf(o.p_unique_ids))
    for name, p in model.named_parameters():
        key = "grad__" + name.replace(".", "_")
        if store_grads_full or name.startswith("layers."):
            out[key] = npf(p.grad)
        else:
            out[key + "__norm"] = np.float64(p.grad.double().norm().item())
            out[key + "__row0"] = npf(p.grad[0])
    # per-level margins of the eval path (ids pinned only on margin-safe rows)
    with torch.no_grad():
        res = model.encode(torch.from_numpy(x_np)).numpy()
        margins = []
        for l in range(L):
            margins.append(top2_margin(res, cbs[l]))
            res = res - cbs[l][ev.sem_ids[:, l].numpy()]
    out["eval_margin"] = np.stack(margins, 1)
    save(f"rqvae_{tag}.npz", **out)


# ------------------------------------------------------------------------ jagged
def jagged_fixture():
    out = {}
    for case, (B, N, D, lens, seed) in {
        "ragged": (6, 11, 8, [3, 11, 1, 7, 11, 5], 31),
        "full": (4, 5, 128, [5, 5, 5, 5], 32),
        "ctx": (5, 33, 16, [1, 33, 17, 32, 9], 33),
    }.items():
        g = gi.rng(seed)
        x = g.standard_normal((B, N, D), dtype=F32)
        lengths = np.array(lens, np.int64)
        xt = torch.from_numpy(x.copy()).requires_grad_(True)
        nt = padded_to_jagged_tensor(xt, torch.from_numpy(lengths), N)
        vals = nt.values()
        gv = g.standard_normal(tuple(vals.shape), dtype=F32)
        (vals * torch.from_numpy(gv)).sum().backward()
        out.update({f"{case}_x": x, f"{case}_lengths": lengths, f"{case}_values": npf(vals),
                    f"{case}_offsets": nt.offsets().detach().numpy().astype(np.int64),
                    f"{case}_gv": gv, f"{case}_grad_x": npf(xt.grad)})
    save("jagged.npz", **out)


# ------------------------------------------------------------------------ decoder
class _DenseLoopSDPA:
    """torch.nn.functional proxy whose SDPA loops over NJT components (CPU substitute)."""

    def __getattr__(self, name):
        return getattr(torch.nn.functional, name)

    @staticmethod
    def scaled_dot_product_attention(q, k, v, dropout_p=0.0, is_causal=False, **kw):
        assert dropout_p == 0.0
        # the reference's NJT offsets are float (ops/triton/jagged.py:47): index with int copies
        qo, ko = q.offsets().long().tolist(), k.offsets().long().tolist()
        assert q._ragged_idx == 2 and k._ragged_idx == 2
        qv, kv, vv = q.values(), k.values(), v.values()          # (H, sum_j, hd) for (B,H,j,hd) NJTs
        outs = [torch.nn.functional.scaled_dot_product_attention(
                    qv[:, qo[b]:qo[b + 1]], kv[:, ko[b]:ko[b + 1]], vv[:, ko[b]:ko[b + 1]], is_causal=is_causal)
                for b in range(len(qo) - 1)]
        vals = torch.cat([o.transpose(0, 1) for o in outs], 0)
        return torch.nested.nested_tensor_from_jagged(vals, q.offsets()).transpose(1, 2)


def tokenized_batch(B, n_max, L1, K, seed):
    g = gi.rng(seed)
    n_items = g.integers(1, n_max + 1, size=B)
    N = n_max * L1
    sem = g.integers(0, K, size=(B, N)).astype(np.int64)
    mask = np.zeros((B, N), bool)
    for b in range(B):
        mask[b, : n_items[b] * L1] = True
    sem[~mask] = -1
    fut = g.integers(0, K, size=(B, L1)).astype(np.int64)
    users = g.integers(0, 10 ** 6, size=(B, 1)).astype(np.int64)
    tt = np.tile(np.arange(L1), (B, n_max)).astype(np.int64)
    tt_fut = np.tile(np.arange(L1), (B, 1)).astype(np.int64)
    return dict(user_ids=users, sem_ids=sem, sem_ids_fut=fut, seq_mask=mask,
                token_type_ids=tt, token_type_ids_fut=tt_fut)


def decoder_fixture(tag, E, A, H, n_layers, K, L1, B, n_max, seed):
    ref_attention.F = _DenseLoopSDPA()
    torch.manual_seed(seed)
    model = EncoderDecoderRetrievalModel(embedding_dim=E, attn_dim=A, dropout=0.0, num_heads=H,
                                         n_layers=n_layers, num_embeddings=K, sem_id_dim=L1,
                                         inference_verifier_fn=None, max_pos=n_max * L1, jagged_mode=True)
    for m in model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    with torch.no_grad():
        for name, p in model.named_parameters():
            p.copy_(torch.from_numpy(gi.named_param(name, p.shape, seed)))
    model.train()
    tb = tokenized_batch(B, n_max, L1, K, seed + 1)
    batch = TokenizedSeqBatch(**{k: torch.from_numpy(v) for k, v in tb.items()})
    o = model(batch)
    o.loss.backward()
    out = dict(E=E, A=A, H=H, n_layers=n_layers, K=K, L1=L1, B=B, n_max=n_max, seed=seed,
               sdpa_substitute=1, loss=npf(o.loss), logits=npf(o.logits), loss_d=npf(o.loss_d), **tb)
    for name, p in model.named_parameters():
        if p.grad is None:
            continue
        if p.numel() <= 16384:
            out["grad__" + name] = npf(p.grad)
        else:   # large FFN weights: norm + first row
            out["grad__" + name + "__norm"] = np.float64(p.grad.double().norm().item())
            out["grad__" + name + "__row0"] = npf(p.grad[0])
    save(f"decoder_{tag}.npz", **out)


# --------------------------------------------------------------------- tokenizer
class _ItemSet:
    def __init__(self, x):
        self.x = torch.from_numpy(x)

    def __len__(self):
        return self.x.shape[0]

    def __getitem__(self, idx):   # same index semantics as reference data/processed.py:353-363
        item_ids = torch.tensor(idx).unsqueeze(0) if not isinstance(idx, torch.Tensor) else idx
        return SeqBatch(user_ids=-1 * torch.ones_like(item_ids.squeeze(0)), ids=item_ids,
                        ids_fut=-1 * torch.ones_like(item_ids.squeeze(0)), x=self.x[idx],
                        x_fut=-1 * torch.ones_like(item_ids.squeeze(0)), seq_mask=torch.ones_like(item_ids, dtype=bool))


def tokenizer_fixture(seed=11):
    inp, hidden, D, K, L = 48, [32], 8, 4, 3     # tiny K => many duplicate tuples
    tok = SemanticIdTokenizer(input_dim=inp, output_dim=D, hidden_dims=hidden, codebook_size=K,
                              n_layers=L, n_cat_feats=0)
    items = gi.items(1300, inp, seed)
    cbs = [gi.residual_rows(K, D, seed + 10 + l, scale=0.5) for l in range(L)]
    tok.rq_vae.load_state_dict(rqvae_state((inp, hidden, D), cbs, seed))
    ids = tok.precompute_corpus_ids(_ItemSet(items))
    seq_ids = gi.rng(seed + 3).integers(-1, 1300, size=(6, 5)).astype(np.int64)
    seq_ids[:, 0] = np.abs(seq_ids[:, 0])
    fut = gi.rng(seed + 4).integers(0, 1300, size=(6, 1)).astype(np.int64)
    sb = SeqBatch(user_ids=torch.arange(6), ids=torch.from_numpy(seq_ids), ids_fut=torch.from_numpy(fut),
                  x=None, x_fut=None, seq_mask=torch.from_numpy(seq_ids >= 0))
    t = tok(sb)
    prefixes = torch.from_numpy(gi.rng(seed + 5).integers(0, K, size=(40, 2)).astype(np.int64))
    out = dict(inp=inp, hidden=np.array(hidden), D=D, K=K, L=L, seed=seed, n_items=1300,
               codebooks=np.stack(cbs), corpus_ids=ids.numpy().astype(np.int64),
               seq_ids=seq_ids, fut_ids=fut, tok_sem_ids=t.sem_ids.numpy().astype(np.int64),
               tok_sem_ids_fut=t.sem_ids_fut.numpy().astype(np.int64), tok_seq_mask=t.seq_mask.numpy(),
               prefixes=prefixes.numpy(), exists_prefix=tok.exists_prefix(prefixes).numpy())
    save("tokenizer.npz", **out)


# ------------------------------------------------------------------------ kmeans
def kmeans_fixture():
    x = gi.residual_rows(600, 8, 5)
    np.random.seed(1234)     # reference draws its init with the global np.random (init/kmeans.py:36)
    init_idx = np.random.choice(600, 16, replace=False)
    np.random.seed(1234)
    torch.manual_seed(0)
    km = Kmeans(k=16, max_iters=50).run(torch.from_numpy(x))
    save("kmeans.npz", x=x, k=16, max_iters=50, np_seed=1234, init_idx=init_idx.astype(np.int64),
         centroids=npf(km.centroids), assignment=km.assignment.numpy().astype(np.int64))


if __name__ == "__main__":
    quantize_fixture("amazon", B=256, D=32, K=256, seed=101, store_inputs=True)
    quantize_fixture("ml32m", B=256, D=64, K=256, seed=202, store_inputs=True)
    quantize_fixture("synth", B=24, D=1024, K=2048, seed=303, store_inputs=False, modes=("rotation", "eval"))
    rqvae_fixture("small", inp=96, hidden=[64, 32], D=16, K=32, L=3, B=128, seed=11, store_grads_full=True)
    rqvae_fixture("ml32m", inp=768, hidden=[512, 256, 128], D=64, K=256, L=3, B=64, seed=12,
                  store_grads_full=False)
    jagged_fixture()
    decoder_fixture("small", E=32, A=64, H=4, n_layers=4, K=16, L1=4, B=6, n_max=5, seed=21)
    tokenizer_fixture()
    kmeans_fixture()
