#!/usr/bin/env python3
"""Generate the golden parity fixtures by importing the READ-ONLY reference.

Test infrastructure only; run in the build container (never on the GPU box, where
/root/reference does not exist):

    python tests/golden/make_golden.py [/root/reference] [fixture names ... (default: all)]

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
REF = next((a for a in sys.argv[1:] if os.path.isdir(a)), "/root/reference")
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gen_inputs as gi  # noqa: E402


try:   # before the stubs: accelerate probes find_spec("swanlab"), which a stub without a spec breaks
    import accelerate  # noqa: E402,F401  (train_rqvae.py:7; only the training-trace fixture needs it)
except ImportError:  # pragma: no cover
    pass


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

from modules.quantize import Quantize, QuantizeForwardMode, QuantizeDistance  # noqa: E402
from modules.rqvae import RqVae  # noqa: E402
from modules.model import EncoderDecoderRetrievalModel  # noqa: E402
from modules.tokenizer.semids import SemanticIdTokenizer  # noqa: E402
from data.schemas import SeqBatch, TokenizedSeqBatch  # noqa: E402
from ops.triton.jagged import padded_to_jagged_tensor  # noqa: E402
from init.kmeans import Kmeans  # noqa: E402
import modules.transformer.attention as ref_attention  # noqa: E402
import distributions.gumbel as ref_gumbel  # noqa: E402
import modules.quantize as ref_quantize  # noqa: E402

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


def rqvae_ties_fixture(inp=768, hidden=(512, 256, 128), D=64, K=256, L=3, B=512, seed=12, pairs=24, eps=3e-6):
    """ML-32M dims with near-tied codebooks: at every level, `pairs` codewords get a twin c + eps * |c| u
    (u a random unit vector), so the items nearest to them sit on a top-2 gap of ~1e-6 — far below the
    'high' margin (1e-4) — and the margin-unsafe branch of the 'high' contract is exercised against the
    reference's own ids. Stores the reference eval ids, per-level residuals and margins."""
    hidden = list(hidden)
    model = RqVae(input_dim=inp, embed_dim=D, hidden_dims=hidden, codebook_size=K,
                  codebook_kmeans_init=False, codebook_mode=QuantizeForwardMode.ROTATION_TRICK,
                  n_layers=L, n_cat_features=0, commitment_weight=0.25)
    cb_items = gi.items(max(4 * K, 512), inp, seed + 100)
    model.load_state_dict(rqvae_state((inp, hidden, D), [np.zeros((K, D), F32)] * L, seed))
    cbs = make_codebooks(model, cb_items, K, L, seed)
    g = gi.rng(seed + 777)
    for l in range(L):
        src = g.permutation(K)[:2 * pairs]
        for a, b in zip(src[:pairs], src[pairs:]):
            u = g.standard_normal(D)
            u /= np.linalg.norm(u)
            cbs[l][b] = (cbs[l][a].astype(np.float64) + eps * np.linalg.norm(cbs[l][a]) * u).astype(F32)
    model.load_state_dict(rqvae_state((inp, hidden, D), cbs, seed))
    x_np = gi.items(B, inp, seed + 300)
    model.eval()
    with torch.no_grad():
        ev = model.get_semantic_ids(torch.from_numpy(x_np))
        res = model.encode(torch.from_numpy(x_np)).numpy()
        margins, res_l = [], []
        for l in range(L):
            res_l.append(res.copy())
            margins.append(top2_margin(res, cbs[l]))
            res = res - cbs[l][ev.sem_ids[:, l].numpy()]
    save("rqvae_ml32m_ties.npz", inp=inp, hidden=np.array(hidden, np.int64), D=D, K=K, L=L, B=B, seed=seed,
         x_checksum=gi.checksum(x_np), codebooks=np.stack(cbs), eval_sem_ids=ev.sem_ids.numpy().astype(np.int64),
         eval_level_residuals=np.stack(res_l).astype(F32), eval_margin=np.stack(margins, 1))


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


def tokenized_batch(B, n_max, L1, K, seed, full_first=False):
    g = gi.rng(seed)
    n_items = g.integers(1, n_max + 1, size=B)
    if full_first:   # the config's longest context: n_max items -> n_max * L1 + 1 tokens
        n_items[0] = n_max
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


def decoder_fixture(tag, E, A, H, n_layers, K, L1, B, n_max, seed, full_first=False):
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
    tb = tokenized_batch(B, n_max, L1, K, seed + 1, full_first)
    batch = TokenizedSeqBatch(**{k: torch.from_numpy(v) for k, v in tb.items()})
    o = model(batch)
    o.loss.backward()
    out = dict(E=E, A=A, H=H, n_layers=n_layers, K=K, L1=L1, B=B, n_max=n_max, seed=seed,
               full_first=int(full_first), sdpa_substitute=1, loss=npf(o.loss), logits=npf(o.logits), loss_d=npf(o.loss_d), **tb)
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


# ------------------------------------------------------------- quantize variants (a4)
def quantize_variants_fixture(B=128, D=64, K=256, seed=404, T=0.2):
    """Gumbel-softmax (the reference's default mode, quantize.py:124-129 with noise injected through
    a patched distributions.gumbel.sample_gumbel), COSINE distance (:113-117), sim_vq (out_proj
    Linear, :64-67) and codebook_normalize (L2-normalised codebook, :68-70) at ML-32M dims."""
    x_np, cb_np = gi.quantize_case(B, D, K, seed)
    g = gi.rng(seed + 1)
    g_emb = g.standard_normal((B, D), dtype=F32)
    g_loss = g.random(B, dtype=F32)
    noise = gi.gumbel_noise((B, K), seed + 2)
    proj_w = gi.linear_weight(D, D, seed + 3)
    out = dict(B=B, D=D, K=K, seed=seed, T=F32(T), x=x_np, codebook=cb_np, g_emb=g_emb, g_loss=g_loss,
               noise_checksum=gi.checksum(noise), proj_w=proj_w)
    variants = {   # name: (forward_mode, distance, sim_vq, codebook_normalize, training)
        "gumbel": (QuantizeForwardMode.GUMBEL_SOFTMAX, QuantizeDistance.L2, False, False, True),
        "gumbel_eval": (QuantizeForwardMode.GUMBEL_SOFTMAX, QuantizeDistance.L2, False, False, False),
        "cosine_rotation": (QuantizeForwardMode.ROTATION_TRICK, QuantizeDistance.COSINE, False, False, True),
        "cosine_eval": (QuantizeForwardMode.ROTATION_TRICK, QuantizeDistance.COSINE, False, False, False),
        "simvq_rotation": (QuantizeForwardMode.ROTATION_TRICK, QuantizeDistance.L2, True, False, True),
        "cbnorm_ste": (QuantizeForwardMode.STE, QuantizeDistance.L2, False, True, True),
        "simvq_gumbel": (QuantizeForwardMode.GUMBEL_SOFTMAX, QuantizeDistance.L2, True, False, True),
    }
    orig = ref_gumbel.sample_gumbel
    ref_gumbel.sample_gumbel = lambda shape, device, eps=1e-20: torch.from_numpy(noise.copy()).reshape(shape)
    try:
        for name, (fm, dm, sim, cbn, training) in variants.items():
            q = Quantize(D, K, do_kmeans_init=False, codebook_normalize=cbn, sim_vq=sim, forward_mode=fm,
                         distance_mode=dm)
            with torch.no_grad():
                q.embedding.weight.copy_(torch.from_numpy(cb_np))
                if sim:
                    q.out_proj[0].weight.copy_(torch.from_numpy(proj_w))
            q.train(training)
            x = torch.from_numpy(x_np.copy()).requires_grad_(True)
            o = q(x, temperature=T)
            ((o.embeddings * torch.from_numpy(g_emb)).sum() + (o.loss * torch.from_numpy(g_loss)).sum()).backward()
            out.update({f"{name}_ids": o.ids.numpy().astype(np.int64), f"{name}_emb": npf(o.embeddings),
                        f"{name}_loss": npf(o.loss), f"{name}_grad_x": npf(x.grad),
                        f"{name}_grad_cb": npf(q.embedding.weight.grad)})
            if sim:
                out[f"{name}_grad_proj"] = npf(q.out_proj[0].weight.grad)
    finally:
        ref_gumbel.sample_gumbel = orig
    out["variants"] = np.array(list(variants))
    save("quantize_variants.npz", **out)


# ------------------------------------------------------------------ generation (f3)
def generation_fixture(E=32, A=64, H=4, n_layers=4, K=256, L1=4, B=3, n_max=5, seed=41):
    """EncoderDecoderRetrievalModel.generate_next_sem_id (modules/model.py:149-245) with
    torch.multinomial replaced by a deterministic top-n (gi.topn_multinomial) and a deterministic
    prefix verifier (gi.prefix_verifier) — the same patches the GPU test applies to this build."""
    ref_attention.F = _DenseLoopSDPA()
    model = EncoderDecoderRetrievalModel(embedding_dim=E, attn_dim=A, dropout=0.3, num_heads=H, n_layers=n_layers,
                                         num_embeddings=K, sem_id_dim=L1, inference_verifier_fn=gi.prefix_verifier,
                                         max_pos=n_max * L1, jagged_mode=True)
    with torch.no_grad():
        for name, p in model.named_parameters():
            v = gi.named_param(name, p.shape, seed)
            if name == "out_proj.weight":
                v = v * 4.0     # well-separated candidate probabilities
            p.copy_(torch.from_numpy(v))
    tb = tokenized_batch(B, n_max, L1, K, seed + 1)
    batch = TokenizedSeqBatch(**{k: torch.from_numpy(v) for k, v in tb.items()})
    model.enable_generation = True
    orig = torch.multinomial
    torch.multinomial = gi.topn_multinomial
    try:
        for top_k in (True, False):
            g = model.generate_next_sem_id(batch, temperature=1, top_k=top_k)
            tag = "topk" if top_k else "greedy"
            tb[f"{tag}_sem_ids"] = g.sem_ids.numpy().astype(np.int64)
            tb[f"{tag}_log_probas"] = npf(g.log_probas)
    finally:
        torch.multinomial = orig
    save("generation.npz", E=E, A=A, H=H, n_layers=n_layers, K=K, L1=L1, B=B, n_max=n_max, seed=seed,
         out_proj_scale=F32(4.0), sdpa_substitute=1, **tb)


# ------------------------------------------------------------ checkpoints (f4)
def checkpoint_fixture(seed=11, steps=3, lr=5e-4, wd=0.01):
    """A checkpoint in the reference's train_rqvae.py:209-221 layout {"iter", "model", "optimizer"}
    (tensors / plain containers only, so it loads with weights_only=True; the reference's
    model_config pickles the module itself, SURVEY A-13) written by the reference RqVae + torch AdamW
    after `steps` steps, plus the reference's NEXT step from it (loss, updated parameters). Also the
    reference's state-dict key/shape manifests of RqVae and EncoderDecoderRetrievalModel."""
    inp, hidden, D, K, L = 96, [64, 32], 16, 32, 3
    model = RqVae(input_dim=inp, embed_dim=D, hidden_dims=hidden, codebook_size=K, codebook_kmeans_init=False,
                  codebook_mode=QuantizeForwardMode.ROTATION_TRICK, n_layers=L, n_cat_features=0)
    z = np.load(os.path.join(HERE, "rqvae_small.npz"))
    model.load_state_dict(rqvae_state((inp, hidden, D), list(z["codebooks"]), seed))
    opt = torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=wd)

    def step(i):
        x = torch.from_numpy(gi.items(64, inp, 700 + i))
        opt.zero_grad()
        o = model(SeqBatch(None, None, None, x, None, None), gumbel_t=0.2)
        o.loss.backward()
        opt.step()
        return float(o.loss)
    for i in range(steps):
        step(i)
    torch.save({"iter": steps - 1, "model": model.state_dict(), "optimizer": opt.state_dict()},
               os.path.join(HERE, "ckpt_rqvae_small.pt"))
    print("wrote ckpt_rqvae_small.pt")
    loss = step(steps)
    out = {"next_loss": np.float64(loss), "iter": steps - 1, "lr": lr, "wd": wd, "seed": seed}
    for name, p in model.named_parameters():
        out["next__" + name] = npf(p)
    for name, t in RqVae(input_dim=768, embed_dim=32, hidden_dims=[512, 256, 128], codebook_size=256,
                         codebook_kmeans_init=False, n_layers=3, n_cat_features=0).state_dict().items():
        out["rqvae_keys__" + name] = np.array(t.shape, np.int64)
    dec = EncoderDecoderRetrievalModel(embedding_dim=128, attn_dim=512, dropout=0.3, num_heads=8, n_layers=8,
                                       num_embeddings=256, sem_id_dim=4, inference_verifier_fn=None, max_pos=80)
    for name, t in dec.state_dict().items():
        out["decoder_keys__" + name] = np.array(t.shape, np.int64)
    out["decoder_n_params"] = np.int64(sum(p.numel() for p in dec.parameters()))
    save("checkpoint.npz", **out)


# ----------------------------------------------------------- C1 loss trace (train_rqvae.train)
def train_trace_fixture(iterations=24, batch_size=64, seed=0, np_seed=2024, sampler_seed=5, w_seed=13):
    """A (iterations+1)-step run of the reference's own train_rqvae.train() at configs/rqvae_amazon.gin
    dims (768 -> [512,256,128] -> 32, K=256, L=3, ROTATION_TRICK, AdamW 1e-4 / 0.01, k-means init on
    the first min(20000, N) items), on the build's seeded synthetic Amazon-sized corpus. Patched into
    the reference module: ItemData (synthetic corpus), RandomSampler (seeded permutation per epoch,
    gi.batch_permutation), RqVae (numpy-seeded MLP weights after construction, per-step loss
    recording), np.random.seed(np_seed) for the k-means init draws. Records the batch indices, the
    post-k-means codebooks and the per-step losses."""
    import train_rqvae as tr
    from torch.utils.data import Sampler
    x_train, x_eval, x_all = gi.synthetic_item_corpus(12101, seed)

    class _Items:
        def __init__(self, *a, train_test_split="all", **k):
            self.x = torch.from_numpy({"train": x_train, "eval": x_eval}.get(train_test_split, x_all))

        def __len__(self):
            return self.x.shape[0]

        def __getitem__(self, idx):
            item_ids = torch.tensor(idx).unsqueeze(0) if not isinstance(idx, torch.Tensor) else idx
            neg = -torch.ones_like(item_ids.squeeze(0))
            return SeqBatch(user_ids=neg, ids=item_ids, ids_fut=neg, x=self.x[idx, :768], x_fut=neg,
                            seq_mask=torch.ones_like(item_ids, dtype=torch.bool))

    class _Sampler(Sampler):
        epochs = {}

        def __init__(self, ds):
            self.n = len(ds)
            self.key = id(ds)

        def __len__(self):
            return self.n

        def __iter__(self):
            e = _Sampler.epochs.get(self.key, 0)
            _Sampler.epochs[self.key] = e + 1
            return iter(gi.batch_permutation(self.n, sampler_seed, e).tolist())

    record = {"loss": [], "rl": [], "vl": [], "pu": [], "idx": []}
    kmeans_cbs = []
    orig_init = ref_quantize.kmeans_init_

    def kmeans_rec(tensor, x):
        orig_init(tensor, x)
        kmeans_cbs.append(tensor.detach().numpy().copy())

    class _RqVae(RqVae):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            enc = gi.mlp_weights([self.input_dim] + list(self.hidden_dims) + [self.embed_dim], w_seed)
            dec = gi.mlp_weights([self.embed_dim] + list(self.hidden_dims)[::-1] + [self.input_dim], w_seed + 1)
            with torch.no_grad():
                for j, w in enumerate(enc):
                    self.encoder.mlp[2 * j].weight.copy_(torch.from_numpy(w))
                for j, w in enumerate(dec):
                    self.decoder.mlp[2 * j].weight.copy_(torch.from_numpy(w))

        def forward(self, batch, gumbel_t):
            o = super().forward(batch, gumbel_t)
            if self.training and batch.x.shape[0] == batch_size:
                record["loss"].append(float(o.loss))
                record["rl"].append(float(o.reconstruction_loss))
                record["vl"].append(float(o.rqvae_loss))
                record["pu"].append(float(o.p_unique_ids))
                record["idx"].append(batch.ids.numpy().astype(np.int64).copy())
            return o

    saved = (tr.ItemData, tr.RandomSampler, tr.RqVae, ref_quantize.kmeans_init_, torch.save)
    tr.ItemData, tr.RandomSampler, tr.RqVae, ref_quantize.kmeans_init_ = _Items, _Sampler, _RqVae, kmeans_rec
    torch.save = lambda *a, **k: None   # the end-of-run checkpoint pickles the (local) model class
    cwd = os.getcwd()
    import tempfile
    try:
        with tempfile.TemporaryDirectory() as d:
            os.chdir(d)
            np.random.seed(np_seed)
            torch.manual_seed(0)
            tr.train(iterations=iterations, batch_size=batch_size, learning_rate=1e-4, weight_decay=0.01,
                     vae_input_dim=768, vae_embed_dim=32, vae_hidden_dims=[512, 256, 128], vae_codebook_size=256,
                     vae_n_layers=3, vae_n_cat_feats=0, vae_codebook_mode=QuantizeForwardMode.ROTATION_TRICK,
                     commitment_weight=0.25, use_kmeans_init=True, do_eval=True, save_dir_root=d + "/",
                     eval_every=10 ** 9, save_model_every=10 ** 9)
    finally:
        os.chdir(cwd)
        tr.ItemData, tr.RandomSampler, tr.RqVae, ref_quantize.kmeans_init_, torch.save = saved
    assert len(record["loss"]) == iterations + 1, len(record["loss"])
    save("train_trace_amazon.npz", iterations=iterations, batch_size=batch_size, seed=seed, np_seed=np_seed,
         sampler_seed=sampler_seed, w_seed=w_seed, lr=1e-4, wd=0.01, n_train=x_train.shape[0],
         kmeans_codebooks=np.stack(kmeans_cbs), batch_idx=np.stack(record["idx"]),
         loss=np.array(record["loss"]), reconstruction_loss=np.array(record["rl"]),
         rqvae_loss=np.array(record["vl"]), p_unique_ids=np.array(record["pu"]))


FIXTURES = {
    "quantize_amazon": lambda: quantize_fixture("amazon", B=256, D=32, K=256, seed=101, store_inputs=True),
    "quantize_ml32m": lambda: quantize_fixture("ml32m", B=256, D=64, K=256, seed=202, store_inputs=True),
    "quantize_synth": lambda: quantize_fixture("synth", B=24, D=1024, K=2048, seed=303, store_inputs=False,
                                               modes=("rotation", "eval")),
    "rqvae_small": lambda: rqvae_fixture("small", inp=96, hidden=[64, 32], D=16, K=32, L=3, B=128, seed=11,
                                         store_grads_full=True),
    "rqvae_ml32m": lambda: rqvae_fixture("ml32m", inp=768, hidden=[512, 256, 128], D=64, K=256, L=3, B=64, seed=12,
                                         store_grads_full=False),
    "rqvae_ml32m_ties": rqvae_ties_fixture,
    "jagged": jagged_fixture,
    "decoder_small": lambda: decoder_fixture("small", E=32, A=64, H=4, n_layers=4, K=16, L1=4, B=6, n_max=5, seed=21),
    # configs[3] (decoder_ml32m.gin: A=384, H=6, 8 layers, E=128): one sequence of 200 items = 801 ctx tokens
    "decoder_dm": lambda: decoder_fixture("dm", E=128, A=384, H=6, n_layers=8, K=256, L1=4, B=3, n_max=200, seed=22,
                                          full_first=True),
    # configs[4] jagged half (DA dims, L=4 -> 5 tokens per item, K=2048): one sequence of 256 items = 1281 tokens
    "decoder_c5": lambda: decoder_fixture("c5", E=128, A=512, H=8, n_layers=8, K=2048, L1=5, B=2, n_max=256, seed=23,
                                          full_first=True),
    "tokenizer": tokenizer_fixture,
    "kmeans": kmeans_fixture,
    "quantize_variants": quantize_variants_fixture,
    "generation": generation_fixture,
    "checkpoint": checkpoint_fixture,
    "train_trace": train_trace_fixture,
}


if __name__ == "__main__":
    names = [a for a in sys.argv[1:] if a in FIXTURES] or list(FIXTURES)
    for n in names:
        FIXTURES[n]()
