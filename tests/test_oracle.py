"""Pin the CPU oracle against golden vectors captured from the reference itself.

Tolerances: ids / offsets / ranks exact; floats rtol 1e-5 (+ small atol) — the oracle is
float32 numpy vs the reference's float32 torch-CPU, so only summation order differs.
"""
import numpy as np
import pytest

import gen_inputs as gi
from oracle import quantize as Q, jagged as J, unique as U, rqvae as R, kmeans as KM, attention as A

MODE = {"rotation": Q.MODE_ROTATION, "ste": Q.MODE_STE, "eval": Q.MODE_EVAL}


def _close(a, b, rtol=1e-5, atol=1e-6, what=""):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    err = np.abs(a - b) - (atol + rtol * np.abs(b))
    assert err.max() <= 0, f"{what}: max abs diff {np.abs(a - b).max():.3e}"


def _quantize_inputs(z):
    if "x" in z:
        return z["x"], z["codebook"]
    x, cb = gi.quantize_case(int(z["B"]), int(z["D"]), int(z["K"]), int(z["seed"]))
    assert gi.checksum(x) == pytest.approx(float(z["x_checksum"]), abs=0)
    assert gi.checksum(cb) == pytest.approx(float(z["cb_checksum"]), abs=0)
    return x, cb


@pytest.mark.parametrize("tag", ["amazon", "ml32m", "synth"])
def test_quantize_level(golden, tag):
    z = golden(f"quantize_{tag}")
    x, cb = _quantize_inputs(z)
    safe = z["margin"] > 1e-5
    for mname in [str(m) for m in z["modes"]]:
        mode = MODE[mname]
        ids, emb, loss, aux = Q.level_fwd(x, cb, mode)
        assert np.array_equal(ids[safe], z[f"{mname}_ids"][safe]), mname
        assert (ids == z[f"{mname}_ids"]).all(), f"{mname}: near-tie flip"
        _close(emb, z[f"{mname}_emb"], 2e-5, 2e-6, f"{mname} emb")
        _close(loss, z[f"{mname}_loss"], 2e-5, 1e-6, f"{mname} loss")
        gx, gcb = Q.level_bwd(x, ids, cb.shape[0], mode, aux, z["g_emb"], z["g_loss"])
        _close(gx, z[f"{mname}_grad_x"], 2e-4, 1e-5, f"{mname} grad_x")
        rows = z[f"{mname}_gcb_rows"]
        assert set(np.nonzero(np.abs(gcb).sum(1))[0]) <= set(rows)
        _close(gcb[rows], z[f"{mname}_gcb"], 2e-4, 1e-5, f"{mname} grad_cb")


def test_quantize_chain_near_ties(golden):
    """The oracle's argmin on the reference's own level residuals of the near-tie fixture (twin codewords,
    top-2 gaps ~1e-6): the reference's ids on every row whose fp64 gap exceeds fp32 resolution (1e-6),
    lowest index among exact ties (torch.min, quantize.py:121)."""
    z = golden("rqvae_ml32m_ties")
    res, cbs, ref, margin = z["eval_level_residuals"], z["codebooks"], z["eval_sem_ids"], z["eval_margin"]
    for l in range(int(z["L"])):
        ids = Q.argmin_first(Q.l2_dist(res[l], cbs[l]))
        ok = margin[:, l] > 1e-6
        assert ok.mean() > 0.8
        assert np.array_equal(ids[ok], ref[ok, l]), l


def _rqvae_state(z):
    inp, hidden, D, L, seed = int(z["inp"]), [int(h) for h in z["hidden"]], int(z["D"]), int(z["L"]), int(z["seed"])
    enc = gi.mlp_weights([inp] + hidden + [D], seed)
    dec = gi.mlp_weights([D] + hidden[::-1] + [inp], seed + 1)
    st = {f"encoder.mlp.{2 * j}.weight": w for j, w in enumerate(enc)}
    st.update({f"decoder.mlp.{2 * j}.weight": w for j, w in enumerate(dec)})
    st.update({f"layers.{l}.embedding.weight": z["codebooks"][l] for l in range(L)})
    return st


@pytest.mark.parametrize("tag", ["small", "ml32m"])
def test_rqvae_step(golden, tag):
    z = golden(f"rqvae_{tag}")
    x = gi.items(int(z["B"]), int(z["inp"]), int(z["seed"]) + 200)
    assert gi.checksum(x) == float(z["x_checksum"])
    model = R.RqVaeOracle(_rqvae_state(z), int(z["L"]))
    # eval-mode semantic ids (tokenizer path)
    res0, _ = R.mlp_fwd(x, [model.state[k] for k in model.enc_keys], False)
    ev = Q.rq_fwd(res0, model.codebooks(), Q.MODE_EVAL)
    assert np.array_equal(ev["ids"], z["eval_sem_ids"])
    _close(ev["emb"].transpose(1, 2, 0), z["eval_embeddings"], 1e-4, 1e-6, "eval emb")
    _close(ev["res"].transpose(1, 2, 0), z["eval_residuals"], 1e-4, 1e-5, "eval res")
    out, grads = model.forward_backward(x)
    assert np.array_equal(out["sem_ids"], z["train_sem_ids"])
    _close(out["loss"], z["loss"], 1e-5, 0, "loss")
    _close(out["reconstruction_loss"], z["reconstruction_loss"], 1e-5, 0, "recon")
    _close(out["rqvae_loss"], z["rqvae_loss"], 1e-5, 0, "rqvae_loss")
    _close(out["embs_norm"], z["embs_norm"], 1e-5, 1e-6, "embs_norm")
    assert out["p_unique_ids"] == pytest.approx(float(z["p_unique_ids"]), abs=1e-7)
    for k, g in grads.items():
        key = "grad__" + k.replace(".", "_")
        if key in z:
            _close(g, z[key], 5e-4, 1e-6, key)
        else:
            assert np.linalg.norm(g.astype(np.float64)) == pytest.approx(float(z[key + "__norm"]), rel=1e-4)
            _close(g[0], z[key + "__row0"], 5e-4, 1e-6, key + " row0")


def test_jagged(golden):
    z = golden("jagged")
    for case in ("ragged", "full", "ctx"):
        x, lens = z[f"{case}_x"], z[f"{case}_lengths"]
        vals, off = J.padded_to_jagged(x, lens)
        assert np.array_equal(off, z[f"{case}_offsets"])
        assert np.array_equal(vals.view(np.uint32), z[f"{case}_values"].view(np.uint32)), "bitwise (x+1)-1"
        g = J.jagged_to_padded_grad(z[f"{case}_gv"], lens, x.shape[1])
        assert np.array_equal(g, z[f"{case}_grad_x"])


def test_plus_one_minus_one_is_not_identity(golden):
    z = golden("jagged")
    x, lens = z["ragged_x"], z["ragged_lengths"]
    raw, _ = J.padded_to_jagged(x, lens, add_one_sub_one=False)
    assert not np.array_equal(raw, z["ragged_values"])


def test_unique_and_dedup(golden):
    z = golden("tokenizer")
    ids = z["corpus_ids"]
    assert np.array_equal(U.dedup_rank(ids[:, :-1]), ids[:, -1])
    r = golden("rqvae_small")
    assert U.count_unique_rows(r["train_sem_ids"]) / r["train_sem_ids"].shape[0] == pytest.approx(float(r["p_unique_ids"]))


def test_kmeans(golden):
    z = golden("kmeans")
    c, a = KM.kmeans(z["x"], z["init_idx"], int(z["max_iters"]))
    assert np.array_equal(a, z["assignment"])
    _close(c, z["centroids"], 1e-5, 1e-6, "centroids")


def test_attention_oracle_self_consistent():
    """Finite-difference check of the attention VJP (the reference attention is torch SDPA;
    the decoder fixture pins the whole model that uses it, see test_decoder_*)."""
    g = gi.rng(5)
    cu = np.array([0, 3, 3, 8])
    q, k, v = (g.standard_normal((8, 2, 4)) for _ in range(3))
    do = g.standard_normal((8, 2, 4))
    for causal in (False, True):
        dq, dk, dv = A.attn_bwd(q, k, v, do, cu, cu, causal)
        eps = 1e-6
        for arr, grad in ((q, dq), (k, dk), (v, dv)):
            idx = (4, 1, 2)
            arr[idx] += eps
            fp = (A.attn_fwd(q, k, v, cu, cu, causal)[0] * do).sum()
            arr[idx] -= 2 * eps
            fm = (A.attn_fwd(q, k, v, cu, cu, causal)[0] * do).sum()
            arr[idx] += eps
            assert (fp - fm) / (2 * eps) == pytest.approx(grad[idx], rel=1e-5, abs=1e-8)


@pytest.mark.parametrize("tag", ["small", "dm"])
def test_decoder_oracle_vs_reference(golden, tag):
    """oracle/decoder.py (padded + masks, plain torch CPU) against the reference's own decoder fixture:
    loss, logits, per-position loss and the parameter gradients."""
    import torch
    from oracle import decoder as Dm
    z = golden(f"decoder_{tag}")
    E, A, H, nl, K, L1, n_max, seed = (int(z[k]) for k in ("E", "A", "H", "n_layers", "K", "L1", "n_max", "seed"))
    names = [k[len("grad__"):].replace("__norm", "") for k in z if k.startswith("grad__") and not k.endswith("__row0")]
    shapes = {n: (z["grad__" + n].shape if "grad__" + n in z else None) for n in names}
    # parameter shapes: small tensors are stored whole; the rest from the module layout
    from modules.model import EncoderDecoderRetrievalModel
    m = EncoderDecoderRetrievalModel(embedding_dim=E, attn_dim=A, dropout=0.0, num_heads=H, n_layers=nl,
                                     num_embeddings=K, sem_id_dim=L1, inference_verifier_fn=None, max_pos=n_max * L1)
    P = {n: torch.from_numpy(gi.named_param(n, p.shape, seed)).requires_grad_(True) for n, p in m.named_parameters()}
    keys = ("user_ids", "sem_ids", "sem_ids_fut", "seq_mask", "token_type_ids", "token_type_ids_fut")
    batch = {k: torch.from_numpy(z[k]) for k in keys}
    loss, logits, loss_d = Dm.decoder_forward(P, batch, K, L1, H, nl, dropout=0.0)
    loss.backward()
    assert float(loss) == pytest.approx(float(z["loss"]), rel=2e-6)
    assert np.abs(logits.detach().numpy() - z["logits"]).max() <= 2e-6 * np.abs(z["logits"]).max()
    assert np.allclose(loss_d.detach().numpy(), z["loss_d"], rtol=1e-5, atol=1e-7)
    checked = 0
    for n in names:
        g = P[n].grad
        if "grad__" + n in z:
            ref = z["grad__" + n]
            assert np.abs(g.numpy() - ref).max() <= 2e-5 * np.abs(ref).max() + 1e-7, n
        else:
            assert g.double().norm().item() == pytest.approx(float(z["grad__" + n + "__norm"]), rel=2e-5), n
        checked += 1
    assert checked == len(names) and shapes


def test_rqvae_torch_cpu_matches_numpy_oracle():
    """bench.py's eager torch-CPU RQ-VAE baseline (oracle/rqvae_torch.py) computes the pinned numpy
    oracle's step: same ids, loss and parameter gradients (rotation-trick mode, small dims)."""
    from oracle.rqvae_torch import RqVaeTorchCPU
    inp, hid, D, K, L, B = 96, [64, 32], 16, 32, 3, 256
    st = {f"encoder.mlp.{2 * j}.weight": w for j, w in enumerate(gi.mlp_weights([inp] + hid + [D], 1))}
    st.update({f"decoder.mlp.{2 * j}.weight": w for j, w in enumerate(gi.mlp_weights([D] + hid[::-1] + [inp], 2))})
    st.update({f"layers.{l}.embedding.weight": gi.residual_rows(K, D, 10 + l, 0.5) for l in range(L)})
    x = gi.items(B, inp, 3)
    out, grads = R.RqVaeOracle(st, L).forward_backward(x)
    loss, ids, tgrads = RqVaeTorchCPU(st, L).forward_backward(x)
    assert np.array_equal(ids, out["sem_ids"])
    assert loss == pytest.approx(float(out["loss"]), rel=1e-5)
    for k, g in grads.items():
        np.testing.assert_allclose(tgrads[k], g, rtol=2e-4, atol=1e-6, err_msg=k)
