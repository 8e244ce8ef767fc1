"""Residual quantization (one level and the L-level chain) — numpy float32 restatement.

Reference: modules/quantize.py, modules/loss.py, modules/rqvae.py (AdamLTy/RQ-VAE-Recommender).
Test infrastructure only (see oracle/__init__.py).
"""
import numpy as np

F32 = np.float32
MODE_EVAL, MODE_GUMBEL, MODE_STE, MODE_ROTATION = 0, 1, 2, 3


def l2_dist(x, cb):
    """dist = (x^2).sum(1,keepdim) + (c^T^2).sum(0,keepdim) - 2 x c^T   (modules/quantize.py:108-112)."""
    x = x.astype(F32)
    cb = cb.astype(F32)
    return ((x * x).sum(1, keepdims=True, dtype=F32) + (cb * cb).sum(1, dtype=F32)[None, :]) - (F32(2) * x) @ cb.T


def argmin_first(dist):
    """ids = dist.min(axis=1).indices; ties resolve to the lowest index (modules/quantize.py:121)."""
    return np.argmin(dist, axis=1).astype(np.int64)


def _norm(v):
    return np.sqrt((v.astype(F32) * v).sum(-1, keepdims=True, dtype=F32)).astype(F32)


def rotation_fwd(x, emb):
    """efficient_rotation_trick_transform(u, q, e=x) * (|emb| / (|x|+1e-6)).detach()

    modules/quantize.py:34-45 (transform) and :135-142 (call + rescale):
      u = x/(|x|+1e-8), q = emb/(|emb|+1e-8), w = normalize(u+q, eps=1e-6)
      out = e - 2 (e.w) w + 2 (e.u) q
    Returns (emb_out, aux) where aux holds the detached constants the VJP needs.
    """
    xn, en = _norm(x), _norm(emb)
    u = (x / (xn + F32(1e-8))).astype(F32)
    q = (emb / (en + F32(1e-8))).astype(F32)
    s = (u + q).astype(F32)
    w = (s / np.maximum(_norm(s), F32(1e-6))).astype(F32)
    ew = (x * w).sum(-1, keepdims=True, dtype=F32)
    eu = (x * u).sum(-1, keepdims=True, dtype=F32)
    out = (x - F32(2) * (ew * w)) + F32(2) * (eu * q)
    lam = (en / (xn + F32(1e-6))).astype(F32)
    return (out * lam).astype(F32), dict(u=u, q=q, w=w, lam=lam)


def rotation_vjp(g, aux):
    """d emb_out / d x applied to g:  lam * (g - 2 (g.w) w + 2 (g.q) u)  (u,q,w,lam detached)."""
    u, q, w, lam = aux["u"], aux["q"], aux["w"], aux["lam"]
    gw = (g * w).sum(-1, keepdims=True, dtype=F32)
    gq = (g * q).sum(-1, keepdims=True, dtype=F32)
    return (lam * ((g - F32(2) * gw * w) + F32(2) * gq * u)).astype(F32)


def quantize_loss(x, emb, beta):
    """QuantizeLoss: |sg(x)-emb|^2 + beta |x-sg(emb)|^2 per row (modules/loss.py:34-42)."""
    d = (x - emb).astype(F32)
    s = (d * d).sum(-1, dtype=F32)
    return (s + F32(beta) * s).astype(F32)


def level_fwd(x, cb, mode, beta=0.25):
    """One Quantize.forward for L2 distance (modules/quantize.py:99-156).

    mode: MODE_ROTATION / MODE_STE (training) or MODE_EVAL (self.training False).
    Returns ids, emb_out, loss, aux.
    """
    x = x.astype(F32)
    ids = argmin_first(l2_dist(x, cb))
    emb = cb[ids].astype(F32)                       # get_item_embeddings: out_proj = Identity (:96-97)
    aux = dict(emb=emb)
    if mode == MODE_ROTATION:
        emb_out, r = rotation_fwd(x, emb)
        aux.update(r)
    elif mode == MODE_STE:
        emb_out = (x + (emb - x)).astype(F32)       # x + (emb - x).detach()  (:132)
    elif mode == MODE_EVAL:
        emb_out = emb                               # (:149)
    else:
        raise ValueError("mode")
    return ids, emb_out, quantize_loss(x, emb, beta), aux


def level_bwd(x, ids, K, mode, aux, g_emb, g_loss, beta=0.25):
    """VJP of level_fwd. Returns (grad_x, grad_codebook (K,D)).

    Gradients of the reference graph: emb_out depends on x only (rotation/STE; u,q,w,lam
    detached) or on the codebook only (eval); QuantizeLoss gives d/demb = 2(emb-x) g_loss,
    d/dx = 2 beta (x-emb) g_loss; the codebook grad is the embedding backward (index-add).
    """
    emb = aux["emb"]
    gl = g_loss.astype(F32)[:, None]
    D = x.shape[1]
    gcb = np.zeros((K, D), F32)
    if mode == MODE_ROTATION:
        gx = rotation_vjp(g_emb.astype(F32), aux)
    elif mode == MODE_STE:
        gx = g_emb.astype(F32).copy()
    else:
        gx = np.zeros_like(x, dtype=F32)
        np.add.at(gcb, ids, g_emb.astype(F32))
    gx = gx + F32(2 * beta) * gl * (x - emb)
    np.add.at(gcb, ids, (F32(2) * gl * (emb - x)).astype(F32))
    return gx.astype(F32), gcb


def rq_fwd(res0, codebooks, mode, beta=0.25):
    """RqVae.get_semantic_ids loop (modules/rqvae.py:114-138): res_{l+1} = res_l - emb_out_l.

    Returns dict with ids (B,L), emb (L,B,D), res (L,B,D), qloss (B,), auxs (per level).
    (The reference returns embeddings/residuals rearranged to (B,D,L) and sem_ids (B,L).)
    """
    res = res0.astype(F32)
    L = codebooks.shape[0]
    ids, embs, ress, auxs = [], [], [], []
    qloss = np.zeros(res.shape[0], F32)
    for l in range(L):
        ress.append(res)
        i, e, lo, a = level_fwd(res, codebooks[l], mode, beta)
        qloss = (qloss + lo).astype(F32)
        res = (res - e).astype(F32)
        ids.append(i)
        embs.append(e)
        auxs.append(a)
    return dict(ids=np.stack(ids, 1), emb=np.stack(embs), res=np.stack(ress), qloss=qloss, auxs=auxs)


def rq_bwd(fwd, codebooks, mode, g_emb_sum=None, g_emb=None, g_qloss=None, beta=0.25):
    """VJP of rq_fwd wrt (res0, codebooks). g_emb_sum: grad of sum_l emb_out_l (B,D);
    g_emb: per-level grads (L,B,D); g_qloss: grad of the summed quantize loss (B,)."""
    L, B, D = fwd["res"].shape
    K = codebooks.shape[1]
    g_next = np.zeros((B, D), F32)
    gcb = np.zeros_like(codebooks, dtype=F32)
    gl = np.zeros(B, F32) if g_qloss is None else g_qloss.astype(F32)
    for l in range(L - 1, -1, -1):
        g_out = np.zeros((B, D), F32)
        if g_emb_sum is not None:
            g_out = g_out + g_emb_sum.astype(F32)
        if g_emb is not None:
            g_out = g_out + g_emb[l].astype(F32)
        g_out = (g_out - g_next).astype(F32)
        gx, gc = level_bwd(fwd["res"][l], fwd["ids"][:, l], K, mode, fwd["auxs"][l], g_out, gl, beta)
        gcb[l] = gc
        g_next = (g_next + gx).astype(F32)
    return g_next, gcb


def p_unique_ids(sem_ids):
    """#distinct L-tuples / B (modules/rqvae.py:152-157, restated as a sort-unique count)."""
    return np.float32(np.unique(sem_ids, axis=0).shape[0] / sem_ids.shape[0])
