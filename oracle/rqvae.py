"""RqVae train step (encoder MLP -> L-level RQ -> decoder MLP -> losses -> AdamW) in numpy.

Reference: modules/rqvae.py:140-165 (forward), modules/encoder.py:7-36 (MLP),
modules/normalize.py:7-8 (l2norm eps 1e-12), modules/loss.py:5-10 (ReconstructionLoss),
torch.optim.AdamW (train_rqvae.py:96-100). n_cat_features = 0 as in every config
(the cat/l2norm at rqvae.py:146 is then a no-op).
Float32 numpy; used as the pinned checker and as bench.py's CPU baseline ("port").
Test infrastructure only.
"""
import numpy as np

from . import quantize as Q

F32 = np.float32


def _silu(z):
    return (z / (F32(1) + np.exp(-z))).astype(F32)


def _silu_grad(z):
    s = (F32(1) / (F32(1) + np.exp(-z))).astype(F32)
    return (s * (F32(1) + z * (F32(1) - s))).astype(F32)


def mlp_fwd(x, weights, normalize):
    """Linear(no bias) -> SiLU ... -> Linear [-> l2norm]   (modules/encoder.py:18-36)."""
    cache = []
    h = x.astype(F32)
    for j, w in enumerate(weights):
        z = (h @ w.T).astype(F32)
        cache.append((h, z))
        h = _silu(z) if j < len(weights) - 1 else z
    pre = h
    if normalize:
        n = np.maximum(np.sqrt((h * h).sum(-1, keepdims=True, dtype=F32)), F32(1e-12))
        h = (h / n).astype(F32)
        cache.append(("norm", n, h))
    return h, (cache, pre)


def mlp_bwd(g, weights, state, normalize):
    cache, pre = state
    grads = [None] * len(weights)
    if normalize:
        _, n, y = cache[-1]
        g = ((g - y * (g * y).sum(-1, keepdims=True, dtype=F32)) / n).astype(F32)
        cache = cache[:-1]
    for j in range(len(weights) - 1, -1, -1):
        h, z = cache[j]
        if j < len(weights) - 1:
            g = (g * _silu_grad(z)).astype(F32)
        grads[j] = (g.T @ h).astype(F32)
        g = (g @ weights[j]).astype(F32)
    return g, grads


class RqVaeOracle:
    """Parameters keyed by the reference state-dict names (encoder.mlp.{2j}.weight, ...)."""

    def __init__(self, state, n_layers, mode=Q.MODE_ROTATION, beta=0.25):
        self.state = {k: np.asarray(v, F32).copy() for k, v in state.items()}
        self.L = n_layers
        self.mode = mode
        self.beta = beta
        self.enc_keys = sorted([k for k in state if k.startswith("encoder.")], key=lambda s: int(s.split(".")[2]))
        self.dec_keys = sorted([k for k in state if k.startswith("decoder.")], key=lambda s: int(s.split(".")[2]))
        self.cb_keys = [f"layers.{l}.embedding.weight" for l in range(n_layers)]
        self.adam = {}

    def codebooks(self):
        return np.stack([self.state[k] for k in self.cb_keys])

    def forward_backward(self, x):
        """One RqVae.forward + loss.backward(); returns (outputs dict, grads dict)."""
        enc_w = [self.state[k] for k in self.enc_keys]
        dec_w = [self.state[k] for k in self.dec_keys]
        cbs = self.codebooks()
        res0, enc_state = mlp_fwd(x, enc_w, normalize=False)
        f = Q.rq_fwd(res0, cbs, self.mode, self.beta)
        emb_sum = f["emb"].sum(0, dtype=F32)
        x_hat, dec_state = mlp_fwd(emb_sum, dec_w, normalize=True)
        d = (x_hat - x).astype(F32)
        recon = (d * d).sum(-1, dtype=F32)
        B = x.shape[0]
        loss = F32((recon + f["qloss"]).mean(dtype=F32))
        # backward: d loss / d recon_b = d loss / d qloss_b = 1/B
        g_xhat = (F32(2.0 / B) * d).astype(F32)
        g_embsum, g_dec = mlp_bwd(g_xhat, dec_w, dec_state, normalize=True)
        g_res0, g_cb = Q.rq_bwd(f, cbs, self.mode, g_emb_sum=g_embsum,
                                g_qloss=np.full(B, 1.0 / B, F32), beta=self.beta)
        _, g_enc = mlp_bwd(g_res0, enc_w, enc_state, normalize=False)
        grads = {}
        for k, g in zip(self.enc_keys, g_enc):
            grads[k] = g
        for k, g in zip(self.dec_keys, g_dec):
            grads[k] = g
        for l, k in enumerate(self.cb_keys):
            grads[k] = g_cb[l]
        out = dict(loss=loss, reconstruction_loss=F32(recon.mean(dtype=F32)), rqvae_loss=F32(f["qloss"].mean(dtype=F32)),
                   sem_ids=f["ids"], embs_norm=np.sqrt((f["emb"] ** 2).sum(-1)).T.astype(F32),
                   p_unique_ids=Q.p_unique_ids(f["ids"]))
        return out, grads

    def adamw_step(self, grads, lr, weight_decay, betas=(0.9, 0.999), eps=1e-8):
        """torch.optim.AdamW (decoupled weight decay; bias-corrected moments)."""
        b1, b2 = betas
        for k, g in grads.items():
            p = self.state[k]
            st = self.adam.setdefault(k, dict(t=0, m=np.zeros_like(p), v=np.zeros_like(p)))
            st["t"] += 1
            p *= F32(1 - lr * weight_decay)
            st["m"] = (b1 * st["m"] + (1 - b1) * g).astype(F32)
            st["v"] = (b2 * st["v"] + (1 - b2) * g * g).astype(F32)
            mh = st["m"] / (1 - b1 ** st["t"])
            vh = st["v"] / (1 - b2 ** st["t"])
            p -= (lr * mh / (np.sqrt(vh) + eps)).astype(F32)

    def train_step(self, x, lr=5e-4, weight_decay=0.01):
        out, grads = self.forward_backward(x)
        self.adamw_step(grads, lr, weight_decay)
        return out
