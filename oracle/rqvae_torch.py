"""RqVae train step in eager PyTorch on the host CPU: bench.py's CPU baseline leg for the RQ-VAE metric
(the reference CPU path as eager PyTorch-CPU on the affinity cores). Test infrastructure
only — never imported by the product package.

Same math as the numpy oracle (oracle/rqvae.py, pinned by the golden fixtures) and as the reference:
  modules/encoder.py:7-36       MLP: bias-free Linear -> SiLU ... -> Linear [-> l2norm, eps 1e-12]
  modules/quantize.py:107-121   L2 distances |x|^2 + |c|^2 - 2 x c^T, argmin (lowest index on ties)
  modules/quantize.py:34-45,133-142  rotation trick (u, q, w detached; gradient through x only), rescale
  modules/loss.py:34-42         QuantizeLoss |sg(x) - e|^2 + beta |x - sg(e)|^2
  modules/rqvae.py:114-165      residual chain over L levels, decoder(sum of level outputs), losses
  torch.optim.AdamW             (train_rqvae.py:96-100)
tests/test_oracle.py checks loss and gradients against the numpy oracle.
"""
import numpy as np
import torch
import torch.nn.functional as F


class RqVaeTorchCPU:
    """Parameters keyed by the reference state-dict names (encoder.mlp.{2j}.weight, decoder.mlp.{2j}.weight,
    layers.{l}.embedding.weight)."""

    def __init__(self, state, n_layers, beta=0.25, lr=5e-4, weight_decay=0.01):
        self.p = {k: torch.tensor(np.asarray(v, np.float32), requires_grad=True) for k, v in state.items()}
        order = lambda pre: sorted([k for k in state if k.startswith(pre)], key=lambda s: int(s.split(".")[2]))  # noqa: E731
        self.enc_keys, self.dec_keys = order("encoder."), order("decoder.")
        self.cb_keys = [f"layers.{l}.embedding.weight" for l in range(n_layers)]
        self.beta = beta
        self.opt = torch.optim.AdamW(list(self.p.values()), lr=lr, weight_decay=weight_decay)

    def _mlp(self, h, keys, normalize):
        for j, k in enumerate(keys):
            h = h @ self.p[k].T
            if j < len(keys) - 1:
                h = F.silu(h)
        if normalize:
            h = h / h.norm(dim=-1, keepdim=True).clamp_min(1e-12)
        return h

    def _level(self, r, cb):
        """One quantize level on residual r: (rotated output, ids, per-row loss)."""
        dist = (r * r).sum(1, keepdim=True) + (cb * cb).sum(1)[None, :] - 2.0 * (r @ cb.T)
        ids = dist.detach().argmin(1)
        e = cb[ids]
        with torch.no_grad():
            u = r / (r.norm(dim=1, keepdim=True) + 1e-8)
            q = e / (e.norm(dim=1, keepdim=True) + 1e-8)
            w = F.normalize(u + q, dim=1, eps=1e-6)
            scale = e.norm(dim=1, keepdim=True) / (r.norm(dim=1, keepdim=True) + 1e-6)
        out = r - 2.0 * (r * w).sum(1, keepdim=True) * w + 2.0 * (r * u).sum(1, keepdim=True) * q
        loss = ((r.detach() - e) ** 2).sum(1) + self.beta * ((r - e.detach()) ** 2).sum(1)
        return out * scale, ids, loss

    def forward(self, x):
        res = self._mlp(x, self.enc_keys, False)
        outs, qloss, ids = [], 0.0, []
        for k in self.cb_keys:
            o, i, lv = self._level(res, self.p[k])
            outs.append(o)
            ids.append(i)
            qloss = qloss + lv
            res = res - o
        x_hat = self._mlp(torch.stack(outs).sum(0), self.dec_keys, True)
        recon = ((x_hat - x) ** 2).sum(-1)
        return (recon + qloss).mean(), torch.stack(ids, 1)

    def forward_backward(self, x):
        """loss, ids and parameter gradients (keyed like the state) of one step, without stepping."""
        for p in self.p.values():
            p.grad = None
        loss, ids = self.forward(torch.as_tensor(x))
        loss.backward()
        return float(loss.detach()), ids.numpy(), {k: p.grad.numpy().copy() for k, p in self.p.items()}

    def train_step(self, x):
        self.opt.zero_grad(set_to_none=True)
        loss, _ = self.forward(x)
        loss.backward()
        self.opt.step()
        return float(loss.detach())
