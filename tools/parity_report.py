#!/usr/bin/env python3
"""Measured deviation from the reference's golden fixtures at 'highest' and 'high' matmul precision
(the numbers behind the tolerances in tests/test_reference_fixtures_gpu.py). One JSON line per case."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "rq-vae-recommender_amd"), ROOT, os.path.join(ROOT, "tests", "golden"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gen_inputs as gi  # noqa: E402


def load(name):
    return dict(np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False))


def rel_grad_err(got, ref):
    ref = np.asarray(ref, np.float64)
    return float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-30))


def decoder(tag, prec, dev):
    from test_reference_fixtures_gpu import _decoder_model, _tokenized
    z = load(f"decoder_{tag}")
    m = _decoder_model(z, dev)
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    m.train()
    torch.set_float32_matmul_precision(prec)
    out = m(_tokenized(z, dev))
    out.loss.backward()
    worst_g, worst_n = 0.0, 0.0
    for name, p in m.named_parameters():
        k = "grad__" + name
        if k in z:
            worst_g = max(worst_g, rel_grad_err(p.grad.double().cpu().numpy(), z[k]))
        elif k + "__norm" in z:
            worst_n = max(worst_n, abs(p.grad.double().norm().item() / float(z[k + "__norm"]) - 1))
            worst_g = max(worst_g, rel_grad_err(p.grad[0].double().cpu().numpy(), z[k + "__row0"]))
    lg = out.logits.detach().cpu().numpy()
    return dict(case=f"decoder_{tag}", precision=prec, ctx_max=int(z["seq_mask"].sum(1).max()) + 1,
                loss_rel=abs(float(out.loss) / float(z["loss"]) - 1),
                logits_err_over_max=float(np.abs(lg - z["logits"]).max() / np.abs(z["logits"]).max()),
                grad_err_over_max=worst_g, grad_norm_rel=worst_n)


def rqvae(prec, dev):
    from data.schemas import SeqBatch
    from test_quantize_gpu import _rqvae
    z = load("rqvae_ml32m")
    m = _rqvae(z, dev)
    x = torch.from_numpy(gi.items(int(z["B"]), int(z["inp"]), int(z["seed"]) + 200)).to(dev)
    torch.set_float32_matmul_precision(prec)
    m.eval()
    with torch.no_grad():
        ids = m.get_semantic_ids(x).sem_ids.cpu().numpy()
    m.train()
    out = m(SeqBatch(None, None, None, x, None, None), gumbel_t=0.2)
    out.loss.backward()
    safe = (z["eval_margin"] > 1e-4).all(1)
    gn = max(abs(p.grad.double().norm().item() / (float(np.linalg.norm(z["grad__" + n.replace(".", "_")]))
                                                  if "grad__" + n.replace(".", "_") in z
                                                  else float(z["grad__" + n.replace(".", "_") + "__norm"])) - 1)
             for n, p in m.named_parameters())
    return dict(case="rqvae_ml32m", precision=prec, rows=int(len(ids)), margin_safe_rows=int(safe.sum()),
                id_rows_differing=int((ids != z["eval_sem_ids"]).any(1).sum()),
                id_rows_differing_on_safe=int((ids[safe] != z["eval_sem_ids"][safe]).any(1).sum()),
                min_margin=float(z["eval_margin"].min()),
                loss_rel=abs(float(out.loss) / float(z["loss"]) - 1), grad_norm_rel=gn)


def main():
    dev = torch.device("cuda", 0)
    for prec in ("highest", "high"):
        print(json.dumps(rqvae(prec, dev)), flush=True)
        for tag in ("small", "dm", "c5"):
            print(json.dumps(decoder(tag, prec, dev)), flush=True)


if __name__ == "__main__":
    main()
