"""Checkpoint / state-dict interchange with the reference, CPU only.

The manifests in checkpoint.npz were written by make_golden.py from the reference's own modules
(RqVae at rqvae_amazon.gin dims, EncoderDecoderRetrievalModel at decoder_amazon.gin dims): this
build's modules must expose exactly the same state-dict keys and shapes, so checkpoints move both
ways with strict loading. ckpt_rqvae_small.pt is a checkpoint in the reference's train_rqvae.py:209-221
layout written by the reference (tensors and plain containers: loads with weights_only=True).
"""
import os

import numpy as np
import pytest
import torch

import gen_inputs as gi

GOLDEN = os.path.dirname(gi.__file__)


def _manifest(z, prefix):
    return {k[len(prefix):]: tuple(int(s) for s in z[k]) for k in z if k.startswith(prefix)}


def test_rqvae_state_dict_matches_reference(golden):
    from modules.quantize import QuantizeForwardMode
    from modules.rqvae import RqVae
    ref = _manifest(golden("checkpoint"), "rqvae_keys__")
    m = RqVae(input_dim=768, embed_dim=32, hidden_dims=[512, 256, 128], codebook_size=256, codebook_kmeans_init=False,
              n_layers=3, n_cat_features=0, codebook_mode=QuantizeForwardMode.ROTATION_TRICK)
    ours = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert ours == ref


def test_decoder_state_dict_matches_reference(golden):
    from modules.model import EncoderDecoderRetrievalModel
    z = golden("checkpoint")
    ref = _manifest(z, "decoder_keys__")
    m = EncoderDecoderRetrievalModel(embedding_dim=128, attn_dim=512, dropout=0.3, num_heads=8, n_layers=8,
                                     num_embeddings=256, sem_id_dim=4, inference_verifier_fn=None, max_pos=80)
    ours = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert ours == ref
    assert sum(p.numel() for p in m.parameters()) == int(z["decoder_n_params"])


def test_reference_checkpoint_loads_weights_only():
    from modules.quantize import QuantizeForwardMode
    from modules.rqvae import RqVae
    from rqvae_hip import optim as hip_optim
    ck = torch.load(os.path.join(GOLDEN, "ckpt_rqvae_small.pt"), map_location="cpu", weights_only=True)
    assert set(ck) == {"iter", "model", "optimizer"}
    m = RqVae(input_dim=96, embed_dim=16, hidden_dims=[64, 32], codebook_size=32, codebook_kmeans_init=False,
              codebook_mode=QuantizeForwardMode.ROTATION_TRICK, n_layers=3, n_cat_features=0)
    m.load_state_dict(ck["model"], strict=True)
    opt = hip_optim.AdamW(m.parameters(), lr=5e-4, weight_decay=0.01)
    opt.load_state_dict(ck["optimizer"])
    steps = {float(st["step"]) for st in opt.state.values()}
    assert steps == {float(ck["iter"]) + 1}
    assert all(st["step"].device.type == "cpu" and st["step"].dtype == torch.float32 for st in opt.state.values())
    # a torch AdamW state asking for amsgrad / maximize is refused rather than silently stepped as plain AdamW
    bad = {"state": ck["optimizer"]["state"],
           "param_groups": [dict(g, amsgrad=True) for g in ck["optimizer"]["param_groups"]]}
    from rqvae_hip._lib import RqHipError
    with pytest.raises(RqHipError):
        hip_optim.AdamW(m.parameters(), lr=5e-4).load_state_dict(bad)
