"""Drop-in training entry points (train_rqvae.train / train_decoder.train) run end to end on the GPU
with the reference configs' shapes (few iterations), incl. k-means init, eval, checkpoint + resume; their
default hipGraph step (rqvae_hip.graph.GraphedSteps) against the eager step (cuda_graphs=False)."""
import glob

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_train_rqvae_amazon_dims(tmp_path, device):
    import numpy as np
    import train_rqvae
    from data.processed import RecDataset
    from modules.quantize import QuantizeForwardMode
    np.random.seed(0)
    kw = dict(iterations=30, batch_size=64, learning_rate=0.0005, weight_decay=0.01, dataset=RecDataset.AMAZON,
              vae_input_dim=768, vae_n_cat_feats=0, vae_hidden_dims=[512, 256, 128], vae_embed_dim=32,
              vae_codebook_size=256, vae_codebook_mode=QuantizeForwardMode.ROTATION_TRICK, vae_n_layers=3,
              save_dir_root=str(tmp_path) + "/", save_model_every=15, eval_every=30, do_eval=True, log_every=10)
    model = train_rqvae.train(**kw)
    assert all(layer.kmeans_initted for layer in model.layers)
    ckpts = sorted(glob.glob(str(tmp_path / "checkpoint_*.pt")))
    assert ckpts
    state = torch.load(ckpts[-1], map_location="cpu", weights_only=True)
    assert "layers.0.embedding.weight" in state["model"] and "encoder.mlp.0.weight" in state["model"]
    # resume from the checkpoint (pretrained path disables k-means, loads optimizer state)
    kw.update(iterations=3, pretrained_rqvae_path=ckpts[-1], save_model_every=10 ** 9, do_eval=False)
    train_rqvae.train(**kw)


def test_train_decoder_small(tmp_path, device):
    import numpy as np
    import train_decoder
    import train_rqvae
    from data.processed import RecDataset
    from modules.quantize import QuantizeForwardMode
    vae = dict(vae_input_dim=768, vae_embed_dim=32, vae_hidden_dims=[512, 256, 128], vae_codebook_size=256,
               vae_n_cat_feats=0, vae_n_layers=3)
    np.random.seed(1)
    train_rqvae.train(iterations=10, batch_size=256, dataset=RecDataset.AMAZON, do_eval=False, save_model_every=10,
                      vae_codebook_mode=QuantizeForwardMode.ROTATION_TRICK, save_dir_root=str(tmp_path / "vae") + "/",
                      **vae)
    ckpt = sorted(glob.glob(str(tmp_path / "vae" / "checkpoint_*.pt")))[-1]
    with pytest.raises(ValueError, match="codebook size"):   # untrained tokenizer: fails loudly on the host
        train_decoder.train(iterations=1, batch_size=8, dataset=RecDataset.AMAZON, **vae)
    m = train_decoder.train(iterations=4, batch_size=32, learning_rate=0.0003, dataset=RecDataset.AMAZON,
                            pretrained_rqvae_path=ckpt, decoder_embed_dim=64, dropout_p=0.3, attn_heads=4,
                            attn_embed_dim=128, attn_layers=4, save_dir_root=str(tmp_path) + "/", log_every=2, **vae)
    assert m.sem_id_embedder.emb.weight.grad is not None
    assert glob.glob(str(tmp_path / "checkpoint_*.pt"))


def _trace(capsys):
    import json
    return [json.loads(l) for l in capsys.readouterr().out.splitlines() if l.startswith('{"iter"') and '"loss"' in l]


def test_train_rqvae_graphed_matches_eager(tmp_path, device, capsys):
    """The graphed trainer replays the same kernels as the eager one: identical per-step losses."""
    import numpy as np
    import train_rqvae
    from data.processed import RecDataset
    from modules.quantize import QuantizeForwardMode
    kw = dict(iterations=12, batch_size=64, learning_rate=0.0005, dataset=RecDataset.AMAZON, vae_input_dim=768,
              vae_n_cat_feats=0, vae_hidden_dims=[512, 256, 128], vae_embed_dim=32, vae_codebook_size=256,
              vae_codebook_mode=QuantizeForwardMode.ROTATION_TRICK, vae_n_layers=3, do_eval=False,
              save_dir_root=str(tmp_path) + "/", save_model_every=10 ** 9, log_every=1, seed=3)
    traces = {}
    for graphs in (False, True):
        np.random.seed(0)
        capsys.readouterr()
        train_rqvae.train(cuda_graphs=graphs, **kw)
        traces[graphs] = _trace(capsys)
        run = dict(train_rqvae.LAST_RUN)
        assert run["step_mode"] == ("hipgraph" if graphs else "eager")
        if graphs:
            assert run["graphs"] == 1 and run["eager_steps"] == 1, run
    assert len(traces[True]) == len(traces[False]) == 13
    for a, b in zip(traces[False], traces[True]):
        for k in ("loss", "rl", "vl", "p_unique_ids"):
            assert a[k] == pytest.approx(b[k], rel=1e-6, abs=1e-9), (k, a, b)


def test_train_decoder_graphed(tmp_path, device, capsys, monkeypatch):
    """The graphed decoder trainer: one graph per context row bucket, gradients in the flat buckets, and —
    with dropout 0 everywhere (dropout_p=0 and the model's hard-coded Dropout(0.5), reference
    modules/model.py:67, patched to p=0) — every replayed step's loss equal to the eager trainer's."""
    import numpy as np
    import train_decoder
    import train_rqvae
    from data.processed import RecDataset
    from modules import model as model_mod
    from modules.quantize import QuantizeForwardMode
    init = model_mod.EncoderDecoderRetrievalModel.__init__

    def init_no_dropout(self, *a, **k):
        init(self, *a, **k)
        self.do.p = 0.0
    monkeypatch.setattr(model_mod.EncoderDecoderRetrievalModel, "__init__", init_no_dropout)
    vae = dict(vae_input_dim=768, vae_embed_dim=32, vae_hidden_dims=[512, 256, 128], vae_codebook_size=256,
               vae_n_cat_feats=0, vae_n_layers=3)
    np.random.seed(1)
    train_rqvae.train(iterations=10, batch_size=256, dataset=RecDataset.AMAZON, do_eval=False, save_model_every=10,
                      vae_codebook_mode=QuantizeForwardMode.ROTATION_TRICK, save_dir_root=str(tmp_path / "vae") + "/",
                      **vae)
    ckpt = sorted(glob.glob(str(tmp_path / "vae" / "checkpoint_*.pt")))[-1]
    kw = dict(iterations=12, batch_size=32, learning_rate=0.0003, dataset=RecDataset.AMAZON, pretrained_rqvae_path=ckpt,
              decoder_embed_dim=64, dropout_p=0.0, attn_heads=4, attn_embed_dim=128, attn_layers=4,
              save_dir_root=str(tmp_path) + "/", save_model_every=10 ** 9, log_every=1, **vae)
    traces = {}
    for graphs in (False, True):
        capsys.readouterr()
        train_decoder.train(cuda_graphs=graphs, **kw)
        traces[graphs] = _trace(capsys)
        run = dict(train_decoder.LAST_RUN)
        assert run["step_mode"] == ("hipgraph" if graphs else "eager")
        if graphs:
            assert run["graphs"] >= 1 and run["eager_steps"] == 1, run
            if "host_ms_per_iter" in run:   # a steady span (no capture in the last 3 iterations)
                assert set(run["host_ms_per_iter"]) >= {"feed_wait", "tokenize", "step", "exchange", "optimizer"}
    assert len(traces[True]) == len(traces[False]) == 12
    for a, b in zip(traces[False], traces[True]):
        assert np.isfinite(b["loss"])
        assert b["loss"] == pytest.approx(a["loss"], rel=1e-5), (a, b)


def test_train_rqvae_amp_flag(tmp_path, device, capsys):
    """amp=True (the reference's accelerate fp16 autocast switch, train_rqvae.py:36,62,147) is accepted with a
    warning: every op of the step is an fp32 HIP kernel autocast leaves alone, so the per-step losses are the
    amp=False ones."""
    import numpy as np
    import train_rqvae
    from data.processed import RecDataset
    from modules.quantize import QuantizeForwardMode
    kw = dict(iterations=6, batch_size=64, learning_rate=0.0005, dataset=RecDataset.AMAZON, vae_input_dim=768,
              vae_n_cat_feats=0, vae_hidden_dims=[512, 256, 128], vae_embed_dim=32, vae_codebook_size=256,
              vae_codebook_mode=QuantizeForwardMode.ROTATION_TRICK, vae_n_layers=3, do_eval=False,
              save_dir_root=str(tmp_path) + "/", save_model_every=10 ** 9, log_every=1, seed=3)
    traces = {}
    for amp in (False, True):
        np.random.seed(0)
        capsys.readouterr()
        if amp:
            with pytest.warns(UserWarning, match="amp=True"):
                train_rqvae.train(amp=True, **kw)
        else:
            train_rqvae.train(**kw)
        traces[amp] = _trace(capsys)
    assert len(traces[True]) == len(traces[False]) > 0
    for a, b in zip(traces[False], traces[True]):
        for k in ("loss", "rl", "vl"):
            assert a[k] == pytest.approx(b[k], rel=1e-6, abs=1e-9), (k, a, b)
