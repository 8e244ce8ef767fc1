"""gin subset (modules/ginlite.py) — the constructs the reference configs use.
CPU only. When the read-only reference tree is present (build container), its own config files
are parsed too; elsewhere those cases skip."""
import importlib
import os

import pytest

REF_CONFIGS = "/root/reference/configs"


def _fresh():
    from modules.ginlite import _GinLite
    g = _GinLite()
    from modules.quantize import QuantizeForwardMode
    from data.processed import RecDataset
    g.constants_from_enum(QuantizeForwardMode, module="modules.quantize")
    g.constants_from_enum(RecDataset, module="data.processed")
    return g


def test_subset_constructs():
    g = _fresh()

    @g.configurable
    def train(iterations=1, hidden=[1], lr=0.1, mode=None, path=None, flag=False, ds=None):
        return dict(iterations=iterations, hidden=hidden, lr=lr, mode=mode, path=path, flag=flag, ds=ds)

    g.parse_config('''import data.processed
import modules.quantize

# full-line comment
train.iterations=400000
train.hidden=[512, 256, 128]
train.lr=0.0005
train.mode=%modules.quantize.QuantizeForwardMode.ROTATION_TRICK
train.path="/mnt/data # not a comment"  # trailing comment
train.flag=True
train.ds=%data.processed.RecDataset.AMAZON''')
    out = train(lr=1.0)
    from modules.quantize import QuantizeForwardMode
    from data.processed import RecDataset
    assert out == dict(iterations=400000, hidden=[512, 256, 128], lr=1.0, mode=QuantizeForwardMode.ROTATION_TRICK,
                       path="/mnt/data # not a comment", flag=True, ds=RecDataset.AMAZON)


def test_unknown_parameter_raises():
    g = _fresh()

    @g.configurable
    def train(a=1):
        return a

    with pytest.raises(ValueError, match="attn_dropout"):
        g.parse_config("train.attn_dropout=0.1")


@pytest.mark.parametrize("name,script", [("rqvae_amazon.gin", "train_rqvae"), ("rqvae_ml32m.gin", "train_rqvae"),
                                         ("rqvae_amazon_custom_path_example.gin", "train_rqvae"),
                                         ("decoder_amazon.gin", "train_decoder"), ("decoder_ml32m.gin", "train_decoder")])
def test_reference_configs(name, script):
    path = os.path.join(REF_CONFIGS, name)
    if not os.path.exists(path):
        pytest.skip("reference tree not present")
    from modules import ginlite
    if not isinstance(ginlite.gin, ginlite._GinLite):
        pytest.skip("real gin-config installed")
    ginlite.gin.clear_config()
    mod = importlib.reload(importlib.import_module(script))
    if name == "decoder_ml32m.gin":   # binds a parameter train() does not have (SURVEY A-8)
        with pytest.raises(ValueError, match="attn_dropout"):
            ginlite.gin.parse_config_file(path)
        return
    ginlite.gin.parse_config_file(path)
    assert callable(mod.train)
    assert ginlite.gin.query_parameter("train.vae_input_dim") == 768
    ginlite.gin.clear_config()
