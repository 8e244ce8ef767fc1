"""Find host-device synchronisations in the drop-in decoder trainer's loop: train_rqvae.train (a small
tokenizer checkpoint), then train_decoder.train at the bench's Amazon config with
torch.cuda.set_sync_debug_mode("warn"); prints each distinct synchronising call site with the count."""
import collections
import glob
import os
import sys
import tempfile
import traceback
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import bench
    import train_decoder
    import train_rqvae
    from data.processed import RecDataset
    from modules.quantize import QuantizeForwardMode
    CFG, DEC = bench.CFG, bench.DEC
    vae = dict(vae_input_dim=CFG["input_dim"], vae_embed_dim=CFG["D"], vae_hidden_dims=CFG["hidden"],
               vae_codebook_size=CFG["K"], vae_n_cat_feats=0, vae_n_layers=CFG["L"])
    np.random.seed(0)
    tmp = tempfile.mkdtemp()
    train_rqvae.train(iterations=10, batch_size=4096, dataset=RecDataset.ML_32M, do_eval=False, save_dir_root=tmp + "/vae/",
                      log_every=10 ** 9, vae_codebook_mode=QuantizeForwardMode.ROTATION_TRICK, **vae)
    ckpt = sorted(glob.glob(tmp + "/vae/checkpoint_*.pt"))[-1]
    sites = collections.Counter()
    orig = warnings.showwarning

    def show(message, category, filename, lineno, file=None, line=None):
        if "synchroniz" in str(message).lower():
            st = [f for f in traceback.extract_stack()[:-1] if "site-packages" not in f.filename]
            sites["; ".join(f"{os.path.basename(f.filename)}:{f.lineno} {f.name}" for f in st[-4:])] += 1
        else:
            orig(message, category, filename, lineno, file, line)
    warnings.showwarning = show
    warnings.simplefilter("always")
    torch.cuda.set_sync_debug_mode("warn")
    train_decoder.train(iterations=30, batch_size=DEC["B"], learning_rate=DEC["lr"], weight_decay=DEC["wd"],
                        dataset=RecDataset.AMAZON, pretrained_rqvae_path=ckpt, decoder_embed_dim=DEC["E"],
                        dropout_p=DEC["dropout"], attn_heads=DEC["H"], attn_embed_dim=DEC["A"],
                        attn_layers=DEC["layers"], save_dir_root=tmp + "/dec/", log_every=10 ** 9,
                        save_model_every=10 ** 9, **vae)
    torch.cuda.set_sync_debug_mode(0)
    for site, n in sites.most_common(40):
        print(f"{n:6d}  {site}")
    print(dict(train_decoder.LAST_RUN))


if __name__ == "__main__":
    main()
