"""Child process of tests/test_dist_trainers_gpu.py: the drop-in trainers (train_rqvae.train, then
train_decoder.train) at world 1 or as one rank of a gloo world on a one-GPU box
(RQVAE_DIST_BACKEND=gloo, RQVAE_SHARE_DEVICE=1: every rank on cuda:0, gloo moving the gradients
through the host). The real data sharding runs — disjoint RQ-VAE item slices, token-balanced decoder
shards with their shard weights, the bucketed exchange after each replayed step graph — on the HIP
kernels. Rank 0 writes the RQ-VAE checkpoint of every iteration and the decoder's final one under argv[1],
and prints both trainers' per-iteration global-batch loss lines; the test compares them with the world-1
run at the same global batch.

    python tools/dist_trainer_probe.py OUT_DIR [TOKENIZER_CKPT]

The decoder runs with dropout 0 everywhere (dropout_p=0 and the model's hard-coded Dropout(0.5),
reference modules/model.py:67, patched to p=0): masks drawn per element of a rank's rows cannot
match a single process's, everything else must."""
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402


def main():
    out = sys.argv[1]
    tok_ckpt = sys.argv[2] if len(sys.argv) > 2 else None
    import train_decoder
    import train_rqvae
    from data.processed import RecDataset
    from modules import model as model_mod
    from modules.quantize import QuantizeForwardMode

    init = model_mod.EncoderDecoderRetrievalModel.__init__

    def init_no_dropout(self, *a, **k):
        init(self, *a, **k)
        self.do.p = 0.0
    model_mod.EncoderDecoderRetrievalModel.__init__ = init_no_dropout

    import numpy as np
    np.random.seed(0)   # the k-means init draws its initial rows from the global numpy RNG (reference init/kmeans.py:36)
    vae = dict(vae_input_dim=768, vae_embed_dim=32, vae_hidden_dims=[512, 256, 128], vae_codebook_size=256,
               vae_n_cat_feats=0, vae_n_layers=3)
    train_rqvae.train(iterations=int(os.environ.get("PROBE_RQ_ITERS", "6")), batch_size=2048, learning_rate=0.0005,
                      dataset=RecDataset.AMAZON, do_eval=False, vae_codebook_mode=QuantizeForwardMode.ROTATION_TRICK,
                      save_dir_root=out + "/vae/", save_model_every=1, log_every=1, seed=2,
                      cuda_graphs=os.environ.get("PROBE_GRAPHS", "1") == "1", **vae)
    rq = dict(train_rqvae.LAST_RUN)
    if os.environ.get("PROBE_RQ_ONLY") == "1":
        import json
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "rqvae": rq}), flush=True)
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
            torch.distributed.destroy_process_group()
        return
    if tok_ckpt is None:
        tok_ckpt = sorted(glob.glob(out + "/vae/checkpoint_*.pt"))[-1] if os.path.isdir(out + "/vae") else None
    if tok_ckpt is None:   # rank > 0 of the world run: the test passes the world-1 tokenizer explicitly
        raise SystemExit("no tokenizer checkpoint")
    train_decoder.train(iterations=8, batch_size=64, learning_rate=0.0003, dataset=RecDataset.AMAZON,
                        pretrained_rqvae_path=tok_ckpt, decoder_embed_dim=64, dropout_p=0.0, attn_heads=4,
                        attn_embed_dim=128, attn_layers=4, save_dir_root=out + "/dec/", save_model_every=10 ** 9,
                        log_every=1, seed=4, **vae)
    dec = dict(train_decoder.LAST_RUN)
    import json
    print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "rqvae": rq, "decoder": dec}), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
