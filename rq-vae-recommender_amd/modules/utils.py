"""Helpers — reference semantics: modules/utils.py:9-78 (decorators, column selection,
repeat-interleave, parse_config, debug metrics)."""
import argparse
import functools

import torch
from torch import Tensor


def reset_kv_cache(fn):
    @functools.wraps(fn)
    def inner(self, *args, **kwargs):
        self.decoder.reset_kv_cache()
        try:
            return fn(self, *args, **kwargs)
        finally:
            self.decoder.reset_kv_cache()
    return inner


def reset_encoder_cache(fn):
    @functools.wraps(fn)
    def inner(self, *args, **kwargs):
        if self.jagged_mode:
            self.transformer.cached_enc_output = None
        out = fn(self, *args, **kwargs)
        if self.jagged_mode:
            self.transformer.cached_enc_output = None
        return out
    return inner


def eval_mode(fn):
    @functools.wraps(fn)
    def inner(self, *args, **kwargs):
        was_training = self.training
        self.eval()
        try:
            return fn(self, *args, **kwargs)
        finally:
            self.train(was_training)
    return inner


def select_columns_per_row(x: Tensor, indices: Tensor) -> Tensor:
    assert x.shape[0] == indices.shape[0]
    assert indices.shape[1] <= x.shape[1]
    return torch.gather(x, 1, indices) if x.dim() == 2 else x[torch.arange(x.shape[0], device=x.device)[:, None], indices]


def maybe_repeat_interleave(x, repeats, dim):
    return x.repeat_interleave(repeats, dim=dim) if isinstance(x, Tensor) else x


def parse_config():
    """`python train_X.py cfg.gin` -> bind the gin file (gin-config when installed, else the
    built-in subset parser ginlite, which covers every construct the reference configs use)."""
    parser = argparse.ArgumentParser()
    parser.add_argument("config_path", type=str, help="Path to gin config file.")
    args = parser.parse_args()
    from modules.ginlite import gin
    gin.parse_config_file(args.config_path)


@torch.no_grad()
def compute_debug_metrics(batch, model_output=None, prefix: str = "") -> dict:
    lengths = batch.seq_mask.sum(axis=1).to(torch.float32)
    qs = torch.tensor([0.25, 0.5, 0.75, 0.9, 1.0], device=lengths.device)
    vals = torch.quantile(lengths, qs).tolist()
    p = prefix + "_"
    out = {f"{p}seq_length_p{q}": v for q, v in zip([0.25, 0.5, 0.75, 0.9, 1], vals)}
    if model_output is not None:
        ld = model_output.loss_d.detach().tolist()
        out.update({f"{p}loss_{d}": ld[d] for d in range(batch.sem_ids_fut.shape[1])})
    return out
