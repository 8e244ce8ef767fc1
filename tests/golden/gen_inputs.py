"""Seeded synthetic inputs shared by the golden-fixture generator and the tests.

Test infrastructure only. Every array here is regenerated bit-identically from a
numpy PCG64 seed, so large inputs never need to be committed: a fixture stores
the seed plus a float64 checksum of each regenerated input, and the test checks
the checksum before trusting the regenerated array.

Distributions follow SURVEY.md §8(d):
  * items: rows ~ N(0, I) then L2-normalised (sentence-T5 embeddings are unit norm,
    reference data/processed.py:76 slices x[:, :768]);
  * MLP weights: U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (torch nn.Linear default bound);
  * sequence lengths: n_items ~ U{2..max_items} (reference data/processed.py:139-146).
"""
import numpy as np


def rng(seed: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(seed))


def checksum(a: np.ndarray) -> float:
    return float(np.asarray(a, dtype=np.float64).sum())


def items(n: int, dim: int, seed: int) -> np.ndarray:
    x = rng(seed).standard_normal((n, dim), dtype=np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    return x.astype(np.float32)


def residual_rows(n: int, dim: int, seed: int, scale: float = 1.0) -> np.ndarray:
    """Rows shaped like encoder outputs / residuals: N(0, scale^2/dim)."""
    g = rng(seed)
    return (g.standard_normal((n, dim), dtype=np.float32) * np.float32(scale / np.sqrt(dim))).astype(np.float32)


def linear_weight(out_dim: int, in_dim: int, seed: int) -> np.ndarray:
    b = 1.0 / np.sqrt(in_dim)
    return rng(seed).uniform(-b, b, size=(out_dim, in_dim)).astype(np.float32)


def mlp_weights(dims, seed: int):
    """Weights of a bias-free Linear chain dims[0]->dims[1]->...; torch layout (out, in)."""
    return [linear_weight(o, i, seed * 1000 + j) for j, (i, o) in enumerate(zip(dims[:-1], dims[1:]))]


def quantize_case(B: int, D: int, K: int, seed: int):
    """x (B,D) residual-like rows and a codebook (K,D) drawn from the same law."""
    x = residual_rows(B, D, seed)
    cb = residual_rows(K, D, seed + 7919)
    return x, cb


def seq_lengths(B: int, max_items: int, seed: int, min_items: int = 2) -> np.ndarray:
    return rng(seed).integers(min_items, max_items + 1, size=B).astype(np.int64)


def named_param(name: str, shape, seed: int) -> np.ndarray:
    """Deterministic value for a named parameter (decoder fixtures), independent of init code.

    1-D weights (RMSNorm, incl. ``ff.0.weight``) ~ 1 + U(-0.1, 0.1); ``bos_emb`` and embedding
    tables (``*emb.weight``, ``wpe``, ``tte``, ``tte_fut``) ~ N(0, 0.3^2); 2-D Linear weights ~
    U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (torch default bound).
    """
    import zlib
    g = rng(seed * 100003 + zlib.crc32(name.encode()))
    shape = tuple(int(s) for s in shape)
    if name == "bos_emb" or name.endswith(("emb.weight", "wpe.weight", "tte.weight", "tte_fut.weight")):
        return (0.3 * g.standard_normal(shape)).astype(np.float32)
    if len(shape) == 1:
        return (1.0 + g.uniform(-0.1, 0.1, size=shape)).astype(np.float32)
    b = 1.0 / np.sqrt(shape[-1])
    return g.uniform(-b, b, size=shape).astype(np.float32)


def gumbel_noise(shape, seed: int, eps: float = 1e-20) -> np.ndarray:
    """Gumbel(0, 1) noise as the reference draws it (distributions/gumbel.py:8-11:
    -log(-log(U + eps) + eps), U ~ U[0, 1)) but from a seeded PCG64 stream, so a fixture can inject
    the same noise into the reference and into this build."""
    u = rng(seed).random(shape, dtype=np.float32)
    e = np.float32(eps)
    return (-np.log(-np.log(u + e) + e)).astype(np.float32)


def topn_multinomial(probs, num_samples, replacement=False, *, generator=None, out=None):
    """Deterministic stand-in for torch.multinomial in generation fixtures (reference
    modules/model.py:178): the num_samples most probable classes, highest first, ties to the lower
    class index. Patched identically into the reference and into this build."""
    import torch
    return torch.sort(probs, dim=-1, descending=True, stable=True).indices[..., :num_samples]


def prefix_verifier(prefix):
    """Deterministic inference_verifier_fn for generation fixtures (stands in for
    SemanticIdTokenizer.exists_prefix): a prefix is valid unless sum(ids) % 7 == 3."""
    return (prefix.sum(-1) % 7) != 3


def batch_permutation(n: int, seed: int, epoch: int) -> np.ndarray:
    """Index order of one epoch of the deterministic sampler used by the training-trace fixture."""
    return rng(seed * 1000 + epoch).permutation(n).astype(np.int64)


def synthetic_item_corpus(n: int, seed: int, eval_fraction: float = 0.05):
    """(train, eval, all) item features of the build's synthetic ItemData (data/processed.py):
    unit-norm 768-d rows from PCG64(seed), train/eval split from PCG64(seed + 1)."""
    x = items(n, 768, seed)
    is_train = rng(seed + 1).random(n) >= eval_fraction
    return x[is_train], x[~is_train], x
