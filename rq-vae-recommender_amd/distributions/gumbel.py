"""Gumbel-softmax sampling — reference semantics: distributions/gumbel.py:8-41.
Used only by QuantizeForwardMode.GUMBEL_SOFTMAX (no config selects it)."""
import math

import torch
import torch.nn.functional as F

__all__ = ["sample_gumbel", "gumbel_softmax_sample", "TemperatureScheduler"]


def sample_gumbel(shape, device, eps=1e-20):
    u = torch.rand(shape, device=device)
    return -torch.log(eps - torch.log(u + eps))


def gumbel_softmax_sample(logits, temperature, device):
    noisy = logits + sample_gumbel(logits.shape, device)
    return F.softmax(noisy / temperature, dim=-1)


class TemperatureScheduler:
    """t <- max(t * exp(-anneal_rate * iter), min_t) at the last iter of every step_size window."""

    def __init__(self, t0: float, min_t: float, anneal_rate: float, step_size: int) -> None:
        self.t0, self.min_t, self.anneal_rate, self.step_size = t0, min_t, anneal_rate, step_size
        self.t = t0

    def update_t(self, iter):
        if (iter + 1) % self.step_size == 0:
            self.t = max(self.t * math.exp(-self.anneal_rate * iter), self.min_t)

    def get_t(self, iter):
        self.update_t(iter)
        return self.t
