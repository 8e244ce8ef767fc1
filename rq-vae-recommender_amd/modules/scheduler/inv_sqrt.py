"""Inverse-square-root LR with warmup (reference modules/scheduler/inv_sqrt.py:5-15):
lr = base for step <= warmup, else base * sqrt(warmup / step), step = last_epoch + 1."""
from torch.optim.lr_scheduler import LRScheduler


class InverseSquareRootScheduler(LRScheduler):
    def __init__(self, optimizer, warmup_steps: int, last_epoch: int = -1):
        self.warmup_steps = warmup_steps
        super().__init__(optimizer, last_epoch)

    def get_lr(self):
        step = self.last_epoch + 1
        scale = 1.0 if step <= self.warmup_steps else (self.warmup_steps / step) ** 0.5
        return [base * scale for base in self.base_lrs]
