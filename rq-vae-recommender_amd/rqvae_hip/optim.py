"""AdamW whose step is one HIP launch per parameter group (rq_adamw_step, csrc/optim.hip).

Same constructor, hyper-parameters, update rule and state keys (`step`, `exp_avg`, `exp_avg_sq`) as
torch.optim.AdamW, which the reference's loops step (train_rqvae.py:96-100,168-172;
train_decoder.py:151-160,203), so `state_dict()` round-trips with torch's optimizer. torch's fused
AdamW splits each tensor into 64 Ki-element blocks, which leaves most of the GPU idle for the
RQ-VAE's 1.18 M parameters; here every 4096-element chunk of every tensor is its own workgroup, and the
segment table rides in the kernel arguments (no upload, no sync when grads are re-allocated).

Supported: fp32 CUDA parameters with dense contiguous grads, amsgrad=False, maximize=False.
No CPU fallback (RqHipError, like every other op of this package).
"""
import ctypes
import math

import torch

from ._lib import RqHipError, call, load, require_gpu, stream_handle


def _check(p):
    require_gpu(p, p.grad, what="AdamW")
    if p.dtype != torch.float32 or p.grad.dtype != torch.float32:
        raise RqHipError("rqvae_hip.optim.AdamW: fp32 parameters and grads only")
    if p.grad.is_sparse or not (p.is_contiguous() and p.grad.is_contiguous()):
        raise RqHipError("rqvae_hip.optim.AdamW: dense contiguous parameters and grads only")


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False,
                 maximize=False, **unused):
        if amsgrad or maximize:
            raise RqHipError("rqvae_hip.optim.AdamW: amsgrad / maximize are not supported")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= weight_decay:
            raise ValueError(f"invalid AdamW hyper-parameters lr={lr} eps={eps} weight_decay={weight_decay}")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"invalid betas {betas}")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                                      amsgrad=False, maximize=False))
        self._tables = {}
        self._checked = {}
        load()   # fail loudly here if the HIP library is missing

    @staticmethod
    def _check_group(group):
        if group.get("amsgrad", False) or group.get("maximize", False):
            raise RqHipError("rqvae_hip.optim.AdamW: amsgrad / maximize are not supported")

    def load_state_dict(self, state_dict):
        """torch.optim.AdamW state (e.g. a reference checkpoint's "optimizer", train_rqvae.py:110-112):
        groups asking for amsgrad / maximize are rejected, and every `step` counter is kept as a CPU
        float32 tensor (a checkpoint loaded with map_location=<gpu> would otherwise make each step read
        it back with a blocking device sync)."""
        for g in state_dict.get("param_groups", []):
            self._check_group(g)
        super().load_state_dict(state_dict)
        for st in self.state.values():
            if "step" in st:
                st["step"] = torch.tensor(float(st["step"]), dtype=torch.float32)
        self._tables, self._checked = {}, {}

    def _table(self, slot, live):
        """Host (ctypes) segment table {p, g, exp_avg, exp_avg_sq, n} per tensor, rebuilt only when a
        pointer changes (grads re-allocated after zero_grad(set_to_none=True)); never uploaded."""
        key = tuple((p.data_ptr(), p.grad.data_ptr(), s["exp_avg"].data_ptr(), s["exp_avg_sq"].data_ptr(), p.numel())
                    for p, s in live)
        hit = self._tables.get(slot)
        if hit is not None and hit[0] == key:
            return hit[1]
        table = (ctypes.c_int64 * (5 * len(key)))(*[v for row in key for v in row])
        self._tables[slot] = (key, table)
        return table

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            self._check_group(group)
            live = [p for p in group["params"] if p.grad is not None and p.numel() > 0]
            if not live:
                continue
            # validate BEFORE any state changes, whenever a tensor changed since the last check
            key = tuple((p.data_ptr(), p.grad.data_ptr()) for p in live)
            if self._checked.get(gi) != key:
                for p in live:
                    _check(p)
                self._checked[gi] = key
            states = []
            for p in live:
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                states.append(st)
            steps = [st["step"] for st in states]
            torch._foreach_add_(steps, 1)   # one host op for the group's step counters (as torch's AdamW)
            by_step = {}   # torch keeps a step count per parameter: one launch per distinct count
            for p, st, t in zip(live, states, steps):
                by_step.setdefault(t.item(), []).append((p, st))
            b1, b2 = group["betas"]
            for k, (step, members) in enumerate(sorted(by_step.items())):
                bc1 = 1.0 - b1 ** step
                bc2s = math.sqrt(1.0 - b2 ** step)
                table = self._table((gi, k), members)
                call("rq_adamw_step", table, len(members), group["lr"], b1, b2, group["eps"],
                     group["weight_decay"], bc1, bc2s, stream_handle(members[0][0].device))
        return loss
