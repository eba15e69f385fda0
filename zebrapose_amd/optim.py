"""Adam on the device through ``zp_adam`` (torch.optim.Adam semantics: no weight decay, no
amsgrad; the update order of torch's implementation -- lerp of the first moment, bias-corrected
step size, sqrt(v)/sqrt(bc2) + eps).  Reference use: train_v6.py:268-269 (Adam(lr)), :338 (step).
State dict layout matches torch.optim.Adam ('step', 'exp_avg', 'exp_avg_sq' per parameter) so
checkpoints stay interchangeable (utils_v2.py:15-23)."""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L


class FusedAdam(torch.optim.Optimizer):
    """capturable=True (torch.optim.Adam's flag of the same name): the per-parameter 'step' counts
    live on the device and the kernels read the count there (zp_adam_multi_dev), so a step captured
    in a hipGraph replays with the current count (zebrapose_amd.graphs.GraphedTrainStep)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, capturable=False):
        if weight_decay != 0.0:
            raise NotImplementedError("weight decay is not used by the ZebraPose trainers")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=0.0))
        self.capturable = capturable

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._steps = {}

    @torch.no_grad()
    def step(self, closure=None):
        """All parameters of a group that share a step count go through one zp_adam_multi call
        (ceil(n / 40) launches instead of one launch per parameter).  The per-parameter 'step'
        tensors of torch's state layout are advanced with one foreach op; a host-side int mirror
        (self._steps) avoids a .item() per parameter."""
        loss = closure() if closure is not None else None
        st = L.stream_ptr()
        steps = self.__dict__.setdefault("_steps", {})
        for group in self.param_groups:
            b1, b2 = group["betas"]
            live, step_t = [], []
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.dtype != torch.float32 or not p.is_contiguous() or not p.grad.is_contiguous():
                    raise ValueError("FusedAdam expects contiguous float32 parameters and gradients")
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = torch.zeros((), dtype=torch.float32, device=p.device) if self.capturable else \
                        torch.tensor(0.0)
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    steps[p] = 0
                elif p not in steps:
                    steps[p] = int(state["step"].item())
                    if self.capturable and state["step"].device != p.device:
                        state["step"] = state["step"].to(p.device)
                steps[p] += 1
                live.append(p)
                step_t.append(state["step"])
            if not live:
                continue
            torch._foreach_add_(step_t, 1.0)
            by_step = {}
            for p in live:
                by_step.setdefault(steps[p], []).append(p)
            for step, ps in by_step.items():
                n = len(ps)
                arr = C.c_void_p * n
                args = (n, arr(*[p.data_ptr() for p in ps]), arr(*[p.grad.data_ptr() for p in ps]),
                        arr(*[self.state[p]["exp_avg"].data_ptr() for p in ps]),
                        arr(*[self.state[p]["exp_avg_sq"].data_ptr() for p in ps]),
                        (C.c_longlong * n)(*[p.numel() for p in ps]), float(group["lr"]), float(b1), float(b2),
                        float(group["eps"]))
                if self.capturable:  # every tensor of this launch group is at the same (device) count
                    L.call("zp_adam_multi_dev", *args, self.state[ps[0]]["step"].data_ptr(), st)
                else:
                    L.call("zp_adam_multi", *args, step, st)
                # the kernel wrote p in place behind autograd's back: bump its version counter so
                # version-keyed caches (packed eval weights in the engine) see the update
                for p in ps:
                    torch.autograd.graph.increment_version(p)
        return loss
