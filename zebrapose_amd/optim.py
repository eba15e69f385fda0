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
        self._stale = False
        super().load_state_dict(state_dict)
        self._steps = {}
        self._plans = {}

    def _sync_steps(self):
        """Write the host mirror into the (CPU) 'step' tensors the fast path leaves behind: a
        foreach add over ~150 CPU scalars costs ~0.9 ms of host time per training step."""
        if self.__dict__.get("_stale"):
            for p, n in self._steps.items():
                self.state[p]["step"].fill_(float(n))
            self._stale = False

    def state_dict(self):
        self._sync_steps()
        return super().state_dict()

    def add_param_group(self, param_group):
        super().add_param_group(param_group)
        self._plans = {}

    def zero_grad(self, set_to_none=True):
        """set_to_none drops the gradients with a plain loop (torch's version walks the same list
        under a profiler scope and per-tensor checks: ~0.5 ms of host time per training step)."""
        if not set_to_none:
            return super().zero_grad(set_to_none=False)
        for group in self.param_groups:
            for p in group["params"]:
                p.grad = None

    def _plan(self, gi, group, steps):
        """Launch plan of a group whose parameters all have gradients and state at one step count:
        the ctypes arrays of parameter / moment pointers and sizes (stable across steps; only the
        gradient pointers are rebuilt per step).  None when the group needs the general path."""
        plans = self.__dict__.setdefault("_plans", {})
        ps = group["params"]
        plan = plans.get(gi)
        # (valid while every step of the group went through the fast path: the general path drops it)
        if plan is not None and plan[0] == len(ps) and all(a is b for a, b in zip(plan[1], ps)):
            return plan
        if not ps or any(len(self.state[p]) == 0 or p not in steps for p in ps):
            return None
        if len({steps[p] for p in ps}) != 1:
            return None
        if any(p.dtype != torch.float32 or not p.is_contiguous() for p in ps):
            return None
        n = len(ps)
        arr = C.c_void_p * n
        plan = (n, tuple(ps), arr(*[p.data_ptr() for p in ps]),
                arr(*[self.state[p]["exp_avg"].data_ptr() for p in ps]),
                arr(*[self.state[p]["exp_avg_sq"].data_ptr() for p in ps]),
                (C.c_longlong * n)(*[p.numel() for p in ps]), [self.state[p]["step"] for p in ps], arr)
        plans[gi] = plan
        return plan

    @torch.no_grad()
    def step(self, closure=None):
        """All parameters of a group that share a step count go through one zp_adam_multi call
        (ceil(n / 40) launches instead of one launch per parameter).  The per-parameter 'step'
        tensors of torch's state layout are advanced with one foreach op; a host-side int mirror
        (self._steps) avoids a .item() per parameter.  Steady state (every parameter of the group
        has a gradient, all at one count) reuses a cached launch plan (_plan)."""
        loss = closure() if closure is not None else None
        st = L.stream_ptr()
        steps = self.__dict__.setdefault("_steps", {})
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            hp = (float(group["lr"]), float(b1), float(b2), float(group["eps"]))
            plan = self._plan(gi, group, steps)
            if plan is not None:
                n, ps, pp, m1, m2, nel, step_t, arr = plan
                grads = [p.grad for p in ps]
                if all(g is not None and g.is_contiguous() for g in grads):
                    step = steps[ps[0]] + 1
                    for p in ps:
                        steps[p] = step
                    if self.capturable:
                        torch._foreach_add_(step_t, 1.0)
                    else:  # host-side step tensors are written from the mirror when read (_sync_steps)
                        self._stale = True
                    args = (n, pp, arr(*[g.data_ptr() for g in grads]), m1, m2, nel) + hp
                    if self.capturable:
                        L.call("zp_adam_multi_dev", *args, step_t[0].data_ptr(), st)
                    else:
                        L.call("zp_adam_multi", *args, step, st)
                    torch.autograd.graph.increment_version(list(ps))
                    continue
            self._sync_steps()
            # the general path may advance only part of the group (a parameter without a gradient):
            # the cached plan assumed one shared step count, so it is rebuilt once they agree again
            self.__dict__.setdefault("_plans", {}).pop(gi, None)
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
                        (C.c_longlong * n)(*[p.numel() for p in ps])) + hp
                if self.capturable:  # every tensor of this launch group is at the same (device) count
                    L.call("zp_adam_multi_dev", *args, self.state[ps[0]]["step"].data_ptr(), st)
                else:
                    L.call("zp_adam_multi", *args, step, st)
                # the kernel wrote p in place behind autograd's back: bump its version counter so
                # version-keyed caches (packed eval weights in the engine) see the update
                torch.autograd.graph.increment_version(ps)
        return loss
