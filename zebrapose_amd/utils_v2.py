"""Checkpoint files in the reference's layout (zebrapose/utils_v2.py:4-51).

A checkpoint is a ``torch.save`` dict with keys ``model_state_dict`` (``net.*`` keys, or
``module.net.*`` when saved from a DDP-wrapped network), ``optimizer_state_dict``,
``iteration_step``, ``best_score``, ``lr_scheduler_state_dict``; periodic checkpoints are named by
step and rotated (keep ``max_to_keep``), the best one is named ``'{:.4f}'.replace('.', '_') +
'step' + N``.  Packed / bf16 / BN-folded weights are derived at run time and never stored.
"""
from __future__ import annotations

import os

import torch


def save_checkpoint(path, net, iteration_step, best_score, optimizer, lr_scheduler, max_to_keep):
    """utils_v2.py:4-24."""
    os.makedirs(path, exist_ok=True)
    saved = sorted(int(f) for f in os.listdir(path) if os.path.isfile(os.path.join(path, f)) and f.isdigit())
    if len(saved) >= max_to_keep:
        os.remove(os.path.join(path, str(saved[0])))
    out = os.path.join(path, str(iteration_step))
    torch.save({"model_state_dict": net.state_dict(), "optimizer_state_dict": optimizer.state_dict(),
                "iteration_step": iteration_step, "best_score": best_score,
                "lr_scheduler_state_dict": lr_scheduler.state_dict()}, out)
    return out


def get_checkpoint(path):
    """utils_v2.py:26-30: the highest-step checkpoint file in `path`."""
    saved = sorted(int(f) for f in os.listdir(path) if os.path.isfile(os.path.join(path, f)) and f.isdigit())
    return os.path.join(path, str(saved[-1]))


def save_best_checkpoint(best_score_path, net, optimizer, lr_scheduler, best_score, iteration_step):
    """utils_v2.py:32-51 (replaces the previous best file)."""
    os.makedirs(best_score_path, exist_ok=True)
    for f in os.listdir(best_score_path):
        if os.path.isfile(os.path.join(best_score_path, f)):
            os.remove(os.path.join(best_score_path, f))
            break
    name = "{:.4f}".format(best_score).replace(".", "_") + "step" + str(iteration_step)
    out = os.path.join(best_score_path, name)
    torch.save({"model_state_dict": net.state_dict(), "optimizer_state_dict": optimizer.state_dict(),
                "best_score": best_score, "iteration_step": iteration_step,
                "lr_scheduler_state_dict": lr_scheduler.state_dict()}, out)
    print("best check point saved in ", out)
    return out


def load_model_state(net, state_dict, strict=True):
    """Load a reference checkpoint's model_state_dict into a bare (non-DDP) module, accepting the
    ``module.`` prefix DDP adds (test_v5.py:204-207 wraps in DDP instead)."""
    if any(k.startswith("module.") for k in state_dict):
        state_dict = {k[len("module."):] if k.startswith("module.") else k: v for k, v in state_dict.items()}
    return net.load_state_dict(state_dict, strict=strict)


def load_checkpoint_file(path, map_location="cpu"):
    """torch.load with weights_only=True (checkpoints hold tensors, ints and floats only)."""
    return torch.load(path, map_location=map_location, weights_only=True)
