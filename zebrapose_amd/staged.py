"""Stage-by-stage autograd graph for the libzp network, so that torch's own
``DistributedDataParallel(net, device_ids=[gpu])`` -- the unchanged line train_v6.py:259 -- overlaps
its gradient all-reduce with the backward.

The network's forward / backward is one engine pass each (zebrapose_amd.engine).  Wrapped as ONE
autograd node, all 152 gradients reach DDP's AccumulateGrad hooks together, after the whole backward
has been enqueued, so every bucket's all-reduce waits for the end of the backward
(INTEGRATION.md).  Here the forward output is passed through a chain of identity nodes, one per
network stage in forward order (stem, layer1, layer2, layer4, layer5, aspp, up1, up2, head
[, aspp_v3]), each taking that stage's parameters as inputs.  Autograd runs the chain backwards:
the head node's backward starts the engine's reverse pass (Engine.backward_iter) and advances it
until every head parameter has its gradient enqueued, then returns them -- DDP's hooks fire and its
bucket all-reduces are launched (on the process group's stream, after the kernels enqueued so far)
while the next node advances the reverse pass through up2, and so on.  The weight gradients of a
stage run on the engine's side stream; the current stream waits for them at the stage boundary so
the returned tensors are complete in stream order (as autograd assumes).

Used when torch.distributed is initialised and no GradBuckets is attached (GradBuckets has its own
per-gradient overlap), or with ZP_STAGED_BACKWARD=1.  Numerically identical to the single node: the
same kernels in the same order.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

STAGE_ORDER = ["stem", "layer1", "layer2", "layer4", "layer5", "aspp", "up1", "up2", "head", "aspp_v3"]


def stage_of(name):
    """Network stage of a parameter (named relative to DeepLabV3)."""
    if name.startswith("aspp_v3."):
        return "aspp_v3"
    if name.startswith("aspp.upsample_1."):
        return "up1"
    if name.startswith("aspp.upsample_2."):
        return "up2"
    if name.startswith("aspp.conv_1x1_4."):
        return "head"
    if name.startswith("aspp."):
        return "aspp"
    if name.startswith("resnet.layer4."):
        return "layer4"
    if name.startswith("resnet.layer5."):
        return "layer5"
    if name.startswith("resnet.resnet.4.") or name.startswith("resnet.resnet_layer_1."):
        return "layer1"
    if name.startswith("resnet.resnet.5.") or name.startswith("resnet.resnet_layer_2."):
        return "layer2"
    return "stem"


def stage_params(module):
    """[(stage, [params])] in forward order, every parameter exactly once."""
    by = {}
    for name, p in module.named_parameters():
        by.setdefault(stage_of(name), []).append(p)
    return [(s, by[s]) for s in STAGE_ORDER if s in by]


def enabled(module):
    """Staged backward: under torch DDP (a process group of world size > 1) or ZP_STAGED_BACKWARD=1 --
    never with a GradBuckets attached, whose reducer is fed by the single-node path (grads_sink /
    finish_grads); ZP_STAGED_BACKWARD=0 turns it off."""
    if getattr(module, "_grad_buckets", None) is not None:
        return False
    env = os.environ.get("ZP_STAGED_BACKWARD")
    if env is not None:
        return env == "1"
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


class _State:
    def __init__(self, engine, tape, nstage):
        self.engine, self.tape = engine, tape
        self.gen = None
        self.grads = {}
        self.left = nstage

    def advance_until(self, params, head_grads):
        if self.gen is None:
            self.gen = self.engine.backward_iter(self.tape, *head_grads, grads=self.grads)
        need = [p for p in params]
        while self.gen is not None and any(p not in self.grads for p in need):
            try:
                next(self.gen)
            except StopIteration:  # the reverse pass is done: a parameter it never reached gets None
                self.gen = None   # (as the single node's by_ptr.get does)
        self.left -= 1
        if self.left == 0:  # the last stage: finish the pass (joins the side stream)
            for _ in self.gen or ():
                pass
            self.gen = None
            self.tape = None
        else:
            self.engine.side_join_current()
        return [self.grads.get(p) for p in need]


class _StageFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, state, nout, *args):
        outs, params = args[:nout], args[nout:]
        ctx.state, ctx.nout, ctx.params = state, nout, params
        return tuple(o.view_as(o) for o in outs)

    @staticmethod
    def backward(ctx, *gouts):
        # the network's output gradients (mask, [entire,] code) pass through unchanged; the first node
        # to run (the last stage) hands them to the engine's reverse pass
        st = ctx.state
        if st.gen is None:
            g = [None if x is None else x.contiguous() for x in gouts]
            head = (g[0], g[-1]) if ctx.nout == 2 else (g[0], g[2], g[1])  # (dmask, dcode[, dentire])
        else:
            head = None
        grads = st.advance_until(ctx.params, head)
        ctx.state = None
        return (None, None) + tuple(gouts) + tuple(grads)


def staged(module, engine, outs, tape):
    """Chain the forward outputs through one identity node per stage (see the module docstring)."""
    sp = stage_params(module)
    st = _State(engine, tape, len(sp))
    outs = tuple(outs)
    for _, ps in sp:
        outs = _StageFn.apply(st, len(outs), *outs, *ps)
    return outs
