"""hipGraph capture of the inference step (forward + on-device decode).

The reference's evaluation loop runs one crop at a time (test.py:190, 248).  At bs=1 the eager
path is bound by host work, not the GPU: about 50 libzp launches, each with its ctypes argument
struct built in Python (tools/host_overhead.py).  torch.cuda.CUDAGraph is hipGraph on ROCm.
Every libzp launch goes to torch's current stream, so one capture records the whole forward and
decode, and each later call is one graph launch.

Inputs and outputs are static device tensors owned by the graph: a call copies the crops (and
boxes) in, replays, and returns views that stay valid until the next call.  Weight packings and
BN folds are cached by the eager warm-up run and referenced by address, so build a new
GraphedInference after changing the weights (load_state_dict, an optimizer step): a call after
such a change raises instead of replaying kernels that read stale (or freed) packings.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L


def _engines(net):
    out = []
    for m in net.modules():
        e = getattr(m, "_engine", None)
        if e is not None:
            out.append(e)
        out.extend(getattr(m, "_engines_split", {}).values())
    return out


def _deeplabs(net):
    """The modules of ``net`` that carry the fp32 eval engines' range guard (model.BinaryCodeNet.DeepLabV3)."""
    return [m for m in net.modules() if hasattr(m, "h2_active")]


def _state_tensors(net):
    return list(net.parameters()) + list(net.buffers())


def _state_stamp(ts, engines):
    """The version counter of every parameter and buffer (what the engine's packing / fold caches
    are keyed on), plus each engine's BN-fold epoch and cache generation (bumped whenever a packing
    or fold buffer is allocated, replaced or dropped -- this catches re-addressed tensors too).
    ~35 us for the R34 net's 296 tensors; (version, data_ptr) pairs cost 3x that per call."""
    return [t._version for t in ts], [(e._fold_epoch, e._cache_gen) for e in engines]


class GraphedInference:
    def __init__(self, net, batch: int, size: int = 256, decoder=None, bbox_size: int = 128, warmup: int = 2,
                 device=None):
        if net.training:
            raise ValueError("GraphedInference captures the eval forward: call net.eval() first")
        dev = torch.device(device) if device is not None else next(net.parameters()).device
        if dev.type != "cuda":
            raise ValueError("GraphedInference needs the network on a HIP device")
        self.net, self.decoder, self.bbox_size = net, decoder, int(bbox_size)
        self.warmup, self.dev = warmup, dev
        self.x = torch.zeros((batch, 3, size, size), dtype=torch.float32, device=dev)
        self.bb = torch.zeros((batch, 4), dtype=torch.int32, device=dev)
        self.bb[:, 2:] = size  # any valid box for the warm-up; callers pass their own
        self.range_fallbacks = 0
        self._capture()

    def _capture(self):
        net, dev, warmup = self.net, self.dev, self.warmup
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.no_grad(), torch.cuda.stream(side):
            for _ in range(max(1, warmup)):  # fills the weight-pack / BN-fold caches outside the capture
                self._step()
        torch.cuda.current_stream(dev).wait_stream(side)
        # the two-plane split engine's range guard (after the eager warm-up, which checks itself and
        # may already have switched a network to x3): the captured forward clears the device flag at
        # its start (Engine._forward_main), _replay reads it after each replay
        self._guarded = [m for m in _deeplabs(net) if m.h2_active() and m.range_check]
        # each guarded network's engine word (Engine.range_word): the captured forwards clear and
        # raise their own words, read together after each replay
        words = [m.eval_engine().range_word(dev) for m in self._guarded]
        self._flag = None if not words else words[0] if len(words) == 1 else words
        self.graph = torch.cuda.CUDAGraph()
        # thread_local: under torch.distributed the RCCL watchdog thread may query events meanwhile
        with torch.no_grad(), torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            out = self._step()
        # the static outputs keep their identity across a re-capture (the x3 fallback): a new graph's
        # outputs are copied into the first capture's tensors after each replay (_out_copy)
        if getattr(self, "out", None) is None:
            self.out, self._out_copy = out, None
        else:
            self._out_copy = out
        self._tensors, self._engs = _state_tensors(net), _engines(net)
        self._stamp = _state_stamp(self._tensors, self._engs)

    def _flag_hit(self):
        """The guarded networks' range words after a replay: one blocking 4-byte read (the host waits
        for the replay), or one per network group via a max on the device."""
        if self._flag is None:
            return False
        f = self._flag if torch.is_tensor(self._flag) else torch.cat(self._flag).max()
        return bool(int(f.item()))

    def _replay(self):
        self.graph.replay()
        if self._flag_hit():
            # a value beyond fp16's range: the networks switch to the full-range x3 engine, and the
            # step is captured again (the warm-up and capture leave the static inputs alone) and
            # replayed
            for m in self._guarded:
                m.range_fallback()
            self.range_fallbacks += 1
            self._capture()
            self.graph.replay()
        if self._out_copy is not None:
            for d, o in zip(self.out, self._out_copy):
                d.copy_(o)

    def _step(self):
        mask, code = self.net(self.x)
        if self.decoder is None:
            return mask, code
        counts, xy, xyz = self.decoder(mask, code, self.bb, bbox_size=self.bbox_size)
        return mask, code, counts, xy, xyz

    def __call__(self, x, bboxes=None):
        """x f32 [B, 3, size, size] (device or host); bboxes [B, 4] (x, y, w, h) when a decoder is
        attached -> (mask, code) or (mask, code, counts, xy, xyz), the graph's static outputs (the
        same tensors on every call, a range fallback's re-capture included).  With a two-plane
        network under the range guard, each call waits for its replay (the 4-byte flag read)."""
        if tuple(x.shape) != tuple(self.x.shape):
            raise ValueError(f"captured for input {tuple(self.x.shape)}, got {tuple(x.shape)}")
        if _state_stamp(self._tensors, self._engs) != self._stamp:
            raise RuntimeError("GraphedInference: the network's weights or BN buffers changed since capture "
                               "(the graph reads the packings made then); build a new GraphedInference")
        self.x.copy_(x, non_blocking=True)
        if bboxes is not None:
            self.bb.copy_(torch.as_tensor(np.asarray(bboxes), dtype=torch.int32).reshape(self.bb.shape),
                          non_blocking=False)
        self._replay()
        return self.out


class GraphedTrainStep:
    """One training step (TrainStep: forward, loss, backward, FusedAdam) captured in a hipGraph for
    a fixed batch shape; each call copies the batch into the graph's static inputs and replays.

    The training step is GPU-bound (tools/host_overhead.py), but its ~400 launches each leave a
    gap on the queue; a replay issues them back to back.  Requirements: one process (no
    data-parallel buckets: their collectives are not captured) and TrainStep(capturable=True),
    whose FusedAdam keeps the step counts on the device.  The warm-up steps run eagerly and are
    real optimizer steps.  Parameters, gradients and optimizer state keep their storage, so
    state_dict / checkpointing work between calls.
    """

    def __init__(self, ts, x, gt_code, gt_mask, warmup: int = 2):
        if ts.buckets is not None or ts.net is not ts.module:
            raise ValueError("GraphedTrainStep runs single-process steps (no data-parallel wrapper)")
        if not getattr(ts.optimizer, "capturable", False):
            raise ValueError("GraphedTrainStep needs TrainStep(..., capturable=True)")
        self.ts = ts
        self.x, self.gc, self.gm = x.clone(), gt_code.clone(), gt_mask.clone()
        dev = self.x.device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                ts(self.x, self.gc, self.gm)
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            self.out = ts(self.x, self.gc, self.gm)
        # the replayed FusedAdam launches carry lr / betas / eps as captured
        self._hyper = self._hyperparams()

    def _hyperparams(self):
        return [(g["lr"], tuple(g["betas"]), g["eps"]) for g in self.ts.optimizer.param_groups]

    def __call__(self, x, gt_code, gt_mask):
        """-> (loss, loss_b, loss_m), the graph's static output tensors (valid until the next call)."""
        if self._hyperparams() != self._hyper:
            raise RuntimeError("GraphedTrainStep: optimizer lr / betas / eps changed since capture (the graph "
                               "replays the captured values); capture a new GraphedTrainStep after a schedule step")
        self.x.copy_(x, non_blocking=True)
        self.gc.copy_(gt_code, non_blocking=True)
        self.gm.copy_(gt_mask, non_blocking=True)
        self.graph.replay()
        # the replay changed parameters, Adam state and BN running statistics on the device behind
        # the host's version counters: bump them (and the engines' fold epochs) so the engine's
        # eval packings / BN folds are rebuilt by the next eager or eval forward
        net = self.ts.module
        with torch.no_grad():
            for t in list(net.parameters()) + list(net.buffers()):
                torch.autograd.graph.increment_version(t)
        for e in _engines(net):
            e._fold_epoch += 1
        return self.out
