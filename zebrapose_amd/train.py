"""The ZebraPose training step on MI355X (train_v6.py:319-338 semantics) and its data-parallel
wrapper (train_v6.py:47-51, 82-91, 252-264).

Per step: forward (train-mode BN) -> visible-mask threshold on device (train_v6.py:325-326 does
it on the host in f64) -> loss_b = BinaryCodeLoss('BCE', True, 2, hist=True) (f64) and
loss_m = MaskLoss -> loss = 3 loss_b + loss_m -> backward -> Adam.  Under torch.distributed
(one process per GPU, backend 'nccl' = RCCL over xGMI) the network is wrapped in DDP exactly as
the reference does (parallel.GradBuckets: DDP's bucketed mean, its all-reduces started while the
backward is still running; ZP_TORCH_DDP=1 selects torch's DDP wrapper), so the gradient
all-reduce (mean) runs over RCCL; lr is multiplied and the
iteration budget divided by the world size (train_v6.py:82-91); BN statistics stay per rank and
rank 0's BN buffers are broadcast at every forward (DDP default broadcast_buffers=True).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .model.BinaryCodeNet import BinaryCodeLoss, MaskLoss
from .optim import FusedAdam
from .parallel import attach_grad_buckets


def scale_for_world(learning_rate, total_iteration, world_size):
    """train_v6.py:82-91."""
    return learning_rate * world_size, total_iteration // world_size


class TrainStep:
    def __init__(self, net, learning_rate=2e-4, binary_loss_weight=3.0, ddp=None, device=None, bucket_mb=25.0,
                 capturable=False):
        self.module = net
        self.net = net
        if ddp is None:
            ddp = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self.buckets = None
        if ddp:
            if any(hasattr(m, "_engine") for m in net.modules()) and os.environ.get("ZP_TORCH_DDP", "0") != "1":
                # DDP semantics with the all-reduce overlapped with the libzp backward
                self.buckets = attach_grad_buckets(net, bucket_mb=bucket_mb)
            else:
                dev = device if device is not None else torch.cuda.current_device()
                self.net = torch.nn.parallel.DistributedDataParallel(net, device_ids=[dev])
        self.binary_loss_weight = binary_loss_weight
        self.code_loss = BinaryCodeLoss("BCE", True, 2, use_histgramm_weighted_binary_loss=True)
        self.mask_loss = MaskLoss()
        # capturable: device-side Adam step counts, for zebrapose_amd.graphs.GraphedTrainStep
        self.optimizer = FusedAdam(self.net.parameters(), lr=learning_rate, capturable=capturable)
        self.events = None  # optional list: (label, event) at step start / before backward / after backward / end

    def _mark(self, label):
        if self.events is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self.events.append((label, ev))

    def __call__(self, x, gt_code, gt_mask, gt_entire_mask=None):
        """x f32 [B,3,H,W]; gt_code u8/f64 [B,L,H/2,W/2]; gt_mask f32 [B,H/2,W/2] -> (loss, loss_b, loss_m).
        With the 3-head BinaryCodeNet_Deeplab_v3 (train_v5.py:321-332) gt_entire_mask f32 [B,H/2,W/2] is
        required and loss = w * loss_b + loss_mask + loss_entire_mask."""
        self._mark("start")
        self.optimizer.zero_grad(set_to_none=True)
        if self.buckets is not None:
            self.buckets.sync_buffers()
        out = self.net(x)
        if len(out) == 3:
            if gt_entire_mask is None:
                raise ValueError("the 3-head network needs gt_entire_mask")
            mask, entire, code = out
        else:
            mask, code = out
        loss_b = self.code_loss.forward_from_logits(code, mask, gt_code)
        loss_m = self.mask_loss(mask, gt_mask)
        loss = self.binary_loss_weight * loss_b + loss_m
        if len(out) == 3:
            loss = loss + self.mask_loss(entire, gt_entire_mask)
        self._mark("backward")
        loss.backward()
        self._mark("optimizer")
        self.optimizer.step()
        self._mark("end")
        return loss.detach(), loss_b.detach(), loss_m.detach()
