"""Network executor: runs BinaryCodeNet_Deeplab's forward / backward as a sequence of libzp
calls over NHWC activation buffers (host orchestration only -- every arithmetic op is a
HIP kernel in libzp.so).

Reference forward (what is executed, in order):
  model/BinaryCodeNet.py:161-174  DeepLabV3.forward (concat branch) -> split [1, L]
  model/resnet.py:233-246         stem (torchvision conv1/bn1/relu) -> x_128; maxpool + layer1 -> x_64;
                                  layer2 -> x_32; layer4 (d2) -> x_16; layer5 (d4) -> x_high
  model/aspp.py:83-114            4 ASPP branches + image pool -> cat(1280) -> 1x1 -> upsample_1
                                  -> cat(x_64) -> upsample_2 -> cat(x_128) -> conv_1x1_4
The torch.cat's are never materialised: producers write into channel slices of one buffer.

Modes
  eval  : BatchNorm folded into a per-channel scale/shift applied in the conv epilogue
          (with bias, residual add and ReLU), one launch per conv (ASPP's four branches in one).
  train : BatchNorm with batch statistics (per-channel sums emitted by the conv epilogue,
          finalised on device, running stats updated with momentum 0.1, unbiased var), then
          a fused scale/shift/residual/ReLU pass; the tape keeps what the backward needs.
Backward (train): for each recorded op in reverse, BN backward (two passes), weight
gradient (split-K implicit GEMM), data gradient (implicit GEMM accumulating into the
input's gradient buffer).
"""
from __future__ import annotations

import os
import ctypes as C
import weakref

import torch

from . import _lib as L
from . import geometry as G
from .model.resnet import TVBottleneck

_KE = {L.ZP_F32: 32, L.ZP_BF16: 64, L.ZP_F16: 64, L.ZP_F32X3: 32, L.ZP_F32H2: 32}
_E = {L.ZP_F32: 4, L.ZP_BF16: 8, L.ZP_F16: 8, L.ZP_F32X3: 8, L.ZP_F32H2: 8}
# bytes per element (x3: three bf16 planes, h2: two fp16 planes)
_ES = {L.ZP_F32: 4, L.ZP_BF16: 2, L.ZP_F16: 2, L.ZP_F32X3: 6, L.ZP_F32H2: 4}
_TN = {L.ZP_F32: "f32", L.ZP_BF16: "bf16", L.ZP_F16: "f16", L.ZP_F32X3: "x3", L.ZP_F32H2: "h2"}
# the split-fp32 storage forms (include/zp.h): dtype code -> (planes, plane element type, the f32
# call's out_mode that writes it)
SPLIT = {L.ZP_F32X3: (3, torch.bfloat16, L.ZP_OUT_NHWC_X3), L.ZP_F32H2: (2, torch.float16, L.ZP_OUT_NHWC_H2)}


class Act:
    """A channel slice [c0, c0 + C) of an NHWC buffer [B, H, W, ld]."""
    __slots__ = ("buf", "c0", "C")

    def __init__(self, buf, c0=0, C=None):
        self.buf, self.c0 = buf, c0
        self.C = buf.shape[3] - c0 if C is None else C

    B = property(lambda s: s.buf.shape[0])
    H = property(lambda s: s.buf.shape[1])
    W = property(lambda s: s.buf.shape[2])
    ld = property(lambda s: s.buf.shape[3])
    P = property(lambda s: s.buf.shape[0] * s.buf.shape[1] * s.buf.shape[2])
    ptr = property(lambda s: s.buf.data_ptr())


class NchwInput(Act):
    """The f32 NCHW input [B, 3, H, W] seen as the stem's (8-channel) NHWC input: ld 0 tells
    zp_stem_split to read the NCHW tensor itself (include/zp.h)."""
    ld = property(lambda s: 0)


def joined(buf):
    """The f32 values of an activation buffer: itself, or -- for a split engine's plane-0 view --
    (hi + mid) + lo of a [3, ...] bf16 tensor (exact, include/zp.h ZP_F32X3), or hi + lo * 2^-11 of a
    [2, ...] fp16 tensor (ZP_F32H2)."""
    base = buf._base
    if base is not None and base.dim() == buf.dim() + 1 and base.data_ptr() == buf.data_ptr():
        if buf.dtype == torch.bfloat16 and base.shape[0] == 3:
            return (base[0].float() + base[1].float()) + base[2].float()
        if buf.dtype == torch.float16 and base.shape[0] == 2:
            return base[0].float() + base[1].float() * (1.0 / 2048.0)
    return buf.float()


def _i32arr(v):
    return (C.c_int * len(v))(*v)


class Unit:
    """conv / transposed conv (+ bias) (+ BatchNorm) (+ residual) (+ ReLU)."""

    def __init__(self, conv, bn=None, relu=True, cin_act=None):
        self.conv, self.bn, self.relu = conv, bn, relu
        self.kind = "convT" if isinstance(conv, torch.nn.ConvTranspose2d) else "conv"
        self.k = conv.kernel_size[0]
        self.s = conv.stride[0]
        self.p = conv.padding[0]
        self.d = conv.dilation[0]
        self.cin_w, self.cout = conv.in_channels, conv.out_channels
        self.cin = cin_act or self.cin_w

    # geometry ---------------------------------------------------------------------------------
    def fwd_plan(self, IH, IW):
        if self.kind == "convT":
            return G.convT_fwd(IH, IW, self.k, self.s, self.p, self.conv.output_padding[0])
        return G.conv_fwd(IH, IW, self.k, self.s, self.p, self.d)

    def dgrad_plan(self, IH, IW):
        if self.kind == "convT":
            return G.convT_dgrad(IH, IW, self.k, self.s, self.p)
        return G.conv_dgrad(IH, IW, self.k, self.s, self.p, self.d)

    def out_hw(self, IH, IW):
        if self.kind == "convT":
            op = self.conv.output_padding[0]
            return (IH - 1) * self.s - 2 * self.p + self.k + op, (IW - 1) * self.s - 2 * self.p + self.k + op
        return G.out_size(IH, self.k, self.s, self.p, self.d), G.out_size(IW, self.k, self.s, self.p, self.d)


class Tape:
    def __init__(self):
        self.recs = []


class Engine:
    """Executes a BinaryCodeNet_Deeplab module tree (zebrapose_amd.model) with libzp."""

    def __init__(self, net, dtype=torch.bfloat16, x3=False, split=None):
        """split: fp32 in a split form (include/zp.h), eval-mode forward only -- the fp32 network's
        training path keeps the exact-f32 MFMA engine:
          "x3" (x3=True): three bf16 planes (hi, mid, lo) summing exactly to the f32 value, every
                conv product from its six leading terms on bf16 MFMAs (ZP_F32X3);
          "h2": two fp16 planes, v = hi + lo * 2^-11 (22 bits), three fp16 MFMA terms (ZP_F32H2)."""
        self._net = weakref.ref(net)
        if x3:
            split = "x3"
        assert split in (None, "x3", "h2"), split
        self.split = split
        self.x3 = split is not None  # any split-fp32 form
        self.dt = {"x3": L.ZP_F32X3, "h2": L.ZP_F32H2}[split] if split else L.dtype_code(dtype)
        self.npl, self.dtype, self.split_out = SPLIT[self.dt] if split else (1, dtype, None)
        # split forms: the stem as im2col + split GEMM (ZP_SPLIT_STEM=0: the exact-f32 small-Cin
        # kernel writing split output)
        self.split_stem = os.environ.get("ZP_SPLIT_STEM", "1") != "0"
        # two planes: the stem in one launch from the f32 image (zp_stem_split); ZP_STEM_DIRECT=0 keeps
        # im2col + GEMM
        self.stem_direct = os.environ.get("ZP_STEM_DIRECT", "1") != "0"
        self._packed = {}
        self._jobs = []  # (cache key, weight, PackJob) of every cached packing, for _prepack
        self._job_table = None
        self._folds = {}
        self._fold_epoch = 0
        self._cache_gen = 0  # bumped when a packing / fold buffer is allocated or dropped (graphs.py)
        self.timing = None  # optional list of (label, start_event, end_event) for conv launches
        # optional list: every eval-mode op appends (kind, unit, x, out, res) with the buffers it
        # read and wrote (kept alive by the list) -- the teacher-forced layer parity tests replay
        # each op on the host from the device's own stored inputs (tests/test_gpu_bench_geometry.py)
        self.trace = None
        # optional list: every conv launch appends (stage, kernel label, flops, algorithmic bytes) in
        # launch order; self.stage names the network stage being enqueued (stem, layer1, layer2,
        # layer4, layer5, aspp, up1, up2, head) -- tools/prof_stages.py attributes rocprofv3's
        # per-dispatch counters to stages with it
        self.stage_log = None
        self.stage = None
        # optional list: every training-backward op appends a dict with the buffers it read and the
        # gradients it wrote (accumulated gradient slices as (before, after) copies) -- the
        # teacher-forced train-step parity test replays each one on the host (tests/test_gpu_train_tf.py)
        self.bwd_trace = None
        # training backward: each unit's weight gradient runs on a second HIP stream, concurrently
        # with its input gradient and the next unit's BN backward on the main stream (the wgrad
        # kernel is L2/MFMA-bound, the BN passes HBM-bound; both fill the other's tail).  The
        # streams join at the end of backward().  ZP_SIDE_WGRAD=0 keeps everything on one stream.
        self.side_wgrad = os.environ.get("ZP_SIDE_WGRAD", "1") != "0"
        self.convT_wgrad_swap = os.environ.get("ZP_CONVT_WGRAD_SWAP", "1") != "0"
        self._side = None
        self._side_used = False
        self.bn_mask_from_raw = True  # BN+ReLU backward without residual: mask from raw (A/B knob)
        # the reduce of a BN + ReLU backward taken by its reader's dgrad launch (_bnr_fusable)
        self.bn_bwd_fused = os.environ.get("ZP_BN_BWD_FUSED", "1") != "0"
        # two-plane eval forward: up2's last conv and the head in one launch (zp_conv2d_head);
        # ZP_FUSE_HEAD=0 keeps them apart
        self.fuse_head = os.environ.get("ZP_FUSE_HEAD", "1") != "0"
        # the two-plane form's range word (range_word) and whether packings were made since its
        # reader last looked (unread_packs: set by _pack, cleared by the readers)
        self._rflag = None
        self.unread_packs = False
        self.range_probe = None  # optional list (tests): see _probe

    def range_word(self, device):
        """This engine's zp_split_range_flag word on ``device`` (int32 [1]): raised by any of its
        two-plane stores or weight packs that meets a value beyond the form's range (include/zp.h)."""
        dev = torch.device(device)
        if dev.index is None:
            dev = torch.device(dev.type, torch.cuda.current_device())
        if self._rflag is None or self._rflag.device != dev:
            self._rflag = torch.zeros(1, dtype=torch.int32, device=dev)
        return self._rflag

    # ------------------------------------------------------------------ weight / BN caches
    def invalidate(self):
        self._cache_gen += 1
        self._packed.clear()
        self._jobs = []
        self._job_table = None
        self._folds.clear()

    def _empty(self, shape, dev):
        """An activation buffer of this engine's storage: plane 0 (a [B, H, W, C] view) of a
        [NPL, B, H, W, C] tensor in a split mode."""
        if self.x3:
            return torch.empty((self.npl,) + tuple(shape), dtype=self.dtype, device=dev)[0]
        return torch.empty(shape, dtype=self.dtype, device=dev)

    def _pack(self, unit, sub, transposed, cstride, k_pad, rows, tag, cache=True, dt=None):
        """Packed weights of one (conv, sub-problem, role), cached on the weight's version counter.
        Every packing is also recorded as a job of the batched repack (_prepack).  dt overrides the
        engine's dtype code (the x3 engine's f32 stem)."""
        dt = self.dt if dt is None else dt
        w = unit.conv.weight
        key = (id(unit.conv), tag, tuple(sub.taps), cstride, k_pad, dt)
        ver = (w._version, w.data_ptr())
        hit = self._packed.get(key) if cache else None
        if hit is not None and hit[0] == ver:
            return hit[1]
        d0, d1 = w.shape[0], w.shape[1]
        shape = (SPLIT[dt][0], rows, k_pad) if dt in SPLIT else (rows, k_pad)
        if hit is not None and tuple(hit[1].shape) == shape:
            out = hit[1]
        else:
            tdt = SPLIT[dt][1] if dt in SPLIT else {L.ZP_F32: torch.float32, L.ZP_BF16: torch.bfloat16,
                                                      L.ZP_F16: torch.float16}[dt]
            out = torch.empty(shape, dtype=tdt, device=w.device)
            self._cache_gen += 1
        if dt == L.ZP_F32H2:
            self.unread_packs = True
        ky = [t[0] for t in sub.taps]
        kx = [t[1] for t in sub.taps]
        L.call("zp_pack_weight", w.data_ptr(), d0, d1, w.shape[2], w.shape[3], transposed, len(sub.taps),
               _i32arr(ky), _i32arr(kx), cstride, dt, out.data_ptr(), rows, k_pad, L.stream_ptr())
        if cache:
            if key not in self._packed:
                j = L.PackJob()
                j.src, j.dst = w.data_ptr(), out.data_ptr()
                j.d0, j.d1, j.kh, j.kw = d0, d1, w.shape[2], w.shape[3]
                j.transposed, j.ntaps, j.cstride, j.rows_pad, j.k_pad, j.dtype = \
                    transposed, len(sub.taps), cstride, rows, k_pad, dt
                for t, (a, b) in enumerate(zip(ky, kx)):
                    j.ky[t], j.kx[t] = a, b
                self._jobs.append((key, w, j))
                self._job_table = None
            self._packed[key] = (ver, out)
        return out

    def _prepack(self, device):
        """Batched repack (training): once the optimizer has changed the weights, every recorded
        packing job runs in ONE zp_pack_weight_multi launch and the cache is revalidated, so the
        forward / backward below hit the cache instead of launching ~110 pack kernels."""
        if not self._jobs:
            return
        if all(self._packed[k][0] == (w._version, w.data_ptr()) for k, w, _ in self._jobs):
            return
        if self._job_table is None or any(self._packed[k][1].data_ptr() != j.dst or w.data_ptr() != j.src
                                          for k, w, j in self._jobs):
            for k, w, j in self._jobs:
                j.src, j.dst = w.data_ptr(), self._packed[k][1].data_ptr()
            n = len(self._jobs)
            arr = (L.PackJob * n)(*[j for _, _, j in self._jobs])
            table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(device)
            pre = [0]
            for _, _, j in self._jobs:
                pre.append(pre[-1] + j.rows_pad * j.k_pad)
            self._job_table = (table, torch.tensor(pre, dtype=torch.int64).to(device), n, pre[-1])
        table, prefix, n, total = self._job_table
        L.call("zp_pack_weight_multi", n, table.data_ptr(), prefix.data_ptr(), total, L.stream_ptr())
        for key, w, _ in self._jobs:
            self._packed[key] = ((w._version, w.data_ptr()), self._packed[key][1])

    def _fold(self, unit):
        bn, bias = unit.bn, unit.conv.bias
        if bn is None:
            return None, bias
        key = id(bn)
        vers = (bn.weight._version, bn.bias._version, bn.running_mean._version, bn.running_var._version,
                None if bias is None else bias._version, self._fold_epoch)
        hit = self._folds.get(key)
        if hit is not None and hit[0] == vers:
            return hit[1], hit[2]
        dev = bn.weight.device
        if hit is not None:  # refold in place: a captured graph keeps reading these addresses
            scale, shift = hit[1], hit[2]
        else:
            scale = torch.empty(unit.cout, dtype=torch.float32, device=dev)
            shift = torch.empty_like(scale)
            self._cache_gen += 1
        L.call("zp_bn_fold", bn.weight.data_ptr(), bn.bias.data_ptr(), bn.running_mean.data_ptr(),
               bn.running_var.data_ptr(), L.ptr(bias), C.c_float(bn.eps), unit.cout, scale.data_ptr(),
               shift.data_ptr(), L.stream_ptr())
        self._folds[key] = (vers, scale, shift)
        return scale, shift

    # ------------------------------------------------------------------ conv launch
    def _conv(self, x: Act, plan, cout, weights, k_pad, rows, outs, res=None, relu=False,
              out_mode=L.ZP_OUT_NHWC, stats=None, small=None, label=None, dt=None, head=None, bnr=None):
        """weights / outs: per sub.  outs[i] = (y_ptr, ldy, cy0, OH, OW, scale, shift, y2).  dt
        overrides the engine's dtype code (the x3 engine's f32 stem).  head: (L.HeadArgs, head FLOPs,
        head bytes) -- the conv feeds the fused 1x1 head (zp_conv2d_head) instead of storing.
        bnr: (raw, save, P) of the train-mode BN whose output gradient this data-gradient launch
        writes: the launch also takes that BN backward's reduce (zp.h bnr_*); returns (partials,
        parts) in place of (stats, parts)."""
        dt = self.dt if dt is None else dt
        a = L.ConvArgs()
        a.dtype = dt
        a.x = x.ptr
        a.ldx, a.cx0, a.IH, a.IW, a.Cin = x.ld, x.c0, x.H, x.W, x.C
        a.N, a.GH, a.GW, a.sy, a.sx = x.B, plan.GH, plan.GW, plan.sy, plan.sy
        a.Cout, a.k_pad, a.w_rows = cout, k_pad, rows
        if res is not None:
            a.res, a.ldr, a.cr0 = res.ptr, res.ld, res.c0
        a.relu, a.out_mode = int(relu), out_mode
        a.nsub = len(plan.subs)
        for i, sb in enumerate(plan.subs):
            s = a.sub[i]
            y, ldy, cy0, OH, OW, scale, shift, y2 = outs[i]
            s.w = weights[i].data_ptr()
            s.scale, s.shift = L.ptr(scale), L.ptr(shift)
            s.y, s.y2 = y, y2
            s.ldy, s.cy0, s.OH, s.OW = ldy, cy0, OH, OW
            s.oys, s.oyo, s.oxs, s.oxo = sb.oys, sb.oyo, sb.oxs, sb.oxo
            s.ntaps = len(sb.taps)
            for t, (ty, tx) in enumerate(sb.offs):
                s.ty[t], s.tx[t] = ty, tx
            if small is not None:
                s.kw, s.dil, s.pad = small
        parts = 0
        if bnr is not None:
            raw, save, P = bnr
            parts = L.lib.zp_conv2d_bnr_parts(C.byref(a))
            rows_ = max(parts, L.lib.zp_bn_bwd_parts(P, cout)) + 1
            stats = torch.empty(2 * rows_ * cout, dtype=torch.float32, device=x.buf.device)
            a.bnr_x, a.bnr_save, a.bnr_part = raw.data_ptr(), save.data_ptr(), stats.data_ptr()
        elif stats == "alloc":
            parts = L.lib.zp_conv2d_stat_parts(C.byref(a))
            stats = torch.empty(L.lib.zp_bn_finalize_floats(parts, cout), dtype=torch.float32, device=x.buf.device)
        if bnr is not None:
            pass
        elif stats is not None:
            a.stats = stats.data_ptr()
        elif dt in SPLIT:  # split-K workspace of a small split-fp32 launch (zp_conv2d_split_ws)
            nb = L.lib.zp_conv2d_split_ws(C.byref(a))
            if nb > 0:
                stats = torch.empty(nb // 4, dtype=torch.float32, device=x.buf.device)
                a.stats = stats.data_ptr()
        st = L.stream_ptr()

        def launch():
            if head is not None:
                L.check(L.lib.zp_conv2d_head(C.byref(a), C.byref(head[0]), st), "zp_conv2d_head")
            else:
                L.check(L.lib.zp_conv2d(C.byref(a), st), "zp_conv2d")
        if self.timing is not None or self.stage_log is not None or self.range_probe is not None:
            if self.timing is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
            launch()
            if self.timing is not None:
                e1.record()
            flops = 2.0 * x.B * plan.GH * plan.GW * sum(len(sb.taps) for sb in plan.subs) * x.C * cout
            kname = self._kname(a, plan, x, dt)
            if head is not None:
                flops += head[1]
                kname = kname.replace("k_conv3w<", "k_conv3w_head<").replace("k_conv_strip2<", "k_conv_strip2_head<")
            geo = (f"{label}:{x.C}->{cout} taps{max(len(sb.taps) for sb in plan.subs)} "
                   f"{x.H}x{x.W}->{plan.GH}x{plan.GW}x{a.nsub}")
            # algorithmic HBM bytes: the input slice and every output read / written once, the
            # packed weights of each sub-problem once (the residual, when fused, read once)
            es = _ES[dt]
            osz = 4 if out_mode == L.ZP_OUT_HEAD_NCHW else (6 if out_mode == L.ZP_OUT_NHWC_X3 else
                                                            (4 if out_mode == L.ZP_OUT_NHWC_H2 else es))
            mgrid = x.B * plan.GH * plan.GW
            nbytes = (x.P * x.C * es + len(plan.subs) * mgrid * cout * osz
                      + sum(w.numel() * w.element_size() for w in weights) + (0 if res is None else mgrid * cout * es))
            if head is not None:  # no conv output stored; the head's inputs / outputs instead
                nbytes += head[2] - len(plan.subs) * mgrid * cout * osz
            if self.timing is not None:
                self.timing.append((geo, e0, e1, flops, kname, nbytes))
            if self.stage_log is not None:
                self.stage_log.append((self.stage, kname, flops, nbytes, geo))
            self._probe(kname)
        else:
            launch()
        return stats, parts

    def _probe(self, kname):
        """range_probe (tests): after each launch, a device copy of this engine's range word, so a
        test can name the first launch that raised it."""
        if self.range_probe is not None and self._rflag is not None:
            self.range_probe.append((self.stage, kname, self._rflag.clone()))

    def _kname(self, a, plan, x, dt=None):
        """rocprofv3's kernel instantiation of this launch, in the label form tools/prof_summary.py
        maps the demangled names to."""
        dt = self.dt if dt is None else dt
        tc, tp, stages, var = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        L.call("zp_conv2d_config", C.byref(a), C.byref(tc), C.byref(tp), C.byref(stages), C.byref(var))
        tn = _TN[dt]
        if var.value == 6:  # rocprofv3 name: k_conv3w<ABL, DM, HEAD, .., NUM, TPX> (TPX 128: the 256 x 128 tile)
            return f"k_conv3w<{tn}>" if tp.value == 256 else f"k_conv3w<{tn},TP={tp.value}>"
        if var.value == 5:  # rocprofv3 name: k_conv3s<NPL, WC>
            return f"k_conv3s<{tn},WC={tc.value // 32}>"
        if var.value == 4:  # rocprofv3 name: k_conv3<NPL, WC, WP, NWP, ST, PIPE>
            return f"k_conv3<{tn},WC={tc.value // 32},NWP={tp.value // 64}>"
        if var.value == 1:  # rocprofv3 name: k_conv_strip<T, WC, STAGES, SPW = 5>
            return f"k_conv_strip<{tn},WC={tc.value // 32},ST=3>"
        if var.value == 3:  # rocprofv3 name: k_conv_quad<T, W>
            return f"k_conv_quad<{tn},W={plan.GW}>"
        if var.value == 7:  # rocprofv3 name: k_conv1x1n<T> (narrow-K 1x1: the head's data gradient)
            return f"k_conv1x1n<{tn}>"
        if var.value == 2:  # rocprofv3 name: k_conv_strip2<T, WC, SPW = 5>
            return f"k_conv_strip2<{tn},WC={tc.value // 32}>"
        # rocprofv3 name: k_conv<T, WC = tc / 32, WP = 4, NWP = tp / 64, STAGES, smallC>
        return (f"k_conv<{tn},WC={tc.value // 32},WP=4,"
                f"NWP={tp.value // 64},ST={stages.value},smallC={int(x.C < _KE[dt])}>")

    def _kpad(self, ntaps, cin):
        return G.ceil_to(ntaps * cin, _KE[self.dt])

    def _fwd_weights(self, unit, plan, cache, dt=None):
        dt = self.dt if dt is None else dt
        kp = max(G.ceil_to(len(sb.taps) * unit.cin, _KE[dt]) for sb in plan.subs)
        rows = L.lib.zp_conv_rows_pad(unit.cout)
        tr = 1 if unit.kind == "convT" else 0
        ws = [self._pack(unit, sb, tr, unit.cin, kp, rows, "fwd", cache, dt=dt) for sb in plan.subs]
        return ws, kp, rows

    def _small(self, cin, k, d, p):
        return (k, d, p) if cin < _KE[self.dt] else None

    # ------------------------------------------------------------------ unit forward
    def unit_fwd(self, unit, x: Act, out: Act, tape, res: Act = None, label=None):
        assert x.C == unit.cin, (x.C, unit.cin)
        plan = unit.fwd_plan(x.H, x.W)
        OH, OW = unit.out_hw(x.H, x.W)
        assert (out.H, out.W, out.C) == (OH, OW, unit.cout), ((out.H, out.W, out.C), (OH, OW, unit.cout))
        train = tape is not None
        if self.x3 and unit.cin < _KE[self.dt] and unit.s == 2 and unit.d == 1 and self.split_stem:
            # the split-mode stem as a GEMM: the f32 image's 7x7 / s2 patches (k*k*3 = 147 -> 160
            # channels, zp_im2col_split) in split form, then a 1x1 split-fp32 conv over them with the
            # 7x7 weights packed tap-major (k = tap * 3 + c, the im2col order)
            assert not train, "the split engine runs eval forwards only"
            cr = unit.conv.weight.shape[1]
            kp = G.ceil_to(unit.k * unit.k * cr, 32)
            if self._stem_direct_ok(unit, OH, OW, out.ld, out.c0, x.ld):
                # one launch from the f32 image (zp_stem_split): no patch tensor
                taps = [(ky, kx) for ky in range(unit.k) for kx in range(unit.k)]
                rows = G.ceil_to(unit.cout, 128)
                w = self._pack(unit, G.Sub(taps, [(0, 0)] * len(taps)), 0, cr, kp, rows, "stem_im2col")
                scale, shift = self._fold(unit)
                L.call("zp_stem_split", x.ptr, x.B, x.H, x.W, x.ld, w.data_ptr(), rows, kp, scale.data_ptr(),
                       shift.data_ptr(), self.dt, out.ptr, out.ld, out.c0, OH, OW, L.stream_ptr())
                if self.stage_log is not None:
                    fl = 2.0 * x.B * OH * OW * unit.k * unit.k * cr * unit.cout
                    nb = x.P * (x.ld or 3) * 4 + x.B * OH * OW * unit.cout * 4 + w.numel() * w.element_size()
                    self.stage_log.append((self.stage, "k_stem_h2", fl, nb, f"{label}:{cr}->{unit.cout} 7x7s2"))
                self._probe("k_stem_h2")
                if self.trace is not None:
                    self.trace.append(("conv", unit, x, out, res))
                return
            if isinstance(x, NchwInput):
                raise AssertionError("the NCHW stem input reached the im2col stem (nchw_stem / unit_fwd disagree)")
            col = Act(self._empty((x.B, OH, OW, kp), x.buf.device))
            L.call("zp_im2col_split", x.ptr, x.B, x.H, x.W, x.ld, cr, unit.k, unit.s, unit.p, OH, OW, kp, self.dt,
                   col.ptr, L.stream_ptr())
            taps = [(ky, kx) for ky in range(unit.k) for kx in range(unit.k)]
            rows = G.ceil_to(unit.cout, 128)
            w = self._pack(unit, G.Sub(taps, [(0, 0)] * len(taps)), 0, cr, kp, rows, "stem_im2col")
            scale, shift = self._fold(unit)
            plan = G.conv_fwd(OH, OW, 1, 1, 0)
            outs = [(out.ptr, out.ld, out.c0, OH, OW, scale, shift, None)]
            self._conv(col, plan, unit.cout, [w], kp, rows, outs, res, unit.relu, label=label)
            if self.trace is not None:
                self.trace.append(("conv", unit, x, out, res))
            return
        if isinstance(x, NchwInput):
            raise AssertionError("the NCHW stem input reaches zp_stem_split only (nchw_stem / unit_fwd disagree)")
        if self.x3 and unit.cin < _KE[self.dt]:
            # the split-mode stem: its 3 (-> 8) input channels are below k_conv3's 32-channel K step;
            # it runs the exact-f32 small-Cin kernel on the f32 NHWC input and writes split output
            assert not train, "the x3 engine runs eval forwards only"
            ws, kp, rows = self._fwd_weights(unit, plan, cache=True, dt=L.ZP_F32)
            scale, shift = self._fold(unit)
            outs = [(out.ptr, out.ld, out.c0, OH, OW, scale, shift, None)] * len(plan.subs)
            self._conv(x, plan, unit.cout, ws, kp, rows, outs, res, unit.relu, out_mode=self.split_out,
                       small=(unit.k, unit.d, unit.p), label=label, dt=L.ZP_F32)
            if self.trace is not None:
                self.trace.append(("conv", unit, x, out, res))
            return
        ws, kp, rows = self._fwd_weights(unit, plan, cache=True)
        small = self._small(unit.cin, unit.k, unit.d, unit.p)
        if not train or unit.bn is None:
            scale, shift = self._fold(unit)
            outs = [(out.ptr, out.ld, out.c0, OH, OW, scale, shift, None)] * len(plan.subs)
            self._conv(x, plan, unit.cout, ws, kp, rows, outs, res, unit.relu, small=small, label=label)
            if self.trace is not None and not train:
                self.trace.append(("conv", unit, x, out, res))
            if train:
                tape.recs.append(("plain", unit, x, out, res, None, None))
            return
        bn = unit.bn
        if bn.momentum is None:
            raise NotImplementedError("BatchNorm momentum=None (cumulative average) is not supported")
        P = x.B * OH * OW
        if P <= 1:
            raise ValueError("Expected more than 1 value per channel when training")
        raw = torch.empty((x.B, OH, OW, unit.cout), dtype=self.dtype, device=x.buf.device)
        outs = [(raw.data_ptr(), unit.cout, 0, OH, OW, None, None, None)] * len(plan.subs)
        stats, parts = self._conv(x, plan, unit.cout, ws, kp, rows, outs, None, False, stats="alloc", small=small,
                                  label=label)
        dev = x.buf.device
        scale = torch.empty(unit.cout, dtype=torch.float32, device=dev)
        shift = torch.empty_like(scale)
        save = torch.empty(4 * unit.cout, dtype=torch.float32, device=dev)  # mean, invstd, scale, shift
        L.call("zp_bn_train_finalize", stats.data_ptr(), parts, unit.cout, P, C.c_float(bn.eps),
               C.c_float(bn.momentum), bn.weight.data_ptr(), bn.bias.data_ptr(), L.ptr(unit.conv.bias),
               bn.running_mean.data_ptr(), bn.running_var.data_ptr(), bn.num_batches_tracked.data_ptr(),
               scale.data_ptr(), shift.data_ptr(), save.data_ptr(), L.stream_ptr())
        L.call("zp_bn_apply", raw.data_ptr(), P, unit.cout, scale.data_ptr(), shift.data_ptr(),
               None if res is None else res.ptr, 0 if res is None else res.ld, 0 if res is None else res.c0,
               int(unit.relu), self.dt, out.ptr, out.ld, out.c0, L.stream_ptr())
        self._fold_epoch += 1
        for buf in (bn.running_mean, bn.running_var, bn.num_batches_tracked):  # written in place by the kernel
            torch.autograd.graph.increment_version(buf)
        tape.recs.append(("bn", unit, x, out, res, raw, save))

    def aspp_branches_fwd(self, units, x: Act, outs_act, tape):
        """The four parallel ASPP branches (aspp.py:89-92) -- one launch with four sub-problems in
        eval mode (same input, own weights / BN / output slice)."""
        if tape is not None:
            for u, o in zip(units, outs_act):
                self.unit_fwd(u, x, o, tape, label="aspp")
            return
        plans = [u.fwd_plan(x.H, x.W) for u in units]
        kp = max(self._kpad(len(p.subs[0].taps), x.C) for p in plans)
        rows = L.lib.zp_conv_rows_pad(256)
        merged = G.Plan(plans[0].GH, plans[0].GW, 1, [p.subs[0] for p in plans])
        ws, outs = [], []
        for u, p, o in zip(units, plans, outs_act):
            ws.append(self._pack(u, p.subs[0], 0, x.C, kp, rows, "fwd", True))
            scale, shift = self._fold(u)
            outs.append((o.ptr, o.ld, o.c0, o.H, o.W, scale, shift, None))
        self._conv(x, merged, 256, ws, kp, rows, outs, None, True, label="aspp")
        if self.trace is not None:
            for u, o in zip(units, outs_act):
                self.trace.append(("conv", u, x, o, None))

    def head_fwd(self, unit, x: Act, mask, code, tape, key="head"):
        """Head conv writing f32 NCHW channel 0 -> mask, channels 1.. -> code (code None when the
        head has one channel); ``key`` names its output gradient in the backward's gmap."""
        plan = unit.fwd_plan(x.H, x.W)
        OH, OW = unit.out_hw(x.H, x.W)
        ws, kp, rows = self._fwd_weights(unit, plan, cache=True)
        outs = [(mask.data_ptr(), 0, 0, OH, OW, None, unit.conv.bias, L.ptr(code))]
        self._conv(x, plan, unit.cout, ws, kp, rows, outs, None, False, out_mode=L.ZP_OUT_HEAD_NCHW,
                   small=self._small(unit.cin, unit.k, unit.d, unit.p), label="head")
        if tape is not None:
            tape.recs.append(("head", unit, x, key, None, None, None))
        elif self.trace is not None:
            self.trace.append(("head", unit, x, (mask, code), None))

    def _stem_direct_ok(self, unit, OH, OW, out_ld, out_c0, x_ld):
        """The one-launch two-plane stem (zp_stem_split) takes this 7x7 / s2 conv: split stem on,
        output width <= 128 dividing 256, whole 256-pixel tiles, 16-byte output rows and input rows
        of 4 floats (x_ld 0: the NCHW input itself)."""
        cr = unit.conv.weight.shape[1]
        return (self.x3 and self.split_stem and self.dt == L.ZP_F32H2 and self.stem_direct
                and unit.cin < _KE[self.dt] and unit.d == 1
                and (unit.k, unit.s, unit.p, cr, unit.cout) == (7, 2, 3, 3, 64)
                and OW <= 128 and 256 % OW == 0 and (OH * OW) % 256 == 0 and out_ld % 8 == 0 and out_c0 % 8 == 0
                and x_ld % 4 == 0)

    def nchw_stem(self, stem_unit, H, W, tape):
        """True when the two-plane stem (zp_stem_split) reads the f32 NCHW input directly: eval, no
        trace (the teacher-forced replays start from the NHWC copy), and the stem unit takes
        unit_fwd's zp_stem_split branch (same predicate) on the 64-channel x_128 output."""
        if tape is not None or self.trace is not None:
            return False
        OH, OW = stem_unit.out_hw(H, W)
        return (OH, OW) == (H // 2, W // 2) and self._stem_direct_ok(stem_unit, OH, OW, 64, 0, 0)

    def head_fusable(self, B, H, W):
        """True when up2's last conv (3x3, 256 -> 256) and the 1x1 head run fused (zp_conv2d_head):
        eval forward, no trace, and -- two-plane engine -- the 256 x 256 tile eligible at this grid, or
        -- bf16 / fp16 -- the strip tile (conv + per-cout-tile head partials, then their combine)."""
        if self.dt not in (L.ZP_F32H2, L.ZP_BF16, L.ZP_F16) or not self.fuse_head or self.trace is not None:
            return False
        a = L.ConvArgs()
        a.dtype, a.Cin, a.Cout, a.N, a.GH, a.GW, a.IH, a.IW = self.dt, 256, 256, B, H, W, H, W
        a.w_rows = int(L.lib.zp_conv_rows_pad(256))
        a.ldx, a.cx0, a.sy, a.sx, a.k_pad = 256, 0, 1, 1, 9 * 256
        a.out_mode, a.nsub = L.ZP_OUT_NHWC, 1
        s = a.sub[0]
        s.ldy, s.cy0, s.OH, s.OW, s.oys, s.oxs, s.ntaps = 256, 0, H, W, 1, 1, 9
        for t in range(9):
            s.ty[t], s.tx[t] = t // 3 - 1, t % 3 - 1
        return bool(L.lib.zp_conv2d_head_ok(C.byref(a)))

    def unit_fwd_head(self, unit, x: Act, head_unit, x2: Act, mask, code):
        """unit (3x3 conv + BN + ReLU, Cout 256) feeding the head conv over [its output | x2] in one
        launch (zp_conv2d_head): the reference's upsample_2[6:9] then conv_1x1_4(torch.cat([x, x_128]))
        (aspp.py:105-112) and the mask / code split (BinaryCodeNet.py:172)."""
        plan = unit.fwd_plan(x.H, x.W)
        OH, OW = unit.out_hw(x.H, x.W)
        ws, kp, rows = self._fwd_weights(unit, plan, cache=True)
        scale, shift = self._fold(unit)
        hp = head_unit.fwd_plan(OH, OW)
        hk = G.ceil_to(head_unit.cin, 32)
        hw = self._pack(head_unit, hp.subs[0], 0, head_unit.cin, hk, 32, "head_fused", True)
        h = L.HeadArgs()
        h.w, h.k_pad, h.bias, h.cout = hw.data_ptr(), hk, L.ptr(head_unit.conv.bias), head_unit.cout
        h.x2, h.ldx2, h.cx20, h.C2 = x2.ptr, x2.ld, x2.c0, x2.C
        h.mask, h.code = mask.data_ptr(), L.ptr(code)
        B = x.B
        hws = None
        if self.dt in (L.ZP_BF16, L.ZP_F16):  # the cout tiles' head partials (zp_conv2d_head_ws)
            hws = torch.empty(2 * 32 * B * OH * OW, dtype=torch.float32, device=x.buf.device)
            h.ws = hws.data_ptr()
        hflops = 2.0 * B * OH * OW * head_unit.cin * head_unit.cout
        hbytes = B * OH * OW * (x2.C * _ES[self.dt] + head_unit.cout * 4) + hw.numel() * hw.element_size()
        outs = [(mask.data_ptr(), 256, 0, OH, OW, scale, shift, None)]  # (y: never written by the fused launch)
        self._conv(x, plan, unit.cout, ws, kp, rows, outs, None, unit.relu, label="upconv+head",
                   head=(h, hflops, hbytes))
        del hws  # (the partials buffer's block returns to the stream's pool: the launches are enqueued)

    # ------------------------------------------------------------------ backward pieces
    def _grad_buf(self, gmap, act: Act):
        """gradient buffer twin of an activation buffer; allocated uninitialised and recorded as
        fresh (no writer yet) in gmap["__fresh__"]."""
        key = act.buf.data_ptr()
        g = gmap.get(key)
        if g is None:
            g = torch.empty_like(act.buf)
            gmap[key] = g
            gmap.setdefault("__fresh__", set()).add(key)
        return key, g

    def _grad(self, gmap, act: Act):
        """gradient slice twin of an activation slice, to be read or accumulated into: a fresh
        buffer is zeroed first."""
        key, g = self._grad_buf(gmap, act)
        fresh = gmap.setdefault("__fresh__", set())
        if key in fresh:
            fresh.discard(key)
            g.zero_()
        return Act(g, act.c0, act.C)

    def _grad_out(self, gmap, act: Act, whole_write):
        """gradient slice a kernel is about to write -> (slice, accumulate).  The first writer of a
        buffer that writes all of it (whole_write: every pixel; the slice spans every channel)
        overwrites instead of accumulating, so the buffer needs no zero fill."""
        key, g = self._grad_buf(gmap, act)
        fresh = gmap.setdefault("__fresh__", set())
        if key in fresh:
            fresh.discard(key)
            if whole_write and act.c0 == 0 and act.C == act.ld:
                return Act(g, act.c0, act.C), False
            g.zero_()
        return Act(g, act.c0, act.C), True

    def _convT_wgrad_swap(self, unit, x: Act, dy: Act):
        """True when a ConvTranspose2d(3, s2, p1, op1) weight gradient runs as the stride-2 conv's
        over dy with x as its output gradient (zp_conv.hip k_wgrad2, stride 2): dW[ci][co][ky][kx] =
        sum_g x[g][ci] dy[2 g + (ky, kx) - 1][co], the ConvT weight's own [in][out][k][k] layout.
        16-bit only (the lean kernel's dtype); the four-phase form otherwise (ZP_CONVT_WGRAD_SWAP=0)."""
        return (self.convT_wgrad_swap and unit.kind == "convT" and self.dt == L.ZP_BF16
                and (unit.k, unit.s, unit.p, unit.conv.output_padding[0]) == (3, 2, 1, 1)
                and x.C == unit.cin_w and (dy.H, dy.W) == (2 * x.H, 2 * x.W))

    def _wgrad(self, unit, x: Act, plan, dy: Act, dw):
        # (i, o): the launch's input and output-gradient activations; (x, dy) unless exchanged
        i_act, o_act, cout, cw, tw = x, dy, unit.cout, unit.cin_w, 1 if unit.kind == "convT" else 0
        if self._convT_wgrad_swap(unit, x, dy):
            plan = G.convT_dgrad(x.H, x.W, unit.k, unit.s, unit.p)
            i_act, o_act, cout, cw, tw = dy, x, unit.cin_w, unit.cout, 0
        a = L.WgradArgs()
        a.dtype = self.dt
        a.x, a.ldx, a.cx0, a.IH, a.IW, a.Cin = i_act.ptr, i_act.ld, i_act.c0, i_act.H, i_act.W, i_act.C
        a.N, a.GH, a.GW, a.sy, a.sx = i_act.B, plan.GH, plan.GW, plan.sy, plan.sy
        a.Cout, a.Cw, a.kh, a.kw = cout, cw, unit.k, unit.k
        a.transposed_w = tw
        a.nsub = len(plan.subs)
        for i, sb in enumerate(plan.subs):
            s = a.sub[i]
            s.dy, s.lddy, s.cdy0, s.OH, s.OW = o_act.ptr, o_act.ld, o_act.c0, o_act.H, o_act.W
            s.oys, s.oyo, s.oxs, s.oxo = sb.oys, sb.oyo, sb.oxs, sb.oxo
            s.ntaps = len(sb.taps)
            for t, ((ky, kx), (ty, tx)) in enumerate(zip(sb.taps, sb.offs)):
                s.ky[t], s.kx[t], s.ty[t], s.tx[t] = ky, kx, ty, tx
        a.dw = dw.data_ptr()
        a.accumulate = 0
        nbytes = L.lib.zp_conv2d_wgrad_ws_bytes(C.byref(a))
        ws = torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=dw.device)
        if self.timing is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            L.check(L.lib.zp_conv2d_wgrad(C.byref(a), ws.data_ptr(), L.stream_ptr()), "zp_conv2d_wgrad")
            e1.record()
            flops = 2.0 * x.B * plan.GH * plan.GW * sum(len(sb.taps) for sb in plan.subs) * x.C * unit.cout
            geo = (f"wgrad:{x.C}->{unit.cout} taps{max(len(sb.taps) for sb in plan.subs)} "
                   f"{x.H}x{x.W}->{plan.GH}x{plan.GW}x{a.nsub}")
            # algorithmic bytes: x and dy read once (16-bit), dw written once (f32)
            esz = x.buf.element_size()
            nbytes = (x.P * x.C + dy.P * unit.cout) * esz + dw.numel() * 4
            self.timing.append((geo, e0, e1, flops, "k_wgrad+reduce", nbytes))
            return
        L.check(L.lib.zp_conv2d_wgrad(C.byref(a), ws.data_ptr(), L.stream_ptr()), "zp_conv2d_wgrad")

    def _side_stream(self, dev):
        if not self.side_wgrad or dev.type != "cuda" or self.timing is not None or self.bwd_trace is not None:
            return None  # the per-launch timing (bench breakdown) wants the serial order
        if self._side is None:
            self._side = torch.cuda.Stream(dev)
        return self._side

    def _side_join(self, dev):
        if self._side is not None and self._side_used:
            torch.cuda.current_stream(dev).wait_stream(self._side)
        self._side_used = False

    def _dgrad(self, unit, gy: Act, gx: Act, accumulate=True, bnr=None):
        """gx (+)= dgrad(gy): accumulate into the input gradient slice (residual = itself), or
        overwrite it (accumulate False: its first writer, see _grad_out).  bnr: see _conv (the
        overwrite form only); returns _conv's (partials, parts)."""
        plan = unit.dgrad_plan(gx.H, gx.W)
        cin_l = gy.C  # = cout (padded for the head)
        kp = max(self._kpad(len(sb.taps), cin_l) for sb in plan.subs)
        rows = L.lib.zp_conv_rows_pad(unit.cin)
        tr = 0 if unit.kind == "convT" else 1
        ws = [self._pack(unit, sb, tr, cin_l, kp, rows, "dgrad") for sb in plan.subs]
        outs = [(gx.ptr, gx.ld, gx.c0, gx.H, gx.W, None, None, None)] * len(plan.subs)
        small = self._small(cin_l, unit.k, -unit.d, -unit.p) if unit.kind == "conv" and unit.s == 1 else None
        if cin_l < _KE[self.dt]:
            assert small is not None, "small-channel dgrad only for stride-1 convs"
        assert bnr is None or not accumulate
        return self._conv(gy, plan, unit.cin, ws, kp, rows, outs, res=gx if accumulate else None, relu=False,
                          small=small, label="dgrad", bnr=bnr)

    @staticmethod
    def _snap(a: Act):
        """copy of a gradient slice (bwd_trace): [B, H, W, C]"""
        return a.buf[..., a.c0:a.c0 + a.C].clone()

    def _dgrad_whole(self, unit, x: Act):
        """True when the dgrad launch writes every input pixel (one sub whose grid is x's pixels)."""
        plan = unit.dgrad_plan(x.H, x.W)
        if len(plan.subs) != 1 or plan.GH != x.H or plan.GW != x.W:
            return False
        sb = plan.subs[0]
        return (sb.oys, sb.oyo, sb.oxs, sb.oxo) == (1, 0, 1, 0)

    def unit_bwd(self, rec, gmap, grads, need_dx=True):
        kind, unit, x, out, res, raw, save = rec
        conv, bn = unit.conv, unit.bn
        dev = x.buf.device
        st = L.stream_ptr()
        plan = unit.fwd_plan(x.H, x.W)
        pending = {}  # this unit's gradients, handed over with the weight gradient
        # where a gradient is written: the parameter's bucket slice when the sink offers one
        # (parallel.GradBuckets.dest, gradient as bucket view), else a fresh tensor
        sink_dest = getattr(grads, "dest", None)

        def dest(p):
            v = sink_dest(p) if sink_dest is not None else None
            return torch.empty_like(p) if v is None else v
        tr = None if self.bwd_trace is None else {"kind": kind, "unit": unit, "x": x, "out": out, "res": res,
                                                   "raw": raw, "save": save}
        if kind == "head":
            gy = gmap[out]
        else:
            gout = self._grad(gmap, out)
            if kind == "bn":
                P = out.P
                parts = L.lib.zp_bn_bwd_parts(P, unit.cout)
                if out.buf.data_ptr() not in gmap.get("__bnr__", {}):
                    partials = torch.empty(2 * (parts + 1) * unit.cout, dtype=torch.float32, device=dev)
                dgamma = dest(bn.weight)
                dbeta = dest(bn.bias)
                # ReLU without a residual: the mask is recomputed from raw (mode 2), out is not read
                rm = (2 if res is None and self.bn_mask_from_raw else 1) if unit.relu else 0
                fused = gmap.get("__bnr__", {}).pop(out.buf.data_ptr(), None)
                if fused is not None:  # the consumer's dgrad launch took the reduce (_bnr_fusable)
                    assert rm == 2
                    partials, fparts = fused
                    L.call("zp_bn_bwd_totals", partials.data_ptr(), fparts, unit.cout, parts, dgamma.data_ptr(),
                           dbeta.data_ptr(), 0, st)
                else:
                    L.call("zp_bn_bwd_reduce", gout.ptr, gout.ld, gout.c0, out.ptr, out.ld, out.c0, raw.data_ptr(),
                           P, unit.cout, save.data_ptr(), rm, self.dt, partials.data_ptr(), dgamma.data_ptr(),
                           dbeta.data_ptr(), 0, st)
                graw = torch.empty_like(raw)
                gres, racc = self._grad_out(gmap, res, True) if res is not None else (None, True)
                gres_before = self._snap(gres) if tr is not None and gres is not None and racc else None
                L.call("zp_bn_bwd_apply", gout.ptr, gout.ld, gout.c0, out.ptr, out.ld, out.c0, raw.data_ptr(), P,
                       unit.cout, save.data_ptr(), partials.data_ptr(), bn.weight.data_ptr(), rm,
                       self.dt, graw.data_ptr(), None if gres is None else gres.ptr,
                       0 if gres is None else gres.ld, 0 if gres is None else gres.c0, int(racc), st)
                pending[bn.weight] = dgamma
                pending[bn.bias] = dbeta
                if tr is not None:
                    tr.update(gout=gout, graw=graw, dgamma=dgamma, dbeta=dbeta,
                              gres=None if gres is None else (gres_before, self._snap(gres)))
                if conv.bias is not None:
                    # train-mode BN removes the per-channel mean: d loss / d conv bias == 0 exactly
                    pending[conv.bias] = dest(conv.bias).zero_()
                gy = Act(graw)
            else:
                raise NotImplementedError("eval-mode backward")
        if kind == "head" and conv.bias is not None:
            partials = torch.empty(2 * (L.lib.zp_bn_bwd_parts(gy.P, gy.ld) + 1) * gy.ld, dtype=torch.float32,
                                   device=dev)
            db = torch.empty(gy.ld, dtype=torch.float32, device=dev)
            L.call("zp_bn_bwd_reduce", gy.ptr, gy.ld, 0, None, 0, 0, None, gy.P, gy.ld, None, 0, self.dt,
                   partials.data_ptr(), None, db.data_ptr(), 0, st)
            pending[conv.bias] = db[:unit.cout]
        if tr is not None and kind == "head":
            tr.update(gy=gy, dbias=pending.get(conv.bias))
        wdy = Act(gy.buf, 0, unit.cout) if kind == "head" else gy
        side = self._side_stream(dev)
        if side is None:
            dw = dest(conv.weight)
            self._wgrad(unit, x, plan, wdy, dw)
            for k, v in pending.items():  # (item by item: dict.update would bypass _ReadyDict's reporting)
                grads[k] = v
            grads[conv.weight] = dw
        else:
            # the side stream starts after everything enqueued so far (gy, dgamma / dbeta, the head
            # bias); the gradients are handed over (grads / GradBuckets.ready copies) from the side
            # stream too, so a bucket's all-reduce is ordered after its weight gradients
            side.wait_stream(torch.cuda.current_stream(dev))
            # dw is allocated on the main stream, which consumes and frees it (Adam, zero_grad):
            # the block belongs to that stream's pool, and record_stream keeps it from being
            # reused there before the side stream's wgrad has written it
            dw = dest(conv.weight)
            dw.record_stream(side)  # (a bucket slice: its storage is never freed; harmless)
            with torch.cuda.stream(side):
                self._wgrad(unit, x, plan, wdy, dw)
                for k, v in pending.items():
                    grads[k] = v
                grads[conv.weight] = dw
            gy.buf.record_stream(side)  # freed below on the main stream; reused only after the wgrad
            self._side_used = True  # x (the tape's activation) and the gradients outlive the join
        if tr is not None:
            tr["dw"] = dw
        if need_dx:
            gx, acc = self._grad_out(gmap, x, self._dgrad_whole(unit, x))
            before = self._snap(gx) if tr is not None and acc else None
            prod = None if acc else gmap.get("__bnr_prod__", {}).get(x.buf.data_ptr())
            if prod is not None:
                # x is the output of a BN + ReLU (mode 2) whose only reader is this unit: the dgrad
                # launch that writes its whole gradient also takes that BN backward's reduce
                _, praw, psave = prod
                fused = self._dgrad(unit, gy, gx, accumulate=False, bnr=(praw, psave, x.P))
                gmap.setdefault("__bnr__", {})[x.buf.data_ptr()] = fused
            else:
                self._dgrad(unit, gy, gx, accumulate=acc)
            if tr is not None:
                tr["gx"] = (before, self._snap(gx))
        if tr is not None:
            self.bwd_trace.append(tr)

    # ------------------------------------------------------------------ network
    # ------------------------------------------------------------------ batch chunks
    # Every libzp launch addresses its input and weights with 32-bit buffer offsets, so one launch's
    # input stays below 2 GiB (zp_conv2d refuses more).  The widest conv input of any network here
    # sits at half resolution with at most 384 channels (v3's [up_2 | x_128 | mask | 0] concat; the
    # main network's unfused head input has 320), so an eval forward whose batch would reach that
    # runs in equal batch chunks: crops are independent in eval mode.  Training keeps
    # one batch -- its BatchNorm statistics are over the whole batch (train_v6.py:320-321).
    _CHUNK_BYTES = (1 << 31) - 1

    def eval_batch_limit(self, H, W):
        """The largest batch one eval forward of this engine runs in a single pass at H x W."""
        per_crop = (H // 2) * (W // 2) * 384 * _ES[self.dt]
        return max(1, self._CHUNK_BYTES // per_crop)

    def _chunks(self, x, train):
        B, _, H, W = x.shape
        lim = self.eval_batch_limit(H, W)
        if train or B <= lim:
            return None
        n = -(-B // lim)
        step = -(-B // n)
        return [x[i:i + step] for i in range(0, B, step)]

    def forward(self, x, train):
        """x f32 NCHW [B, 3, H, W] -> (mask [B,1,H/2,W/2], code [B,L,H/2,W/2]) f32, tape (train)."""
        parts = self._chunks(x, train)
        if parts is not None:
            rs = [self._forward_main(c, train, first=i == 0) for i, c in enumerate(parts)]
            return torch.cat([r["mask"] for r in rs]), torch.cat([r["code"] for r in rs]), None
        r = self._forward_main(x, train)
        return r["mask"], r["code"], r["tape"]

    def forward_v3(self, x, train):
        """BinaryCodeNet_Deeplab_v3 (BinaryCodeNet_v3.py:152-169): the main network, then the
        entire-mask head ASPP_v3 on (mask logits, x_high, x_128, x_64) (aspp_v3.py:78-102)
        -> (mask, entire_mask, code, tape)."""
        parts = self._chunks(x, train)
        if parts is not None:
            outs = []
            for i, c in enumerate(parts):
                r = self._forward_main(c, train, first=i == 0)
                outs.append((r["mask"], self._aspp_v3(r), r["code"]))
            return tuple(torch.cat(t) for t in zip(*outs)) + (None,)
        r = self._forward_main(x, train)
        entire = self._aspp_v3(r)
        return r["mask"], entire, r["code"], r["tape"]

    def _forward_main(self, x, train, first=True):
        dl = self._net()
        rn, aspp = dl.resnet, dl.aspp
        if not rn.concat_decoder:
            raise NotImplementedError("concat=False: the reference forward cannot run this configuration "
                                      "(aspp.py:112 concatenates x_128=None)")
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError(f"expected input [B, 3, H, W], got {tuple(x.shape)}")
        if x.dtype != torch.float32 or not x.is_cuda:
            raise ValueError("input must be a float32 CUDA (HIP) tensor")
        x = x.contiguous()
        B, _, H, W = x.shape
        if H % 8 or W % 8:
            raise ValueError("input height / width must be multiples of 8")
        dev, dt = x.device, self.dtype
        tape = Tape() if train else None
        if self.x3 and train:
            raise RuntimeError("the split-fp32 (x3) engine runs eval forwards only")

        def new(h, w, c):
            return Act(self._empty((B, h, w, c), dev))

        if self.dt == L.ZP_F32H2:
            # the range guard (include/zp.h zp_split_range_flag): this engine's own word, registered
            # and cleared at the start of every forward, eager or captured (a captured forward
            # clears it at the start of each replay), before the weight packing, whose |w| >= 32
            # check raises it too.  Its readers -- DeepLabV3.forward after an eager forward,
            # GraphedInference after a replay -- therefore see this forward's stores only: not a
            # word left set by an unguarded run, nor another network's
            # (weights packed by a forward whose word nobody read -- an unguarded run -- keep it
            # set: their |w| >= 32 check runs only at packing time)
            flag = self.range_word(dev)
            L.register_range_flag(flag)
            # (a chunked forward clears it before its first chunk only: the word covers the batch)
            if first and (not self.unread_packs or torch.cuda.is_current_stream_capturing()):
                flag.zero_()
        self._prepack(dev)
        st = L.stream_ptr()
        self.stage = "stem"
        r = rn.resnet
        stem_unit = self._u(r[0], r[1], True, cin_act=8)
        if self.nchw_stem(stem_unit, H, W, tape):  # zp_stem_split reads the NCHW input itself (ldx 0)
            xin = NchwInput(x.permute(0, 2, 3, 1), 0, 8)
        elif self.x3:  # the stem reads f32 (exact-f32 small-Cin kernel) and writes split output
            xin = Act(torch.empty((B, H, W, 8), dtype=torch.float32, device=dev))
            L.call("zp_nchw_to_nhwc", x.data_ptr(), B, 3, H, W, 8, L.ZP_F32, xin.ptr, st)
        else:
            xin = new(H, W, 8)
            L.call("zp_nchw_to_nhwc", x.data_ptr(), B, 3, H, W, 8, self.dt, xin.ptr, st)
        if self.trace is not None and tape is None:
            self.trace.append(("input", None, x, xin, None))
        r = rn.resnet
        H2, W2 = H // 2, W // 2
        H4, W4, H8, W8 = H // 4, W // 4, H // 8, W // 8
        c64 = 64 if rn.num_layers == 34 else 256
        fuse = tape is None and rn.num_layers == 34 and self.head_fusable(B, H2, W2)
        if fuse:  # the head reads x_128 itself: no [up2 | x_128] concat buffer
            head_in = None
            x128 = Act(self._empty((B, H2, W2, 64), dev))
        else:
            head_in = self._empty((B, H2, W2, 320), dev)
            x128 = Act(head_in, 256, 64)
        self.unit_fwd(stem_unit, xin, x128, tape, label="stem")
        self.stage = "layer1"
        pooled = new(H4, W4, 64)
        L.call("zp_maxpool3s2", x128.ptr, B, H2, W2, x128.ld, x128.c0, 64, self.dt, pooled.ptr, H4, W4, 64, 0, st)
        if tape is not None:
            tape.recs.append(("maxpool", x128, pooled))
        elif self.trace is not None:
            self.trace.append(("maxpool", None, x128, pooled, None))
        up2_in = self._empty((B, H4, W4, 256 + c64), dev)
        x64 = Act(up2_in, 256, c64)
        h = self._layer(r[4], pooled, x64, tape)
        self.stage = "layer2"
        h = self._layer(r[5], h, None, tape)
        self.stage = "layer4"
        h = self._layer(rn.layer4, h, None, tape)
        self.stage = "layer5"
        xh = self._layer(rn.layer5, h, None, tape)
        # ---- ASPP (aspp.py:83-99)
        self.stage = "aspp"
        A = self._empty((B, H8, W8, 1280), dev)
        br = [self._u(aspp.conv_1x1_1, aspp.bn_conv_1x1_1), self._u(aspp.conv_3x3_1, aspp.bn_conv_3x3_1),
              self._u(aspp.conv_3x3_2, aspp.bn_conv_3x3_2), self._u(aspp.conv_3x3_3, aspp.bn_conv_3x3_3)]
        self.aspp_branches_fwd(br, xh, [Act(A, 256 * i, 256) for i in range(4)], tape)
        pool = Act(self._empty((B, 1, 1, xh.C), dev))
        L.call("zp_global_avgpool", xh.ptr, B, H8, W8, xh.ld, xh.c0, xh.C, self.dt, pool.ptr, st)
        if tape is not None:  # tape order = forward order (the backward walks it reversed)
            tape.recs.append(("avgpool", xh, pool))
        elif self.trace is not None:
            self.trace.append(("avgpool", None, xh, pool, None))
        imgo = Act(self._empty((B, 1, 1, 256), dev))
        self.unit_fwd(self._u(aspp.conv_1x1_2, aspp.bn_conv_1x1_2), pool, imgo, tape, label="aspp_pool")
        L.call("zp_broadcast_hw", imgo.ptr, B, 256, self.dt, A.data_ptr(), H8, W8, 1280, 1024, st)
        if tape is not None:
            tape.recs.append(("broadcast", imgo, Act(A, 1024, 256)))
        elif self.trace is not None:
            self.trace.append(("broadcast", None, imgo, Act(A, 1024, 256), None))
        o = new(H8, W8, 256)
        self.unit_fwd(self._u(aspp.conv_1x1_3, aspp.bn_conv_1x1_3), Act(A), o, tape, label="aspp_proj")
        # ---- decoder (aspp.py:101-112)
        self.stage = "up1"
        self._upsample(aspp.upsample_1, o, Act(up2_in, 0, 256), tape)
        self.stage = "up2"
        ncls = aspp.conv_1x1_4.out_channels
        mask = torch.empty((B, 1, H2, W2), dtype=torch.float32, device=dev)
        code = torch.empty((B, ncls - 1, H2, W2), dtype=torch.float32, device=dev)
        if fuse:
            self._upsample(aspp.upsample_2, Act(up2_in), None, tape,
                           head=(self._u(aspp.conv_1x1_4, None, False), x128, mask, code))
        else:
            self._upsample(aspp.upsample_2, Act(up2_in), Act(head_in, 0, 256), tape)
            self.stage = "head"
            self.head_fwd(self._u(aspp.conv_1x1_4, None, False), Act(head_in), mask, code, tape)
        r = {"mask": mask, "code": code, "tape": tape, "xh": xh, "x64": x64, "x128": x128}
        if tape is not None and self.bwd_trace is not None:
            self.last_fwd = r  # the traced training step's outputs and tape (teacher-forced tests)
        return r

    def _aspp_v3(self, r):
        """ASPP_v3.forward (aspp_v3.py:78-102).  The concats are channel slices of three buffers
        whose widths are padded to the MFMA K step (1025 -> 1088, 321 -> 384 channels, zero
        padding, zero weight columns): [3 branches | image pool | mask_32 | 0], [up_1 | x_64 |
        mask_64 | 0], [up_2 | x_128 | mask | 0]; x_64 / x_128 are copied in (16 / 64 KB per crop)."""
        dl = self._net()
        a3 = dl.aspp_v3
        xh, x64, x128, mask, tape = r["xh"], r["x64"], r["x128"], r["mask"], r["tape"]
        if x64.C != 64:
            raise NotImplementedError("ASPP_v3 expects the ResNet34 encoder (64-channel x_64)")
        if (x64.H, x64.W) != (64, 64):
            raise ValueError("BinaryCodeNet_Deeplab_v3 runs 256x256 inputs only: aspp_v3.py:95 resamples the mask "
                             "to a fixed 64x64 before concatenating it with x_64")
        B, H8, W8 = xh.B, xh.H, xh.W
        H4, W4, H2, W2 = x64.H, x64.W, x128.H, x128.W
        dev, dt = xh.buf.device, self.dtype
        st = L.stream_ptr()
        A = torch.zeros((B, H8, W8, 1088), dtype=dt, device=dev)
        br = [self._u(a3.conv_1x1_1, a3.bn_conv_1x1_1), self._u(a3.conv_3x3_1, a3.bn_conv_3x3_1),
              self._u(a3.conv_3x3_2, a3.bn_conv_3x3_2)]
        self.aspp_branches_fwd(br, xh, [Act(A, 256 * i, 256) for i in range(3)], tape)
        pool = Act(torch.empty((B, 1, 1, xh.C), dtype=dt, device=dev))
        L.call("zp_global_avgpool", xh.ptr, B, H8, W8, xh.ld, xh.c0, xh.C, self.dt, pool.ptr, st)
        if tape is not None:
            tape.recs.append(("avgpool", xh, pool))
        imgo = Act(torch.empty((B, 1, 1, 256), dtype=dt, device=dev))
        self.unit_fwd(self._u(a3.conv_1x1_2, a3.bn_conv_1x1_2), pool, imgo, tape, label="aspp_pool")
        L.call("zp_broadcast_hw", imgo.ptr, B, 256, self.dt, A.data_ptr(), H8, W8, 1088, 768, st)
        if tape is not None:
            tape.recs.append(("broadcast", imgo, Act(A, 768, 256)))
        self._mask_interp(mask, Act(A, 1024, 1), tape)
        o = Act(torch.empty((B, H8, W8, 256), dtype=dt, device=dev))
        self.unit_fwd(self._u(a3.conv_1x1_3, a3.bn_conv_1x1_3, cin_act=1088), Act(A), o, tape, label="aspp_proj")
        up2 = torch.zeros((B, H4, W4, 384), dtype=dt, device=dev)
        self._upsample(a3.upsample_1, o, Act(up2, 0, 256), tape)
        self._copy(x64, Act(up2, 256, 64), tape)
        self._mask_interp(mask, Act(up2, 320, 1), tape)
        hin = torch.zeros((B, H2, W2, 384), dtype=dt, device=dev)
        self._upsample(a3.upsample_2, Act(up2), Act(hin, 0, 256), tape, cin_act=384)
        self._copy(x128, Act(hin, 256, 64), tape)
        self._mask_interp(mask, Act(hin, 320, 1), tape)
        entire = torch.empty((B, 1, H2, W2), dtype=torch.float32, device=dev)
        self.head_fwd(self._u(a3.conv_1x1_4, None, False, cin_act=384), Act(hin), entire, None, tape, key="head3")
        return entire

    def _mask_interp(self, mask, dst: Act, tape):
        B, _, H, W = mask.shape
        L.call("zp_mask_interp", mask.data_ptr(), B, H, W, dst.H, dst.W, self.dt, dst.ptr, dst.ld, dst.c0,
               L.stream_ptr())
        if tape is not None:
            tape.recs.append(("interp", dst))

    def _copy(self, src: Act, dst: Act, tape):
        L.call("zp_copy_slice", src.ptr, src.ld, src.c0, self.dt, dst.ptr, dst.ld, dst.c0, self.dt, src.P, src.C, 0,
               L.stream_ptr())
        if tape is not None:
            tape.recs.append(("copy", src, dst))

    def _u(self, conv, bn=None, relu=True, cin_act=None):
        key = (id(conv), id(bn), relu, cin_act)
        cache = self.__dict__.setdefault("_units", {})
        u = cache.get(key)
        if u is None:
            u = cache[key] = Unit(conv, bn, relu, cin_act)
        return u

    def _upsample(self, seq, x: Act, out: Act, tape, cin_act=None, head=None):
        """aspp.py:60-80 (ConvT + BN + ReLU, 2 x (conv + BN + ReLU)); head = (head unit, x2, mask,
        code): the last conv feeds the fused head instead of writing ``out``."""
        h1 = self._u(seq[0], seq[1], cin_act=cin_act)
        OH, OW = h1.out_hw(x.H, x.W)
        dev = x.buf.device
        t1 = Act(self._empty((x.B, OH, OW, 256), dev))
        self.unit_fwd(h1, x, t1, tape, label="upconvT")
        t2 = Act(self._empty((x.B, OH, OW, 256), dev))
        self.unit_fwd(self._u(seq[3], seq[4]), t1, t2, tape, label="upconv")
        if head is not None:
            self.unit_fwd_head(self._u(seq[6], seq[7]), t2, head[0], head[1], head[2], head[3])
        else:
            self.unit_fwd(self._u(seq[6], seq[7]), t2, out, tape, label="upconv")

    def _layer(self, seq, x: Act, final_out: Act, tape):
        n = len(seq)
        for i, blk in enumerate(seq):
            x = self._block(blk, x, final_out if i == n - 1 else None, tape)
        return x

    def _block(self, blk, x: Act, out: Act, tape):
        dev, dt = x.buf.device, self.dtype
        if isinstance(blk, TVBottleneck):
            u1 = self._u(blk.conv1, blk.bn1)
            u2 = self._u(blk.conv2, blk.bn2)
            u3 = self._u(blk.conv3, blk.bn3)
            h1, w1 = u1.out_hw(x.H, x.W)
            t1 = Act(self._empty((x.B, h1, w1, u1.cout), dev))
            self.unit_fwd(u1, x, t1, tape, label="enc")
            h2, w2 = u2.out_hw(h1, w1)
            t2 = Act(self._empty((x.B, h2, w2, u2.cout), dev))
            self.unit_fwd(u2, t1, t2, tape, label="enc")
            last, mid = u3, t2
        else:
            u1 = self._u(blk.conv1, blk.bn1)
            h1, w1 = u1.out_hw(x.H, x.W)
            t1 = Act(self._empty((x.B, h1, w1, u1.cout), dev))
            self.unit_fwd(u1, x, t1, tape, label="enc")
            last, mid = self._u(blk.conv2, blk.bn2, True), t1
        ds = blk.downsample
        if ds is not None and len(ds) > 0:
            ud = self._u(ds[0], ds[1], False)
            hd, wd = ud.out_hw(x.H, x.W)
            res = Act(self._empty((x.B, hd, wd, ud.cout), dev))
            self.unit_fwd(ud, x, res, tape, label="enc_ds")
        else:
            res = x
        if out is None:
            oh, ow = last.out_hw(mid.H, mid.W)
            out = Act(self._empty((x.B, oh, ow, last.cout), dev))
        self.unit_fwd(last, mid, out, tape, res=res, label="enc")
        return out

    def backward(self, tape, dmask, dcode, dentire=None, grads=None):
        """Returns {parameter: gradient} for every parameter of the network.  With the v3 head
        (tape holds a "head3" record), dentire is the entire-mask logits' gradient and the mask
        resamplings add their gradient into the visible-mask head's before it runs.  ``grads`` is
        the dict the gradients are assigned into as they are enqueued (parallel.grads_sink: a
        data-parallel run starts each bucket's all-reduce from those assignments)."""
        grads = {} if grads is None else grads
        for _ in self.backward_iter(tape, dmask, dcode, dentire, grads):
            pass
        return grads

    def side_join_current(self):
        """Make the current stream wait for the weight-gradient side stream (stage boundaries of
        the staged backward, zebrapose_amd.staged)."""
        if self._side is not None and self._side_used:
            torch.cuda.current_stream(self._side.device).wait_stream(self._side)
            self._side_used = False

    def _bnr_fusable(self, tape):
        """{activation buffer: (unit, raw, save)} of the train-mode BN + ReLU outputs whose backward
        reduce can run inside the data-gradient launch of their reader (zp.h bnr_*): relu mask from
        the raw conv output (mode 2: no residual), the output is a whole buffer (no channel slice of a
        concat), and exactly one taped op reads that buffer -- a conv unit with its own BN or none,
        not the head -- so that reader's dgrad, which writes every pixel of the gradient (overwrite,
        _grad_out), is its only writer.  f32 / bf16 engines (the kernels' epilogue), ZP_BN_BWD_FUSED=0
        turns it off."""
        if not self.bn_bwd_fused or self.dt not in (L.ZP_F32, L.ZP_BF16):
            return {}
        readers = {}

        def read(act):
            if act is not None:
                k = act.buf.data_ptr()
                readers[k] = readers.get(k, 0) + 1
        kinds = {}
        for rec in tape.recs:
            kind = rec[0]
            if kind in ("plain", "bn", "head"):
                read(rec[2])
                read(rec[4])
                kinds.setdefault(rec[2].buf.data_ptr(), []).append((kind, rec[1], rec[2]))
            elif kind in ("maxpool", "broadcast", "copy", "avgpool"):
                read(rec[1])
        out = {}
        for rec in tape.recs:
            if rec[0] != "bn":
                continue
            _, unit, _x, o, res, raw, save = rec
            k = o.buf.data_ptr()
            if not unit.relu or res is not None or not self.bn_mask_from_raw or o.c0 != 0 or o.C != o.ld:
                continue
            rd = kinds.get(k)
            if readers.get(k) != 1 or not rd or rd[0][0] == "head" or not self._dgrad_whole(rd[0][1], rd[0][2]):
                continue
            out[k] = (unit, raw, save)
        return out

    def backward_iter(self, tape, dmask, dcode, dentire=None, grads=None):
        """Engine.backward as a generator: yields after each taped op's backward has been enqueued
        (the staged autograd chain of zebrapose_amd.staged advances it stage by stage)."""
        gmap = {}
        grads = {} if grads is None else grads
        self.bwd_progress = (0, len(tape.recs))  # taped ops whose backward is enqueued / all
        st = L.stream_ptr()
        head_rec = next(r for r in tape.recs if r[0] == "head" and r[3] == "head")
        hin = head_rec[2]
        B, H2, W2 = hin.B, hin.H, hin.W
        ncls = head_rec[1].cout
        dev = hin.buf.device
        if dmask is None:
            dmask = torch.zeros((B, 1, H2, W2), dtype=torch.float32, device=dev)
        if dcode is None:
            dcode = torch.zeros((B, ncls - 1, H2, W2), dtype=torch.float32, device=dev)
        dmask, dcode = dmask.contiguous().float(), dcode.contiguous().float()
        if self.bwd_trace is not None:
            self.last_head_grads = (dmask, dcode)
        ldh = 32 if ncls <= 32 else G.ceil_to(ncls, 64)
        v3 = any(r[0] == "head" and r[3] == "head3" for r in tape.recs)
        if v3:
            # the v3 head's mask inputs accumulate into a private copy of dmask
            dmask = dmask.clone()
            if dentire is None:
                dentire = torch.zeros((B, 1, H2, W2), dtype=torch.float32, device=dev)
            g3 = torch.empty((B, H2, W2, 32), dtype=self.dtype, device=dev)
            L.call("zp_head_grad_to_nhwc", dentire.contiguous().float().data_ptr(), None, B, 0, H2, W2, 32, self.dt,
                   g3.data_ptr(), st)
            gmap["head3"] = Act(g3)

        def main_head_grad():
            ghead = torch.empty((B, H2, W2, ldh), dtype=self.dtype, device=dev)
            L.call("zp_head_grad_to_nhwc", dmask.data_ptr(), dcode.data_ptr(), B, ncls - 1, H2, W2, ldh, self.dt,
                   ghead.data_ptr(), st)
            gmap["head"] = Act(ghead)

        if not v3:
            main_head_grad()
        gmap["__bnr_prod__"] = self._bnr_fusable(tape)
        for rec in reversed(tape.recs):
            kind = rec[0]
            if kind == "head" and rec[3] == "head" and v3:
                main_head_grad()  # every mask resampling of the v3 head has been differentiated
            if kind in ("plain", "bn", "head"):
                need_dx = rec[2].ld != 8  # the NHWC image input needs no gradient
                self.unit_bwd(rec, gmap, grads, need_dx=need_dx)
            elif kind == "maxpool":
                _, xa, pa = rec
                gp = self._grad(gmap, pa)
                gx = self._grad(gmap, xa)
                before = self._snap(gx) if self.bwd_trace is not None else None
                L.call("zp_maxpool3s2_bwd", xa.ptr, xa.ld, xa.c0, gp.ptr, gp.ld, gp.c0, xa.B, xa.H, xa.W, xa.C, pa.H,
                       pa.W, self.dt, gx.ptr, gx.ld, gx.c0, 1, st)
                if self.bwd_trace is not None:
                    self.bwd_trace.append({"kind": "maxpool", "x": xa, "gp": gp, "gx": (before, self._snap(gx))})
            elif kind == "broadcast":
                _, src, dst = rec
                gd = self._grad(gmap, dst)
                gs = self._grad(gmap, src)
                before = self._snap(gs) if self.bwd_trace is not None else None
                L.call("zp_sum_hw", gd.ptr, gd.B, gd.H, gd.W, gd.ld, gd.c0, gd.C, self.dt, gs.ptr, st)
                if self.bwd_trace is not None:
                    self.bwd_trace.append({"kind": "broadcast", "gd": gd, "gx": (before, self._snap(gs))})
            elif kind == "interp":
                _, dst = rec
                gd = self._grad(gmap, dst)
                L.call("zp_mask_interp_bwd", gd.ptr, gd.ld, gd.c0, B, dst.H, dst.W, H2, W2, self.dt, dmask.data_ptr(),
                       1, st)
            elif kind == "copy":
                _, src, dst = rec
                gd = self._grad(gmap, dst)
                gs = self._grad(gmap, src)
                L.call("zp_copy_slice", gd.ptr, gd.ld, gd.c0, self.dt, gs.ptr, gs.ld, gs.c0, self.dt, gd.P, gd.C, 1, st)
            elif kind == "avgpool":
                _, xa, pa = rec
                gp = self._grad(gmap, pa)
                gx = self._grad(gmap, xa)
                before = self._snap(gx) if self.bwd_trace is not None else None
                L.call("zp_add_broadcast_hw", gp.ptr, C.c_float(1.0 / (xa.H * xa.W)), xa.B, xa.C, self.dt, gx.ptr,
                       xa.H, xa.W, gx.ld, gx.c0, 1, st)
                if self.bwd_trace is not None:
                    self.bwd_trace.append({"kind": "avgpool", "gp": gp, "gx": (before, self._snap(gx))})
            self.bwd_progress = (self.bwd_progress[0] + 1, len(tape.recs))
            yield rec
        self._side_join(dev)

