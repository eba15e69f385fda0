"""Capture golden vectors from the REAL reference code -- TEST INFRASTRUCTURE ONLY.

Run in the build container (where /root/reference exists):

    PYTHONDONTWRITEBYTECODE=1 python -B -m oracle.capture_fixtures [--only=fwd256,gt,add] [--r50] [--v3]

It imports ``/root/reference/zebrapose`` read-only through a small import shim
(SURVEY §8c): the reference's only missing imports are torchvision (its ResNet
module layout is restated in ``oracle/tv_layout.py`` / ``_tv_resnet`` below: the
reference reuses torchvision's children, resnet.py:183-221), cv2 (used only by PnP,
CNN_output_to_pose.py:155-158, never reached here) and the pretrained backbone
file (resnet.py:187-189, absent; every weight is overwritten by the synthetic
checkpoint anyway).  Outputs go to ``tests/golden/``; nothing is written under
/root/reference.
"""
from __future__ import annotations

import os
import sys
import types
import copy

sys.dont_write_bytecode = True

import numpy as np
import torch
import torch.nn as nn

REF = "/root/reference/zebrapose"
HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(os.path.dirname(HERE), "tests", "golden")
sys.path.insert(0, os.path.dirname(HERE))

from oracle import ref_cpu, tv_layout  # noqa: E402


# ----------------------------------------------------------------------------- shim
class _TVBasic(nn.Module):
    expansion = 1

    def __init__(self, cin, cout, stride):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        o = self.relu(self.bn1(self.conv1(x)))
        o = self.bn2(self.conv2(o))
        idn = x if self.downsample is None else self.downsample(x)
        return self.relu(o + idn)


class _TVBottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride):
        super().__init__()
        cout = width * 4
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        o = self.relu(self.bn1(self.conv1(x)))
        o = self.relu(self.bn2(self.conv2(o)))
        o = self.bn3(self.conv3(o))
        idn = x if self.downsample is None else self.downsample(x)
        return self.relu(o + idn)


class _TVResNet(nn.Module):
    def __init__(self, variant):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        if variant == 34:
            mk = lambda cin, cout, n, s: nn.Sequential(*[_TVBasic(cin if i == 0 else cout, cout, s if i == 0 else 1) for i in range(n)])
            self.layer1, self.layer2 = mk(64, 64, 3, 1), mk(64, 128, 4, 2)
            self.layer3, self.layer4 = mk(128, 256, 6, 2), mk(256, 512, 3, 2)
            nfc = 512
        else:
            mk = lambda cin, w, n, s: nn.Sequential(*[_TVBottleneck(cin if i == 0 else w * 4, w, s if i == 0 else 1) for i in range(n)])
            self.layer1, self.layer2 = mk(64, 64, 3, 1), mk(256, 128, 4, 2)
            self.layer3, self.layer4 = mk(512, 256, 6, 2), mk(1024, 512, 3, 2)
            nfc = 2048
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(nfc, 1000)


def install_shim():
    tv = types.ModuleType("torchvision")
    tvm = types.ModuleType("torchvision.models")
    tvm.resnet34 = lambda *a, **k: _TVResNet(34)
    tvm.resnet50 = lambda *a, **k: _TVResNet(50)
    tvm.resnet18 = None
    tv.models = tvm
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.models"] = tvm
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    real_load = torch.load

    def fake_load(f, *a, **k):
        if isinstance(f, str) and "pretrained_backbone" in f:
            return _TVResNet(50 if "resnet50" in f else 34).state_dict()
        return real_load(f, *a, **k)

    torch.load = fake_load
    if REF not in sys.path:
        sys.path.insert(0, REF)


def build_reference(variant):
    from model.BinaryCodeNet import BinaryCodeNet_Deeplab
    import contextlib, io
    with contextlib.redirect_stdout(io.StringIO()):
        return BinaryCodeNet_Deeplab(num_resnet_layers=variant, concat=True, binary_code_length=16,
                                     divided_number_each_iteration=2, output_kernel_size=1)


def check_layout(net, variant):
    sd = net.state_dict()
    entries, aliases = tv_layout.state_spec(variant, 16)
    got = [(k, tuple(v.shape)) for k, v in sd.items()]
    want = [(k, tuple(s)) for k, s, _ in entries]
    assert got == want, "state-dict layout mismatch"
    for ak, ck in aliases.items():
        assert sd[ak].data_ptr() == sd[ck].data_ptr(), ak
    with open(os.path.join(GOLDEN, f"state_keys_r{variant}.txt"), "w") as f:
        for k, s in got:
            f.write(f"{k} {list(s)}\n")
    nparam = sum(p.numel() for p in net.parameters())
    print(f"r{variant}: {len(got)} keys, {len(aliases)} aliases, {nparam} params")
    return nparam


def calibrate_bn(net, x):
    """BN running stats := batch statistics of one train-mode pass (momentum=None)."""
    bns = [m for m in net.modules() if isinstance(m, nn.BatchNorm2d)]
    for m in bns:
        m.momentum = None
        m.reset_running_stats()
    net.train()
    with torch.no_grad():
        net(x)
    for m in bns:
        m.momentum = 0.1
    net.eval()


def canonical_bn_buffers(net, variant):
    entries, aliases = tv_layout.state_spec(variant, 16)
    sd = net.state_dict()
    return {k: sd[k].numpy().copy() for k, _, kind in entries
            if kind in ("bn_rm", "bn_rv", "bn_nbt") and k not in aliases}


def seeded(shape, seed, kind="normal"):
    g = np.random.default_rng(seed)
    if kind == "normal":
        return torch.from_numpy(g.standard_normal(shape).astype(np.float32))
    raise ValueError(kind)


def capture_network(variant=34):
    net = build_reference(variant)
    check_layout(net, variant)
    sd = ref_cpu.synthetic_state(variant, 16, seed=0)
    net.load_state_dict(sd)
    calibrate_bn(net, seeded((4, 3, 64, 64), 1))
    bnbuf = canonical_bn_buffers(net, variant)
    np.savez(os.path.join(GOLDEN, f"r{variant}_bn_buffers.npz"), **bnbuf)
    out = {}
    with torch.no_grad():
        x = seeded((2, 3, 64, 64), 0)
        m, c = net(x)
        out["fwd64_x"], out["fwd64_mask"], out["fwd64_code"] = x.numpy(), m.numpy(), c.numpy()
    np.savez(os.path.join(GOLDEN, f"r{variant}_fwd64.npz"), **out)
    # the oracle must agree with the reference it restates
    sd2 = ref_cpu.synthetic_state(variant, 16, seed=0, bn_buffers=bnbuf)
    with torch.no_grad():
        om, oc = ref_cpu.forward(sd2, torch.from_numpy(out["fwd64_x"]), variant)
    print(f"r{variant} fwd64 oracle vs reference: mask {np.abs(om.numpy() - out['fwd64_mask']).max():.3g}"
          f" code {np.abs(oc.numpy() - out['fwd64_code']).max():.3g}"
          f" |logit| max {np.abs(out['fwd64_code']).max():.3g}")
    return net, bnbuf


def capture_train_step(net):
    """One train_v6.py:319-338 step (loss part + backward) and a second loss call (EMA)."""
    from model.BinaryCodeNet import BinaryCodeLoss, MaskLoss
    from common_ops import from_output_to_class_mask
    net = copy.deepcopy(net)
    net.train()
    g = np.random.default_rng(7)
    x = seeded((2, 3, 64, 64), 3)
    gt_code = torch.from_numpy((g.random((2, 16, 32, 32)) < 0.5).astype(np.float64))
    gt_mask = torch.from_numpy((g.random((2, 32, 32)) < 0.7).astype(np.float32))
    gt_code2 = torch.from_numpy((g.random((2, 16, 32, 32)) < 0.5).astype(np.float64))
    bcl = BinaryCodeLoss("BCE", True, 2, use_histgramm_weighted_binary_loss=True)
    ml = MaskLoss()
    net.zero_grad()
    pm, pc = net(x)
    mask01 = torch.tensor(from_output_to_class_mask(pm))
    loss_b = bcl(pc, mask01, gt_code)
    loss_m = ml(pm, gt_mask)
    loss = 3 * loss_b + loss_m
    loss.backward()
    hist1 = bcl.histogram.detach().numpy().copy()
    with torch.no_grad():
        loss_b2 = bcl(pc.detach(), mask01, gt_code2)
    grads = {}
    keys = ["net.aspp.conv_1x1_4.weight", "net.aspp.conv_1x1_4.bias", "net.resnet.layer5.2.conv2.weight",
            "net.aspp.upsample_2.0.weight", "net.resnet.resnet.0.weight", "net.aspp.bn_conv_1x1_3.weight",
            "net.resnet.layer4.0.downsample.0.weight"]
    named = dict(net.named_parameters())
    for k in keys:
        g_ = named[k].grad.numpy()
        grads["grad:" + k] = g_[:8].copy()          # leading slice (full tensors are too big to commit)
        grads["gradsum:" + k] = np.array([g_.astype(np.float64).sum(), (g_.astype(np.float64) ** 2).sum()])
    sd = net.state_dict()
    after = {"after:" + k: sd[k].numpy().copy() for k in
             ["net.resnet.resnet.1.running_mean", "net.resnet.resnet.1.running_var",
              "net.aspp.upsample_2.7.running_var", "net.resnet.layer5.2.bn2.running_mean"]}
    np.savez(os.path.join(GOLDEN, "r34_train_step.npz"), x=x.numpy(), gt_code=gt_code.numpy(),
             gt_mask=gt_mask.numpy(), gt_code2=gt_code2.numpy(), mask_logits=pm.detach().numpy(),
             code_logits=pc.detach().numpy(), mask01=mask01.numpy(), loss_b=loss_b.detach().numpy(),
             loss_m=loss_m.detach().numpy(), loss=loss.detach().numpy(), hist1=hist1,
             hist2=bcl.histogram.numpy(), loss_b2=loss_b2.numpy(), **grads, **after)
    print("train step: loss_b", float(loss_b), "loss_m", float(loss_m), "dtype", loss_b.dtype)


def planted_logits(rng, shape):
    v = rng.standard_normal(shape).astype(np.float32) * 3
    special = np.array([0.0, 1e-8, -1e-8, 8.940696716308594e-08, 8.94069742685133e-08, -8.94069742685133e-08,
                        1.1920929e-07, 5.9604645e-08, 1.0e-7, np.nan, np.inf, -np.inf, 30.0, -30.0, 1e-45],
                       dtype=np.float32)
    flat = v.reshape(-1)
    idx = rng.choice(flat.size, size=flat.size // 16, replace=False)
    flat[idx] = special[rng.integers(0, special.size, idx.size)]
    return v


def capture_decode():
    from common_ops import from_output_to_class_mask, from_output_to_class_binary_code
    from binary_code_helper.class_id_encoder_decoder import class_code_images_to_class_id_image
    from binary_code_helper.CNN_output_to_pose import (load_dict_class_id_3D_points,
                                                       build_non_unique_2D_3D_correspondence,
                                                       mapping_pixel_position_to_original_position)
    from binary_code_helper.generate_new_dict import generate_new_corres_dict
    rng = np.random.default_rng(11)
    B, H, W = 2, 128, 128
    mask_logits = planted_logits(rng, (B, 1, H, W))
    mask_logits[0, 0, :40] = -5.0     # ragged: a band of background rows
    mask_logits[1] -= 2.0             # second crop sparser
    code_logits = planted_logits(rng, (B, 16, H, W))
    lut = rng.standard_normal((65536, 3)) * 50.0
    lut[::97] = np.nan
    lut[5::1031, 1] = np.nan
    # LUT text file in the generator's format (Generate_Mesh_with_GT_Color.cpp:616-624)
    path = "/tmp/zp_lut_capture.txt"
    with open(path, "w") as f:
        f.write("65536 2 16\n")
        for i in range(65536):
            f.write(f"{i} {float(lut[i,0])!r} {float(lut[i,1])!r} {float(lut[i,2])!r}\n")
    _, _, _, lut_dict = load_dict_class_id_3D_points(path)
    lut_loaded = np.stack([lut_dict[float(i)] for i in range(65536)])
    assert np.array_equal(np.isnan(lut_loaded), np.isnan(lut))
    bboxes = np.array([[-37, 12, 203, 203], [301, -9, 77, 77]], dtype=np.int64)
    masks = from_output_to_class_mask(torch.from_numpy(mask_logits))
    codes = from_output_to_class_binary_code(torch.from_numpy(code_logits), "BCE")
    out = dict(mask_logits=mask_logits, code_logits=code_logits, lut=lut_loaded, bboxes=bboxes,
               mask_bits=masks.astype(np.uint8), code_bits=codes.astype(np.uint8))
    for ignore_bit in (0, 2):
        d = lut_dict if ignore_bit == 0 else generate_new_corres_dict(lut_dict, 16, 16 - ignore_bit)
        if ignore_bit:
            out[f"lut_ib{ignore_bit}"] = np.stack([np.asarray(d[i]).reshape(3) for i in range(2 ** (16 - ignore_bit))])
        pm = masks.transpose(0, 2, 3, 1).squeeze(-1).astype("uint8")
        pc = codes.transpose(0, 2, 3, 1)
        for b in range(B):
            bits = pc[b] if ignore_bit == 0 else pc[b][:, :, :-ignore_bit]
            ids = class_code_images_to_class_id_image(bits, 2)
            p2 = pm[b].nonzero()
            P2D, P3D = build_non_unique_2D_3D_correspondence(p2, ids, d)
            O2D = mapping_pixel_position_to_original_position(P2D, bboxes[b], 128)
            out[f"ib{ignore_bit}_b{b}_ids"] = ids.astype(np.int64)
            out[f"ib{ignore_bit}_b{b}_p2d"] = O2D.astype(np.int64)
            out[f"ib{ignore_bit}_b{b}_p3d"] = P3D.astype(np.float32)
            out[f"ib{ignore_bit}_b{b}_count"] = np.int64(len(O2D))
    np.savez_compressed(os.path.join(GOLDEN, "decode.npz"), **out)
    # boundary table of the CPU sigmoid threshold
    probe = np.array([8.940696716308594e-08, 8.94069742685133e-08], np.float32)
    print("threshold probe", from_output_to_class_mask(torch.from_numpy(probe)))
    print("decode counts", [int(out[f"ib0_b{b}_count"]) for b in range(B)])


def capture_v3():
    """BinaryCodeNet_Deeplab_v3: layout, 256x256 forward (3 heads) and one
    train_v5.py:321-334 step (3 * loss_b + loss_mask + loss_entire_mask, backward).  The reference
    resamples the mask to a fixed 64x64 (aspp_v3.py:95), so only 256x256 inputs run."""
    from model.BinaryCodeNet_v3 import BinaryCodeNet_Deeplab_v3, BinaryCodeLoss, MaskLoss
    from common_ops import from_output_to_class_mask
    import contextlib, io
    with contextlib.redirect_stdout(io.StringIO()):
        net = BinaryCodeNet_Deeplab_v3(num_resnet_layers=34, concat=True, binary_code_length=16,
                                       divided_number_each_iteration=2, output_kernel_size=1)
    entries, aliases = tv_layout.state_spec("v3", 16)
    got = [(k, tuple(v.shape)) for k, v in net.state_dict().items()]
    assert got == [(k, tuple(sh)) for k, sh, _ in entries], "v3 state-dict layout mismatch"
    with open(os.path.join(GOLDEN, "state_keys_r34v3.txt"), "w") as f:
        for k, sh in got:
            f.write(f"{k} {list(sh)}\n")
    net.load_state_dict(ref_cpu.synthetic_state("v3", 16, seed=0))
    calibrate_bn(net, seeded((2, 3, 256, 256), 1))
    bnbuf = {k: net.state_dict()[k].numpy().copy() for k, _, kind in entries
             if kind in ("bn_rm", "bn_rv", "bn_nbt") and k not in aliases}
    np.savez(os.path.join(GOLDEN, "r34v3_bn_buffers.npz"), **bnbuf)
    x = seeded((1, 3, 256, 256), 0)
    with torch.no_grad():
        m, e, c = net(x)
    np.savez(os.path.join(GOLDEN, "r34v3_fwd256.npz"), x=x.numpy(), mask=m.numpy(), entire=e.numpy(), code=c.numpy())
    sd2 = ref_cpu.synthetic_state("v3", 16, seed=0, bn_buffers=bnbuf)
    with torch.no_grad():
        om, oe, oc = ref_cpu.forward_v3(sd2, x)
    print(f"v3 fwd256 oracle vs reference: mask {np.abs(om.numpy() - m.numpy()).max():.3g} entire "
          f"{np.abs(oe.numpy() - e.numpy()).max():.3g} code {np.abs(oc.numpy() - c.numpy()).max():.3g}")
    # one training step
    net.train()
    g = np.random.default_rng(17)
    xt = seeded((2, 3, 256, 256), 5)
    gt_code = torch.from_numpy((g.random((2, 16, 128, 128)) < 0.5).astype(np.float64))
    gt_mask = torch.from_numpy((g.random((2, 128, 128)) < 0.7).astype(np.float32))
    gt_entire = torch.from_numpy((g.random((2, 128, 128)) < 0.8).astype(np.float32))
    bcl = BinaryCodeLoss("BCE", True, 2, use_histgramm_weighted_binary_loss=True)
    ml = MaskLoss()
    net.zero_grad()
    pm, pe, pc = net(xt)
    mask01 = torch.tensor(from_output_to_class_mask(pm))
    loss_b = bcl(pc, mask01, gt_code)
    loss_m = ml(pm, gt_mask)
    loss_e = ml(pe, gt_entire)
    loss = 3 * loss_b + loss_m + loss_e
    loss.backward()
    keys = ["net.aspp_v3.conv_1x1_4.weight", "net.aspp_v3.conv_1x1_4.bias", "net.aspp_v3.conv_1x1_3.weight",
            "net.aspp_v3.upsample_2.0.weight", "net.aspp_v3.bn_conv_1x1_1.weight", "net.aspp.conv_1x1_4.weight",
            "net.aspp.upsample_2.3.weight", "net.resnet.layer5.2.conv2.weight", "net.resnet.resnet.0.weight"]
    named = dict(net.named_parameters())
    grads = {}
    for k in keys:
        g_ = named[k].grad.numpy()
        grads["grad:" + k] = g_[:8].copy()
        grads["gradsum:" + k] = np.array([g_.astype(np.float64).sum(), (g_.astype(np.float64) ** 2).sum()])
    np.savez_compressed(os.path.join(GOLDEN, "r34v3_train_step.npz"), x=xt.numpy(),
             gt_code=gt_code.numpy().astype(np.uint8), gt_mask=gt_mask.numpy().astype(np.uint8),
             gt_entire=gt_entire.numpy().astype(np.uint8), mask_logits=pm.detach().numpy(),
             entire_logits=pe.detach().numpy(), loss_b=loss_b.detach().numpy(),
             loss_m=loss_m.detach().numpy(), loss_e=loss_e.detach().numpy(), loss=loss.detach().numpy(), **grads)
    print("v3 train step: loss", float(loss), "loss_e", float(loss_e))


def capture_fwd256():
    """The bench geometry's parity anchor (configs[1]: 256x256 crops): the R34 net with the
    synthetic weights, BN running stats calibrated on four 256x256 crops (so the logits sit in the
    range a trained model's do, not the 64x64-calibrated fixture's 300), forward of two other
    256x256 crops (model/BinaryCodeNet.py:161-174)."""
    net = build_reference(34)
    net.load_state_dict(ref_cpu.synthetic_state(34, 16, seed=0))
    calibrate_bn(net, seeded((4, 3, 256, 256), 21))
    bnbuf = canonical_bn_buffers(net, 34)
    np.savez(os.path.join(GOLDEN, "r34_bn_buffers256.npz"), **bnbuf)
    x = seeded((2, 3, 256, 256), 22)
    with torch.no_grad():
        m, c = net(x)
    np.savez_compressed(os.path.join(GOLDEN, "r34_fwd256.npz"), x=x.numpy(), mask=m.numpy(), code=c.numpy())
    sd2 = ref_cpu.synthetic_state(34, 16, seed=0, bn_buffers=bnbuf)
    with torch.no_grad():
        om, oc = ref_cpu.forward(sd2, x, 34)
    print(f"r34 fwd256 (256-calibrated BN): |logit| max {np.abs(c.numpy()).max():.3g}; oracle vs reference: "
          f"mask {np.abs(om.numpy() - m.numpy()).max():.3g} code {np.abs(oc.numpy() - c.numpy()).max():.3g}")


def capture_r50_256(seeds=(0, 1, 2)):
    """configs[4]'s network at its own geometry (R50 + ASPP_50, 256x256 crops, one network per
    object as test_vivo.py:99-114 builds them): per object seed, the synthetic weights with BN
    running stats calibrated on four 256x256 crops by the reference itself (r50_bn256_s<seed>.npz);
    for seed 0 also the reference's forward of two other 256x256 crops (r50_fwd256.npz) -- the
    anchor that pins ref_cpu.forward(.., 50) at 256x256 for tests/test_gpu_multi_object.py."""
    for seed in seeds:
        net = build_reference(50)
        net.load_state_dict(ref_cpu.synthetic_state(50, 16, seed=seed))
        calibrate_bn(net, seeded((4, 3, 256, 256), 51 + seed))
        bnbuf = canonical_bn_buffers(net, 50)
        np.savez_compressed(os.path.join(GOLDEN, f"r50_bn256_s{seed}.npz"), **bnbuf)
        if seed != 0:
            continue
        x = seeded((2, 3, 256, 256), 52)
        with torch.no_grad():
            m, c = net(x)
        np.savez_compressed(os.path.join(GOLDEN, "r50_fwd256.npz"), x=x.numpy(), mask=m.numpy(), code=c.numpy())
        sd2 = ref_cpu.synthetic_state(50, 16, seed=0, bn_buffers=bnbuf)
        with torch.no_grad():
            om, oc = ref_cpu.forward(sd2, x, 50)
        print(f"r50 fwd256 (256-calibrated BN): |logit| max {np.abs(c.numpy()).max():.3g}; oracle vs reference: "
              f"mask {np.abs(om.numpy() - m.numpy()).max():.3g} code {np.abs(oc.numpy() - c.numpy()).max():.3g}")


def capture_gt_codes():
    """GT code planes: the reference's RGB_image_to_class_id_image +
    class_id_image_to_class_code_images (class_id_encoder_decoder.py:6-15, 43-63) on BGR GT crops
    as bop_dataset_pytorch.py:311-312 calls them (base 2, 16 iterations, 65536 classes), then the
    transform_pre permute to CHW (:345).  Random colours plus planted extremes (0, 255, ids above
    2^16 whose high byte must be ignored)."""
    from binary_code_helper.class_id_encoder_decoder import (RGB_image_to_class_id_image,
                                                             class_id_image_to_class_code_images)
    rng = np.random.default_rng(31)
    gt = rng.integers(0, 256, (3, 128, 128, 3), dtype=np.uint8)
    gt[1, :16] = 0
    gt[1, 16:32] = 255
    gt[2, :, :, 0] = rng.integers(1, 256, (128, 128), dtype=np.uint8)  # B != 0: id >= 2^16
    codes = []
    for b in range(gt.shape[0]):
        cid = RGB_image_to_class_id_image(gt[b])
        cc = class_id_image_to_class_code_images(cid, 2, 16, 65536)
        codes.append(torch.from_numpy(cc).permute(2, 0, 1).numpy())
    codes = np.stack(codes)
    assert set(np.unique(codes)) <= {0.0, 1.0}
    np.savez_compressed(os.path.join(GOLDEN, "gt_codes.npz"), gt_bgr=gt, code=codes.astype(np.uint8),
                        code_dtype=np.array(str(codes.dtype)))
    print("gt codes:", codes.shape, codes.dtype)


def _import_pose_error():
    """lib/pysixd/pose_error.py imports lib.utils.logger (needs termcolor, absent) and
    lib.pysixd.misc / visibility (need cv2 and mmcv, absent).  add / adi use only numpy, scipy and
    the module's own transform_pts_Rt, so those imports are stubbed with empty modules."""
    tc = types.ModuleType("termcolor")
    tc.colored = lambda s, *a, **k: s
    sys.modules.setdefault("termcolor", tc)
    import lib.pysixd as P
    for n in ("misc", "visibility"):
        if "lib.pysixd." + n not in sys.modules:
            m = types.ModuleType("lib.pysixd." + n)
            sys.modules["lib.pysixd." + n] = m
            setattr(P, n, m)
    from lib.pysixd import pose_error
    return pose_error


def _rot(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def capture_add_adi():
    """ADD / ADI: the reference's lib/pysixd/pose_error.add / adi (:297-336)
    on model points and pose pairs (identical, small and large errors, a symmetric flip)."""
    pose_error = _import_pose_error()
    rng = np.random.default_rng(41)
    pts = rng.uniform(-60, 60, (2000, 3)).astype(np.float32)
    n = 6
    Rg = np.stack([_rot(rng) for _ in range(n)])
    tg = rng.uniform(-50, 50, (n, 3)) + np.array([0, 0, 800])
    Re = Rg.copy()
    te = tg.copy()
    Re[1] = Rg[1] @ _rot(np.random.default_rng(5)) * 1.0
    te[2] = tg[2] + rng.normal(0, 5, 3)
    Re[3] = Rg[3] @ np.diag([-1.0, -1.0, 1.0])  # 180 deg about z
    Re[4] = _rot(rng)
    te[4] = tg[4] + rng.normal(0, 40, 3)
    te[5] = tg[5] + np.array([0, 0, 1e-3])
    add = np.array([pose_error.add(Re[b], te[b].reshape(3, 1), Rg[b], tg[b].reshape(3, 1), pts) for b in range(n)])
    adi = np.array([pose_error.adi(Re[b], te[b].reshape(3, 1), Rg[b], tg[b].reshape(3, 1), pts) for b in range(n)])
    np.savez(os.path.join(GOLDEN, "add_adi.npz"), pts=pts, R_est=Re, t_est=te, R_gt=Rg, t_gt=tg, add=add, adi=adi)
    print("add", add, "adi", adi)


def main():
    os.makedirs(GOLDEN, exist_ok=True)
    install_shim()
    torch.manual_seed(0)
    torch.set_num_threads(8)
    only = None
    for a in sys.argv[1:]:
        if a.startswith("--only="):
            only = set(a[7:].split(","))
    if only is None:
        net, _ = capture_network(34)
        capture_train_step(net)
        capture_decode()
    if only is None or "fwd256" in only:
        capture_fwd256()
    if only is None or "gt" in only:
        capture_gt_codes()
    if only is None or "add" in only:
        capture_add_adi()
    if "--r50" in sys.argv:
        capture_network(50)
    if only is not None and "r50_256" in only:
        capture_r50_256()
    if "--v3" in sys.argv:
        capture_v3()


if __name__ == "__main__":
    main()
