"""State-dict layout of ``BinaryCodeNet_Deeplab(34|50, L, 2, concat=True, 1)`` -- TEST INFRASTRUCTURE.

The encoder reuses torchvision's ResNet34/ResNet50 children (reference
``zebrapose/model/resnet.py:183-227``).  torchvision (README pins 0.10.0) is a
third-party dependency absent from /root/reference; its published module layout
is restated here:

* ``ResNet`` children: conv1(7x7 s2 p3), bn1, relu, maxpool(3,2,1), layer1..layer4, avgpool, fc
* ``BasicBlock``: conv1(3x3, stride), bn1, relu, conv2(3x3), bn2, downsample=Sequential(conv1x1(stride), bn)
* ``Bottleneck`` (v1.5, stride on the 3x3): conv1(1x1), bn1, conv2(3x3, stride), bn2, conv3(1x1, x4), bn3, relu, downsample

``oracle/capture_fixtures.py`` checks this list against the real reference's
``state_dict()`` (key order and shapes) and commits the key list to
``tests/golden/state_keys_r{34,50}.txt``.
"""
from __future__ import annotations


def _conv(key, cout, cin, k, kind="conv"):
    return [(key + ".weight", (cout, cin, k, k), kind)]


def _bn(prefix, c):
    return [(prefix + ".weight", (c,), "bn_w"), (prefix + ".bias", (c,), "bn_b"),
            (prefix + ".running_mean", (c,), "bn_rm"), (prefix + ".running_var", (c,), "bn_rv"),
            (prefix + ".num_batches_tracked", (), "bn_nbt")]


def _tv_basic(p, cin, cout, stride):
    e = _conv(p + ".conv1", cout, cin, 3) + _bn(p + ".bn1", cout)
    e += _conv(p + ".conv2", cout, cout, 3) + _bn(p + ".bn2", cout)
    if stride != 1 or cin != cout:
        e += _conv(p + ".downsample.0", cout, cin, 1) + _bn(p + ".downsample.1", cout)
    return e


def _tv_bottleneck(p, cin, width, stride):
    cout = width * 4
    e = _conv(p + ".conv1", width, cin, 1) + _bn(p + ".bn1", width)
    e += _conv(p + ".conv2", width, width, 3) + _bn(p + ".bn2", width)
    e += _conv(p + ".conv3", cout, width, 1) + _bn(p + ".bn3", cout)
    if stride != 1 or cin != cout:
        e += _conv(p + ".downsample.0", cout, cin, 1) + _bn(p + ".downsample.1", cout)
    return e


def _tv_children(p, variant):
    """children[:-4] of torchvision resnet34/50 -> Sequential indices 0..5."""
    e = _conv(p + ".0", 64, 3, 7) + _bn(p + ".1", 64)
    if variant == 34:
        for i in range(3):
            e += _tv_basic(f"{p}.4.{i}", 64, 64, 1)
        for i in range(4):
            e += _tv_basic(f"{p}.5.{i}", 64 if i == 0 else 128, 128, 2 if i == 0 else 1)
    else:
        for i in range(3):
            e += _tv_bottleneck(f"{p}.4.{i}", 64 if i == 0 else 256, 64, 1)
        for i in range(4):
            e += _tv_bottleneck(f"{p}.5.{i}", 256 if i == 0 else 512, 128, 2 if i == 0 else 1)
    return e


def _zp_basic(p, cin, cout):
    """resnet.py:20-51 BasicBlock (registration order conv1, bn1, conv2, bn2, downsample)."""
    e = _conv(p + ".conv1", cout, cin, 3) + _bn(p + ".bn1", cout)
    e += _conv(p + ".conv2", cout, cout, 3) + _bn(p + ".bn2", cout)
    if cin != cout:
        e += _conv(p + ".downsample.0", cout, cin, 1) + _bn(p + ".downsample.1", cout)
    return e


def _upsample(p, cin, cout):
    """aspp.py:60-80 Sequential indices 0 ConvT, 1 BN, 3 conv, 4 BN, 6 conv, 7 BN."""
    e = [(p + ".0.weight", (cin, cout, 3, 3), "convT")] + _bn(p + ".1", cout)
    e += _conv(p + ".3", cout, cout, 3) + _bn(p + ".4", cout)
    e += _conv(p + ".6", cout, cout, 3) + _bn(p + ".7", cout)
    return e


def state_spec(variant: int = 34, code_bits: int = 16):
    """variant 34 | 50 (BinaryCodeNet_Deeplab) or "v3" (BinaryCodeNet_Deeplab_v3, ResNet34: the
    same keys followed by net.aspp_v3.*, aspp_v3.py:8-55)."""
    if variant == "v3":
        entries, aliases = state_spec(34, code_bits)
        a = "net.aspp_v3"

        def cb3(name, bn, cin, cout, k):
            return (_conv(f"{a}.{name}", cout, cin, k) + [(f"{a}.{name}.bias", (cout,), "bias")]
                    + _bn(f"{a}.{bn}", cout))
        entries += cb3("conv_1x1_1", "bn_conv_1x1_1", 512, 256, 1)
        entries += cb3("conv_3x3_1", "bn_conv_3x3_1", 512, 256, 3)
        entries += cb3("conv_3x3_2", "bn_conv_3x3_2", 512, 256, 3)
        entries += cb3("conv_1x1_2", "bn_conv_1x1_2", 512, 256, 1)
        entries += cb3("conv_1x1_3", "bn_conv_1x1_3", 1025, 256, 1)
        entries += _upsample(f"{a}.upsample_1", 256, 256)
        entries += _upsample(f"{a}.upsample_2", 321, 256)
        entries += _conv(f"{a}.conv_1x1_4", 1, 321, 1) + [(f"{a}.conv_1x1_4.bias", (1,), "bias")]
        return entries, aliases
    if variant not in (34, 50):
        raise ValueError("variant must be 34 or 50")
    r = "net.resnet"
    entries = _tv_children(r + ".resnet", variant)
    aliases = {}
    # resnet_layer_1 = children[:-7] (conv1,bn1,relu); _2 = children[-7:-5] (maxpool, layer1);
    # _3 = children[-5:-4] (layer2)   (resnet.py:195-199, 217-221)
    for key, shape, kind in list(entries):
        rest = key[len(r + ".resnet."):]
        idx, tail = rest.split(".", 1)
        idx = int(idx)
        if idx in (0, 1):
            ak = f"{r}.resnet_layer_1.{idx}.{tail}"
        elif idx == 4:
            ak = f"{r}.resnet_layer_2.1.{tail}"
        elif idx == 5:
            ak = f"{r}.resnet_layer_3.0.{tail}"
        else:
            continue
        aliases[ak] = key
    alias_entries = []
    lookup = {k: (s, kd) for k, s, kd in entries}
    for grp in ("resnet_layer_1", "resnet_layer_2", "resnet_layer_3"):
        for ak, ck in aliases.items():
            if ak.startswith(f"{r}.{grp}."):
                s, kd = lookup[ck]
                alias_entries.append((ak, s, kd))
    entries = entries + alias_entries
    c16, chigh = (256, 512) if variant == 34 else (1024, 2048)
    c32 = 128 if variant == 34 else 512
    c64 = 64 if variant == 34 else 256
    for i in range(6):
        entries += _zp_basic(f"{r}.layer4.{i}", c32 if i == 0 else c16, c16)
    for i in range(3):
        entries += _zp_basic(f"{r}.layer5.{i}", c16 if i == 0 else chigh, chigh)
    a = "net.aspp"
    ncls = code_bits + 1
    def cb(name, bn, cin, cout, k):
        return (_conv(f"{a}.{name}", cout, cin, k) + [(f"{a}.{name}.bias", (cout,), "bias")]
                + _bn(f"{a}.{bn}", cout))
    entries += cb("conv_1x1_1", "bn_conv_1x1_1", chigh, 256, 1)
    entries += cb("conv_3x3_1", "bn_conv_3x3_1", chigh, 256, 3)
    entries += cb("conv_3x3_2", "bn_conv_3x3_2", chigh, 256, 3)
    entries += cb("conv_3x3_3", "bn_conv_3x3_3", chigh, 256, 3)
    entries += cb("conv_1x1_2", "bn_conv_1x1_2", chigh, 256, 1)
    entries += cb("conv_1x1_3", "bn_conv_1x1_3", 1280, 256, 1)
    entries += _upsample(f"{a}.upsample_1", 256, 256)
    entries += _upsample(f"{a}.upsample_2", 256 + c64, 256)
    entries += _conv(f"{a}.conv_1x1_4", ncls, 256 + 64, 1) + [(f"{a}.conv_1x1_4.bias", (ncls,), "bias")]
    return entries, aliases
