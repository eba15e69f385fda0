"""Range guard of the two-plane split-fp32 engine at the geometry the bench runs (VERDICT r4 #1:
BASELINE.json configs[1], ResNet34 + DeepLabv3, bs=32, 256x256).  Reference anchor:
model/BinaryCodeNet.py:161-174 (plain f32 over the whole range).

At bs=32 the headline kernels are the wide two-plane tile k_conv3w (256 x 256: layer5, the
decoder's 3x3s and ConvT phases), the fused up2-conv + head launch (k_conv3w_head, whose conv output
is never stored: the overflow check runs on the values it feeds to the head) and, for layer4,
k_conv3's 128 x 256 tile.  The 64x64 tests in test_gpu_range.py never dispatch them.  Here one BN's
gamma / beta is scaled so that the FIRST launch whose stores leave fp16's range is the named wide
kernel (asserted from the engine's per-launch range probe), and the forward must
  * raise the flag, warn, fall back to the full-range x3 engine;
  * give logits within 1e-3 of the logit scale of the CPU oracle (ref_cpu.forward, f32) for crops
    0 / 13 / 31.
The same through GraphedInference, with an input-dependent overflow (the graph is captured on h2
with in-range crops, and a replay of scaled crops overflows first in a layer5 k_conv3w launch): the
replay detects it, re-captures on x3, and returns the oracle's logits in the same output tensors.
"""
import numpy as np
import pytest
import torch

from tests.test_gpu_bench_geometry import B, S, SAMPLE, bench_crops

pytestmark = pytest.mark.gpu


def _net(golden, mutate=None):
    from oracle import ref_cpu
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    sd = ref_cpu.synthetic_state(34, 16, 0, dict(golden("r34_bn_buffers256.npz")))
    if mutate is not None:
        mutate(sd)
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="fp32")
    net.load_state_dict(sd)
    net.net.f32_split = "h2"
    return net.cuda().eval(), sd


def _scale_bn(key, s):
    def f(sd):
        sd[key + ".weight"].mul_(s)
        sd[key + ".bias"].mul_(s)
    return f


def _oracle(sd, x):
    from oracle import ref_cpu
    with torch.no_grad():
        m, c = ref_cpu.forward(sd, x[list(SAMPLE)].cpu(), 34)
    return m.numpy(), c.numpy()


def _close(m, c, ref, what):
    scale = max(float(np.abs(r).max()) for r in ref)
    for g, r in ((m, ref[0]), (c, ref[1])):
        g = g.detach().cpu()[list(SAMPLE)].numpy()
        assert np.isfinite(g).all(), f"{what}: non-finite output"
        d = float(np.abs(g - r).max())
        print(f"{what}: logit scale {scale:.3g}, max |d| {d:.3g} ({d / scale:.2e} of the scale)")
        assert d <= 1e-3 * scale, (what, d, scale)


def _first_raising(net, x):
    """(stage, kernel label) of the first launch of an unguarded h2 forward after which the
    engine's range word is set (Engine.range_probe)."""
    eng = net.net.eval_engine()
    assert eng.split == "h2"
    net.net.range_check = False
    eng.range_probe = []
    try:
        with torch.no_grad():
            net(x)
        probe = [(st, k, int(f.item())) for st, k, f in eng.range_probe]
    finally:
        eng.range_probe = None
        net.net.range_check = True
        eng.unread_packs = False  # (the packs were checked here: the next forward clears the word)
    hits = [(st, k) for st, k, v in probe if v]
    assert hits, "expected the unguarded two-plane forward to raise the range word"
    print("launches before the first raise:", len(probe) - len(hits), "first raising:", hits[0])
    return hits[0]


# (BN scaled by 1e5, the stage and wide kernel whose epilogue must raise the flag first)
CASES = [
    ("layer5", "net.resnet.layer5.0.bn1", "layer5", "k_conv3w<h2>"),
    ("layer4", "net.resnet.layer4.1.bn1", "layer4", "k_conv3<h2,WC=4,NWP=4>"),
    ("up1_convT", "net.aspp.upsample_1.1", "up1", "k_conv3w<h2>"),
    ("fused_head", "net.aspp.upsample_2.7", "up2", "k_conv3w_head<h2>"),
]


@pytest.mark.parametrize("case,bn,stage,kernel", CASES, ids=[c[0] for c in CASES])
def test_bench_geometry_overflow_falls_back(golden, case, bn, stage, kernel):
    net, sd = _net(golden, _scale_bn(bn, 1e5))
    x = bench_crops().cuda()
    assert _first_raising(net, x) == (stage, kernel)
    ref = _oracle(sd, x)
    with pytest.warns(RuntimeWarning, match="fp16's range"):
        with torch.no_grad():
            m, c = net(x)
    assert net.net.range_fallbacks == 1 and net.net.eval_engine().split == "x3"
    _close(m, c, ref, f"bs=32 eager {case}")


def _scale_bn_renormalised(block, s):
    """layer5's first conv's BN (gamma, beta) x s and the next BN's running mean / var x s / s^2:
    only that conv's stored output is scaled by s; the block's output and everything after it are
    unchanged (conv2 is linear, bn2's statistics absorb the scale)."""
    def f(sd):
        sd[block + ".bn1.weight"].mul_(s)
        sd[block + ".bn1.bias"].mul_(s)
        sd[block + ".bn2.running_mean"].mul_(s)
        sd[block + ".bn2.running_var"].mul_(s * s)
    return f


def test_bench_geometry_graph_replay_overflow(golden):
    """Input-dependent overflow at replay time in a layer5 k_conv3w launch.  layer5.0.conv1's stored
    output is scaled (renormalised by the next BN) to ~40000 on the bench crops -- inside fp16's
    range -- so the graph captures and replays on h2; crops scaled by 3 push that launch (and nothing
    before it: the stages before layer5 peak ~100x lower) past 65520.  The probe confirms where the
    scaled forward first raises the word; the replay must detect it, re-capture on x3 and return the
    oracle's logits in the same output tensors."""
    from zebrapose_amd.engine import joined
    from zebrapose_amd.graphs import GraphedInference
    x = bench_crops().cuda()
    net0, _ = _net(golden)
    names = {id(m): n for n, m in net0.named_modules()}
    eng = net0.net.eval_engine()
    eng.trace = []
    with torch.no_grad():
        net0(x)
    pre = l51 = 0.0
    for kind, unit, _x, out, _r in eng.trace:
        if kind != "conv":
            continue
        n = names.get(id(unit.conv), "")
        v = float(joined(out.buf)[..., out.c0:out.c0 + out.C].abs().max())
        if n.startswith("net.resnet.") and not n.startswith("net.resnet.layer5"):
            pre = max(pre, v)
        if n == "net.resnet.layer5.0.conv1":
            l51 = v
    eng.trace = None
    del net0
    s = 40000.0 / l51
    k = 3.0
    print(f"in-range maxima: before layer5 {pre:.3g}, layer5.0.conv1 {l51:.3g}; s {s:.4g}, crop scale {k}")
    assert pre * k * 4 < 65520, pre
    net, sd = _net(golden, _scale_bn_renormalised("net.resnet.layer5.0", s))
    assert _first_raising(net, x * k) == ("layer5", "k_conv3w<h2>")
    gi = GraphedInference(net, batch=B, size=S)
    assert gi._flag is not None and net.net.eval_engine().split == "h2"
    m, c = gi(x)
    assert gi.range_fallbacks == 0 and net.net.eval_engine().split == "h2"
    _close(m, c, _oracle(sd, x), "graph h2, in range")
    with pytest.warns(RuntimeWarning, match="fp16's range"):
        m2, c2 = gi(x * k)
    assert gi.range_fallbacks == 1 and net.net.f32_split == "x3"
    assert m2 is m and c2 is c  # the static outputs keep their identity across the re-capture
    _close(m2, c2, _oracle(sd, x * k), "graph after fallback, scaled crops")
