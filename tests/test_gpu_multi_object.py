"""Batched multi-object inference (configs[4]; zebrapose_amd/multi_object.py) against the
reference's per-object loop (test_vivo.py:99-175: one net + one LUT per object, one crop at a
time), run here through the same drop-ins crop by crop: grouping crops by object, decoding the
whole batch with per-crop LUT indices and solving PnP in one launch must not change a single
bit of any crop's result."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

K = np.array([[572.4114, 0.0, 325.2611], [0.0, 573.57043, 242.04899], [0.0, 0.0, 1.0]])


def _net(seed, bn, layers=34):
    from oracle import ref_cpu
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    net = BinaryCodeNet_Deeplab(layers, 16, 2, concat=True, output_kernel_size=1)
    sd = ref_cpu.synthetic_state(layers, 16, seed, bn)
    net.load_state_dict(sd)
    return net.cuda().eval()


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_multi_object_matches_per_object_loop(gpu, golden, precision):
    from zebrapose_amd.decode import Decoder
    from zebrapose_amd.multi_object import MultiObjectPose
    from zebrapose_amd.pnp import PnP
    rng = np.random.default_rng(3)
    bn = dict(golden("r34_bn_buffers.npz"))
    nets = [_net(s, bn) for s in (0, 1, 2)]
    luts = [rng.uniform(-60, 60, (65536, 3)) for _ in nets]
    luts[1][::97] = np.nan
    mo = MultiObjectPose(nets, luts, precision=precision)
    B = 7
    obj = np.array([2, 0, 2, 1, 0, 2, 1])
    x = torch.from_numpy(rng.normal(0, 1, (B, 3, 128, 128)).astype(np.float32)).cuda()
    bb = np.stack([rng.integers(-20, 300, B), rng.integers(-20, 200, B), rng.integers(64, 300, B),
                   rng.integers(64, 300, B)], 1)
    Ks = np.broadcast_to(K, (B, 3, 3)).copy()
    Ks[:, 0, 2] += np.arange(B)
    out = mo(x, obj, bb, Ks)
    torch.cuda.synchronize()
    assert out["mask"].shape == (B, 1, 64, 64) and out["code"].shape == (B, 16, 64, 64)
    for b in range(B):
        net = nets[obj[b]]
        m, c = net(x[b:b + 1])
        assert torch.equal(m, out["mask"][b:b + 1]) and torch.equal(c, out["code"][b:b + 1]), b
        dec = Decoder(luts[obj[b]])
        counts, xy, xyz = dec(m, c, bb[b:b + 1], bbox_size=128)
        n = int(counts[0])
        assert n == int(out["counts"][b])
        assert torch.equal(xy[0, :n], out["xy"][b, :n]) and torch.equal(xyz[0, :n], out["xyz"][b, :n])
        R, t, ok, inl = PnP()(counts, xy, xyz, Ks[b])
        assert bool(ok[0]) == bool(out["success"][b])
        if bool(ok[0]):
            assert torch.equal(R[0], out["R"][b]) and torch.equal(t[0], out["t"][b])
            assert int(inl[0]) == int(out["inliers"][b])


def test_multi_object_rejects_bad_index(gpu, golden):
    from zebrapose_amd.multi_object import MultiObjectPose
    nets = [_net(0, dict(golden("r34_bn_buffers.npz")))]
    mo = MultiObjectPose(nets, [np.zeros((65536, 3))])
    x = torch.zeros(2, 3, 64, 64, device="cuda")
    with pytest.raises(ValueError):
        mo(x, [0, 1], np.zeros((2, 4), int))
