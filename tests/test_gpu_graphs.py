"""hipGraph-captured inference (zebrapose_amd.graphs.GraphedInference): a replay must give
bit-identical mask / code logits and decoded correspondences to the eager path, for several
inputs through the same captured graph, at bs=1 (the reference's test.py:190, 248 loop) and bs=4."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def net(golden):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import ref_cpu
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    n = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="bf16")
    n.load_state_dict(ref_cpu.synthetic_state(34, 16, 0, dict(golden("r34_bn_buffers256.npz"))))
    return n.cuda().eval()


@pytest.mark.parametrize("B", [1, 4])
def test_graph_replay_matches_eager(net, B):
    from zebrapose_amd.decode import Decoder
    from zebrapose_amd.graphs import GraphedInference
    rng = np.random.default_rng(B)
    lut = rng.standard_normal((65536, 3)) * 50
    dec = Decoder(lut, device="cuda")
    g = GraphedInference(net, B, 256, decoder=dec, bbox_size=128)
    for seed in (1, 2, 3):
        x = torch.randn(B, 3, 256, 256, generator=torch.Generator().manual_seed(seed)).cuda()
        side = rng.integers(64, 401, B)
        bb = np.stack([rng.integers(0, 300, B), rng.integers(0, 200, B), side, side], 1)
        with torch.no_grad():
            m, c = net(x)
            counts, xy, xyz = dec(m, c, bb, bbox_size=128)
        gm, gc, gcounts, gxy, gxyz = g(x, bb)
        torch.cuda.synchronize()
        assert torch.equal(gm, m) and torch.equal(gc, c), seed
        assert torch.equal(gcounts, counts), seed
        for b in range(B):
            n = int(counts[b])
            assert torch.equal(gxy[b, :n], xy[b, :n]) and torch.equal(gxyz[b, :n], xyz[b, :n])


def test_graph_rejects_training_mode_and_bad_shapes(net):
    from zebrapose_amd.graphs import GraphedInference
    net.train()
    try:
        with pytest.raises(ValueError):
            GraphedInference(net, 1, 256)
    finally:
        net.eval()
    g = GraphedInference(net, 1, 256)
    with pytest.raises(ValueError):
        g(torch.zeros(2, 3, 256, 256, device="cuda"))
