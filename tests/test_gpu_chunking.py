"""Eval batches past one launch's 2 GiB input.  Every libzp launch addresses its
input with 32-bit buffer offsets (zp_conv2d refuses an input of 2 GiB or more); the reference runs
whatever batch the config gives (train_v6.py:320-321; test.py's loader).  An eval forward whose
widest conv input would reach that runs in equal batch chunks (Engine.eval_batch_limit): fp32 at
bs=128, 256x256 is two chunks of 64 on the two-plane engine and three of <= 56 after an x3 (range)
fallback.  Crops are independent in eval mode, so every sampled crop's logits must equal the same
crop's logits from a bs=32 forward: bit for bit on x3 (the dispatch at bs = 43 picks the same tiles
as at bs = 32), and up to the f32 rounding of a different tile choice on h2 (at bs = 64 layer4 and
conv_1x1_3 fill 256 workgroups of the wide 256 x 256 tile, which flushes its correction sums per K
step where k_conv3's 128 x 256 tile flushes per half tile: observed 1e-6 of the logit scale, bound
4e-6).  The only cross-chunk state is the range word, which the chunks share."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _crops(n, seed=5):
    g = torch.Generator(device="cpu").manual_seed(seed)
    u8 = torch.randint(0, 256, (n, 3, 256, 256), generator=g, dtype=torch.uint8)
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    return (u8.float() / 255.0 - mean) / std


@pytest.mark.parametrize("split,nchunks", [("h2", 2), ("x3", 3)])
def test_bs128_fp32_runs_in_chunks(golden, split, nchunks):
    from oracle import ref_cpu
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    sd = ref_cpu.synthetic_state(34, 16, 0, dict(golden("r34_bn_buffers256.npz")))
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="fp32")
    net.load_state_dict(sd)
    net = net.cuda().eval()
    net.net.f32_split = split
    eng = net.net.eval_engine()
    lim = eng.eval_batch_limit(256, 256)
    assert -(-128 // lim) == nchunks, lim
    x = _crops(128).cuda()
    with torch.no_grad():
        m, c = net(x)
    torch.cuda.synchronize()
    assert m.shape == (128, 1, 128, 128) and c.shape == (128, 16, 128, 128)
    assert net.net.range_fallbacks == 0 and net.net.eval_engine().split == split
    for b0 in (0, 32, 96):  # crops 0..31, 32..63 (across the h2 chunk border at 64), 96..127
        with torch.no_grad():
            m32, c32 = net(x[b0:b0 + 32])
        torch.cuda.synchronize()
        dm = float((m[b0:b0 + 32] - m32).abs().max())
        dc = float((c[b0:b0 + 32] - c32).abs().max())
        print(f"{split}: crops {b0}..{b0 + 31} at bs=128 (chunks of <= {lim}) vs bs=32: max |d| mask {dm:.3g} code {dc:.3g}")
        if split == "x3":
            assert torch.equal(m[b0:b0 + 32], m32) and torch.equal(c[b0:b0 + 32], c32)
        else:
            scale = float(c32.abs().max())
            assert max(dm, dc) <= 4e-6 * scale, (dm, dc, scale)
    # one crop against the oracle (the chunked path is the network's, not a copy of the bs=32 one)
    with torch.no_grad():
        rm, rc = ref_cpu.forward(sd, x[127:128].cpu(), 34)
    for got, ref in ((m[127:128].cpu().numpy(), rm.numpy()), (c[127:128].cpu().numpy(), rc.numpy())):
        np.testing.assert_allclose(got, ref, atol=1e-3, rtol=0)
    del net
    torch.cuda.empty_cache()
