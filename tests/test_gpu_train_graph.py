"""hipGraph-captured training (zebrapose_amd.graphs.GraphedTrainStep) and the capturable FusedAdam
it needs (device-side step counts, zp_adam_multi_dev)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_capturable_adam_matches_torch():
    """FusedAdam(capturable=True): device step counts (zp_adam_multi_dev) against torch.optim.Adam."""
    from zebrapose_amd.optim import FusedAdam
    torch.manual_seed(3)
    ref = [torch.randn(n, requires_grad=True) for n in (5, 4097, 300)]
    dev = [r.detach().clone().cuda().requires_grad_(True) for r in ref]
    o_ref, o = torch.optim.Adam(ref, lr=3e-4), FusedAdam(dev, lr=3e-4, capturable=True)
    for s in range(4):
        for r, d in zip(ref, dev):
            g = torch.randn(r.numel()) * (s + 1)
            r.grad, d.grad = g.clone(), g.cuda()
        o_ref.step()
        o.step()
    torch.cuda.synchronize()
    for r, d in zip(ref, dev):
        np.testing.assert_allclose(d.detach().cpu().numpy(), r.detach().numpy(), rtol=1e-5, atol=1e-7)
    assert o.state_dict()["state"][0]["step"].item() == 4


def test_graphed_train_step_matches_eager(golden):
    """Five bf16 train steps eagerly vs two eager warm-up steps + three hipGraph replays from the
    same initial state: losses and parameters agree (the same kernels; Adam's bias corrections are
    computed on the device in the capturable form)."""
    from oracle import ref_cpu
    from zebrapose_amd.graphs import GraphedTrainStep
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    from zebrapose_amd.train import TrainStep
    sd = ref_cpu.synthetic_state(34, 16, 0, dict(golden("r34_bn_buffers.npz")))
    B, S = 4, 128
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, 3, S, S, generator=g).cuda()
    gc = torch.randint(0, 2, (B, 16, S // 2, S // 2), generator=g, dtype=torch.uint8).cuda()
    gm = torch.randint(0, 2, (B, S // 2, S // 2), generator=g).float().cuda()
    nets, losses = [], []
    for graphed in (False, True):
        net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="bf16")
        net.load_state_dict(sd)
        net = net.cuda().train()
        ts = TrainStep(net, learning_rate=2e-4, capturable=True)
        ls = []
        if graphed:
            gts = GraphedTrainStep(ts, x, gc, gm, warmup=2)
            for _ in range(3):
                ls.append(float(gts(x, gc, gm)[0]))
        else:
            for _ in range(5):
                ls.append(float(ts(x, gc, gm)[0]))
            ls = ls[2:]
        nets.append(net)
        losses.append(ls)
    np.testing.assert_allclose(losses[1], losses[0], rtol=1e-4)
    pa, pb = dict(nets[0].named_parameters()), dict(nets[1].named_parameters())
    for k in pa:
        np.testing.assert_allclose(pb[k].detach().cpu().numpy(), pa[k].detach().cpu().numpy(), rtol=1e-3, atol=1e-5,
                                   err_msg=k)
