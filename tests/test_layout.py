"""Drop-in boundary on the host: module tree, state_dict keys/shapes/aliases, parameter order,
checkpoint save/load in the reference's layout (utils_v2.py:4-51)."""
import os

import numpy as np
import pytest
import torch

from tests.conftest import GOLDEN


@pytest.fixture(scope="module")
def net():
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    return BinaryCodeNet_Deeplab(num_resnet_layers=34, concat=True, binary_code_length=16,
                                 divided_number_each_iteration=2, output_kernel_size=1)


def test_state_dict_keys_and_shapes(net):
    want = open(os.path.join(GOLDEN, "state_keys_r34.txt")).read().splitlines()
    got = [f"{k} {list(v.shape)}" for k, v in net.state_dict().items()]
    assert got == want


def test_parameters(net):
    ps = list(net.parameters())
    assert len(ps) == 152
    assert sum(p.numel() for p in ps) == 29112977


def test_aliases_share_storage(net):
    sd = net.state_dict()
    from oracle import tv_layout
    _, aliases = tv_layout.state_spec(34, 16)
    for a, c in aliases.items():
        assert sd[a].data_ptr() == sd[c].data_ptr()


def test_r50_variant_layout():
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    from oracle import tv_layout
    n = BinaryCodeNet_Deeplab(50, 16, 2, True, 1)
    entries, _ = tv_layout.state_spec(50, 16)
    assert [(k, tuple(v.shape)) for k, v in n.state_dict().items()] == [(k, tuple(s)) for k, s, _ in entries]
    assert sum(p.numel() for p in n.parameters()) == 339941265


def test_reference_unsupported_configs_fail_loudly():
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab, BinaryCodeLoss
    with pytest.raises(NotImplementedError):
        BinaryCodeNet_Deeplab(34, 16, 4, True, 1)  # CE ablation (DeepLabV3_non_binary)
    with pytest.raises(NotImplementedError):
        BinaryCodeLoss("L1", True, 2)


def test_leaf_layers_never_compute_on_host(net):
    with pytest.raises(RuntimeError):
        net.net.resnet.resnet[0](torch.zeros(1, 3, 8, 8))


def test_checkpoint_roundtrip(tmp_path, net):
    from zebrapose_amd import utils_v2
    from zebrapose_amd.optim import FusedAdam
    from oracle import ref_cpu
    bn = dict(np.load(os.path.join(GOLDEN, "r34_bn_buffers.npz")))
    net.load_state_dict(ref_cpu.synthetic_state(34, 16, 0, bn))
    opt = FusedAdam(net.parameters(), lr=2e-4)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1000, gamma=1)
    for step in (10, 20, 30, 40):
        utils_v2.save_checkpoint(str(tmp_path), net, step, 0.5, opt, sched, max_to_keep=3)
    assert sorted(os.listdir(tmp_path)) == ["20", "30", "40"]
    assert utils_v2.get_checkpoint(str(tmp_path)).endswith("40")
    ck = torch.load(utils_v2.get_checkpoint(str(tmp_path)), weights_only=True)
    assert set(ck) == {"model_state_dict", "optimizer_state_dict", "iteration_step", "best_score",
                       "lr_scheduler_state_dict"}
    # a DDP-written checkpoint (module. prefix) loads into the bare module
    ddp_sd = {"module." + k: v for k, v in ck["model_state_dict"].items()}
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    n2 = BinaryCodeNet_Deeplab(34, 16, 2, True, 1)
    utils_v2.load_model_state(n2, ddp_sd)
    for (k1, v1), (k2, v2) in zip(net.state_dict().items(), n2.state_dict().items()):
        assert k1 == k2 and torch.equal(v1, v2)
    p = utils_v2.save_best_checkpoint(str(tmp_path / "best"), net, opt, sched, 0.90971, 376000)
    assert os.path.basename(p) == "0_9097step376000"


def test_v3_variant_layout():
    """BinaryCodeNet_Deeplab_v3: the reference's module tree and state_dict keys (+ net.aspp_v3.*)."""
    from zebrapose_amd.model.BinaryCodeNet_v3 import BinaryCodeNet_Deeplab_v3
    net = BinaryCodeNet_Deeplab_v3(34, 16, 2, concat=True, output_kernel_size=1)
    want = open(os.path.join(GOLDEN, "state_keys_r34v3.txt")).read().splitlines()
    assert [f"{k} {list(v.shape)}" for k, v in net.state_dict().items()] == want
    with pytest.raises(NotImplementedError):
        BinaryCodeNet_Deeplab_v3(50, 16, 2, concat=True)
