"""parallel.GradBuckets -- DDP's gradient mean (train_v6.py:252-264) with the all-reduces started
from inside the backward.  World-size-2 gloo: on CPU with a small model whose gradients are fed in
backward order (bucket boundaries, parameter broadcast, buffer sync, finish), and on the GPU with
the libzp network (two ranks sharing the one card over gloo) through TrainStep's data-parallel
path, against the mean of each rank's plain single-process gradients."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))


def _cpu_worker(rank, world, port, q):
    _env(rank, world, port)
    from zebrapose_amd import parallel as P
    try:
        P.init_from_env("gloo")
        torch.manual_seed(rank)  # ranks start from different weights: the constructor broadcasts rank 0's
        net = torch.nn.Sequential(torch.nn.Linear(6, 40), torch.nn.BatchNorm1d(40), torch.nn.ReLU(),
                                  torch.nn.Linear(40, 5))
        with torch.no_grad():
            net[1].running_mean.fill_(float(rank))
        red = P.GradBuckets(net, bucket_mb=2e-4)  # ~210 B: three buckets
        nb = len(red.buckets)
        w0 = net[0].weight.detach().clone()
        net.train()
        g = torch.Generator().manual_seed(5)
        xb = torch.randn(8, 6, generator=g)
        out = {}
        for step in range(2):  # the bucket state resets between steps
            for p in net.parameters():
                p.grad = None
            with torch.no_grad():
                net[1].running_mean.add_(float(rank))  # diverge, then sync_buffers restores rank 0's
            red.sync_buffers()
            rm = net[1].running_mean.detach().clone()
            net(xb[rank * 4:(rank + 1) * 4]).pow(2).mean().backward()
            for p in reversed(list(net.parameters())):  # the engine's order
                red.ready(p, p.grad)
            avg = red.finish()
            out[step] = [avg[p].detach().clone().tolist() for p in net.parameters()]
        q.put((rank, nb, w0.tolist(), rm.tolist(), out))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_grad_buckets_gloo_cpu():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_cpu_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] >= 3
    assert res[0][2] == res[1][2]  # rank 0's parameters everywhere
    assert res[0][3] == res[1][3]  # rank 0's buffers before every forward
    # each rank's own half-batch gradient (BN normalises per rank, as DDP without SyncBN does)
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(6, 40), torch.nn.BatchNorm1d(40), torch.nn.ReLU(),
                              torch.nn.Linear(40, 5))
    net.train()
    g = torch.Generator().manual_seed(5)
    xb = torch.randn(8, 6, generator=g)
    per = []
    for r in range(world):
        net.zero_grad()
        net(xb[r * 4:(r + 1) * 4]).pow(2).mean().backward()
        per.append([p.grad.clone() for p in net.parameters()])
    want = [(a / 2 + b / 2) for a, b in zip(*per)]
    for step in (0, 1):
        for r in range(world):
            for got, w in zip(res[r][4][step], want):
                torch.testing.assert_close(torch.tensor(got), w, rtol=1e-5, atol=1e-6)


def _gpu_worker(rank, world, port, q, mode="buckets"):
    _env(rank, world, port)
    if mode == "torch_ddp":  # torch's DistributedDataParallel(net) over the libzp network
        os.environ["ZP_TORCH_DDP"] = "1"
    torch.cuda.set_device(0)
    from zebrapose_amd import parallel as P
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    from zebrapose_amd.train import TrainStep
    try:
        P.init_from_env("gloo")
        dev = torch.device("cuda", 0)
        torch.manual_seed(0)
        net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="bf16").to(dev)
        net.train()
        g = torch.Generator().manual_seed(11)
        x = torch.randn(4, 3, 64, 64, generator=g)[rank * 2:(rank + 1) * 2].to(dev)
        gt = (torch.rand(4, 16, 32, 32, generator=g) < 0.5).to(torch.uint8)[rank * 2:(rank + 1) * 2].to(dev)
        gm = (torch.rand(4, 32, 32, generator=g) < 0.7).float()[rank * 2:(rank + 1) * 2].to(dev)
        names = ["net.aspp.conv_1x1_4.weight", "net.aspp.conv_1x1_4.bias", "net.resnet.layer5.2.conv2.weight",
                 "net.resnet.resnet.0.weight", "net.resnet.resnet.1.weight"]
        params = dict(net.named_parameters())
        # plain local gradients (no exchange)
        ts0 = TrainStep(net, ddp=False, learning_rate=0.0)
        ts0.optimizer.step = lambda: None
        ts0(x, gt, gm)
        local = {n: params[n].grad.detach().double().cpu() for n in names}
        norm_local = sum(float(p.grad.double().pow(2).sum()) for p in net.parameters())
        # data-parallel step: the same forward / backward with the buckets attached
        ts = TrainStep(net, ddp=True, learning_rate=0.0, device=0)
        ts.optimizer.step = lambda: None
        if mode == "torch_ddp":
            assert ts.buckets is None and isinstance(ts.net, torch.nn.parallel.DistributedDataParallel)
        else:
            assert ts.buckets is not None and ts.net is net
        # when each parameter's gradient reached autograd (its AccumulateGrad / DDP hook): the share
        # of the engine's reverse pass enqueued by then.  At world size 2 under torch's DDP the
        # stage-by-stage chain (zebrapose_amd.staged) is taken automatically -- the path an unchanged
        # train_v6.py:259 takes at world 8
        eng = net.net._engine
        seen = {}

        def hook_for(n):
            def hook(t):
                seen.setdefault(n, getattr(eng, "bwd_progress", (0, 1)))
            return hook
        hooks = [p.register_post_accumulate_grad_hook(hook_for(n)) for n, p in net.named_parameters()]
        ts(x, gt, gm)
        torch.cuda.synchronize()
        for h in hooks:
            h.remove()
        avg = {n: params[n].grad.detach().double().cpu() for n in names}
        nb = len(ts.buckets.buckets) if ts.buckets is not None else None
        q.put((rank, nb, {n: local[n].tolist() for n in names}, {n: avg[n].tolist() for n in names}, norm_local,
               {n: list(v) for n, v in seen.items()}))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["buckets", "torch_ddp"])
def test_grad_buckets_engine_two_ranks(gpu, mode):
    """Both data-parallel paths over the libzp network: GradBuckets (default) and torch's own
    DistributedDataParallel(net) (ZP_TORCH_DDP=1, the wrapper train_v6.py:259 uses).  Under torch's
    DDP the staged chain is automatic at world size 2 (no ZP_STAGED_BACKWARD): its hooks must fire
    stage by stage -- the head's with under a quarter of the reverse pass enqueued, the stem's at the
    end."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gpu_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = sorted([q.get(timeout=100) for _ in range(world)], key=lambda r: r[0])
    finally:
        for p in ps:
            p.join(timeout=60)
    for p in ps:
        assert p.exitcode == 0
    if mode == "buckets":
        assert res[0][1] >= 4  # 116 MB of f32 gradients in ~25 MB buckets
    for n in res[0][2]:
        want = (torch.tensor(res[0][2][n]) / 2 + torch.tensor(res[1][2][n]) / 2)
        scale = want.abs().max().item() + 1e-12
        for r in range(world):
            got = torch.tensor(res[r][3][n])
            assert (got - want).abs().max().item() <= 1e-5 * scale, n
    assert res[0][4] > 0 and res[1][4] > 0
    if mode == "torch_ddp":  # the automatic staged chain: head hooks early, the stem's at the end
        for r in range(world):
            hp = res[r][5]
            assert len(hp) == 152
            done, total = hp["net.aspp.conv_1x1_4.weight"]
            assert done < total / 4, (r, done, total)
            done, total = hp["net.resnet.layer5.2.conv2.weight"]
            assert done < total / 2, (r, done, total)
            done, total = hp["net.resnet.resnet.0.weight"]
            assert done == total, (r, done, total)
