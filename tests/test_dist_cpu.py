"""World-size-2 gloo tests (CPU) of the data-parallel plumbing: sampler sharding, crop sharding,
metric all-reduce ([value, 1] SUM, train_v6.py:391-393), max-over-ranks timing, and the
DDP gradient-mean + lr x world rule of train_v6.py:82-91 on a small CPU model."""
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


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from zebrapose_amd import parallel as P
    from zebrapose_amd.train import scale_for_world
    try:
        P.init_from_env("gloo")
        idx = P.sampler_indices(11, rank, world, epoch=3)
        lo, hi = P.crop_shard(33, rank, world)
        m = P.all_reduce_mean_metric(float(rank + 1))
        mx = P.max_over_ranks(float(rank) * 2.0)
        # DDP gradient averaging on CPU: each rank sees half of a batch
        torch.manual_seed(0)
        lin = torch.nn.Linear(4, 3)
        ddp = torch.nn.parallel.DistributedDataParallel(lin)
        g = torch.Generator().manual_seed(1)
        xb = torch.randn(8, 4, generator=g)
        ddp(xb[rank * 4:(rank + 1) * 4]).pow(2).mean().backward()
        lr, iters = scale_for_world(2e-4, 380000, world)
        q.put((rank, idx, (lo, hi), m, mx, lin.weight.grad.numpy().tolist(), lr, iters))  # plain data (no shm fds)
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    idx0, idx1 = res[0][1], res[1][1]
    assert len(idx0) == len(idx1) == 6 and set(idx0) | set(idx1) == set(range(11))
    assert res[0][2] == (0, 17) and res[1][2] == (17, 33)
    assert res[0][3] == res[1][3] == 1.5
    assert res[0][4] == res[1][4] == 2.0
    # DDP mean of per-rank grads == grad of the full-batch mean loss
    torch.manual_seed(0)
    lin = torch.nn.Linear(4, 3)
    g = torch.Generator().manual_seed(1)
    xb = torch.randn(8, 4, generator=g)
    lin(xb).pow(2).mean().backward()
    torch.testing.assert_close(torch.tensor(res[0][5]), lin.weight.grad)
    torch.testing.assert_close(torch.tensor(res[1][5]), lin.weight.grad)
    assert res[0][6] == pytest.approx(4e-4) and res[0][7] == 190000
