"""configs[3]'s gradient exchange over RCCL (backend "nccl"), as far as one GPU allows: a
world-size-1 RCCL process group on cuda:0 drives exactly the data-parallel code of the 8-GPU run
(reference train_v6.py:50-51 init_process_group, :259 DistributedDataParallel, :337 backward
all-reduce): GradBuckets' async all_reduce on the process group's stream, the current-stream ->
RCCL-stream hand-off, finish()'s wait(), the per-forward BN buffer broadcast; and torch's own
DistributedDataParallel(net) over the libzp network (ZP_TORCH_DDP=1).

At world size 1 the mean over ranks is the local gradient, so the averaged gradients must equal
the plain local ones BIT FOR BIT (the backward is deterministic: fixed-order split reductions), and
under GradBuckets every gradient is a view of its bucket (round 6: written there by the engine)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(port, mode, q):
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      ZP_QUIET="1")
    v3 = mode.endswith("_v3")
    mode = mode[:-3] if v3 else mode
    if mode in ("torch_ddp", "torch_ddp_staged"):
        os.environ["ZP_TORCH_DDP"] = "1"
    if mode == "torch_ddp_staged":  # zebrapose_amd.staged (automatic at world size > 1)
        os.environ["ZP_STAGED_BACKWARD"] = "1"
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        from zebrapose_amd import parallel as P
        from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
        from zebrapose_amd.train import TrainStep
        torch.manual_seed(0)
        if v3:  # the 3-head network (train_v5.py) through the same exchange paths; it runs 256 x 256 only
            from zebrapose_amd.model.BinaryCodeNet_v3 import BinaryCodeNet_Deeplab_v3
            net = BinaryCodeNet_Deeplab_v3(34, 16, 2, concat=True, output_kernel_size=1, precision="bf16").to(dev)
            hw = 256
        else:
            net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="bf16").to(dev)
            hw = 64
        net.train()
        g = torch.Generator().manual_seed(5)
        x = torch.randn(2, 3, hw, hw, generator=g).to(dev)
        gt = (torch.rand(2, 16, hw // 2, hw // 2, generator=g) < 0.5).to(torch.uint8).to(dev)
        gm = (torch.rand(2, hw // 2, hw // 2, generator=g) < 0.7).float().to(dev)
        ge = (torch.rand(2, hw // 2, hw // 2, generator=g) < 0.8).float().to(dev) if v3 else None
        extra = (ge,) if v3 else ()
        ts0 = TrainStep(net, ddp=False, learning_rate=0.0)
        ts0.optimizer.step = lambda: None
        ts0(x, gt, gm, *extra)
        local = {n: p.grad.detach().clone() for n, p in net.named_parameters()}
        # count the BN-buffer broadcasts (DDP broadcast_buffers=True: one per forward)
        # (round 6: GradBuckets broadcasts its flat buffer tensors in place, one dist.broadcast each;
        # torch's DDP uses _broadcast_coalesced)
        calls = {"bcast": 0, "bcast_flat": 0}
        orig = dist._broadcast_coalesced
        orig_b = dist.broadcast

        def counting(*a, **k):
            calls["bcast"] += 1
            return orig(*a, **k)

        def counting_b(*a, **k):
            calls["bcast_flat"] += 1
            return orig_b(*a, **k)
        dist._broadcast_coalesced = counting
        dist.broadcast = counting_b
        ts = TrainStep(net, ddp=True, learning_rate=0.0, device=0)
        ts.optimizer.step = lambda: None
        works = []
        if mode == "buckets":
            assert ts.buckets is not None and ts.net is net
            assert dist.get_backend() == "nccl"
            launch = ts.buckets._launch

            def recording(b):
                launch(b)
                works.append(ts.buckets.buckets[b][3])
            ts.buckets._launch = recording
            ts.buckets.timing = []
        else:
            assert ts.buckets is None and isinstance(ts.net, torch.nn.parallel.DistributedDataParallel)
        # when each parameter's gradient reached autograd (its AccumulateGrad / DDP hook): the share
        # of the engine's reverse pass enqueued by then
        eng = net.net._engine
        seen = {}
        def hook_for(n):
            def hook(t):
                seen.setdefault(n, getattr(eng, "bwd_progress", (0, 1)))
            return hook
        hooks = [p.register_post_accumulate_grad_hook(hook_for(n)) for n, p in net.named_parameters()]
        bc0, bf0 = calls["bcast"], calls["bcast_flat"]
        ts(x, gt, gm, *extra)
        torch.cuda.synchronize()
        for h in hooks:
            h.remove()
        diffs = {n: int((p.grad != local[n]).sum().item()) for n, p in net.named_parameters()}
        res = {"mode": mode, "diffs": diffs, "bcast": calls["bcast"] - bc0, "bcast_flat": calls["bcast_flat"] - bf0,
               "nparams": len(local),
               "hook_progress": {n: list(v) for n, v in seen.items()}}
        if mode == "buckets":
            res["avg"] = ts.buckets._avg  # RCCL's ReduceOp.AVG accepted (the 8-GPU run's mean)
            res["nflats"] = len(ts.buckets._buf_flats)
            # every BN buffer is a view of one of those flat tensors
            res["buf_outside"] = [n for n, b in net.named_buffers()
                                  if not any(f.data_ptr() <= b.data_ptr() < f.data_ptr() + f.numel() * f.element_size()
                                             for f in ts.buckets._buf_flats)]
            # gradient as bucket view (round 6): every p.grad lies inside its bucket's flat buffer --
            # written there by the engine, adopted by AccumulateGrad without a clone
            spans = [(bk[0].data_ptr(), bk[0].data_ptr() + bk[0].numel() * bk[0].element_size())
                     for bk in ts.buckets.buckets]
            res["outside_bucket"] = [n for n, p in net.named_parameters()
                                     if not any(lo <= p.grad.data_ptr() < hi for lo, hi in spans)]
            res["nbuckets"] = len(ts.buckets.buckets)
            res["launched"] = len(works)
            res["completed"] = sum(1 for w in works if w.is_completed())
            tl = ts.buckets.timing
            res["done_event"] = sum(1 for b, _ in tl if b == "done")
            # the exchange itself, standalone: every bucket all-reduced on the RCCL stream
            flats = [bk[0] for bk in ts.buckets.buckets]
            ref = [f.clone() for f in flats]
            for f in flats:
                dist.all_reduce(f, op=dist.ReduceOp.SUM)
            torch.cuda.synchronize()
            res["allreduce_identity"] = all(torch.equal(a, b) for a, b in zip(flats, ref))
        q.put(res)
    except Exception as e:  # reported to the parent as a failure message
        q.put({"error": repr(e)})
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["buckets", "torch_ddp", "torch_ddp_staged", "torch_ddp_staged_v3"])
def test_rccl_world1_grad_exchange(gpu, mode):
    """torch_ddp_staged: torch's DistributedDataParallel(net) -- the unchanged train_v6.py:259 line --
    over the stage-by-stage autograd chain (zebrapose_amd.staged): the head's gradients must reach
    DDP's hooks while most of the reverse pass is still to be enqueued, the stem's at its end."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), mode, q))
    p.start()
    try:
        res = q.get(timeout=110)
    finally:
        p.join(timeout=60)
    assert "error" not in res, res.get("error")
    assert p.exitcode == 0
    bad = {n: d for n, d in res["diffs"].items() if d}
    assert not bad, f"averaged gradients differ from the local ones: {bad}"
    v3 = mode.endswith("_v3")
    nparams = res["nparams"]
    assert nparams == (192 if v3 else 152), nparams
    hp = res["hook_progress"]
    assert len(hp) == nparams
    if v3:  # ASPP_v3's head runs last in the forward, first in the reverse pass; its first staged
        # segment also holds the three-head split and the up blocks (measured: 19 of 71 units)
        done, total = hp["net.aspp_v3.conv_1x1_4.weight"]
        assert done < total / 3, (done, total)
        done, total = hp["net.resnet.resnet.0.weight"]
        assert done == total
    elif mode == "torch_ddp_staged":
        done, total = hp["net.aspp.conv_1x1_4.weight"]
        assert done < total / 4, (done, total)  # head gradients handed over early
        done, total = hp["net.resnet.layer5.2.conv2.weight"]
        assert done < total / 2, (done, total)
        done, total = hp["net.resnet.resnet.0.weight"]
        assert done == total
    elif mode == "torch_ddp":  # one autograd node: every hook after the whole reverse pass
        assert all(d == t for d, t in hp.values())
    if mode == "buckets":
        assert res["nbuckets"] >= 4  # 116 MB of f32 gradients in ~25 MB buckets
        assert res["launched"] == res["nbuckets"] == res["completed"]
        assert res["done_event"] == 1
        # rank 0's BN buffers broadcast before the forward: one in-place broadcast per flat buffer
        # tensor (f32 running stats, int64 num_batches_tracked), no coalescing copies
        assert res["bcast"] == 0 and res["bcast_flat"] == res["nflats"] == 2, res
        assert not res["buf_outside"], res["buf_outside"]
        assert res["allreduce_identity"]
        assert not res["outside_bucket"], res["outside_bucket"]
        assert res["avg"] is True, res["avg"]  # the buckets' mean is RCCL's ReduceOp.AVG
