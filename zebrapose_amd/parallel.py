"""Process-group plumbing for the data-parallel path (one process per GPU; backend 'nccl' is RCCL
over xGMI on ROCm, 'gloo' for CPU tests).

Reference: train_v6.py:47-51 (init_process_group), :82-91 (lr x world, iterations / world),
:149/168/223 (DistributedSampler), :391-393 (metric all-reduce of [value, 1]).
Inference shards crops by rank with no collective; training all-reduces gradients through DDP.
"""
from __future__ import annotations

import math
import os

import torch
import torch.distributed as dist


def init_from_env(backend="nccl"):
    """torchrun-style env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT); returns (rank, world, local)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return rank, world, local


def sampler_indices(n, rank, world, epoch=0, shuffle=True, seed=0):
    """torch DistributedSampler semantics (drop_last=False): pad by wrapping to a multiple of
    world, then every world-th index starting at rank."""
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        idx = torch.randperm(n, generator=g).tolist()
    else:
        idx = list(range(n))
    total = int(math.ceil(n / world)) * world
    idx += idx[: total - len(idx)]
    return idx[rank:total:world]


def crop_shard(n, rank, world):
    """Contiguous crop range [lo, hi) of rank for inference (no collective needed)."""
    per = (n + world - 1) // world
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def all_reduce_mean_metric(value, device=None):
    """train_v6.py:391-393: all_reduce SUM of [value, 1] -> value / count."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value), 1.0], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return (t[0] / t[1]).item()


def max_over_ranks(seconds, device=None):
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(seconds)
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


class GradBuckets:
    """DDP's gradient exchange (train_v6.py:252-264 wraps the net in DistributedDataParallel),
    overlapped with the libzp backward.

    torch's DDP sees the network as one autograd node that returns all 152 gradients at once, so
    its buckets could only all-reduce after the whole backward.  Here the engine reports each
    gradient as it is enqueued (``ready``), and when a bucket is complete it is all-reduced with
    ``async_op=True``.  The collective is ordered after the kernels enqueued so far on the current
    stream and runs on the process group's own stream (RCCL over xGMI for 'nccl') while the rest of
    the backward is computed.  ``finish`` makes the current stream wait for every bucket and returns
    the averaged gradients.

    Gradient as bucket view (round 6; DDP's ``gradient_as_bucket_view=True``): the engine asks
    ``dest(p)`` for the parameter's slice of its bucket's flat buffer and writes the gradient there
    (weight gradients by zp_conv2d_wgrad's split reduce, dgamma / dbeta by the BN backward), so no
    per-gradient copy is made; a gradient produced elsewhere is still copied in.  The mean over
    ranks is RCCL's ncclAvg (``ReduceOp.AVG``: each input pre-multiplied by 1 / world inside the
    collective, exact for world sizes that are powers of two), so no separate division pass runs;
    backends without AVG (gloo) divide the bucket first, as DDP does; at world size 1 the mean is
    the gradient itself.  ``finish`` returns fresh views of the buckets, which autograd's
    AccumulateGrad adopts as ``p.grad`` without cloning them.

    DDP semantics kept: parameters broadcast from rank 0 at construction, module buffers (BN
    running statistics) broadcast from rank 0 before every forward (broadcast_buffers=True),
    buckets of ~25 MB over the parameters in reverse registration order (the backward's order),
    gradient = mean over ranks (pre-divided, then summed, as DDP does).  Every rank issues the same
    collectives in the same order because the backward is deterministic.
    """

    def __init__(self, module, bucket_mb=25.0, group=None):
        self.module = module
        self.group = group
        self.world = dist.get_world_size(group)
        self.params = [p for p in module.parameters() if p.requires_grad]
        with torch.no_grad():
            states = [t for t in list(module.parameters()) + list(module.buffers())]
            if states:
                dist._broadcast_coalesced(self._pg(), states, 250 * 1024 * 1024, 0)
        self._flatten_buffers()
        cap = int(bucket_mb * 1024 * 1024)
        self.buckets = []  # [flat, [params], pending count, work]
        self.slot = {}  # param -> (bucket index, view)
        cur, size = [], 0
        for p in reversed(self.params):
            cur.append(p)
            size += p.numel() * p.element_size()
            if size >= cap:
                self._add_bucket(cur)
                cur, size = [], 0
        if cur:
            self._add_bucket(cur)
        # optional per-step timeline (bench.py's DDP leg): (bucket, event recorded on the current
        # stream when the bucket's all-reduce is enqueued); finish() appends ("done", event)
        self.timing = None
        self._avg = None  # the backend's ReduceOp.AVG in use (decided at the first launch)
        self._reset()

    def describe(self, names=None):
        """Bucket layout in launch order: [(bucket, MB, n params, first / last parameter name)]."""
        names = names or {}
        return [(b, round(bk[0].numel() * bk[0].element_size() / 2 ** 20, 2), len(bk[1]),
                 names.get(bk[1][0], "?"), names.get(bk[1][-1], "?")) for b, bk in enumerate(self.buckets)]

    def _pg(self):
        return self.group if self.group is not None else dist.distributed_c10d._get_default_group()

    def _add_bucket(self, ps):
        dt, dev = ps[0].dtype, ps[0].device
        if any(p.dtype != dt or p.device != dev for p in ps):
            raise ValueError("GradBuckets: one dtype / device per bucket")
        flat = torch.zeros(sum(p.numel() for p in ps), dtype=dt, device=dev)
        b = len(self.buckets)
        off = 0
        for p in ps:
            self.slot[p] = (b, flat[off:off + p.numel()].view_as(p), off)
            off += p.numel()
        self.buckets.append([flat, ps, 0, None])

    def _reset(self):
        for bk in self.buckets:
            bk[2] = len(bk[1])
            bk[3] = None
        self.seen = set()

    def _flatten_buffers(self):
        """The module's buffers (BN running mean / var, num_batches_tracked) become views of one flat
        tensor per (dtype, device), so that the per-forward broadcast is one collective per flat
        tensor in place -- _broadcast_coalesced flattened ~150 buffers into a scratch tensor and copied
        each back: ~0.6 ms of copy launches per step (BENCH r06 train.rccl_world1)."""
        groups, seen = {}, {}
        for m in self.module.modules():
            for name, b in m._buffers.items():
                if b is None:
                    continue
                groups.setdefault((b.dtype, b.device), []).append((m, name, b))
        self._buf_flats = []
        with torch.no_grad():
            for (dt, dev), items in groups.items():
                uniq = [b for b in {id(b): b for _, _, b in items}.values()]
                flat = torch.empty(sum(b.numel() for b in uniq), dtype=dt, device=dev)
                off = 0
                for b in uniq:
                    v = flat[off:off + b.numel()].view_as(b)
                    v.copy_(b)
                    seen[id(b)] = v
                    off += b.numel()
                for m, name, b in items:
                    m._buffers[name] = seen[id(b)]
                self._buf_flats.append(flat)

    def sync_buffers(self):
        """DDP broadcast_buffers=True: rank 0's BN running statistics before every forward (one
        in-place broadcast per flat buffer tensor; their version counters are bumped, as the copy
        back of a coalesced broadcast did, so version-keyed caches -- the eval BN folds -- refresh)."""
        if not self._buf_flats:
            return
        with torch.no_grad():
            for f in self._buf_flats:
                dist.broadcast(f, 0, group=self.group)
        torch.autograd.graph.increment_version(self._buf_flats)

    def _launch(self, b):
        bk = self.buckets[b]
        if self.timing is not None and torch.cuda.is_available() and bk[0].is_cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self.timing.append((b, ev))
        if self._avg is None:
            self._avg = dist.get_backend(self._pg()) == "nccl" and hasattr(dist.ReduceOp, "AVG")
        if self._avg:  # (also at world size 1, where it is the identity: the RCCL path stays exercised)
            try:
                bk[3] = dist.all_reduce(bk[0], op=dist.ReduceOp.AVG, group=self.group, async_op=True)
                return
            except (RuntimeError, ValueError):  # a backend build without ncclAvg: divide, then sum
                self._avg = False
        if self.world > 1:
            bk[0].div_(self.world)
        bk[3] = dist.all_reduce(bk[0], op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def dest(self, p):
        """The slice of p's bucket the engine writes p's gradient into (None: p is not bucketed)."""
        s = self.slot.get(p)
        return None if s is None else s[1]

    def ready(self, p, g):
        """Gradient g of parameter p has been enqueued on the current stream (written into dest(p),
        or anywhere else: then copied in)."""
        s = self.slot.get(p)
        if s is None:
            return
        if p in self.seen:
            raise RuntimeError("GradBuckets: a parameter received two gradients in one backward")
        self.seen.add(p)
        b, view = s[0], s[1]
        if g.data_ptr() != view.data_ptr():
            view.copy_(g)
        self.buckets[b][2] -= 1
        if self.buckets[b][2] == 0:
            self._launch(b)

    def finish(self):
        """Launch any bucket still open (gradients never produced count as zero, in the same order
        on every rank), wait for all, and return {parameter: averaged gradient view}."""
        for b, bk in enumerate(self.buckets):
            if bk[3] is None:
                for p in bk[1]:
                    if p not in self.seen:
                        self.slot[p][1].zero_()
                self._launch(b)
        for bk in self.buckets:
            bk[3].wait()
        if self.timing is not None and torch.cuda.is_available() and self.buckets and self.buckets[0][0].is_cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()  # the current stream has waited for every bucket
            self.timing.append(("done", ev))
        # fresh views (the slot's own view stays referenced here, so autograd would clone it)
        out = {p: self.buckets[self.slot[p][0]][0][self.slot[p][2]:self.slot[p][2] + p.numel()].view_as(p)
               for p in self.params}
        self._reset()
        return out


class _ReadyDict(dict):
    """The engine's {parameter: gradient} map; each assignment reports to GradBuckets.ready.
    ``dest(p)``: where the engine may write p's gradient (its bucket slice)."""

    def __init__(self, reducer):
        super().__init__()
        self._reducer = reducer
        self.dest = reducer.dest

    def __setitem__(self, k, v):
        super().__setitem__(k, v)
        self._reducer.ready(k, v)


def grads_sink(module):
    """The dict the engine backward writes into: a plain dict, or one feeding the module's
    attached GradBuckets (see attach_grad_buckets)."""
    red = getattr(module, "_grad_buckets", None)
    return {} if red is None else _ReadyDict(red)


def finish_grads(module, grads):
    """After the engine backward: the averaged gradients when GradBuckets is attached."""
    red = getattr(module, "_grad_buckets", None)
    return grads if red is None else red.finish()


def attach_grad_buckets(net, bucket_mb=25.0, group=None):
    """Attach a GradBuckets to the libzp-executed module(s) inside net (the DeepLabV3 whose
    autograd node runs the engine backward); returns it."""
    inner = [m for m in net.modules() if hasattr(m, "_engine")]
    if len(inner) != 1:
        raise ValueError("attach_grad_buckets: expected exactly one engine-executed module")
    red = GradBuckets(net, bucket_mb=bucket_mb, group=group)
    object.__setattr__(inner[0], "_grad_buckets", red)
    return red
