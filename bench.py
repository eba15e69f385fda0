#!/usr/bin/env python3
"""ZebraPose hot-path benchmark on MI355X (BASELINE.json metric: 256x256 crops/s/GPU).

One *step* = one pass of the hot path over one batch of synthetic crops resident in HBM:
BinaryCodeNet_Deeplab(34, 16, 2, concat=True) forward at bs=32 in fp32 (the reference's own
arithmetic, BinaryCodeNet.py:161-174: no AMP) + the on-device code->vertex decode (configs[1] of
BASELINE.json); the same step in bf16 (bf16 MFMA, f32 accumulate) is a labelled leg.  `value` is the whole-job
throughput (crops/s summed over ranks; each rank runs its own independent batch: the inference
path shards by crop with no collective -> weak scaling).

Extra fields: the training step (configs[2]/[3]: bs=32 per GPU, hist-weighted BCE + mask loss,
backward, Adam; DDP over RCCL when N > 1), the dominant kernel's roofline (HIP events around its
launches over a timed pass), and the CPU baseline (the oracle restatement on the host cores,
rank 0, N = 1, bounded sample).

Also the configs[4] leg (rank 0, N = 1): R50 fp16 batched multi-object inference + decode + PnP.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-train] [--no-cpu] [--no-multi]
    torchrun --nproc-per-node N bench.py --gpus N ...

``--gpus N`` (N > 1) without a torchrun environment launches the N ranks itself (one process per
GPU, torch.multiprocessing spawn, as train_v6.py:465-468 does with mp.spawn); the parent process
never touches the GPU.  Each rank joins the process group (RCCL for the GPU run); ``n_gpus`` is
the size of the group that actually formed.  ``--dry-run`` swaps the network for a CPU stub and
RCCL for gloo: it exercises exactly this launcher / rendezvous / timing path on a host without a
GPU (tests/test_bench_launcher.py).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
os.environ.setdefault("ZP_QUIET", "1")

PEAK = {"bf16": 2516.6, "fp32": 157.3}  # TFLOP/s dense MFMA (256 CU x 4 SIMD x 2.4 GHz; MI355X_MICROARCH.md)
# The split-fp32 kernels (k_conv3 / k_conv3s, include/zp.h) form each f32 product from 6 bf16 MFMA
# products (ZP_F32X3) or 3 fp16 ones (ZP_F32H2): their MFMA ceiling in f32 FLOP/s is the dense
# 16-bit peak / 6 or / 3 (bf16 and fp16 MFMAs take the same cycles).
PEAK_X3 = PEAK["bf16"] / 6.0
PEAK_H2 = PEAK["bf16"] / 3.0


def peak_of(kname, precision):
    """(peak TFLOP/s, basis) for the dominant kernel instance."""
    if kname.startswith("k_conv3") and "<h2" in kname:
        return PEAK_H2, ("split-fp32 kernel (two fp16 planes): dense fp16 MFMA peak 2516.6 / 3 fp16 products "
                         "per f32 MAC (f32 MFMA peak 157.3)")
    if kname.startswith("k_conv3"):  # k_conv3 / k_conv3s
        return PEAK_X3, ("split-fp32 kernel: dense bf16 MFMA peak 2516.6 / 6 bf16 products per f32 MAC "
                         "(f32 MFMA peak 157.3)")
    if "<f32" in kname:
        return PEAK["fp32"], "dense f32 MFMA peak (v_mfma_f32_16x16x4_f32)"
    return PEAK["bf16"], "dense bf16 MFMA peak"
FWD_GFLOP_PER_CROP = 109.136  # 2 x 54,568,026,112 MAC per 256x256 crop (R34)
R50_GFLOP_PER_CROP = 747.68  # ResNet50_OS8 + ASPP_50 forward per crop


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--precision", default="fp32", choices=["bf16", "fp32"],
                    help="headline precision; fp32 = the reference's own arithmetic (bf16 runs as a labelled leg)")
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--train-steps", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=60.0, help="bound on each CPU-baseline timing loop")
    ap.add_argument("--layer-report", default=None, help="write per-launch conv timings (JSON) here")
    ap.add_argument("--no-multi", action="store_true", help="skip the configs[4] multi-object leg")
    ap.add_argument("--mo-objects", type=int, default=30)
    ap.add_argument("--mo-crops", type=int, default=8, help="crops per object per step (configs[4] leg)")
    ap.add_argument("--no-bf16", action="store_true", help="skip the bf16 inference leg")
    ap.add_argument("--no-rccl", action="store_true", help="N = 1: no world-size-1 RCCL group for the train leg")
    ap.add_argument("--no-bs1", action="store_true", help="skip the bs=1 eager vs hipGraph latency leg")
    ap.add_argument("--eager", action="store_true", help="time the eager launches instead of the hipGraph replay")
    ap.add_argument("--dry-run", action="store_true", help="CPU stub workload over gloo (launcher test)")
    return ap.parse_args(argv)


def calibrate_bn(net, x):
    """Synthetic checkpoint: BN running stats := batch statistics of one train-mode pass."""
    bns = [m for m in net.modules() if isinstance(m, torch.nn.BatchNorm2d)]
    for m in bns:
        m.momentum = 1.0
    net.train()
    with torch.no_grad():
        net(x)
    for m in bns:
        m.momentum = 0.1
    net.eval()


def synthetic_crops(B, S, device, seed):
    """uint8 HWC crops normalised as the reference's loader does (bop_dataset_pytorch.py:333-347;
    BGR order with RGB ImageNet constants)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    u8 = torch.randint(0, 256, (B, 3, S, S), generator=g, dtype=torch.uint8)
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    return ((u8.float() / 255.0 - mean) / std).to(device)


def synthetic_lut(seed=0):
    rng = np.random.default_rng(seed)
    lut = rng.standard_normal((65536, 3)) * 50.0
    lut[::97] = np.nan
    return lut


def kernel_name(dt, cout, cin_l):
    wc = 4 if cout > 64 else (2 if cout > 32 else 1)
    small = cin_l < (64 if dt == "bf16" else 32)
    return f"k_conv<{'bf16' if dt == 'bf16' else 'f32'},WC={wc},WP=4,smallC={int(small)}>"


def _device_init_(net, seed):
    """Synthetic weights generated on the device (SURVEY §8d recipe: He-normal convs, BN
    gamma~U(0.5,1.5), beta~N(0,0.1)); used for the 30 R50 objects of the configs[4] leg, whose
    f32 masters (41 GB) are never built on the host."""
    g = torch.Generator(device=next(net.parameters()).device).manual_seed(seed)
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, (torch.nn.Conv2d, torch.nn.ConvTranspose2d)):
                w = m.weight
                fan = (w.shape[1] if isinstance(m, torch.nn.Conv2d) else w.shape[0] / 4.0) * w.shape[2] * w.shape[3]
                w.normal_(0.0, float(np.sqrt(2.0 / fan)), generator=g)
                if m.bias is not None:
                    m.bias.normal_(0.0, 0.01, generator=g)
            elif isinstance(m, torch.nn.BatchNorm2d):
                m.weight.uniform_(0.5, 1.5, generator=g)
                m.bias.normal_(0.0, 0.1, generator=g)
                m.running_mean.zero_()
                m.running_var.fill_(1.0)
                m.num_batches_tracked.zero_()


def _cpu_model():
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def cpu_baseline(args, net, x, bboxes):
    """SURVEY §8(d) / BASELINE.md CPU-baseline protocol: the oracle (oracle/ref_cpu.py: the reference's
    op sequence on the torch CPU backend, fp32; decode in the reference's own per-pixel-loop form,
    CNN_output_to_pose.py:53-64) on the host cores, 2 warm-ups then the median of 10 timed iterations,
    at bs=1 and bs=32, forward / decode / end-to-end.  Threads: torch's default, i.e. OMP_NUM_THREADS
    when set -- on the GPU box that is 16, the CPU share one GPU's job is given there (the machine
    shows more CPUs, reported as host_cpus, but belongs to 8 GPUs' jobs)."""
    from oracle import ref_cpu
    threads = torch.get_num_threads()
    sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    lut = synthetic_lut()
    ld = ref_cpu.lut_dict(lut)
    res = {}
    t_all = time.perf_counter()
    with torch.no_grad():
        for bs in (1, x.shape[0]):
            xb = x[:bs].cpu()
            fw = []
            n_it = 10
            it = 0
            while it < 2 + n_it:
                t0 = time.perf_counter()
                m, c = ref_cpu.forward(sd, xb, 34)
                dtf = time.perf_counter() - t0
                if it >= 2:
                    fw.append(dtf)
                elif it == 1 and dtf * n_it > args.cpu_seconds:  # bound the sample (reported below)
                    n_it = max(3, int(args.cpu_seconds / dtf))
                it += 1
            dec = []
            for b in range(bs):
                t0 = time.perf_counter()
                ref_cpu.decode_crop_loop(m[b, 0].numpy(), c[b].numpy(), ld, bboxes[b])
                dec.append(time.perf_counter() - t0)
            f_med = float(np.median(fw))
            d_crop = float(np.median(dec))
            res[f"bs{bs}"] = {"forward_ms": round(f_med * 1e3, 1), "forward_crops_per_s": round(bs / f_med, 3),
                              "decode_ms_per_crop": round(d_crop * 1e3, 2), "e2e_crops_per_s":
                              round(bs / (f_med + sum(dec)), 3), "timed_forward_iterations": len(fw)}
    total = time.perf_counter() - t_all
    big = res[f"bs{x.shape[0]}"]
    return {"value": big["e2e_crops_per_s"], "unit": "crops/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(), "cpu_model": _cpu_model(), **res,
            "sample": f"oracle/ref_cpu.py forward (torch CPU fp32, {threads} threads) + the reference-form per-pixel "
                      f"decode loop, 256x256 synthetic crops; 2 warm-ups then the median of the timed iterations "
                      f"at bs=1 and bs={x.shape[0]}; value = bs={x.shape[0]} end-to-end; {total:.0f} s of CPU work"}


def train_breakdown(ts, tnet, x, gt_code, gt_mask, world, rank, steps=3):
    """Per-step timeline of the train step from HIP events on the compute stream: forward + loss,
    backward (engine reverse pass; at N > 1 up to the moment the current stream has waited for every
    gradient bucket's RCCL all-reduce), optimizer.  At N > 1 also: when each bucket's all-reduce
    was enqueued relative to the backward start, the exposed communication (last bucket enqueued ->
    all buckets complete), and the same buckets all-reduced standalone (no overlapping compute).
    Per-rank bucket order goes to stderr (BASELINE.md configs[3]: all-reduce time vs backward)."""
    rows = []
    ts.events = []
    if ts.buckets is not None:
        ts.buckets.timing = []
    for _ in range(steps):
        ts.events.clear()
        if ts.buckets is not None:
            ts.buckets.timing.clear()
        ts(x, gt_code, gt_mask)
        torch.cuda.synchronize()
        ev = dict(ts.events)
        r = {"fwd_loss_ms": ev["start"].elapsed_time(ev["backward"]),
             "backward_ms": ev["backward"].elapsed_time(ev["optimizer"]),
             "optimizer_ms": ev["optimizer"].elapsed_time(ev["end"])}
        if ts.buckets is not None:
            tl = ts.buckets.timing
            launches = [(b, e) for b, e in tl if b != "done"]
            done = [e for b, e in tl if b == "done"][0]
            r["bucket_enqueue_ms"] = [round(ev["backward"].elapsed_time(e), 3) for _, e in launches]
            r["exposed_comm_ms"] = launches[-1][1].elapsed_time(done)
        rows.append(r)
    ts.events = None
    med = {k: round(float(np.median([r[k] for r in rows])), 3) for k in rows[0] if not isinstance(rows[0][k], list)}
    out = dict(med, steps=steps)
    if ts.buckets is not None:
        out["bucket_enqueue_ms"] = rows[-1]["bucket_enqueue_ms"]
        ts.buckets.timing = None
        names = {p: n for n, p in tnet.named_parameters()}
        layout = ts.buckets.describe(names)
        flats = [bk[0] for bk in ts.buckets.buckets]
        nbytes = sum(f.numel() * f.element_size() for f in flats)
        times = []
        for _ in range(5):
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for f in flats:
                dist.all_reduce(f, op=dist.ReduceOp.SUM)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        ar = float(np.median(times))
        out.update(buckets=len(flats), bucket_mb=[b[1] for b in layout], grad_mb=round(nbytes / 2 ** 20, 2),
                   allreduce_ms_standalone=round(ar * 1e3, 3), allreduce_algbw_GBps=round(nbytes / ar / 1e9, 1),
                   backend=dist.get_backend(), world=world)
        if world > 1:  # ring bus bandwidth 2 (N - 1) / N x bytes / time (0 at N = 1: nothing crosses a link)
            out["allreduce_busbw_GBps"] = round(2 * (world - 1) / world * nbytes / ar / 1e9, 1)
        print(f"[rank {rank}] grad buckets (launch order): " + "; ".join(
            f"#{b} {mb} MB {n} params {first}..{last}" for b, mb, n, first, last in layout)
            + f" | enqueue ms into backward {out['bucket_enqueue_ms']} | exposed comm {out['exposed_comm_ms']} ms",
            file=sys.stderr, flush=True)
    return out


def bs1_leg(net, dec, S, dev, iters=50):
    """The reference's per-crop evaluation loop (test.py:190, 248: bs=1): forward + decode of one
    crop, eager (about 50 launches whose arguments are packed in Python: host-bound) vs one
    hipGraph replay of the same captured step (zebrapose_amd.graphs)."""
    from zebrapose_amd.graphs import GraphedInference
    x1 = synthetic_crops(1, S, dev, seed=7)
    bb = np.array([[100, 80, 200, 200]])

    def eager():
        with torch.no_grad():
            m, c = net(x1)
            return dec(m, c, bb, bbox_size=S // 2)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / iters * 1e3

    te = timed(eager)
    g = GraphedInference(net, 1, S, decoder=dec, bbox_size=S // 2)
    tg = timed(lambda: g(x1, bb))
    return {"eager_ms_per_crop": round(te, 3), "graph_ms_per_crop": round(tg, 3),
            "graph_crops_per_s": round(1e3 / tg, 1), "speedup": round(te / tg, 2), "iterations": iters}


def multi_object_leg(args, dev):
    """configs[4]: ResNet50 + ASPP_50, fp16 MFMA, batched multi-object inference (T-LESS-style 30
    objects, one weight set + LUT each) with the code->vertex decode and PnP on the device
    (zebrapose_amd/multi_object.py).  One step = mo_crops crops of every object, grouped by object,
    one forward per object, one decode and one PnP launch over the whole batch."""
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    from zebrapose_amd.multi_object import MultiObjectPose
    nobj, per = args.mo_objects, args.mo_crops
    B = nobj * per
    x = synthetic_crops(B, 256, dev, seed=500)
    nets = []
    for o in range(nobj):
        with torch.device("meta"):
            n = BinaryCodeNet_Deeplab(50, 16, 2, concat=True, output_kernel_size=1, precision="fp16")
        n = n.to_empty(device=dev)
        _device_init_(n, 1000 + o)
        calibrate_bn(n, x[o * per:(o + 1) * per])
        nets.append(n)
    luts = [synthetic_lut(o) for o in range(nobj)]
    mo = MultiObjectPose(nets, luts, precision="fp16")
    rng = np.random.default_rng(11)
    obj = rng.permutation(np.repeat(np.arange(nobj), per))  # crops arrive interleaved
    side = rng.integers(64, 401, B)
    bb = np.stack([rng.integers(0, 300, B), rng.integers(0, 200, B), side, side], 1)
    mo(x, obj, bb)
    torch.cuda.synchronize()
    steps = 3
    t0 = time.perf_counter()
    for _ in range(steps):
        out = mo(x, obj, bb)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    res = {"workload": f"configs[4]: R50+ASPP_50 fp16, {nobj} objects x {per} crops (256x256) per step, "
                       "grouped forward + one decode + one PnP launch", "crops_per_s": round(B / el, 1),
           "ms_per_step": round(el * 1e3, 2), "steps": steps, "dtype": "f16",
           "network_tflops": round(R50_GFLOP_PER_CROP * 1e9 * B / el / 1e12, 1),
           "pnp_success": int(out["success"].sum().item())}
    del mo, nets
    torch.cuda.empty_cache()
    return res


# ---------------------------------------------------------------------------------- launcher
def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _rank_main(local_rank, args, port):
    """One spawned rank: the torchrun environment, then the normal single-rank body."""
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(args.gpus),
                      LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    run(args)


def launch(args):
    """``bench.py --gpus N`` without torchrun: spawn N ranks (train_v6.py:465-468 mp.spawn).  The
    parent only counts devices (no GPU initialisation on this image) and never runs GPU work."""
    import torch.multiprocessing as mp
    if not args.dry_run:
        n = torch.cuda.device_count()
        if n < args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but only {n} GPU(s) are visible")
    mp.start_processes(_rank_main, args=(args, _free_port()), nprocs=args.gpus, join=True, start_method="spawn")


def dry_run(args, world, rank):
    """The launcher / rendezvous / barrier / max-over-ranks path with a CPU stub step (gloo)."""
    torch.manual_seed(rank)
    a = torch.randn(256, 256)
    for _ in range(args.warmup):
        a = torch.tanh(a @ a) * 0.5
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        a = torch.tanh(a @ a) * 0.5
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    if rank == 0:
        print(json.dumps({"metric": "dry-run stub steps/s", "value": round(world * args.steps / el, 2),
                          "unit": "steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "f32",
                          "data": "dry-run: CPU stub step over gloo, no GPU work",
                          "config": {"workload": "launcher dry run", "parallelism": f"replicas{world}",
                                     "backend": dist.get_backend() if world > 1 else "none"}}), flush=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        launch(args)
        return
    run(args)


def lib_sha16():
    """Identity of the libzp.so build being benched (PMC traffic files carry the one they measured)."""
    import hashlib
    from zebrapose_amd import _lib
    with open(_lib.LIB_PATH, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


def pmc_traffic(kname):
    """HBM bytes per launch of kernel instance ``kname`` from the newest committed PMC pass
    (tools/prof_round.sh + tools/prof_summary.py -> profiles/<tag>_pmc_traffic.json) that was
    measured on THIS libzp.so build (its lib_sha16); a pass of another build is refused, so the
    number cannot go stale silently.  rocprofv3 cannot run inside this process."""
    sha = lib_sha16()
    for pf in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")), reverse=True):
        if "_train_" in os.path.basename(pf):  # the eval (folded-BN) launches are the ones timed here
            continue
        with open(pf) as fh:
            d = json.load(fh)
        if d.get("lib_sha16") != sha:
            continue
        t = d.get("by_label", {}).get(kname)
        if t is not None:
            return t, os.path.relpath(pf, ROOT)
    return None, f"no committed PMC pass of this libzp.so build (lib_sha16 {sha})"


def train_pmc():
    """The newest committed training-step PMC summary (tools/prof_train.py ->
    profiles/<tag>_train_pmc_traffic.json) measured on THIS libzp.so build, or (None, reason)."""
    sha = lib_sha16()
    for pf in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_train_pmc_traffic.json")), reverse=True):
        with open(pf) as fh:
            d = json.load(fh)
        if d.get("lib_sha16") == sha and "step" in d:
            return d, os.path.relpath(pf, ROOT)
    return None, f"no committed training PMC pass of this libzp.so build (lib_sha16 {sha})"


def train_kernel_roofline(ts, tnet, x, gt_code, gt_mask, steps=2):
    """The dominant training kernel (largest total time over one step's conv / weight-gradient
    launches): every launch bracketed by HIP events on the stream it runs on (engine timing: the
    weight gradients then run on the compute stream, not the side stream); achieved = algorithmic
    FLOPs / launch time against the bf16 dense peak; traffic per launch from the training PMC pass of
    this build."""
    eng = tnet.net._engine
    per = {}
    for _ in range(steps):
        eng.timing = []
        ts(x, gt_code, gt_mask)
        torch.cuda.synchronize()
        for label, e0, e1, flops, kname, nbytes in eng.timing:
            d = per.setdefault(kname, [0.0, 0.0, 0, 0.0])
            d[0] += flops
            d[1] += e0.elapsed_time(e1) * 1e-3
            d[2] += 1
            d[3] += nbytes
    eng.timing = None
    kname, (fl, tsec, nl, nb) = max(per.items(), key=lambda kv: kv[1][1])
    pmc, src = train_pmc()
    row = (pmc or {}).get("by_label", {}).get(kname)
    traffic = None if row is None else row["hbm_bytes_per_launch"]
    achieved = fl / tsec / 1e12
    return {"kernel": kname, "launches_per_step": nl // steps, "avg_launch_us": round(tsec / nl * 1e6, 2),
            "achieved": round(achieved, 2), "peak": PEAK["bf16"], "unit": "TFLOP/s",
            "frac": round(achieved / PEAK["bf16"], 4), "algorithmic_flop_per_launch": round(fl / nl),
            "algorithmic_bytes_per_launch": round(nb / nl), "traffic": traffic,
            "traffic_over_algorithmic": None if traffic is None else round(traffic / (nb / nl), 3),
            "traffic_source": src if row is not None else (src if pmc is None else f"{src}: no row for {kname}"),
            "share_of_conv_time": round(tsec / sum(v[1] for v in per.values()), 3)}


def time_infer(net, x, dec, bboxes, steps, warmup, world, dev, rank, use_graph=True):
    """configs[1] step = forward + on-device decode of one bs=B batch resident in HBM.  The timed
    step is one hipGraph replay of that step (zebrapose_amd.graphs; the crops are copied into the
    graph's static input each step -- a device copy, timed); every kernel of the eager step runs,
    only the ~50 per-launch host round trips are gone.  Barrier + synchronize on both sides of
    the K timed steps; the max over ranks is the job time."""
    B, S = x.shape[0], x.shape[-1]

    def eager_step():
        with torch.no_grad():
            m, c = net(x)
            return dec(m, c, bboxes, bbox_size=S // 2)

    graph = None
    if use_graph:
        from zebrapose_amd.graphs import GraphedInference
        try:
            graph = GraphedInference(net, B, S, decoder=dec, bbox_size=S // 2)
            graph.bb.copy_(torch.as_tensor(bboxes, dtype=torch.int32))
        except RuntimeError as e:  # the same kernels, launched one by one (launch says which)
            print(f"[bench] rank {rank}: hipGraph capture failed ({e}); timing the eager launches",
                  file=sys.stderr, flush=True)
            graph = None

    def step():
        if graph is None:
            return eager_step()
        return graph(x)[2:]

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    n_corr = int(out[0].sum().item())
    res = {"el": el, "ms_per_step": el / steps * 1e3, "value": world * B * steps / el, "n_corr": n_corr,
           "launch": "eager" if graph is None else "hipgraph", "out": tuple(t.clone() for t in out)}
    del graph
    return res


def conv_roofline(net, x, steps, precision, ms_per_step, layer_report=None, rank=0):
    """Roofline of the dominant conv kernel instance (largest total time over the step's launches):
    every conv launch of `steps` eager forwards bracketed by HIP events on the stream it runs on
    (torch's current stream, where libzp enqueues); achieved = sum of algorithmic FLOPs
    (2 * M * taps * Cin * Cout per launch) / sum of launch durations."""
    eng = net.net.eval_engine()
    eng.timing = []
    with torch.no_grad():
        for _ in range(steps):
            net(x)
    torch.cuda.synchronize()
    per = {}
    eng_t = eng.timing
    eng.timing = None
    for label, e0, e1, flops, kname, nbytes in eng_t:
        d = per.setdefault(kname, [0.0, 0.0, 0, 0.0])
        d[0] += flops
        d[1] += e0.elapsed_time(e1) * 1e-3
        d[2] += 1
        d[3] += nbytes
    if layer_report and rank == 0:
        lay = {}
        for label, e0, e1, flops, kname, _ in eng_t:
            d = lay.setdefault(label, [kname, 0.0, 0.0, 0])
            d[1] += e0.elapsed_time(e1) * 1e3
            d[2] += flops
            d[3] += 1
        rows = [{"label": k, "kernel": v[0], "us": round(v[1] / v[3], 2), "tflops": round(v[2] / v[1] * 1e-6, 1)}
                for k, v in lay.items()]
        with open(layer_report, "w") as f:
            json.dump(rows, f, indent=0)
    kname, (fl, tsec, nl, algo_bytes) = max(per.items(), key=lambda kv: kv[1][1])
    achieved = fl / tsec / 1e12
    traffic, traffic_src = pmc_traffic(kname)
    algo_per_launch = algo_bytes / nl
    B = x.shape[0]
    all_fl = sum(v[0] for v in per.values())
    all_t = sum(v[1] for v in per.values())
    peak, basis = peak_of(kname, precision)
    return {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 2), "peak": round(peak, 2),
            "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "peak_basis": basis,
            "frac_of_f32_mfma_peak": round(achieved / PEAK["fp32"], 4) if precision == "fp32" else None,
            "traffic": traffic,
            "traffic_source": traffic_src, "algorithmic_bytes_per_launch": round(algo_per_launch),
            "traffic_over_algorithmic": None if traffic is None else round(traffic / algo_per_launch, 3),
            "launches_per_step": nl // steps, "avg_launch_us": round(tsec / nl * 1e6, 2),
            "algorithmic_flop_per_launch": round(fl / nl),
            "all_conv_tflops": round(all_fl / all_t / 1e12, 2),
            "conv_ms_per_step": round(all_t / steps * 1e3, 3),
            "whole_step_tflops": round(FWD_GFLOP_PER_CROP * 1e9 * B / (ms_per_step * 1e-3) / 1e12, 2),
            "lib_sha16": lib_sha16()}


def run(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo", rank=rank, world_size=world)
            world = dist.get_world_size()
        dry_run(args, world, rank)
        if world > 1:
            dist.destroy_process_group()
        return
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    rccl1 = False
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        world = dist.get_world_size()  # the ranks that actually joined the RCCL group
    elif not args.no_rccl and not args.no_train:
        # N = 1: a world-size-1 RCCL group, so the train leg's data-parallel gradient exchange
        # (configs[3]'s code path: GradBuckets' async all_reduce on the RCCL stream) runs for real
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                device_id=dev)
        rccl1 = True

    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    from zebrapose_amd.decode import Decoder

    torch.manual_seed(1234)
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision=args.precision).to(dev)
    B, S = args.batch, args.size
    x = synthetic_crops(B, S, dev, seed=100 + rank)
    calibrate_bn(net, x)
    dec = Decoder(synthetic_lut(), device=dev)
    rng = np.random.default_rng(rank)
    side = rng.integers(64, 401, B)
    bboxes = np.stack([rng.integers(0, 300, B), rng.integers(0, 200, B), side, side], 1)

    def eager_step():
        with torch.no_grad():
            m, c = net(x)
            return dec(m, c, bboxes, bbox_size=S // 2)

    # ------------------------------------------------------------------ inference (value)
    main = time_infer(net, x, dec, bboxes, args.steps, args.warmup, world, dev, rank, use_graph=not args.eager)
    value, ms_per_step, n_corr, out = main["value"], main["ms_per_step"], main["n_corr"], main["out"]
    roofline = conv_roofline(net, x, args.steps, args.precision, ms_per_step, args.layer_report, rank)

    # (the training leg runs right after the headline: measured inside the full bench after the bf16
    # and bs=1 hipGraph legs with the world-size-1 RCCL group alive, the same step read ~1 ms slower
    # (16.95 vs 15.9-16.0 ms with any one of the three absent, tools/plans/r05_g34.txt) -- an
    # interaction of the process's earlier legs, not of the step)
    # ------------------------------------------------------------------ training step (extra)
    # configs[2]: bs=32 per GPU, bf16 (BASELINE.json), hist-weighted BCE + mask loss, backward, Adam;
    # configs[3] at N > 1 (DDP over RCCL).  At N = 1 the same step also runs through a world-size-1
    # RCCL group (rccl_world1): every bucket's all_reduce is a real RCCL collective on its stream.
    train = None
    tprec = "bf16"
    if not args.no_train:
        from zebrapose_amd.train import TrainStep
        tnet = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision=tprec).to(dev)
        calibrate_bn(tnet, x)
        tnet.train()
        lr = 2e-4 * world  # train_v6.py:89-91
        g = torch.Generator(device="cpu").manual_seed(7 + rank)
        gt_code = (torch.rand((B, 16, S // 2, S // 2), generator=g) < 0.5).to(torch.uint8).to(dev)
        gt_mask = (torch.rand((B, S // 2, S // 2), generator=g) < 0.7).float().to(dev)
        K = args.train_steps or max(3, args.steps // 2)

        def timed_train(ts):
            # (the first steps initialise the Adam state and grow the caching allocator: W full
            # warm-up steps, not W / 2, so the timed steps are steady-state)
            for _ in range(max(3, args.warmup)):
                ts(x, gt_code, gt_mask)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            for _ in range(K):
                loss = ts(x, gt_code, gt_mask)
            torch.cuda.synchronize()
            tel = time.perf_counter() - t0
            if world > 1:
                t = torch.tensor([tel], device=dev, dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                tel = t.item()
            return tel, loss

        ts = TrainStep(tnet, learning_rate=lr)
        tel, loss = timed_train(ts)
        train = {"crops_per_s": round(world * B * K / tel, 2), "ms_per_step": round(tel / K * 1e3, 3),
                 "steps": K, "global_batch": world * B, "dtype": tprec, "loss": round(float(loss[0].item()), 5),
                 "achieved_tflops": round(3 * FWD_GFLOP_PER_CROP * 1e9 * world * B * K / tel / 1e12 / world, 2),
                 "parallelism": f"ddp{world}" if world > 1 else "single"}
        tpk = PEAK["bf16"] if tprec in ("bf16", "fp16") else PEAK["fp32"]
        train["roofline"] = {"bound": "mfma", "achieved": train["achieved_tflops"], "peak": tpk, "unit": "TFLOP/s",
                             "frac": round(train["achieved_tflops"] / tpk, 4), "traffic": None,
                             "scope": "whole step, wall clock: 3 x the forward's algorithmic FLOPs (forward, data "
                                      "gradient, weight gradient) over the step time, against the dense MFMA peak"}
        pmc, psrc = train_pmc()
        if pmc is not None:  # whole-step HBM bytes from the training PMC passes of this build
            st = pmc["step"]
            train["roofline"].update(
                traffic=st["hbm_bytes"], traffic_unit="HBM bytes per training step (PMC, one-stream step)",
                traffic_source=psrc,
                hbm_gbps_over_step=round(st["hbm_bytes"] / (train["ms_per_step"] * 1e-3) / 1e9, 1))
        else:
            train["roofline"]["traffic_source"] = psrc
        train["breakdown"] = train_breakdown(ts, tnet, x, gt_code, gt_mask, world, rank)
        train["roofline"]["dominant_kernel"] = train_kernel_roofline(ts, tnet, x, gt_code, gt_mask)
        del ts
        if rccl1:
            ts = TrainStep(tnet, learning_rate=lr, ddp=True, device=local)
            tel, _ = timed_train(ts)
            train["rccl_world1"] = {
                "what": "the same step through a world-size-1 RCCL process group (backend nccl): GradBuckets' "
                        "bucketed async all_reduce on the RCCL stream, overlapped with the backward, plus the "
                        "per-forward BN buffer broadcast -- configs[3]'s exchange code, on one GPU",
                "ms_per_step": round(tel / K * 1e3, 3), "crops_per_s": round(B * K / tel, 2),
                "breakdown": train_breakdown(ts, tnet, x, gt_code, gt_mask, 1, rank)}
            del ts
        del tnet

    # ------------------------------------------------------------------ bf16 leg (throughput mode)
    # the same step with bf16 storage / bf16 MFMA (f32 accumulate): narrower than the reference's
    # fp32, so a labelled extra with its own roofline, not the headline
    bf16 = None
    if args.precision != "bf16" and not args.no_bf16:
        net.set_precision("bf16")
        r = time_infer(net, x, dec, bboxes, args.steps, args.warmup, world, dev, rank, use_graph=not args.eager)
        bf16 = {"crops_per_s": round(r["value"], 2), "ms_per_step": round(r["ms_per_step"], 3), "dtype": "bf16",
                "launch": r["launch"], "steps": args.steps,
                "roofline": conv_roofline(net, x, args.steps, "bf16", r["ms_per_step"])}
        net.set_precision(args.precision)
        torch.cuda.empty_cache()

    # ------------------------------------------------------------------ bs=1 latency: eager vs hipGraph
    bs1 = None
    if not args.no_bs1 and rank == 0:
        bs1 = bs1_leg(net, dec, S, dev)
        bs1["dtype"] = args.precision
        # the benched batch launched eagerly, one launch at a time (value is the graph replay)
        for _ in range(2):
            eager_step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            eager_step()
        torch.cuda.synchronize()
        ele = time.perf_counter() - t0
        bs1["bs%d_eager_crops_per_s" % B] = round(B * args.steps / ele, 1)
        bs1["bs%d_eager_ms_per_step" % B] = round(ele / args.steps * 1e3, 3)

    # ------------------------------------------------------------------ on-device PnP (extra, §8f rank 1)
    # RANSAC-EPnP (150 iterations, 2 px) over the last step's decoded correspondences; the random
    # network gives random correspondences, i.e. the worst case (no early RANSAC termination)
    from zebrapose_amd.pnp import PnP
    pnp = PnP()
    counts, xy, xyz = out
    pnp(counts, xy, xyz)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        pnp(counts, xy, xyz)
    e1.record()
    torch.cuda.synchronize()
    pnp_ms = e0.elapsed_time(e1) / 5
    pnp_res = {"ms_per_batch": round(pnp_ms, 3), "crops_per_s": round(B / (pnp_ms * 1e-3), 1), "iterations": 150,
               "correspondences_per_crop": round(n_corr / B),
               "what": "the random network's decoded correspondences: no RANSAC early termination (worst case)"}
    # the same on realistic scenes: 32 crops of 7000 correspondences from a known pose (0.5 px
    # noise, 30% outliers) -- OpenCV's adaptive bound stops RANSAC after ~25 iterations
    g = torch.Generator().manual_seed(7)
    ns, HWs = 7000, 7000
    Kc = torch.tensor([[572.4114, 0.0, 325.2611], [0.0, 573.57043, 242.04899], [0.0, 0.0, 1.0]], dtype=torch.float64)
    sc_xy = torch.zeros(B, HWs, 2, dtype=torch.int32)
    sc_xyz = torch.zeros(B, HWs, 3, dtype=torch.float32)
    for b in range(B):
        ang = torch.randn(3, generator=g, dtype=torch.float64) * 0.6
        th = float(ang.norm())
        kx = torch.tensor([[0, -ang[2], ang[1]], [ang[2], 0, -ang[0]], [-ang[1], ang[0], 0]], dtype=torch.float64) / th
        Rm = torch.eye(3, dtype=torch.float64) + np.sin(th) * kx + (1 - np.cos(th)) * kx @ kx
        tv = torch.tensor([0.0, 0.0, 800.0], dtype=torch.float64) + torch.rand(3, generator=g, dtype=torch.float64) * 100 - 50
        pw = torch.rand(ns, 3, generator=g, dtype=torch.float64) * 120 - 60
        Xc = pw @ Rm.T + tv
        uv = torch.stack([Kc[0, 0] * Xc[:, 0] / Xc[:, 2] + Kc[0, 2], Kc[1, 1] * Xc[:, 1] / Xc[:, 2] + Kc[1, 2]], 1)
        uv = uv + torch.randn(uv.shape, generator=g, dtype=torch.float64) * 0.5
        outl = torch.rand(ns, generator=g) < 0.3
        uv[outl] += torch.rand(int(outl.sum()), 2, generator=g, dtype=torch.float64) * 240 - 120
        sc_xy[b] = uv.round().int()
        sc_xyz[b] = pw.float()
    sc = (torch.full((B,), ns, dtype=torch.int32, device=dev), sc_xy.to(dev), sc_xyz.to(dev))
    pnp(*sc, Kc.numpy())
    torch.cuda.synchronize()
    e0.record()
    for _ in range(5):
        r_sc = pnp(*sc, Kc.numpy())
    e1.record()
    torch.cuda.synchronize()
    sc_ms = e0.elapsed_time(e1) / 5
    pnp_res["scenes"] = {"ms_per_batch": round(sc_ms, 3), "crops_per_s": round(B / (sc_ms * 1e-3), 1),
                         "correspondences_per_crop": ns, "outliers": 0.3, "success": int(r_sc[2].sum().item()),
                         "what": "synthetic scenes from a known pose (0.5 px noise, 30% outliers): RANSAC stops early"}

    # ------------------------------------------------------------------ device crop pipeline (extra, §8f rank 2)
    from zebrapose_amd.crop import CropPipeline
    cp = CropPipeline()
    g = torch.Generator(device="cpu").manual_seed(3)
    imgs = torch.randint(0, 256, (8, 480, 640, 3), generator=g, dtype=torch.uint8).to(dev)
    gts = torch.randint(0, 256, (8, 480, 640, 3), generator=g, dtype=torch.uint8).to(dev)
    msk = torch.randint(0, 256, (8, 480, 640), generator=g, dtype=torch.uint8).to(dev)
    raw = np.stack([rng.integers(0, 500, B), rng.integers(0, 350, B), rng.integers(40, 200, B),
                    rng.integers(40, 200, B)], 1)
    pad, _ = cp.boxes(raw, 640, 480)
    cidx = np.arange(B) % 8
    cp(imgs, cidx, pad, gts, msk, msk)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        cp(imgs, cidx, pad, gts, msk, msk)
    e1.record()
    torch.cuda.synchronize()
    crop_ms = e0.elapsed_time(e1) / 10
    crop_res = {"ms_per_batch": round(crop_ms, 3), "crops_per_s": round(B / (crop_ms * 1e-3), 1),
                "what": "640x480 BGR images -> 256 px INTER_LINEAR normalised crop + 128 px GT code planes and "
                        "2 masks (INTER_NEAREST), padding 1.5"}
    del imgs, gts, msk

    # ------------------------------------------------------------------ 3-head v3 network (extra, §8f rank 3)
    v3 = None
    if not args.no_train:
        from zebrapose_amd.model.BinaryCodeNet_v3 import BinaryCodeNet_Deeplab_v3
        from zebrapose_amd.train import TrainStep
        n3 = BinaryCodeNet_Deeplab_v3(34, 16, 2, concat=True, output_kernel_size=1, precision=tprec).to(dev)
        calibrate_bn(n3, x)
        with torch.no_grad():
            n3(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.no_grad():
            for _ in range(args.steps):
                n3(x)
        torch.cuda.synchronize()
        inf_ms = (time.perf_counter() - t0) / args.steps * 1e3
        n3.train()
        ts3 = TrainStep(n3, learning_rate=2e-4 * world)
        g = torch.Generator(device="cpu").manual_seed(9 + rank)
        gt_code = (torch.rand((B, 16, S // 2, S // 2), generator=g) < 0.5).to(torch.uint8).to(dev)
        gt_mask = (torch.rand((B, S // 2, S // 2), generator=g) < 0.7).float().to(dev)
        gt_ent = (torch.rand((B, S // 2, S // 2), generator=g) < 0.8).float().to(dev)
        for _ in range(2):
            ts3(x, gt_code, gt_mask, gt_ent)
        torch.cuda.synchronize()
        K3 = max(3, args.steps // 4)
        t0 = time.perf_counter()
        for _ in range(K3):
            ts3(x, gt_code, gt_mask, gt_ent)
        torch.cuda.synchronize()
        tr_ms = (time.perf_counter() - t0) / K3 * 1e3
        v3 = {"model": "BinaryCodeNet_Deeplab_v3(34, 16, 2, concat=True) (train_v5.py)", "batch": B, "dtype": tprec,
              "infer_crops_per_s": round(B / (inf_ms * 1e-3), 1), "infer_ms_per_step": round(inf_ms, 3),
              "train_crops_per_s": round(B / (tr_ms * 1e-3), 1), "train_ms_per_step": round(tr_ms, 3)}
        del ts3, n3

    # ------------------------------------------------------------------ configs[4] multi-object leg (extra)
    multi = None
    if rank == 0 and world == 1 and not args.no_multi:
        multi = multi_object_leg(args, dev)

    # ------------------------------------------------------------------ CPU baseline (rank 0, N = 1)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args, net, x, bboxes)

    if rank == 0:
        dname = {"fp32": "f32", "bf16": "bf16"}[args.precision]
        line = {"metric": "256x256 crops/sec (R34 DeepLabv3 inference bs=32, forward + code->vertex decode)",
                "value": round(value, 2), "unit": "crops/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": dname, "data": "synthetic",
                "config": {"workload": "configs[1]: ResNet34+DeepLabv3 inference bs=32 on 1xMI355X, synthetic "
                                       "256x256 crops, 16-bit code head, on-device decode",
                           "model": "BinaryCodeNet_Deeplab(34, 16, 2, concat=True)", "global_batch": world * B,
                           "per_gpu_batch": B, "input": f"{S}x{S}", "parallelism": f"replicas{world}",
                           "precision": args.precision, "launch": main["launch"],
                           "fp32_engine": ("two-plane fp16 split fp32 (ZP_F32H2; range-guarded, full-range "
                                           "x3 fallback)" if args.precision == "fp32" else None),
                           "correspondences_last_step": n_corr},
                "roofline": roofline, "bf16": bf16, "bs1": bs1, "cpu_baseline": cpu, "train": train, "pnp": pnp_res,
                "crop": crop_res, "v3": v3, "multi_object": multi}
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
