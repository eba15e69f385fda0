#!/usr/bin/env python3
"""ZebraPose hot-path benchmark on MI355X (BASELINE.json metric: 256x256 crops/s/GPU).

One *step* = one pass of the hot path over one batch of synthetic crops resident in HBM:
BinaryCodeNet_Deeplab(34, 16, 2, concat=True) forward at bs=32 (bf16 MFMA, f32 accumulate)
+ the on-device code->vertex decode (configs[1] of BASELINE.json).  `value` is the whole-job
throughput (crops/s summed over ranks; each rank runs its own independent batch: the inference
path shards by crop with no collective -> weak scaling).

Extra fields: the training step (configs[2]/[3]: bs=32 per GPU, hist-weighted BCE + mask loss,
backward, Adam; DDP over RCCL when N > 1), the dominant kernel's roofline (HIP events around its
launches over a timed pass), and the CPU baseline (the oracle restatement on the host cores,
rank 0, N = 1, bounded sample).

Also the configs[4] leg (rank 0, N = 1): R50 fp16 batched multi-object inference + decode + PnP.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-train] [--no-cpu] [--no-multi]
    torchrun --nproc-per-node N bench.py --gpus N ...
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
FWD_GFLOP_PER_CROP = 109.136  # 2 x 54,568,026,112 MAC per 256x256 crop (R34)
R50_GFLOP_PER_CROP = 747.68  # ResNet50_OS8 + ASPP_50 forward per crop


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--train-steps", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--layer-report", default=None, help="write per-launch conv timings (JSON) here")
    ap.add_argument("--no-multi", action="store_true", help="skip the configs[4] multi-object leg")
    ap.add_argument("--mo-objects", type=int, default=30)
    ap.add_argument("--mo-crops", type=int, default=8, help="crops per object per step (configs[4] leg)")
    return ap.parse_args()


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


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

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

    def step():
        with torch.no_grad():
            m, c = net(x)
            return dec(m, c, bboxes, bbox_size=S // 2)

    # ------------------------------------------------------------------ inference (value)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    ms_per_step = el / args.steps * 1e3
    value = world * B * args.steps / el
    n_corr = int(out[0].sum().item())

    # ------------------------------------------------------------------ roofline of the dominant kernel
    eng = net.net._engine
    eng.timing = []
    with torch.no_grad():
        for _ in range(args.steps):
            net(x)
    torch.cuda.synchronize()
    per = {}
    eng_t = eng.timing
    eng.timing = None
    # group launches by kernel instantiation (the names rocprofv3 reports)
    for rec in eng_t:
        label, e0, e1, flops, kname = rec
        d = per.setdefault(kname, [0.0, 0.0, 0])
        d[0] += flops
        d[1] += e0.elapsed_time(e1) * 1e-3
        d[2] += 1
    if args.layer_report and rank == 0:
        lay = {}
        for label, e0, e1, flops, kname in eng_t:
            d = lay.setdefault(label, [kname, 0.0, 0.0, 0])
            d[1] += e0.elapsed_time(e1) * 1e3
            d[2] += flops
            d[3] += 1
        rows = [{"label": k, "kernel": v[0], "us": round(v[1] / v[3], 2), "tflops": round(v[2] / v[1] * 1e-6, 1)}
                for k, v in lay.items()]
        with open(args.layer_report, "w") as f:
            json.dump(rows, f, indent=0)
    dom = max(per.items(), key=lambda kv: kv[1][1])
    kname, (fl, tsec, nl) = dom
    achieved = fl / tsec / 1e12
    traffic = None
    # HBM bytes per launch of this kernel instance from the committed PMC passes (rocprofv3 cannot
    # run inside this process): tools/prof_round.sh + tools/prof_summary.py -> profiles/<tag>_pmc_traffic.json
    pmc = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    if pmc:
        with open(pmc[-1]) as fh:
            traffic = json.load(fh).get("by_label", {}).get(kname)
    all_conv_flops = sum(v[0] for v in per.values())
    all_conv_time = sum(v[1] for v in per.values())
    roofline = {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 2), "peak": PEAK[args.precision],
                "unit": "TFLOP/s", "frac": round(achieved / PEAK[args.precision], 4), "traffic": traffic,
                "launches_per_step": nl // args.steps, "avg_launch_us": round(tsec / nl * 1e6, 2),
                "all_conv_tflops": round(all_conv_flops / all_conv_time / 1e12, 2),
                "whole_step_tflops": round(FWD_GFLOP_PER_CROP * 1e9 * B / (ms_per_step * 1e-3) / 1e12, 2)}

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
               "correspondences_per_crop": round(n_corr / B)}

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

    # ------------------------------------------------------------------ training step (extra)
    train = None
    if not args.no_train:
        from zebrapose_amd.train import TrainStep
        tnet = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision=args.precision).to(dev)
        calibrate_bn(tnet, x)
        tnet.train()
        lr = 2e-4 * world  # train_v6.py:89-91
        ts = TrainStep(tnet, learning_rate=lr)
        g = torch.Generator(device="cpu").manual_seed(7 + rank)
        gt_code = (torch.rand((B, 16, S // 2, S // 2), generator=g) < 0.5).to(torch.uint8).to(dev)
        gt_mask = (torch.rand((B, S // 2, S // 2), generator=g) < 0.7).float().to(dev)
        K = args.train_steps or max(3, args.steps // 2)
        for _ in range(max(2, args.warmup // 2)):
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
        train = {"crops_per_s": round(world * B * K / tel, 2), "ms_per_step": round(tel / K * 1e3, 3),
                 "steps": K, "global_batch": world * B, "loss": round(float(loss[0].item()), 5),
                 "achieved_tflops": round(3 * FWD_GFLOP_PER_CROP * 1e9 * world * B * K / tel / 1e12 / world, 2),
                 "parallelism": f"ddp{world}" if world > 1 else "single"}
        del ts, tnet

    # ------------------------------------------------------------------ 3-head v3 network (extra, §8f rank 3)
    v3 = None
    if not args.no_train:
        from zebrapose_amd.model.BinaryCodeNet_v3 import BinaryCodeNet_Deeplab_v3
        from zebrapose_amd.train import TrainStep
        n3 = BinaryCodeNet_Deeplab_v3(34, 16, 2, concat=True, output_kernel_size=1, precision=args.precision).to(dev)
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
        v3 = {"model": "BinaryCodeNet_Deeplab_v3(34, 16, 2, concat=True) (train_v5.py)", "batch": B,
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
        from oracle import ref_cpu
        threads = min(16, os.cpu_count() or 1)
        torch.set_num_threads(threads)
        sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
        xb = x[:2].cpu()
        lut = synthetic_lut()
        with torch.no_grad():
            ref_cpu.forward(sd, xb, 34)
            n = 0
            t0 = time.perf_counter()
            while True:
                m, c = ref_cpu.forward(sd, xb, 34)
                for b in range(xb.shape[0]):
                    ref_cpu.decode_crop(m[b, 0].numpy(), c[b].numpy(), lut, bboxes[b])
                n += xb.shape[0]
                if time.perf_counter() - t0 > args.cpu_seconds:
                    break
            cel = time.perf_counter() - t0
        cpu = {"value": round(n / cel, 3), "unit": "crops/s", "cores": threads, "kind": "port",
               "sample": f"{n} crops (batches of 2, 256x256) through oracle/ref_cpu.py forward (torch CPU fp32) + "
                         f"numpy decode, {cel:.1f} s on {threads} threads"}

    if rank == 0:
        line = {"metric": "256x256 crops/sec (R34 DeepLabv3 inference bs=32, forward + code->vertex decode)",
                "value": round(value, 2), "unit": "crops/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": args.precision, "data": "synthetic",
                "config": {"workload": "configs[1]: ResNet34+DeepLabv3 inference bs=32 on 1xMI355X, synthetic "
                                       "256x256 crops, 16-bit code head, on-device decode",
                           "model": "BinaryCodeNet_Deeplab(34, 16, 2, concat=True)", "global_batch": world * B,
                           "per_gpu_batch": B, "input": f"{S}x{S}", "parallelism": f"replicas{world}",
                           "correspondences_last_step": n_corr},
                "roofline": roofline, "cpu_baseline": cpu, "train": train, "pnp": pnp_res, "crop": crop_res, "v3": v3,
                "multi_object": multi}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
