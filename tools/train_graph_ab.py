#!/usr/bin/env python3
"""bs=32 256x256 bf16 train step: eager TrainStep vs GraphedTrainStep (same process, ms per step)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from zebrapose_amd.graphs import GraphedTrainStep
    from zebrapose_amd.model.BinaryCodeNet import BinaryCodeNet_Deeplab
    from zebrapose_amd.train import TrainStep
    B, S, K = 32, 256, 10
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = BinaryCodeNet_Deeplab(34, 16, 2, concat=True, output_kernel_size=1, precision="bf16").to(dev).train()
    x = torch.randn(B, 3, S, S, device=dev)
    gc = torch.randint(0, 2, (B, 16, S // 2, S // 2), device=dev, dtype=torch.uint8)
    gm = torch.randint(0, 2, (B, S // 2, S // 2), device=dev).float()
    ts = TrainStep(net, capturable=True)

    def timed(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / K * 1e3

    te = timed(lambda: ts(x, gc, gm))
    g = GraphedTrainStep(ts, x, gc, gm)
    tg = timed(lambda: g(x, gc, gm))
    print(f"train bs{B}: eager {te:.3f} ms/step, hipGraph {tg:.3f} ms/step ({te / tg:.3f}x)")


if __name__ == "__main__":
    main()
