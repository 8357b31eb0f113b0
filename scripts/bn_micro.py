#!/usr/bin/env python
"""Micro-benchmark of the BatchNorm-backward passes on the flagship U-Net's BN shapes.

For every BN layer of the 256^2 width/2 U-Net (batch --batch): ``bn_backward`` with a
plain incoming gradient (BN1 of each block) and with the max-pool route (BN2 of the encoder
blocks: skip gradient + pooled gradient).  Prints time per call and the achieved HBM rate
over the bytes a perfect implementation moves (reduce: read dA (+dP) + y; apply: read them
again + write dY).  Run under ``rocprofv3 --kernel-trace --stats`` for the per-kernel split.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

LAYERS = [("l1", 256, 32), ("l2", 128, 64), ("l3", 64, 128), ("l4", 32, 256), ("l5", 16, 256),
          ("mid", 8, 256)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from ddlpc.ops import _ext
    F = _ext.ops()
    dev = "cuda"
    tot = 0.0
    for name, H, C in LAYERS:
        for pool in (False, True):
            if pool and name == "mid":
                continue
            N = a.batch
            y = torch.randn(N, H, H, C, device=dev).bfloat16()
            dA = (torch.randn(N, H, H, C, device=dev) * 1e-3).bfloat16()
            dP = (torch.randn(N, H // 2, H // 2, C, device=dev) * 1e-3).bfloat16() if pool else None
            mean = torch.randn(C, device=dev) * 0.1
            inv = torch.rand(C, device=dev) + 0.5
            gam = torch.rand(C, device=dev) + 0.5
            st4 = torch.stack([mean, inv, gam * inv, torch.randn(C, device=dev) * 0.1]).contiguous()
            for _ in range(2):
                F.bn_backward(dA, dP, y, st4, gam, None)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                F.bn_backward(dA, dP, y, st4, gam, None)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.iters * 1e3
            n = y.numel()
            pbytes = (n // 4) * 2 if pool else 0
            ideal = (2 * n * 2 + 2 * pbytes) + (2 * n * 2 + pbytes + n * 2)
            tot += us
            print(f"{name:4s} {H:4d}^2 x{C:4d} {'pool' if pool else '    '} {us:9.1f} us "
                  f"{ideal / us / 1e3:7.0f} GB/s (two-pass bytes {ideal / 2**20:7.1f} MiB)", flush=True)
    print(f"total {tot:.1f} us (each layer once)")
    # forward BN2 + ReLU + 2x2 max-pool of the encoder blocks (deferred skip: only the pooled
    # activation is written): ideal bytes = read y + write pooled
    for name, H, C in LAYERS[:-1]:
        N = a.batch
        y = torch.randn(N, H, H, C, device=dev).bfloat16()
        st4 = torch.stack([torch.zeros(C, device=dev), torch.ones(C, device=dev),
                           torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1]).contiguous()
        for _ in range(2):
            F.bn_relu_apply(y, st4, True, False)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            F.bn_relu_apply(y, st4, True, False)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.iters * 1e3
        ideal = y.numel() * 2 * 5 // 4
        print(f"fwd-pool {name:4s} {H:4d}^2 x{C:4d} {us:9.1f} us {ideal / us / 1e3:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
