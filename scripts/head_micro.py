#!/usr/bin/env python
"""Micro-benchmark of the fused head kernels at the flagship shape (batch 128, 256^2, 32
channels, 6 classes, deferred BN): the training forward + statistics pass and the
recompute + BN-backward apply pass.  Run under rocprofv3 --pmc for counters."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from ddlpc.ops import _ext
    F = _ext.ops()
    dev = "cuda"
    N, H, C, K = a.batch, 256, 32, 6
    y = torch.randn(N, H, H, C, device=dev).bfloat16()
    bn4 = torch.stack([torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5,
                       torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1]).contiguous()
    wh = torch.randn(K, C, device=dev) * 0.3
    bh = torch.randn(K, device=dev) * 0.1
    lab = torch.randint(0, K, (N, H, H), device=dev)
    gamma = torch.rand(C, device=dev) + 0.5
    o, wrows, brows = F.head_ce_fwd_stats(y, wh, bh, lab, -100, bn4)
    scale = torch.ones(1, device=dev) / o[2:3]
    fns = {"fwd_stats": lambda: F.head_ce_fwd_stats(y, wh, bh, lab, -100, bn4),
           "bn_apply": lambda: F.head_ce_bn_bwd(y, wh, bh, lab, o, None, -100, bn4, brows, gamma,
                                                None, None, scale)}
    for name, fn in fns.items():
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        e1.synchronize()
        print(f"{name:10s} {e0.elapsed_time(e1) * 1e3 / a.iters:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
