#!/usr/bin/env python
"""Time the 3-D weight gradient of the 32-output-channel layers of BASELINE config #5
(3-D U-Net, batch 8, 128^3): enc1.b / dec1.b (32 -> 32, BN prologue), dec1.a (concat
32 + 64 -> 32), and the 64^3 / 32^3 levels' enc2.b, dec2.a, enc3.b.  The kernel is chosen by the environment (DDLPC_CONV3D_WGRAD_DS=0: the v3
per-depth-tap-plane kernel; DDLPC_WGDS_PF=2: the streaming kernel with two steps in flight), so
A/B runs are separate processes:

    python scripts/wgrad3d_micro.py [--batch 8] [--iters 10]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    from ddlpc.ops import _ext
    _ext.load(strict=True)
    ops = torch.ops.ddlpc
    dev = torch.device("cuda:0")
    N, S = args.batch, args.size
    tag = "v3" if os.environ.get("DDLPC_CONV3D_WGRAD_DS") == "0" else f"ds_pf{os.environ.get('DDLPC_WGDS_PF', '1')}"
    for name, sz, c1, c2, co, pro in [("enc1.b", S, 32, 0, 32, True), ("dec1.a", S, 32, 64, 32, False),
                                      ("enc2.b", S // 2, 64, 0, 64, True), ("dec2.a", S // 2, 128, 64, 64, False),
                                      ("enc3.b", S // 4, 128, 0, 128, True)]:
        x1 = torch.randn(N, sz, sz, sz, c1, device=dev).bfloat16()
        x2 = torch.randn(N, sz, sz, sz, c2, device=dev).bfloat16() if c2 else None
        dy = torch.randn(N, sz, sz, sz, co, device=dev).bfloat16()
        sc = torch.rand(c1, device=dev) + 0.5 if pro else None
        sh = torch.randn(c1, device=dev) * 0.1 if pro else None
        fn = lambda: ops.conv3_wgrad(dy, x1, x2, sc, sh)  # noqa: E731
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.iters
        flop = 2.0 * N * sz ** 3 * 27 * co * (c1 + c2)
        print(f"{tag:7s} {name:7s} {us:9.1f} us  {flop / us / 1e6:8.1f} TFLOP/s", flush=True)
        del x1, x2, dy


if __name__ == "__main__":
    main()
