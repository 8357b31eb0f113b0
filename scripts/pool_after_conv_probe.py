#!/usr/bin/env python
"""Is a memory-bound kernel slower right after a heavy MFMA kernel than in a tight loop of its
own?  Times the encoder's forward BN + ReLU + 2x2 max-pool (bn_relu_pool2_kernel, enc1.b shape:
batch 256, 256^2 x 32) (a) back to back and (b) each call right after the enc1.b forward conv
that produces its input, with events around the pool call only.

    python scripts/pool_after_conv_probe.py [--batch 256] [--iters 10]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from ddlpc.ops import _ext
    from ddlpc.ops.fused_unet import _ConvPack
    F = _ext.ops()
    dev = "cuda"
    N, H, C = a.batch, 256, 32
    x = torch.randn(N, H, H, C, device=dev).bfloat16()
    conv = torch.nn.Module()
    conv.weight = torch.nn.Parameter(torch.randn(C, C, 3, 3, device=dev) * 0.05)
    pk = _ConvPack(conv, 0, True)
    F.weight_pack(torch.tensor([pk.entry()], dtype=torch.int64, device=dev), 1, pk.numel())
    sc = torch.rand(C, device=dev) + 0.5
    sh = torch.randn(C, device=dev) * 0.1
    y, _, _ = F.conv3_fwd(x, None, pk.fwd, None, sc, sh, C, 0, True)
    st4 = torch.stack([torch.zeros(C, device=dev), torch.ones(C, device=dev),
                       torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1]).contiguous()
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

    def pool_only():
        ts = []
        for _ in range(a.iters):
            e0, e1 = ev(), ev()
            e0.record()
            F.bn_relu_apply(y, st4, True, False)
            e1.record()
            ts.append((e0, e1))
        torch.cuda.synchronize()
        return [e0.elapsed_time(e1) * 1e3 for e0, e1 in ts]

    def after_conv():
        ts, tc = [], []
        for _ in range(a.iters):
            c0, c1, e0, e1 = ev(), ev(), ev(), ev()
            c0.record()
            yy, _, _ = F.conv3_fwd(x, None, pk.fwd, None, sc, sh, C, 0, True)
            c1.record()
            e0.record()
            F.bn_relu_apply(yy, st4, True, False)
            e1.record()
            ts.append((e0, e1))
            tc.append((c0, c1))
        torch.cuda.synchronize()
        return [e0.elapsed_time(e1) * 1e3 for e0, e1 in ts], [c0.elapsed_time(c1) * 1e3 for c0, c1 in tc]

    pool_only()
    after_conv()
    for r in range(3):
        p = sorted(pool_only())
        q, c = after_conv()
        q = sorted(q)
        print(f"round {r}: pool alone median {p[len(p) // 2]:7.1f} us | after conv median "
              f"{q[len(q) // 2]:7.1f} us (conv {sorted(c)[len(c) // 2]:7.1f} us)", flush=True)


if __name__ == "__main__":
    main()
