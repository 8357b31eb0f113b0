#!/usr/bin/env python
"""Per-layer micro-benchmark of the 3x3 conv kernels on the flagship U-Net shapes (B=32, 256^2).

Prints one line per (layer, pass) with time and TFLOP/s; run under rocprofv3 --pmc to get
counters per kernel.  ``--only`` filters layers by name substring.
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

LAYERS = [  # name, H, C1, C2, Cout, prologue
    ("enc1.a", 256, 8, 0, 32, False), ("enc1.b", 256, 32, 0, 32, True),
    ("enc2.a", 128, 32, 0, 64, False), ("enc2.b", 128, 64, 0, 64, True),
    ("enc3.a", 64, 64, 0, 128, False), ("enc3.b", 64, 128, 0, 128, True),
    ("enc4.a", 32, 128, 0, 256, False), ("enc4.b", 32, 256, 0, 256, True),
    ("enc5.a", 16, 256, 0, 256, False), ("enc5.b", 16, 256, 0, 256, True),
    ("mid.a", 8, 256, 0, 256, False), ("mid.b", 8, 256, 0, 256, True),
    ("dec5.a", 16, 256, 256, 256, False), ("dec5.b", 16, 256, 0, 256, True),
    ("dec4.a", 32, 256, 256, 256, False), ("dec4.b", 32, 256, 0, 256, True),
    ("dec3.a", 64, 256, 128, 128, False), ("dec3.b", 64, 128, 0, 128, True),
    ("dec2.a", 128, 128, 64, 64, False), ("dec2.b", 128, 64, 0, 64, True),
    ("dec1.a", 256, 64, 32, 32, False), ("dec1.b", 256, 32, 0, 32, True),
]


def _time(fn, iters):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--passes", default="fwd,dgrad,wgrad")
    ap.add_argument("--dims", type=int, default=2)
    ap.add_argument("--tile", type=int, default=256, help="top-level image size (layer sizes scale)")
    ap.add_argument("--ab", default="",
                    help="KNOB:v0,v1[,..] — interleaved same-process A/B of a kernel knob "
                         "(torch.ops.ddlpc.set_knob), e.g. CONV_CFG5:0,1; medians over --rounds")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    from ddlpc.ops import _ext
    from ddlpc.ops.fused_unet import _ConvPack
    F = _ext.ops()
    dev = "cuda"
    fns_ref_us = {}
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "dgradbn": 0.0}
    for name, H, C1, C2, Co, pro in LAYERS:
        if a.only and a.only not in name:
            continue
        N = a.batch
        H = H * a.tile // 256
        sp = (H,) * a.dims
        x1 = torch.randn(N, *sp, C1, device=dev).bfloat16()
        x2 = torch.randn(N, *sp, C2, device=dev).bfloat16() if C2 else None
        dy = torch.randn(N, *sp, Co, device=dev).bfloat16()
        conv = torch.nn.Module()
        conv.weight = torch.nn.Parameter(torch.randn(Co, C1 + C2, *(3,) * a.dims, device=dev) * 0.05)
        pk = _ConvPack(conv, 0, True)
        F.weight_pack(torch.tensor([pk.entry()], dtype=torch.int64, device=dev), 1, pk.numel())
        sc = torch.rand(C1, device=dev) + 0.5 if pro else None
        sh = torch.randn(C1, device=dev) * 0.1 if pro else None
        flops = 2.0 * N * H ** a.dims * Co * 3 ** a.dims * (C1 + C2)
        fns = {
            "fwd": lambda: F.conv3_fwd(x1, x2, pk.fwd, None, sc, sh, Co, 0, True),
            "dgrad": lambda: F.conv3_fwd(dy, None, pk.dgrad, None, None, None, C1 + C2,
                                         C1 if C2 else 0, False),
            # (the image layer: 3 real channels of the 8-channel padded input)
            "wgrad": lambda: F.conv3_wgrad(dy, x1, x2, sc, sh, cin_real=3 if C1 == 8 else 0),
            # data gradient with the BN-backward reduction against y fused into its epilogue
            "dgradbn": lambda: F.conv3_fwd(dy, None, pk.dgrad, None, None, None, C1, 0, False,
                                           None, None, x1, bn4),
        }
        bn4 = torch.stack([torch.randn(C1, device=dev) * 0.1, torch.rand(C1, device=dev) + 0.5,
                           torch.rand(C1, device=dev) + 0.5, torch.randn(C1, device=dev) * 0.1]).contiguous()
        for ps in a.passes.split(","):
            if ps.startswith("t"):
                continue
            if ps.startswith("dgrad") and name == "enc1.a":
                continue
            if ps == "dgradbn" and (C2 or a.dims != 2):
                continue
            fn = fns[ps]
            if a.ab:
                knob, vals = a.ab.split(":")
                vals = [int(v) for v in vals.split(",")]
                samples = {v: [] for v in vals}
                for v in vals:                       # warm every variant once
                    F.set_knob(knob, v)
                    fn()
                for _ in range(a.rounds):
                    for v in vals:
                        F.set_knob(knob, v)
                        samples[v].append(_time(fn, a.iters))
                med = {v: sorted(x)[len(x) // 2] for v, x in samples.items()}
                for v in vals:
                    tot[f"{ps}@{v}"] = tot.get(f"{ps}@{v}", 0.0) + med[v]
                print(f"{name:8s} {ps:6s} " + "  ".join(
                    f"{knob}={v}: {med[v]:8.1f} us {flops / med[v] / 1e6:7.1f} TF/s" for v in vals)
                    + f"  ({med[vals[1]] / med[vals[0]]:.3f}x)", flush=True)
                continue
            fn()
            torch.cuda.synchronize()
            us = _time(fn, a.iters)
            tot[ps] += us
            if ps == "dgradbn":
                tot["dgrad_b_layers"] = tot.get("dgrad_b_layers", 0.0) + fns_ref_us.get(name, 0.0)
            if ps == "dgrad":
                fns_ref_us[name] = us
            print(f"{name:8s} {ps:6s} {us:9.1f} us  {flops / us / 1e6:8.1f} TF/s", flush=True)
    # transposed-conv up-sampling (2x2 stride 2), channels preserved: (name, Hin, C)
    UPS = [("up5", 8, 256), ("up4", 16, 256), ("up3", 32, 256), ("up2", 64, 128), ("up1", 128, 64)]
    tpasses = [p for p in a.passes.split(",") if p.startswith("t")]
    for name, H, C in UPS:
        if not tpasses or (a.only and a.only not in name):
            continue
        N = a.batch
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        dout = torch.randn(N, 2 * H, 2 * H, C, device=dev).bfloat16()
        up = torch.nn.Module()
        up.weight = torch.nn.Parameter(torch.randn(C, C, 2, 2, device=dev) * 0.05)
        pk = _ConvPack(up, 1, True)
        F.weight_pack(torch.tensor([pk.entry()], dtype=torch.int64, device=dev), 1, pk.numel())
        b = torch.zeros(C, device=dev)
        flops = 2.0 * N * H * H * C * 4 * C
        bn4 = torch.stack([torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5,
                           torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1]).contiguous()
        fns = {"tfwd": lambda: F.convt_fwd(x, pk.fwd, b, C),
               "tfwdbn": lambda: F.convt_fwd(x, pk.fwd, b, C, bn4),
               "tdgrad": lambda: F.convt_dgrad(dout, pk.dgrad, C)[0],
               "tdgradbn": lambda: F.convt_dgrad(dout, pk.dgrad, C, x, bn4)[0],
               "twgrad": lambda: F.convt_wgrad(x, dout),
               # full backward with the deferred BN: fused kernel vs the separate pair
               "tbwdf": lambda: F.convt_bwd_fused(x, dout, pk.dgrad, None, None, None, bn4),
               "tbwds": lambda: (F.convt_dgrad(dout, pk.dgrad, C, x, bn4), F.convt_wgrad(x, dout, None, None, None, bn4))}
        for ps in tpasses:
            fn = fns[ps]
            if a.ab:
                knob, vals = a.ab.split(":")
                vals = [int(v) for v in vals.split(",")]
                samples = {v: [] for v in vals}
                for v in vals:                       # warm every variant once
                    F.set_knob(knob, v)
                    fn()
                for _ in range(a.rounds):
                    for v in vals:
                        F.set_knob(knob, v)
                        samples[v].append(_time(fn, a.iters))
                med = {v: sorted(x)[len(x) // 2] for v, x in samples.items()}
                print(f"{name:8s} {ps:6s} " + "  ".join(
                    f"{knob}={v}: {med[v]:8.1f} us {flops / med[v] / 1e6:7.1f} TF/s" for v in vals),
                    flush=True)
                continue
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.iters
            tot[ps] = tot.get(ps, 0.0) + us
            gbs = (x.numel() + dout.numel()) * 2 / us / 1e3
            print(f"{name:8s} {ps:6s} {us:9.1f} us  {flops / us / 1e6:8.1f} TF/s  {gbs:7.1f} GB/s", flush=True)
    print("totals (us):", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
