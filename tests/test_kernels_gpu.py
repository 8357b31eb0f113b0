"""Numerics of every hand-written HIP kernel against a plain PyTorch fp32 reference.

Each test builds bf16 inputs, runs the gfx950 kernel through ``torch.ops.ddlpc`` and compares
with the same op computed by stock PyTorch in fp32 on the bf16-valued inputs.  Tolerances
reflect bf16 OUTPUT rounding (the kernels accumulate in fp32).
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    from ddlpc.ops import _ext
    return _ext.ops()


def nhwc(x):           # NCHW(D) -> channel-last shape
    return x.permute(0, *range(2, x.dim()), 1).contiguous()


def nchw(x):
    return x.permute(0, x.dim() - 1, *range(1, x.dim() - 1))


def assert_stats(st, ref, atol0, atol1):
    """BN-statistics partial rows [rows][2][C] of a forward conv: per-channel (sum, sum^2) of
    the kernel's fp32 outputs (before the bf16 store) against the fp32 torch reference — the
    same bf16 operands, so only fp32 summation order separates them"""
    s = st.sum(0)
    dims = (0,) + tuple(range(2, ref.dim()))
    assert torch.allclose(s[0], ref.sum(dims), rtol=1e-3, atol=atol0)
    assert torch.allclose(s[1], (ref * ref).sum(dims), rtol=1e-3, atol=atol1)


def rel_err(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def pack_conv(ops, w, need_dgrad=True):
    """pack an OIHW fp32 conv weight with the library's packer"""
    from ddlpc.ops.fused_unet import _ConvPack
    conv = torch.nn.Module()
    conv.weight = torch.nn.Parameter(w.contiguous())
    kind = 0 if w.shape[-1] == 3 else 1
    pk = _ConvPack(conv, kind, need_dgrad)
    ent = torch.tensor([pk.entry()], dtype=torch.int64, device=w.device)
    ops.weight_pack(ent, 1, pk.numel())
    return pk


@pytest.mark.parametrize("N,H,W,C1,C2,Cout", [
    (2, 16, 16, 32, 0, 32), (2, 32, 32, 64, 0, 64), (1, 16, 16, 64, 64, 128),
    (2, 8, 8, 256, 0, 256), (2, 32, 32, 3, 0, 32), (1, 16, 16, 64, 32, 96),
    (2, 24, 20, 32, 0, 64), (1, 64, 64, 32, 64, 32)])
def test_conv3_fwd(ops, N, H, W, C1, C2, Cout):
    torch.manual_seed(0)
    x1 = torch.randn(N, C1, H, W, device=DEV).bfloat16()
    x2 = torch.randn(N, C2, H, W, device=DEV).bfloat16() if C2 else None
    w = torch.randn(Cout, C1 + C2, 3, 3, device=DEV) * (1.0 / math.sqrt(9 * (C1 + C2)))
    b = torch.randn(Cout, device=DEV) * 0.1
    pk = pack_conv(ops, w)
    xin1 = ops.to_nhwc_bf16(x1, 8) if C1 % 8 else nhwc(x1)     # first layer: 3 -> 8 channels
    y, _, st = ops.conv3_fwd(xin1, nhwc(x2) if x2 is not None else None, pk.fwd, b, None,
                             None, Cout, 0, True)
    xin = torch.cat([x1, x2], 1) if x2 is not None else x1
    ref = F.conv2d(xin.float(), w.bfloat16().float(), b, padding=1)
    assert rel_err(nchw(y), ref) < 1e-2
    assert_stats(st, ref, 1e-2, 1e-1)


# shapes that fill the chip with 512-pixel (32 x 16) tiles: the BM-512 configuration (cfg 5,
# bias and BN statistics accumulated in LDS), incl. a concat input, the BN prologue and the
# split data-gradient output
@pytest.mark.parametrize("N,H,W,C1,C2,Cout,pro,co1", [
    (32, 64, 64, 128, 0, 128, True, 0), (32, 64, 64, 256, 128, 128, False, 0),
    (64, 32, 32, 256, 0, 256, True, 0), (64, 32, 32, 128, 0, 384, False, 256),
    (8, 128, 128, 128, 64, 64, True, 0)])
def test_conv3_fwd_bigtile(ops, N, H, W, C1, C2, Cout, pro, co1):
    torch.manual_seed(5)
    x1 = torch.randn(N, C1, H, W, device=DEV).bfloat16()
    x2 = torch.randn(N, C2, H, W, device=DEV).bfloat16() if C2 else None
    w = torch.randn(Cout, C1 + C2, 3, 3, device=DEV) * (1.0 / math.sqrt(9 * (C1 + C2)))
    b = torch.randn(Cout, device=DEV) * 0.1 if not co1 else None
    scale = torch.rand(C1, device=DEV) + 0.5 if pro else None
    shift = torch.randn(C1, device=DEV) * 0.5 if pro else None
    pk = pack_conv(ops, w)
    y, y2, st = ops.conv3_fwd(nhwc(x1), nhwc(x2) if x2 is not None else None, pk.fwd, b, scale,
                              shift, Cout, co1, True)
    a1 = x1.float()
    if pro:
        a1 = torch.relu(a1 * scale[None, :, None, None] + shift[None, :, None, None]).bfloat16().float()
    xin = torch.cat([a1, x2.float()], 1) if x2 is not None else a1
    ref = F.conv2d(xin, w.bfloat16().float(), b, padding=1)
    out = torch.cat([nchw(y), nchw(y2)], 1) if co1 else nchw(y)
    assert rel_err(out, ref) < 1e-2
    assert_stats(st, ref, 1e-1, 1.0)


def test_conv3_fwd_prologue(ops):
    torch.manual_seed(1)
    N, H, W, C, Cout = 2, 32, 32, 64, 64
    x = torch.randn(N, C, H, W, device=DEV).bfloat16()
    scale = torch.rand(C, device=DEV) + 0.5
    shift = torch.randn(C, device=DEV) * 0.5
    w = torch.randn(Cout, C, 3, 3, device=DEV) / math.sqrt(9 * C)
    pk = pack_conv(ops, w)
    y, _, _ = ops.conv3_fwd(nhwc(x), None, pk.fwd, None, scale, shift, Cout, 0, False)
    a = torch.relu(x.float() * scale[None, :, None, None] + shift[None, :, None, None]).bfloat16()
    ref = F.conv2d(a.float(), w.bfloat16().float(), padding=1)
    assert rel_err(nchw(y), ref) < 1e-2


@pytest.mark.parametrize("N,H,W", [(4, 128, 128), (4, 136, 120)])
def test_conv3_dgrad_96_channel_split_sums(ops, N, H, W):
    """The first decoder conv's data gradient (dY 32 ch -> d[up | skip] = 64 + 32 ch) on the
    resident 96-channel tile: both outputs vs fp32 torch, and its statistics rows = the
    per-channel column sums (the up-conv's bias gradient) with zero sum^2 rows (ops.h
    ConvFwdArgs::stats)."""
    torch.manual_seed(23)
    Cin, Cout, co1 = 32, 96, 64                 # the dgrad: 32 -> 96 channels
    w = torch.randn(Cin, Cout, 3, 3, device=DEV) / math.sqrt(9 * Cout)   # the fwd conv 96 -> 32
    pk = pack_conv(ops, w)
    dy = torch.randn(N, Cin, H, W, device=DEV).bfloat16()
    dx1, dx2, st = ops.conv3_fwd(nhwc(dy), None, pk.dgrad, None, None, None, Cout, co1, True)
    ref = F.conv_transpose2d(dy.float(), w.bfloat16().float(), padding=1)
    assert rel_err(nchw(dx1), ref[:, :co1]) < 1e-2
    assert rel_err(nchw(dx2), ref[:, co1:]) < 1e-2
    s = st.sum(0)
    assert torch.allclose(s[0], ref.sum((0, 2, 3)), rtol=1e-3, atol=1e-1)
    if DEV == "cuda":            # (the resident 96-channel GPU kernel writes zero sum^2 rows)
        assert torch.count_nonzero(s[1]) == 0


# shapes that take the resident-weight kernel (conv3x3_res.hip): high resolution, few
# channels, enough 16x16 tiles to fill the chip
@pytest.mark.parametrize("N,H,W,C1,C2,Cout,pro", [
    (2, 256, 256, 32, 0, 32, True), (2, 256, 256, 3, 0, 32, False),
    (2, 256, 256, 64, 32, 32, True), (2, 256, 256, 32, 0, 64, False),
    (2, 256, 256, 64, 0, 64, True), (3, 200, 232, 32, 0, 32, True),
    (2, 128, 128, 64, 0, 96, False),
    # streaming kernel, 8-wave 256x128 tiles (cfg 4)
    (16, 64, 64, 128, 0, 128, True), (8, 64, 64, 128, 64, 256, False)])
def test_conv3_fwd_resident(ops, N, H, W, C1, C2, Cout, pro):
    torch.manual_seed(4)
    x1 = torch.randn(N, C1, H, W, device=DEV).bfloat16()
    x2 = torch.randn(N, C2, H, W, device=DEV).bfloat16() if C2 else None
    w = torch.randn(Cout, C1 + C2, 3, 3, device=DEV) * (1.0 / math.sqrt(9 * (C1 + C2)))
    b = torch.randn(Cout, device=DEV) * 0.1
    scale = torch.rand(C1, device=DEV) + 0.5 if pro else None
    shift = torch.randn(C1, device=DEV) * 0.5 if pro else None
    pk = pack_conv(ops, w)
    xin1 = ops.to_nhwc_bf16(x1, 8) if C1 % 8 else nhwc(x1)
    y, _, st = ops.conv3_fwd(xin1, nhwc(x2) if x2 is not None else None, pk.fwd, b, scale,
                             shift, Cout, 0, True)
    a1 = x1.float()
    if pro:
        a1 = torch.relu(a1 * scale[None, :, None, None] + shift[None, :, None, None]).bfloat16().float()
    xin = torch.cat([a1, x2.float()], 1) if x2 is not None else a1
    ref = F.conv2d(xin, w.bfloat16().float(), b, padding=1)
    assert rel_err(nchw(y), ref) < 1e-2
    assert_stats(st, ref, 1e-1, 1.0)


@pytest.mark.parametrize("C1,C2,Cout", [(64, 32, 32), (32, 0, 32), (64, 128, 64), (128, 0, 128)])
def test_conv3_dgrad_resident(ops, C1, C2, Cout):
    torch.manual_seed(5)
    N, H, W = 2, 256, 256
    Cin = C1 + C2
    w = torch.randn(Cout, Cin, 3, 3, device=DEV) / math.sqrt(9 * Cin)
    dy = torch.randn(N, Cout, H, W, device=DEV).bfloat16()
    pk = pack_conv(ops, w)
    dx1, dx2, _ = ops.conv3_fwd(nhwc(dy), None, pk.dgrad, None, None, None, Cin,
                                C1 if C2 else 0, False)
    ref = F.conv_transpose2d(dy.float(), w.bfloat16().float(), padding=1)
    assert rel_err(nchw(dx1), ref[:, :C1]) < 1e-2
    if C2:
        assert rel_err(nchw(dx2), ref[:, C1:]) < 1e-2


# BN-backward reduction fused into the data-gradient epilogue (ConvFwdArgs::bnb_y): shapes
# covering the resident kernel (BN 32 / 64, ragged edges), the streaming kernel (cfg 0/1,
# cfg 4 super-stages and its 2-deep path for an odd chunk count) and the split-K finalize
@pytest.mark.parametrize("N,H,W,Cin,Cout", [
    (2, 256, 256, 32, 32), (2, 256, 256, 64, 64), (3, 200, 232, 32, 32),
    (16, 64, 64, 128, 128), (16, 64, 64, 128, 96), (2, 16, 16, 32, 32), (2, 32, 32, 64, 64),
    (1, 16, 16, 128, 128), (2, 8, 8, 256, 256), (48, 64, 64, 128, 128), (8, 128, 128, 64, 128)])
def test_conv3_dgrad_bn_backward_epilogue(ops, N, H, W, Cin, Cout):
    torch.manual_seed(11)
    w = torch.randn(Cout, Cin, 3, 3, device=DEV) / math.sqrt(9 * Cin)
    dy = torch.randn(N, Cout, H, W, device=DEV).bfloat16()
    y = torch.randn(N, Cin, H, W, device=DEV).bfloat16()
    mean = torch.randn(Cin, device=DEV) * 0.2
    invstd = torch.rand(Cin, device=DEV) + 0.5
    gamma = torch.rand(Cin, device=DEV) + 0.5
    beta = torch.randn(Cin, device=DEV) * 0.3
    scale = gamma * invstd
    s4 = torch.stack([mean, invstd, scale, beta - mean * scale]).contiguous()
    pk = pack_conv(ops, w)
    da0, _, _ = ops.conv3_fwd(nhwc(dy), None, pk.dgrad, None, None, None, Cin, 0, False)
    da, _, part = ops.conv3_fwd(nhwc(dy), None, pk.dgrad, None, None, None, Cin, 0, False,
                                None, None, nhwc(y), s4)
    assert torch.equal(da, da0)                       # the epilogue only adds the partials
    # the partials reduce the kernel's fp32 dA (before its bf16 store): reference = the fp32
    # data gradient of the same bf16 operands (only summation order differs)
    p = part.double().sum(0)
    yf = nchw(nhwc(y)).double()
    df = F.conv_transpose2d(dy.float(), w.bfloat16().float(), padding=1).double()
    a = yf * scale.double()[None, :, None, None] + s4[3].double()[None, :, None, None]
    dyh = torch.where(a > 0, df, torch.zeros_like(df))
    xh = (yf - mean.double()[None, :, None, None]) * invstd.double()[None, :, None, None]
    ref1, ref2 = dyh.sum((0, 2, 3)), (dyh * xh).sum((0, 2, 3))
    assert torch.allclose(p[0], ref1, rtol=1e-4, atol=1e-3 * math.sqrt(N * H * W))
    assert torch.allclose(p[1], ref2, rtol=1e-4, atol=1e-3 * math.sqrt(N * H * W))
    # the BN backward from those partials: dgamma / dbeta are the fp32 sums above; dY matches
    # the path with its own reduction pass over the stored dA (which differs from the fp32
    # sums by the bf16 rounding of dA, ~2^-9 relative)
    dY0, dg0, db0 = ops.bn_backward(da, None, nhwc(y), s4, gamma, None)
    dY1, dg1, db1 = ops.bn_backward(da, None, nhwc(y), s4, gamma, None, None, None, part)
    assert rel_err(dY1, dY0) < 2e-3
    assert rel_err(dg1, ref2.float()) < 1e-4 and rel_err(db1, ref1.float()) < 1e-4


@pytest.mark.parametrize("C1,C2,Cout", [(64, 32, 32), (0, 64, 32), (256, 256, 256)])
def test_conv3_dgrad_split(ops, C1, C2, Cout):
    torch.manual_seed(2)
    if C1 == 0:
        C1, C2 = C2, 0
    N, H, W = 2, 16, 16
    Cin = C1 + C2
    w = torch.randn(Cout, Cin, 3, 3, device=DEV) / math.sqrt(9 * Cin)
    dy = torch.randn(N, Cout, H, W, device=DEV).bfloat16()
    pk = pack_conv(ops, w)
    dx1, dx2, _ = ops.conv3_fwd(nhwc(dy), None, pk.dgrad, None, None, None, Cin,
                                C1 if C2 else 0, False)
    xin = torch.zeros(N, Cin, H, W, device=DEV, requires_grad=True)
    out = F.conv2d(xin, w.bfloat16().float(), padding=1)
    (g,) = torch.autograd.grad(out, xin, dy.float())
    assert rel_err(nchw(dx1), g[:, :C1]) < 1e-2
    if C2:
        assert rel_err(nchw(dx2), g[:, C1:]) < 1e-2


@pytest.mark.parametrize("N,H,W,C1,C2,Cout,pro", [
    (2, 16, 16, 32, 0, 32, False), (2, 32, 32, 64, 0, 64, True), (1, 16, 16, 64, 64, 128, False),
    (4, 8, 8, 256, 0, 256, True), (2, 32, 32, 3, 0, 32, False), (1, 16, 16, 64, 32, 32, False),
    (2, 64, 64, 64, 32, 32, True), (2, 72, 40, 32, 0, 64, True), (1, 128, 128, 128, 64, 64, False),
    (2, 48, 48, 128, 0, 96, True),
    (4, 256, 256, 32, 0, 32, True),      # > 64 split-K rows: the one-launch wide reduction
    # the 128-output-channel v3 tiles (Cout >= 128, H*W >= 32^2: the default for the deep
    # layers, ref.py:579,582 at C_out >= 128), with and without the prologue / a concat input
    (4, 32, 32, 256, 0, 256, True), (2, 64, 64, 128, 0, 128, False),
    (2, 32, 32, 256, 256, 256, False), (1, 64, 64, 256, 256, 256, True),
    (2, 64, 64, 128, 128, 128, True), (2, 40, 56, 128, 0, 128, True),
    # the first decoder conv's shape (32 output channels over a 64 + 32 concat input):
    # partial tiles, full size
    (3, 80, 72, 64, 32, 32, False), (1, 256, 256, 64, 32, 32, False)])
def test_conv3_wgrad(ops, N, H, W, C1, C2, Cout, pro):
    torch.manual_seed(3)
    x1 = torch.randn(N, C1, H, W, device=DEV).bfloat16()
    x2 = torch.randn(N, C2, H, W, device=DEV).bfloat16() if C2 else None
    dy = torch.randn(N, Cout, H, W, device=DEV).bfloat16()
    scale = shift = None
    a1 = x1.float()
    if pro:
        scale = torch.rand(C1, device=DEV) + 0.5
        shift = torch.randn(C1, device=DEV) * 0.5
        a1 = torch.relu(x1.float() * scale[None, :, None, None] + shift[None, :, None, None]).bfloat16().float()
    xin = torch.cat([a1, x2.float()], 1) if x2 is not None else a1
    xin1 = ops.to_nhwc_bf16(x1, 8) if C1 % 8 else nhwc(x1)
    dw = ops.conv3_wgrad(nhwc(dy), xin1, nhwc(x2) if x2 is not None else None, scale, shift)
    dw = dw[:, :C1 + C2]
    w = torch.zeros(Cout, C1 + C2, 3, 3, device=DEV, requires_grad=True)
    out = F.conv2d(xin, w, padding=1)
    (g,) = torch.autograd.grad(out, w, dy.float())
    assert dw.shape == g.shape
    assert rel_err(dw, g) < 5e-3


@pytest.mark.parametrize("R,N", [(1, 100), (64, 9216), (65, 37), (300, 9216), (1024, 130), (4096, 130),
                                 (5000, 70)])
def test_reduce_rows(ops, R, N):
    """Deterministic fp64 column sums of an fp32 [R][N] slab (single pass for R <= 64, the
    one-launch 16-wave form up to 1024 rows, the two-pass chunk form beyond)."""
    torch.manual_seed(R)
    x = torch.randn(R, N, device=DEV)
    got = ops.reduce_rows(x, R, N)
    ref = x.double().sum(0)
    assert got.dtype == torch.float64
    assert float((got - ref).abs().max()) < 1e-9 * max(1.0, float(ref.abs().max())) + 1e-9
    assert torch.equal(got, ops.reduce_rows(x, R, N))        # run to run: bit for bit


@pytest.mark.parametrize("N,H,W,C,pool", [
    (4, 16, 16, 64, True), (2, 64, 64, 32, True), (2, 32, 32, 256, True), (2, 8, 8, 512, True),
    (2, 32, 32, 128, False), (3, 24, 40, 32, False)])
def test_bn_forward_backward(ops, N, H, W, C, pool):
    torch.manual_seed(4)
    y = (torch.randn(N, C, H, W, device=DEV) * 2 + 0.5).bfloat16()
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.1
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    nbt = torch.zeros((), dtype=torch.long, device=DEV)
    yf = y.float()
    partial = torch.stack([yf.sum((0, 2, 3)), (yf * yf).sum((0, 2, 3))])[None].contiguous()
    s4 = ops.bn_finalize(partial, float(N * H * W), gamma, beta, rm, rv, 0.1, 1e-5, True, nbt)
    bn = torch.nn.BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(gamma)
        bn.bias.copy_(beta)
    yr = yf.clone().requires_grad_(True)
    ar = torch.relu(bn(yr))
    assert torch.allclose(rm, bn.running_mean, atol=1e-5)
    assert torch.allclose(rv, bn.running_var, rtol=1e-4, atol=1e-5)
    assert int(nbt) == 1
    a, p = ops.bn_relu_apply(nhwc(y), s4, True)
    assert rel_err(nchw(a), ar) < 5e-3
    assert rel_err(nchw(p), F.max_pool2d(nchw(a).float(), 2)) < 1e-6
    # backward through BN + ReLU + max-pool + skip sum
    dA = torch.randn(N, C, H, W, device=DEV).bfloat16()
    dP = torch.randn(N, C, H // 2, W // 2, device=DEV).bfloat16()
    dy, dg, db = ops.bn_backward(nhwc(dA), nhwc(dP) if pool else None, nhwc(y), s4, gamma, None)
    ar2 = torch.relu(bn(yr))
    a_bf = ar2.bfloat16().float()
    pooled = F.max_pool2d(a_bf, 2)
    loss = (ar2 * dA.float()).sum()
    if pool:
        loss = loss + (F.max_pool2d(ar2, 2) * dP.float()).sum()
    gy, gg, gb = torch.autograd.grad(loss, [yr, bn.weight, bn.bias])
    assert rel_err(nchw(dy), gy) < 2e-2
    assert rel_err(dg, gg) < 1e-2
    assert rel_err(db, gb) < 1e-2
    del pooled


@pytest.mark.parametrize("N,D,H,W,C,pool", [
    (2, 4, 8, 16, 32, True), (1, 6, 12, 8, 64, True), (1, 4, 16, 16, 256, True),
    (2, 3, 8, 8, 32, False), (1, 2, 4, 6, 128, False)])
def test_bn3d_forward_backward(ops, N, D, H, W, C, pool):
    torch.manual_seed(14)
    y = (torch.randn(N, C, D, H, W, device=DEV) * 2 + 0.5).bfloat16()
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.1
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    yf = y.float()
    partial = torch.stack([yf.sum((0, 2, 3, 4)), (yf * yf).sum((0, 2, 3, 4))])[None].contiguous()
    s4 = ops.bn_finalize(partial, float(N * D * H * W), gamma, beta, rm, rv, 0.1, 1e-5, True, None)
    bn = torch.nn.BatchNorm3d(C).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(gamma)
        bn.bias.copy_(beta)
    yr = yf.clone().requires_grad_(True)
    ar = torch.relu(bn(yr))
    a, p = ops.bn_relu_apply(nhwc(y), s4, pool)
    assert rel_err(nchw(a), ar) < 5e-3
    if pool:
        assert rel_err(nchw(p), F.max_pool3d(nchw(a).float(), 2)) < 1e-6
    dA = torch.randn(N, C, D, H, W, device=DEV).bfloat16()
    dP = torch.randn(N, C, D // 2, H // 2, W // 2, device=DEV).bfloat16()
    dy, dg, db = ops.bn_backward(nhwc(dA), nhwc(dP) if pool else None, nhwc(y), s4, gamma, None)
    loss = (ar * dA.float()).sum()
    if pool:   # the kernel routes the pooled gradient by the bf16 activations' arg-max
        idx = F.max_pool3d(ar.bfloat16().float(), 2, return_indices=True)[1]
        loss = loss + (ar.flatten(2).gather(2, idx.flatten(2)) * dP.float().flatten(2)).sum()
    gy, gg, gb = torch.autograd.grad(loss, [yr, bn.weight, bn.bias])
    assert rel_err(nchw(dy), gy) < 2e-2
    assert rel_err(dg, gg) < 1e-2
    assert rel_err(db, gb) < 1e-2


# (resident-weight forward: Cin % 32 == 0, Cin <= 256, 4*Cout % 128 == 0; 12x12 leaves a
# partial 128-pixel tile, Cin 96 / 512 exercise the GEMM fallback)
@pytest.mark.parametrize("N,H,W,Cin,Cout", [(2, 8, 8, 256, 256), (2, 16, 16, 64, 64), (1, 32, 32, 128, 128),
                                            (3, 12, 12, 64, 32), (2, 8, 8, 96, 64), (1, 64, 64, 64, 32),
                                            (2, 8, 8, 64, 96), (1, 8, 8, 512, 64)])
def test_convt(ops, N, H, W, Cin, Cout):
    torch.manual_seed(5)
    x = torch.randn(N, Cin, H, W, device=DEV).bfloat16()
    w = torch.randn(Cin, Cout, 2, 2, device=DEV) / math.sqrt(Cin)
    b = torch.randn(Cout, device=DEV) * 0.1
    pk = pack_conv(ops, w)
    out = ops.convt_fwd(nhwc(x), pk.fwd, b, Cout)
    xr = x.float().requires_grad_(True)
    wr = w.bfloat16().float().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    ref = F.conv_transpose2d(xr, wr, br, stride=2)
    assert rel_err(nchw(out), ref) < 1e-2
    dout = torch.randn_like(ref).bfloat16()
    gx, gw, gb = torch.autograd.grad(ref, [xr, wr, br], dout.float())
    dx = ops.convt_dgrad(nhwc(dout), pk.dgrad, Cin)[0]
    assert rel_err(nchw(dx), gx) < 1e-2
    dw, db = ops.convt_wgrad(nhwc(x), nhwc(dout))
    assert rel_err(dw, gw) < 5e-3
    assert rel_err(db, gb) < 1e-3


@pytest.mark.parametrize("N,H,Cin,Cout", [(9, 60, 256, 256), (4, 36, 512, 128), (3, 52, 256, 512),
                                           (20, 60, 256, 256), (17, 64, 256, 512)])
def test_convt_fwd_persistent_gemm(ops, N, H, Cin, Cout):
    """The persistent XCD-aware forward GEMM (gemm_nt_fwd2_kernel: shapes the resident convT
    kernel declines, Cin 256 / 512): several m tiles per workgroup, so epilogue stores drain
    under the next tile's DMA stages; a partial last m tile; plain and deferred-BN input.
    The last two shapes (>= 65536 input pixels, 4 Cout % 256 == 0) take the 256-column tiles."""
    torch.manual_seed(12)
    x = torch.randn(N, Cin, H, H, device=DEV).bfloat16()
    w = torch.randn(Cin, Cout, 2, 2, device=DEV) / math.sqrt(Cin)
    b = torch.randn(Cout, device=DEV) * 0.1
    pk = pack_conv(ops, w)
    out = ops.convt_fwd(nhwc(x), pk.fwd, b, Cout)
    ref = F.conv_transpose2d(x.float(), w.bfloat16().float(), b, stride=2)
    assert rel_err(nchw(out), ref) < 1e-2
    y = nhwc(x)
    bn4 = _bn4(Cin, 2)
    a = ops.bn_relu_apply(y, bn4, False)[0]
    assert torch.equal(ops.convt_fwd(y, pk.fwd, b, Cout, bn4), ops.convt_fwd(a, pk.fwd, b, Cout))


@pytest.mark.parametrize("C,K", [(32, 6), (64, 6), (16, 3), (8, 2), (64, 11), (32, 16), (8, 1),
                                 (64, 2)])
def test_head_ce(ops, C, K):
    """Any K <= 16 classes for C in {8, 16, 32, 64} (padded class slots, runtime K)."""
    torch.manual_seed(6)
    N, H, W = 2, 32, 32
    a = torch.relu(torch.randn(N, C, H, W, device=DEV)).bfloat16()
    wh = torch.randn(K, C, device=DEV) * 0.3
    bh = torch.randn(K, device=DEV) * 0.1
    y = torch.randint(0, K, (N, H, W), device=DEV)
    y[0, 0, :5] = -100
    out3 = ops.head_ce_fwd(nhwc(a), wh, bh, y, -100)
    ar = a.float().requires_grad_(True)
    whr = wh.clone().requires_grad_(True)
    bhr = bh.clone().requires_grad_(True)
    logits = torch.einsum("nchw,kc->nkhw", ar, whr) + bhr[None, :, None, None]
    loss = F.cross_entropy(logits, y)
    assert abs(float(out3[0]) - float(loss)) < 1e-4 * max(1.0, float(loss))
    assert int(out3[1]) == int((logits.argmax(1) == y).sum())
    assert int(out3[2]) == int((y != -100).sum())
    g = torch.tensor([0.5], device=DEV)
    da, dw, db, _ = ops.head_ce_bwd(nhwc(a), wh, bh, y, out3, g, -100)
    ga, gw, gb = torch.autograd.grad(loss * 0.5, [ar, whr, bhr])
    assert rel_err(nchw(da), ga) < 1e-2
    assert rel_err(dw, gw) < 1e-3
    assert rel_err(db, gb) < 1e-3
    lg = ops.head_logits(nhwc(a), wh, bh)
    assert rel_err(lg, logits) < 1e-5


def test_adam_matches_torch(ops):
    torch.manual_seed(7)
    n = 10_007
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    pr = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([pr], lr=1e-3)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    for t in range(1, 4):
        pr.grad = g.clone()
        opt.step()
        bc1, bc2 = 1 - 0.9 ** t, 1 - 0.999 ** t
        ops.adam_step(p, g, m, v, 0.9, 0.999, 1e-8, 0.0, 1e-3 / bc1, 1 / math.sqrt(bc2))
    assert torch.allclose(p, pr.detach(), atol=1e-6, rtol=1e-5)


def test_adam_device_scalars_match_torch(ops):
    """adam_step_dev: bias corrections advanced on the device (graph-capturable)."""
    torch.manual_seed(7)
    n = 10_007
    p = torch.randn(n, device=DEV)
    pr = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([pr], lr=1e-3, weight_decay=0.01)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    scal = torch.zeros(3, device=DEV)
    for t in range(1, 6):
        g = torch.randn(n, device=DEV)
        pr.grad = g.clone()
        opt.step()
        ops.adam_step_dev(p, g, m, v, scal, 1e-3, 0.9, 0.999, 1e-8, 0.01)
    assert float(scal[0]) == 5.0
    assert torch.allclose(p, pr.detach(), atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("codec", ["fp16_absmax", "int8_absmax"])
def test_codec_matches_oracle(codec):
    from ddlpc.ops import codec_ops
    from ddlpc.parallel import codec as C
    torch.manual_seed(8)
    g = torch.randn(100_003, device=DEV) * 1e-3
    segs = [(0, 50_000), (50_000, 100_003)]
    q, s = codec_ops.encode_segments(g, segs, codec)
    qc, sc = C.encode_segments(g.cpu(), segs, codec)
    assert torch.equal(s.cpu(), sc)
    assert torch.equal(q.cpu(), qc)
    out = torch.empty_like(g)
    codec_ops.decode_sum_segments(out, [q, q], [s, s], segs, codec, [0.25, 0.75])
    ref = torch.zeros_like(g).cpu()
    for w in (0.25, 0.75):                             # the torch oracle, rank order
        C.decode_segments_accumulate(ref, qc, sc, segs, codec, weight=w)
    assert torch.allclose(out.cpu(), ref, rtol=1e-6, atol=1e-12)
    if DEV == "cpu":                                   # the C++ kernel: the oracle's bits
        assert torch.equal(out, ref)


def test_to_nhwc_pad(ops):
    x = torch.randn(2, 3, 8, 8, device=DEV)
    y = ops.to_nhwc_bf16(x, 8)
    assert y.shape == (2, 8, 8, 8)
    assert torch.equal(y[..., :3], nhwc(x).bfloat16()) and not y[..., 3:].any()
    xc = x.bfloat16().to(memory_format=torch.channels_last)
    assert torch.equal(ops.to_nhwc_bf16(xc, 8), y)


def test_bilinear(ops):
    torch.manual_seed(9)
    x = torch.randn(2, 32, 8, 8, device=DEV).bfloat16()
    y = ops.bilinear_up2(nhwc(x))
    xr = x.float().requires_grad_(True)
    ref = F.interpolate(xr, scale_factor=2, mode="bilinear", align_corners=True)
    assert rel_err(nchw(y), ref) < 1e-2
    dy = torch.randn_like(ref).bfloat16()
    (gx,) = torch.autograd.grad(ref, xr, dy.float())
    dx = ops.bilinear_up2_bwd(nhwc(dy))
    assert rel_err(nchw(dx), gx) < 1e-2


def test_trilinear_3d(ops):
    """3-D up-sampling (UpBlock bilinear mode with dims=3 -> trilinear, align_corners)."""
    torch.manual_seed(19)
    x = torch.randn(1, 16, 4, 6, 8, device=DEV).bfloat16()
    y = ops.bilinear_up2(nhwc(x))
    xr = x.float().requires_grad_(True)
    ref = F.interpolate(xr, scale_factor=2, mode="trilinear", align_corners=True)
    assert rel_err(nchw(y), ref) < 1e-2
    dy = torch.randn_like(ref).bfloat16()
    (gx,) = torch.autograd.grad(ref, xr, dy.float())
    dx = ops.bilinear_up2_bwd(nhwc(dy))
    assert rel_err(nchw(dx), gx) < 1e-2


@pytest.mark.parametrize("C,K,H", [(32, 6, 12), (16, 3, 9), (64, 2, 8), (8, 16, 5)])
def test_head_fused_forward_stats(ops, C, K, H):
    """Training forward fused with the backward's statistics pass (unit gradient scale,
    scaled on the device in backward) against the separate forward + stats pass: loss /
    hits / count, dWh, dbh, and the BatchNorm backward (dgamma, dbeta, dY) to fp32 rounding."""
    torch.manual_seed(8)
    N, W = 2, H + 5
    yh = torch.randn(N, H, W, C, device=DEV).bfloat16()
    bnh = _bn4(C, 4)
    wh = torch.randn(K, C, device=DEV) * 0.3
    bh = torch.randn(K, device=DEV) * 0.1
    lab = torch.randint(0, K, (N, H, W), device=DEV)
    lab[1, 0, :3] = -100
    o_ref = ops.head_ce_fwd(yh, wh, bh, lab, -100, bnh)
    o, wrows, brows = ops.head_ce_fwd_stats(yh, wh, bh, lab, -100, bnh)
    assert torch.allclose(o, o_ref, rtol=1e-5, atol=0)
    gs = torch.tensor([0.5], device=DEV)
    _, dw_ref, db_ref, part_ref = ops.head_ce_bwd(yh, wh, bh, lab, o_ref, gs, -100, None, None, bnh, False)
    scale = ops.head_grad_scale(o, gs)
    assert torch.allclose(scale, gs / o[2:3], rtol=1e-6, atol=0)
    assert torch.allclose(ops.head_grad_scale(o), 1.0 / o[2:3], rtol=1e-6, atol=0)
    dw, db = ops.head_wgrad_from_rows(wrows, scale, K, C)
    assert rel_err(dw, dw_ref) < 1e-5 and rel_err(db, db_ref) < 1e-5
    # into adjacent (weight, bias) views of one flat buffer: the single-launch scatter
    flat = torch.zeros(K * C + K, device=DEV)
    ops.head_wgrad_from_rows(wrows, scale, K, C, flat[:K * C].view(K, C), flat[K * C:])
    assert torch.equal(flat[:K * C].view(K, C), dw) and torch.equal(flat[K * C:], db)
    gamma = torch.rand(C, device=DEV) + 0.5
    ref = ops.head_ce_bn_bwd(yh, wh, bh, lab, o_ref, gs, -100, bnh, part_ref, gamma)
    got = ops.head_ce_bn_bwd(yh, wh, bh, lab, o, gs, -100, bnh, brows, gamma, None, None, scale)
    assert rel_err(got[1], ref[1]) < 5e-3 and rel_err(got[2], ref[2]) < 5e-3
    assert rel_err(got[0], ref[0]) < 1e-2


@pytest.mark.parametrize("N,H,W", [(2, 32, 32), (3, 24, 40), (1, 20, 18)])
def test_conv3_wgrad_dy_prologue(ops, N, H, W):
    """First-layer weight gradient with BatchNorm backward applied on load (dY prologue:
    dy holds dA, the kernel forms k (dA [relu active] - m1 - xhat m2) from y) equals the
    separate path (bn_backward writing dY, then conv3_wgrad) — same arithmetic, so equal up
    to fp32 summation order at most; partial 16x16 tiles via odd H/W."""
    torch.manual_seed(23)
    Cin, Cout = 8, 32
    x = torch.randn(N, H, W, Cin, device=DEV).bfloat16()
    y = torch.randn(N, H, W, Cout, device=DEV).bfloat16()
    da = torch.randn(N, H, W, Cout, device=DEV).bfloat16()
    s4 = _bn4(Cout, 9)
    gamma = torch.rand(Cout, device=DEV) + 0.5
    # partial rows as the data-gradient epilogue would produce them: one reduction pass
    ref_dy, ref_dg, ref_db = ops.bn_backward(da, None, y, s4, gamma, None)
    part = torch.zeros(1, 2, Cout, device=DEV)
    a = y.float() * s4[2] + s4[3]
    dyh = torch.where(a > 0, da.float(), torch.zeros_like(a))
    xh = (y.float() - s4[0]) * s4[1]
    part[0, 0] = dyh.sum((0, 1, 2))
    part[0, 1] = (dyh * xh).sum((0, 1, 2))
    dy_sep, dg, db = ops.bn_backward(da, None, y, s4, gamma, None, None, None, part)
    coefs, dg2, db2 = ops.bn_grad_coefs(part, y, s4, gamma)
    assert torch.equal(dg, dg2) and torch.equal(db, db2)
    w_sep = ops.conv3_wgrad(dy_sep, x, None, None, None)
    w_pro = ops.conv3_wgrad(da, x, None, None, None, None, None, None, y, s4, coefs)
    assert rel_err(w_pro, w_sep) < 1e-6, rel_err(w_pro, w_sep)
    assert rel_err(dy_sep, ref_dy) < 1e-2


@pytest.mark.parametrize("N,H,W,Cout,pro", [(2, 32, 32, 32, False), (3, 40, 24, 32, True),
                                            (1, 20, 18, 32, True), (2, 36, 52, 64, False),
                                            (2, 64, 64, 64, True)])
def test_conv3_wgrad_image_layer(ops, N, H, W, Cout, pro):
    """First-layer weight gradient on the (tap, channel)-packed image kernel (cin_real = 3 of
    the 8-channel padded image) against fp32 autograd, against the generic v2 path (cin_real
    0: same products, different fp32 summation order) and with the BN-backward dY prologue;
    gradients of the padding channels must be exactly zero.  Partial 16-pixel tiles via odd
    sizes."""
    torch.manual_seed(31)
    x = torch.randn(N, 3, H, W, device=DEV).bfloat16()
    xin = ops.to_nhwc_bf16(x, 8)
    if pro:
        y = torch.randn(N, H, W, Cout, device=DEV).bfloat16()
        da = torch.randn(N, H, W, Cout, device=DEV).bfloat16()
        s4 = _bn4(Cout, 5)
        gamma = torch.rand(Cout, device=DEV) + 0.5
        part = torch.zeros(1, 2, Cout, device=DEV)
        a = y.float() * s4[2] + s4[3]
        dyh = torch.where(a > 0, da.float(), torch.zeros_like(a))
        part[0, 0] = dyh.sum((0, 1, 2))
        part[0, 1] = (dyh * (y.float() - s4[0]) * s4[1]).sum((0, 1, 2))
        dy, _, _ = ops.bn_backward(da, None, y, s4, gamma, None, None, None, part)
        coefs, _, _ = ops.bn_grad_coefs(part, y, s4, gamma)
        w_img = ops.conv3_wgrad(da, xin, None, None, None, None, None, None, y, s4, coefs, cin_real=3)
        w_gen = ops.conv3_wgrad(da, xin, None, None, None, None, None, None, y, s4, coefs)
    else:
        dy = torch.randn(N, H, W, Cout, device=DEV).bfloat16()
        w_img = ops.conv3_wgrad(dy, xin, None, None, None, cin_real=3)
        w_gen = ops.conv3_wgrad(dy, xin, None, None, None)
    assert w_img.shape == (Cout, 8, 3, 3)
    assert torch.count_nonzero(w_img[:, 3:]) == 0
    assert rel_err(w_img, w_gen) < 1e-5, rel_err(w_img, w_gen)
    w = torch.zeros(Cout, 3, 3, 3, device=DEV, requires_grad=True)
    out = F.conv2d(x.float(), w, padding=1)
    (g,) = torch.autograd.grad(out, w, dy.permute(0, 3, 1, 2).float())
    assert rel_err(w_img[:, :3], g) < 5e-3


@pytest.mark.parametrize("N,D,H,W,Cout", [(2, 6, 32, 32, 32), (1, 5, 20, 18, 32), (1, 4, 24, 40, 64)])
def test_conv3d_wgrad_image_layer(ops, N, D, H, W, Cout):
    """3-D first-layer weight gradient: the packed image kernel per depth tap plane (depth
    borders, partial tiles) vs fp32 autograd and vs the generic path; padding channels zero."""
    torch.manual_seed(37)
    x = torch.randn(N, 3, D, H, W, device=DEV).bfloat16()
    xin = ops.to_nhwc_bf16(x, 8)
    dy = torch.randn(N, D, H, W, Cout, device=DEV).bfloat16()
    w_img = ops.conv3_wgrad(dy, xin, None, None, None, cin_real=3)
    w_gen = ops.conv3_wgrad(dy, xin, None, None, None)
    assert w_img.shape == (Cout, 8, 3, 3, 3)
    assert torch.count_nonzero(w_img[:, 3:]) == 0
    assert rel_err(w_img, w_gen) < 1e-5, rel_err(w_img, w_gen)
    w = torch.zeros(Cout, 3, 3, 3, 3, device=DEV, requires_grad=True)
    out = F.conv3d(x.float(), w, padding=1)
    (g,) = torch.autograd.grad(out, w, dy.permute(0, 4, 1, 2, 3).float())
    assert rel_err(w_img[:, :3], g) < 5e-3


@pytest.mark.parametrize("N,H,W,bn", [(2, 16, 16, False), (3, 12, 20, True), (1, 40, 24, True),
                                      (4, 8, 8, True)])
def test_convt_bwd_fused(ops, N, H, W, bn):
    """Fused data + weight gradient of the 64 -> 64 transposed conv (dOut read once) against
    the separate kernels (dx and the BN partials bit for bit: same MFMA k order is not
    guaranteed, so dx to bf16 rounding; dW / db / partials to fp32 tolerance) and fp32 torch.
    Odd pixel counts leave partial 32-pixel stages; the deferred BN of x is applied to the
    weight-gradient operand in registers."""
    torch.manual_seed(21)
    C = 64
    x = torch.randn(N, H, W, C, device=DEV).bfloat16()
    w = torch.randn(C, C, 2, 2, device=DEV) / math.sqrt(C)
    pk = pack_conv(ops, w)
    dout = torch.randn(N, 2 * H, 2 * W, C, device=DEV).bfloat16()
    bn4 = _bn4(C, 7) if bn else None
    dx, part, dw, db = ops.convt_bwd_fused(x, dout, pk.dgrad, None, None, None, bn4)
    rdx, rpart = ops.convt_dgrad(dout, pk.dgrad, C, x if bn else None, bn4)
    rdw, rdb = ops.convt_wgrad(x, dout, None, None, None, bn4)
    assert rel_err(dx, rdx) < 1e-2
    assert rel_err(dw, rdw) < 1e-4 and rel_err(db, rdb) < 1e-5
    # vs fp32 torch (deferred BN: the activation relu(x*scale+shift) rounded to bf16)
    xa = ops.bn_relu_apply(x, bn4, False)[0] if bn else x
    xr = xa.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.bfloat16().float().requires_grad_(True)
    ref = F.conv_transpose2d(xr, wr, None, stride=2)
    gx, gw = torch.autograd.grad(ref, [xr, wr], dout.float().permute(0, 3, 1, 2))
    assert rel_err(dw, gw) < 5e-3
    if not bn:
        assert rel_err(dx.permute(0, 3, 1, 2), gx) < 1e-2
        return
    gamma = torch.rand(C, device=DEV) + 0.5
    a = ops.bn_backward(dx, None, x, bn4, gamma, None, None, None, part)
    b = ops.bn_backward(dx, None, x, bn4, gamma, None)
    for u, v in zip(a, b):
        assert rel_err(u, v) < 2e-3
    # into caller buffers (direct grads): accumulated
    dwo, dbo = torch.ones_like(dw), torch.ones_like(db)
    ops.convt_bwd_fused(x, dout, pk.dgrad, dwo, dbo, None, bn4)
    assert torch.allclose(dwo, dw + 1, atol=1e-5) and torch.allclose(dbo, db + 1, atol=1e-5)


@pytest.mark.parametrize("N,D,H,W,Cin,Cout", [(1, 4, 4, 8, 64, 64), (2, 4, 8, 8, 128, 64)])
def test_convt3d(ops, N, D, H, W, Cin, Cout):
    """ConvTranspose3d(k2, s2) forward / data / weight gradients vs fp32 torch."""
    torch.manual_seed(20)
    x = torch.randn(N, Cin, D, H, W, device=DEV).bfloat16()
    w = torch.randn(Cin, Cout, 2, 2, 2, device=DEV) / math.sqrt(Cin)
    b = torch.randn(Cout, device=DEV) * 0.1
    pk = pack_conv(ops, w)
    out = ops.convt_fwd(nhwc(x), pk.fwd, b, Cout)
    xr = x.float().requires_grad_(True)
    wr = w.bfloat16().float().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    ref = F.conv_transpose3d(xr, wr, br, stride=2)
    assert rel_err(nchw(out), ref) < 1e-2
    dout = torch.randn_like(ref).bfloat16()
    gx, gw, gb = torch.autograd.grad(ref, [xr, wr, br], dout.float())
    dx = ops.convt_dgrad(nhwc(dout), pk.dgrad, Cin)[0]
    assert rel_err(nchw(dx), gx) < 1e-2
    dw, db = ops.convt_wgrad(nhwc(x), nhwc(dout))
    assert rel_err(dw.view_as(gw), gw) < 5e-3
    assert rel_err(db, gb) < 1e-3


def test_conv3d_fwd_wgrad(ops):
    torch.manual_seed(10)
    N, D, H, W, C, Cout = 1, 8, 8, 16, 32, 64
    x = torch.randn(N, C, D, H, W, device=DEV).bfloat16()
    w = torch.randn(Cout, C, 3, 3, 3, device=DEV) / math.sqrt(27 * C)
    pk = pack_conv(ops, w)
    y, _, _ = ops.conv3_fwd(nhwc(x), None, pk.fwd, None, None, None, Cout, 0, False)
    ref = F.conv3d(x.float(), w.bfloat16().float(), padding=1)
    assert rel_err(nchw(y), ref) < 1e-2
    dy = torch.randn_like(ref).bfloat16()
    dw = ops.conv3_wgrad(nhwc(dy), nhwc(x), None, None, None)
    wr = torch.zeros_like(w, requires_grad=True)
    (g,) = torch.autograd.grad(F.conv3d(x.float(), wr, padding=1), wr, dy.float())
    assert rel_err(dw, g) < 5e-3
    dx, _, _ = ops.conv3_fwd(nhwc(dy), None, pk.dgrad, None, None, None, C, 0, False)
    xr = torch.zeros(N, C, D, H, W, device=DEV, requires_grad=True)
    (gx,) = torch.autograd.grad(F.conv3d(xr, w.bfloat16().float(), padding=1), xr, dy.float())
    assert rel_err(nchw(dx), gx) < 1e-2


@pytest.mark.parametrize("N,D,H,W", [(2, 32, 64, 64), (12, 5, 48, 40)])
def test_conv3d_image_layer_resident(ops, N, D, H, W):
    """3-D image layer (8-channel padded input -> 32): the resident kernel's (tap, channel)-
    packed path over depth slices with 3-plane halos (conv3x3_res.hip TAP8 = 3), incl.
    partial tiles and depth borders; output, bias and BN statistics vs fp32 torch."""
    torch.manual_seed(19)
    Cin, Cout = 8, 32
    x = torch.randn(N, Cin, D, H, W, device=DEV).bfloat16()
    x[:, 3:] = 0                                        # the engine's zero channel padding
    w = torch.randn(Cout, Cin, 3, 3, 3, device=DEV) / math.sqrt(27 * 3)
    b = torch.randn(Cout, device=DEV) * 0.1
    pk = pack_conv(ops, w)
    y, _, st = ops.conv3_fwd(nhwc(x), None, pk.fwd, b, None, None, Cout, 0, True)
    ref = F.conv3d(x.float(), w.bfloat16().float(), b, padding=1)
    assert rel_err(nchw(y), ref) < 1e-2
    assert_stats(st, ref, 1e-1, 1.0)


@pytest.mark.parametrize("N,D,H,W,C1,C2,Cout,pro,co1", [
    (2, 24, 64, 32, 32, 32, 32, True, 0),      # 8-wave 3-D config 6: 6x4x16 tiles, BN 32
    (2, 32, 32, 32, 64, 0, 64, False, 0),      # config 7: 4x4x16, BN 64
    (1, 32, 32, 32, 128, 0, 128, True, 0),     # config 8: 2x4x16, BN 128
    (1, 16, 32, 32, 128, 128, 256, False, 0),  # config 8, two channel tiles, concat
    (2, 32, 32, 32, 32, 0, 96, False, 64)])    # config 9: BN 96, split output (dec1.a dgrad)
def test_conv3d_fwd_8wave(ops, N, D, H, W, C1, C2, Cout, pro, co1):
    """3-D streaming conv on the 8-wave tile configurations (bindings.cpp conv3_fwd picks them
    when the layer fills the chip): output, bias, BN prologue, concat input, split output and
    statistics."""
    torch.manual_seed(17)
    x1 = torch.randn(N, C1, D, H, W, device=DEV).bfloat16()
    x2 = torch.randn(N, C2, D, H, W, device=DEV).bfloat16() if C2 else None
    w = torch.randn(Cout, C1 + C2, 3, 3, 3, device=DEV) * (1.0 / math.sqrt(27 * (C1 + C2)))
    b = torch.randn(Cout, device=DEV) * 0.1 if not co1 else None
    scale = torch.rand(C1, device=DEV) + 0.5 if pro else None
    shift = torch.randn(C1, device=DEV) * 0.5 if pro else None
    pk = pack_conv(ops, w)
    y, y2, st = ops.conv3_fwd(nhwc(x1), nhwc(x2) if x2 is not None else None, pk.fwd, b, scale,
                              shift, Cout, co1, True)
    a1 = x1.float()
    if pro:
        a1 = torch.relu(a1 * scale.view(1, -1, 1, 1, 1) + shift.view(1, -1, 1, 1, 1)).bfloat16().float()
    xin = torch.cat([a1, x2.float()], 1) if x2 is not None else a1
    ref = F.conv3d(xin, w.bfloat16().float(), b, padding=1)
    out = torch.cat([nchw(y), nchw(y2)], 1) if co1 else nchw(y)
    assert rel_err(out, ref) < 1e-2
    assert_stats(st, ref, 1e-1, 1.0)


@pytest.mark.parametrize("N,D,H,W,C1,C2,Cout,pro", [
    (2, 5, 12, 20, 32, 0, 64, True), (1, 4, 16, 16, 32, 32, 32, True),
    (2, 3, 8, 16, 64, 64, 64, False), (1, 4, 8, 16, 3, 0, 32, False),
    (1, 3, 8, 8, 32, 0, 64, False)])
def test_conv3d_wgrad(ops, N, D, H, W, C1, C2, Cout, pro):
    # 3-D weight gradient: LDS-DMA kernel (one depth tap plane per workgroup, W >= 16) and
    # the legacy kernel (W < 16)
    torch.manual_seed(13)
    x1 = torch.randn(N, C1, D, H, W, device=DEV).bfloat16()
    x2 = torch.randn(N, C2, D, H, W, device=DEV).bfloat16() if C2 else None
    dy = torch.randn(N, Cout, D, H, W, device=DEV).bfloat16()
    scale = shift = None
    a1 = x1.float()
    if pro:
        scale = torch.rand(C1, device=DEV) + 0.5
        shift = torch.randn(C1, device=DEV) * 0.5
        bc = (None, slice(None), None, None, None)
        a1 = torch.relu(x1.float() * scale[bc] + shift[bc]).bfloat16().float()
    xin = torch.cat([a1, x2.float()], 1) if x2 is not None else a1
    xin1 = ops.to_nhwc_bf16(x1, 8) if C1 % 8 else nhwc(x1)
    dw = ops.conv3_wgrad(nhwc(dy), xin1, nhwc(x2) if x2 is not None else None, scale, shift)
    dw = dw[:, :C1 + C2]
    w = torch.zeros(Cout, C1 + C2, 3, 3, 3, device=DEV, requires_grad=True)
    (g,) = torch.autograd.grad(F.conv3d(xin, w, padding=1), w, dy.float())
    assert dw.shape == g.shape
    assert rel_err(dw, g) < 5e-3


def _bn4(C, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    mean = torch.randn(C, device=DEV, generator=g) * 0.2
    invstd = torch.rand(C, device=DEV, generator=g) + 0.5
    scale = torch.randn(C, device=DEV, generator=g)
    shift = torch.randn(C, device=DEV, generator=g) * 0.3
    return torch.stack([mean, invstd, scale, shift]).contiguous()


@pytest.mark.parametrize("Cin,Cout,H", [(64, 64, 16), (128, 64, 12), (128, 128, 8), (512, 256, 8),
                                        (256, 128, 12)])
def test_deferred_bn_consumers_match_materialised(ops, Cin, Cout, H):
    """Deferred BatchNorm activations (engine: block output kept pre-BN, BN + ReLU applied
    on load by the transposed-conv / head kernels) equal the materialised path bit for bit,
    and the BN-backward partial sums emitted by the consumers' backward epilogues give the
    same BatchNorm backward as the standalone reduction pass.  (Cin, Cout) cover the
    resident-weight convT kernels' 128- and 64-wide n tiles in both directions; H = 12
    leaves a partial 128-pixel tile; 512 / 256 input channels take the GEMM data gradient,
    whose BN-partial rows are one per launched tile, each fully written.)"""
    torch.manual_seed(11)
    N, W, C = 2, H, Cin
    y = torch.randn(N, H, W, C, device=DEV).bfloat16()
    bn4 = _bn4(C, 1)
    a = ops.bn_relu_apply(y, bn4, False)[0]                     # materialised activation
    w = torch.randn(C, Cout, 2, 2, device=DEV) / math.sqrt(C)
    b = torch.randn(Cout, device=DEV) * 0.1
    pk = pack_conv(ops, w)
    assert torch.equal(ops.convt_fwd(y, pk.fwd, b, Cout, bn4), ops.convt_fwd(a, pk.fwd, b, Cout))
    dout = torch.randn(N, 2 * H, 2 * W, Cout, device=DEV).bfloat16()
    dw1, db1 = ops.convt_wgrad(y, dout, None, None, None, bn4)
    dw2, db2 = ops.convt_wgrad(a, dout)
    assert torch.equal(dw1, dw2) and torch.equal(db1, db2)
    dx1, part = ops.convt_dgrad(dout, pk.dgrad, C, y, bn4)
    dx2, _ = ops.convt_dgrad(dout, pk.dgrad, C)
    assert torch.equal(dx1, dx2) and part.dim() == 3 and part.shape[1:] == (2, C)
    gamma = torch.rand(C, device=DEV) + 0.5
    r_pre = ops.bn_backward(dx1, None, y, bn4, gamma, None, None, None, part)
    r_ref = ops.bn_backward(dx1, None, y, bn4, gamma, None)
    for u, v in zip(r_pre, r_ref):
        assert rel_err(u, v) < 2e-3
    if Cin != 64:
        return
    # head: C = 32, K = 6
    Ch, K = 32, 6
    yh = torch.randn(N, H, W, Ch, device=DEV).bfloat16()
    bnh = _bn4(Ch, 2)
    ah = ops.bn_relu_apply(yh, bnh, False)[0]
    wh = torch.randn(K, Ch, device=DEV) * 0.3
    bh = torch.randn(K, device=DEV) * 0.1
    lab = torch.randint(0, K, (N, H, W), device=DEV)
    o1 = ops.head_ce_fwd(yh, wh, bh, lab, -100, bnh)
    o2 = ops.head_ce_fwd(ah, wh, bh, lab, -100)
    assert torch.equal(o1, o2)
    da1, dwh1, dbh1, hpart = ops.head_ce_bwd(yh, wh, bh, lab, o1, None, -100, None, None, bnh)
    da2, dwh2, dbh2, _ = ops.head_ce_bwd(ah, wh, bh, lab, o2, None, -100)
    assert torch.equal(da1, da2) and torch.equal(dwh1, dwh2) and torch.equal(dbh1, dbh2)
    gh = torch.rand(Ch, device=DEV) + 0.5
    h_pre = ops.bn_backward(da1, None, yh, bnh, gh, None, None, None, hpart)
    h_ref = ops.bn_backward(da1, None, yh, bnh, gh, None)
    for u, v in zip(h_pre, h_ref):
        assert rel_err(u, v) < 2e-3
    assert torch.equal(ops.head_logits(yh, wh, bh, bnh), ops.head_logits(ah, wh, bh))


@pytest.mark.parametrize("C,K,H", [(32, 6, 12), (16, 3, 9), (64, 2, 8), (8, 16, 5)])
def test_head_two_pass_bn_backward(ops, C, K, H):
    """Two-pass head backward (stats pass without the dA store, then head_ce_bn_bwd: dA
    recomputed and the deferred BatchNorm's backward applied in registers) equals the
    one-pass path — head_ce_bwd storing dA, then bn_backward on it with the same partials —
    bit for bit: dWh, dbh, the BN partials, dgamma, dbeta and dY.  Odd H leaves a partial
    pixel pair / workgroup step; ignore_index pixels included."""
    torch.manual_seed(5)
    N, W = 2, H + 3
    yh = torch.randn(N, H, W, C, device=DEV).bfloat16()
    bnh = _bn4(C, 3)
    wh = torch.randn(K, C, device=DEV) * 0.3
    bh = torch.randn(K, device=DEV) * 0.1
    lab = torch.randint(0, K, (N, H, W), device=DEV)
    lab[0, 0, :2] = -100
    o = ops.head_ce_fwd(yh, wh, bh, lab, -100, bnh)
    gs = torch.tensor([0.75], device=DEV)
    gamma = torch.rand(C, device=DEV) + 0.5
    da1, dw1, db1, part1 = ops.head_ce_bwd(yh, wh, bh, lab, o, gs, -100, None, None, bnh)
    d0, dw2, db2, part2 = ops.head_ce_bwd(yh, wh, bh, lab, o, gs, -100, None, None, bnh, False)
    assert d0.numel() == 0
    assert torch.equal(dw1, dw2) and torch.equal(db1, db2) and torch.equal(part1, part2)
    ref = ops.bn_backward(da1, None, yh, bnh, gamma, None, None, None, part1)
    got = ops.head_ce_bn_bwd(yh, wh, bh, lab, o, gs, -100, bnh, part2, gamma)
    for u, v in zip(got, ref):
        assert torch.equal(u, v)
    # accumulate into caller buffers (direct-grad mode)
    dgo, dbo = torch.ones(C, device=DEV), torch.ones(C, device=DEV)
    ops.head_ce_bn_bwd(yh, wh, bh, lab, o, gs, -100, bnh, part2, gamma, dgo, dbo)
    assert torch.allclose(dgo, ref[1] + 1) and torch.allclose(dbo, ref[2] + 1)


def test_out_params_respect_bounds(ops):
    """Kernels that write into caller-provided buffers (in training: views into the one flat
    fp32 gradient buffer) are given views into sentinel-filled guard buffers; the guard
    regions on both sides must come back untouched (bounds checking)."""
    torch.manual_seed(12)
    G, S = 4099, 12345.0

    def guarded(*shape):
        n = math.prod(shape)
        buf = torch.full((n + 2 * G,), S, device=DEV)
        v = buf[G:G + n]
        v.zero_()
        return buf, v.view(*shape)

    def intact(buf, v):
        n = v.numel()
        return bool((buf[:G] == S).all()) and bool((buf[G + n:] == S).all())

    N, H, W, Ci, Co = 2, 24, 40, 32, 64
    x = torch.randn(N, H, W, Ci, device=DEV).bfloat16()
    dy = torch.randn(N, H, W, Co, device=DEV).bfloat16()
    b, v = guarded(Co, Ci, 3, 3)
    ops.conv3_wgrad(dy, x, None, None, None, v)
    assert intact(b, v) and bool(v.abs().sum() > 0)
    y = torch.randn(N, H, W, Co, device=DEV).bfloat16()
    bg, vg = guarded(Co)
    bb, vb = guarded(Co)
    ops.bn_backward(dy, None, y, _bn4(Co, 3), torch.rand(Co, device=DEV) + 0.5, None, vg, vb)
    assert intact(bg, vg) and intact(bb, vb)
    xt = torch.randn(N, 8, 8, 64, device=DEV).bfloat16()
    dout = torch.randn(N, 16, 16, 64, device=DEV).bfloat16()
    bw, vw = guarded(64, 64, 2, 2)
    bdb, vdb = guarded(64)
    ops.convt_wgrad(xt, dout, vw, vdb)
    assert intact(bw, vw) and intact(bdb, vdb)
    a = torch.relu(torch.randn(N, H, W, 32, device=DEV)).bfloat16()
    wh = torch.randn(6, 32, device=DEV) * 0.3
    bh = torch.zeros(6, device=DEV)
    lab = torch.randint(0, 6, (N, H, W), device=DEV)
    out3 = ops.head_ce_fwd(a, wh, bh, lab, -100)
    bhw, vhw = guarded(6, 32)
    bhb, vhb = guarded(6)
    ops.head_ce_bwd(a, wh, bh, lab, out3, None, -100, vhw, vhb)
    assert intact(bhw, vhw) and intact(bhb, vhb)
    n = 10_003
    bufs = [guarded(n) for _ in range(4)]
    p, g, m, v2 = (t for _, t in bufs)
    p.copy_(torch.randn(n, device=DEV))
    g.copy_(torch.randn(n, device=DEV))
    ops.adam_step(p, g, m, v2, 0.9, 0.999, 1e-8, 0.0, 1e-3, 1.0)
    assert all(intact(bb_, t) for bb_, t in bufs)


@pytest.mark.parametrize("H,C1,C2,Cout", [(32, 64, 32, 32), (16, 128, 64, 64), (64, 32, 32, 32)])
def test_deferred_skip_prologue_matches_materialised(ops, H, C1, C2, Cout):
    """Deferred skip (encoder a2 never materialised): the concat conv's X2 prologue applies
    BN + ReLU on load in the forward kernels (resident / streaming) and the weight-gradient
    kernels bit-identically to the materialised activation; bn_relu_apply(full=False) writes
    the same pooled tensor."""
    torch.manual_seed(21)
    N, W = 2, H
    up = torch.randn(N, H, W, C1, device=DEV).bfloat16()
    y = torch.randn(N, H, W, C2, device=DEV).bfloat16()
    bn4 = _bn4(C2, 3)
    a, p_full = ops.bn_relu_apply(y, bn4, True)
    _, p_def = ops.bn_relu_apply(y, bn4, True, False)
    assert torch.equal(p_full, p_def)
    w = torch.randn(Cout, C1 + C2, 3, 3, device=DEV) / math.sqrt(9 * (C1 + C2))
    pk = pack_conv(ops, w)
    b = torch.randn(Cout, device=DEV) * 0.1
    y_mat, _, st_mat = ops.conv3_fwd(up, a, pk.fwd, b, None, None, Cout, 0, True)
    y_def, _, st_def = ops.conv3_fwd(up, y, pk.fwd, b, None, None, Cout, 0, True, bn4[2], bn4[3])
    assert torch.equal(y_mat, y_def) and torch.equal(st_mat, st_def)
    dy = torch.randn(N, H, W, Cout, device=DEV).bfloat16()
    dw_mat = ops.conv3_wgrad(dy, up, a, None, None)
    dw_def = ops.conv3_wgrad(dy, up, y, None, None, None, bn4[2], bn4[3])
    assert torch.equal(dw_mat, dw_def)


def test_meter_add_single_launch(ops):
    """DeviceMeter on the HIP path (meter_add: one launch) accumulates exactly what the
    elementwise path does: fp64 sums of loss, correct, pixels and the micro-batch count."""
    from ddlpc.utils.metrics import DeviceMeter
    m = DeviceMeter(DEV)
    out3 = torch.tensor([0.75, 1000.0, 4096.0], device=DEV)
    for k in range(3):
        m.add(out3[0] * (k + 1), out3[1], 4096)
    torch.cuda.synchronize()
    assert m.buf.tolist() == [0.75 * 6, 3000.0, 3 * 4096.0, 3.0]
    r = m.reduce()
    assert abs(r["loss"] - 1.5) < 1e-12 and abs(r["pixel_acc"] - 1000.0 / 4096.0) < 1e-12


# ------------------------------------------------------------------ per-micro-batch BN groups
def bn_relu_pool_backward_oracle(y, dA, dP, gamma, beta, eps, s4):
    """fp32 autograd through train-mode BatchNorm + ReLU (+ 2x2 max-pool) of ONE statistics
    group (channel-last y [n, H, W, C]): -> (dY, dgamma, dbeta).  The ReLU mask and the
    pool's arg-max come from the kernels' bf16-rounded activation fma(y, scale, shift) (the
    values the forward stored), so a bf16 tie cannot route the pooled gradient elsewhere;
    every gradient value is fp32 autograd of the BatchNorm formula."""
    x = nchw(y).float().detach().requires_grad_(True)
    g = gamma.detach().clone().requires_grad_(True)
    b = beta.detach().clone().requires_grad_(True)
    z = F.batch_norm(x, None, None, g, b, training=True, eps=eps)
    sc, sh = s4[2].view(1, -1, 1, 1), s4[3].view(1, -1, 1, 1)
    zk = torch.addcmul(sh, nchw(y).float(), sc).bfloat16().float().detach()
    a = torch.where(zk > 0, z, torch.zeros_like(z))
    loss = (a * (nchw(dA).float() if dA is not None else 0)).sum()
    if dP is not None:
        _, idx = F.max_pool2d(torch.relu(zk), 2, return_indices=True)
        pooled = torch.gather(a.flatten(2), 2, idx.flatten(2)).view_as(idx)
        loss = loss + (pooled * nchw(dP).float()).sum()
    loss.backward()
    return x.grad.permute(0, 2, 3, 1), g.grad, b.grad


@pytest.mark.parametrize("G,n,H,W,C,pool", [(5, 1, 32, 32, 32, True), (3, 2, 16, 16, 256, False),
                                            (4, 1, 64, 64, 64, False), (50, 1, 16, 16, 128, True),
                                            (2, 1, 8, 8, 256, False), (2, 1, 16, 16, 512, True),
                                            (3, 2, 8, 8, 1024, True)])
def test_bn_group_kernels(ops, G, n, H, W, C, pool):
    """bn_group_finalize / bn_group_apply / bn_group_backward (a batched window of G
    micro-batches, each its own BatchNorm statistics group) against the fp32 per-group
    oracle and the single-group kernels run group by group."""
    torch.manual_seed(G * 7 + C)
    N = G * n
    y = (torch.randn(N, H, W, C, device=DEV) * 2 + 0.5).bfloat16()
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.3
    eps = 1e-5
    arena = torch.zeros(G, 3 * C + 16, device=DEV)
    s4 = ops.bn_group_finalize(y, G, gamma, beta, eps, arena, 16)
    assert s4.shape == (G, 4, C)
    yg = y.float().view(G, n * H * W, C).double()
    mean = yg.mean(1)
    var = yg.var(1, unbiased=False)
    inv = 1.0 / torch.sqrt(var + eps)
    assert torch.allclose(s4[:, 0].double(), mean, rtol=1e-5, atol=1e-6)
    assert torch.allclose(s4[:, 1].double(), inv, rtol=1e-5)
    sc = gamma.double() * inv
    assert torch.allclose(s4[:, 2].double(), sc, rtol=1e-5)
    assert torch.allclose(s4[:, 3].double(), beta.double() - mean * sc, rtol=1e-5, atol=1e-5)
    assert torch.allclose(arena[:, 16:16 + C].double(), mean, rtol=1e-5, atol=1e-6)
    assert torch.allclose(arena[:, 16 + C:16 + 2 * C].double(), yg.var(1, unbiased=True), rtol=1e-5)
    # apply (+ pool)
    a, p = ops.bn_group_apply(y, s4, G, pool)
    ref = torch.relu(y.float().view(G, -1, C) * s4[:, 2][:, None] + s4[:, 3][:, None])
    ref = ref.view(N, H, W, C)
    # (the kernel rounds fma(y, scale, shift) once; the oracle rounds the product first)
    assert float((a.float() - ref).abs().max()) <= 1e-2 * float(ref.abs().max())
    assert rel_err(a, ref) < 3e-3
    if pool:
        pr = F.max_pool2d(nchw(a).float(), 2)        # max over the stored activations
        assert torch.equal(nchw(p).float(), pr)
    # backward vs fp32 autograd through BatchNorm + ReLU (+ pool) per group, and vs the
    # single-group kernel run group by group
    dA = torch.randn(N, H, W, C, device=DEV).bfloat16()
    dP = torch.randn(N, H // 2, W // 2, C, device=DEV).bfloat16() if pool else None
    dg = torch.zeros(C, device=DEV)
    db = torch.zeros(C, device=DEV)
    dY, _, _ = ops.bn_group_backward(dA, dP, y, s4, gamma, G, dg, db)
    dg_ref = torch.zeros(C, device=DEV, dtype=torch.float64)
    db_ref = torch.zeros(C, device=DEV, dtype=torch.float64)
    dg_k = torch.zeros(C, device=DEV, dtype=torch.float64)
    for g in range(G):
        sl = slice(g * n, (g + 1) * n)
        dPg = dP[sl].contiguous() if pool else None
        dYo, dgo, dbo = bn_relu_pool_backward_oracle(y[sl], dA[sl], dPg, gamma, beta, eps, s4[g])
        assert rel_err(dY[sl], dYo) < 1e-2, (g, rel_err(dY[sl], dYo))
        dg_ref += dgo.double()
        db_ref += dbo.double()
        dYg, dgg, _ = ops.bn_backward(dA[sl].contiguous(), dPg, y[sl].contiguous(),
                                      s4[g].contiguous(), gamma, None)
        assert rel_err(dY[sl], dYg) < 2e-3, g
        dg_k += dgg.double()
    assert torch.allclose(dg.double(), dg_ref, rtol=1e-3, atol=1e-2 * float(dg_ref.abs().max())), \
        float((dg.double() - dg_ref).abs().max())
    assert torch.allclose(db.double(), db_ref, rtol=1e-3, atol=1e-3 * float(db_ref.abs().max()) + 1e-3)
    assert torch.allclose(dg.double(), dg_k, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("G,n,H,W,Cin,Cmid", [(2, 1, 256, 256, 32, 32), (3, 2, 64, 64, 64, 64),
                                              (4, 1, 128, 128, 8, 32), (50, 1, 16, 16, 64, 128),
                                              (2, 2, 96, 80, 32, 64)])
def test_conv_bn_group_fusion(ops, G, n, H, W, Cin, Cmid):
    """The fused BN-group path of a batched window (``UNetEngine.group_fused``): convs walking
    their tiles group-major write per-group statistic rows (forward (sum, sum^2), and the
    BN-backward partials of the data gradient), the second conv and its weight gradient apply
    each group's BN + ReLU on load.  Against fp32 torch per group and the unfused kernels."""
    torch.manual_seed(G * 13 + Cmid)
    N = G * n
    x = torch.randn(N, H, W, Cin, device=DEV).bfloat16()
    w1 = torch.randn(Cmid, Cin, 3, 3, device=DEV) / math.sqrt(9 * Cin)
    w2 = torch.randn(Cmid, Cmid, 3, 3, device=DEV) / math.sqrt(9 * Cmid)
    b1 = torch.randn(Cmid, device=DEV) * 0.1
    gamma = torch.rand(Cmid, device=DEV) + 0.5
    beta = torch.randn(Cmid, device=DEV) * 0.3
    eps = 1e-5
    pk1, pk2 = pack_conv(ops, w1), pack_conv(ops, w2)
    count = float(n * H * W)
    # conv1: group-major statistic rows
    y1, _, r1 = ops.conv3_fwd(x, None, pk1.fwd, b1, None, None, Cmid, 0, True, None, None, None, None, G)
    assert r1.shape[0] % G == 0 and r1.shape[1:] == (2, Cmid)
    ref1 = F.conv2d(nchw(x).float(), w1.bfloat16().float(), b1, padding=1)
    assert rel_err(nchw(y1), ref1) < 1e-2
    rows = r1.view(G, -1, 2, Cmid).sum(1)
    for g in range(G):
        rg = ref1[g * n:(g + 1) * n]
        assert torch.allclose(rows[g, 0], rg.sum((0, 2, 3)), rtol=1e-3, atol=1e-1)
        assert torch.allclose(rows[g, 1], (rg * rg).sum((0, 2, 3)), rtol=1e-3, atol=1e-1)
    s1 = ops.bn_group_finalize_rows(r1, G, count, gamma, beta, eps)
    s1y = ops.bn_group_finalize(y1, G, gamma, beta, eps)       # (statistics of the bf16 y)
    assert torch.allclose(s1[:, 0], s1y[:, 0], rtol=1e-2, atol=1e-3)
    assert torch.allclose(s1[:, 1], s1y[:, 1], rtol=1e-2)
    # conv2 with the per-group BN1 + ReLU prologue
    y2, _, r2 = ops.conv3_fwd(y1, None, pk2.fwd, None, s1[:, 2], s1[:, 3], Cmid, 0, True,
                              None, None, None, None, G)
    a1 = torch.relu(y1.float().view(G, -1, Cmid) * s1[:, 2][:, None] + s1[:, 3][:, None])
    a1 = a1.bfloat16().float().view(N, H, W, Cmid)
    ref2 = F.conv2d(nchw(a1), w2.bfloat16().float(), None, padding=1)
    assert rel_err(nchw(y2), ref2) < 1e-2, rel_err(nchw(y2), ref2)
    rows2 = r2.view(G, -1, 2, Cmid).sum(1)
    assert torch.allclose(rows2[:, 0], ref2.view(G, n, Cmid, H, W).sum((1, 3, 4)), rtol=2e-3, atol=0.5)
    # weight gradient of conv2 with the per-group prologue
    dy = (torch.randn(N, H, W, Cmid, device=DEV) * 0.1).bfloat16()
    dW = ops.conv3_wgrad(dy, y1, None, s1[:, 2], s1[:, 3], groups=G)
    dW_ref = torch.nn.grad.conv2d_weight(nchw(a1), w2.shape, nchw(dy).float(), padding=1)
    assert rel_err(dW.view_as(dW_ref), dW_ref) < 1e-2, rel_err(dW.view_as(dW_ref), dW_ref)
    # data gradient with the per-group BN-backward epilogue vs the unfused kernels group by group
    da, _, part = ops.conv3_fwd(dy, None, pk2.dgrad, None, None, None, Cmid, 0, False,
                                None, None, y1, s1, G)
    assert part.shape[0] % G == 0
    prow = part.view(G, -1, 2, Cmid).sum(1)
    for g in range(G):
        sl = slice(g * n, (g + 1) * n)
        da_g, _, part_g = ops.conv3_fwd(dy[sl].contiguous(), None, pk2.dgrad, None, None, None, Cmid,
                                        0, False, None, None, y1[sl].contiguous(), s1[g].contiguous())
        assert rel_err(da[sl], da_g) < 1e-2
        pg = part_g.sum(0)
        assert torch.allclose(prow[g], pg, rtol=1e-3, atol=1e-3 * float(pg.abs().max()) + 1e-4), g
    dg0, db0 = torch.zeros(Cmid, device=DEV), torch.zeros(Cmid, device=DEV)
    dg1, db1 = torch.zeros(Cmid, device=DEV), torch.zeros(Cmid, device=DEV)
    dY0, _, _ = ops.bn_group_backward(da, None, y1, s1, gamma, G, dg0, db0)
    dY1, _, _ = ops.bn_group_backward(da, None, y1, s1, gamma, G, dg1, db1, part)
    assert rel_err(dY1, dY0) < 2e-3, rel_err(dY1, dY0)
    assert torch.allclose(dg1, dg0, rtol=2e-3, atol=2e-3 * float(dg0.abs().max()))
    assert torch.allclose(db1, db0, rtol=2e-3, atol=2e-3 * float(db0.abs().max()))


@pytest.mark.parametrize("G,n,H,W,K", [(4, 1, 32, 32, 6), (3, 2, 16, 24, 6), (50, 1, 16, 16, 6),
                                       (2, 1, 64, 48, 16)])
def test_head_bn_groups(ops, G, n, H, W, K):
    """The C = 32 head with the last decoder block's BatchNorm deferred in a batched window
    of G micro-batches (per-group statistics, group-major workgroups): the fused training
    forward (loss, hits, dWh rows, BN partial rows) and the two-pass backward's per-group BN
    apply against fp32 autograd through each group's BatchNorm + ReLU, the 1x1 head and the
    cross-entropy over the whole window."""
    torch.manual_seed(G * 3 + K)
    C, N = 32, G * n
    eps = 1e-5
    y = (torch.randn(N, H, W, C, device=DEV) * 1.5 + 0.3).bfloat16()
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.3
    s4 = ops.bn_group_finalize(y, G, gamma, beta, eps)
    wh = torch.randn(K, C, device=DEV) * 0.3
    bh = torch.randn(K, device=DEV) * 0.1
    lab = torch.randint(0, K, (N, H, W), device=DEV)
    lab[0, 0, :3] = -100
    out3, wrows, brows = ops.head_ce_fwd_stats(y, wh, bh, lab, -100, s4, G)
    assert brows.shape[0] % G == 0
    # fp32 reference: per-group BN + ReLU as the kernel forms it (fma, bf16, max 0)
    sc = s4[:, 2].repeat_interleave(n, 0)[:, None, None, :]
    sh = s4[:, 3].repeat_interleave(n, 0)[:, None, None, :]
    a = torch.relu(torch.addcmul(sh, y.float(), sc).bfloat16().float()).requires_grad_(True)
    w_ = wh.clone().requires_grad_(True)
    b_ = bh.clone().requires_grad_(True)
    logits = a @ w_.t() + b_
    loss = F.cross_entropy(logits.reshape(-1, K), lab.reshape(-1), ignore_index=-100)
    loss.backward()
    valid = lab != -100
    hits = ((logits.argmax(-1) == lab) & valid).sum()
    assert abs(float(out3[0]) - float(loss)) <= 2e-3 * float(loss), (float(out3[0]), float(loss))
    assert float(out3[2]) == float(valid.sum())
    assert abs(float(out3[1]) - float(hits)) <= 0.002 * float(valid.sum()) + 2
    scale = ops.head_grad_scale(out3, None)
    dw, db = ops.head_wgrad_from_rows(wrows, scale, K, C)
    assert rel_err(dw, w_.grad) < 1e-2 and rel_err(db, b_.grad) < 1e-2
    dY, dg, dbeta = ops.head_ce_bn_bwd(y, wh, bh, lab, out3, None, -100, s4, brows, gamma, None,
                                       None, scale, G)
    dg_ref = torch.zeros(C, device=DEV, dtype=torch.float64)
    db_ref = torch.zeros(C, device=DEV, dtype=torch.float64)
    for g in range(G):
        sl = slice(g * n, (g + 1) * n)
        dYo, dgo, dbo = bn_relu_pool_backward_oracle(y[sl], a.grad[sl], None, gamma, beta, eps, s4[g])
        assert rel_err(dY[sl], dYo) < 2e-2, (g, rel_err(dY[sl], dYo))
        dg_ref += dgo.double()
        db_ref += dbo.double()
    assert torch.allclose(dg.double(), dg_ref, rtol=1e-2, atol=2e-2 * float(dg_ref.abs().max()))
    assert torch.allclose(dbeta.double(), db_ref, rtol=1e-2, atol=2e-2 * float(db_ref.abs().max()))


@pytest.mark.parametrize("N,H,W", [(2, 32, 32), (3, 24, 40), (1, 50, 18), (300, 16, 16)])
def test_conv3_bwd32(ops, N, H, W):
    """The fused backward of a 32 -> 32-channel conv on relu(bn1(y)) (data gradient + BN1
    partials + weight gradient from one pass over dY and y) against fp32 torch and against
    the separate kernels it replaces (resident data gradient with the BN-backward epilogue,
    v3 weight gradient with the BN prologue).  Partial 16x16 tiles and more tiles than CUs
    (persistent workgroups) included."""
    torch.manual_seed(N + H)
    C = 32
    y = (torch.randn(N, H, W, C, device=DEV) * 1.3 + 0.2).bfloat16()
    dy = (torch.randn(N, H, W, C, device=DEV) * 0.1).bfloat16()
    w = torch.randn(C, C, 3, 3, device=DEV) / math.sqrt(9 * C)
    s4 = _bn4(C, 7)
    pk = pack_conv(ops, w)
    dA, part, dW = ops.conv3_bwd32(dy, y, s4, pk.dgrad)
    # fp32 references on the bf16-rounded a1 = relu(bf16(y * scale + shift))
    a1 = torch.relu(torch.addcmul(s4[3], y.float(), s4[2]).bfloat16().float())
    dW_ref = torch.nn.grad.conv2d_weight(nchw(a1), w.shape, nchw(dy).float(), padding=1)
    dA_ref = torch.nn.grad.conv2d_input(nchw(a1).shape, w.bfloat16().float(), nchw(dy).float(), padding=1)
    assert rel_err(dW, dW_ref) < 5e-3, rel_err(dW, dW_ref)
    assert rel_err(nchw(dA), dA_ref) < 1e-2, rel_err(nchw(dA), dA_ref)
    # against the kernels it replaces
    dA0, _, part0 = ops.conv3_fwd(dy, None, pk.dgrad, None, None, None, C, 0, False, None, None, y, s4)
    dW0 = ops.conv3_wgrad(dy, y, None, s4[2], s4[3])
    assert rel_err(dA, dA0) < 2e-3 and rel_err(dW, dW0) < 1e-3, (rel_err(dA, dA0), rel_err(dW, dW0))
    ps, ps0 = part.sum(0), part0.sum(0)
    assert torch.allclose(ps, ps0, rtol=2e-3, atol=2e-3 * float(ps0.abs().max())), \
        float((ps - ps0).abs().max())
    # accumulate into a caller buffer (direct-grad mode)
    acc = torch.ones_like(w)
    _, _, none = ops.conv3_bwd32(dy, y, s4, pk.dgrad, acc)
    assert none.numel() == 0 and torch.allclose(acc, dW + 1, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("G,n,H,W", [(4, 1, 32, 32), (3, 2, 24, 40), (50, 1, 16, 16)])
def test_conv3_bwd32_groups(ops, G, n, H, W):
    """The fused 32-channel backward in a batched window (per-group BN1 statistics, group-
    major workgroups): each group's partial rows and data gradient equal the single-group
    kernel run on that group; the weight gradient is the sum over groups."""
    torch.manual_seed(G * 5 + H)
    C, N = 32, G * n
    y = (torch.randn(N, H, W, C, device=DEV) * 1.3 + 0.2).bfloat16()
    dy = (torch.randn(N, H, W, C, device=DEV) * 0.1).bfloat16()
    w = torch.randn(C, C, 3, 3, device=DEV) / math.sqrt(9 * C)
    s4 = torch.stack([_bn4(C, 11 + g) for g in range(G)]).contiguous()
    pk = pack_conv(ops, w)
    dA, part, dW = ops.conv3_bwd32(dy, y, s4, pk.dgrad, None, G)
    assert part.shape[0] % G == 0
    rows = part.view(G, -1, 2, C).sum(1)
    dW_sum = torch.zeros_like(dW)
    for g in range(G):
        sl = slice(g * n, (g + 1) * n)
        dA_g, part_g, dW_g = ops.conv3_bwd32(dy[sl].contiguous(), y[sl].contiguous(), s4[g].contiguous(),
                                             pk.dgrad)
        assert rel_err(dA[sl], dA_g) < 1e-3, g
        pg = part_g.sum(0)
        assert torch.allclose(rows[g], pg, rtol=1e-3, atol=1e-3 * float(pg.abs().max()) + 1e-5), g
        dW_sum += dW_g
    assert rel_err(dW, dW_sum) < 1e-4


@pytest.mark.parametrize("N,D,H,W,pro,bias", [(4, 6, 128, 128, True, True), (4, 5, 120, 120, False, True),
                                              (2, 3, 256, 136, True, False), (300, 2, 16, 16, False, False)])
def test_conv3d_depth_streaming(ops, N, D, H, W, pro, bias):
    """The 3-D 32 -> 32-channel depth-streaming resident kernel (conv3x3x3_ds.hip; chosen by
    conv3_fwd when the layer has at least one 16x16 tile column per CU) against F.conv3d:
    output, bias, BN prologue, statistics rows; partial (h, w) tiles, shallow volumes (the
    first / last planes skip the missing depth taps) and more columns than CUs."""
    torch.manual_seed(D * 7 + H)
    C = 32
    x = torch.randn(N, C, D, H, W, device=DEV).bfloat16()
    w = torch.randn(C, C, 3, 3, 3, device=DEV) / math.sqrt(27 * C)
    b = torch.randn(C, device=DEV) * 0.1 if bias else None
    scale = torch.rand(C, device=DEV) + 0.5 if pro else None
    shift = torch.randn(C, device=DEV) * 0.5 if pro else None
    pk = pack_conv(ops, w)
    y, _, st = ops.conv3_fwd(nhwc(x), None, pk.fwd, b, scale, shift, C, 0, True)
    a1 = x.float()
    if pro:
        a1 = torch.relu(a1 * scale.view(1, -1, 1, 1, 1) + shift.view(1, -1, 1, 1, 1)).bfloat16().float()
    ref = F.conv3d(a1, w.bfloat16().float(), b, padding=1)
    assert rel_err(nchw(y), ref) < 1e-2, rel_err(nchw(y), ref)
    assert_stats(st, ref, 1.0, 10.0)
    # data-gradient use (flipped, transposed pack; no prologue)
    dy = torch.randn(N, D, H, W, C, device=DEV).bfloat16()
    dx, _, _ = ops.conv3_fwd(dy, None, pk.dgrad, None, None, None, C, 0, False)
    dref = torch.nn.grad.conv3d_input(a1.shape, w.bfloat16().float(), nchw(dy).float(), padding=1)
    assert rel_err(nchw(dx), dref) < 1e-2, rel_err(nchw(dx), dref)


@pytest.mark.parametrize("N,H,W,C1,C2,pro,pro2", [
    (32, 128, 128, 32, 64, True, True), (40, 120, 136, 32, 64, False, True),
    (32, 128, 128, 32, 32, True, False)])
def test_conv3_wgrad_c32_all_chunks(ops, N, H, W, C1, C2, pro, pro2):
    """The 2-D weight gradient of the 32-output-channel concat convs with every input chunk
    per workgroup (conv3x3_wgrad_c32.hip; dec1.a) against the fp32 autograd weight gradient:
    BN prologues on either input, partial tiles, 2 and 3 input chunks."""
    torch.manual_seed(H + C2)
    x1 = torch.randn(N, C1, H, W, device=DEV).bfloat16()
    x2 = torch.randn(N, C2, H, W, device=DEV).bfloat16()
    dy = torch.randn(N, 32, H, W, device=DEV).bfloat16()
    bc = (None, slice(None), None, None)

    def pro_of(x, C, on):
        if not on:
            return x.float(), None, None
        sc = torch.rand(C, device=DEV) + 0.5
        sh = torch.randn(C, device=DEV) * 0.5
        return torch.relu(x.float() * sc[bc] + sh[bc]).bfloat16().float(), sc, sh

    a1, s1, h1 = pro_of(x1, C1, pro)
    a2, s2, h2 = pro_of(x2, C2, pro2)
    dw = ops.conv3_wgrad(nhwc(dy), nhwc(x1), nhwc(x2), s1, h1, None, s2, h2)
    w = torch.zeros(32, C1 + C2, 3, 3, device=DEV, requires_grad=True)
    (g,) = torch.autograd.grad(F.conv2d(torch.cat([a1, a2], 1), w, padding=1), w, dy.float())
    assert dw.shape == g.shape
    assert rel_err(dw, g) < 5e-3, rel_err(dw, g)


@pytest.mark.parametrize("H,W,C1,C2", [(256, 256, 64, 32), (240, 264, 32, 32)])
def test_conv3_wgrad_c32_bn_prologue_emits_dy(ops, H, W, C1, C2):
    """dec1.a's weight gradient with BN1's backward applied on load (conv3x3_wgrad_c32.hip, dY
    prologue): the kernel forms dY = k (dA [y*scale + shift > 0] - m1 - xhat m2) from dA and y
    in LDS, stores it (dy_out) for the data gradient, and its weight gradient equals the plain
    c32 kernel's on that stored dY bit for bit.  dY against the fp32 formula, dW against fp32
    autograd; partial tiles in the second case."""
    ncu = int(ops.set_cu_reserve(-1))
    tiles = -(-H // 16) * -(-W // 16)
    N = -(-8 * ncu // tiles)                     # the c32 kernel's eligibility: 8 tiles per CU
    torch.manual_seed(H + C1)
    x1 = nhwc(torch.randn(N, C1, H, W, device=DEV).bfloat16())
    x2 = nhwc(torch.randn(N, C2, H, W, device=DEV).bfloat16())
    da = nhwc((torch.randn(N, 32, H, W, device=DEV) * 1e-2).bfloat16())
    y = nhwc(torch.randn(N, 32, H, W, device=DEV).bfloat16())
    mean = torch.randn(32, device=DEV) * 0.1
    inv = torch.rand(32, device=DEV) + 0.5
    sc = (torch.rand(32, device=DEV) + 0.5) * inv * torch.where(torch.arange(32, device=DEV) % 5 == 0, -1.0, 1.0)
    sh = torch.randn(32, device=DEV) * 0.3
    s4 = torch.stack([mean, inv, sc, sh]).contiguous()
    coefs = torch.stack([torch.rand(32, device=DEV) + 0.5, torch.randn(32, device=DEV) * 1e-3,
                         torch.randn(32, device=DEV) * 1e-3]).contiguous()
    dy_out = torch.empty_like(da)
    dw = ops.conv3_wgrad(da, x1, x2, None, None, None, None, None, y, s4, coefs, dy_out=dy_out)
    # dY against the formula (fp32; the kernel's fused multiply-adds may round 1 bf16 ulp apart)
    yf, df = y.float(), da.float()
    a = yf * sc + sh
    dyh = torch.where(a > 0, df, torch.zeros_like(df))
    xh = yf * inv - mean * inv
    ref = coefs[0] * (dyh - coefs[1] - xh * coefs[2])
    assert rel_err(dy_out, ref) < 5e-3, rel_err(dy_out, ref)
    assert float((dy_out.float() - ref.bfloat16().float()).ne(0).float().mean()) < 1e-2
    # the weight gradient is the plain kernel's on the stored dY, bit for bit
    dw_plain = ops.conv3_wgrad(dy_out, x1, x2, None, None)
    assert torch.equal(dw, dw_plain)
    w = torch.zeros(32, C1 + C2, 3, 3, device=DEV, requires_grad=True)
    (g,) = torch.autograd.grad(F.conv2d(torch.cat([nchw(x1).float(), nchw(x2).float()], 1), w,
                                        padding=1), w, nchw(dy_out).float())
    assert rel_err(dw, g) < 5e-3, rel_err(dw, g)


@pytest.mark.parametrize("N,D,H,W,Cout,co1,pro,bias", [
    (2, 5, 128, 120, 64, 0, True, True), (2, 4, 96, 136, 96, 32, False, False),
    (1, 3, 256, 256, 96, 64, False, True)])
def test_conv3d_depth_streaming_chunks(ops, N, D, H, W, Cout, co1, pro, bias):
    """The depth-streaming 3-D conv with several 32-channel output chunks (conv3x3x3_ds.hip:
    enc2.a's 32 -> 64 forward, dec1.a's 32 -> 96 data gradient split into the two concat
    inputs' gradients): outputs, bias, prologue and the per-workgroup statistics rows (chunks a
    workgroup never met are zero) against F.conv3d; item ranges cross chunk boundaries."""
    torch.manual_seed(D * 5 + W)
    C = 32
    x = torch.randn(N, C, D, H, W, device=DEV).bfloat16()
    w = torch.randn(Cout, C, 3, 3, 3, device=DEV) / math.sqrt(27 * C)
    b = torch.randn(Cout, device=DEV) * 0.1 if bias else None
    scale = torch.rand(C, device=DEV) + 0.5 if pro else None
    shift = torch.randn(C, device=DEV) * 0.5 if pro else None
    pk = pack_conv(ops, w, need_dgrad=False)
    y1, y2, st = ops.conv3_fwd(nhwc(x), None, pk.fwd, b, scale, shift, Cout, co1, True)
    a1 = x.float()
    if pro:
        a1 = torch.relu(a1 * scale.view(1, -1, 1, 1, 1) + shift.view(1, -1, 1, 1, 1)).bfloat16().float()
    ref = F.conv3d(a1, w.bfloat16().float(), b, padding=1)
    c1 = co1 if co1 else Cout
    assert y1.shape[-1] == c1 and (co1 == 0 or y2.shape[-1] == Cout - co1)
    assert rel_err(nchw(y1), ref[:, :c1]) < 1e-2, rel_err(nchw(y1), ref[:, :c1])
    if co1:
        assert rel_err(nchw(y2), ref[:, c1:]) < 1e-2, rel_err(nchw(y2), ref[:, c1:])
    assert st.shape[-1] == Cout
    assert_stats(st, ref, 1.0, 10.0)


@pytest.mark.parametrize("N,D,H,W,C1,C2,pro,pro2", [
    (4, 6, 128, 128, 32, 0, True, False), (2, 5, 120, 120, 32, 64, True, True),
    (300, 4, 16, 16, 32, 0, False, False), (1, 4, 256, 136, 64, 32, False, True),
    (2, 24, 64, 64, 32, 32, True, False)])
def test_conv3d_wgrad_depth_streaming(ops, N, D, H, W, C1, C2, pro, pro2):
    """The depth-streaming 3-D weight gradient of the 32-output-channel layers
    (conv3x3x3_wgrad_ds.hip; chosen by conv3_wgrad when (input chunk, tile column) pairs fill
    the chip) against the fp32 autograd weight gradient: BN prologues on either input of a
    concat, partial (h, w) tiles, shallow volumes (missing depth taps), uneven item ranges
    crossing chunk boundaries, depth segments (the last shape: 4 segments of 6 planes)."""
    _wgrad_ds_check(ops, N, D, H, W, C1, C2, 32, pro, pro2)


@pytest.mark.parametrize("N,D,H,W,C1,C2,Cout,pro,pro2", [
    (8, 8, 64, 64, 64, 0, 64, True, False), (4, 6, 64, 64, 64, 64, 64, False, True),
    (2, 8, 80, 72, 32, 32, 96, True, True)])
def test_conv3d_wgrad_depth_streaming_co_chunks(ops, N, D, H, W, C1, C2, Cout, pro, pro2):
    """The depth-streaming 3-D weight gradient with several 32-channel output chunks (the 64^3
    level: items = (output chunk, input chunk) pairs x columns x depth segments) against the
    fp32 autograd weight gradient."""
    _wgrad_ds_check(ops, N, D, H, W, C1, C2, Cout, pro, pro2)


def _wgrad_ds_check(ops, N, D, H, W, C1, C2, Cout, pro, pro2):
    torch.manual_seed(D * 11 + H + C2 + Cout)
    x1 = torch.randn(N, C1, D, H, W, device=DEV).bfloat16()
    x2 = torch.randn(N, C2, D, H, W, device=DEV).bfloat16() if C2 else None
    dy = torch.randn(N, Cout, D, H, W, device=DEV).bfloat16()
    bc = (None, slice(None), None, None, None)

    def pro_of(x, C, on):
        if not on:
            return x.float(), None, None
        sc = torch.rand(C, device=DEV) + 0.5
        sh = torch.randn(C, device=DEV) * 0.5
        return torch.relu(x.float() * sc[bc] + sh[bc]).bfloat16().float(), sc, sh

    a1, s1, h1 = pro_of(x1, C1, pro)
    xin = a1
    s2 = h2 = None
    if x2 is not None:
        a2, s2, h2 = pro_of(x2, C2, pro2)
        xin = torch.cat([a1, a2], 1)
    dw = ops.conv3_wgrad(nhwc(dy), nhwc(x1), nhwc(x2) if x2 is not None else None, s1, h1,
                         None, s2, h2)
    w = torch.zeros(Cout, C1 + C2, 3, 3, 3, device=DEV, requires_grad=True)
    (g,) = torch.autograd.grad(F.conv3d(xin, w, padding=1), w, dy.float())
    assert dw.shape == g.shape
    assert rel_err(dw, g) < 5e-3, rel_err(dw, g)
