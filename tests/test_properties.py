"""Hypothesis property tests ("Hypothesis-generated shapes").

CPU part: the lossy gradient codec against the reference formulas (ref.py:354,375,304,313)
for arbitrary sizes / magnitudes / segmentations, and the U-Net's shape contract for
arbitrary (depth, width divisor, up-sample mode, tile).

GPU part (``-m gpu``): the hand-written kernels on generated geometries — odd and
non-power-of-two H/W, batch 1-3, concat inputs, BN prologue on/off — against the plain
PyTorch fp32 op on the same bf16 inputs.  Channel counts stay inside the kernels' documented
domain (multiples of 8; concat first input a multiple of 32; Cout in the U-Net's set).
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from ddlpc.parallel import codec as C

_SET = settings(max_examples=25, deadline=None,
                suppress_health_check=[HealthCheck.function_scoped_fixture,
                                       HealthCheck.too_slow])


# ----------------------------------------------------------------------------- CPU: codec
@_SET
@given(n=st.integers(1, 4000), mag=st.floats(1e-8, 1e3), seed=st.integers(0, 2**31 - 1),
       codec=st.sampled_from(["fp16_absmax", "int8_absmax"]))
def test_codec_bit_exact_any_size(n, mag, seed, codec):
    L, dtype = (100, np.float16) if codec == "fp16_absmax" else (10, np.int8)
    g = torch.randn(n, generator=torch.Generator().manual_seed(seed)) * mag
    mx = g.abs().max()
    ref_q = torch.round(g / mx * L).numpy().astype(dtype)          # ref.py:354,375
    q = C.encode(g, mx, codec)
    assert np.array_equal(q.numpy(), ref_q)
    assert int(np.abs(ref_q.astype(np.int32)).max()) <= L
    ref_d = torch.from_numpy(ref_q.astype(np.float32)) / L * mx     # ref.py:304,313
    assert torch.equal(C.decode(q, mx, codec), ref_d)


@_SET
@given(sizes=st.lists(st.integers(1, 300), min_size=1, max_size=8),
       seed=st.integers(0, 2**31 - 1), codec=st.sampled_from(["fp16_absmax", "int8_absmax"]))
def test_codec_segments_roundtrip(sizes, seed, codec):
    gen = torch.Generator().manual_seed(seed)
    parts = [torch.randn(s, generator=gen) * 10.0 ** float(torch.randint(-6, 2, (1,), generator=gen))
             for s in sizes]
    flat = torch.cat(parts)
    segs, o = [], 0
    for s in sizes:
        segs.append((o, o + s))
        o += s
    q, scales = C.encode_segments(flat, segs, codec)
    acc = torch.zeros_like(flat)
    C.decode_segments_accumulate(acc, q, scales, segs, codec)
    L = 100 if codec == "fp16_absmax" else 10
    for (a, b), p in zip(segs, parts):
        # per-segment absmax scale: error bounded by half a quantisation level of that segment
        step = float(p.abs().max()) / L
        assert float((acc[a:b] - p).abs().max()) <= 0.5 * step * (1 + 1e-3) + 1e-30


# ----------------------------------------------------------------------------- CPU: model
@settings(max_examples=12, deadline=None)
@given(depth=st.sampled_from([4, 5]), div=st.sampled_from([2, 4, 8]),
       mode=st.sampled_from(["conv_transpose", "bilinear"]), k=st.integers(1, 3),
       classes=st.integers(2, 8))
def test_unet_shape_contract(depth, div, mode, k, classes):
    from ddlpc.models import UNet
    tile = 2 ** depth * k                       # any multiple of the total down-sampling
    m = UNet(out_classes=classes, width_divisor=div, depth=depth, up_sample_mode=mode)
    with torch.no_grad():
        out = m(torch.rand(2, 3, tile, tile))   # batch 2: training-mode BN at a 1x1 bottleneck
    assert out.shape == (2, classes, tile, tile)
    assert all(k.startswith(("down_conv", "double_conv", "up_conv", "conv_last"))
               for k in m.state_dict())


# ----------------------------------------------------------------------------- GPU kernels
DEV = "cuda"


def _nhwc(x):
    return x.permute(0, *range(2, x.dim()), 1).contiguous()


def _nchw(x):
    return x.permute(0, x.dim() - 1, *range(1, x.dim() - 1))


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.fixture(scope="module")
def ops():
    from ddlpc.ops import _ext
    return _ext.ops()


def _pack(ops, w):
    from ddlpc.ops.fused_unet import _ConvPack
    conv = torch.nn.Module()
    conv.weight = torch.nn.Parameter(w.contiguous())
    pk = _ConvPack(conv, 0, True)
    ops.weight_pack(torch.tensor([pk.entry()], dtype=torch.int64, device=w.device), 1, pk.numel())
    return pk


_CH = st.sampled_from([(32, 0), (64, 0), (128, 0), (32, 32), (64, 32), (64, 64), (128, 64),
                       (256, 0)])
_CO = st.sampled_from([32, 64, 96, 128, 256])


@pytest.mark.gpu
@_SET
@given(n=st.integers(1, 3), h=st.integers(3, 40), w=st.integers(3, 40), ch=_CH, cout=_CO,
       pro=st.booleans())
def test_conv3_fwd_dgrad_wgrad_any_geometry(ops, n, h, w, ch, cout, pro):
    c1, c2 = ch
    cin = c1 + c2
    g = torch.Generator(device=DEV).manual_seed(n * 7919 + h * 31 + w)
    x1 = torch.randn(n, c1, h, w, device=DEV, generator=g).bfloat16()
    x2 = torch.randn(n, c2, h, w, device=DEV, generator=g).bfloat16() if c2 else None
    wt = torch.randn(cout, cin, 3, 3, device=DEV, generator=g) / math.sqrt(9 * cin)
    b = torch.randn(cout, device=DEV, generator=g) * 0.1
    sc = torch.rand(c1, device=DEV, generator=g) + 0.5 if pro else None
    sh = torch.randn(c1, device=DEV, generator=g) * 0.5 if pro else None
    pk = _pack(ops, wt)
    a1 = x1.float()
    if pro:
        a1 = torch.relu(a1 * sc[None, :, None, None] + sh[None, :, None, None]).bfloat16().float()
    xin = torch.cat([a1, x2.float()], 1) if c2 else a1
    wb = wt.bfloat16().float()
    # forward (+ BN statistics of the fp32 outputs, before the bf16 store)
    y, _, stt = ops.conv3_fwd(_nhwc(x1), _nhwc(x2) if c2 else None, pk.fwd, b, sc, sh, cout, 0,
                              True)
    ref_y = F.conv2d(xin, wb, b, padding=1)
    assert _rel(_nchw(y), ref_y) < 1e-2
    assert torch.allclose(stt.sum(0)[0], ref_y.sum((0, 2, 3)), rtol=1e-3, atol=1e-1)
    assert torch.allclose(stt.sum(0)[1], (ref_y * ref_y).sum((0, 2, 3)), rtol=1e-3, atol=1.0)
    # data gradient, split across the concat inputs
    dy = torch.randn(n, cout, h, w, device=DEV, generator=g).bfloat16()
    dx1, dx2, _ = ops.conv3_fwd(_nhwc(dy), None, pk.dgrad, None, None, None, cin,
                                c1 if c2 else 0, False)
    ref_dx = F.conv_transpose2d(dy.float(), wb, padding=1)
    assert _rel(_nchw(dx1), ref_dx[:, :c1]) < 1e-2
    if c2:
        assert _rel(_nchw(dx2), ref_dx[:, c1:]) < 1e-2
    # weight gradient (BN prologue re-applied on the first input)
    dw = ops.conv3_wgrad(_nhwc(dy), _nhwc(x1), _nhwc(x2) if c2 else None, sc, sh)
    wz = torch.zeros(cout, cin, 3, 3, device=DEV, requires_grad=True)
    (gw,) = torch.autograd.grad(F.conv2d(xin, wz, padding=1), wz, dy.float())
    assert _rel(dw.reshape(gw.shape), gw) < 5e-3


@pytest.mark.gpu
@_SET
@given(n=st.integers(1, 3), h2=st.integers(1, 24), w2=st.integers(1, 24),
       c=st.sampled_from([32, 64, 128, 256]), pool=st.booleans())
def test_bn_backward_any_geometry(ops, n, h2, w2, c, pool):
    h, w = 2 * h2, 2 * w2                     # max-pool needs even extents
    g = torch.Generator(device=DEV).manual_seed(n * 131 + h * 17 + w + c)
    y = (torch.randn(n, c, h, w, device=DEV, generator=g) * 2 + 0.5).bfloat16()
    gamma = torch.rand(c, device=DEV, generator=g) + 0.5
    beta = torch.randn(c, device=DEV, generator=g) * 0.1
    yf = y.float()
    part = torch.stack([yf.sum((0, 2, 3)), (yf * yf).sum((0, 2, 3))])[None].contiguous()
    s4 = ops.bn_finalize(part, float(n * h * w), gamma, beta, torch.zeros(c, device=DEV),
                         torch.ones(c, device=DEV), 0.1, 1e-5, True, None)
    bn = torch.nn.BatchNorm2d(c).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(gamma)
        bn.bias.copy_(beta)
    yr = yf.clone().requires_grad_(True)
    ar = torch.relu(bn(yr))
    a, p = ops.bn_relu_apply(_nhwc(y), s4, pool)
    assert _rel(_nchw(a), ar) < 5e-3
    dA = torch.randn(n, c, h, w, device=DEV, generator=g).bfloat16()
    dP = torch.randn(n, c, h // 2, w // 2, device=DEV, generator=g).bfloat16()
    dy, dg, db = ops.bn_backward(_nhwc(dA), _nhwc(dP) if pool else None, _nhwc(y), s4, gamma,
                                 None)
    loss = (ar * dA.float()).sum()
    if pool:   # the kernel routes the pooled gradient by the bf16 activations' arg-max
        assert _rel(_nchw(p), F.max_pool2d(_nchw(a).float(), 2)) < 1e-6
        idx = F.max_pool2d(ar.bfloat16().float(), 2, return_indices=True)[1]
        loss = loss + (ar.flatten(2).gather(2, idx.flatten(2)) * dP.float().flatten(2)).sum()
    gy, gg, gb = torch.autograd.grad(loss, [yr, bn.weight, bn.bias])
    assert _rel(_nchw(dy), gy) < 2e-2
    assert _rel(dg, gg) < 1e-2
    assert _rel(db, gb) < 1e-2
