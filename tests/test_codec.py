"""Lossy gradient codec parity with the reference formulas (ref.py:328-545) — CPU."""
import numpy as np
import pytest
import torch

from ddlpc.parallel import codec as C


@pytest.mark.parametrize("codec,L,dtype", [("fp16_absmax", 100, np.float16),
                                           ("int8_absmax", 10, np.int8)])
def test_encode_decode_bit_exact_with_reference(codec, L, dtype):
    torch.manual_seed(0)
    g = torch.randn(1000) * 1e-3
    mx = g.abs().max()
    # reference: torch.round(grad / max_grad * L).to(dtype)  (ref.py:354,375)
    ref_q = torch.round(g / mx * L).numpy().astype(dtype)
    q = C.encode(g, mx, codec)
    assert np.array_equal(q.numpy(), ref_q)
    # reference decode: from_numpy(frombuffer(b)).to(float32) / L * max_grad (ref.py:304,313)
    ref_d = torch.from_numpy(np.frombuffer(ref_q.tobytes(), dtype=dtype).copy()).to(torch.float32) / L * mx
    assert torch.equal(C.decode(q, mx, codec), ref_d)


def test_levels_used_and_zero_grad():
    g = torch.linspace(-1, 1, 1001)
    q = C.encode(g, g.abs().max(), "int8_absmax")
    assert q.min() == -10 and q.max() == 10
    z = torch.zeros(10)
    assert torch.equal(C.encode(z, z.abs().max(), "fp16_absmax").float(), z)


def test_reference_weights_match_survey_table():
    assert C.reference_weights(2) == [1.0, 1.0]                      # M=1: a sum
    w = C.reference_weights(3)
    assert w == pytest.approx([0.25, 0.25, 0.5])                     # M=2
    w4 = C.reference_weights(4)
    assert w4 == pytest.approx([1 / 27, 1 / 27, 1 / 9, 1 / 3])      # M=3
    # (SURVEY.md §2.6 lists the sum as 13/27; the weights it lists add up to 14/27)
    assert sum(w4) == pytest.approx(14 / 27)


def test_segments_roundtrip_and_global_zeroing():
    torch.manual_seed(1)
    big = torch.randn(500) * 1.0
    small = torch.randn(500) * 1e-4
    flat = torch.cat([big, small])
    # global scale zeroes the small-magnitude tensor
    q, s = C.encode_segments(flat, [(0, 1000)], "int8_absmax")
    assert int((q[500:] != 0).sum()) == 0
    # per-tensor scales keep it
    q2, s2 = C.encode_segments(flat, [(0, 500), (500, 1000)], "int8_absmax")
    assert int((q2[500:] != 0).sum()) > 100
    acc = torch.zeros(1000)
    C.decode_segments_accumulate(acc, q2, s2, [(0, 500), (500, 1000)], "int8_absmax")
    assert C.relative_l2_error(small, "int8_absmax") < 0.5
    assert float((acc[500:] - small).norm() / small.norm()) < 0.5
