"""U-Net structure parity with the reference (ref.py:575-656) — CPU."""
import pytest
import torch

from ddlpc.models import UNet


def _expected_keys(depth=5, mode="conv_transpose"):
    keys = []
    bn = ["weight", "bias", "running_mean", "running_var", "num_batches_tracked"]

    def dc(prefix):
        out = []
        for i in (0, 3):
            out += [f"{prefix}.double_conv.{i}.weight", f"{prefix}.double_conv.{i}.bias"]
            out += [f"{prefix}.double_conv.{i + 1}.{b}" for b in bn]
        return out

    for k in range(1, depth + 1):
        keys += dc(f"down_conv{k}.double_conv")
    keys += dc("double_conv")
    for k in range(depth, 0, -1):
        if mode == "conv_transpose":
            keys += [f"up_conv{k}.up_sample.weight", f"up_conv{k}.up_sample.bias"]
        keys += dc(f"up_conv{k}.double_conv")
    keys += ["conv_last.weight", "conv_last.bias"]
    return keys


def test_reference_state_dict_keys_and_counts():
    m = UNet(out_classes=6)
    sd = m.state_dict()
    assert len(sd) == 166
    assert len(list(m.parameters())) == 100
    assert sum(p.numel() for p in m.parameters()) == 8_723_558
    assert sum(b.numel() for b in m.buffers()) == 6_934
    assert set(sd) == set(_expected_keys())


def test_width_divisor_and_bilinear_counts():
    assert sum(p.numel() for p in UNet(out_classes=6, width_divisor=1).parameters()) == 34_869_446
    mb = UNet(out_classes=6, up_sample_mode="bilinear")
    assert sum(p.numel() for p in mb.parameters()) == 7_854_246
    assert len(list(mb.parameters())) == 90
    assert len(mb.state_dict()) == 156
    assert set(mb.state_dict()) == set(_expected_keys(mode="bilinear"))


def test_layer_shapes_match_reference_widths():
    m = UNet(out_classes=6)
    # (ref.py:625-641) widths 64,128,256,512,512 // 2; decoder concat widths 512,512,384,192,96
    assert m.down_conv1.double_conv.double_conv[0].weight.shape == (32, 3, 3, 3)
    assert m.down_conv5.double_conv.double_conv[3].weight.shape == (256, 256, 3, 3)
    assert m.up_conv5.up_sample.weight.shape == (256, 256, 2, 2)
    assert m.up_conv3.double_conv.double_conv[0].weight.shape == (128, 384, 3, 3)
    assert m.up_conv1.double_conv.double_conv[0].weight.shape == (32, 96, 3, 3)
    assert m.conv_last.weight.shape == (6, 32, 1, 1)


@pytest.mark.parametrize("depth,dims,tile", [(5, 2, 64), (4, 2, 32), (3, 3, 16)])
def test_forward_shapes(depth, dims, tile):
    m = UNet(out_classes=4, depth=depth, dims=dims, width_divisor=8)
    x = torch.randn((2, 3) + (tile,) * dims)
    assert m(x).shape == (2, 4) + (tile,) * dims


def test_invalid_upsample_mode():
    with pytest.raises(ValueError):
        UNet(up_sample_mode="nearest")


def test_upsampled_tensor_first_in_concat():
    """cat([up, skip]): the first in-channels of up_conv1's conv come from the up-sample."""
    m = UNet(out_classes=2, width_divisor=8, depth=2)
    ub = m.up_conv1
    seen = {}
    def hook(mod, inp, out):
        seen["x"] = inp[0]

    h = ub.double_conv.double_conv[0].register_forward_hook(hook)
    m(torch.randn(1, 3, 16, 16))
    h.remove()
    up_ch = ub.up_sample.out_channels
    assert seen["x"].shape[1] == up_ch + m.enc_widths[0]


def test_loss_and_correct_torch_path():
    torch.manual_seed(0)
    m = UNet(out_classes=3, width_divisor=16, depth=2)
    x = torch.randn(2, 3, 16, 16)
    y = torch.randint(0, 3, (2, 16, 16))
    loss, correct = m.loss_and_correct(x, y)
    ref = torch.nn.functional.cross_entropy(m(x), y)
    assert torch.allclose(loss, ref)
    assert int(correct) == int((m(x).argmax(1) == y).sum())
