"""Flat fused Adam vs torch.optim.Adam, checkpoint format and resume — CPU."""
import copy

import torch

from ddlpc.models import UNet
from ddlpc.ops.adam import FlatAdam
from ddlpc.parallel import flatten_module
from ddlpc.train.checkpoint import load_checkpoint, save_checkpoint


def _grads(m, seed):
    g = torch.Generator().manual_seed(seed)
    for p in m.parameters():
        p.grad.copy_(torch.randn(p.shape, generator=g))


def test_flat_adam_matches_torch_adam():
    torch.manual_seed(0)
    a = UNet(out_classes=2, width_divisor=16, depth=2)
    b = copy.deepcopy(a)
    flat = flatten_module(a)
    opt_a = FlatAdam(flat, lr=1e-3)
    opt_b = torch.optim.Adam(b.parameters(), lr=1e-3)
    for step in range(3):
        _grads(a, step)
        for p in b.parameters():
            p.grad = torch.zeros_like(p)
        _grads(b, step)
        opt_a.step()
        opt_b.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.allclose(pa, pb, atol=1e-6, rtol=1e-5)
    # state_dict is torch.optim.Adam format: loads into stock Adam
    sd = opt_a.state_dict()
    opt_c = torch.optim.Adam(copy.deepcopy(b).parameters(), lr=1e-3)
    opt_c.load_state_dict(sd)
    assert float(sd["state"][0]["step"]) == 3
    assert torch.allclose(opt_c.state_dict()["state"][5]["exp_avg"], opt_b.state_dict()["state"][5]["exp_avg"], atol=1e-7)


def test_checkpoint_roundtrip_keeps_flat_views(tmp_path):
    torch.manual_seed(0)
    m = UNet(out_classes=2, width_divisor=16, depth=2)
    flat = flatten_module(m)
    opt = FlatAdam(flat)
    _grads(m, 0)
    opt.step()
    path = save_checkpoint(str(tmp_path / "c.pt"), m, opt, epoch=3, step=7)
    m2 = UNet(out_classes=2, width_divisor=16, depth=2)
    flat2 = flatten_module(m2)
    opt2 = FlatAdam(flat2)
    blob = load_checkpoint(path, m2, opt2)
    assert blob["epoch"] == 3 and blob["step"] == 7
    assert flat2.check_bound()
    for a, b in zip(m.state_dict().values(), m2.state_dict().values()):
        assert torch.equal(a, b)
    assert opt2.step_count == 1
    assert torch.equal(opt2.exp_avg, opt.exp_avg)
    # checkpoint has the reference-compatible key set and loads into a plain UNet
    plain = UNet(out_classes=2, width_divisor=16, depth=2)
    plain.load_state_dict(torch.load(path, weights_only=True)["model"])
