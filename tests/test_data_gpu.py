"""Device input pipeline and the device-fed ``train()`` / ``validate()`` path.

* ``synth_tiles`` (csrc/data.hip) renders exactly the bits of the PyTorch twin
  ``render_synthetic`` (labels equal, images equal after bf16 rounding);
* ``tile_gather`` (HBM-resident uint8 dataset) equals ``TileDataset.get`` (/255, NCHW);
* ``Trainer.fit()`` + ``validate()`` run on the HIP engine fed by those kernels, for the
  synthetic source and a Vaihingen-convention directory, resident and host-streamed.
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("classes,tile,dims,grid", [(6, 64, 2, 8), (3, 50, 2, 8), (10, 32, 2, 8),
                                                    (6, 16, 3, 4), (10, 16, 3, 4), (2, 33, 2, 5)])
def test_synth_tiles_kernel_matches_torch_twin(classes, tile, dims, grid):
    from ddlpc.data import SyntheticTiles
    from ddlpc.data.datasets import render_synthetic
    idx = [0, 7, 123456, 2**31 + 5]
    dev = SyntheticTiles(10, tile, classes=classes, seed=11, dims=dims, grid=grid,
                         device="cuda", layout="engine")
    x, y = dev.get(idx)
    xp = x._ddlpc_nhwc
    assert xp.shape == (len(idx),) + (tile,) * dims + (8,) and xp.dtype == torch.bfloat16
    assert not xp[..., 3:].any()                                 # zero channel padding
    xr, yr = render_synthetic(idx, 11, classes, 3, tile, dims, grid=grid)
    assert torch.equal(y.cpu(), yr)
    want = xr.permute(0, *range(2, xr.dim()), 1).to(torch.bfloat16)
    got = xp[..., :3].cpu()
    bad = (got != want).nonzero()
    assert bad.numel() == 0, (bad.shape[0], bad[:6].tolist(),
                              [(float(got[tuple(i)]), float(want[tuple(i)]),
                                float(xr.permute(0, *range(2, xr.dim()), 1)[tuple(i)]))
                               for i in bad[:6].tolist()])
    # the NCHW view the model API sees
    assert x.shape == (len(idx), 3) + (tile,) * dims


def test_device_prefetcher_hands_out_each_batch_intact():
    """``DevicePrefetcher`` (bench.py's input pipeline): batch k renders on a side stream
    under step k - 1; every batch handed out equals a direct render of the same indices,
    with the consumer allocating / freeing memory and running kernels in between (the
    allocator must not recycle a batch the current stream still reads)."""
    from ddlpc.data import DevicePrefetcher, SyntheticTiles
    ds = SyntheticTiles(1 << 20, 64, classes=6, seed=5, device="cuda", layout="engine")

    def make(k):
        return ds.get(torch.arange(8 * k, 8 * k + 8, device="cuda"))

    pf = DevicePrefetcher(make, "cuda")
    for k in range(6):
        x, y = pf.get(k)
        junk = torch.randn(4 << 20, device="cuda")          # allocator churn + device work
        s = float((x._ddlpc_nhwc.float().sum() + y.sum()).item()) + float(junk.sum().item())
        xr, yr = make(k)
        assert torch.equal(x._ddlpc_nhwc, xr._ddlpc_nhwc) and torch.equal(y, yr), k
        del x, y, junk, s
    assert 6 in pf.pending                                   # the next batch is in flight


def test_tile_gather_matches_host_dataset():
    from ddlpc.data import TileDataset
    rng = np.random.default_rng(0)
    xs = rng.integers(0, 256, (9, 24, 40, 3), dtype=np.uint8)
    ys = rng.integers(0, 6, (9, 24, 40), dtype=np.uint8)
    ds = TileDataset(xs, ys)
    idx = [8, 0, 3, 3]
    xh, yh = ds.get(idx)
    for budget in (None, 0):                      # resident in HBM / pinned host + copy stream
        dd = ds.to_device("cuda", "engine", budget)
        assert dd.resident == (budget is None)
        x, y = dd.get(idx)
        assert torch.equal(y.cpu(), yh)
        assert torch.equal(x._ddlpc_nhwc[..., :3].cpu(), xh.permute(0, 2, 3, 1).bfloat16())
        dn = ds.to_device("cuda", "nchw", budget)
        x2, y2 = dn.get(idx)                      # (torch's GPU /255 is a reciprocal multiply)
        assert torch.allclose(x2.cpu(), xh, rtol=1e-6, atol=0) and torch.equal(y2.cpu(), yh)


def _cfg(tmp_path, **kw):
    from ddlpc.config import ModelConfig, TrainConfig
    base = dict(model=ModelConfig(out_classes=6), tile=64, batch_per_gpu=4, num_samples=48,
                test_holdout=8, impl="hip", epochs=2, log_every=2,
                log_dir=str(tmp_path / "log"), ckpt_dir=str(tmp_path / "ck"))
    base.update(kw)
    return TrainConfig(**base)


def test_fit_and_validate_on_hip_engine(tmp_path):
    """fit() on device-rendered synthetic tiles: the engine input is the generator's buffer
    (no conversion pass), the loss falls, metrics/checkpoints are written, validate() runs."""
    from ddlpc.train.trainer import Trainer
    tr = Trainer(_cfg(tmp_path, epochs=3), device="cuda")
    x, _ = tr.train_set.get([0, 1, 2, 3])
    assert getattr(x, "_ddlpc_nhwc", None) is not None
    assert tr.model._engine.to_nhwc(x) is x._ddlpc_nhwc            # zero-copy engine input
    m = tr.fit()
    v = tr.validate()
    tr.close()
    assert np.isfinite(m["loss"]) and m["steps"] == 3 * (48 // 4)
    assert set(v) >= {"val_loss", "val_pixel_acc", "val_iou", "val_miou"}
    assert 0.0 <= v["val_pixel_acc"] <= 1.0 and len(v["val_iou"]) == 6
    lines = (tmp_path / "log" / "metrics.jsonl").read_text().splitlines()
    steps = [json.loads(line) for line in lines]
    losses = [r["loss"] for r in steps if "images_per_s" in r]
    assert losses[-1] < losses[0], losses
    assert os.path.exists(tmp_path / "ck" / "ckpt_36.pt")


def test_fit_vaihingen_dir_hbm_and_streamed(tmp_path):
    from PIL import Image
    from ddlpc.train.trainer import Trainer
    d = tmp_path / "data"
    d.mkdir()
    rng = np.random.default_rng(1)
    for i in range(12):
        Image.fromarray(rng.integers(0, 255, (64, 64, 3), dtype=np.uint8)).save(d / f"t{i:02d}.png")
        np.save(d / f"t{i:02d}_label.npy", rng.integers(0, 6, (64, 64)))
    out = []
    for gb in (None, 0.0):
        tr = Trainer(_cfg(tmp_path / str(gb), data="vaihingen_dir", data_dir=str(d),
                          test_holdout=4, epochs=2, data_hbm_gb=gb, shuffle=False,
                          log_dir=None, ckpt_dir=None), device="cuda")
        assert tr.train_set.resident == (gb is None)
        m = tr.fit()
        v = tr.validate()
        out.append((tr.flat.param_buf.clone(), m["loss"], v["val_loss"]))
        tr.close()
    # the two data paths feed bit-identical batches -> bit-identical training (the held-out
    # loss goes through torch's GPU cross_entropy sum, whose reduction order may vary)
    assert torch.equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]
    assert abs(out[0][2] - out[1][2]) <= 1e-6 * abs(out[0][2])
