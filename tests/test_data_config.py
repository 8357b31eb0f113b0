"""Data loaders, sampler and config — CPU."""
import json
import os

import numpy as np
import pytest
import torch

from ddlpc.config import ModelConfig, TrainConfig, add_config_args, config_from_args
from ddlpc.data import ShardedSampler, SyntheticTiles, TileDataset, load_files, to_tensors


def _write_dir(tmp_path, n=35, size=16):
    from PIL import Image
    rng = np.random.default_rng(0)
    for i in range(n):
        Image.fromarray(rng.integers(0, 255, (size, size, 3), dtype=np.uint8)).save(
            tmp_path / f"tile_{i:03d}.png")
        np.save(tmp_path / f"tile_{i:03d}_label.npy", rng.integers(0, 6, (size, size)))
    return tmp_path


def test_load_files_reference_convention(tmp_path):
    d = _write_dir(tmp_path)
    xtr, ytr, xte, yte = load_files(str(d))
    assert xtr.shape == (5, 16, 16, 3) and xte.shape == (30, 16, 16, 3)   # last 30 held out
    assert ytr.dtype == np.uint8 and yte.shape == (30, 16, 16)
    x, y = to_tensors(xtr, ytr)
    assert x.shape == (5, 3, 16, 16) and x.dtype == torch.float32 and float(x.max()) <= 1.0
    assert y.dtype == torch.int64
    # NCHW transpose is the reference's swapaxes(1,3).swapaxes(2,3) (ref.py:737)
    ref = torch.from_numpy(xtr.astype("float32") / 255).swapaxes(1, 3).swapaxes(2, 3)
    assert torch.allclose(x, ref)
    tr, te = TileDataset.from_dir(str(d))
    assert len(tr) == 5 and len(te) == 30
    xg, yg = tr.get([1, 4])                     # host get(): the reference's tensors
    assert torch.equal(xg, x[[1, 4]]) and torch.equal(yg, y[[1, 4]])


def test_synthetic_deterministic_and_learnable_shape():
    ds = SyntheticTiles(10, 32, classes=6, seed=3)
    x1, y1 = ds.get([2, 5])
    x2, y2 = ds.get([2, 5])
    assert torch.equal(x1, x2) and torch.equal(y1, y2)
    assert x1.shape == (2, 3, 32, 32) and y1.shape == (2, 32, 32)
    assert int(y1.max()) < 6
    x3, y3 = SyntheticTiles(4, 8, classes=2, dims=3).get([0])
    assert x3.shape == (1, 3, 8, 8, 8) and y3.shape == (1, 8, 8, 8)


def test_sharded_sampler_disjoint_and_replicated():
    parts = [ShardedSampler(20, r, 4, shard=True, seed=1).indices() for r in range(4)]
    flat = sorted(i for p in parts for i in p)
    assert flat == list(range(20))
    rep = [ShardedSampler(20, r, 4, shard=False, shuffle=False).indices() for r in range(4)]
    assert all(r == list(range(20)) for r in rep)      # reference replicated mode
    s = ShardedSampler(20, 0, 2, seed=1)
    e0 = s.indices()
    s.set_epoch(1)
    assert s.indices() != e0


def test_config_roundtrip_and_cli(tmp_path):
    cfg = TrainConfig(model=ModelConfig(depth=4, width_divisor=4), tile=128, accum_steps=50)
    d = cfg.to_dict()
    cfg2 = TrainConfig.from_dict(json.loads(json.dumps(d)))
    assert cfg2.to_dict() == d
    p = tmp_path / "c.json"
    cfg.save(str(p))
    import argparse
    ap = add_config_args(argparse.ArgumentParser())
    args = ap.parse_args(["--config", str(p), "--lr", "0.01", "--depth", "5",
                          "--grad-codec", "int8_absmax", "--shard-data", "false"])
    c3 = config_from_args(args)
    assert c3.lr == 0.01 and c3.model.depth == 5 and c3.accum_steps == 50
    assert c3.grad_codec == "int8_absmax" and c3.shard_data is False
    with pytest.raises(ValueError):
        TrainConfig(grad_codec="zip").validate()
    with pytest.raises(ValueError):
        TrainConfig.from_dict({"bogus": 1})


def test_yaml_config(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text("model:\n  depth: 4\n  out_classes: 2\ntile: 128\nbatch_per_gpu: 2\n")
    c = TrainConfig.load(str(p))
    assert c.model.depth == 4 and c.tile == 128 and c.batch_per_gpu == 2


def test_config_precision_is_honest():
    """The HIP kernels compute in bf16: asking them for fp32 (the reference's precision,
    ref.py:702-704) is an error, not a silent bf16 run; fp32 runs on stock ops."""
    import pytest
    import torch
    from ddlpc.config import TrainConfig
    from ddlpc.train.trainer import resolve_impl
    with pytest.raises(ValueError):
        TrainConfig(impl="hip", dtype="fp32").validate()
    TrainConfig(impl="torch", dtype="fp32").validate()
    gpu = torch.device("cuda", 0)
    assert resolve_impl("auto", gpu, "fp32") == "torch"
    assert resolve_impl("auto", gpu, "bf16") == "hip"
    # the precision picks the path, not the device: the engine's operators dispatch by
    # tensor device (CPU kernels: csrc/cpu_ref.cpp)
    assert resolve_impl("auto", torch.device("cpu"), "bf16") == "hip"
    assert resolve_impl("auto", torch.device("cpu"), "fp32") == "torch"


def test_resume_missing_explicit_checkpoint_raises(tmp_path):
    """An explicit resume path that does not exist fails loudly on rank 0 (it would otherwise
    start from scratch and broadcast that state); resume='auto' tolerates an empty dir."""
    import pytest
    from ddlpc.config import ModelConfig, TrainConfig
    from ddlpc.train.trainer import Trainer
    kw = dict(model=ModelConfig(out_classes=3, depth=3, width_divisor=8), tile=32,
              batch_per_gpu=1, num_samples=2, test_holdout=0, impl="torch")
    with pytest.raises(FileNotFoundError):
        Trainer(TrainConfig(resume=str(tmp_path / "nope.pt"), **kw), device="cpu")
    Trainer(TrainConfig(resume="auto", ckpt_dir=str(tmp_path), **kw), device="cpu").close()


def test_device_dataset_rejects_out_of_range_host_indices():
    import pytest
    import torch
    from ddlpc.data.datasets import DeviceTileDataset, TileDataset
    base = TileDataset(torch.zeros(3, 8, 8, 3, dtype=torch.uint8), torch.zeros(3, 8, 8, dtype=torch.uint8))
    ds = DeviceTileDataset.__new__(DeviceTileDataset)
    ds.base = base
    with pytest.raises(IndexError):
        DeviceTileDataset.get(ds, [0, 3])


def test_split_batch_views_rejoin_without_copy():
    """A whole accumulation window rendered at once (bench.py) is handed to the trainer as
    zero-copy micro-batch views; ``Trainer._cat_window`` joins them back without a copy, and
    anything else (separately allocated micro-batches) still concatenates by copy."""
    import torch
    from ddlpc.data import cat_adjacent, split_batch
    from ddlpc.data.datasets import engine_input
    from ddlpc.train.trainer import Trainer
    xp = torch.randn(6, 4, 4, 8)
    x, y = engine_input(xp, 3), torch.randint(0, 5, (6, 4, 4))
    mbs = split_batch(x, y, 3)
    assert [tuple(m[0].shape) for m in mbs] == [(2, 3, 4, 4)] * 3
    assert all(m[0]._ddlpc_nhwc.shape == (2, 4, 4, 8) for m in mbs)
    xw, yw = Trainer._cat_window(mbs)
    assert xw._ddlpc_nhwc.data_ptr() == xp.data_ptr() and torch.equal(xw._ddlpc_nhwc, xp)
    assert yw.data_ptr() == y.data_ptr() and torch.equal(yw, y)
    parts = [y[:2].clone(), y[2:4].clone()]
    joined = cat_adjacent(parts)
    assert joined.data_ptr() != parts[0].data_ptr() and torch.equal(joined, y[:4])
    # out of order views are copied in the given order
    assert torch.equal(cat_adjacent([y[2:4], y[:2]]), torch.cat([y[2:4], y[:2]]))
    try:
        split_batch(x, y, 4)
        raise AssertionError("uneven split accepted")
    except ValueError:
        pass
