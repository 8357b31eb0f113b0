"""Data-parallel correctness on a gloo world of 2 CPU processes (no cluster needed)."""
import copy

import pytest
import torch

from dist_utils import run


def _small_model():
    from ddlpc.models import UNet
    torch.manual_seed(0)
    return UNet(out_classes=3, width_divisor=16, depth=2)


def _batch(seed, n=2, tile=16):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(n, 3, tile, tile, generator=g), torch.randint(0, 3, (n, tile, tile), generator=g)


def _reducer_vs_big_batch(rank, world, codec, reduce, double_report=False):
    import torch.distributed as dist
    import torch.nn.functional as F
    from ddlpc.parallel import GradBucketReducer, broadcast_module, flatten_module, init_distributed
    init_distributed(device="cpu")
    m = _small_model().eval()          # eval: BN uses running stats -> per-sample independence
    flat = flatten_module(m)
    broadcast_module(m)
    red = GradBucketReducer(flat, bucket_mb=0.01, reduce=reduce, grad_codec=codec)
    if double_report:           # a second readiness source (as kernels writing .grad directly)
        for q in flat.order:
            q.register_post_accumulate_grad_hook(red.mark_ready)
    x, y = _batch(100 + rank)
    red.prepare(sync=True)
    F.cross_entropy(m(x), y).backward()
    red.finish()
    g = flat.grad_buf.clone()
    gs = [torch.empty_like(g) for _ in range(world)]
    dist.all_gather(gs, g)
    return {"grad": g, "all_same": all(torch.equal(gs[0], t) for t in gs),
            "buckets": len(red.buckets), "in_backward": red.stats["launched_in_backward"]}


def _single_process_grads(world, reduce):
    import torch.nn.functional as F
    from ddlpc.parallel import flatten_module
    m = _small_model().eval()
    flat = flatten_module(m)
    for r in range(world):
        x, y = _batch(100 + r)
        loss = F.cross_entropy(m(x), y)
        (loss / world if reduce == "mean" else loss).backward()
    return flat.grad_buf.clone()


@pytest.mark.parametrize("reduce,double", [("mean", False), ("sum", False), ("reference", False),
                                           ("mean", True)])
def test_bucketed_allreduce_equals_big_batch(reduce, double):
    res = run(_reducer_vs_big_batch, 2, ("none", reduce, double))
    ref = _single_process_grads(2, "mean" if reduce == "mean" else "sum")
    for r in (0, 1):
        assert res[r]["all_same"]
        assert res[r]["buckets"] > 1 and res[r]["in_backward"] == res[r]["buckets"]
        assert torch.allclose(res[r]["grad"], ref, atol=1e-6, rtol=1e-4)


@pytest.mark.parametrize("codec", ["fp16_absmax", "int8_absmax"])
def test_codec_allgather_identical_and_close(codec):
    res = run(_reducer_vs_big_batch, 2, (codec, "mean"))
    ref = _single_process_grads(2, "mean")
    assert torch.equal(res[0]["grad"], res[1]["grad"])
    err = float((res[0]["grad"] - ref).norm() / ref.norm())
    assert err < (0.05 if codec == "fp16_absmax" else 0.5)


def _train_ranks(rank, world, accum, codec):
    from ddlpc.config import ModelConfig, TrainConfig
    from ddlpc.parallel import params_checksum
    from ddlpc.train.trainer import Trainer
    cfg = TrainConfig(model=ModelConfig(out_classes=2, depth=3, width_divisor=16), tile=32, dtype="fp32",
                      num_samples=12, test_holdout=4, batch_per_gpu=2, accum_steps=accum,
                      epochs=2, check_consistency_every=1, bucket_mb=0.05, grad_codec=codec,
                      log_every=0, timeout_s=60)
    tr = Trainer(cfg, device="cpu")
    m = tr.fit()
    v = tr.validate()
    cs = float(params_checksum(tr.model))
    tr.close()
    return {"checksum": cs, "steps": tr.step_count, "loss": m["loss"], "val": v}


@pytest.mark.parametrize("accum,codec", [(1, "none"), (2, "none"), (1, "int8_absmax")])
def test_replicas_stay_bit_identical(accum, codec):
    res = run(_train_ranks, 2, (accum, codec))
    assert res[0]["checksum"] == res[1]["checksum"]
    assert res[0]["steps"] == res[1]["steps"] > 0
    assert res[0]["val"]["val_pixel_acc"] == res[1]["val"]["val_pixel_acc"]


def _init_broadcast(rank, world):
    from ddlpc.models import UNet
    from ddlpc.parallel import broadcast_module, init_distributed, params_checksum
    init_distributed(device="cpu")
    torch.manual_seed(rank)                 # deliberately different init per rank
    m = UNet(out_classes=2, width_divisor=16, depth=2)
    broadcast_module(m)
    return float(params_checksum(m))


def test_rank0_broadcast_replaces_pickled_model():
    res = run(_init_broadcast, 3)
    assert res[0] == res[1] == res[2]


def _fault(rank, world):
    import os
    import time
    from ddlpc.config import ModelConfig, TrainConfig
    from ddlpc.data import SyntheticTiles
    from ddlpc.train.trainer import Trainer
    cfg = TrainConfig(model=ModelConfig(out_classes=2, depth=2, width_divisor=16), tile=16, dtype="fp32",
                      num_samples=8, test_holdout=0, batch_per_gpu=1, timeout_s=20)
    tr = Trainer(cfg, device="cpu")
    x, y = SyntheticTiles(4, 16, classes=2).get([0])
    for step in range(4):
        if rank == 1 and step == 2:
            os._exit(3)                      # fault injection: a worker PC dies mid-run
        tr.train_step([(x, y)])
    return "finished"


def test_fault_injection_dead_peer_raises_not_hangs():
    out = run(_fault, 2, timeout=120, allow_fail=True)
    assert 0 in out and out[0][0] == "err", out      # rank 0 errors out instead of hanging


def _fresh_reducer_arming(rank, world):
    """A fresh reducer (and one after ``finish()``) is disarmed: readiness reports from an
    accumulation micro-batch's backward launch nothing; only ``prepare(sync=True)`` arms."""
    import torch.nn.functional as F
    from ddlpc.parallel import GradBucketReducer, broadcast_module, flatten_module, init_distributed
    init_distributed(device="cpu")
    m = _small_model().eval()
    flat = flatten_module(m)
    broadcast_module(m)
    red = GradBucketReducer(flat, bucket_mb=0.01)
    x, y = _batch(100 + rank)
    F.cross_entropy(m(x), y).backward()              # no prepare(): accumulation
    n_fresh = red.stats["launched_in_backward"]
    red.prepare(sync=True)
    F.cross_entropy(m(x), y).backward()
    n_armed = red.stats["launched_in_backward"]
    red.finish()
    F.cross_entropy(m(x), y).backward()              # after the exchange: disarmed again
    return {"fresh": n_fresh, "armed": n_armed, "after": red.stats["launched_in_backward"],
            "buckets": len(red.buckets)}


def test_fresh_reducer_is_disarmed():
    res = run(_fresh_reducer_arming, 2)
    for r in (0, 1):
        o = res[r]
        assert o["fresh"] == 0 and o["armed"] == o["buckets"] > 1 and o["after"] == o["armed"], o


def _resume_missing(rank, world, tmp):
    from ddlpc.config import ModelConfig, TrainConfig
    from ddlpc.train.trainer import Trainer
    cfg = TrainConfig(model=ModelConfig(out_classes=2, depth=2, width_divisor=16), tile=16, dtype="fp32",
                      num_samples=4, test_holdout=0, timeout_s=600,
                      resume=tmp + "/no_such_ckpt.pt")
    try:
        Trainer(cfg, device="cpu")
    except FileNotFoundError as e:
        return f"raised: {e}"
    return "no error"


def test_missing_resume_path_fails_every_rank_fast(tmp_path):
    """An explicit resume path missing on rank 0 raises on EVERY rank at once (ranks > 0
    must not block in the state broadcast until the 30-minute collective timeout)."""
    import time
    t0 = time.time()
    res = run(_resume_missing, 2, (str(tmp_path),), timeout=120)
    assert all(str(v).startswith("raised") for v in res.values()), res
    assert time.time() - t0 < 100
