"""train()/validate() integration, resume, logs and PNG dumps on CPU (BASELINE config #1 shape)."""
import json
import os
import subprocess
import sys

import pytest
import torch

from ddlpc.config import ModelConfig, TrainConfig
from ddlpc.train import Trainer, train, validate


def _cfg(tmp_path, **kw):
    # fp32 = the reference's precision on the stock-op path (the narrow test widths are below
    # the engine's geometry floor)
    base = dict(model=ModelConfig(out_classes=2, depth=4, width_divisor=8), tile=64, dtype="fp32",
                num_samples=16, test_holdout=4, batch_per_gpu=2, accum_steps=2, epochs=3,
                log_every=1, log_dir=str(tmp_path / "logs"), ckpt_dir=str(tmp_path / "ck"))
    base.update(kw)
    return TrainConfig(**base)


def test_train_loss_decreases_and_logs(tmp_path):
    cfg = _cfg(tmp_path, png_dir=str(tmp_path / "png"), png_count=2)
    m, tr = train(cfg, device="cpu", return_trainer=True)
    lines = [json.loads(l) for l in open(tmp_path / "logs" / "metrics.jsonl")]
    losses = [l["loss"] for l in lines if "step" in l and "epoch_end" not in l]
    assert losses[-1] < losses[0]
    otus = (tmp_path / "logs" / "otus_float32.txt").read_text()
    assert "batch_size" in otus and otus.count("ep:") == 3
    assert sorted(os.listdir(tmp_path / "png")) == [
        "Image 0.png", "Image 1.png", "Label 0.png", "Label 1.png", "Model 0.png", "Model 1.png"]
    v = tr.validate()
    assert 0.0 <= v["val_pixel_acc"] <= 1.0 and len(v["val_iou"]) == 2
    assert os.path.exists(tmp_path / "ck" / f"ckpt_{tr.step_count}.pt")


def test_resume_gives_identical_next_step(tmp_path):
    cfg = _cfg(tmp_path, epochs=1, max_steps=2, shuffle=False)
    _, tr = train(cfg, device="cpu", return_trainer=True)
    ck = tr.save(str(tmp_path / "mid.pt"))
    batch = [tr._to_device(*tr.train_set.get([0, 1])), tr._to_device(*tr.train_set.get([2, 3]))]
    tr.train_step(batch)
    after = {k: v.clone() for k, v in tr.model.state_dict().items()}
    cfg2 = _cfg(tmp_path, epochs=1, max_steps=2, shuffle=False, resume=ck)
    tr2 = Trainer(cfg2, device="cpu")
    assert tr2.step_count == tr.step_count - 1
    tr2.train_step(batch)
    for k, v in tr2.model.state_dict().items():
        assert torch.allclose(v.float(), after[k].float(), atol=1e-6), k


def test_validate_from_checkpoint(tmp_path):
    cfg = _cfg(tmp_path, epochs=1)
    _, tr = train(cfg, device="cpu", return_trainer=True)
    path = tr.save(str(tmp_path / "v.pt"))
    v = validate(_cfg(tmp_path, epochs=1), checkpoint=path, device="cpu")
    assert abs(v["val_pixel_acc"] - tr.validate()["val_pixel_acc"]) < 1e-9


def test_profiler_trace_and_throughput_metrics(tmp_path):
    cfg = _cfg(tmp_path, epochs=2, max_steps=6, profile_dir=str(tmp_path / "prof"),
               profile_steps=1, trace_ranges=True)
    train(cfg, device="cpu")
    assert os.path.exists(tmp_path / "prof" / "trace_rank0.json")
    trace = json.load(open(tmp_path / "prof" / "trace_rank0.json"))
    names = {e.get("name") for e in trace.get("traceEvents", [])}
    assert any(n and "conv" in n for n in names)
    lines = [json.loads(l) for l in open(tmp_path / "logs" / "metrics.jsonl")]
    steps = [l for l in lines if "step" in l and "epoch_end" not in l]
    assert steps and all(l["images_per_s"] > 0 for l in steps)


def test_phase_timer_on_cpu_uses_the_host_clock():
    """On a CPU device (gloo rehearsal) the phase marks are host clock readings: every op is
    synchronous there, so the per-phase means are real (bench.py's comm_wait_ms on CPU)."""
    import time
    from ddlpc.utils.tracing import PhaseTimer, trace_range
    pt = PhaseTimer(torch.device("cpu"))
    for _ in range(2):
        pt.mark("start")
        with trace_range("x"):
            time.sleep(0.01)
            pt.mark("a")
        pt.mark("b")
        pt.end_step()
    r = pt.read()
    assert set(r) == {"a_ms", "b_ms", "step_ms"}
    assert 9.0 <= r["a_ms"] < 500 and 0 <= r["b_ms"] < r["a_ms"]
    assert abs(r["step_ms"] - r["a_ms"] - r["b_ms"]) < 1e-6
    assert pt.read() == {}                     # reset after a read


def test_bench_cpu_json_contract():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--impl", "torch",
                          "--steps", "1", "--warmup", "1", "--batch", "2", "--tile", "64",
                          "--width-divisor", "16"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in rec
    assert rec["n_gpus"] == 1 and rec["steps"] == 1 and rec["value"] > 0


def test_bench_torchrun_two_ranks_gloo():
    """The driver's N>1 launch line (torch.distributed.run, 127.0.0.1) on CPU/gloo: one JSON
    line from rank 0 with the whole-job aggregate, and the run's self-validation: the
    backend and world size the collectives really used, bit-identical replicas after the
    timed steps, the exposed communication wait per step."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="2")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "2", "--rdzv-backend", "c10d",
                          "--rdzv-endpoint", "127.0.0.1:0", os.path.join(root, "bench.py"),
                          "--gpus", "2", "--impl", "torch", "--steps", "2", "--warmup", "1",
                          "--batch", "2", "--tile", "64", "--width-divisor", "16",
                          "--wire-dtype", "bf16", "--bucket-mb", "0.5", "--bucket-sweep", "0.25,1"],
                         capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["global_batch"] == 4 and rec["value"] > 0
    # multi-GPU reporting fields: bucket count, wire dtype, the bucket sweep
    c = rec["config"]
    assert c["wire_dtype"] == "bf16" and c["buckets"] >= 2 and "comm_wait_ms" in c
    assert set(c["bucket_sweep"]) == {"0.25", "1.0"}
    assert c["bucket_sweep"]["0.25"]["buckets"] > c["bucket_sweep"]["1.0"]["buckets"]
    assert rec["dist_backend"] == "gloo" and rec["world_size"] == 2
    assert rec["replicas_identical"] is True and rec["rccl_version"] is None
    assert rec["comm_wait_ms"] is not None and rec["comm_wait_ms"] >= 0
    # the readiness plan re-cut from one measured step (same cuts on both ranks, or the
    # bucket all-reduces of the timed steps would not have matched up)
    cal = c["bucket_plan_calibration"]
    assert cal is not None and cal["backward_ms"] > 0 and cal["buckets"] >= 1
    assert len(cal["predicted_end_ms"]) == cal["buckets"] == len(cal["bucket_mb"])


def test_bench_self_spawns_torchrun_for_gpus_n():
    """``bench.py --gpus 2`` outside torchrun launches torchrun itself (a child process) and
    the ranks report the world they really formed."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "2"
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                          "--impl", "torch", "--steps", "1", "--warmup", "1", "--batch", "2",
                          "--tile", "64", "--width-divisor", "16"],
                         capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2 and rec["replicas_identical"] is True


def test_bench_refuses_world_size_mismatch():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                          "--impl", "torch", "--steps", "1", "--warmup", "0"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 2 and "refusing" in out.stderr


def test_resume_with_max_steps_inside_an_epoch(tmp_path):
    """max_steps stopping mid-epoch must not advance the epoch: a resume with a larger
    max_steps continues inside the same epoch and reaches the same weights as one run."""
    full = _cfg(tmp_path / "a", epochs=2, max_steps=None, shuffle=True, ckpt_dir=None,
                log_dir=None)
    _, t_full = train(full, device="cpu", return_trainer=True)
    # 16 samples / (2 x 2) = 4 steps per epoch; stop after 3 (inside epoch 0), then resume
    part = _cfg(tmp_path / "b", epochs=2, max_steps=3, shuffle=True, log_dir=None)
    _, t1 = train(part, device="cpu", return_trainer=True)
    assert (t1.epoch, t1.epoch_step, t1.step_count) == (0, 3, 3)
    res = _cfg(tmp_path / "b", epochs=2, max_steps=None, shuffle=True, resume="auto",
               log_dir=None)
    _, t2 = train(res, device="cpu", return_trainer=True)
    assert t2.step_count == t_full.step_count == 8
    assert torch.allclose(t2.flat.param_buf, t_full.flat.param_buf, atol=1e-6)


def test_latest_checkpoint_ignores_non_step_names(tmp_path):
    from ddlpc.train.checkpoint import latest_checkpoint
    for n in ("ckpt_3.pt", "ckpt_12.pt", "ckpt_final.pt", "ckpt_7.pt.tmp", "other.pt"):
        (tmp_path / n).write_bytes(b"x")
    assert latest_checkpoint(str(tmp_path)).endswith("ckpt_12.pt")


def test_synthetic_sample_independent_of_batch_and_rank():
    """Sample i renders identically whatever batch / rank / order asks for it (counter-based
    hash), and the generator is learnable-shaped: piecewise-constant labels, bounded pixels."""
    from ddlpc.data import SyntheticTiles
    from ddlpc.data.datasets import render_synthetic, synthetic_palette
    ds = SyntheticTiles(100, 32, classes=6, seed=5)
    xa, ya = ds.get([3, 17, 42])
    xb, yb = ds.get([42, 3])
    assert torch.equal(xa[2], xb[0]) and torch.equal(ya[0], yb[1])
    assert float(xa.min()) >= 0.0 and float(xa.max()) <= 1.0
    assert ya[0, :4, :4].unique().numel() == 1          # one lattice cell (32/8 = 4 px)
    x3, y3 = render_synthetic([1], 0, 10, 4, 8, 3, grid=2)
    assert x3.shape == (1, 4, 8, 8, 8) and int(y3.max()) < 10
    assert synthetic_palette(10, 4).shape == (10, 4)


def _resume_rank(rank, world, ckdir):
    import os as _os
    from ddlpc.config import ModelConfig, TrainConfig
    from ddlpc.train.trainer import Trainer
    cfg = TrainConfig(model=ModelConfig(out_classes=2, depth=4, width_divisor=8), tile=32, dtype="fp32",
                      num_samples=8, test_holdout=0, batch_per_gpu=2, epochs=1,
                      ckpt_dir=_os.path.join(ckdir, f"rank{rank}"), resume="auto")
    tr = Trainer(cfg, device="cpu")
    out = {"step": tr.step_count, "epoch_step": tr.epoch_step,
           "opt_step": tr.optimizer.step_count,
           "p": float(tr.flat.param_buf.double().sum()),
           "m": float(tr.optimizer.exp_avg.double().abs().sum())}
    tr.close()
    return out


def test_resume_rank0_state_broadcast_without_shared_fs(tmp_path):
    """Only rank 0 has the checkpoint file (no shared filesystem): every rank must adopt
    rank 0's restored weights, Adam moments and counters."""
    from dist_utils import run
    cfg = _cfg(tmp_path, epochs=1, max_steps=3, ckpt_dir=str(tmp_path / "rank0"),
               model=ModelConfig(out_classes=2, depth=4, width_divisor=8), tile=32,
               num_samples=8, test_holdout=0, batch_per_gpu=2, accum_steps=1, log_dir=None)
    _, tr = train(cfg, device="cpu", return_trainer=True)
    want_p = float(tr.flat.param_buf.double().sum())
    res = run(_resume_rank, 2, (str(tmp_path),), timeout=200)
    for r in (0, 1):
        o = res[r]
        assert (o["step"], o["epoch_step"], o["opt_step"]) == (3, 3, 3), o
        assert abs(o["p"] - want_p) < 1e-9 and o["m"] > 0, o


def test_window_size_policy_and_concat():
    """bn_window policy (the batched accumulation window with per-micro-batch BatchNorm
    groups runs on the HIP engine only) and the window batch assembly: engine-layout inputs
    stay in that layout, labels concatenate in micro-batch order."""
    from ddlpc.config import ModelConfig, TrainConfig
    from ddlpc.data.datasets import engine_input
    from ddlpc.train.trainer import Trainer
    from ddlpc.utils.flops import unet_activation_elems_per_sample
    cfg = TrainConfig(model=ModelConfig(out_classes=2, depth=2, width_divisor=8), tile=16,
                      num_samples=4, test_holdout=0, accum_steps=4, log_every=0, dtype="fp32")
    tr = Trainer(cfg, device="cpu")
    assert tr._window_size(4) == 0                      # stock-op (CPU) path: no window
    tr.impl, tr.device = "hip", torch.device("cuda")    # policy only (nothing runs)
    cfg.bn_window = -1
    cfg.batch_per_gpu, cfg.tile = 1, 512
    assert tr._window_size(50) == 50                    # the reference regime: one pass
    assert tr._window_size(100) == 64                   # WINDOW_PIXELS caps a pass
    assert tr._window_size(1) == 0
    cfg.tile = 1024
    assert tr._window_size(50) == 0                     # large micro-batches: one by one
    cfg.bn_window = 8
    assert tr._window_size(50) == 8
    cfg.bn_window = 0
    assert tr._window_size(50) == 0
    # activation memory bounds the auto window (half of what the allocator can hand out)
    cfg.bn_window, cfg.tile = -1, 512
    per = tr.WINDOW_BYTES_PER_ELEM * unet_activation_elems_per_sample(cfg.model, 512)
    tr._allocator_bytes_available = lambda: 2 * 10.5 * per
    tr._window_cache = {}
    assert tr._window_size(50) == 10
    tr._allocator_bytes_available = lambda: 2 * 1.5 * per
    tr._window_cache = {}
    assert tr._window_size(50) == 0                     # not even two fit: one by one
    del tr._allocator_bytes_available
    tr._window_cache = {}
    cfg.recompute = 1
    assert tr._window_size(50) == 0                     # the grouped pass ignores recompute
    cfg.recompute = 0
    cfg.tile = 24                                       # 24 >> 1 = 12 >> 1 = 6: ok (depth 2)
    assert tr._window_size(50) == 50
    tr.impl, tr.device = "torch", torch.device("cpu")
    mbs = []
    for j in range(3):
        xp = torch.full((1, 8, 8, 8), float(j))
        mbs.append((engine_input(xp, 3), torch.full((1, 8, 8), j, dtype=torch.int64)))
    x, y = Trainer._cat_window(mbs)
    assert x.shape == (3, 3, 8, 8) and x._ddlpc_nhwc.shape == (3, 8, 8, 8)
    assert [int(v) for v in y[:, 0, 0]] == [0, 1, 2]
    assert [float(v) for v in x._ddlpc_nhwc[:, 0, 0, 0]] == [0.0, 1.0, 2.0]
    # micro-batches of unequal size cannot form one window (their BatchNorm groups and loss
    # weights would be wrong)
    mbs.append((engine_input(torch.zeros(2, 8, 8, 8), 3), torch.zeros(2, 8, 8, dtype=torch.int64)))
    with pytest.raises(ValueError):
        Trainer._cat_window(mbs)
    tr.close()


def test_bn_group_support_geometry():
    """The grouped BatchNorm kernels' shape contract, checked before a window is chosen:
    the standard U-Net widths (width divisor 1: 512 pooled channels) are supported; a BN
    width whose C / 8 is not a power of two, or an odd pooled extent, is not."""
    from ddlpc.models import UNet
    from ddlpc.ops.fused_unet import bn_groups_supported
    assert bn_groups_supported(UNet(out_classes=6, width_divisor=1), 512)
    assert bn_groups_supported(UNet(out_classes=6, width_divisor=2), 128)
    assert not bn_groups_supported(UNet(out_classes=6, width_divisor=2), 48)   # 48 >> 4 = 3
    m = UNet(out_classes=6, width_divisor=2, base_widths=(24, 48, 96, 192, 192))
    assert not bn_groups_supported(m, 256)                                    # C / 8 = 3


def test_collective_model_fit_recovers_latency_and_bandwidth():
    from ddlpc.parallel.bucket_plan import fit_collective_model
    world, gbps, lat_us = 8, 150.0, 25.0
    f = 2.0 * (world - 1) / world
    sizes = [1e6, 4e6, 8e6, 16e6]
    ms = [lat_us * 1e-3 + f * b / (gbps * 1e6) for b in sizes]
    g, l = fit_collective_model(sizes, ms, world)
    assert abs(g - gbps) < 1e-6 * gbps and abs(l - lat_us) < 1e-6
    assert fit_collective_model([4e6, 4e6], [0.1, 0.1], world) is None
