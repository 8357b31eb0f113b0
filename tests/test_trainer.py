"""train()/validate() integration, resume, logs and PNG dumps on CPU (BASELINE config #1 shape)."""
import json
import os
import subprocess
import sys

import torch

from ddlpc.config import ModelConfig, TrainConfig
from ddlpc.train import Trainer, train, validate


def _cfg(tmp_path, **kw):
    base = dict(model=ModelConfig(out_classes=2, depth=4, width_divisor=8), tile=64,
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


def test_phase_timer_reads_on_cpu_are_empty():
    from ddlpc.utils.tracing import PhaseTimer, trace_range
    pt = PhaseTimer(torch.device("cpu"))
    pt.mark("start")
    with trace_range("x"):
        pt.mark("a")
    pt.end_step()
    assert pt.read() == {}


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
    line from rank 0 with the whole-job aggregate."""
    import socket
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                          "--master-port", str(port), os.path.join(root, "bench.py"),
                          "--gpus", "2", "--impl", "torch", "--steps", "2", "--warmup", "1",
                          "--batch", "2", "--tile", "64", "--width-divisor", "16"],
                         capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["global_batch"] == 4 and rec["value"] > 0
