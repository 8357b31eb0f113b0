"""CLI entry point (``python -m ddlpc``): config resolution, train and validate on CPU."""
import json
import os
import subprocess
import sys

from ddlpc.cli import main

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--tile", "64", "--depth", "4", "--batch-per-gpu", "2", "--num-samples", "8",
         "--test-holdout", "2", "--device", "cpu"]


def test_config_flags(capsys):
    assert main(["config", "--tile", "128", "--max-steps", "7", "--width-divisor", "4",
                 "--grad-codec", "fp16_absmax"]) == 0
    d = json.loads(capsys.readouterr().out)
    assert d["tile"] == 128 and d["max_steps"] == 7 and d["grad_codec"] == "fp16_absmax"
    assert d["model"]["width_divisor"] == 4


def test_train_then_validate_checkpoint(tmp_path, capsys):
    ck = str(tmp_path / "ck")
    assert main(["train", *SMALL, "--max-steps", "2", "--ckpt-dir", ck]) == 0
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert out["cmd"] == "train" and out["steps"] == 2.0
    files = sorted(os.listdir(ck))
    assert files, "train() must write a checkpoint at the end"
    assert main(["validate", *SMALL, "--checkpoint", os.path.join(ck, files[-1])]) == 0
    v = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert v["cmd"] == "validate" and 0.0 <= v["val_pixel_acc"] <= 1.0


def test_module_entry_point():
    r = subprocess.run([sys.executable, "-m", "ddlpc", "config", "--depth", "3"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout)["model"]["depth"] == 3
