"""Restart-based elasticity: a rank dies mid-epoch (fault-injection
hook), ``torchrun --max-restarts`` relaunches the job, ``--resume auto`` picks up the last
checkpoint — including the position inside the epoch — and the run ends with exactly the
weights of an uninterrupted run.  CPU / gloo, 2 ranks."""
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--impl", "torch", "--device", "cpu", "--tile", "32", "--depth", "4",
        "--width-divisor", "16", "--num-samples", "16", "--test-holdout", "4",
        "--batch-per-gpu", "2", "--epochs", "5", "--max-steps", "4", "--ckpt-every", "1",
        "--log-every", "0"]


def _torchrun(extra, restarts=0):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    # c10d rendezvous on port 0: torchrun's agent binds the store's port itself (no
    # probe-then-bind race with other processes for a "free" port)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--rdzv-backend", "c10d", "--rdzv-endpoint", "127.0.0.1:0",
           "--max-restarts", str(restarts), "-m", "ddlpc", "train", *ARGS, *extra]
    return subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)


def test_rank_failure_restart_resumes_to_identical_weights(tmp_path):
    ref_dir, el_dir = str(tmp_path / "ref"), str(tmp_path / "elastic")
    r = _torchrun(["--ckpt-dir", ref_dir])
    assert r.returncode == 0, r.stderr[-3000:]
    r = _torchrun(["--ckpt-dir", el_dir, "--resume", "auto", "--fault-rank", "1",
                   "--fault-step", "2"], restarts=1)
    assert r.returncode == 0, r.stderr[-3000:]
    # the injected failure happened (marker written by the dying rank), and torchrun restarted
    assert os.path.exists(os.path.join(el_dir, "fault_rank1_step2.marker")), os.listdir(el_dir)
    assert "exitcode: 17" in r.stderr or "exitcode  : 17" in r.stderr, r.stderr[-2000:]
    a = torch.load(os.path.join(ref_dir, "ckpt_4.pt"), weights_only=True)
    b = torch.load(os.path.join(el_dir, "ckpt_4.pt"), weights_only=True)
    assert a["step"] == b["step"] == 4 and a["epoch"] == b["epoch"]
    for k, v in a["model"].items():
        assert torch.equal(v, b["model"][k]), k
