"""End-to-end engine tests of ``test_unet_gpu.py`` on the CPU kernels.

``UNetEngine`` is one code path for both devices (``torch.ops.ddlpc`` dispatches to the
gfx950 kernels or to ``csrc/cpu_ref.cpp``), so the engine-level checks — against the fp32
stock-module oracle, exact checkpoint resume, accumulation, activation recompute, deferred
skips — run here on CPU tensors with the GPU tests' own bounds.  Tests of GPU-only mechanisms
(hipGraph capture, side / micro-batch streams, the schedule probe, HBM accounting) and the
largest shapes stay GPU-only (``_CPU`` lists what runs here).
"""
import os

import pytest

_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "test_unet_gpu.py")
_src = open(_path).read()
assert 'DEV = "cuda"' in _src and "pytestmark = pytest.mark.gpu" in _src
_src = _src.replace('DEV = "cuda"', 'DEV = "cpu"', 1).replace(
    "pytestmark = pytest.mark.gpu", "pytestmark = []", 1)
_ns = {"__name__": __name__, "__file__": _path}
exec(compile(_src, _path, "exec"), _ns)

# (the two gradient-direction tests bound the engine against CUDA autocast; on the CPU the
# same checks run against fp32 with CPU-autocast margins in tests/test_engine_cpu.py)
_CPU = ["test_trainer_hip_step_decreases_loss", "test_hip_checkpoint_resume_is_exact",
        "test_hip_grad_accumulation_matches_fp32_oracle", "test_deferred_skips_match_materialised_engine"]
for _k, _v in _ns.items():
    if _k.startswith("__"):
        continue
    if not _k.startswith("test_") or _k in _CPU:
        globals()[_k] = _v
