"""The kernel numerics suite of ``test_kernels_gpu.py`` run against the CPU kernels.

``torch.ops.ddlpc`` has two kernels per operator: the gfx950 HIP kernel (GPU tensors) and the
C++ / ATen reference of ``csrc/cpu_ref.cpp`` (CPU tensors), chosen by PyTorch's dispatcher
(SURVEY.md §7.4).  This module re-runs every test of ``test_kernels_gpu.py`` on CPU tensors
(same inputs, same fp32 references, same tolerances), so both kernels of an operator are held
to one specification.  Tests of GPU-only mechanisms (kernel variants selected by launch
geometry, device-side scalars inside captured graphs, guard-page bounds) or shapes too large
for a CPU test run are listed in ``_GPU_ONLY`` and skipped here.
"""
import os

import pytest

_src = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "test_kernels_gpu.py")).read()
assert 'DEV = "cuda"' in _src and "pytestmark = pytest.mark.gpu" in _src
_src = _src.replace("pytestmark = pytest.mark.gpu", "pytestmark = []", 1).replace(
    'DEV = "cuda"', 'DEV = "cpu"', 1)
exec(compile(_src, os.path.join(os.path.dirname(os.path.abspath(__file__)), "test_kernels_gpu.py"),
             "exec"), globals())

# GPU-only mechanisms: one-launch device accumulation checked with device synchronisation
_GPU_ONLY = {"test_meter_add_single_launch"}
for _name in _GPU_ONLY:
    del globals()[_name]
