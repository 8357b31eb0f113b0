"""The generated-geometry kernel properties of ``test_properties.py`` on the CPU kernels.

Same hypothesis strategies, same fp32 oracles, same tolerances as the GPU part of
``test_properties.py``, run on CPU tensors so ``torch.ops.ddlpc`` dispatches to the C++
reference kernels of ``csrc/cpu_ref.cpp`` (the CPU-only tests of that module are not
repeated here).
"""
import os

_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "test_properties.py")
_src = open(_path).read()
assert 'DEV = "cuda"' in _src and "@pytest.mark.gpu" in _src
_src = _src.replace('DEV = "cuda"', 'DEV = "cpu"', 1).replace("@pytest.mark.gpu\n", "")
_ns = {"__name__": __name__, "__file__": _path}
exec(compile(_src, _path, "exec"), _ns)
# keep the kernel properties (the ones that were GPU-marked), not the CPU-only ones
for _k, _v in _ns.items():
    if _k.startswith("test_") and "ops" in getattr(_v, "__code__", type("", (), {"co_varnames": ()})).co_varnames:
        globals()[_k] = _v
    elif not _k.startswith("test_"):
        globals().setdefault(_k, _v)
