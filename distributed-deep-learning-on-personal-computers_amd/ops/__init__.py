"""Hand-written HIP/CDNA4 operators (``csrc/*.hip``) and their Python/autograd glue."""
from . import _ext

__all__ = ["_ext"]
