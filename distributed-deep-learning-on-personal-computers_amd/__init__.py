"""MI355X-native distributed U-Net segmentation trainer.

Capabilities of NikolayKrivosheev/Distributed-deep-learning-on-personal-computers
(one script, ``/root/reference/Vaihingen PyTorch 2 (кластер).py``), rebuilt for AMD
MI355X: hand-written HIP/CDNA4 kernels for the U-Net hot path, RCCL data parallelism
over xGMI, and a CPU/gloo path for tests.  See SURVEY.md for the component map.
"""
from .config import ModelConfig, TrainConfig
from .models.unet import UNet

__version__ = "0.1.0"

__all__ = ["ModelConfig", "TrainConfig", "UNet", "__version__"]
