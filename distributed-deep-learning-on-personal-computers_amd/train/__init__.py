from .checkpoint import latest_checkpoint, load_checkpoint, save_checkpoint
from .trainer import Trainer, train, validate

__all__ = ["Trainer", "train", "validate", "save_checkpoint", "load_checkpoint",
           "latest_checkpoint"]
