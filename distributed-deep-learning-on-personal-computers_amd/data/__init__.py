from .datasets import (SyntheticTiles, TileDataset, device_random_batch, load_files,
                       to_tensors)
from .sampler import ShardedSampler

__all__ = ["SyntheticTiles", "TileDataset", "ShardedSampler", "load_files", "to_tensors",
           "device_random_batch"]
