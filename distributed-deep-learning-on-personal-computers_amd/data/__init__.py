from .datasets import (DevicePrefetcher, SyntheticTiles, TileDataset, cat_adjacent,
                       device_random_batch, load_files, split_batch, to_tensors)
from .sampler import ShardedSampler

__all__ = ["SyntheticTiles", "TileDataset", "ShardedSampler", "load_files", "to_tensors",
           "device_random_batch", "split_batch", "cat_adjacent", "DevicePrefetcher"]
