"""Per-rank sharded, seeded index streams.

The reference loads the SAME directory in the SAME order on every PC (ref.py:732,849)
and never applies its per-epoch shuffle (``indxs`` is computed and unused,
ref.py:722-723); so its "data parallelism" adds no new data per step.

``ShardedSampler`` gives each rank a disjoint, rank-strided slice of a seeded per-epoch
permutation (``shard=True``, the default), or reproduces the reference's replicated mode
(``shard=False``: every rank sees every sample in order).
"""
from __future__ import annotations

from typing import Iterator, List

import torch


class ShardedSampler:
    def __init__(self, length: int, rank: int = 0, world_size: int = 1, shard: bool = True,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = True):
        self.length, self.rank, self.world = length, rank, world_size
        self.shard, self.shuffle, self.seed, self.drop_last = shard, shuffle, seed, drop_last
        self.epoch = 0

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def indices(self) -> List[int]:
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + 7919 * self.epoch)
            order = torch.randperm(self.length, generator=g).tolist()
        else:
            order = list(range(self.length))
        if not self.shard or self.world == 1:
            return order
        if self.drop_last:
            n = (self.length // self.world) * self.world
            order = order[:n]
        return order[self.rank::self.world]

    def __len__(self):
        if not self.shard or self.world == 1:
            return self.length
        return self.length // self.world if self.drop_last else -(-self.length // self.world)

    def __iter__(self) -> Iterator[int]:
        return iter(self.indices())

    def batches(self, batch_size: int) -> Iterator[List[int]]:
        idx = self.indices()
        for i in range(0, len(idx) - batch_size + 1 if self.drop_last else len(idx), batch_size):
            yield idx[i:i + batch_size]
