from .dist import (DistInfo, assert_replicas_identical, broadcast_buffers, broadcast_module,
                   broadcast_tensors, init_distributed, params_checksum, shutdown)
from .flat import FlatParams, flatten_module
from .reducer import GradBucketReducer

__all__ = ["DistInfo", "init_distributed", "shutdown", "broadcast_module",
           "broadcast_buffers", "broadcast_tensors", "assert_replicas_identical", "params_checksum",
           "FlatParams", "flatten_module", "GradBucketReducer"]
