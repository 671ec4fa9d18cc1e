"""Multi-GPU / multi-process parallelism (template-bank sharding over RCCL)."""
from .dist import (DistContext, ShardedSearch, allgather_tables, barrier, init_distributed,  # noqa: F401
                   max_over_ranks, merge_tables, shard_range)
