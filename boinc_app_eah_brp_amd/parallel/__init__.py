"""Multi-GPU / multi-process parallelism (template-bank sharding over RCCL)."""
from .dist import (CollectiveError, DistContext, ShardedSearch, allgather_tables, barrier, degrade,  # noqa: F401
                   init_distributed, max_floors_over_ranks, max_over_ranks, merge_tables, shard_range,
                   sharded_merge, table_floors)
