from .comm import NO_COMM, TPComm, TPRankProxyComm
from .dist import ParallelContext, init_distributed, single_process_context
from .partition import (Mesh, P, PartitionSpec, get_llama_param_partition_spec, get_partition_spec,
                        shard_tree, with_named_sharding_constraint, with_sharding_constraint)

__all__ = ["TPComm", "TPRankProxyComm", "NO_COMM", "ParallelContext", "init_distributed", "single_process_context", "Mesh",
           "P", "PartitionSpec", "get_llama_param_partition_spec", "get_partition_spec", "shard_tree",
           "with_named_sharding_constraint", "with_sharding_constraint"]
