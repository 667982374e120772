"""Multi-GPU data parallelism (one process per GPU, RCCL over xGMI)."""
from .membership import ElasticCounterReducer, ElasticGroup, Membership
from .dp import (CounterReducer, DistContext, EpochPipeline, all_max, all_sum, assign_partitions, barrier,
                 broadcast_blob, broadcast_model, hist_quantile, init_distributed, resolve_row_format, x_group)

__all__ = ["ElasticCounterReducer", "ElasticGroup", "Membership", "CounterReducer", "DistContext", "EpochPipeline", "all_max", "all_sum", "assign_partitions", "barrier",
           "broadcast_blob", "broadcast_model", "hist_quantile", "init_distributed", "resolve_row_format", "x_group"]
