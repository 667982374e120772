"""GPU-resident micro-batching engine (native core in csrc/engine/engine.cpp)."""
from .stream_engine import PartitionLog, PinnedArray, StepStats, StreamEngine

__all__ = ["PartitionLog", "PinnedArray", "StepStats", "StreamEngine"]
