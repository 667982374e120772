"""GPU-resident micro-batching engine (native core in csrc/engine/engine.cpp)."""
from .stream_engine import FlaggedDrainer, PartitionLog, PinnedArray, StepStats, StreamEngine

__all__ = ["FlaggedDrainer", "PartitionLog", "PinnedArray", "StepStats", "StreamEngine"]
