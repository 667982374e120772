"""Seldon-compatible serving (predict() REST) and scoring back-ends."""
from .scorers import CpuScorer, GpuScorer, make_scorer

__all__ = ["CpuScorer", "GpuScorer", "make_scorer"]
