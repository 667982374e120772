"""Training (JupyterHub/Spark workbench replacement): LR/MLP on PyTorch-ROCm, oblivious GBDT."""
from .trainer import TrainConfig, evaluate, train_logistic, train_mlp, train_oblivious_gbdt

__all__ = ["TrainConfig", "evaluate", "train_logistic", "train_mlp", "train_oblivious_gbdt"]
