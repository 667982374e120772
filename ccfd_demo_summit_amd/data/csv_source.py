"""Reader for the Kaggle ``creditcard.csv`` layout (``Time,V1..V28,Amount,Class``).

The reference producer reads it from S3 (``s3bucket``/``filename``,
ProducerDeployment.yaml:92-95).  We read a local path (S3 is optional and needs
network); the file is not shipped, so tests use a synthetic CSV with the same header.
"""
from __future__ import annotations

import csv
from typing import Optional, Tuple

import numpy as np

from ..contracts.transaction import FEATURE_NAMES, N_FEATURES


def read_creditcard_csv(path: str, limit: Optional[int] = None) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    with open(path, newline="") as f:
        rd = csv.reader(f)
        header = [h.strip().strip('"') for h in next(rd)]
        try:
            cols = [header.index(n) for n in FEATURE_NAMES]
        except ValueError as e:
            raise ValueError(f"{path}: missing column ({e})") from None
        ycol = header.index("Class") if "Class" in header else None
        X, y = [], []
        for i, row in enumerate(rd):
            if limit is not None and i >= limit:
                break
            X.append([float(row[c]) for c in cols])
            if ycol is not None:
                y.append(int(float(row[ycol].strip('"'))))
    Xa = np.asarray(X, dtype=np.float32).reshape(-1, N_FEATURES)
    ya = np.asarray(y, dtype=np.uint8) if ycol is not None else None
    return Xa, ya


def write_creditcard_csv(path: str, X: np.ndarray, y: Optional[np.ndarray] = None) -> None:
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(list(FEATURE_NAMES) + (["Class"] if y is not None else []))
        for i in range(X.shape[0]):
            row = [repr(float(v)) for v in X[i]]
            if y is not None:
                row.append(str(int(y[i])))
            w.writerow(row)
