"""scikit-learn model import: bring a fraud model trained in the reference's Python workbench
(the JupyterHub / Spark notebooks, deploy/frauddetection_cr.yaml:7-53; the Seldon
``modelfull`` container serves a Python model, deploy/model/modelfull.json:24) onto the
MI355X kernels.

Accepted estimators, fitted on the 30 transaction columns (Time, V1..V28, Amount):

* ``LogisticRegression`` (binary)                       -> ``LogisticModel`` (K2 kernel);
* ``MLPClassifier(hidden_layer_sizes=(128, 64), activation="relu")`` (binary)
                                                       -> ``MLPModel`` (K3 MFMA kernel);
* either of them behind a ``StandardScaler`` in a ``Pipeline`` (or ``make_pipeline``): the
  scaler becomes the model's ``Normalizer`` (mu = mean_, 1/sigma = 1/scale_), which the
  kernels fuse into their prologue -- or, on W64 rows, fold into the first layer.

The MLP kernel is specialised to 30 -> 128 -> 64 -> 1; other architectures are refused
with a clear error.  The estimator object is taken as-is: loading it from disk (joblib /
pickle) is the caller's decision -- only ever do that with files you produced yourself.

    from ccfd_demo_summit_amd.models.sklearn_import import from_sklearn
    model = from_sklearn(fitted_pipeline)      # then save_model(model, "m.safetensors")
"""
from __future__ import annotations

from typing import Any, Optional

import numpy as np

from ..contracts.transaction import N_FEATURES
from .common import Normalizer
from .lr import LogisticModel
from .mlp import H1, H2, MLPModel


def _normalizer(scaler: Optional[Any]) -> Normalizer:
    if scaler is None:
        return Normalizer.identity()
    name = type(scaler).__name__
    if name != "StandardScaler":
        raise ValueError(f"unsupported preprocessing step {name} (only StandardScaler folds into the kernels)")
    mean = getattr(scaler, "mean_", None)
    scale = getattr(scaler, "scale_", None)
    mu = np.zeros(N_FEATURES, np.float32) if mean is None else np.asarray(mean, np.float32)
    isg = np.ones(N_FEATURES, np.float32) if scale is None else (1.0 / np.asarray(scale, np.float64)).astype(np.float32)
    if mu.shape != (N_FEATURES,) or isg.shape != (N_FEATURES,):
        raise ValueError(f"scaler was fitted on {mu.shape[0]} features, transactions have {N_FEATURES}")
    return Normalizer(mu, isg, log_amount=False)


def _binary(est: Any) -> None:
    classes = getattr(est, "classes_", None)
    if classes is None:
        raise ValueError(f"{type(est).__name__} is not fitted")
    if len(classes) != 2:
        raise ValueError(f"{type(est).__name__} has {len(classes)} classes; the fraud scorer is binary")


def from_sklearn(est: Any) -> Any:
    """Fitted scikit-learn estimator or ``Pipeline`` -> LogisticModel / MLPModel whose
    ``predict_proba`` equals the estimator's ``predict_proba(X)[:, 1]`` (up to float32)."""
    scaler = None
    if type(est).__name__ == "Pipeline":
        steps = [s for _, s in est.steps if s is not None and s != "passthrough"]
        if not steps:
            raise ValueError("empty pipeline")
        *pre, est = steps
        if len(pre) > 1:
            raise ValueError(f"pipeline has {len(pre)} preprocessing steps; at most one StandardScaler folds in")
        scaler = pre[0] if pre else None
    norm = _normalizer(scaler)
    name = type(est).__name__
    _binary(est)
    if name == "LogisticRegression":
        coef = np.asarray(est.coef_, np.float64)
        if coef.shape != (1, N_FEATURES):
            raise ValueError(f"LogisticRegression coef_ shape {coef.shape}, expected (1, {N_FEATURES})")
        return LogisticModel(coef[0].astype(np.float32), float(np.asarray(est.intercept_)[0]), norm)
    if name == "MLPClassifier":
        if est.activation != "relu":
            raise ValueError(f"MLPClassifier activation {est.activation!r}: the kernel implements relu")
        shapes = [tuple(w.shape) for w in est.coefs_]
        want = [(N_FEATURES, H1), (H1, H2), (H2, 1)]
        if shapes != want:
            raise ValueError(f"MLPClassifier layer shapes {shapes}; the MLP kernel is 30 -> {H1} -> {H2} -> 1 "
                             f"(hidden_layer_sizes=({H1}, {H2}))")
        W1, W2, W3 = (np.asarray(w, np.float32) for w in est.coefs_)
        b1, b2, b3 = (np.asarray(b, np.float32) for b in est.intercepts_)
        return MLPModel(W1.T.copy(), b1.copy(), W2.T.copy(), b2.copy(), W3[:, 0].copy(), float(b3[0]), norm)
    raise ValueError(f"unsupported estimator {name}: LogisticRegression or MLPClassifier (optionally after a "
                     "StandardScaler) map onto the kernels; oblivious GBDTs import via models.gbdt_import")
