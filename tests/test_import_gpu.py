"""Imported models on the MI355X kernels: a scikit-learn MLP (behind a StandardScaler) and a
CatBoost-schema oblivious ensemble score on the GPU like their source frameworks' own
predict_proba (bf16 MFMA tolerance for the MLP, float summation order for the trees)."""
import warnings

import numpy as np
import pytest

from ccfd_demo_summit_amd.data import generate

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wire", [False, True])
def test_sklearn_mlp_on_the_mfma_kernel(gpu, wire):
    from sklearn.exceptions import ConvergenceWarning
    from sklearn.neural_network import MLPClassifier
    from sklearn.pipeline import make_pipeline
    from sklearn.preprocessing import StandardScaler
    from ccfd_demo_summit_amd.engine import StreamEngine
    from ccfd_demo_summit_amd.models.sklearn_import import from_sklearn
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    X, y = generate(20000, seed=12, fraud_rate=0.05)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", ConvergenceWarning)
        pipe = make_pipeline(StandardScaler(), MLPClassifier(hidden_layer_sizes=(128, 64), max_iter=20,
                                                             random_state=1)).fit(X.astype(np.float64), y)
    m = from_sklearn(pipe)
    eng = StreamEngine(DeviceModel(m, gpu, wire=wire), batch=4096, depth=2)
    p, _ = eng.score(X[:8000])
    eng.close()
    ref = pipe.predict_proba(X[:8000].astype(np.float64))[:, 1]
    assert np.abs(p - ref).max() < 2e-2 and np.abs(p - ref).mean() < 2e-3


def test_catboost_schema_ensemble_on_the_g32_kernel(gpu):
    from ccfd_demo_summit_amd.engine import StreamEngine
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.models.gbdt_import import from_catboost_json, to_catboost_json
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    X, _ = generate(20000, seed=13)
    src = build_model("gbdt", seed=4, X_ref=X, gbdt_trees=300, gbdt_depth=6)   # 300 x 64 leaves: L2 path
    m = from_catboost_json(to_catboost_json(src))
    eng = StreamEngine(DeviceModel(m, gpu, bins=True), batch=4096, depth=2)
    p, _ = eng.score(X[:8000])
    eng.close()
    assert np.abs(p - src.predict_proba(X[:8000])).max() < 2e-5
