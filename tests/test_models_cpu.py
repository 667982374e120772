"""CPU checks of the model families and of the kernel weight packing (the NumPy lane
emulator walks the exact MFMA fragment maps the HIP kernel uses)."""
import numpy as np
import pytest

from ccfd_demo_summit_amd.data import FRAUD_RATE, generate
from ccfd_demo_summit_amd.models import (LogisticModel, MLPModel, ObliviousGBDT, build_model, load_model,
                                         save_model)
from ccfd_demo_summit_amd.models.common import Normalizer, bf16_round
from ccfd_demo_summit_amd.models.mlp import BLOB_BYTES, emulate_packed_kernel


@pytest.fixture(scope="module")
def X():
    return generate(20000, seed=3)[0]


def test_synthetic_shape_and_prior():
    X, y = generate(200_000, seed=1)
    assert X.shape == (200_000, 30) and X.dtype == np.float32
    assert abs(y.mean() - FRAUD_RATE) < 0.001
    assert (X[:, 29] >= 0).all() and X[:, 29].max() <= 25691.16 + 1e-3
    assert np.all(np.diff(X[:, 0]) >= 0)      # Time is monotone
    # fraud rows are shifted on V14/V17 (negative)
    assert X[y == 1, 14].mean() < X[y == 0, 14].mean() - 3


def test_bf16_round_rne():
    x = np.array([1.0, 1.00390625, 1.01171875, -2.5, 3.0e38], np.float32)
    r = bf16_round(x)
    assert r[0] == 1.0
    assert r[1] == 1.0            # tie -> even
    assert r[2] == 1.015625       # tie -> even (up)
    assert r[3] == -2.5


@pytest.mark.parametrize("n", [1, 15, 16, 17, 40])
def test_mlp_packing_emulator_matches_bf16_oracle(X, n):
    m = build_model("mlp", seed=2, X_ref=X)
    blob = m.pack()
    assert len(blob) == BLOB_BYTES
    pe = emulate_packed_kernel(blob, X[:n])
    np.testing.assert_allclose(pe, m.predict_proba(X[:n], emulate_bf16=True), atol=1e-6)
    assert np.abs(pe - m.predict_proba(X[:n])).max() < 1e-2


def test_calibration_hits_target_rate(X):
    for kind in ("lr", "mlp", "gbdt"):
        m = build_model(kind, seed=4, X_ref=X, calibrate_rate=0.01)
        rate = (m.predict_proba(X) >= 0.5).mean()
        assert abs(rate - 0.01) < 0.003, (kind, rate)


def test_gbdt_pack_unpack_and_leaf_index(X):
    g = ObliviousGBDT.random_init(50, 6, seed=1, X_ref=X)
    g2 = ObliviousGBDT.unpack(g.pack())
    np.testing.assert_array_equal(g2.feat, g.feat)
    np.testing.assert_array_equal(g2.leaves, g.leaves)
    idx = g.leaf_index(X[:5])
    assert idx.shape == (5, 50) and idx.max() < 64
    # manual check of one row / tree
    t, r = 7, 3
    manual = sum(int(X[r, g.feat[t, d]] > g.thr[t, d]) << d for d in range(6))
    assert idx[r, t] == manual
    with pytest.raises(ValueError):
        ObliviousGBDT(np.zeros((2, 9), np.int32), np.zeros((2, 9), np.float32), np.zeros((2, 512), np.float32))


def test_normalizer(X):
    nz = Normalizer.fit(X)
    Z = nz(X)
    assert np.abs(Z.mean(0)).max() < 1e-3
    assert np.abs(Z.std(0) - 1).max() < 1e-2


@pytest.mark.parametrize("kind", ["lr", "mlp", "gbdt"])
def test_save_load_roundtrip(tmp_path, X, kind):
    m = build_model(kind, seed=5, X_ref=X)
    p = tmp_path / f"{kind}.safetensors"
    save_model(m, str(p), version="3")
    m2 = load_model(str(p))
    assert type(m2) is type(m)
    np.testing.assert_allclose(m2.predict_proba(X[:100]), m.predict_proba(X[:100]), atol=1e-7)
    assert m2.pack() == m.pack()


def test_lr_predict_one(X):
    m = LogisticModel.random_init(0, Normalizer.fit(X))
    assert abs(m.predict_one(X[0]) - m.predict_proba(X[:1])[0]) < 1e-7


def test_mlp_param_count():
    assert MLPModel.random_init(0).n_params == 12289


# ---------------------------------------------------------------------------------------
# GBDT weight import: CatBoost JSON oblivious trees
def _catboost_doc(rng):
    """Hand-built CatBoost-schema dump: mixed depths, float features mapped onto
    transaction columns out of order, scale and bias."""
    cols = rng.permutation(30)
    ff = [{"feature_index": i, "flat_feature_index": int(cols[i])} for i in range(30)]
    trees = []
    for t in range(12):
        d = int(rng.integers(2, 7))
        trees.append({"leaf_values": rng.normal(0, 0.3, 1 << d).tolist(), "leaf_weights": [1.0] * (1 << d),
                      "splits": [{"border": float(rng.normal()), "float_feature_index": int(rng.integers(0, 30)),
                                  "split_index": 0, "split_type": "FloatFeature"} for _ in range(d)]})
    return {"features_info": {"float_features": ff}, "oblivious_trees": trees, "scale_and_bias": [0.7, [-1.25]]}


def _catboost_raw(doc, X):
    """Independent evaluator of the CatBoost schema: bit d of the leaf index is split d."""
    col = {f["feature_index"]: f["flat_feature_index"] for f in doc["features_info"]["float_features"]}
    raw = np.zeros(len(X))
    for tree in doc["oblivious_trees"]:
        idx = np.zeros(len(X), np.int64)
        for d, s in enumerate(tree["splits"]):
            idx |= (X[:, col[s["float_feature_index"]]] > np.float32(s["border"])).astype(np.int64) << d
        raw += np.asarray(tree["leaf_values"])[idx]
    sc, b = doc["scale_and_bias"]
    return sc * raw + b[0]


def test_catboost_json_import_matches_an_independent_evaluator(tmp_path):
    import json
    from ccfd_demo_summit_amd.models.gbdt_import import from_catboost_json, to_catboost_json
    rng = np.random.default_rng(5)
    doc = _catboost_doc(rng)
    X, _ = generate(5000, seed=8)
    X[:, :] = X / (np.abs(X).max(0) + 1e-6)            # borders ~ N(0,1) split these columns
    p = tmp_path / "cb.json"
    p.write_text(json.dumps(doc))
    m = from_catboost_json(str(p))
    assert m.depth == max(len(t["splits"]) for t in doc["oblivious_trees"]) and m.n_trees == 12
    np.testing.assert_allclose(m.raw_score(X), _catboost_raw(doc, X), rtol=1e-5, atol=1e-5)
    # padded levels never fire, so the G32 table of the import stays exact
    spec = m.bin_spec()
    k = spec.bin_index(m.feat, m.thr)
    np.testing.assert_array_equal(spec.encode(X)[:, m.feat].astype(np.int32) > k[None], X[:, m.feat] > m.thr[None])
    # round trip through the exporter
    m2 = from_catboost_json(to_catboost_json(m))
    np.testing.assert_allclose(m2.raw_score(X), m.raw_score(X), rtol=1e-6, atol=1e-6)


def test_catboost_import_refuses_what_the_kernels_cannot_run():
    from ccfd_demo_summit_amd.models.gbdt_import import from_catboost_json
    doc = _catboost_doc(np.random.default_rng(1))
    doc["oblivious_trees"][0]["splits"][0]["split_type"] = "OneHotFeature"
    with pytest.raises(ValueError, match="FloatFeature"):
        from_catboost_json(doc)
    doc = _catboost_doc(np.random.default_rng(1))
    doc["oblivious_trees"][1]["leaf_values"] = doc["oblivious_trees"][1]["leaf_values"] * 3
    with pytest.raises(ValueError, match="multi-class"):
        from_catboost_json(doc)
    with pytest.raises(ValueError, match="oblivious"):
        from_catboost_json({"trees": []})


def _sk_data(n=6000, seed=8):
    from ccfd_demo_summit_amd.data import generate
    X, y = generate(n, seed=seed, fraud_rate=0.05)
    return X.astype(np.float64), y


def test_sklearn_logistic_regression_import_matches_predict_proba():
    """models/sklearn_import.py: a fitted LogisticRegression (bare and behind a StandardScaler)
    scores like sklearn's own predict_proba[:, 1]."""
    from sklearn.linear_model import LogisticRegression
    from sklearn.pipeline import make_pipeline
    from sklearn.preprocessing import StandardScaler
    from ccfd_demo_summit_amd.models.sklearn_import import from_sklearn
    X, y = _sk_data()
    for est in (make_pipeline(StandardScaler(), LogisticRegression(max_iter=300)),
                LogisticRegression(max_iter=2000, C=0.1)):
        est.fit(X, y)
        m = from_sklearn(est)
        assert m.kind == "lr"
        np.testing.assert_allclose(m.predict_proba(X[:2000]), est.predict_proba(X[:2000])[:, 1], atol=2e-6)


def test_sklearn_mlp_import_matches_predict_proba_and_refuses_other_shapes():
    import warnings
    from sklearn.exceptions import ConvergenceWarning
    from sklearn.neural_network import MLPClassifier
    from sklearn.pipeline import Pipeline
    from sklearn.preprocessing import MinMaxScaler, StandardScaler
    from ccfd_demo_summit_amd.models import load_model, save_model
    from ccfd_demo_summit_amd.models.sklearn_import import from_sklearn
    X, y = _sk_data()
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", ConvergenceWarning)
        pipe = Pipeline([("scale", StandardScaler()),
                         ("mlp", MLPClassifier(hidden_layer_sizes=(128, 64), max_iter=15, random_state=0))]).fit(X, y)
        small = MLPClassifier(hidden_layer_sizes=(32,), max_iter=5, random_state=0).fit(X, y)
        tanh = MLPClassifier(hidden_layer_sizes=(128, 64), activation="tanh", max_iter=3, random_state=0).fit(X, y)
    m = from_sklearn(pipe)
    assert m.kind == "mlp"
    np.testing.assert_allclose(m.predict_proba(X[:2000]), pipe.predict_proba(X[:2000])[:, 1], atol=2e-5)
    import os
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        save_model(m, os.path.join(d, "m.safetensors"))
        back = load_model(os.path.join(d, "m.safetensors"))
    np.testing.assert_allclose(back.predict_proba(X[:500]), m.predict_proba(X[:500]), atol=1e-7)
    with pytest.raises(ValueError, match="30 -> 128 -> 64 -> 1"):
        from_sklearn(small)
    with pytest.raises(ValueError, match="relu"):
        from_sklearn(tanh)
    with pytest.raises(ValueError, match="StandardScaler"):
        from_sklearn(Pipeline([("s", MinMaxScaler()), ("mlp", pipe.steps[-1][1])]))


def test_trained_gbdt_100x6_stays_on_g20_rows():
    """a TRAINED 100 x 6 ensemble (not only the random one) must keep the
    20-byte G20 row format: the trainer's split candidates are capped at 31 borders a feature
    (train/__main__.py --max-borders, n_bins = 32), so however the splits concentrate on few
    features, no feature exceeds 31 distinct thresholds."""
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.train.trainer import train_oblivious_gbdt
    Xt, yt = generate(30_000, seed=5, fraud_rate=0.02)
    m, _ = train_oblivious_gbdt(Xt, yt, n_trees=100, depth=6, device="cpu", n_bins=32)
    spec = m.bin_spec(bits=5)                           # raises if any feature needs > 31 edges
    ne = np.diff(spec.offsets)
    assert spec.row_format == "g20" and ne.max() <= 31
    # without the cap (255 candidates a feature) the same data can exceed G20's 31 edges
    m2, _ = train_oblivious_gbdt(Xt, yt, n_trees=100, depth=6, device="cpu", n_bins=256)
    assert np.diff(m2.bin_spec().offsets).max() >= np.diff(spec.offsets).max()


def test_same_bins_compares_the_whole_table_not_the_stamp():
    """the in-row stamp is 6 bits for G20 -- two different tables collide ~1/63 of
    the time; the host-side checks (log vs model, hot swap) compare the full edge table."""
    from ccfd_demo_summit_amd.engine.stream_engine import same_bins
    from ccfd_demo_summit_amd.models.gbdt import BinSpec
    rng = np.random.default_rng(0)
    base = [np.unique(rng.standard_normal(10).astype(np.float32)) for _ in range(30)]
    a = BinSpec([e.copy() for e in base], bits=5)
    assert same_bins(a, BinSpec([e.copy() for e in base], bits=5))
    assert not same_bins(a, a.with_bits(8))
    # find a different table with the same G20 stamp: the stamp alone would accept it
    for k in range(2000):
        e2 = [e.copy() for e in base]
        e2[k % 30] = np.unique(np.append(e2[k % 30], np.float32(5.0 + k)))
        b = BinSpec(e2, bits=5)
        if b.stamp == a.stamp:
            break
    assert b.stamp == a.stamp and not same_bins(a, b)
