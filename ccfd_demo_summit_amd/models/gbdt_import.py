"""GBDT weight import ("a GBDT weight importer"): oblivious ensembles
trained elsewhere -> ``ObliviousGBDT`` (and from there the G20 / G32 / f32 device kernels).

CatBoost's default trees are oblivious -- the model family of BASELINE.json config 4 -- and
its JSON dump (``model.save_model(path, format="json")``) carries everything the kernels
need:

* ``oblivious_trees[t].splits``: one split per level, ``{"float_feature_index": f,
  "border": b, "split_type": "FloatFeature"}``; split ``d`` of a tree sets bit ``d`` of the
  leaf index when ``x[f] > b`` -- exactly ``ObliviousGBDT.leaf_index``;
* ``oblivious_trees[t].leaf_values``: ``2**depth`` raw values (binary logloss);
* ``scale_and_bias``: ``[scale, [bias]]`` -> raw score = scale * sum(leaves) + bias;
* ``features_info.float_features[i].flat_feature_index``: the input column of float
  feature ``i`` (categorical features are not supported: transactions are 30 floats).

Trees of a smaller depth than the deepest are padded to the common depth with never-firing
splits (NaN threshold: ``x > NaN`` is false, so the leaf index keeps its low bits) and their
leaves are replicated accordingly.  No CatBoost is installed here, so the importer is pinned
by hand-built documents of that schema (tests/test_models_cpu.py); parity with a real dump
is unpinned.
"""
from __future__ import annotations

import json
from typing import Any, Dict, Optional, Union

import numpy as np

from ..contracts.transaction import N_FEATURES
from .gbdt import MAX_DEPTH, ObliviousGBDT


def from_catboost_json(doc: Union[str, Dict[str, Any]], column_of: Optional[Dict[int, int]] = None) -> ObliviousGBDT:
    """CatBoost JSON model (path, JSON text or parsed dict) -> ObliviousGBDT.
    ``column_of``: override of float-feature index -> transaction column (0..29)."""
    if isinstance(doc, str):
        if doc.lstrip().startswith("{"):
            doc = json.loads(doc)
        else:
            with open(doc) as f:
                doc = json.load(f)
    trees = doc.get("oblivious_trees")
    if not trees:
        raise ValueError("not a CatBoost oblivious model: no 'oblivious_trees'")
    ff = (doc.get("features_info") or {}).get("float_features") or []
    if (doc.get("features_info") or {}).get("categorical_features"):
        raise ValueError("categorical features are not supported (transactions are 30 floats)")
    cols = {int(f.get("feature_index", i)): int(f.get("flat_feature_index", f.get("feature_index", i)))
            for i, f in enumerate(ff)}
    cols.update(column_of or {})
    depth = max(len(t.get("splits") or []) for t in trees)
    if not 1 <= depth <= MAX_DEPTH:
        raise ValueError(f"tree depth {depth} outside 1..{MAX_DEPTH}")
    T = len(trees)
    feat = np.zeros((T, depth), np.int32)
    thr = np.full((T, depth), np.nan, np.float32)
    leaves = np.zeros((T, 1 << depth), np.float32)
    for t, tree in enumerate(trees):
        splits = tree.get("splits") or []
        for d, s in enumerate(splits):
            if s.get("split_type", "FloatFeature") != "FloatFeature":
                raise ValueError(f"tree {t}: split type {s.get('split_type')!r} (only FloatFeature)")
            f = int(s["float_feature_index"])
            col = cols.get(f, f)
            if not 0 <= col < N_FEATURES:
                raise ValueError(f"tree {t}: feature {f} maps to column {col} outside 0..{N_FEATURES - 1}")
            feat[t, d] = col
            thr[t, d] = np.float32(s["border"])
        vals = np.asarray(tree.get("leaf_values"), np.float64).reshape(-1)
        dt = len(splits)
        if vals.size != (1 << dt):
            raise ValueError(f"tree {t}: {vals.size} leaf values for depth {dt} (multi-class models are not supported)")
        # padded levels never fire, so leaf index = its low dt bits: replicate the table
        leaves[t] = np.tile(vals, 1 << (depth - dt)).astype(np.float32)
    scale, bias = 1.0, 0.0
    sb = doc.get("scale_and_bias")
    if sb:
        scale = float(sb[0])
        b = sb[1]
        bias = float(b[0] if isinstance(b, (list, tuple)) else b)
    leaves = (leaves.astype(np.float64) * scale).astype(np.float32)
    return ObliviousGBDT(feat, thr, leaves, float(bias))


def to_catboost_json(model: ObliviousGBDT) -> Dict[str, Any]:
    """The inverse (for round trips and for handing an ensemble trained here to CatBoost
    tooling): float feature i == transaction column i."""
    trees = []
    for t in range(model.n_trees):
        trees.append({"leaf_values": model.leaves[t].astype(float).tolist(),
                      "splits": [{"border": float(model.thr[t, d]), "float_feature_index": int(model.feat[t, d]),
                                  "split_type": "FloatFeature"} for d in range(model.depth)]})
    ff = [{"feature_index": i, "flat_feature_index": i} for i in range(N_FEATURES)]
    return {"features_info": {"float_features": ff}, "oblivious_trees": trees,
            "scale_and_bias": [1.0, [float(model.base)]]}
