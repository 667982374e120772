"""The model workbench (examples/model_workbench.py, the JupyterHub/Spark workbench analogue,
SURVEY.md §2.1 C19) runs end to end on the CPU: trains LR/MLP/GBDT, the G32 leaves equal the
f32 model's, the saved safetensors reload to the same probabilities."""
import importlib.util
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def test_workbench_runs_on_cpu(tmp_path):
    spec = importlib.util.spec_from_file_location("model_workbench", ROOT / "examples" / "model_workbench.py")
    wb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(wb)
    r = wb.main(["--rows", "30000", "--trees", "8", "--epochs", "2", "--batch", "1024", "--device", "cpu", "--out", str(tmp_path)])
    assert set(r["models"]) == {"lr", "mlp", "gbdt"}
    assert all(0.9 <= v["roc_auc"] <= 1.0 for v in r["models"].values())
    assert r["g32"]["leaves_equal"] and r["g32"]["rows"] == 6000
    assert sorted(p.name for p in tmp_path.iterdir()) == ["gbdt.safetensors", "lr.safetensors", "mlp.safetensors"]


def test_leaf_index_g32_matches_f32_with_non_finite_inputs():
    import numpy as np
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.models import build_model
    X, _ = generate(5000, seed=4)
    X[3, 2], X[4, 9], X[5, 29] = np.nan, np.inf, -np.inf
    m = build_model("gbdt", seed=2, X_ref=X[10:])
    m.thr[0, 0] = np.nan                                   # a never-firing split
    sp = m.bin_spec()
    np.testing.assert_array_equal(m.leaf_index(X), m.leaf_index_g32(sp.encode(X), sp))



@pytest.mark.gpu
def test_workbench_scores_through_the_hip_kernels(gpu, tmp_path):
    spec = importlib.util.spec_from_file_location("model_workbench", ROOT / "examples" / "model_workbench.py")
    wb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(wb)
    r = wb.main(["--rows", "60000", "--trees", "20", "--epochs", "2", "--batch", "2048", "--device", "cuda:0",
                 "--out", str(tmp_path)])
    assert r["g32"]["leaves_equal"]
    # bf16 MLP vs its fp32 CPU model; LR / GBDT (exact leaves) tighter
    assert r["gpu"]["mlp"]["max_abs_dp"] < 2e-2
    assert r["gpu"]["lr"]["max_abs_dp"] < 1e-3 and r["gpu"]["gbdt"]["max_abs_dp"] < 1e-5
