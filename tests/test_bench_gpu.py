"""bench.py end to end on one MI355X: the JSON contract the driver parses, a sustained
timed region, exact row accounting, per-rank attribution and precision evidence."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_json_contract(gpu):
    r = _run(["--steps", "5", "--warmup", "2", "--min-timed-s", "0.3", "--log-rows", str(1 << 20),
              "--precision-rows", str(1 << 18)])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 5 and d["dtype"] == "bf16"
    assert d["timed_region_s"] >= 0.3
    assert d["rows_scored"] == d["rows_expected"]
    assert abs(d["value"] * d["timed_region_s"] - d["rows_scored"]) / d["rows_scored"] < 1e-3
    assert d["backend"] in ("none", "nccl") and not d["rehearsal"]
    assert len(d["per_rank"]) == 1 and d["per_rank"][0]["rows"] == d["rows_scored"]
    assert d["per_rank"][0]["h2d_zerocopy_GBps"] > 1
    pr = d["precision_vs_fp32"]
    assert pr["rows"] == 1 << 18 and pr["max_abs_dp"] < 1e-2 and pr["route_flips_outside_1e-2_band"] == 0
    assert d["f32_wire_tx_s"] > 0


def test_bench_refuses_gpu_count_mismatch(gpu):
    # an explicit WORLD_SIZE that disagrees with --gpus is refused, never re-launched
    r = _run(["--gpus", "2", "--steps", "2", "--warmup", "1"],
             env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr, r.stderr[-2000:]
    import torch
    if torch.cuda.device_count() < 2:
        # --gpus 2 self-spawns two ranks (launch/local_ranks.py); on a one-GPU box the second
        # rank refuses with a clear message and the parent exits non-zero
        r = _run(["--gpus", "2", "--steps", "2", "--warmup", "1"])
        assert r.returncode != 0 and "visible GPU" in r.stderr, r.stderr[-2000:]
