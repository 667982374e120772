"""bench.py records its environment and refuses an unlabelled number under a diagnostic
variable (utils/benchenv.py)."""
import os
import subprocess
import sys
from pathlib import Path

from ccfd_demo_summit_amd.utils import benchenv

ROOT = Path(__file__).resolve().parents[1]


def test_collect_records_runtime_prefixes_only():
    env = {"CCFD_PERSIST_PIPE": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "0", "HIP_VISIBLE_DEVICES": "0",
           "PATH": "/usr/bin", "HOME": "/root"}
    rec = benchenv.collect(env)
    assert rec == {"CCFD_PERSIST_PIPE": "1", "HIP_VISIBLE_DEVICES": "0", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    d = benchenv.describe(env)
    assert d["tuning"] == ["CCFD_PERSIST_PIPE"] and d["diagnostic"] == []


def test_diagnostic_vars_refuse_unless_labelled():
    for k in ("CCFD_ABLATE", "CCFD_LIB_PATH", "CCFD_FAULTS", "HIP_LAUNCH_BLOCKING", "CCFD_DEBUG_SYNC"):
        env = {k: "576" if k == "CCFD_ABLATE" else "1"}
        assert benchenv.diagnostics(env) == [k]
        msg = benchenv.refusal(env)
        assert msg and k in msg and "--diagnostic" in msg
        assert benchenv.refusal(env, allow=True) is None
    # "0" / empty means unset
    assert benchenv.refusal({"CCFD_DEBUG_SYNC": "0", "HIP_LAUNCH_BLOCKING": ""}) is None


def test_bench_refuses_before_touching_the_gpu():
    """The refusal is the first thing bench.py does (no torch / GPU needed to see it)."""
    env = dict(os.environ, CCFD_ABLATE="576")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 3
    assert "refusing to print a headline number" in r.stderr and "CCFD_ABLATE" in r.stderr
    assert r.stdout.strip() == ""


def test_no_ablation_paths_in_the_default_build_sources():
    """The round-1..4 runtime ablation switches are gone from the kernels and the engine."""
    hits = []
    for p in list((ROOT / "csrc").rglob("*")):
        if p.suffix in (".h", ".hip", ".cpp") and "ABLATE" in p.read_text():
            hits.append(str(p))
    assert hits == []
