"""CCFD_LIB_PATH (ops/_lib.py) selects an A/B build of the native library (scripts/build_ab.py)
without touching the default one."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lib_path(env_extra):
    env = dict(os.environ, **env_extra)
    out = subprocess.run([sys.executable, "-c", "from ccfd_demo_summit_amd.ops import _lib; print(_lib.LIB_PATH)"],
                         cwd=ROOT, env=env, capture_output=True, text=True, check=True)
    return out.stdout.strip()


def test_default_and_override_paths(tmp_path):
    env = {k: "" for k in ("CCFD_LIB_PATH", "CCFD_SANITIZE")}
    assert _lib_path(env).endswith(os.path.join("_native", "libccfd_hip.so"))
    alt = tmp_path / "variant.so"
    assert _lib_path(dict(env, CCFD_LIB_PATH=str(alt))) == str(alt.resolve())
