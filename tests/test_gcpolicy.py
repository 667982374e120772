"""utils/gcpolicy.py: the service GC policy freezes start-up objects and raises thresholds;
CCFD_GC=default leaves CPython's defaults (run in a subprocess: GC state is global)."""
import subprocess
import sys


def _run(env_mode):
    code = ("import gc, os\n"
            "from ccfd_demo_summit_amd.utils.gcpolicy import tune_for_service\n"
            "r = tune_for_service()\n"
            "print(r, gc.get_threshold(), gc.get_freeze_count())\n")
    import os
    env = dict(os.environ)
    if env_mode:
        env["CCFD_GC"] = env_mode
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=60).stdout


def test_service_policy_and_default_switch():
    out = _run(None)
    assert "(10000, 1, 1000000)" in out and out.startswith("frozen")
    assert int(out.split()[-1]) > 1000
    out = _run("default")
    assert out.startswith("default") and "(700, 10, 10)" in out
