"""Progress watchdog (utils/watchdog.py) + the ``stall`` fault (utils/faults.py): a rank that
stops stepping is reported with its state and exits non-zero instead of hanging until the
process-group timeout."""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

from ccfd_demo_summit_amd.utils.faults import FaultPlan
from ccfd_demo_summit_amd.utils.watchdog import EXIT_STALLED, Watchdog

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_watchdog_fires_with_state_and_code():
    codes = []
    wd = Watchdog(0.3, lambda: {"posted": 7, "ticks": 3}, rank=2, exit_fn=codes.append, poll_s=0.02).start()
    for _ in range(5):                       # beating keeps it quiet
        time.sleep(0.1)
        wd.beat("step")
    assert not wd.fired
    time.sleep(0.8)                          # stall
    assert wd.fired and codes == [EXIT_STALLED]
    assert wd.report["rank"] == 2 and wd.report["state"] == {"posted": 7, "ticks": 3}
    assert wd.report["last_progress"] == "step"
    wd.stop()


def test_watchdog_state_error_does_not_mask_stall():
    codes = []

    def bad():
        raise RuntimeError("engine gone")
    wd = Watchdog(0.1, bad, exit_fn=codes.append, poll_s=0.02).start()
    time.sleep(0.5)
    assert codes == [EXIT_STALLED] and "engine gone" in wd.report["state_error"]


def test_stall_fault_parses():
    p = FaultPlan.parse("stall:after_steps=4,rank=1", rank=1)
    assert p.clauses[0].kind == "stall" and p.clauses[0].after_steps == 4


def test_stalled_rank_process_exits_nonzero_with_diagnostic(tmp_path):
    """A child 'rank' steps under the watchdog with CCFD_FAULTS=stall: it must end by itself
    (exit 5) and print the JSON diagnostic on stderr -- no external kill."""
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent(f"""
        import sys, time
        sys.path.insert(0, {ROOT!r})
        from ccfd_demo_summit_amd.utils.faults import FaultPlan
        from ccfd_demo_summit_amd.utils.watchdog import Watchdog
        state = {{"steps": 0, "last_collective": "x2_all_reduce#2"}}
        wd = Watchdog(1.0, lambda: dict(state), rank=1, poll_s=0.05).start()
        plan = FaultPlan.from_env(rank=1)
        for k in range(10_000):
            plan.step()
            state["steps"] += 1
            wd.beat(f"step {{k}}")
            time.sleep(0.01)
        print("finished without stalling")
    """))
    env = dict(os.environ, CCFD_FAULTS="stall:after_steps=5,rank=1")
    t0 = time.time()
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, env=env, timeout=60)
    assert r.returncode == EXIT_STALLED, (r.returncode, r.stdout, r.stderr)
    assert time.time() - t0 < 30
    line = [ln for ln in r.stderr.splitlines() if ln.startswith("[watchdog]")][0]
    rep = json.loads(line.split(" -- ", 1)[1])
    assert rep["rank"] == 1 and rep["state"]["steps"] == 4
    assert rep["state"]["last_collective"] == "x2_all_reduce#2" and rep["last_progress"] == "step 3"


@pytest.mark.gpu
def test_bench_watchdog_fires_on_stalled_rank(gpu):
    """bench.py itself: a rank wedged after 3 steps (CCFD_FAULTS stall) ends with the watchdog
    diagnostic and exit code 5, well inside the driver's limits."""
    env = dict(os.environ, CCFD_FAULTS="stall:after_steps=3")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "2",
                        "--watchdog-s", "8", "--batches-per-step", "16", "--log-rows", str(1 << 18),
                        "--probe-ms", "0", "--host-probe-s", "0", "--precision-rows", "0",
                        "--encode-probe-rows", "0", "--no-unloaded-probe", "--no-f32-probe",
                        "--diagnostic"],                 # fault injection: a labelled diagnostic run
                       capture_output=True, text=True, env=env, timeout=110)
    assert r.returncode == EXIT_STALLED, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    line = [ln for ln in r.stderr.splitlines() if ln.startswith("[watchdog]")][0]
    rep = json.loads(line.split(" -- ", 1)[1])
    assert rep["state"]["phase"] in ("warmup", "calibration") and "engine" in rep["state"]
    assert rep["state"]["engine"]["submitted"] >= rep["state"]["engine"]["completed"]
    # the persistent scoring kernel was asked to leave and drained before the exit
    assert "exit hook returned 0" in r.stderr, r.stderr[-2000:]
