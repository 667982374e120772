"""Restart-on-crash supervisor with graceful drain -- the analogue of the reference's
DeploymentConfig ``restartPolicy: Always`` + rolling strategy (deploy/router.yaml:10-31,
75-76; terminationGracePeriodSeconds 30; SURVEY.md §2.1 C20, §5 failure detection).

* runs the child as its own process (never exec: a GPU-initialised parent must not exec);
* on SIGTERM/SIGINT forwards SIGTERM, waits ``grace_s`` (30 s like the reference), then
  SIGKILLs the child's process group;
* restarts a child that exits non-zero with exponential back-off, up to ``max_restarts``
  within ``window_s`` (crash-loop protection), and returns the child's last exit code.
"""
from __future__ import annotations

import os
import signal
import subprocess
import sys
import time
from typing import List, Optional


def supervise(cmd: List[str], max_restarts: int = 10, backoff_s: float = 1.0, grace_s: float = 30.0,
              window_s: float = 600.0, env: Optional[dict] = None, log=print) -> int:
    if not cmd:
        log("[supervise] no command given")
        return 2
    stopping = {"flag": False}
    child: Optional[subprocess.Popen] = None

    def on_signal(signum, _frame):
        stopping["flag"] = True
        if child is not None and child.poll() is None:
            try:
                os.killpg(child.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    restarts: List[float] = []
    rc = 0
    try:
        while True:
            child = subprocess.Popen(cmd, env=env, start_new_session=True)
            while child.poll() is None:
                try:
                    child.wait(timeout=0.5)
                except subprocess.TimeoutExpired:
                    pass
                if stopping["flag"]:
                    try:
                        child.wait(timeout=grace_s)
                    except subprocess.TimeoutExpired:
                        try:
                            os.killpg(child.pid, signal.SIGKILL)
                        except ProcessLookupError:
                            pass
                        child.wait()
            rc = child.returncode
            if stopping["flag"] or rc == 0:
                return rc
            now = time.monotonic()
            restarts = [t for t in restarts if now - t < window_s] + [now]
            if len(restarts) > max_restarts:
                log(f"[supervise] crash loop: {len(restarts)} restarts in {window_s:.0f}s, giving up (rc={rc})")
                return rc
            delay = backoff_s * (2 ** (len(restarts) - 1))
            log(f"[supervise] child exited rc={rc}; restart #{len(restarts)} in {delay:.1f}s")
            time.sleep(min(delay, 60.0))
    finally:
        for s, h in old.items():
            signal.signal(s, h)


if __name__ == "__main__":
    sys.exit(supervise(sys.argv[1:]))
