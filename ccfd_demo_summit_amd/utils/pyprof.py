"""Opt-in Python profile of a long-running service (the tracing / profiling subsystem of
SURVEY.md §5, for the Python side that rocprofv3 does not see).

``CCFD_PYPROF=<dir>``: the service enables ``cProfile`` on its main (event-loop) thread at
start-up and writes ``<dir>/<name>-<pid>.prof`` when it receives SIGTERM (how the deploy
harness and the operator stop it) or exits; read it with ``python -m pstats``.  Off by
default: the profiler slows a broker's event loop by ~2x.
"""
from __future__ import annotations

import os


def install_from_env(name: str) -> bool:
    out = os.environ.get("CCFD_PYPROF", "")
    if not out:
        return False
    import atexit
    import cProfile
    import signal
    os.makedirs(out, exist_ok=True)
    prof = cProfile.Profile()
    path = os.path.join(out, f"{name}-{os.getpid()}.prof")
    done = [False]

    def dump():
        if not done[0]:
            done[0] = True
            prof.disable()
            prof.dump_stats(path)

    def on_term(*_a):
        dump()
        os._exit(0)
    signal.signal(signal.SIGTERM, on_term)
    atexit.register(dump)
    prof.enable()
    return True
