"""Self-spawn of N local ranks for a script invoked as ``script.py --gpus N``.

``python bench.py --gpus 8`` is how the driver invokes config 2 at N = 1; config 3 (8-way
DP, BASELINE.json ``configs[2]``; the reference's only scale knob is ``replicas``,
/root/reference/deploy/model/modelfull.json:46) must start the same way.  When ``--gpus N > 1``
and no ``WORLD_SIZE`` is set, the script's parent process calls :func:`run_ranks`, which runs
``python -m torch.distributed.run --nnodes 1 --nproc-per-node N --master-addr 127.0.0.1
--master-port P script.py <same argv>`` as a CHILD process:

- the parent never imports torch and never touches the GPU, and it never replaces itself
  (no exec): it waits for the child and exits with the worst rank's code;
- the children's stdout is streamed line by line: the metric JSON line(s) (rank 0 prints
  exactly one) go to the parent's stdout, everything else to its stderr, so stdout carries
  ONE JSON line whatever the ranks print;
- SIGTERM / SIGINT to the parent are forwarded to the launcher (which tears the ranks down);
  the launcher gets SIGTERM if the parent dies (``PR_SET_PDEATHSIG``), so no resident
  kernel outlives the job;
- each rank writes its own exit code into ``CCFD_RANK_RC_DIR`` (:func:`record_rank_rc`), so
  the parent returns the worst per-rank code rather than torchrun's generic 1.

This module must stay torch-free: it runs in the parent before any GPU work.
"""
from __future__ import annotations

import ctypes
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import threading
from pathlib import Path
from typing import Dict, List, Optional, Sequence

RC_DIR_ENV = "CCFD_RANK_RC_DIR"
# env a --rehearsal parent gives its children: N ranks may share the box's GPU(s), and the
# collectives go over gloo (RCCL refuses two ranks on one GPU); bench.py labels the line
REHEARSAL_ENV = {"CCFD_DIST_BACKEND": "gloo", "CCFD_DEVICE_MODULO": "1"}


def needs_spawn(gpus: int, env: Optional[Dict[str, str]] = None) -> bool:
    """True when this process is a plain ``--gpus N>1`` invocation (not already a rank).

    An explicit WORLD_SIZE that disagrees with --gpus is NOT spawned over: the script's own
    topology check refuses it (a mismatched rank count must not be silently re-launched)."""
    env = os.environ if env is None else env
    return int(gpus) > 1 and "WORLD_SIZE" not in env


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_cmd(script: str, argv: Sequence[str], nproc: int, port: int) -> List[str]:
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
            "--master-addr", "127.0.0.1", "--master-port", str(port), script, *argv]


def is_metric_line(line: str) -> bool:
    s = line.strip()
    if not (s.startswith("{") and s.endswith("}")):
        return False
    try:
        d = json.loads(s)
    except ValueError:
        return False
    return isinstance(d, dict) and "metric" in d and "value" in d


def record_rank_rc(code: int) -> None:
    """Called by a rank on its way out: write its exit code where the parent collects it."""
    d = os.environ.get(RC_DIR_ENV)
    if not d:
        return
    try:
        rank = os.environ.get("RANK", "x")
        Path(d, f"rank{rank}.rc").write_text(str(int(code)))
    except OSError:
        pass


def worst_rc(launcher_rc: int, rank_rcs: Dict[int, int]) -> int:
    """The job's exit code: 0 only if the launcher and every reporting rank succeeded; else the
    worst (largest) non-zero per-rank code, or the launcher's own when no rank reported one
    (a rank killed by a signal writes nothing)."""
    bad = [c for c in rank_rcs.values() if c != 0]
    if bad:
        return max(bad)
    return int(launcher_rc)


def read_rank_rcs(d: str) -> Dict[int, int]:
    out = {}
    for p in Path(d).glob("rank*.rc"):
        try:
            out[int(p.stem[4:])] = int(p.read_text().strip())
        except ValueError:
            continue
    return out


def _pdeathsig():
    try:
        libc = ctypes.CDLL("libc.so.6", use_errno=True)
        libc.prctl(1, signal.SIGTERM)        # PR_SET_PDEATHSIG
    except OSError:
        pass


def run_ranks(script: str, argv: Sequence[str], nproc: int, extra_env: Optional[Dict[str, str]] = None,
              out=None, err=None, port: Optional[int] = None) -> int:
    """Run ``script argv`` as ``nproc`` local ranks under torch.distributed.run; returns the
    worst exit code.  ``out`` / ``err`` default to sys.stdout / sys.stderr."""
    out = out or sys.stdout
    err = err or sys.stderr
    rc_dir = tempfile.mkdtemp(prefix="ccfd_rank_rc_")
    env = dict(os.environ)
    env.update(extra_env or {})
    env[RC_DIR_ENV] = rc_dir
    env["PYTHONUNBUFFERED"] = "1"
    cmd = launcher_cmd(script, argv, nproc, port or free_port())
    print(f"[launch] {nproc} local ranks: {' '.join(cmd)}", file=err, flush=True)
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=None, env=env, text=True, bufsize=1,
                            preexec_fn=_pdeathsig)
    forwarded = []

    def _fwd(signum, _frame):
        forwarded.append(signum)
        try:
            proc.send_signal(signum)
        except ProcessLookupError:
            pass
    old = {s: signal.signal(s, _fwd) for s in (signal.SIGTERM, signal.SIGINT)} \
        if threading.current_thread() is threading.main_thread() else {}
    try:
        for line in proc.stdout:
            if is_metric_line(line):
                out.write(line if line.endswith("\n") else line + "\n")
                out.flush()
            else:
                err.write(line)
                err.flush()
        launcher_rc = proc.wait()
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    rcs = read_rank_rcs(rc_dir)
    for p in Path(rc_dir).glob("*"):
        p.unlink()
    os.rmdir(rc_dir)
    rc = worst_rc(launcher_rc, rcs)
    if rc != 0:
        print(f"[launch] launcher rc={launcher_rc}, per-rank rc={dict(sorted(rcs.items()))}"
              + (f", forwarded signals {forwarded}" if forwarded else ""), file=err, flush=True)
    if launcher_rc < 0 and rc == launcher_rc:
        rc = 128 - launcher_rc                 # killed by a signal: shell convention
    return rc
