"""Launcher + supervisor (restart-on-crash, crash-loop give-up, graceful stop)."""
import os
import subprocess
import sys

from ccfd_demo_summit_amd.launch.supervisor import supervise


def test_supervisor_restarts_until_success(tmp_path):
    marker = tmp_path / "count"
    script = tmp_path / "flaky.py"
    script.write_text(
        "import sys, pathlib\n"
        f"p = pathlib.Path({str(marker)!r})\n"
        "n = int(p.read_text()) if p.exists() else 0\n"
        "p.write_text(str(n + 1))\n"
        "sys.exit(0 if n >= 2 else 3)\n")
    logs = []
    rc = supervise([sys.executable, str(script)], max_restarts=5, backoff_s=0.01, log=logs.append)
    assert rc == 0
    assert marker.read_text() == "3"
    assert len(logs) == 2


def test_supervisor_gives_up_on_crash_loop():
    logs = []
    rc = supervise([sys.executable, "-c", "import sys; sys.exit(7)"], max_restarts=2, backoff_s=0.01,
                   log=logs.append)
    assert rc == 7
    assert "crash loop" in logs[-1]


def test_launch_help_and_demo():
    env = dict(os.environ, CCFD_NO_NUMA_BIND="1")
    out = subprocess.run([sys.executable, "-m", "ccfd_demo_summit_amd.launch", "--help"], capture_output=True,
                         text=True, env=env, timeout=120)
    assert out.returncode == 0 and "kafka-lite" in out.stdout
    out = subprocess.run([sys.executable, "-m", "ccfd_demo_summit_amd.launch", "demo", "--device", "cpu",
                          "--seconds", "1", "--batch", "500", "--port", "0"],
                         capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert '"consumed"' in out.stdout


def test_launch_options_after_service_name_are_parsed():
    from ccfd_demo_summit_amd.launch.__main__ import parse_args
    a = parse_args(["engine", "--port", "18091", "--host", "127.0.0.1", "--watch-model", "m.safetensors"])
    assert (a.service, a.port, a.host, a.watch_model, a.cmd) == ("engine", 18091, "127.0.0.1", "m.safetensors", [])
    a = parse_args(["--port", "1", "kafka-lite"])
    assert a.port == 1 and a.service == "kafka-lite"
    a = parse_args(["supervise", "--max-restarts", "3", "--", "python", "-c", "print(1)", "--port", "9"])
    assert a.max_restarts == 3 and a.cmd == ["python", "-c", "print(1)", "--port", "9"] and a.port is None
