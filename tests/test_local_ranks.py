"""``python bench.py --gpus N`` self-spawns N local ranks (launch/local_ranks.py; VERDICT r3
"Next #1"): argv pass-through, one JSON line on stdout, worst per-rank exit code, rehearsal
env, and no re-spawn when WORLD_SIZE is already set.  CPU only: the ranks run a tiny script
(or bench.py itself, which exits on a box without a GPU)."""
import io
import json
import os
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from ccfd_demo_summit_amd.launch import local_ranks  # noqa: E402

RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys
    sys.path.insert(0, {root!r})
    from ccfd_demo_summit_amd.launch.local_ranks import record_rank_rc
    rank = int(os.environ["RANK"])
    print("rank", rank, "chatter on stdout", flush=True)
    if rank == 0:
        print(json.dumps({{"metric": "m", "value": 1.0, "argv": sys.argv[1:],
                          "world": os.environ["WORLD_SIZE"],
                          "backend": os.environ.get("CCFD_DIST_BACKEND"),
                          "modulo": os.environ.get("CCFD_DEVICE_MODULO")}}), flush=True)
    code = int(os.environ.get("FAIL_RANK_CODE", "0")) if rank == int(os.environ.get("FAIL_RANK", "-1")) else 0
    record_rank_rc(code)
    sys.exit(code)
""")


@pytest.fixture()
def script(tmp_path):
    p = tmp_path / "rank_script.py"
    p.write_text(RANK_SCRIPT.format(root=str(ROOT)))
    return str(p)


def _run(script, argv, nproc, extra_env=None, env=None):
    out, err = io.StringIO(), io.StringIO()
    old = dict(os.environ)
    try:
        os.environ.update(env or {})
        rc = local_ranks.run_ranks(script, argv, nproc, extra_env=extra_env, out=out, err=err)
    finally:
        os.environ.clear()
        os.environ.update(old)
    return rc, out.getvalue(), err.getvalue()


def test_argv_passthrough_and_single_json_line(script):
    rc, out, err = _run(script, ["--gpus", "2", "--steps", "3", "--warmup", "1"], 2)
    assert rc == 0, err[-2000:]
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1, out                  # chatter went to stderr
    d = json.loads(lines[0])
    assert d["argv"] == ["--gpus", "2", "--steps", "3", "--warmup", "1"] and d["world"] == "2"
    assert "chatter on stdout" in err


def test_worst_rank_rc_propagates(script):
    rc, out, err = _run(script, [], 2, env={"FAIL_RANK": "1", "FAIL_RANK_CODE": "7"})
    assert rc == 7, err[-2000:]
    assert "per-rank rc={0: 0, 1: 7}" in err


def test_rehearsal_env_reaches_ranks(script):
    rc, out, _ = _run(script, ["--rehearsal"], 2, extra_env=dict(local_ranks.REHEARSAL_ENV))
    d = json.loads(out.strip())
    assert rc == 0 and d["backend"] == "gloo" and d["modulo"] == "1"


def test_worst_rc_rules():
    assert local_ranks.worst_rc(0, {0: 0, 1: 0}) == 0
    assert local_ranks.worst_rc(1, {0: 0, 1: 4}) == 4
    assert local_ranks.worst_rc(1, {0: 3, 1: 4}) == 4
    assert local_ranks.worst_rc(1, {}) == 1            # a rank killed by a signal reports nothing


def test_needs_spawn_only_for_plain_multi_gpu_invocations():
    assert local_ranks.needs_spawn(2, {})
    assert not local_ranks.needs_spawn(1, {})
    # an explicit WORLD_SIZE is never re-launched, even when it disagrees with --gpus: the
    # bench's topology check refuses that (tests/test_bench_topology.py)
    assert not local_ranks.needs_spawn(8, {"WORLD_SIZE": "1"})
    assert not local_ranks.needs_spawn(8, {"WORLD_SIZE": "8"})


def test_is_metric_line():
    assert local_ranks.is_metric_line('{"metric": "x", "value": 1}\n')
    assert not local_ranks.is_metric_line('{"phase": "x"}')
    assert not local_ranks.is_metric_line("[bench] hello")


def test_bench_parent_spawns_and_propagates_rank_failure():
    """bench.py --gpus 2 on a box without a GPU: the parent spawns 2 ranks (it never needs a
    GPU itself), each rank refuses to run, the job fails with their code."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0
    assert "[launch] 2 local ranks" in r.stderr and "--nproc-per-node 2" in r.stderr
    assert "needs a GPU" in r.stderr
    assert r.stdout.strip() == ""


def test_bench_mismatched_world_size_is_not_respawned():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0 and "[launch]" not in r.stderr


def test_host_dram_ceiling_sums_concurrent_rates():
    """Synthetic dp8 on 2 nodes: the concurrent per-rank rates of a node are its share, so the
    node figure is their sum (or the lead's solo probe if larger), never the max."""
    import bench
    per_rank = []
    for r in range(8):
        node = r // 4
        per_rank.append({"rank": r, "host": "h", "numa_node": node,
                         "host_numa_read_GBps": [12.9, 78.1, 40.0, 50.0][r % 4],
                         "host_node_probe_GBps": (150.0 if node == 0 else 400.0) if r % 4 == 0 else None})
    nodes, ceiling = bench.host_dram_ceiling(per_rank, 64)
    assert nodes["h:0"]["concurrent_sum"] == pytest.approx(181.0)
    assert nodes["h:0"]["GBps"] == pytest.approx(181.0)          # sum beats the lead probe
    assert nodes["h:1"]["GBps"] == pytest.approx(400.0)          # lead probe beats the sum
    assert nodes["h:0"]["ranks"] == [0, 1, 2, 3]
    assert ceiling == pytest.approx((181.0 + 400.0) * 1e9 / 64, rel=1e-6)
    # no probes -> no ceiling
    assert bench.host_dram_ceiling([{"rank": 0, "numa_node": None}], 64)[1] is None


def test_node_leads():
    import bench
    leads = bench.node_leads([(3, "a", 0), (1, "a", 0), (2, "a", 1), (0, "b", 0)])
    assert leads == {("a", 0): 1, ("a", 1): 2, ("b", 0): 0}
