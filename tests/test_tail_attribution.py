"""bench/tail_attribution.py on a synthetic trace: a batch that waited while the scoring thread
was out of run() during a GC pause is charged to gc; one that waited inside run() to in_run."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "bench"))


def test_attribution_splits_queue_time(tmp_path):
    import tail_attribution as ta
    from ccfd_demo_summit_amd.ops._lib import BATCH_TRACE_DTYPE
    b = np.zeros(100, BATCH_TRACE_DTYPE)
    us = 1000
    b["t_arrival"] = np.arange(100) * 100 * us + 1
    b["t_submit"] = b["t_arrival"] + 5 * us
    b["t_landed"] = b["t_submit"] + 20 * us
    # batch 50 waits 3 ms: the scoring thread left run() for a 3 ms GC pause
    a50 = int(b["t_arrival"][50])
    b["t_submit"][50] = a50 + 3000 * us
    b["t_landed"][50] = b["t_submit"][50] + 20 * us
    b["dev_start"] = b["t_submit"] + 2 * us           # device clock: its own epoch, only differences count
    b["dev_end"] = b["dev_start"] + 15 * us
    runs = [(0, a50 - 10 * us, 0), (a50 + 2990 * us, 10 ** 12, 0)]
    gc = [(a50 + 100 * us, 0, 2), (a50 + 2900 * us, 1, 2)]
    np.savez(tmp_path / "rank0.npz", batches=b, runs=np.array(runs, np.int64), tasks=np.zeros((0, 2), np.int64),
             task_names=np.array([], "U32"), gc=np.array(gc, np.int64), held=np.zeros((0, 2), np.int64),
             t_dump=np.int64(10 ** 12))
    r = ta.attribute(str(tmp_path / "rank0.npz"), tail_q=0.99)
    bd = r["tail_mean_breakdown_us"]
    assert r["batches"] == 100 and r["tail_batches_ge_p99"] == 1
    assert 2790 <= bd["gc"] <= 2810 and bd["outside_run"] >= 2990 and bd["in_run"] <= 10
    assert bd["flight"] == 20.0
    assert bd["device_exec"] == 15.0 and bd["flight_other"] == 5.0
    # aligned device clock: post -> first claim + last item -> host = 5 us
    assert bd["device_start_wait"] == 5.0 and bd["host_notice"] == 0.0   # the fastest notice defines 0
    assert r["device_exec_us"]["p99"] == 15.0 and r["device_exec_us"]["batches"] == 100
