"""Native library checks that need no GPU: ABI layout and the C++ JSON ingest parser."""
import ctypes as C
import json
import subprocess

import numpy as np
import pytest

from ccfd_demo_summit_amd.contracts import FEATURE_NAMES


@pytest.fixture(scope="module")
def L():
    from ccfd_demo_summit_amd.ops._lib import lib
    return lib()


def test_abi_struct_sizes(L, tmp_path):
    from ccfd_demo_summit_amd.ops._lib import EngineConfig, EngineStats, Flagged, ScoreArgs
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include "ccfd_abi.h"\nint main(){printf("%zu %zu %zu %zu",'
                   'sizeof(ccfd_score_args),sizeof(ccfd_engine_config),sizeof(ccfd_flagged),'
                   'sizeof(ccfd_engine_stats));}\n')
    from ccfd_demo_summit_amd.ops.build import CSRC
    exe = tmp_path / "sz"
    r = subprocess.run(["gcc", str(src), "-I", str(CSRC / "include"), "-o", str(exe)], capture_output=True)
    if r.returncode != 0:
        pytest.skip("no C compiler")
    out = subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()
    assert [int(v) for v in out] == [C.sizeof(ScoreArgs), C.sizeof(EngineConfig), C.sizeof(Flagged),
                                     C.sizeof(EngineStats)]


def _parse(L, msgs):
    bufs = [m if isinstance(m, bytes) else m.encode() for m in msgs]
    buf = b"".join(bufs)
    off = np.cumsum([0] + [len(b) for b in bufs]).astype(np.int64)
    n = len(bufs)
    f = np.zeros((n, 30), np.float32)
    ids = np.zeros(n, np.uint64)
    cu = np.zeros(n, np.uint32)
    rc = L.ccfd_parse_json_batch(buf, off.ctypes.data, n, f.ctypes.data, ids.ctypes.data, cu.ctypes.data)
    return rc, f, ids, cu


def test_json_parser_named_columns(L):
    rng = np.random.default_rng(0)
    vals = rng.standard_normal((50, 30)).astype(np.float32)
    msgs = []
    for i in range(50):
        d = {"id": 100 + i, "customer_id": i * 3, "extra": {"nested": [1, "x", None, True]}}
        d.update({n: float(v) for n, v in zip(FEATURE_NAMES, vals[i])})
        msgs.append(json.dumps(d))
    rc, f, ids, cu = _parse(L, msgs)
    assert rc == 50
    np.testing.assert_allclose(f, vals, rtol=1e-6)
    assert ids.tolist() == list(range(100, 150))
    assert cu.tolist() == [i * 3 for i in range(50)]


@pytest.mark.parametrize("sanitizer", ["thread", "address,undefined"])
def test_spsc_ring_stress_under_sanitizers(tmp_path, sanitizer):
    """The engine's SPSC row ring (csrc/engine/spsc_ring.h) under ThreadSanitizer and
    ASan/UBSan with randomised producer/consumer timing (SURVEY.md §5 race detection)."""
    from ccfd_demo_summit_amd.ops.build import CSRC
    exe = tmp_path / "ring_stress"
    r = subprocess.run(["g++", "-O1", "-g", "-std=c++17", f"-fsanitize={sanitizer}", "-pthread",
                        str(CSRC / "tests" / "ring_stress.cpp"), "-o", str(exe)], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip(f"sanitizer build unavailable: {r.stderr[-300:]}")
    out = subprocess.run([str(exe), "200000", "4093"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "ring stress ok" in out.stdout


def test_json_parser_features_array_and_errors(L):
    rc, f, ids, _ = _parse(L, [json.dumps({"features": list(range(30)), "tx_id": "12"})])
    assert rc == 1 and ids[0] == 12
    np.testing.assert_array_equal(f[0], np.arange(30))
    rc, *_ = _parse(L, [json.dumps({"Amount": 1.0}), "{broken"])
    assert rc == -2
    rc, *_ = _parse(L, [json.dumps({"features": [1, 2, 3]})])
    assert rc == -1
