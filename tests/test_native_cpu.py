"""Native library checks that need no GPU: ABI layout and the C++ JSON ingest parser."""
import ctypes as C
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest

from ccfd_demo_summit_amd.contracts import FEATURE_NAMES


@pytest.fixture(scope="module")
def L():
    from ccfd_demo_summit_amd.ops._lib import lib
    return lib()


def test_abi_struct_sizes(L, tmp_path):
    from ccfd_demo_summit_amd.ops._lib import SCORED_DTYPE, EngineConfig, EngineStats, Flagged, ScoreArgs
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include "ccfd_abi.h"\nint main(){printf("%zu %zu %zu %zu %zu",'
                   'sizeof(ccfd_score_args),sizeof(ccfd_engine_config),sizeof(ccfd_flagged),'
                   'sizeof(ccfd_engine_stats),sizeof(ccfd_scored));}\n')
    from ccfd_demo_summit_amd.ops.build import CSRC
    exe = tmp_path / "sz"
    r = subprocess.run(["gcc", str(src), "-I", str(CSRC / "include"), "-o", str(exe)], capture_output=True)
    if r.returncode != 0:
        pytest.skip("no C compiler")
    out = subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()
    assert [int(v) for v in out] == [C.sizeof(ScoreArgs), C.sizeof(EngineConfig), C.sizeof(Flagged),
                                     C.sizeof(EngineStats), np.dtype(SCORED_DTYPE).itemsize]


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


def test_dedupe_index_stress_under_asan(tmp_path):
    """The KIE tier's windowed dedupe index (csrc/engine/dedupe.cpp) against a reference model
    under ASan/UBSan: repeats within and across batches, keys re-admitted after leaving the
    window, recovery inserts, lookups, a tiny window that wraps the table many times."""
    from ccfd_demo_summit_amd.ops.build import CSRC
    exe = tmp_path / "dedupe_stress"
    r = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined",
                        str(CSRC / "tests" / "dedupe_stress.cpp"), str(CSRC / "engine" / "dedupe.cpp"), "-o", str(exe)],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip(f"sanitizer build unavailable: {r.stderr[-300:]}")
    for rounds, window in ((3000, 1000), (600, 7)):
        out = subprocess.run([str(exe), str(rounds), str(window)], capture_output=True, text=True, timeout=600)
        assert out.returncode == 0, out.stderr[-3000:]
        assert "dedupe stress ok" in out.stdout


def test_json_parser_features_array_and_errors(L):
    rc, f, ids, _ = _parse(L, [json.dumps({"features": list(range(30)), "tx_id": "12"})])
    assert rc == 1 and ids[0] == 12
    np.testing.assert_array_equal(f[0], np.arange(30))
    rc, *_ = _parse(L, [json.dumps({"Amount": 1.0}), "{broken"])
    assert rc == -2
    rc, *_ = _parse(L, [json.dumps({"features": [1, 2, 3]})])
    assert rc == -1


def test_host_runtime_under_asan(tmp_path):
    """Host-sanitizer build of the native runtime: the JSON parser (valid,
    truncated, garbage), W64 / G32 / G20 encoders and CRC-32C run under clang ASan+UBSan in a child
    process with the runtime preloaded; any report fails the test."""
    import os
    import sys
    from ccfd_demo_summit_amd.ops.build import asan_runtime, build
    try:
        build(sanitize="address,undefined", verbose=False)
        rt = asan_runtime()
    except Exception as e:                                   # toolchain without sanitizer runtimes
        pytest.skip(f"sanitizer build unavailable: {e}")
    if not rt or not os.path.exists(rt):
        pytest.skip("clang ASan runtime not found")
    script = tmp_path / "asan_probe.py"
    script.write_text(
        "import json, numpy as np\n"
        "from ccfd_demo_summit_amd.ops._lib import lib\n"
        "from ccfd_demo_summit_amd.contracts import FEATURE_NAMES\n"
        "L = lib()\n"
        "assert 'address' in L._name, L._name\n"
        "rng = np.random.default_rng(0)\n"
        "msgs = [json.dumps({'id': i, **{n: float(v) for n, v in zip(FEATURE_NAMES, rng.standard_normal(30))}}).encode()"
        " for i in range(200)]\n"
        "msgs += [b'{\"id\": 1, \"Time\": 1e', b'', b'\\xff\\xfe{', b'{\"features\": [1,2,3,' + b'9,' * 4000 + b'1]}']\n"
        "for k in range(len(msgs)):\n"
        "    sub = msgs[k:k + 1]\n"
        "    buf = b''.join(sub); off = np.array([0, len(buf)], np.int64)\n"
        "    f = np.zeros((1, 30), np.float32); ids = np.zeros(1, np.uint64); cu = np.zeros(1, np.uint32)\n"
        "    rows = np.zeros((1, 64), np.uint8)\n"
        "    L.ccfd_parse_json_batch(buf, off.ctypes.data, 1, f.ctypes.data, ids.ctypes.data, cu.ctypes.data)\n"
        "    L.ccfd_parse_json_batch_w64(buf, off.ctypes.data, 1, rows.ctypes.data, ids.ctypes.data, cu.ctypes.data)\n"
        "X = rng.standard_normal((1000, 30)).astype(np.float32)\n"
        "out = np.zeros((1000, 64), np.uint8)\n"
        "assert L.ccfd_encode_w64(X.ctypes.data, 1000, 30, out.ctypes.data) == 1000\n"
        "assert L.ccfd_crc32c(bytes(range(256)) * 100, 25600, 0) != 0\n"
        "# G32 encoder (binary search over the bin table), incl. NaN/inf rows and a refused table\n"
        "from ccfd_demo_summit_amd.models.gbdt import ObliviousGBDT\n"
        "spec = ObliviousGBDT.random_init(50, 6, seed=0, X_ref=X).bin_spec()\n"
        "flat, offs = spec.flat, spec.offsets\n"
        "X[3, 4] = np.nan; X[5, 6] = np.inf\n"
        "g = np.zeros((1000, 32), np.uint8); am = np.zeros(1000, np.float32)\n"
        "assert L.ccfd_encode_g32(X.ctypes.data, 1000, 30, flat.ctypes.data, offs.ctypes.data, spec.stamp, g.ctypes.data, am.ctypes.data) == 1000\n"
        "assert (g == spec.encode(X)).all()\n"
        "bad = offs.copy(); bad[5] = bad[6] + 1\n"
        "assert L.ccfd_encode_g32(X.ctypes.data, 1000, 30, flat.ctypes.data, bad.ctypes.data, spec.stamp, g.ctypes.data, None) == -1\n"
        "# G20 encoder (5-bit fields straddling dwords) against the numpy oracle\n"
        "s5 = spec.with_bits(5)\n"
        "g5 = np.zeros((1000, 20), np.uint8)\n"
        "assert L.ccfd_encode_g20(X.ctypes.data, 1000, 30, flat.ctypes.data, offs.ctypes.data, s5.stamp, g5.ctypes.data, am.ctypes.data) == 1000\n"
        "assert (g5 == s5.encode(X)).all()\n"
        "# native Kafka consumer: Fetch/RecordBatch parsing against kafka-lite\n"
        "import time\n"
        "from ccfd_demo_summit_amd.contracts import TxBatch\n"
        "from ccfd_demo_summit_amd.ingest.kafka_lite import KafkaLiteServer\n"
        "from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker\n"
        "from ccfd_demo_summit_amd.ingest.native_consumer import NativeKafkaConsumer\n"
        "srv = KafkaLiteServer('127.0.0.1', 0, default_partitions=1).start_in_thread()\n"
        "kb = KafkaBroker(srv.bootstrap); kb.create_topic('t', 1)\n"
        "kb.produce('t', TxBatch(ids=np.arange(500, dtype=np.uint64), customer=np.zeros(500, np.uint32), features=X[:500]).encode(), partition=0)\n"
        "kb.produce_many('t', msgs[:50], partition=0)\n"
        "for kw in ({'wire': True}, {'bins': spec}):\n"
        "    kc = NativeKafkaConsumer.for_arrays(srv.bootstrap, 't', {0: 0}, capacity=1000, **kw).start()\n"
        "    t0 = time.time()\n"
        "    while kc.stats()['records'] < 51 and time.time() - t0 < 20: time.sleep(0.01)\n"
        "    assert kc.stats()['records'] == 51, kc.stats()\n"
        "    kc.stop(); kc.close()\n"
        "kb.close(); srv.stop()\n"
        "# fuzz the RecordBatch/TXB1/JSON parsers with truncated and bit-flipped record sets\n"
        "from ccfd_demo_summit_amd.ingest.kafka_wire import encode_record_batch\n"
        "good = encode_record_batch([TxBatch(ids=np.arange(64, dtype=np.uint64), customer=np.zeros(64, np.uint32), features=X[:64]).encode()] + msgs[:20], [None] * 21, base_offset=0)\n"
        "fz = NativeKafkaConsumer.for_arrays('127.0.0.1:1', 't', {0: 0}, capacity=100000, wire=False)\n"
        "assert fz.feed(good) == 21\n"
        "r = np.random.default_rng(1)\n"
        "for it in range(3000):\n"
        "    b = bytearray(good)\n"
        "    for _ in range(int(r.integers(1, 8))): b[int(r.integers(0, len(b)))] = int(r.integers(0, 256))\n"
        "    cut = int(r.integers(0, len(b) + 1)) if it % 3 == 0 else len(b)\n"
        "    fz.feed(bytes(b[:cut]))\n"
        "    fz.feed(bytes(r.integers(0, 256, int(r.integers(0, 300)), dtype=np.uint8)))\n"
        "# a CRC-valid batch whose record value length runs past the record (ADVICE r1): rejected, no over-read\n"
        "import struct\n"
        "from ccfd_demo_summit_amd.ingest.kafka_wire import _varint, crc32c, CODEC_GZIP\n"
        "def batch_of(recs, n):\n"
        "    after = struct.pack('>hiqqqhii', 0, n - 1, 0, 0, -1, -1, -1, n) + recs\n"
        "    return struct.pack('>qi', 0, 9 + len(after)) + struct.pack('>ibI', 0, 2, crc32c(after)) + after\n"
        "for vlen in (1 << 20, 40, 11):\n"
        "    body = b'\\x00' + _varint(0) + _varint(0) + _varint(-1) + _varint(vlen) + b'{\"id\": 1}' + _varint(0)\n"
        "    e0 = fz.stats()['errors']\n"
        "    fz.feed(batch_of(_varint(len(body)) + body, 1))\n"
        "    assert fz.stats()['errors'] > e0, vlen\n"
        "gz = encode_record_batch(msgs[:30], compression=CODEC_GZIP)\n"
        "gzc = NativeKafkaConsumer.for_arrays('127.0.0.1:1', 't', {0: 0}, capacity=1000, wire=False)\n"
        "assert gzc.feed(gz) == 30, gzc.last_error()\n"
        "for it in range(500):\n"
        "    b = bytearray(gz)\n"
        "    for _ in range(int(r.integers(1, 8))): b[int(r.integers(61, len(b)))] = int(r.integers(0, 256))\n"
        "    gzc.feed(bytes(b))\n"
        "gzc.close()\n"
        "fz.close()\n"
        "print('asan probe ok')\n")
    env = dict(os.environ, CCFD_SANITIZE="address,undefined", LD_PRELOAD=rt, CCFD_NO_AUTOBUILD="1",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               PYTHONPATH=str(Path(__file__).resolve().parents[1]), HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "asan probe ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


_EDGE_NUMBERS = ["0", "-0.0", "1", "-1.35981", "0.000123456", "123456.789", "1e5", "1E+5", "-2.5e-3",
                 "1.5E-30", "3.4028235e38", "1e-45", "0.1", "0.30000000000000004", "123456789012345678901",
                 "12345678.12345678", "9007199254740993", "1.7976931348623157e300", "4.9406564584124654e-324",
                 "00012.5", "7.", "-.5e1", "+3.25", "1234567890123456789"]


@pytest.mark.parametrize("pad", [0, 24])
def test_json_parser_numbers_match_python_float(L, pad):
    """The fast decimal path (8-digit SWAR + Clinger) returns what strtod returns, at the end of
    a message (per-digit tail) and with 8+ readable bytes after the number (SWAR)."""
    body = []
    for i, s in enumerate(_EDGE_NUMBERS):
        tail = "," + '"x":' + "1" * pad if pad else ""
        body.append('{"features":[' + ",".join([s] * 30) + "]" + tail + "}")
    rc, f, _, _ = _parse(L, body)
    assert rc == len(body)
    for i, s in enumerate(_EDGE_NUMBERS):
        with np.errstate(over="ignore"):
            want = np.float32(float(s))
        assert f[i, 0] == want and f[i, 29] == want, (s, f[i, 0], want)


def test_json_parser_rejects_malformed_numbers(L):
    for bad in ("-", "1e", "1e+", ".", "--1", "1.2.3"):
        rc, _, _, _ = _parse(L, ['{"features":[' + ",".join([bad] * 30) + "]}"])
        assert rc == -1, bad


@pytest.mark.parametrize("field,val", [("id", "-5"), ("id", "1e30"), ("customer_id", "-1"),
                                       ("customer_id", "5000000000"), ("id", "\"-7\"")])
def test_json_ids_out_of_range_are_malformed(L, field, val):
    """negative / oversized ids are rejected instead of an undefined
    float->integer conversion; a bare `true`/`null` at the very end is bounds-checked."""
    feats = ",".join(["0.5"] * 30)
    rc, _, _, _ = _parse(L, ['{"%s": %s, "features": [%s]}' % (field, val, feats)])
    assert rc != 1
    rc, _, ids, _ = _parse(L, ['{"id": 12, "features": [%s], "flag": true}' % feats,
                               '{"id": 13, "features": [%s], "x": null}' % feats])
    assert rc == 2 and ids.tolist() == [12, 13]


def _edge_table(rng, ne_max, g20):
    """A random BinSpec-shaped table: sorted per-feature edges incl. duplicates-free ties with
    the input values, empty features and the format's maximum edge count."""
    edges, offs = [], [0]
    for j in range(30):
        ne = int(rng.integers(0, ne_max + 1)) if j not in (0, 7) else (ne_max if j == 0 else 0)
        e = np.unique(rng.standard_normal(ne).astype(np.float32) * 2)
        edges.append(e)
        offs.append(offs[-1] + len(e))
    flat = np.concatenate(edges).astype(np.float32) if offs[-1] else np.zeros(1, np.float32)
    return np.ascontiguousarray(flat), np.asarray(offs, np.int32)


@pytest.mark.parametrize("g20", [False, True])
def test_simd_encoder_matches_reference(L, g20):
    """The branch-free AVX2 bin encoder (csrc/engine/binenc.h) is bit-exact against the scalar
    binary-search encoder it replaced, for NaN / +-inf / values equal to an edge, every table
    width up to the format's maximum (31 edges G20, 255 G32), and the multi-threaded entry."""
    rng = np.random.default_rng(11 + g20)
    ne_max = 31 if g20 else 255
    rb = 20 if g20 else 32
    for trial in range(6):
        flat, offs = _edge_table(rng, ne_max, g20)
        n = 5000
        X = rng.standard_normal((n, 30)).astype(np.float32) * 2
        # exact ties with edges, specials
        for j in range(30):
            ne = offs[j + 1] - offs[j]
            if ne:
                k = rng.integers(0, n, 200)
                X[k, j] = flat[offs[j] + rng.integers(0, ne, 200)]
        X[rng.integers(0, n, 50), rng.integers(0, 30, 50)] = np.nan
        X[rng.integers(0, n, 50), rng.integers(0, 30, 50)] = np.inf
        X[rng.integers(0, n, 50), rng.integers(0, 30, 50)] = -np.inf
        X[rng.integers(0, n, 20), rng.integers(0, 30, 20)] = -0.0
        stamp = int(rng.integers(1, 63))
        fn, ref = (L.ccfd_encode_g20, L.ccfd_encode_g20_ref) if g20 else (L.ccfd_encode_g32, L.ccfd_encode_g32_ref)
        a = np.zeros((n, rb), np.uint8)
        b = np.zeros((n, rb), np.uint8)
        am = np.zeros(n, np.float32)
        assert fn(X.ctypes.data, n, 30, flat.ctypes.data, offs.ctypes.data, stamp, a.ctypes.data, am.ctypes.data) == n
        assert ref(X.ctypes.data, n, 30, flat.ctypes.data, offs.ctypes.data, stamp, b.ctypes.data, None) == n
        assert (a == b).all(), np.argwhere(a != b)[:5]
        np.testing.assert_array_equal(am, X[:, 29])
        c = np.zeros((n, rb), np.uint8)
        assert L.ccfd_encode_bins_mt(X.ctypes.data, n, 30, flat.ctypes.data, offs.ctypes.data, stamp, int(g20),
                                     c.ctypes.data, None, 3) == n
        assert (c == b).all()


def test_simd_encoder_is_faster(L):
    """Microbench guard: the SIMD encoder beats the scalar binary search it replaced on a
    BASELINE-shaped table (100 x 6 ensemble: ~20 edges a feature); the measured ratio on the
    GPU box's host goes into profiles/r3/encode/ (bench/encode_bench.py)."""
    import time
    rng = np.random.default_rng(3)
    from ccfd_demo_summit_amd.models.gbdt import ObliviousGBDT
    X = rng.standard_normal((200_000, 30)).astype(np.float32)
    spec = ObliviousGBDT.random_init(100, 6, seed=0, X_ref=X[:20000]).bin_spec(bits=5)
    out = np.zeros((len(X), 20), np.uint8)
    flat, offs = spec.flat, spec.offsets
    args = (X.ctypes.data, len(X), 30, flat.ctypes.data, offs.ctypes.data, spec.stamp, out.ctypes.data, None)

    def best(fn):
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            fn(*args)
            ts.append(time.perf_counter() - t0)
        return min(ts)
    t_ref, t_simd = best(L.ccfd_encode_g20_ref), best(L.ccfd_encode_g20)
    assert t_simd * 1.5 < t_ref, (t_simd, t_ref)


def test_host_read_bw_probe(L):
    from ccfd_demo_summit_amd.engine.stream_engine import PinnedArray  # noqa: F401  (GPU-free import)
    buf = np.zeros((64 << 20) // 8 + 8, np.uint64)
    p = buf.ctypes.data
    p = p + (-p) % 32
    gbps = L.ccfd_host_read_bw(C.c_void_p(p), 64 << 20, 2, 0.05)
    assert gbps > 0.5, gbps
    assert L.ccfd_host_read_bw(C.c_void_p(p), 100, 2, 0.01) < 0


def test_corrupt_gzip_batch_stalls_partition(L):
    """a CRC-valid gzip batch that does not inflate must stall the partition (error
    reported, nothing after it consumed) instead of being skipped -- a later batch would move
    the offset past the lost records and they would be committed unread."""
    import struct
    import zlib
    from ccfd_demo_summit_amd.ingest.kafka_wire import CODEC_GZIP, crc32c, encode_record_batch
    from ccfd_demo_summit_amd.ingest.native_consumer import NativeKafkaConsumer
    msgs = [json.dumps({"id": i, **{n: float(i) for n in FEATURE_NAMES}}).encode() for i in range(10)]
    gz = bytearray(encode_record_batch(msgs[:5], compression=CODEC_GZIP, base_offset=0))
    hdr = 12 + 9 + 40          # base/len, epoch/magic/crc, attrs..count
    body = bytearray(gz[hdr:])
    for i in range(12, len(body) - 8):            # wreck the deflate stream, keep the gzip header
        body[i] ^= 0x5A
    after = bytes(gz[21:hdr]) + bytes(body)
    bad = struct.pack(">qi", 0, 9 + len(after)) + struct.pack(">ibI", 0, 2, crc32c(after)) + after
    assert zlib.crc32(bad) != zlib.crc32(bytes(gz))
    good = encode_record_batch(msgs[5:], base_offset=5)
    kc = NativeKafkaConsumer.for_arrays("127.0.0.1:1", "t", {0: 0}, capacity=1000, wire=False)
    try:
        kc.feed(bad + good)
        st = kc.stats()
        assert st["records"] == 0, st                 # the valid batch behind it is NOT consumed
        assert "gzip" in kc.last_error()
        assert kc.committable() == {}
    finally:
        kc.close()


def test_native_crash_report_prints_the_native_stack():
    """A fault in any thread prints the native stack (module + offset per frame) and then
    chains to Python's faulthandler (engine.cpp installs it at ccfd_engine_create)."""
    import pathlib
    import subprocess
    import sys
    code = ("import ctypes, faulthandler, os, signal; faulthandler.enable(); "
            "from ccfd_demo_summit_amd.ops.build import lib_path; L = ctypes.CDLL(str(lib_path(''))); "
            "assert L.ccfd_crash_report_install() == 5; assert L.ccfd_crash_report_install() == 0; "
            "ctypes.string_at(8)")                     # a real SIGSEGV (read of address 8)
    root = pathlib.Path(__file__).resolve().parents[1]
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=str(root))
    assert r.returncode != 0
    assert "[ccfd] native crash: signal 11 at address 0x0000000000000008" in r.stderr, r.stderr[-2000:]
    assert "native stack (module+offset)" in r.stderr and "Fatal Python error" in r.stderr
