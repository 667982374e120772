"""W64 wire rows (64 B: bf16 V1..V28, f32 Time/Amount): NumPy and native encoders agree
bit-for-bit, JSON parses straight into W64, and the wire-order packed blob reproduces the
bf16 oracle through the lane-exact kernel emulator."""
import ctypes as C
import json

import numpy as np
import pytest

from ccfd_demo_summit_amd.contracts import FEATURE_NAMES, WIRE_PERM, decode_wire, encode_wire
from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.models import build_model
from ccfd_demo_summit_amd.models.mlp import emulate_packed_kernel


@pytest.fixture(scope="module")
def L():
    from ccfd_demo_summit_amd.ops._lib import lib
    return lib()


def test_layout_and_roundtrip():
    X, _ = generate(500, seed=9)
    W = encode_wire(X)
    assert W.shape == (500, 64) and W.dtype == np.uint8
    Y = decode_wire(W)
    np.testing.assert_array_equal(Y[:, [0, 29]], X[:, [0, 29]])          # Time / Amount exact
    rel = np.abs(Y[:, 1:29] - X[:, 1:29]) / np.maximum(np.abs(X[:, 1:29]), 1e-30)
    assert rel.max() <= 2 ** -8                                           # bf16 RNE
    assert sorted(WIRE_PERM.tolist()) == list(range(30))
    assert FEATURE_NAMES[WIRE_PERM[28]] == "Time" and FEATURE_NAMES[WIRE_PERM[29]] == "Amount"


def test_native_encoder_bit_exact(L):
    X, _ = generate(1000, seed=2)
    X[0, 3] = np.float32(1.0 + 2 ** -8)          # exact tie -> round to even
    X[1, 4] = -0.0
    X[2, 5] = np.nan
    X[3, 6] = np.float32(np.inf)
    out = np.zeros((1000, 64), np.uint8)
    assert L.ccfd_encode_w64(X.ctypes.data, 1000, 30, out.ctypes.data) == 1000
    np.testing.assert_array_equal(out, encode_wire(X))
    assert np.isnan(decode_wire(out)[2, 5]) and np.isinf(decode_wire(out)[3, 6])


def test_native_json_to_w64(L):
    X, _ = generate(40, seed=5)
    msgs = []
    for i in range(40):
        d = {"id": i + 7, "customer_id": i}
        d.update({n: float(v) for n, v in zip(FEATURE_NAMES, X[i])})
        msgs.append(json.dumps(d).encode())
    buf = b"".join(msgs)
    off = np.cumsum([0] + [len(m) for m in msgs]).astype(np.int64)
    rows = np.zeros((40, 64), np.uint8)
    ids = np.zeros(40, np.uint64)
    cu = np.zeros(40, np.uint32)
    assert L.ccfd_parse_json_batch_w64(buf, off.ctypes.data, 40, rows.ctypes.data, ids.ctypes.data,
                                       cu.ctypes.data) == 40
    # JSON floats round-trip through float64 text -> f32 first, exactly like encode_wire(X)
    np.testing.assert_array_equal(rows, encode_wire(X))
    assert ids.tolist() == list(range(7, 47))


@pytest.mark.parametrize("kind", ["mlp", "lr"])
def test_wire_blob_matches_oracle(kind):
    X, _ = generate(3000, seed=11)
    m = build_model(kind, seed=3, X_ref=X)
    Xw = decode_wire(encode_wire(X[:48]))
    if kind == "mlp":
        got = emulate_packed_kernel(m.pack(wire=True), X[:48])
        np.testing.assert_allclose(got, m.wire_proba(X[:48]), atol=2e-6)
        # folding the V-normalisation into W1 stays within bf16 noise of normalise-then-round
        assert np.abs(got - m.predict_proba(Xw, emulate_bf16=True)).max() < 2e-3
        # and the wire numerics stay within bf16 noise of the f32 model
        assert np.abs(got - m.predict_proba(X[:48])).max() < 5e-3
    blob = np.frombuffer(m.pack(wire=True), np.uint8)
    assert int(np.frombuffer(blob[4:8].tobytes(), np.uint32)[0]) & 2


# ---------------------------------------------------------------------------------------
# G32 rows (GBDT): bins against the ensemble's split table are exact for every float
def _g32_case(seed=0, n=20000):
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.models.gbdt import ObliviousGBDT
    X, _ = generate(n, seed=seed)
    m = ObliviousGBDT.random_init(100, 6, seed=seed, X_ref=X)
    m.thr[3, 2] = np.nan                      # a split that never fires
    X[5, 3] = np.nan
    X[6, 29] = np.nan
    X[7, 2] = np.inf
    X[8, 2] = -np.inf
    X[9, :] = m.thr[0, 0]                     # values equal to thresholds
    X[10, :] = -0.0
    return X, m


def test_g32_bins_reproduce_every_split_decision():
    X, m = _g32_case()
    spec = m.bin_spec()
    k = spec.bin_index(m.feat, m.thr)
    rows = spec.encode(X)
    np.testing.assert_array_equal(rows[:, m.feat].astype(np.int32) > k[None], X[:, m.feat] > m.thr[None])
    assert (rows[:, 31] == spec.stamp).all() and 1 <= spec.stamp <= 255


def test_g32_native_encoder_matches_numpy_oracle():
    from ccfd_demo_summit_amd.engine.stream_engine import G32_ROW_F32, encode_g32
    X, m = _g32_case(seed=1)
    spec = m.bin_spec()
    out = np.empty((X.shape[0], G32_ROW_F32), np.float32)
    am = np.empty(X.shape[0], np.float32)
    encode_g32(X, spec, out.ctypes.data, am.ctypes.data)
    np.testing.assert_array_equal(out.view(np.uint8), spec.encode(X))
    np.testing.assert_array_equal(am, X[:, 29])
    from ccfd_demo_summit_amd.contracts.metric_names import AMOUNT_BUCKETS
    b = np.searchsorted(np.asarray(AMOUNT_BUCKETS, np.float32), X[:, 29], side="left")
    b[np.isnan(X[:, 29])] = 0
    np.testing.assert_array_equal(out.view(np.uint8)[:, 30], b)


def test_g32_blob_and_spec_roundtrip():
    import struct
    from ccfd_demo_summit_amd.models.gbdt import BinSpec, ObliviousGBDT
    X, m = _g32_case(seed=2)
    spec = m.bin_spec()
    s2 = BinSpec.from_bytes(spec.to_bytes())
    assert s2.stamp == spec.stamp and all(np.array_equal(a, b) for a, b in zip(s2.edges, spec.edges))
    blob = m.pack(bins=spec)
    assert blob[:4] == b"GBB1" and struct.unpack_from("<i", blob, 20)[0] == spec.stamp
    off_f, off_k, off_l, end = ObliviousGBDT.blob_offsets(m.n_trees, m.depth)
    k = np.frombuffer(blob, np.int32, m.feat.size, off_k).reshape(m.feat.shape)
    assert k[3, 2] == 255                       # NaN split: no u8 bin exceeds it
    # a superset table accepts the model; a table missing one of its thresholds refuses it
    wide = BinSpec([np.union1d(e, np.float32([1e9])) for e in spec.edges])
    assert wide.contains(spec) and wide.stamp != spec.stamp
    m.pack(bins=wide)
    narrow = BinSpec([e[1:] if j == int(m.feat[0, 0]) else e for j, e in enumerate(spec.edges)])
    with pytest.raises(ValueError, match="not a bin edge"):
        m.pack(bins=narrow)
    with pytest.raises(ValueError):
        BinSpec([np.arange(300, dtype=np.float32)] + [np.zeros(0, np.float32)] * 29)


# ---------------------------------------------------------------------------------------
# G20 rows: the same bins packed 5 bits each (<= 31 edges a feature), equally exact
def _g20_case(seed=0, n=20000):
    X, m = _g32_case(seed=seed, n=n)
    keep = m.bin_spec()
    if not keep.fits_g20:                     # a 100 x 6 draw can exceed 31 on one feature
        m = type(m)(m.feat[:60], m.thr[:60], m.leaves[:60], m.base)
    return X, m


def test_g20_bins_reproduce_every_split_decision():
    from ccfd_demo_summit_amd.contracts import decode_g20_bins
    X, m = _g20_case()
    spec = m.bin_spec(bits=5)
    assert spec.row_format == "g20" and 1 <= spec.stamp <= 63
    rows = spec.encode(X)
    assert rows.shape == (X.shape[0], 20)
    g = decode_g20_bins(rows)
    g32 = m.bin_spec().encode(X)
    np.testing.assert_array_equal(g[:, :31], g32[:, :31])       # bins + amount bucket
    assert (g[:, 31] == spec.stamp).all()
    np.testing.assert_array_equal(m.leaf_index_g32(rows, spec), m.leaf_index(X))


def test_g20_native_encoder_matches_numpy_oracle():
    from ccfd_demo_summit_amd.engine.stream_engine import G20_ROW_F32, encode_g32
    X, m = _g20_case(seed=1)
    spec = m.bin_spec(bits=5)
    out = np.empty((X.shape[0], G20_ROW_F32), np.float32)
    am = np.empty(X.shape[0], np.float32)
    encode_g32(X, spec, out.ctypes.data, am.ctypes.data)
    np.testing.assert_array_equal(out.view(np.uint8), spec.encode(X))
    np.testing.assert_array_equal(am, X[:, 29])


def test_g20_spec_limits_and_roundtrip():
    from ccfd_demo_summit_amd.models.gbdt import BinSpec
    X, m = _g20_case(seed=2)
    spec = m.bin_spec(bits=5)
    s2 = BinSpec.from_bytes(spec.to_bytes(), bits=5)
    assert s2.stamp == spec.stamp and s2.row_format == "g20"
    edges = [np.arange(32, dtype=np.float32)] + [np.zeros(0, np.float32)] * 29
    with pytest.raises(ValueError, match="5 bits"):
        BinSpec(edges, bits=5)
    assert not BinSpec(edges).fits_g20
    from ccfd_demo_summit_amd.ops._lib import lib
    import ctypes as C
    flat, off = BinSpec(edges).flat, BinSpec(edges).offsets
    out = np.zeros((4, 20), np.uint8)
    # the native encoder refuses a table a 5-bit field cannot index, and stamps past 63
    assert lib().ccfd_encode_g20(X.ctypes.data, 4, 30, flat.ctypes.data, off.ctypes.data, 5,
                                 C.c_void_p(out.ctypes.data), None) == -1
    f2, o2 = spec.flat, spec.offsets
    assert lib().ccfd_encode_g20(X.ctypes.data, 4, 30, f2.ctypes.data, o2.ctypes.data, 64,
                                 C.c_void_p(out.ctypes.data), None) == -1
