"""ctypes binding of ``libccfd_hip.so`` (C ABI in csrc/include/ccfd_abi.h).

``torch`` must be imported BEFORE the library is loaded: torch's bundled
``libamdhip64.so`` carries the same soname (``libamdhip64.so.7``), so the dynamic
linker resolves our NEEDED entry to the runtime torch already loaded and both share one
HIP runtime (one context, interchangeable device pointers and streams).
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

import torch  # noqa: F401  (must precede the dlopen, see module doc)

_NATIVE = Path(__file__).resolve().parents[1] / "_native"
# CCFD_SANITIZE=<san>: load the host-sanitizer build (ops/build.py) instead
_SAN = os.environ.get("CCFD_SANITIZE", "")
LIB_PATH = _NATIVE / (f"libccfd_hip_{_SAN.replace(',', '_')}.so" if _SAN else "libccfd_hip.so")
# CCFD_LIB_PATH=<path>: load an A/B build (scripts/build_ab.py) instead
if os.environ.get("CCFD_LIB_PATH"):
    LIB_PATH = Path(os.environ["CCFD_LIB_PATH"]).resolve()

MODEL_LR, MODEL_MLP, MODEL_GBDT = 0, 1, 2
MODEL_IDS = {"lr": MODEL_LR, "mlp": MODEL_MLP, "gbdt": MODEL_GBDT}
N_COUNTER_SLOTS = 64
ENGINE_FLAG_FULL = 1      # ccfd_abi.h CCFD_ENGINE_FLAG_FULL: drain the flagged ring, call again
CNT_WIRE_STALE = 4        # ccfd_abi.h CCFD_CNT_WIRE_STALE
ARG_WIRE_W64, ARG_WIRE_G32, ARG_WIRE_G20 = 2, 4, 8
ROW_FORMATS = {"f32": 0, "w64": 1, "g32": 2, "g20": 3}      # ccfd_engine_config.wire
BIN_FORMATS = ("g32", "g20")                                # rows of per-feature bins (GBDT)


class ScoreArgs(C.Structure):
    _fields_ = [("x", C.c_void_p), ("ld", C.c_int64), ("n", C.c_int32), ("model", C.c_int32),
                ("blob", C.c_void_p), ("threshold", C.c_float), ("gbdt_trees", C.c_int32),
                ("gbdt_depth", C.c_int32), ("flags", C.c_int32), ("proba", C.c_void_p),
                ("route", C.c_void_p), ("counters", C.c_void_p), ("slot_ctl", C.c_void_p),
                ("flag_idx", C.c_void_p), ("done_rec", C.c_void_p), ("done_seq", C.c_uint64),
                ("rules", C.c_void_p)]


class EngineConfig(C.Structure):
    _fields_ = [("device", C.c_int32), ("model", C.c_int32), ("blob", C.c_void_p),
                ("gbdt_trees", C.c_int32), ("gbdt_depth", C.c_int32), ("threshold", C.c_float),
                ("max_batch", C.c_int32), ("depth", C.c_int32), ("n_streams", C.c_int32),
                ("input_mode", C.c_int32), ("output_mode", C.c_int32), ("flag_capacity", C.c_int32),
                ("exec_mode", C.c_int32), ("persist_grid", C.c_int32), ("wire", C.c_int32),
                ("coalesce", C.c_int32), ("persist_items", C.c_int32), ("counters", C.c_void_p * 2),
                ("rules", C.c_void_p)]


class Flagged(C.Structure):
    _fields_ = [("tx_id", C.c_uint64), ("customer", C.c_uint32), ("proba", C.c_float),
                ("amount", C.c_float), ("partition", C.c_uint32)]


class EngineStats(C.Structure):
    _fields_ = [("batches", C.c_uint64), ("rows", C.c_uint64), ("fraud_rows", C.c_uint64),
                ("flagged_dropped", C.c_uint64), ("wall_s", C.c_double), ("lat_p50_us", C.c_double),
                ("lat_p99_us", C.c_double), ("lat_max_us", C.c_double), ("lat_mean_us", C.c_double),
                ("lat_hist", C.c_uint64 * 256), ("host_submit_ns", C.c_uint64), ("host_wait_ns", C.c_uint64),
                ("host_complete_ns", C.c_uint64), ("dev_batches", C.c_uint64), ("dev_exec_ns", C.c_uint64),
                ("dev_hist", C.c_uint64 * 256), ("lat_hist_rows", C.c_uint64 * 256),
                ("dev_hist_rows", C.c_uint64 * 256), ("last_seq", C.c_uint64), ("last_tx_id", C.c_uint64),
                ("last_proba", C.c_float), ("last_amount", C.c_float), ("last_partition", C.c_int32),
                ("last_row_bytes", C.c_int32), ("last_row", C.c_uint8 * 128),
                ("origin_batches", C.c_uint64), ("origin_hist", C.c_uint64 * 256),
                ("origin_hist_rows", C.c_uint64 * 256), ("submitted", C.c_uint64),
                ("flag_full_events", C.c_uint64)]


FLAGGED_DTYPE = [("tx_id", "<u8"), ("customer", "<u4"), ("proba", "<f4"), ("amount", "<f4"),
                 ("partition", "<u4")]

# ccfd_scored (ccfd_abi.h): one record per scored row (opt-in scored ring)
SCORED_DTYPE = [("tx_id", "<u8"), ("customer", "<u4"), ("proba", "<f4"), ("amount", "<f4"),
                ("partition", "<u2"), ("route", "u1"), ("pad", "u1")]

# ccfd_batch_trace (ccfd_abi.h): per-micro-batch stage timestamps
BATCH_TRACE_DTYPE = [("seq", "<i8"), ("partition", "<i4"), ("rows", "<i4"), ("t_arrival", "<i8"),
                     ("t_submit", "<i8"), ("t_landed", "<i8"), ("t_complete", "<i8"), ("dev_start", "<i8"),
                     ("dev_end", "<i8"), ("flagged", "<i4"), ("pad", "<i4")]

_lib = None
_lock = threading.Lock()


class NativeUnavailable(RuntimeError):
    pass


def lib() -> C.CDLL:
    """Load (building first if needed and a toolchain exists) the native library."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not LIB_PATH.exists():
            if os.environ.get("CCFD_NO_AUTOBUILD"):
                raise NativeUnavailable(f"{LIB_PATH} missing (run python -m ccfd_demo_summit_amd.ops.build)")
            from .build import build
            build(verbose=False)
        L = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
        L.ccfd_score_launch.argtypes = [C.POINTER(ScoreArgs), C.c_void_p]
        L.ccfd_score_launch.restype = C.c_int
        L.ccfd_last_error.restype = C.c_char_p
        L.ccfd_host_alloc.argtypes = [C.c_size_t]
        L.ccfd_host_alloc.restype = C.c_void_p
        L.ccfd_host_free.argtypes = [C.c_void_p]
        L.ccfd_host_device_ptr.argtypes = [C.c_void_p]
        L.ccfd_host_device_ptr.restype = C.c_void_p
        L.ccfd_engine_create.argtypes = [C.POINTER(EngineConfig)]
        L.ccfd_engine_create.restype = C.c_void_p
        L.ccfd_engine_destroy.argtypes = [C.c_void_p]
        L.ccfd_engine_set_log.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_int64, C.c_int64]
        L.ccfd_engine_pump.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.POINTER(EngineStats)]
        L.ccfd_engine_score_sync.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
        L.ccfd_engine_flip_epoch.argtypes = [C.c_void_p, C.c_void_p]
        L.ccfd_engine_epoch_complete.argtypes = [C.c_void_p, C.c_int64]
        L.ccfd_engine_set_blob.argtypes = [C.c_void_p, C.c_void_p]
        L.ccfd_engine_drain_flagged.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.ccfd_engine_drain_flagged.restype = C.c_int64
        L.ccfd_engine_scored_enable.argtypes = [C.c_void_p, C.c_int64]
        L.ccfd_engine_drain_scored.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.ccfd_engine_drain_scored.restype = C.c_int64
        L.ccfd_engine_scored_dropped.argtypes = [C.c_void_p]
        L.ccfd_engine_scored_dropped.restype = C.c_int64
        L.ccfd_engine_serve_start.argtypes = [C.c_void_p, C.c_int64, C.c_int64]
        L.ccfd_engine_serve_stop.argtypes = [C.c_void_p]
        L.ccfd_engine_serve_hold.argtypes = [C.c_void_p, C.c_int]
        L.ccfd_engine_serve_stats.argtypes = [C.c_void_p, C.POINTER(EngineStats), C.POINTER(C.c_int64)]
        L.ccfd_engine_serve_collect.argtypes = [C.c_void_p, C.POINTER(EngineStats), C.c_void_p, C.c_int64,
                                                C.POINTER(C.c_int64), C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
        L.ccfd_engine_cursor.argtypes = [C.c_void_p, C.c_int]
        L.ccfd_engine_cursor.restype = C.c_int64
        L.ccfd_engine_reset_stats.argtypes = [C.c_void_p]
        L.ccfd_engine_progress.argtypes = [C.c_void_p, C.c_void_p]
        L.ccfd_engine_emergency_stop.argtypes = [C.c_void_p, C.c_int]
        L.ccfd_engine_trace_enable.argtypes = [C.c_void_p, C.c_int32]
        L.ccfd_engine_trace_read.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        L.ccfd_engine_set_ring.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]
        L.ccfd_engine_ring_acquire.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.POINTER(C.c_int64)]
        L.ccfd_engine_ring_acquire.restype = C.c_int64
        L.ccfd_engine_ring_commit.argtypes = [C.c_void_p, C.c_int, C.c_int64]
        L.ccfd_engine_ring_commit_at.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_int64]
        L.ccfd_engine_run.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.POINTER(EngineStats)]
        L.ccfd_crc32c.argtypes = [C.c_char_p, C.c_size_t, C.c_uint32]
        L.ccfd_crc32c.restype = C.c_uint32
        L.ccfd_parse_json_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                            C.c_void_p]
        L.ccfd_parse_json_batch.restype = C.c_int64
        L.ccfd_parse_json_batch_w64.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                                C.c_void_p]
        L.ccfd_parse_json_batch_w64.restype = C.c_int64
        L.ccfd_encode_w64.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p]
        L.ccfd_encode_w64.restype = C.c_int64
        L.ccfd_encode_g32.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_int32,
                                      C.c_void_p, C.c_void_p]
        L.ccfd_encode_g32.restype = C.c_int64
        L.ccfd_encode_g20.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_int32,
                                      C.c_void_p, C.c_void_p]
        L.ccfd_encode_g20.restype = C.c_int64
        for name in ("ccfd_encode_g32_ref", "ccfd_encode_g20_ref"):       # scalar oracles
            fn = getattr(L, name)
            fn.argtypes = L.ccfd_encode_g32.argtypes
            fn.restype = C.c_int64
        L.ccfd_encode_bins_mt.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_int32,
                                          C.c_int32, C.c_void_p, C.c_void_p, C.c_int32]
        L.ccfd_encode_bins_mt.restype = C.c_int64
        L.ccfd_encode_isa.argtypes = [C.c_int32]
        L.ccfd_encode_isa.restype = C.c_int32
        L.ccfd_host_read_bw.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_double]
        L.ccfd_host_read_bw.restype = C.c_double
        L.ccfd_engine_set_amount.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        _lib = L
        return L


def last_error() -> str:
    return lib().ccfd_last_error().decode(errors="replace")


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed (rc={rc}): {last_error()}")
