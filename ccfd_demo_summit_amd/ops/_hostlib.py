"""The host-only codec library ``libccfd_host.so`` (ops/build.py ``build_host``): CRC-32C,
Kafka RecordBatch framing, JSON transaction parsing and the W64 / G32 / G20 row encoders,
built with the host C++ compiler and linked against nothing from ROCm.  Services that need
only these (kafka-lite, KIE, notifier, producers) load it instead of the engine library, so
they never initialise the HIP runtime or open the GPU."""
from __future__ import annotations

import ctypes as C
import threading
from typing import Optional

from .build import HOST_LIB

_lib: Optional[C.CDLL] = None
_lock = threading.Lock()


def hostlib() -> C.CDLL:
    """Load (building it first when missing and a compiler exists) the host codec library."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not HOST_LIB.exists():
                from .build import build_host
                build_host(verbose=False)
            L = C.CDLL(str(HOST_LIB))
            L.ccfd_crc32c.argtypes = [C.c_char_p, C.c_size_t, C.c_uint32]
            L.ccfd_crc32c.restype = C.c_uint32
            L.ccfd_parse_json_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                                C.c_void_p]
            L.ccfd_parse_json_batch.restype = C.c_int64
            _lib = L
    return _lib
