"""Zero-copy roofline probes (csrc/kernels/probe.hip): the load-width probe behind the bench's
H2D ceiling (bench.py _h2d_probe) returns a plausible PCIe rate for every lane width and
refuses bad arguments."""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_bw_probe_width_all_widths_and_bad_args():
    from ccfd_demo_summit_amd.engine import PinnedArray
    from ccfd_demo_summit_amd.ops._lib import lib
    L = lib()
    L.ccfd_bw_probe_width.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_void_p]
    L.ccfd_bw_probe_width.restype = C.c_double
    nbytes = 32 << 20
    host = PinnedArray(nbytes // 4, "float32")
    host.array[:] = 1.0
    scratch = torch.empty(1 << 16, dtype=torch.uint8, device="cuda")
    try:
        for w in (4, 8, 16):
            gbps = L.ccfd_bw_probe_width(C.c_void_p(host.ptr), nbytes, w, 512, 2, C.c_void_p(scratch.data_ptr()))
            assert 1.0 < gbps < 200.0, (w, gbps)          # PCIe Gen5 x16 is ~64 GB/s
        assert L.ccfd_bw_probe_width(C.c_void_p(host.ptr), nbytes, 12, 512, 1, C.c_void_p(scratch.data_ptr())) == -1.0
        assert L.ccfd_bw_probe_width(None, nbytes, 4, 512, 1, C.c_void_p(scratch.data_ptr())) == -1.0
    finally:
        host.free()


def test_bench_h2d_probe_takes_the_better_width():
    import bench
    from ccfd_demo_summit_amd.ops._lib import lib
    gbps = bench._h2d_probe(lib, 20.0, mb=32)
    assert 1.0 < gbps < 200.0
