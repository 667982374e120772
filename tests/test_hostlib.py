"""The host-only codec library (ops/_hostlib.py): the services that need only CRC-32C, the
Kafka RecordBatch codecs and JSON transaction parsing (kafka-lite, KIE, notifier, producers)
never load the engine library, so they never bring up the HIP runtime or open the GPU."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

CODE = r"""
import sys
from ccfd_demo_summit_amd.ingest.kafka_wire import warm_native, crc32c, encode_record_batch, decode_record_batches
from ccfd_demo_summit_amd.ingest.codec import parse_json_batch
warm_native()
assert crc32c(b"123456789") == 0xE3069283                   # CRC-32C check value
rs = encode_record_batch([b'{"id": %d, "V1": 0.5, "Amount": 2.25}' % i for i in range(16)])
recs = decode_record_batches(bytes(rs), "t", 0, verify_crc=True)
X, ids, cust = parse_json_batch([r.value for r in recs])
assert list(ids) == list(range(16)) and X[3, 1] == 0.5 and X[3, 29] == 2.25
maps = open("/proc/self/maps").read()
print("engine_lib", "ccfd_demo_summit_amd.ops._lib" in sys.modules, "torch" in sys.modules,
      "hip", "libamdhip64" in maps, "host", "libccfd_host" in maps)
"""


def test_codecs_run_without_the_engine_library():
    out = subprocess.run([sys.executable, "-c", CODE], cwd=str(ROOT), capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "engine_lib False False hip False host True" in out.stdout, out.stdout


def test_crc32c_three_way_matches_reference_at_chunk_edges():
    """The native CRC-32C runs three interleaved chains over 12 KB chunks and joins them with
    shift tables: bit-identical to the byte-wise reference at every chunk edge and seed."""
    import os
    import random

    from ccfd_demo_summit_amd.ingest.kafka_wire import _codec_lib, _crc32c_py
    L = _codec_lib()
    rng = random.Random(7)
    for n in (0, 1, 8, 12287, 12288, 12289, 24576, 36871, 65536 + 3):
        b = os.urandom(n)
        seed = rng.randrange(1 << 32)
        ref = _crc32c_py(b, seed) if seed else _crc32c_py(b)
        assert L.ccfd_crc32c(b, n, seed) == ref, (n, seed)
