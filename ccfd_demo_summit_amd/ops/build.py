"""Build the native library ``libccfd_hip.so`` in-tree with hipcc for gfx950.

    python -m ccfd_demo_summit_amd.ops.build [--force] [--jobs N]

Every ``csrc/kernels/*.hip`` (device code, MFMA kernels) and ``csrc/engine/*.cpp``
(host runtime: streaming engine, ingest parser) is compiled to an object under
``build/obj`` and linked into ``ccfd_demo_summit_amd/_native/libccfd_hip.so``.  The .so
is git-ignored but travels to the GPU box with the gpurun snapshot.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
CSRC = ROOT / "csrc"
OBJ = ROOT / "build" / "obj"
NATIVE = Path(__file__).resolve().parents[1] / "_native"
LIB = NATIVE / "libccfd_hip.so"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
# Host-code sanitizer build: CCFD_SANITIZE=address|undefined|address,undefined
# instruments the host runtime (csrc/engine/*.cpp) -- never device code -- and links
# libccfd_hip_<san>.so next to the normal library; load it with the clang runtime preloaded
# (tests/test_native_cpu.py::test_host_runtime_under_asan).
SANITIZE = os.environ.get("CCFD_SANITIZE", "")


# Host-only codecs (CRC-32C, Kafka RecordBatch framing, JSON transaction parsing, row
# encoders) and the KIE tier's start-dedupe index ALSO go into a small library with no HIP dependency: the broker, KIE, notifier
# and producer processes load only this one, so they never bring up the GPU runtime (CPU-only
# pods in the operator's deployment; ~0.3 s with the GIL held in a service that loaded the
# engine library lazily, profiles/r4/kie_handoff/).
HOST_LIB = NATIVE / "libccfd_host.so"
HOST_SOURCES = ("crc32c.cpp", "kafka_codec.cpp", "ingest.cpp", "dedupe.cpp")


def host_sources():
    return [CSRC / "engine" / n for n in HOST_SOURCES]


def build_host(force: bool = False, verbose: bool = True) -> Path:
    """g++ -> libccfd_host.so (plain C++, no offload, no libamdhip64)."""
    OBJ.mkdir(parents=True, exist_ok=True)
    NATIVE.mkdir(parents=True, exist_ok=True)
    cxx = os.environ.get("CXX") or shutil.which("g++") or shutil.which("c++")
    if not cxx:
        raise RuntimeError("no host C++ compiler for libccfd_host.so")
    newest = max([s.stat().st_mtime for s in host_sources()] + [_headers_mtime()])
    if force or not HOST_LIB.exists() or HOST_LIB.stat().st_mtime < newest:
        tmp = HOST_LIB.with_suffix(".so.tmp")
        cmd = [cxx, "-O3", "-fPIC", "-shared", "-std=c++17", "-Wall", "-I", str(CSRC / "include"),
               "-o", str(tmp)] + [str(s) for s in host_sources()] + ["-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"host lib build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, HOST_LIB)
    if verbose:
        print(f"[ccfd build] {HOST_LIB} ({len(HOST_SOURCES)} host sources)")
    return HOST_LIB


def lib_path(sanitize: str = SANITIZE) -> Path:
    return LIB if not sanitize else NATIVE / f"libccfd_hip_{sanitize.replace(',', '_')}.so"


def asan_runtime() -> str:
    out = subprocess.run([str(Path(hipcc()).parent.parent / "lib/llvm/bin/clang"), "-print-file-name=libclang_rt.asan-x86_64.so"],
                         capture_output=True, text=True).stdout.strip()
    return out


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libccfd_hip.so)")


def sources():
    return sorted(CSRC.glob("kernels/*.hip")) + sorted(CSRC.glob("engine/*.cpp"))


def _headers_mtime() -> float:
    hs = list(CSRC.glob("**/*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _compile(src: Path, force: bool, sanitize: str = "") -> Path:
    tag = "" if not sanitize or src.suffix != ".cpp" else "_" + sanitize.replace(",", "_")
    obj = OBJ / (src.parent.name + "_" + src.stem + tag + ".o")
    if not force and obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, _headers_mtime()):
        return obj
    cmd = [hipcc(), "-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall",
           "-Wno-unused-result", "-I", str(CSRC / "include"), "-c", str(src), "-o", str(obj)]
    if src.suffix == ".cpp":
        # host-only translation units: no device code object
        cmd = [hipcc(), "-O1" if sanitize else "-O3", "-fPIC", "-std=c++17", "-Wall",
               "-I", str(CSRC / "include"), "-c", str(src), "-o", str(obj)]
        if sanitize:
            cmd[1:1] = [f"-fsanitize={sanitize}", "-fno-omit-frame-pointer", "-g"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int = 4, verbose: bool = True, sanitize: str = SANITIZE) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    NATIVE.mkdir(parents=True, exist_ok=True)
    srcs = sources()
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, sanitize), srcs))
    newest = max(o.stat().st_mtime for o in objs)
    LIB = lib_path(sanitize)
    if force or not LIB.exists() or LIB.stat().st_mtime < newest:
        tmp = LIB.with_suffix(".so.tmp")
        cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(tmp)] + \
              [str(o) for o in objs] + ["-lpthread", "-lz"] + ([f"-fsanitize={sanitize}", "-shared-libsan"] if sanitize else [])
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
    if verbose:
        print(f"[ccfd build] {LIB} ({len(srcs)} sources, arch {ARCH})")
    if not sanitize:
        build_host(force=force, verbose=verbose)
    return LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=4)
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs)


if __name__ == "__main__":
    sys.exit(main())
