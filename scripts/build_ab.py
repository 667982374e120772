"""Build an A/B variant of the native library: the regular objects, with chosen kernel
sources recompiled under extra -D flags, linked into ccfd_demo_summit_amd/_native/ab/<name>.so.
Load it with CCFD_LIB_PATH=<that path> (ops/_lib.py).  Compile-time variants keep the
default kernels free of runtime A/B branches (a runtime branch measurably slowed the
default path, profiles/r3/load_width/README.md).

    python scripts/build_ab.py --name tb8 --src kernels/score_gbdt_g32_persist.hip -D CCFD_G32_TREE_BLOCK=8

(The round-3 fetch-width variants measured with it -- W64 8- / 4-byte lanes, G20 16-byte
lanes -- were removed from the sources after they lost; evidence: profiles/r3/load_width/,
docs/ROUND3.md.)
"""
import argparse
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--name", required=True)
    ap.add_argument("--src", action="append", required=True, help="csrc-relative source(s) to recompile")
    ap.add_argument("-D", dest="defs", action="append", default=[])
    ap.add_argument("--from-rev", default=None,
                    help="compile the --src files as they were at this git revision (a variant "
                         "removed from the tree after it lost), against today's headers")
    args = ap.parse_args()
    from ccfd_demo_summit_amd.ops import build as B
    B.build(verbose=False)                       # regular objects up to date
    out_dir = ROOT / "ccfd_demo_summit_amd" / "_native" / "ab"
    out_dir.mkdir(parents=True, exist_ok=True)
    objs = {s: B.OBJ / (s.parent.name + "_" + s.stem + ".o") for s in B.sources()}
    for rel in args.src:
        src = B.CSRC / rel
        obj = B.OBJ / f"ab_{args.name}_{src.parent.name}_{src.stem}.o"
        comp = src
        if args.from_rev:
            comp = B.OBJ / f"ab_{args.name}_{src.stem}{src.suffix}"
            text = subprocess.run(["git", "-C", str(ROOT), "show", f"{args.from_rev}:csrc/{rel}"],
                                  check=True, capture_output=True, text=True).stdout
            comp.write_text(text)
        cmd = [B.hipcc(), "-O3", "-fPIC", "-std=c++17", f"--offload-arch={B.ARCH}", "-Wall", "-Wno-unused-result",
               "-I", str(B.CSRC / "include"), "-I", str(src.parent)] + [f"-D{d}" for d in args.defs] + \
              ["-c", str(comp), "-o", str(obj)]
        subprocess.run(cmd, check=True)
        objs[src] = obj
    lib = out_dir / f"{args.name}.so"
    cmd = [B.hipcc(), "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o", str(lib)] + \
          [str(o) for o in objs.values()] + ["-lpthread", "-lz"]
    subprocess.run(cmd, check=True)
    print(lib)


if __name__ == "__main__":
    main()
