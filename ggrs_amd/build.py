"""Build the HIP engine (ggrs_amd/libggrs_amd.so) for gfx950 with hipcc, in-tree.

Flags that matter for parity: -ffp-contract=off (the reference's Rust never fuses a*b+c; the
sincosf restatement places its fmas explicitly), no -ffast-math (keeps correctly rounded f32
division/sqrt and f32 denormals, hipcc's defaults).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libggrs_amd.so")
SOURCES = [os.path.join(CSRC, f) for f in ("engine.hip", "branch.hip", "particles.hip", "p2p.hip", "codec.hip")]
HEADERS = [os.path.join(CSRC, h) for h in ("box_game.h", "glibc_sincosf.h", "common.h", "particles.h")] + [
    os.path.join(ROOT, "include", "ggrs_amd.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "--offload-arch=gfx950", "-ffp-contract=off", "-fPIC", "-shared", "-std=c++17",
         "-Wall", "-Wno-unused-function"]


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(f) > t for f in SOURCES + HEADERS)


def build(force=False, verbose=False):
    if not force and not needs_build():
        return LIB
    cmd = [HIPCC, *FLAGS, "-I", os.path.join(ROOT, "include"), "-I", CSRC, "-o", LIB + ".tmp",
           *SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB)
