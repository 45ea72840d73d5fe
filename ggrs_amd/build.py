"""Build the HIP engine (ggrs_amd/libggrs_amd.so) for gfx950 with hipcc, in-tree.

Flags that matter for parity: -ffp-contract=off (the reference's Rust never fuses a*b+c; the
sincosf restatement places its fmas explicitly), no -ffast-math (keeps correctly rounded f32
division/sqrt and f32 denormals, hipcc's defaults).

Each translation unit compiles to its own object in parallel (ggrs_amd/_obj/), then one link.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "_obj")
LIB = os.path.join(HERE, "libggrs_amd.so")
UNITS = ("engine.hip", "requests.hip", "branch.hip", "particles.hip", "p2p.hip", "p2p_sched.hip", "codec.hip",
         "lane_encode.cpp")
SOURCES = [os.path.join(CSRC, f) for f in UNITS]
HEADERS = [os.path.join(CSRC, h) for h in ("box_game.h", "glibc_sincosf.h", "common.h", "particles.h", "p2p_engine.h",
                                           "engine.h")] + [
    os.path.join(ROOT, "include", "ggrs_amd.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "--offload-arch=gfx950", "-ffp-contract=off", "-fPIC", "-std=c++17",
         "-Wall", "-Wno-unused-function"]
# The step kernels run one wave per SIMD, so a VALU instruction that waits on the previous one's
# result stalls the SIMD; LLVM's max-ilp machine scheduler interleaves the step's independent
# chains (the next sin/cos, the Fletcher sums, the stores) instead of the default
# occupancy-oriented order.  Measured on MI355X (profiles/r03b): the v5 SyncTest launch 0.1951 ->
# 0.1794 ms, the P2P flat kernel 0.1295 -> 0.1209 ms, config 3 2.4 -> 2.3 us per round, config 4
# unchanged; the lane-server unit (requests.hip) was slower with it and keeps the default.  Round 4
# (profiles/r04o, the whole library A/B twice): the default scheduler cost config 2 3 %, the P2P
# kernels 4-6 %, and gained config 3's pipelined prefix kernel (lane-pair trunk split,
# write-through saves) 3 %: 25.8 -> 25.0 us per 16-round step, so branch.hip keeps the default.
# max-ilp on every unit (round 4): codec and the request boundary unchanged; the particle unit's
# checksums changed, which round 5 traced to inline asm (DESIGN.md §3 "No inline asm": LLVM's
# hazard recognizer does not see an asm statement as the reader of a v_dot result, so the 3 wait
# states gfx950 needs were missing).  No unit contains instruction-emitting inline asm any more
# (tests/test_no_inline_asm.py).  Also measured on every unit: max-memory-clause, config 2 and
# the P2P chains 3 % slower, config 3 equal; iterative-ilp crashes this hipcc on particles.hip.
ILP = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
UNIT_FLAGS = {"engine.hip": ILP, "p2p.hip": ILP, "p2p_sched.hip": ILP}


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(f) > t for f in SOURCES + HEADERS + [os.path.abspath(__file__)])


def _compile(src, extra, verbose, obj_dir=OBJ, csrc=CSRC):
    obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
    # an unchanged unit keeps its object (same source, headers, flags and this script)
    if not extra and csrc == CSRC and os.path.exists(obj):
        t = os.path.getmtime(obj)
        if all(os.path.getmtime(f) <= t for f in [src] + HEADERS + [os.path.abspath(__file__)]):
            return obj
    cmd = [HIPCC, *FLAGS, *UNIT_FLAGS.get(os.path.basename(src), []), *extra, "-I", os.path.join(ROOT, "include"), "-I", csrc, "-c", "-o", obj, src]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return obj


def build(force=False, verbose=False, out=LIB, extra=(), csrc=CSRC):
    """Compile every unit for gfx950 and link `out` (default: the product library).  `extra`
    flags and another source directory `csrc` are for experiment builds only
    (tools/exp_build.sh: a scratch copy of csrc/ with tools/exp/*.patch applied), which write
    elsewhere."""
    if csrc != CSRC and out == LIB:
        raise ValueError("an experiment source tree must not overwrite the product library")
    if out == LIB and not extra and not force and not needs_build():
        return LIB
    obj_dir = OBJ if out == LIB else out + ".obj"  # experiment builds keep their own objects
    os.makedirs(obj_dir, exist_ok=True)
    jobs = min(len(SOURCES), max(1, os.cpu_count() or 1), 16)
    srcs = [os.path.join(csrc, f) for f in UNITS]
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, list(extra), verbose, obj_dir, csrc), srcs))
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out + ".tmp", *objs]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


DRIVER_SRC = os.path.join(ROOT, "bench_native", "handler_driver.c")
DRIVER_LIB = os.path.join(ROOT, "bench_native", "libhandler_driver.so")


def build_driver(force=False, verbose=False):
    """bench.py's request-handler driver (bench infrastructure, linked against the engine)."""
    if not force and os.path.exists(DRIVER_LIB) and os.path.getmtime(DRIVER_LIB) >= max(
            os.path.getmtime(DRIVER_SRC), os.path.getmtime(LIB)):
        return DRIVER_LIB
    # -O3 -mavx2: the handler's per-call loops over L lanes (token rows, checksum hand-back) vectorise
    cmd = ["gcc", "-O3", "-mavx2", "-pthread", "-fopenmp", "-shared", "-fPIC", "-I", os.path.join(ROOT, "include"), "-o", DRIVER_LIB + ".tmp",
           DRIVER_SRC, "-L", HERE, "-lggrs_amd", "-Wl,-rpath,$ORIGIN/../ggrs_amd"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(DRIVER_LIB + ".tmp", DRIVER_LIB)
    return DRIVER_LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    build_driver(force="--force" in sys.argv, verbose=True)
    print(LIB)
