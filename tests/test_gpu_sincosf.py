"""GPU KATs of the product step arithmetic.  The sinf/cosf restatement: the order-independent
digest of every f32 in [0, 2*pi] (each reachable ship rotation is in there, SURVEY.md finding 3)
must equal the digest of glibc libm's values pinned in tests/golden/golden.json, both the separate
and the fused form.  The v4 step (advance_player_lean): its clamp square root on every f32 above
49, and the whole player step against the v3 step on random states."""
import ctypes
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))


@pytest.fixture(scope="module")
def katlib(tmp_path_factory):
    so = os.path.join(HERE, "native", "libsincosf_kat_device.so")
    src = os.path.join(HERE, "native", "sincosf_kat_device.hip")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-ffp-contract=off",
                        "-fPIC", "-shared", "-std=c++17", "-I", os.path.join(ROOT, "ggrs_amd", "csrc"),
                        src, "-o", so], check=True)
    L = ctypes.CDLL(so)
    L.kat_digest.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
    L.kat_values.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.kat_sqrt49.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    L.kat_lean_step.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
    L.kat_clamp_div.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
    return L


@pytest.mark.parametrize("fused", [0, 1])
def test_device_digest_0_2pi(katlib, fused):
    g = GOLDEN["sincos_digest_0_2pi"]
    out = ctypes.c_uint64()
    assert katlib.kat_digest(g["lo"], g["hi"], fused, ctypes.byref(out)) == 0
    assert out.value == g["digest"]


def test_device_values(katlib):
    xs = np.array([s["x"] for s in GOLDEN["sincos"]], np.uint32)
    sv, cv = np.zeros_like(xs), np.zeros_like(xs)
    assert katlib.kat_values(ctypes.c_void_p(xs.ctypes.data), xs.size, ctypes.c_void_p(sv.ctypes.data),
                             ctypes.c_void_p(cv.ctypes.data)) == 0
    for i, s in enumerate(GOLDEN["sincos"]):
        if s["x"] in (0x7F800000,):
            continue
        assert (int(sv[i]), int(cv[i])) == (s["sin"], s["cos"]), hex(s["x"])


def test_clamp_sqrt_every_f32_above_49(katlib):
    """The v4 step's square root (taken only when s > 49) equals hipcc's correctly rounded sqrtf
    bit for bit on every f32 in (49, +inf]."""
    bad = ctypes.c_uint64()
    assert katlib.kat_sqrt49(ctypes.byref(bad)) == 0
    assert bad.value == 0


def test_lean_step_equals_domain_step(katlib):
    """advance_player_lean (v4) and advance_player_rec over make_input_rec (the v5 kernel's staged
    input records) == advance_player_domain (v3) bitwise on 2^25 random player states x 16 inputs
    (edges, zero, -0 and subnormal velocities included)."""
    bad = ctypes.c_uint64()
    assert katlib.kat_lean_step(0x6767, 64, ctypes.byref(bad)) == 0
    assert bad.value & 0xfffff == 0, "lean step differs"
    assert bad.value >> 20 == 0, "record step differs"


def test_clamp_division_through_f64_reciprocal(katlib):
    """RN32(a * refined 1/m in binary64) == a / m (correctly rounded) for every f32 divisor m in
    (7, 16] x 1024 random numerators of every exponent below 2^8 (~9.4e9 divisions)."""
    bad = ctypes.c_uint64()
    assert katlib.kat_clamp_div(0x6767, 1024, ctypes.byref(bad)) == 0
    assert bad.value == 0
