"""CPU KAT of the product's glibc sinf/cosf restatement (ggrs_amd/csrc/glibc_sincosf.h), compiled
for the host by hipcc, against this image's libm on every f32 (2^32 inputs, ~15 s on 8 cores),
plus the libm digest over [0, 2*pi] pinned in tests/golden/golden.json."""
import json
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))


@pytest.fixture(scope="module")
def kat_binary(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("kat") / "sincosf_kat_host")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-ffp-contract=off", "-std=c++17",
                    "-I", os.path.join(ROOT, "ggrs_amd", "csrc"),
                    os.path.join(HERE, "native", "sincosf_kat_host.cpp"), "-o", out, "-lpthread"],
                   check=True)
    return out


def test_port_matches_libm_on_0_2pi(kat_binary):
    r = subprocess.run([kat_binary, "0", "40c90fdb", str(os.cpu_count() or 8)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bad_sin 0 bad_cos 0 bad_fused 0 bad_domain 0" in r.stdout


def test_port_matches_libm_on_all_f32(kat_binary):
    r = subprocess.run([kat_binary, "0", "ffffffff", str(os.cpu_count() or 8)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_libm_digest_pinned(oracle):
    g = GOLDEN["sincos_digest_0_2pi"]
    assert oracle.sincos_digest(g["lo"], g["hi"], os.cpu_count() or 8) == g["digest"]
