"""C ABI checks that need no GPU: the in-tree HIP library loads, exports every entry point that
include/ggrs_amd.h declares, and rejects bad configurations before touching the device."""
import os
import re

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def header_symbols():
    src = open(os.path.join(ROOT, "include", "ggrs_amd.h")).read()
    return sorted(set(re.findall(r"\b(ggrs_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    from ggrs_amd import _lib
    assert header_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_every_symbol(engine_lib):
    import ctypes
    for name in header_symbols():
        assert hasattr(engine_lib, name), name
    assert engine_lib.ggrs_abi_version() == 6


def test_nm_exports(engine_lib):
    import subprocess
    from ggrs_amd import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for name in header_symbols():
        assert re.search(rf"\bT {name}\b", out), name


@pytest.mark.parametrize("kw,msg", [
    (dict(check_distance=8, max_prediction=8), "Check distance too big"),
    (dict(num_players=5), "num_players"),
    (dict(num_players=0), "num_players"),
    (dict(num_lanes=0), "num_lanes"),
    (dict(input_capacity=4, check_distance=7, input_delay=2), "input_capacity"),
])
def test_bad_config_rejected_without_device(engine_lib, kw, msg):
    from ggrs_amd import Engine, InvalidRequest
    args = dict(num_lanes=4, num_players=2, max_prediction=8, check_distance=2)
    args.update(kw)
    with pytest.raises(InvalidRequest, match=msg):
        Engine(**args)


@pytest.mark.parametrize("kw,msg", [
    (dict(remote_latency=8, max_prediction=8), "remote_latency"),
    (dict(remote_latency=0), "remote_latency"),
    (dict(local_players=(0, 1)), "remote player"),
    (dict(local_players=(2,)), "local_mask"),
    (dict(predictor=2), "predictor"),
    (dict(max_prediction=-1), "max_prediction"),
])
def test_bad_p2p_config_rejected_without_device(engine_lib, kw, msg):
    from ggrs_amd import InvalidRequest, P2PEngine
    args = dict(num_players=2, remote_latency=3)
    args.update(kw)
    with pytest.raises(InvalidRequest, match=msg):
        P2PEngine(4, **args)


def test_builder_mirrors_reference_check(engine_lib):
    from ggrs_amd import InvalidRequest, SessionBuilder
    with pytest.raises(InvalidRequest, match="Check distance too big"):
        SessionBuilder().with_check_distance(8).start_synctest_session()


def test_no_gpu_is_a_loud_error(engine_lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ggrs_amd import Engine, GgrsError
    with pytest.raises(GgrsError):
        Engine(num_lanes=4)
