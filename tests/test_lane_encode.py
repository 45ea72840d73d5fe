"""ggrs_lane_encode / ggrs_lane_shape (the request handler's per-session encoding, shared by the
Rust crate and the bench's C driver) against the Python encoder (session.encode_lane_lists) on
heterogeneous per-lane P2P request lists from the oracle's P2PSession stream -- rollbacks of
differing depth per lane (p2p_session.rs:304-339,658-714).  Host code only: runs without a GPU."""
import ctypes

import numpy as np
import pytest

from ggrs_amd import _lib
from ggrs_amd._lib import REQ_ADVANCE, REQ_LOAD, REQ_SAVE
from ggrs_amd.session import encode_lane_lists


@pytest.fixture(scope="module")
def L():
    try:
        return _lib.lib()
    except OSError as exc:  # pragma: no cover - the library is built by build()
        pytest.skip(f"engine library not built: {exc}")


class HostBatch:
    """A lane batch laid out in plain host arrays (what ggrs_lane_batch_map returns in pinned memory)."""

    def __init__(self, lanes, players, W, LD, A, S):
        self.tokens = np.full((W, lanes), 0xDEADBEEF, np.uint32)
        self.loads = np.full((LD, lanes), -7, np.int32)
        self.inputs = np.zeros((A, lanes, players), np.uint8)
        self.status = np.zeros((A, lanes, players), np.uint8)
        self.cks = np.zeros((S, lanes), np.uint16)
        self.result = np.zeros(lanes, np.int32)
        vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        self.b = _lib.LaneBatch(W, LD, A, S, ctypes.cast(vp(self.tokens), ctypes.POINTER(ctypes.c_uint32)),
                                ctypes.cast(vp(self.loads), ctypes.POINTER(ctypes.c_int32)),
                                ctypes.cast(vp(self.inputs), ctypes.POINTER(ctypes.c_uint8)),
                                ctypes.cast(vp(self.status), ctypes.POINTER(ctypes.c_uint8)),
                                ctypes.cast(vp(self.cks), ctypes.POINTER(ctypes.c_uint16)),
                                ctypes.cast(vp(self.result), ctypes.POINTER(ctypes.c_int32)))


def encode(L, hb, lanes, players, lane, reqs, inputs, status, lane_frame):
    r = (_lib.Request * max(1, len(reqs)))(*[_lib.Request(k, f) for k, f in reqs])
    inp = np.ascontiguousarray(inputs, np.uint8).reshape(-1)
    st = None if status is None else np.ascontiguousarray(status, np.uint8).reshape(-1)
    bad = ctypes.c_int32()
    rc = L.ggrs_lane_encode(ctypes.byref(hb.b), lanes, players, lane, r, len(reqs),
                            inp.ctypes.data_as(ctypes.c_void_p) if inp.size else None,
                            None if st is None else st.ctypes.data_as(ctypes.c_void_p), lane_frame, ctypes.byref(bad))
    return rc, bad.value


def p2p_lists(oracle, n_lanes, calls, P=2, maxp=8):
    """Per lane: its own P2P session's request lists (jittered arrivals: rollbacks of differing
    depth), as [(kind, frame, inputs, status)] per call."""
    out = []
    for lane in range(n_lanes):
        inputs = oracle.gen_inputs(oracle.session_seed(lane), calls, P, oracle.MODEL_HELD)
        st = oracle.p2p_stream(inputs, oracle.jitter_schedule(calls, maxp, seed=lane), num_players=P,
                               max_prediction=maxp)
        assert st["rc"] == 0
        lane_calls = []
        for c in range(st["calls"]):
            a, b = int(st["call_off"][c]), int(st["call_off"][c + 1])
            lane_calls.append([(int(st["kind"][k]), int(st["frame"][k]), st["inputs"][k], st["status"][k])
                               for k in range(a, b)])
        out.append(lane_calls)
    return out


def test_encode_matches_python_encoder_on_p2p_lists(L, oracle):
    P, lanes, calls = 2, 24, 60
    per_lane = p2p_lists(oracle, lanes, calls, P)
    frames = [0] * lanes
    for c in range(calls):
        lists = [per_lane[l][c] for l in range(lanes)]
        ref = encode_lane_lists(lists, P)
        W, LD, A, S = ref["shape"]
        hb = HostBatch(lanes, P, W, LD, A, S)
        for l, reqs in enumerate(lists):
            rk = [(k, f) for k, f, _, _ in reqs]
            adv = [(i, s) for k, _, i, s in reqs if k == REQ_ADVANCE]
            inp = np.array([i for i, _ in adv], np.uint8).reshape(-1, P)
            st = np.array([s for _, s in adv], np.uint8).reshape(-1, P)
            shape = np.zeros(4, np.int32)
            r = (_lib.Request * max(1, len(rk)))(*[_lib.Request(k, f) for k, f in rk])
            assert L.ggrs_lane_shape(r, len(rk), shape.ctypes.data_as(ctypes.c_void_p)) == 0
            assert tuple(shape) == (-(-len(rk) // 16), sum(k == REQ_LOAD for k, _ in rk), len(adv),
                                    sum(k == REQ_SAVE for k, _ in rk))
            rc, bad = encode(L, hb, lanes, P, l, rk, inp, st, frames[l])
            assert rc == 0 and bad == -1, (c, l, rc, bad)
            # the frame the lane reaches (what lane_result reports after the batch)
            for k, f in rk:
                frames[l] = f if k == REQ_LOAD else (frames[l] + 1 if k == REQ_ADVANCE else frames[l])
        assert (hb.tokens == ref["tokens"]).all(), c
        for l, reqs in enumerate(lists):
            nl = sum(1 for r in reqs if r[0] == REQ_LOAD)
            na = sum(1 for r in reqs if r[0] == REQ_ADVANCE)
            assert (hb.loads[:nl, l] == ref["load_frames"][:nl, l]).all()
            assert (hb.inputs[:na, l] == ref["inputs"][:na, l]).all()
            assert (hb.status[:na, l] == ref["status"][:na, l]).all()
    # the lists really are heterogeneous: differing lengths and rollback depths across lanes
    assert len({len(per_lane[l][c]) for l in range(lanes) for c in range(calls)}) > 3


def test_exactly_full_words_need_no_end_token(L):
    """A list of exactly 16 W requests fills W words (the Rust crate used to ask for W + 1)."""
    P, lanes = 1, 3
    reqs = [(REQ_SAVE, 0), (REQ_ADVANCE, 0)] * 8 + [(REQ_SAVE, 8), (REQ_ADVANCE, 0)] * 0
    frames = [(REQ_SAVE, f // 2) if k == REQ_SAVE else (k, 0) for f, (k, _) in enumerate(reqs)]
    shape = np.zeros(4, np.int32)
    r = (_lib.Request * 16)(*[_lib.Request(k, f) for k, f in frames])
    assert L.ggrs_lane_shape(r, 16, shape.ctypes.data_as(ctypes.c_void_p)) == 0
    assert shape[0] == 1
    hb = HostBatch(lanes, P, 1, 1, 8, 8)
    rc, bad = encode(L, hb, lanes, P, 1, frames, np.arange(8, dtype=np.uint8), None, 0)
    assert rc == 0 and bad == -1
    want = sum(((_lib.TOK_SAVE if k == REQ_SAVE else _lib.TOK_ADVANCE) << (2 * i)) for i, (k, _) in enumerate(frames))
    assert int(hb.tokens[0, 1]) == want
    assert (hb.inputs[:, 1, 0] == np.arange(8)).all()
    assert (hb.status[:, 1, 0] == 0).all()  # status NULL = Confirmed


def test_save_frame_mismatch_rejects_the_lane(L):
    """ex_game.rs:104 asserts a Save's frame equals the state's: the encoder rejects the lane (an
    empty list: it will not run) and names the request."""
    P, lanes = 2, 4
    hb = HostBatch(lanes, P, 2, 1, 4, 4)
    reqs = [(REQ_LOAD, 5), (REQ_ADVANCE, 0), (REQ_SAVE, 6), (REQ_ADVANCE, 0), (REQ_SAVE, 9)]
    rc, bad = encode(L, hb, lanes, P, 2, reqs, np.zeros((2, P), np.uint8), None, 7)
    assert rc == _lib.GGRS_E_PRECONDITION and bad == 4
    assert "ex_game.rs:104" in L.ggrs_last_error().decode()
    assert (hb.tokens[:, 2] == 0xFFFFFFFF).all()  # every token END
    # from the right start frame the same list passes up to the bad Save only
    rc, bad = encode(L, hb, lanes, P, 2, reqs[:4], np.zeros((2, P), np.uint8), None, 7)
    assert rc == 0
    # the NULL_FRAME start skips the check
    rc, bad = encode(L, hb, lanes, P, 3, reqs, np.zeros((2, P), np.uint8), None, -1)
    assert rc == 0 and bad == -1


def test_list_beyond_the_batch_shape_is_invalid(L):
    P, lanes = 2, 2
    hb = HostBatch(lanes, P, 1, 1, 2, 2)
    reqs = [(REQ_SAVE, 0), (REQ_ADVANCE, 0)] * 3
    rc, _ = encode(L, hb, lanes, P, 0, [(k, i // 2) for i, (k, _) in enumerate(reqs)], np.zeros((3, P), np.uint8),
                   None, 0)
    assert rc == _lib.GGRS_E_INVALID
    assert "exceeds the batch" in L.ggrs_last_error().decode()
