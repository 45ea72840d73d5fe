"""Host-side mirror of GGRS's session surface over the batched HIP engine.

The names, defaults, argument meanings and errors follow the reference so that code written
against GGRS reads the same here; every object drives ALL lanes of one engine (one lane = one
(session, branch)), so inputs carry a leading lane axis.

  SessionBuilder          src/sessions/builder.rs:30-78 (defaults :13-27), with_* :120-200,
                          start_synctest_session :346-358
  SyncTestSession         src/sessions/sync_test_session.rs:11-218
  GgrsRequest variants    src/lib.rs:171-195 (SaveGameState, LoadGameState, AdvanceFrame)
  BoxGameHandler          the user's request handler, examples/ex_game/ex_game.rs:79-127
  MismatchedChecksum      src/error.rs:44-50

There is no CPU path: the engine's HIP library must be built and a GPU present.
"""
import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import (GgrsError, InvalidRequest, PreconditionError, NULL_FRAME, REQ_ADVANCE, REQ_LOAD,
                   REQ_SAVE, LANE_MISMATCH)

# builder.rs:13-27
DEFAULT_PLAYERS = 2
DEFAULT_INPUT_DELAY = 0
DEFAULT_MAX_PREDICTION_FRAMES = 8
DEFAULT_CHECK_DISTANCE = 2


class MismatchedChecksum(GgrsError):
    """GgrsError::MismatchedChecksum { current_frame, mismatched_frames } (error.rs:44-50).

    Raised when at least one lane's SyncTest found a resimulated checksum differing from the
    first one recorded.  `current_frame`/`mismatched_frames` describe the first such lane;
    `lanes` lists every halted lane (they stop, like a reference session that returned Err).
    """

    def __init__(self, current_frame, mismatched_frames, lanes):
        super().__init__(0, f"Detected checksum mismatch during rollback on frame {current_frame}, "
                            f"mismatched frames: {mismatched_frames} (lanes {list(lanes)[:8]}...)")
        self.current_frame = current_frame
        self.mismatched_frames = mismatched_frames
        self.lanes = lanes


def _vp(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class Engine:
    """Owns one ggrs_engine_t (C ABI include/ggrs_amd.h)."""

    def __init__(self, num_lanes, num_players=DEFAULT_PLAYERS,
                 max_prediction=DEFAULT_MAX_PREDICTION_FRAMES, check_distance=DEFAULT_CHECK_DISTANCE,
                 input_delay=DEFAULT_INPUT_DELAY, input_capacity=0, device=0, trace_capacity=0):
        self._L = _lib.lib()
        cfg = _lib.Config(num_lanes, num_players, max_prediction, check_distance, input_delay,
                          input_capacity, device, trace_capacity)
        h = ctypes.c_void_p()
        _lib.check(self._L.ggrs_engine_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        out = _lib.Config()
        _lib.check(self._L.ggrs_engine_config(self._h, ctypes.byref(out)))
        self.cfg = out
        self.num_lanes = num_lanes
        self.num_players = num_players
        self.ring_len = max_prediction + 1
        self.state_bytes = 36 + 20 * num_players

    def close(self):
        if getattr(self, "_h", None):
            self._L.ggrs_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- inputs / programs
    def add_local_inputs(self, first_frame, inputs):
        a = np.ascontiguousarray(inputs, np.uint8)
        if a.ndim != 3 or a.shape[1:] != (self.num_lanes, self.num_players):
            raise InvalidRequest(-1, f"inputs must be [n][{self.num_lanes}][{self.num_players}], got {a.shape}")
        _lib.check(self._L.ggrs_add_local_inputs(self._h, first_frame, a.shape[0], _vp(a)))

    def add_local_inputs_device(self, first_frame, n_frames, device_ptr):
        _lib.check(self._L.ggrs_add_local_inputs_device(self._h, first_frame, n_frames,
                                                          ctypes.c_void_p(device_ptr)))

    def synctest_advance_frames(self, n):
        _lib.check(self._L.ggrs_synctest_advance_frames(self._h, n))

    def set_synctest_path(self, path):
        """_lib.PATH_PIPELINED (default) or _lib.PATH_SEQUENTIAL."""
        _lib.check(self._L.ggrs_set_synctest_path(self._h, path))

    def handle_requests(self, reqs, inputs=None, status=None):
        arr = (_lib.Request * len(reqs))(*[_lib.Request(k, f) for k, f in reqs])
        i = None if inputs is None else np.ascontiguousarray(inputs, np.uint8)
        s = None if status is None else np.ascontiguousarray(status, np.uint8)
        _lib.check(self._L.ggrs_handle_requests(self._h, arr, len(reqs), _vp(i), _vp(s)))

    def synchronize(self):
        _lib.check(self._L.ggrs_synchronize(self._h))

    def corrupt_on_load(self, lane, frame):
        _lib.check(self._L.ggrs_debug_corrupt_on_load(self._h, lane, frame))

    # ---- reads
    def current_frame(self):
        v = ctypes.c_int32()
        _lib.check(self._L.ggrs_current_frame(self._h, ctypes.byref(v)))
        return v.value

    def mismatches(self):
        n = self.num_lanes
        st, mf, mm = np.zeros(n, np.int32), np.zeros(n, np.int32), np.zeros(n, np.uint64)
        _lib.check(self._L.ggrs_read_mismatches(self._h, _vp(st), _vp(mf), _vp(mm)))
        return st, mf, mm

    def save_checksums(self, frame):
        out = np.zeros(self.num_lanes, np.uint16)
        _lib.check(self._L.ggrs_read_save_checksums(self._h, frame, _vp(out)))
        return out

    def state(self, lane):
        out = np.zeros(self.state_bytes, np.uint8)
        _lib.check(self._L.ggrs_read_state(self._h, lane, _vp(out)))
        return out

    def ring(self, lane):
        fr = np.zeros(self.ring_len, np.int32)
        ck = np.zeros(self.ring_len, np.uint16)
        st = np.zeros((self.ring_len, self.state_bytes), np.uint8)
        _lib.check(self._L.ggrs_read_ring(self._h, lane, _vp(fr), _vp(ck), _vp(st)))
        return fr, ck, st

    def trace(self, first_frame, n):
        out = np.zeros((n, self.num_lanes), np.uint16)
        _lib.check(self._L.ggrs_read_trace(self._h, first_frame, n, _vp(out)))
        return out

    def timing_reset(self):
        _lib.check(self._L.ggrs_timing_reset(self._h))

    def timing_read(self):
        """(summed device ms of the fused launches since timing_reset, launch count)."""
        ms, n = ctypes.c_float(), ctypes.c_int32()
        _lib.check(self._L.ggrs_timing_read(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def last_launch_ms(self):
        v = ctypes.c_float()
        _lib.check(self._L.ggrs_last_launch_ms(self._h, ctypes.byref(v)))
        return v.value


class SessionBuilder:
    """builder.rs:30-78, with the batched-engine extras with_num_lanes / with_device."""

    def __init__(self):
        self.num_players = DEFAULT_PLAYERS
        self.max_prediction = DEFAULT_MAX_PREDICTION_FRAMES
        self.input_delay = DEFAULT_INPUT_DELAY
        self.check_dist = DEFAULT_CHECK_DISTANCE
        self.num_lanes = 1
        self.device = 0
        self.input_capacity = 0
        self.trace_capacity = 0

    def with_num_players(self, n):
        self.num_players = n
        return self

    def with_max_prediction_window(self, window):
        self.max_prediction = window
        return self

    def with_input_delay(self, delay):
        self.input_delay = delay
        return self

    def with_check_distance(self, check_distance):
        self.check_dist = check_distance
        return self

    def with_num_lanes(self, lanes):
        self.num_lanes = lanes
        return self

    def with_device(self, device):
        self.device = device
        return self

    def with_input_capacity(self, frames):
        self.input_capacity = frames
        return self

    def with_trace_capacity(self, frames):
        self.trace_capacity = frames
        return self

    def start_synctest_session(self):
        """builder.rs:346-358: InvalidRequest("Check distance too big.") if check >= max_pred."""
        if self.check_dist >= self.max_prediction:
            raise InvalidRequest(-1, "Check distance too big.")
        return SyncTestSession(Engine(self.num_lanes, self.num_players, self.max_prediction,
                                      self.check_dist, self.input_delay, self.input_capacity,
                                      self.device, self.trace_capacity),
                               self.max_prediction, self.check_dist)


class SyncTestSession:
    """sync_test_session.rs:11-218 over L lanes: inputs are per lane, frames are shared."""

    def __init__(self, engine, max_prediction, check_distance):
        self.engine = engine
        self._max_prediction = max_prediction
        self._check_distance = check_distance
        self._pending = {}
        self._added = 0
        self._reported = np.zeros(engine.num_lanes, bool)

    def num_players(self):
        return self.engine.num_players

    def max_prediction(self):
        return self._max_prediction

    def check_distance(self):
        return self._check_distance

    def current_frame(self):
        return self.engine.current_frame()

    def add_local_input(self, player_handle, inputs):
        """:61-74 -- `inputs` holds this player's input for every lane ([num_lanes] u8)."""
        if not 0 <= player_handle < self.engine.num_players:
            raise InvalidRequest(-1, "The player handle you provided is not valid.")
        a = np.asarray(inputs, np.uint8).reshape(-1)
        if a.size != self.engine.num_lanes:
            raise InvalidRequest(-1, f"expected {self.engine.num_lanes} lane inputs, got {a.size}")
        self._pending[player_handle] = a

    def advance_frame(self):
        """:85-150 + the handler's execution of the returned requests, on every lane."""
        if len(self._pending) != self.engine.num_players:
            raise InvalidRequest(-1, "Missing local input while calling advance_frame().")
        frame = np.stack([self._pending[p] for p in range(self.engine.num_players)], axis=1)[None]
        self._pending.clear()
        self.add_local_inputs(frame)
        self.advance_frames(1)

    def add_local_inputs(self, inputs):
        """Batched add_local_input for consecutive frames: inputs[n][num_lanes][num_players]."""
        a = np.asarray(inputs, np.uint8)
        self.engine.add_local_inputs(self._added, a)
        self._added += a.shape[0]

    def advance_frames(self, n, check=True):
        """n fused advance_frame calls.  With check=True, raise MismatchedChecksum if a lane
        halted (each lane reported once)."""
        self.engine.synctest_advance_frames(n)
        if check:
            self.raise_on_mismatch()

    def raise_on_mismatch(self):
        st, mf, mm = self.engine.mismatches()
        bad = (st == LANE_MISMATCH) & ~self._reported
        if bad.any():
            self._reported |= bad
            lanes = np.nonzero(bad)[0]
            first = lanes[np.argmin(mf[lanes])]
            cur = int(mf[first])
            frames = [cur - self._check_distance + k for k in range(64) if (int(mm[first]) >> k) & 1]
            raise MismatchedChecksum(cur, frames, lanes)


# -------------------------------------------------------------------- GgrsRequest (lib.rs:171-195)
@dataclass
class SaveGameState:
    frame: int


@dataclass
class LoadGameState:
    frame: int


@dataclass
class AdvanceFrame:
    inputs: np.ndarray                    # [num_lanes][num_players] Input.inp
    status: np.ndarray = field(default=None)  # [num_lanes][num_players] InputStatus (None: confirmed)


class BoxGameHandler:
    """The ex_game request handler (ex_game.rs:79-127) executing a GGRS request list on all
    lanes in one fused launch; saved states stay in the engine's HBM ring and the checksum each
    save produced is returned per lane (what a handler passes to GameStateCell::save)."""

    def __init__(self, engine):
        self.engine = engine

    def handle_requests(self, requests):
        reqs, inputs, status, saves = [], [], [], []
        any_status = any(isinstance(r, AdvanceFrame) and r.status is not None for r in requests)
        for r in requests:
            if isinstance(r, SaveGameState):
                reqs.append((REQ_SAVE, r.frame))
                saves.append(r.frame)
            elif isinstance(r, LoadGameState):
                reqs.append((REQ_LOAD, r.frame))
            elif isinstance(r, AdvanceFrame):
                reqs.append((REQ_ADVANCE, 0))
                inputs.append(np.asarray(r.inputs, np.uint8))
                if any_status:
                    st = r.status if r.status is not None else np.zeros_like(inputs[-1])
                    status.append(np.asarray(st, np.uint8))
            else:
                raise InvalidRequest(-1, f"unknown request {r!r}")
        inp = np.stack(inputs) if inputs else None
        st = np.stack(status) if status else None
        self.engine.handle_requests(reqs, inp, st)
        return {f: self.engine.save_checksums(f) for f in saves}


__all__ = ["Engine", "SessionBuilder", "SyncTestSession", "BoxGameHandler", "SaveGameState",
           "LoadGameState", "AdvanceFrame", "GgrsError", "InvalidRequest", "PreconditionError",
           "MismatchedChecksum", "NULL_FRAME"]
