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
import weakref
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

    def handle_requests_lanes(self, reqs, offsets, inputs=None, status=None, check=True):
        """Per-lane request lists (ggrs_handle_requests_lanes): reqs [n][2] (kind, frame) of every
        lane back to back, offsets [num_lanes + 1], inputs / status [n_advance][num_players] in the
        same order.  Returns (checksum of every Save in order, lane_result [num_lanes]: >= 0 the
        lane's frame after its list, -(1 + k) its failing request).  With check, a failed lane
        raises LanesFailed (the other lanes ran)."""
        r = np.ascontiguousarray(reqs, np.int32).reshape(-1, 2)
        off = np.ascontiguousarray(offsets, np.int32)
        if off.shape != (self.num_lanes + 1,):
            raise InvalidRequest(-1, f"offsets must have {self.num_lanes + 1} entries")
        i = None if inputs is None else np.ascontiguousarray(inputs, np.uint8)
        st = None if status is None else np.ascontiguousarray(status, np.uint8)
        n_save = int((r[:, 0] == REQ_SAVE).sum())
        cks = np.zeros(max(n_save, 1), np.uint16)
        res = np.zeros(self.num_lanes, np.int32)
        rc = self._L.ggrs_handle_requests_lanes(self._h, _vp(r), _vp(off), _vp(i), _vp(st), _vp(cks), _vp(res))
        self._check_batches()  # the CSR form may have grown (and freed) the mapped lane batch
        if rc == _lib.GGRS_E_PRECONDITION:
            if check:
                raise LanesFailed(self._L.ggrs_last_error().decode(errors="replace"), res)
        else:
            _lib.check(rc)
        return cks[:n_save], res

    def lane_batch(self, token_words, load_slots, adv_rows, save_rows):
        """The engine's mapped per-lane batch (ggrs_lane_batch_map) as numpy views.  Views of an
        earlier, smaller mapping are invalidated when this one grows it."""
        b = LaneBatch(self, token_words, load_slots, adv_rows, save_rows)
        self._check_batches()
        self.__dict__.setdefault("_batches", []).append(weakref.ref(b))
        return b

    def _check_batches(self):
        """Invalidate LaneBatch views whose mapping the engine has replaced (their memory is freed)."""
        live = [w() for w in self.__dict__.get("_batches", [])]
        live = [b for b in live if b is not None and b.valid]
        if not live:
            self._batches = []
            return
        cur = _lib.LaneBatch()
        _lib.check(self._L.ggrs_lane_batch_map(self._h, 0, 0, 0, 0, ctypes.byref(cur)))
        addr = ctypes.cast(cur.tokens, ctypes.c_void_p).value
        for b in live:
            if b.tokens_addr != addr:
                b._invalidate()
        self._batches = [weakref.ref(b) for b in live if b.valid]

    def set_lane_server(self, on=True):
        """ggrs_lane_server: per-lane batches through one persistent kernel (default) or one
        launch each."""
        _lib.check(self._L.ggrs_lane_server(self._h, int(bool(on))))

    def lane_frames(self):
        out = np.zeros(self.num_lanes, np.int32)
        _lib.check(self._L.ggrs_read_lane_frames(self._h, _vp(out)))
        return out

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

    def save_checksums_frames(self, frames):
        """[len(frames)][num_lanes] checksums of the saved cells of `frames`, one transfer wait."""
        fr = np.ascontiguousarray(frames, np.int32)
        out = np.zeros((len(fr), self.num_lanes), np.uint16)
        _lib.check(self._L.ggrs_read_save_checksums_frames(self._h, _vp(fr), len(fr), _vp(out)))
        return out

    def state(self, lane):
        out = np.zeros(self.state_bytes, np.uint8)
        _lib.check(self._L.ggrs_read_state(self._h, lane, _vp(out)))
        return out

    def states(self):
        """state(lane) for every lane, one transfer: [num_lanes][state_bytes]."""
        out = np.zeros((self.num_lanes, self.state_bytes), np.uint8)
        _lib.check(self._L.ggrs_read_states(self._h, _vp(out)))
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

    def timing_stop(self):
        """Record the span's end behind the last launch without waiting (timing_read reports it)."""
        _lib.check(self._L.ggrs_timing_stop(self._h))

    def timing_read(self):
        """(summed device ms of the fused launches since timing_reset, launch count)."""
        ms, n = ctypes.c_float(), ctypes.c_int32()
        _lib.check(self._L.ggrs_timing_read(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def last_launch_ms(self):
        v = ctypes.c_float()
        _lib.check(self._L.ggrs_last_launch_ms(self._h, ctypes.byref(v)))
        return v.value


class LanesFailed(PreconditionError):
    """Some lanes' request lists failed validation (a reference session would have panicked):
    `lane_result[l] = -(1 + k)` names lane l's failing request; the other lanes ran."""

    def __init__(self, msg, lane_result):
        super().__init__(_lib.GGRS_E_PRECONDITION, msg)
        self.lane_result = lane_result
        self.lanes = np.nonzero(lane_result < 0)[0]


class LaneBatch:
    """Numpy views of an engine's mapped lane batch (ggrs_lane_batch_t; pinned host memory the
    kernel reads and writes in place).  Fill tokens / load_frames / inputs (/ status), then run()."""

    def __init__(self, engine, token_words, load_slots, adv_rows, save_rows):
        self.engine = engine
        b = _lib.LaneBatch()
        _lib.check(engine._L.ggrs_lane_batch_map(engine._h, token_words, load_slots, adv_rows, save_rows,
                                                 ctypes.byref(b)))
        self._b = b
        self.valid = True
        self.tokens_addr = ctypes.cast(b.tokens, ctypes.c_void_p).value
        L, P = engine.num_lanes, engine.num_players
        W, LD, A, S = b.token_words, b.load_slots, b.adv_rows, b.save_rows
        view = np.ctypeslib.as_array
        self.tokens = view(b.tokens, shape=(W, L))
        self.load_frames = view(b.load_frames, shape=(LD, L))
        self.inputs = view(b.inputs, shape=(A, L, P))
        self.status = view(b.status, shape=(A, L, P))
        self.checksums = view(b.checksums, shape=(S, L))
        self.lane_result = view(b.lane_result, shape=(L,))
        self.shape = (W, LD, A, S)

    def _invalidate(self):
        self.valid = False
        self.tokens = self.load_frames = self.inputs = self.status = self.checksums = self.lane_result = None

    def run(self, token_words=None, load_slots=None, adv_rows=None, save_rows=None, status=False):
        """ggrs_lane_batch_run with the given counts (default: the mapped shape); returns the number
        of lanes that failed validation (their lane_result < 0)."""
        if not self.valid:
            raise _lib.GgrsError(_lib.GGRS_E_STATE, "lane batch views are stale: the engine re-mapped the "
                                                           "batch (ggrs_lane_batch_map)")
        b = self._run_struct(token_words, load_slots, adv_rows, save_rows)
        n = ctypes.c_int32()
        rc = self.engine._L.ggrs_lane_batch_run(self.engine._h, ctypes.byref(b), _lib.BATCH_STATUS if status else 0,
                                                ctypes.byref(n))
        if rc != _lib.GGRS_E_PRECONDITION:
            _lib.check(rc)
        return n.value


    def encode(self, lane, reqs, inputs=None, status=None, lane_frame=NULL_FRAME):
        """ggrs_lane_encode: lane `lane`'s ordered list -- reqs [(kind, frame)], inputs / status
        [n_advance][P] -- into this batch (the C encoder the Rust handler and the bench driver
        share).  lane_frame: the lane's frame before the list (NULL_FRAME skips the Save-frame
        check).  Returns -1, or the index of the rejected Save (the lane was encoded empty)."""
        if not self.valid:
            raise _lib.GgrsError(_lib.GGRS_E_STATE, "lane batch views are stale")
        P = self.engine.num_players
        r = (_lib.Request * max(1, len(reqs)))(*[_lib.Request(int(k), int(f)) for k, f in reqs])
        i = None if inputs is None else np.ascontiguousarray(inputs, np.uint8).reshape(-1)
        st = None if status is None else np.ascontiguousarray(status, np.uint8).reshape(-1)
        bad = ctypes.c_int32()
        rc = self.engine._L.ggrs_lane_encode(ctypes.byref(self._b), self.engine.num_lanes, P, lane, r, len(reqs),
                                             _vp(i), _vp(st), lane_frame, ctypes.byref(bad))
        if rc == _lib.GGRS_E_PRECONDITION:
            return bad.value
        _lib.check(rc)
        return -1

    def _run_struct(self, token_words, load_slots, adv_rows, save_rows):
        W, LD, A, S = self.shape
        return _lib.LaneBatch(W if token_words is None else token_words, LD if load_slots is None else load_slots,
                              A if adv_rows is None else adv_rows, S if save_rows is None else save_rows,
                              self._b.tokens, self._b.load_frames, self._b.inputs, self._b.status,
                              self._b.checksums, self._b.lane_result)

    def submit(self, token_words=None, load_slots=None, adv_rows=None, save_rows=None, status=False):
        """ggrs_lane_batch_submit: publish the batch and return at once (wait() collects it)."""
        if not self.valid:
            raise _lib.GgrsError(_lib.GGRS_E_STATE, "lane batch views are stale")
        b = self._run_struct(token_words, load_slots, adv_rows, save_rows)
        _lib.check(self.engine._L.ggrs_lane_batch_submit(self.engine._h, ctypes.byref(b),
                                                         _lib.BATCH_STATUS if status else 0))

    def wait(self):
        """ggrs_lane_batch_wait: the submitted batch's results are in host memory; returns the
        number of lanes that failed validation."""
        n = ctypes.c_int32()
        rc = self.engine._L.ggrs_lane_batch_wait(self.engine._h, ctypes.byref(n))
        if rc != _lib.GGRS_E_PRECONDITION:
            _lib.check(rc)
        return n.value


def encode_lane_lists(lists, num_players):
    """Per-lane request lists -> the batch encoding (tests and tools): lists[l] is lane l's
    requests as (kind, frame, inputs[P] or None, status[P] or None).  Returns dict of tokens
    [W][L], load_frames [LD][L], inputs / status [A][L][P] and the shape (W, LD, A, S)."""
    L = len(lists)
    n_tok = max((len(x) for x in lists), default=0)
    W = max(1, -(-n_tok // _lib.TOKENS_PER_WORD))
    LD = max(1, max(sum(1 for r in x if r[0] == REQ_LOAD) for x in lists))
    A = max(1, max(sum(1 for r in x if r[0] == REQ_ADVANCE) for x in lists))
    S = max(1, max(sum(1 for r in x if r[0] == REQ_SAVE) for x in lists))
    tok = np.full((W * _lib.TOKENS_PER_WORD, L), _lib.TOK_END, np.uint64)
    loads = np.full((LD, L), NULL_FRAME, np.int32)
    inp = np.zeros((A, L, num_players), np.uint8)
    st = np.zeros((A, L, num_players), np.uint8)
    kind_tok = {REQ_SAVE: _lib.TOK_SAVE, REQ_ADVANCE: _lib.TOK_ADVANCE, REQ_LOAD: _lib.TOK_LOAD}
    for l, reqs in enumerate(lists):
        nl = na = 0
        for k, (kind, frame, i, s) in enumerate(reqs):
            tok[k, l] = kind_tok[kind]
            if kind == REQ_LOAD:
                loads[nl, l] = frame
                nl += 1
            elif kind == REQ_ADVANCE:
                inp[na, l] = i
                if s is not None:
                    st[na, l] = s
                na += 1
    shifts = (2 * np.arange(_lib.TOKENS_PER_WORD, dtype=np.uint64))[None, :, None]
    words = (tok.reshape(W, _lib.TOKENS_PER_WORD, L) << shifts).sum(axis=1).astype(np.uint32)
    return dict(tokens=words, load_frames=loads, inputs=inp, status=st, shape=(W, LD, A, S))


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
        self._unchecked = False  # frames advanced since the device's mismatch state was last read

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
        """:85-150 + the handler's execution of the returned requests, on every lane.  Error order
        as the reference: a lane's MismatchedChecksum (:89-102) before the missing-input
        InvalidRequest (:108-113).  The device's mismatch state is re-read only when frames were
        advanced without a check since the last one (advance_frames(check=True) already read it)."""
        if self._unchecked:
            self.raise_on_mismatch()
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
        self._unchecked = True
        if check:
            self.raise_on_mismatch()

    def raise_on_mismatch(self):
        st, mf, mm = self.engine.mismatches()
        self._unchecked = False
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
        cks = self.engine.save_checksums_frames(saves) if saves else []
        return {f: cks[k] for k, f in enumerate(saves)}


class LaneBoxGameHandler:
    """The ex_game request handler (ex_game.rs:79-127) for lanes that are independent GGRS
    sessions: handle_requests(lists) executes lists[l] -- lane l's own Vec<GgrsRequest> from its
    own advance_frame() -- for every lane in one launch (ggrs_handle_requests_lanes) and returns,
    per lane, the checksum of each SaveGameState in order (what the handler passes to
    GameStateCell::save)."""

    def __init__(self, engine):
        self.engine = engine

    def handle_requests(self, lists):
        P = self.engine.num_players
        reqs, offsets, inputs, status = [], [0], [], []
        any_status = any(isinstance(r, AdvanceFrame) and r.status is not None for x in lists for r in x)
        for x in lists:
            for r in x:
                if isinstance(r, SaveGameState):
                    reqs.append((REQ_SAVE, r.frame))
                elif isinstance(r, LoadGameState):
                    reqs.append((REQ_LOAD, r.frame))
                elif isinstance(r, AdvanceFrame):
                    reqs.append((REQ_ADVANCE, 0))
                    inputs.append(np.asarray(r.inputs, np.uint8).reshape(P))
                    if any_status:
                        st = r.status if r.status is not None else np.zeros(P, np.uint8)
                        status.append(np.asarray(st, np.uint8).reshape(P))
                else:
                    raise InvalidRequest(-1, f"unknown request {r!r}")
            offsets.append(len(reqs))
        cks, _ = self.engine.handle_requests_lanes(
            np.array(reqs, np.int32).reshape(-1, 2), np.array(offsets, np.int32),
            np.stack(inputs) if inputs else None, np.stack(status) if status else None)
        out, k = [], 0
        for x in lists:
            n = sum(1 for r in x if isinstance(r, SaveGameState))
            out.append(cks[k:k + n])
            k += n
        return out


__all__ = ["Engine", "SessionBuilder", "SyncTestSession", "BoxGameHandler", "LaneBoxGameHandler", "LaneBatch",
           "LanesFailed", "encode_lane_lists", "SaveGameState",
           "LoadGameState", "AdvanceFrame", "GgrsError", "InvalidRequest", "PreconditionError",
           "MismatchedChecksum", "NULL_FRAME"]
