"""P2P rollback decision over the engine's C ABI (include/ggrs_amd.h, ggrs_p2p_*).

One P2PEngine holds S sessions of one peer.  Each call of advance_frames(n) runs n x
P2PSession::advance_frame (src/sessions/p2p_session.rs:265-426) + the ex_game handler for every
session: the remote players' inputs of frame f - remote_latency arrive, mispredictions found by
InputQueue (src/input_queue.rs:190-230) roll the session back (adjust_gamestate, :658-714), the
current frame is saved and advanced with synchronized inputs (remote players predicted,
src/lib.rs:390-406).  The device decides per session whether and how far to roll back.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import InvalidRequest

PREDICT_REPEAT_LAST, PREDICT_DEFAULT = 0, 1


class P2PConfig(ctypes.Structure):
    _fields_ = [
        ("num_sessions", ctypes.c_int32),
        ("num_players", ctypes.c_int32),
        ("local_mask", ctypes.c_int32),
        ("input_delay", ctypes.c_int32),
        ("max_prediction", ctypes.c_int32),
        ("remote_latency", ctypes.c_int32),
        ("predictor", ctypes.c_int32),
        ("input_capacity", ctypes.c_int32),
        ("trace_capacity", ctypes.c_int32),
        ("device", ctypes.c_int32),
    ]


_bound = False


def _bind(L):
    global _bound
    if _bound:
        return
    vp = ctypes.c_void_p
    P = ctypes.POINTER
    i32 = ctypes.c_int32
    L.ggrs_p2p_engine_create.argtypes = [P(P2PConfig), P(vp)]
    L.ggrs_p2p_engine_destroy.argtypes = [vp]
    L.ggrs_p2p_engine_config.argtypes = [vp, P(P2PConfig)]
    L.ggrs_p2p_add_inputs.argtypes = [vp, i32, i32, vp]
    L.ggrs_p2p_advance_frames.argtypes = [vp, i32]
    L.ggrs_p2p_current_frame.argtypes = [vp, P(i32)]
    L.ggrs_p2p_calls.argtypes = [vp, P(i32)]
    L.ggrs_p2p_synchronize.argtypes = [vp]
    L.ggrs_p2p_read_state.argtypes = [vp, i32, vp]
    L.ggrs_p2p_read_states.argtypes = [vp, vp]
    L.ggrs_p2p_read_ring.argtypes = [vp, i32, vp, vp, vp]
    L.ggrs_p2p_read_stats.argtypes = [vp, vp, vp]
    L.ggrs_p2p_read_queues.argtypes = [vp, vp]
    L.ggrs_p2p_read_trace.argtypes = [vp, i32, i32, vp]
    L.ggrs_p2p_timing_reset.argtypes = [vp]
    L.ggrs_p2p_timing_stop.argtypes = [vp]
    L.ggrs_p2p_timing_read.argtypes = [vp, P(ctypes.c_float), P(i32)]
    L.ggrs_p2p_set_desync_detection.argtypes = [vp, i32]
    L.ggrs_p2p_local_checksums.argtypes = [vp, i32, vp, i32]
    L.ggrs_p2p_compare_checksums.argtypes = [vp, i32, vp, i32, vp, P(i32)]
    L.ggrs_p2p_debug_desync.argtypes = [vp, i32, i32]
    L.ggrs_p2p_set_sparse_saving.argtypes = [vp, i32]
    L.ggrs_p2p_set_unstaged.argtypes = [vp, i32]
    L.ggrs_p2p_set_arrival_schedule.argtypes = [vp, i32]
    L.ggrs_p2p_add_arrivals.argtypes = [vp, i32, i32, vp, vp]
    L.ggrs_p2p_add_peer_reports.argtypes = [vp, i32, i32, vp]
    L.ggrs_p2p_read_sessions.argtypes = [vp, vp, vp, vp]
    L.ggrs_p2p_read_reports.argtypes = [vp, i32, i32, vp, vp, vp, vp]
    for name in _lib.EXPORTS:
        if name.startswith("ggrs_p2p_"):
            getattr(L, name).restype = ctypes.c_int
    _bound = True


def peer_report(player, reporter, frame):
    """GGRS_PEER_REPORT: remote player `reporter`'s endpoint reports remote player `player`
    disconnected with last frame `frame`."""
    return 16 | player | reporter << 2 | (frame + 1) << 5


def _vp(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class P2PEngine:
    """S sessions of one peer: local players `local_players`, every other player remote."""

    def __init__(self, num_sessions, num_players=2, local_players=(0,), input_delay=0,
                 max_prediction=8, remote_latency=4, predictor=PREDICT_REPEAT_LAST,
                 input_capacity=0, trace_capacity=0, device=0):
        self._L = _lib.lib()
        _bind(self._L)
        mask = 0
        for p in local_players:
            mask |= 1 << p
        cfg = P2PConfig(num_sessions, num_players, mask, input_delay, max_prediction, remote_latency,
                        predictor, input_capacity, trace_capacity, device)
        h = ctypes.c_void_p()
        _lib.check(self._L.ggrs_p2p_engine_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self.num_sessions, self.num_players, self.local_mask = num_sessions, num_players, mask
        self.input_delay, self.max_prediction = input_delay, max_prediction
        self.remote_latency, self.predictor = remote_latency, predictor
        self.ring_len = max_prediction + 1
        self.state_bytes = 36 + 20 * num_players

    def close(self):
        if getattr(self, "_h", None):
            self._L.ggrs_p2p_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_inputs(self, first_frame, inputs):
        """inputs [n][S][P]: row g = local players' add_local_input of call g, remote players'
        input of frame g."""
        a = np.ascontiguousarray(inputs, np.uint8)
        if a.ndim != 3 or a.shape[1:] != (self.num_sessions, self.num_players):
            raise InvalidRequest(-1, f"inputs must be [n][{self.num_sessions}][{self.num_players}]")
        _lib.check(self._L.ggrs_p2p_add_inputs(self._h, first_frame, a.shape[0], _vp(a)))

    def advance_frames(self, n=1):
        _lib.check(self._L.ggrs_p2p_advance_frames(self._h, n))

    def current_frame(self):
        v = ctypes.c_int32()
        _lib.check(self._L.ggrs_p2p_current_frame(self._h, ctypes.byref(v)))
        return v.value

    def calls(self):
        """advance_frame calls made (current_frame() is the session's frame: the same in rollback
        mode, behind it in lockstep mode)."""
        v = ctypes.c_int32()
        _lib.check(self._L.ggrs_p2p_calls(self._h, ctypes.byref(v)))
        return v.value

    def synchronize(self):
        _lib.check(self._L.ggrs_p2p_synchronize(self._h))

    def state(self, session):
        out = np.zeros(self.state_bytes, np.uint8)
        _lib.check(self._L.ggrs_p2p_read_state(self._h, session, _vp(out)))
        return out

    def states(self):
        """state(session) for every session, one transfer: [num_sessions][state_bytes]."""
        out = np.zeros((self.num_sessions, self.state_bytes), np.uint8)
        _lib.check(self._L.ggrs_p2p_read_states(self._h, _vp(out)))
        return out

    def ring(self, session):
        frames = np.zeros(self.ring_len, np.int32)
        cks = np.zeros(self.ring_len, np.uint16)
        states = np.zeros((self.ring_len, self.state_bytes), np.uint8)
        _lib.check(self._L.ggrs_p2p_read_ring(self._h, session, _vp(frames), _vp(cks), _vp(states)))
        return frames, cks, states

    def queues(self):
        """[4][P][S] int32: every session's InputQueue prediction frame, prediction input, first
        incorrect frame and last requested frame."""
        out = np.zeros((4, self.num_players, self.num_sessions), np.int32)
        _lib.check(self._L.ggrs_p2p_read_queues(self._h, _vp(out)))
        return out

    def stats(self):
        rb = np.zeros(self.num_sessions, np.int32)
        rs = np.zeros(self.num_sessions, np.int64)
        _lib.check(self._L.ggrs_p2p_read_stats(self._h, _vp(rb), _vp(rs)))
        return rb, rs

    def trace(self, first_frame, n):
        out = np.zeros((n, self.num_sessions), np.uint16)
        _lib.check(self._L.ggrs_p2p_read_trace(self._h, first_frame, n, _vp(out)))
        return out

    def timing_reset(self):
        _lib.check(self._L.ggrs_p2p_timing_reset(self._h))

    def timing_stop(self):
        """Record the span's end behind the last launch without waiting (timing_read reports it)."""
        _lib.check(self._L.ggrs_p2p_timing_stop(self._h))

    def timing_read(self):
        ms, n = ctypes.c_float(), ctypes.c_int32()
        _lib.check(self._L.ggrs_p2p_timing_read(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    # ---- desync detection (include/ggrs_amd.h, ggrs_p2p_*_desync*/checksums)
    def set_desync_detection(self, interval):
        """DesyncDetection::On{interval} (0 = Off) for every session; before the first call."""
        _lib.check(self._L.ggrs_p2p_set_desync_detection(self._h, interval))
        self.desync_interval = interval

    def local_checksums(self, frame, out=None):
        """This peer's checksum report of `frame` for every session: numpy [S] u16, or into a
        device tensor `out` (torch, uint16/int16, S elements)."""
        if out is not None and hasattr(out, "data_ptr"):
            _lib.check(self._L.ggrs_p2p_local_checksums(self._h, frame, ctypes.c_void_p(out.data_ptr()), 1))
            return out
        a = np.zeros(self.num_sessions, np.uint16)
        _lib.check(self._L.ggrs_p2p_local_checksums(self._h, frame, _vp(a), 0))
        return a

    def compare_checksums(self, frame, remote):
        """Sessions whose local report of `frame` differs from `remote` ([S] u16 numpy, or a device
        tensor): numpy array of session indices (compared on the device)."""
        words = np.zeros((self.num_sessions + 63) // 64, np.uint64)
        n = ctypes.c_int32()
        if hasattr(remote, "data_ptr"):
            ptr, dev = ctypes.c_void_p(remote.data_ptr()), 1
        else:
            remote = np.ascontiguousarray(remote, np.uint16)
            ptr, dev = _vp(remote), 0
        _lib.check(self._L.ggrs_p2p_compare_checksums(self._h, frame, ptr, dev, _vp(words), ctypes.byref(n)))
        if n.value == 0:
            return np.zeros(0, np.int64)
        bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:self.num_sessions]
        return np.nonzero(bits)[0]

    def debug_desync(self, session, frame):
        """Test hook: session's AdvanceFrame from `frame` flips a bit, on every (re)simulation."""
        _lib.check(self._L.ggrs_p2p_debug_desync(self._h, session, frame))

    def set_sparse_saving(self, on=True):
        """SessionBuilder::with_sparse_saving_mode for every session; before the first call."""
        _lib.check(self._L.ggrs_p2p_set_sparse_saving(self._h, int(bool(on))))
        self.sparse_saving = bool(on)

    # ---- arrival schedules (include/ggrs_amd.h, ggrs_p2p_*arrival*; p2p_sched.hip)
    def set_arrival_schedule(self, on=True):
        """Per-session remote-arrival tables instead of the fixed remote_latency (before the first
        call): each session rolls back to its own earliest misprediction, stops advancing at the
        prediction threshold (p2p_session.rs:393-423), and handles disconnects (:618-655)."""
        _lib.check(self._L.ggrs_p2p_set_arrival_schedule(self._h, int(bool(on))))
        self.arrival_schedule = bool(on)

    def add_arrivals(self, first_call, arrive_upto, events=None):
        """arrive_upto [n][S] int32: the newest remote frame each session's poll delivered at calls
        first_call .. first_call + n - 1; events [n][S] uint8 (bit k: Event::Disconnected for
        remote player k at that call, after its arrivals) or None."""
        a = np.ascontiguousarray(arrive_upto, np.int32)
        if a.ndim != 2 or a.shape[1] != self.num_sessions:
            raise InvalidRequest(-1, f"arrive_upto must be [n][{self.num_sessions}]")
        ev = None
        if events is not None:
            ev = np.ascontiguousarray(events, np.uint8)
            if ev.shape != a.shape:
                raise InvalidRequest(-1, "events must have arrive_upto's shape")
        _lib.check(self._L.ggrs_p2p_add_arrivals(self._h, first_call, a.shape[0], _vp(a), _vp(ev)))

    def add_peer_reports(self, first_call, reports):
        """reports [n][S] int32 (peer_report(player, reporter, frame) or 0): the peers' disconnect
        reports received by calls first_call .. first_call + n - 1 (after their add_arrivals); each
        stands until its reporter disconnects (update_player_disconnects, p2p_session.rs:748-783)."""
        r = np.ascontiguousarray(reports, np.int32)
        if r.ndim != 2 or r.shape[1] != self.num_sessions:
            raise InvalidRequest(-1, f"reports must be [n][{self.num_sessions}]")
        _lib.check(self._L.ggrs_p2p_add_peer_reports(self._h, first_call, r.shape[0], _vp(r)))

    def sessions(self):
        """(frames, skipped, errors) [S] int32 each: every session's current frame, its calls that
        did not advance (prediction threshold), and its error (0, or where the reference panics)."""
        out = [np.zeros(self.num_sessions, np.int32) for _ in range(3)]
        _lib.check(self._L.ggrs_p2p_read_sessions(self._h, *(_vp(a) for a in out)))
        return tuple(out)

    def reports(self, first_call, n_calls):
        """Desync detection under arrival schedules: dict of [n][S] arrays for calls first_call ..
        first_call + n - 1 -- frame (the checksum report check_checksum_send_interval sent, -1
        none), checksum, last_confirmed (the frame compare_local_checksums_against_peers compared
        against) and local_last (the local players' last queued frame after the call)."""
        shape = (n_calls, self.num_sessions)
        out = dict(frame=np.zeros(shape, np.int32), checksum=np.zeros(shape, np.uint16),
                   last_confirmed=np.zeros(shape, np.int32), local_last=np.zeros(shape, np.int32))
        _lib.check(self._L.ggrs_p2p_read_reports(self._h, first_call, n_calls, _vp(out["frame"]),
                                                  _vp(out["checksum"]), _vp(out["last_confirmed"]),
                                                  _vp(out["local_last"])))
        return out

    KERNEL_FORMS = {"default": 0, "unstaged": 1, "lockstep": 2, "flat": 3, "chains": 4, "flat_queues": 5,
                    "canonical": 6}

    def set_unstaged(self, on=True):
        """Calls in lockstep with input rows read from global memory (for comparison)."""
        self.set_kernel_form("unstaged" if on else "default")

    def set_kernel_form(self, form):
        """"default" (flat whenever input rows can be staged, with the block's session rings in LDS
        for the launch where they fit; the chains form instead when the sessions fill at most one
        wave per CU), "flat" (each session's calls as its own step sequence, rings in HBM),
        "lockstep" (calls in lockstep, rows staged in LDS), "unstaged" (lockstep, rows from global
        memory), "chains" (every call as a chain of remote_latency + 1 advances from the confirmed
        state, chains pipelined over lanes; plain launches only), "flat_queues" (the flattened form
        with LDS rings stepping the InputQueue bookkeeping) or "canonical" (the flattened form with
        the rollback decision read off the inputs, the default's choice for plain launches, sparse
        saving included)."""
        _lib.check(self._L.ggrs_p2p_set_unstaged(self._h, self.KERNEL_FORMS[form]))
