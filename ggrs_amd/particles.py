"""Config-5 particle world: the SyncTest program on ~1 MB states, over the C ABI
(include/ggrs_amd.h, ggrs_particle_*).  Game definition: ggrs_amd/csrc/particles.h."""
import ctypes

import numpy as np

from . import _lib
from ._lib import InvalidRequest, LANE_MISMATCH


class ParticleConfig(ctypes.Structure):
    _fields_ = [
        ("num_sessions", ctypes.c_int32),
        ("num_entities", ctypes.c_int32),
        ("num_players", ctypes.c_int32),
        ("max_prediction", ctypes.c_int32),
        ("check_distance", ctypes.c_int32),
        ("input_capacity", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("first_session_id", ctypes.c_int32),
    ]


_bound = False


def _bind(L):
    global _bound
    if _bound:
        return
    vp, P = ctypes.c_void_p, ctypes.POINTER
    L.ggrs_particle_engine_create.argtypes = [P(ParticleConfig), P(vp)]
    L.ggrs_particle_engine_destroy.argtypes = [vp]
    L.ggrs_particle_add_local_inputs.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp]
    L.ggrs_particle_synctest_advance_frames.argtypes = [vp, ctypes.c_int32]
    L.ggrs_particle_synchronize.argtypes = [vp]
    L.ggrs_particle_current_frame.argtypes = [vp, P(ctypes.c_int32)]
    L.ggrs_particle_read_mismatches.argtypes = [vp, vp, vp, vp]
    L.ggrs_particle_read_state.argtypes = [vp, ctypes.c_int32, vp]
    L.ggrs_particle_read_saved.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, P(ctypes.c_uint16), vp]
    L.ggrs_particle_debug_corrupt_on_load.argtypes = [vp, ctypes.c_int32, ctypes.c_int32]
    L.ggrs_particle_timing_reset.argtypes = [vp]
    L.ggrs_particle_timing_stop.argtypes = [vp]
    L.ggrs_particle_timing_read.argtypes = [vp, P(ctypes.c_float), P(ctypes.c_int32)]
    for name in _lib.EXPORTS:
        if name.startswith("ggrs_particle_"):
            getattr(L, name).restype = ctypes.c_int
    _bound = True


def _vp(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class ParticleEngine:
    def __init__(self, num_sessions, num_entities=10000, num_players=2, max_prediction=17,
                 check_distance=16, input_capacity=0, device=0, first_session_id=0):
        self._L = _lib.lib()
        _bind(self._L)
        cfg = ParticleConfig(num_sessions, num_entities, num_players, max_prediction, check_distance,
                             input_capacity, device, first_session_id)
        h = ctypes.c_void_p()
        _lib.check(self._L.ggrs_particle_engine_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self.num_sessions, self.num_entities, self.num_players = num_sessions, num_entities, num_players
        self.check_distance = check_distance
        self.state_bytes = 4 + 100 * num_entities
        self._added = 0

    def close(self):
        if getattr(self, "_h", None):
            self._L.ggrs_particle_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_local_inputs(self, inputs):
        a = np.ascontiguousarray(inputs, np.uint8)
        if a.ndim != 3 or a.shape[1:] != (self.num_sessions, self.num_players):
            raise InvalidRequest(-1, f"inputs must be [n][{self.num_sessions}][{self.num_players}]")
        _lib.check(self._L.ggrs_particle_add_local_inputs(self._h, self._added, a.shape[0], _vp(a)))
        self._added += a.shape[0]

    def synctest_advance_frames(self, n):
        _lib.check(self._L.ggrs_particle_synctest_advance_frames(self._h, n))

    def synchronize(self):
        _lib.check(self._L.ggrs_particle_synchronize(self._h))

    def current_frame(self):
        v = ctypes.c_int32()
        _lib.check(self._L.ggrs_particle_current_frame(self._h, ctypes.byref(v)))
        return v.value

    def mismatches(self):
        n = self.num_sessions
        st, mf, mm = np.zeros(n, np.int32), np.zeros(n, np.int32), np.zeros(n, np.uint64)
        _lib.check(self._L.ggrs_particle_read_mismatches(self._h, _vp(st), _vp(mf), _vp(mm)))
        return st, mf, mm

    def state(self, session):
        out = np.zeros(self.state_bytes, np.uint8)
        _lib.check(self._L.ggrs_particle_read_state(self._h, session, _vp(out)))
        return out

    def saved(self, session, frame, with_state=True):
        ck = ctypes.c_uint16()
        out = np.zeros(self.state_bytes, np.uint8) if with_state else None
        _lib.check(self._L.ggrs_particle_read_saved(self._h, session, frame, ctypes.byref(ck), _vp(out)))
        return int(ck.value), out

    def corrupt_on_load(self, session, frame):
        _lib.check(self._L.ggrs_particle_debug_corrupt_on_load(self._h, session, frame))

    def timing_reset(self):
        _lib.check(self._L.ggrs_particle_timing_reset(self._h))

    def timing_stop(self):
        """Record the span's end behind the last launch without waiting (timing_read reports it)."""
        _lib.check(self._L.ggrs_particle_timing_stop(self._h))

    def timing_read(self):
        ms, n = ctypes.c_float(), ctypes.c_int32()
        _lib.check(self._L.ggrs_particle_timing_read(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value
