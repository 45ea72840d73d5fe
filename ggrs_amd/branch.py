"""Speculative branch rollback (P2P) over the engine's C ABI (include/ggrs_amd.h, ggrs_branch_*).

One BranchEngine holds S sessions x B branches.  Each round: speculate() replays the window from
each session's confirmed trunk with the branch generator's remote inputs (P2PSession::
adjust_gamestate, src/sessions/p2p_session.rs:658-714, with InputQueue prediction replaced), then
confirm() applies the confirmed remote inputs of the trunk frame: the trunk advances, each lane
learns whether its branch survived, and the per-session checksum + survival bits form the report
that a multi-GPU run all-gathers (the ChecksumReport exchange, p2p_session.rs:939-975).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import InvalidRequest


class BranchConfig(ctypes.Structure):
    _fields_ = [
        ("num_sessions", ctypes.c_int32),
        ("num_players", ctypes.c_int32),
        ("remote_mask", ctypes.c_int32),
        ("window", ctypes.c_int32),
        ("branches", ctypes.c_int32),
        ("alphabet", ctypes.c_int32),
        ("input_capacity", ctypes.c_int32),
        ("device", ctypes.c_int32),
    ]


_bound = False


def _bind(L):
    global _bound
    if _bound:
        return
    vp = ctypes.c_void_p
    P = ctypes.POINTER
    L.ggrs_branch_engine_create.argtypes = [P(BranchConfig), P(vp)]
    L.ggrs_branch_engine_destroy.argtypes = [vp]
    L.ggrs_branch_engine_config.argtypes = [vp, P(BranchConfig)]
    L.ggrs_branch_add_inputs.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp]
    L.ggrs_branch_speculate.argtypes = [vp]
    L.ggrs_branch_confirm.argtypes = [vp, vp]
    L.ggrs_branch_report_bytes.argtypes = [vp, P(ctypes.c_int64)]
    L.ggrs_branch_synchronize.argtypes = [vp]
    L.ggrs_branch_trunk_frame.argtypes = [vp, P(ctypes.c_int32)]
    L.ggrs_branch_read_report.argtypes = [vp, vp, vp]
    L.ggrs_branch_read_desync.argtypes = [vp, vp]
    L.ggrs_branch_read_trunk.argtypes = [vp, ctypes.c_int32, vp]
    L.ggrs_branch_read_lane.argtypes = [vp, ctypes.c_int64, ctypes.c_int32, P(ctypes.c_uint16), vp]
    L.ggrs_branch_read_cells.argtypes = [vp, ctypes.c_int32, vp, vp]
    L.ggrs_branch_timing_reset.argtypes = [vp]
    L.ggrs_branch_timing_stop.argtypes = [vp]
    L.ggrs_branch_timing_read.argtypes = [vp, P(ctypes.c_float), P(ctypes.c_int32)]
    L.ggrs_branch_rounds.argtypes = [vp, ctypes.c_int32]
    L.ggrs_branch_set_round_launches.argtypes = [vp, ctypes.c_int32]
    L.ggrs_branch_set_stream.argtypes = [vp, vp]
    L.ggrs_branch_use_own_stream.argtypes = [vp]
    L.ggrs_branch_round.argtypes = [vp, vp]
    i32 = ctypes.c_int32
    L.ggrs_branch_compare_peer.argtypes = [vp, vp, i32, i32, i32, i32, vp, vp]
    L.ggrs_branch_compare_peer_rows.argtypes = [vp, vp, i32, i32, i32, i32, i32, i32, vp, vp]
    L.ggrs_branch_rounds_reports.argtypes = [vp, i32, vp]
    for name in _lib.EXPORTS:
        if name.startswith("ggrs_branch_"):
            getattr(L, name).restype = ctypes.c_int
    _bound = True


def _vp(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class BranchEngine:
    def __init__(self, num_sessions, num_players=2, remote_mask=0b10, window=4, branches=1,
                 alphabet=16, input_capacity=0, device=0):
        self._L = _lib.lib()
        _bind(self._L)
        cfg = BranchConfig(num_sessions, num_players, remote_mask, window, branches, alphabet,
                           input_capacity, device)
        h = ctypes.c_void_p()
        _lib.check(self._L.ggrs_branch_engine_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self.num_sessions, self.num_players = num_sessions, num_players
        self.remote_mask, self.window, self.branches, self.alphabet = remote_mask, window, branches, alphabet
        self.num_lanes = num_sessions * branches
        self.ring_len = window + 1
        self.state_bytes = 36 + 20 * num_players
        n = ctypes.c_int64()
        _lib.check(self._L.ggrs_branch_report_bytes(self._h, ctypes.byref(n)))
        self.report_bytes = n.value
        self.report_ck_bytes = (2 * num_sessions + 7) & ~7
        self.report_words = (self.num_lanes + 63) // 64

    def close(self):
        if getattr(self, "_h", None):
            self._L.ggrs_branch_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_inputs(self, first_frame, inputs):
        a = np.ascontiguousarray(inputs, np.uint8)
        if a.ndim != 3 or a.shape[1:] != (self.num_sessions, self.num_players):
            raise InvalidRequest(-1, f"inputs must be [n][{self.num_sessions}][{self.num_players}]")
        _lib.check(self._L.ggrs_branch_add_inputs(self._h, first_frame, a.shape[0], _vp(a)))

    def speculate(self):
        _lib.check(self._L.ggrs_branch_speculate(self._h))

    def confirm(self, report_device_ptr=None):
        ptr = ctypes.c_void_p(report_device_ptr) if report_device_ptr else None
        _lib.check(self._L.ggrs_branch_confirm(self._h, ptr))

    def set_stream(self, stream_ptr):
        """Enqueue all work on this hipStream_t (an int handle, e.g. torch.cuda.current_stream()
        .cuda_stream; 0 or None = HIP's null stream, which is what torch's default stream reports).
        Work queued before the switch is ordered before work queued after it."""
        _lib.check(self._L.ggrs_branch_set_stream(self._h, ctypes.c_void_p(stream_ptr) if stream_ptr else None))

    def use_own_stream(self):
        """Back to the engine's own non-blocking stream (the one it was created with)."""
        _lib.check(self._L.ggrs_branch_use_own_stream(self._h))

    def confirm_to_tensor(self, t):
        """confirm() with the round's report written into torch uint8 tensor `t`: a device tensor
        receives it on the engine's stream (no host sync); a CPU tensor through a host read."""
        if t.is_cuda:
            self.confirm(t.data_ptr())
            return
        self.confirm()
        self._report_into(t)

    def round_to_tensor(self, t):
        """One round (speculate + confirm) as one launch, its report written into device uint8
        tensor `t` by the kernel itself (ggrs_branch_round); a CPU tensor through a host read."""
        if t.is_cuda:
            _lib.check(self._L.ggrs_branch_round(self._h, ctypes.c_void_p(t.data_ptr())))
            return
        _lib.check(self._L.ggrs_branch_round(self._h, None))
        self._report_into(t)

    def rounds_to_tensor(self, t, n):
        """n rounds in one launch, round r's report written into row r of device uint8 tensor
        `t` ([>= n][report_bytes], contiguous) by the kernel (ggrs_branch_rounds_reports)."""
        if not t.is_cuda or not t.is_contiguous() or t.shape[-1] != self.report_bytes or t.shape[0] < n:
            raise ValueError("rounds_to_tensor needs a contiguous device tensor [>= n][report_bytes]")
        _lib.check(self._L.ggrs_branch_rounds_reports(self._h, n, ctypes.c_void_p(t.data_ptr())))

    def compare_peer(self, gathered, rank, peer, frame, count, first_frame):
        """Queue the peer checksum comparison of one all-gathered report block (device tensors:
        gathered [world][report_bytes] u8, count and first_frame int64 scalars)."""
        _lib.check(self._L.ggrs_branch_compare_peer(
            self._h, ctypes.c_void_p(gathered.data_ptr()), gathered.shape[0], rank, peer, frame,
            ctypes.c_void_p(count.data_ptr()), ctypes.c_void_p(first_frame.data_ptr())))

    def compare_peer_rows(self, gathered, n_rows, rank, peer, first_frame, count, first):
        """The same over a batch: gathered [world][rows][report_bytes] u8 (device), rows 0 ..
        n_rows-1 compared, row k = frame first_frame + k; one launch."""
        _lib.check(self._L.ggrs_branch_compare_peer_rows(
            self._h, ctypes.c_void_p(gathered.data_ptr()), gathered.shape[0], gathered.shape[1], n_rows, rank, peer,
            first_frame, ctypes.c_void_p(count.data_ptr()), ctypes.c_void_p(first.data_ptr())))

    def _report_into(self, t):
        ck, bits = self.report()
        raw = np.zeros(self.report_bytes, np.uint8)
        raw[:2 * self.num_sessions] = ck.view(np.uint8)
        raw[self.report_ck_bytes:self.report_ck_bytes + 8 * self.report_words] = bits.view(np.uint8)
        import torch
        t.copy_(torch.from_numpy(raw))

    def rounds(self, n):
        """n rounds of speculate + confirm from native code (no report copy): one launch by
        default, or 2 n back-to-back launches after set_round_launches(True)."""
        _lib.check(self._L.ggrs_branch_rounds(self._h, n))

    def set_round_launches(self, on=True):
        _lib.check(self._L.ggrs_branch_set_round_launches(self._h, int(bool(on))))

    ROUND_FORMS = {"fused": 0, "per_round": 1, "full": 2}

    def set_round_form(self, form):
        """rounds(): "fused" (one launch; prefix-shared when the enumerated player is the only
        remote one), "per_round" (2 n launches of speculate / confirm) or "full" (one launch, every
        lane replaying and saving its whole window)."""
        _lib.check(self._L.ggrs_branch_set_round_launches(self._h, self.ROUND_FORMS[form]))

    def synchronize(self):
        _lib.check(self._L.ggrs_branch_synchronize(self._h))

    def trunk_frame(self):
        v = ctypes.c_int32()
        _lib.check(self._L.ggrs_branch_trunk_frame(self._h, ctypes.byref(v)))
        return v.value

    def report(self):
        ck = np.zeros(self.num_sessions, np.uint16)
        bits = np.zeros(self.report_words, np.uint64)
        _lib.check(self._L.ggrs_branch_read_report(self._h, _vp(ck), _vp(bits)))
        return ck, bits

    def survivors(self):
        _, bits = self.report()
        return unpack_bits(bits, self.num_lanes)

    def desync(self):
        out = np.zeros(self.num_sessions, np.int32)
        _lib.check(self._L.ggrs_branch_read_desync(self._h, _vp(out)))
        return out

    def trunk(self, session):
        out = np.zeros(self.state_bytes, np.uint8)
        _lib.check(self._L.ggrs_branch_read_trunk(self._h, session, _vp(out)))
        return out

    def lane_state(self, lane, frame):
        out = np.zeros(self.state_bytes, np.uint8)
        ck = ctypes.c_uint16()
        _lib.check(self._L.ggrs_branch_read_lane(self._h, lane, frame, ctypes.byref(ck), _vp(out)))
        return int(ck.value), out

    def cells(self, frame, states=True):
        """lane_state for every lane: (checksums [num_lanes], states [num_lanes][sb] or None)."""
        ck = np.zeros(self.num_lanes, np.uint16)
        st = np.zeros((self.num_lanes, self.state_bytes), np.uint8) if states else None
        _lib.check(self._L.ggrs_branch_read_cells(self._h, frame, _vp(ck), _vp(st) if states else None))
        return ck, st

    def timing_reset(self):
        _lib.check(self._L.ggrs_branch_timing_reset(self._h))

    def timing_stop(self):
        """Record the span's end behind the last launch without waiting (timing_read reports it)."""
        _lib.check(self._L.ggrs_branch_timing_stop(self._h))

    def timing_read(self):
        ms, n = ctypes.c_float(), ctypes.c_int32()
        _lib.check(self._L.ggrs_branch_timing_read(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    # ---- the branch generator, restated on the host for checking and scheduling
    def assumed_remote(self, branch, k, last_confirmed):
        """Remote inputs lane `branch` plays on speculated frame k, per player (None = local)."""
        out = []
        first_remote = next(q for q in range(self.num_players) if self.remote_mask >> q & 1)
        E = 0
        v = 1
        while v < self.branches:
            v *= self.alphabet
            E += 1
        for q in range(self.num_players):
            if not self.remote_mask >> q & 1:
                out.append(None)
            elif q == first_remote and self.branches > 1:
                kk = min(k, E - 1)
                out.append((branch // self.alphabet ** kk) % self.alphabet)
            else:
                out.append(int(last_confirmed[q]))
        return out


def unpack_bits(words, n):
    bits = np.unpackbits(np.ascontiguousarray(words, "<u8").view(np.uint8), bitorder="little")
    return bits[:n].astype(bool)
