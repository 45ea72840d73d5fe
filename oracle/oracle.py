"""ctypes binding of the C oracle (oracle/ggrs_oracle.c).  TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker
or the CPU baseline.  The product (ggrs_amd/) never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libggrs_oracle.so")

REQ_SAVE, REQ_LOAD, REQ_ADVANCE = 0, 1, 2
MODEL_UNIFORM, MODEL_HELD = 0, 1


class SyncTestCfg(ctypes.Structure):
    _fields_ = [
        ("num_players", ctypes.c_int32),
        ("max_prediction", ctypes.c_int32),
        ("check_distance", ctypes.c_int32),
        ("input_delay", ctypes.c_int32),
        ("predictor", ctypes.c_int32),
        ("random_checksums", ctypes.c_int32),
        ("rng_seed", ctypes.c_uint64),
        ("corrupt_frame", ctypes.c_int32),
        ("pad_", ctypes.c_int32),
    ]


class SyncTestResult(ctypes.Structure):
    _fields_ = [
        ("status", ctypes.c_int32),
        ("frames_done", ctypes.c_int32),
        ("mismatch_frame", ctypes.c_int32),
        ("mismatch_mask", ctypes.c_uint64),
        ("n_load", ctypes.c_int64),
        ("n_save", ctypes.c_int64),
        ("n_advance", ctypes.c_int64),
        ("n_resim", ctypes.c_int64),
    ]


class P2PCfg(ctypes.Structure):
    _fields_ = [
        ("num_players", ctypes.c_int32),
        ("max_prediction", ctypes.c_int32),
        ("input_delay", ctypes.c_int32),
        ("latency", ctypes.c_int32),
        ("local_mask", ctypes.c_int32),
        ("predictor", ctypes.c_int32),
        ("sparse_saving", ctypes.c_int32),
    ]


class P2PResult(ctypes.Structure):
    _fields_ = [
        ("status", ctypes.c_int32),
        ("frames_done", ctypes.c_int32),
        ("rollbacks", ctypes.c_int64),
        ("resim", ctypes.c_int64),
        ("n_load", ctypes.c_int64),
        ("n_save", ctypes.c_int64),
        ("n_advance", ctypes.c_int64),
    ]


def build():
    """Compile the oracle with its Makefile (gcc; seconds)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER
        u8p, u16p, i32p = P(ctypes.c_uint8), P(ctypes.c_uint16), P(ctypes.c_int32)
        L.oracle_synctest_run.argtypes = [P(SyncTestCfg), ctypes.c_int32, u8p, u16p, u8p,
                                          ctypes.c_int64, i32p, u8p, i32p, u16p, u8p,
                                          P(SyncTestResult)]
        L.oracle_synctest_run.restype = ctypes.c_int
        L.oracle_gen_inputs.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64,
                                        ctypes.c_int, u8p]
        L.oracle_fletcher16.argtypes = [u8p, ctypes.c_size_t]
        L.oracle_fletcher16.restype = ctypes.c_uint16
        L.oracle_state_new_bytes.argtypes = [ctypes.c_int32, u8p]
        L.oracle_state_advance_bytes.argtypes = [u8p, u8p, u8p, u8p]
        for fn in ("oracle_sinf", "oracle_cosf"):
            getattr(L, fn).argtypes = [ctypes.c_float]
            getattr(L, fn).restype = ctypes.c_float
        L.oracle_sincos_digest.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int]
        L.oracle_sincos_digest.restype = ctypes.c_uint64
        L.oracle_sincos_range.argtypes = [ctypes.c_uint32, ctypes.c_uint32, P(ctypes.c_uint32),
                                          P(ctypes.c_uint32)]
        L.oracle_synctest_bench.argtypes = [P(SyncTestCfg), ctypes.c_int, ctypes.c_uint64,
                                            ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, u16p,
                                            P(ctypes.c_double)]
        L.oracle_synctest_bench.restype = ctypes.c_int64
        L.oracle_p2p_replay.argtypes = [ctypes.c_int32, u8p, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32, u8p, u8p, u8p, u16p, u8p]
        L.oracle_p2p_replay.restype = ctypes.c_int
        i32 = ctypes.c_int32
        L.oracle_branch_bench.argtypes = [i32, i32, i32, i32, ctypes.c_uint32, i32, i32, i32, i32,
                                          ctypes.c_uint64, P(ctypes.c_double), u16p]
        L.oracle_branch_bench.restype = ctypes.c_int64
        L.oracle_particles_synctest_run.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                     ctypes.c_int32, ctypes.c_uint64, ctypes.c_int32,
                                                     u8p, ctypes.c_int32, u16p, u8p, i32p, u16p, u8p,
                                                     P(SyncTestResult)]
        L.oracle_particles_synctest_run.restype = ctypes.c_int
        L.oracle_input_queue_sequence.argtypes = [ctypes.c_int32, ctypes.c_int32, i32p, u8p,
                                                  ctypes.c_int, i32p, u8p, i32p]
        L.oracle_p2p_run.argtypes = [P(P2PCfg), ctypes.c_int32, u8p, u16p, i32p, u8p, ctypes.c_int64,
                                     i32p, u8p, i32p, u16p, u8p, P(P2PResult)]
        L.oracle_p2p_run.restype = ctypes.c_int
        i64p = P(ctypes.c_int64)
        L.oracle_p2p_stream.argtypes = [P(P2PCfg), ctypes.c_int32, u8p, i32p, ctypes.c_int64, i64p, i32p, i32p,
                                        u8p, u8p, P(P2PResult)]
        L.oracle_p2p_stream.restype = ctypes.c_int
        L.oracle_handler_run.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, i32p, i32p, u8p, u8p,
                                         u16p, u8p, i32p, u16p, u8p]
        L.oracle_handler_run.restype = ctypes.c_int
        L.oracle_p2p_desync_pair_run.argtypes = [
            ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, i32p, ctypes.c_int32, ctypes.c_int32,
            ctypes.c_int32, u8p, ctypes.c_int32, ctypes.c_int32, i32p, u16p, ctypes.c_int32, i32p, i32p,
            i32p, u16p, u16p, i32p, u16p]
        L.oracle_p2p_desync_pair_run.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct)) if a is not None else None


def state_bytes(p):
    return 36 + 20 * p


def gen_inputs(seed, frames, players, model=MODEL_UNIFORM):
    out = np.zeros((frames, players), np.uint8)
    lib().oracle_gen_inputs(seed, frames, players, model, _ptr(out, ctypes.c_uint8))
    return out


def session_seed(session, base=0x6767525300000000):
    return (base + session) & 0xFFFFFFFFFFFFFFFF


def fletcher16(b):
    a = np.frombuffer(bytes(b), np.uint8).copy()
    return int(lib().oracle_fletcher16(_ptr(a, ctypes.c_uint8), a.size))


def state_new(p):
    out = np.zeros(state_bytes(p), np.uint8)
    lib().oracle_state_new_bytes(p, _ptr(out, ctypes.c_uint8))
    return out


def state_advance(state, inputs, status=None):
    state = np.ascontiguousarray(state, np.uint8)
    p = (state.size - 36) // 20
    inp = np.ascontiguousarray(inputs, np.uint8)
    st = np.zeros(p, np.uint8) if status is None else np.ascontiguousarray(status, np.uint8)
    out = np.zeros_like(state)
    lib().oracle_state_advance_bytes(_ptr(state, ctypes.c_uint8), _ptr(inp, ctypes.c_uint8),
                                     _ptr(st, ctypes.c_uint8), _ptr(out, ctypes.c_uint8))
    return out


def synctest_run(inputs, num_players=2, max_prediction=8, check_distance=2, input_delay=0,
                 random_checksums=False, rng_seed=1, req_cap=None, corrupt_frame=-1):
    """Run the restated SyncTest loop; returns a dict of numpy arrays and the result struct."""
    inputs = np.ascontiguousarray(inputs, np.uint8).reshape(-1, num_players)
    frames = inputs.shape[0]
    R = max_prediction + 1
    sb = state_bytes(num_players)
    cfg = SyncTestCfg(num_players, max_prediction, check_distance, input_delay, 0,
                      1 if random_checksums else 0, rng_seed, corrupt_frame, 0)
    res = SyncTestResult()
    req_cap = req_cap if req_cap is not None else frames * (2 * check_distance + 3)
    out = dict(
        cksum=np.zeros(frames, np.uint16),
        req=np.zeros(max(req_cap, 1), np.uint8),
        req_len=np.zeros(frames, np.int32),
        final_state=np.zeros(sb, np.uint8),
        ring_frames=np.zeros(R, np.int32),
        ring_cksums=np.zeros(R, np.uint16),
        ring_states=np.zeros((R, sb), np.uint8),
    )
    rc = lib().oracle_synctest_run(
        ctypes.byref(cfg), frames, _ptr(inputs, ctypes.c_uint8), _ptr(out["cksum"], ctypes.c_uint16),
        _ptr(out["req"], ctypes.c_uint8), req_cap, _ptr(out["req_len"], ctypes.c_int32),
        _ptr(out["final_state"], ctypes.c_uint8), _ptr(out["ring_frames"], ctypes.c_int32),
        _ptr(out["ring_cksums"], ctypes.c_uint16), _ptr(out["ring_states"], ctypes.c_uint8),
        ctypes.byref(res))
    out["rc"] = rc
    out["result"] = res
    return out


def input_queue_sequence(delay, frames, inputs, read=True):
    """Add (frame, input) pairs to one InputQueue; returns (add_input results, input(frame)
    read back after each add, queue length after each add)."""
    fr = np.ascontiguousarray(frames, np.int32)
    ins = np.ascontiguousarray(inputs, np.uint8)
    n = fr.size
    added, got, length = np.zeros(n, np.int32), np.zeros(n, np.uint8), np.zeros(n, np.int32)
    lib().oracle_input_queue_sequence(delay, n, _ptr(fr, ctypes.c_int32), _ptr(ins, ctypes.c_uint8),
                                      1 if read else 0, _ptr(added, ctypes.c_int32),
                                      _ptr(got, ctypes.c_uint8), _ptr(length, ctypes.c_int32))
    return added, got, length


def p2p_replay(state, load_frame, inputs, max_prediction=None, status=None):
    """P2PSession::adjust_gamestate from `state` (the cell of load_frame) over len(inputs) frames
    + the save of the current frame; returns (saved states [count][sb], checksums [count], final)."""
    state = np.ascontiguousarray(state, np.uint8)
    P = (state.size - 36) // 20
    inp = np.ascontiguousarray(inputs, np.uint8).reshape(-1, P)
    count = inp.shape[0]
    st = None if status is None else np.ascontiguousarray(status, np.uint8).reshape(-1, P)
    mp = max_prediction or count
    states = np.zeros((count, state.size), np.uint8)
    cks = np.zeros(count, np.uint16)
    final = np.zeros(state.size, np.uint8)
    rc = lib().oracle_p2p_replay(P, _ptr(state, ctypes.c_uint8), load_frame, count, mp,
                                 _ptr(inp, ctypes.c_uint8), _ptr(st, ctypes.c_uint8),
                                 _ptr(states, ctypes.c_uint8), _ptr(cks, ctypes.c_uint16),
                                 _ptr(final, ctypes.c_uint8))
    if rc != 0:
        raise ValueError("bad p2p replay arguments")
    return states, cks, final


def p2p_run(inputs, num_players=2, local_mask=0b01, input_delay=0, max_prediction=8, latency=4,
            predictor=0, req_cap=0, sparse_saving=False):
    """One peer's P2P session over len(inputs) calls (oracle_p2p_run in ggrs_oracle.c):
    inputs[g] = local add_local_input of call g / remote input of frame g."""
    inputs = np.ascontiguousarray(inputs, np.uint8).reshape(-1, num_players)
    frames = inputs.shape[0]
    R = max_prediction + 1
    sb = state_bytes(num_players)
    cfg = P2PCfg(num_players, max_prediction, input_delay, latency, local_mask, predictor, int(sparse_saving))
    res = P2PResult()
    out = dict(ck_trace=np.zeros(frames, np.uint16), rb_frame=np.zeros(frames, np.int32),
               req_trace=np.zeros(max(req_cap, 1), np.uint8), req_len=np.zeros(frames, np.int32),
               final_state=np.zeros(sb, np.uint8), ring_frames=np.zeros(R, np.int32),
               ring_cksums=np.zeros(R, np.uint16), ring_states=np.zeros((R, sb), np.uint8))
    rc = lib().oracle_p2p_run(
        ctypes.byref(cfg), frames, _ptr(inputs, ctypes.c_uint8), _ptr(out["ck_trace"], ctypes.c_uint16),
        _ptr(out["rb_frame"], ctypes.c_int32), _ptr(out["req_trace"], ctypes.c_uint8), req_cap,
        _ptr(out["req_len"], ctypes.c_int32), _ptr(out["final_state"], ctypes.c_uint8),
        _ptr(out["ring_frames"], ctypes.c_int32), _ptr(out["ring_cksums"], ctypes.c_uint16),
        _ptr(out["ring_states"], ctypes.c_uint8), ctypes.byref(res))
    out["rc"] = rc
    out["result"] = res
    return out


def jitter_schedule(frames, max_prediction, seed, max_lag=None):
    """arrive_upto[f] for oracle_p2p_stream: the newest remote frame delivered by call f, from a
    random per-call lag in [1, max_lag] (default max_prediction - 1), kept non-decreasing, so
    inputs arrive in bursts of differing size."""
    rng = np.random.default_rng(seed)
    max_lag = max_lag or max_prediction - 1
    lag = rng.integers(1, max_lag + 1, frames)
    upto = np.maximum.accumulate(np.arange(frames) - lag)
    return upto.astype(np.int32)


def p2p_stream(inputs, arrive_upto, num_players=2, local_mask=0b01, input_delay=0, max_prediction=8,
               predictor=0, sparse_saving=False):
    """The request lists one P2P session emits per call under a jittery network
    (oracle_p2p_stream): dict with call_off [calls + 1] and per request kind, frame, inputs [P],
    status [P]."""
    inputs = np.ascontiguousarray(inputs, np.uint8).reshape(-1, num_players)
    frames = inputs.shape[0]
    upto = np.ascontiguousarray(arrive_upto, np.int32)
    cap = frames * (4 * max_prediction + 8)
    cfg = P2PCfg(num_players, max_prediction, input_delay, 1, local_mask, predictor, int(sparse_saving))
    res = P2PResult()
    off = np.zeros(frames + 1, np.int64)
    kind, frame = np.zeros(cap, np.int32), np.zeros(cap, np.int32)
    inp, st = np.zeros((cap, num_players), np.uint8), np.zeros((cap, num_players), np.uint8)
    rc = lib().oracle_p2p_stream(ctypes.byref(cfg), frames, _ptr(inputs, ctypes.c_uint8), _ptr(upto, ctypes.c_int32),
                                 cap, _ptr(off, ctypes.c_int64), _ptr(kind, ctypes.c_int32),
                                 _ptr(frame, ctypes.c_int32), _ptr(inp, ctypes.c_uint8), _ptr(st, ctypes.c_uint8),
                                 ctypes.byref(res))
    n = int(off[res.frames_done])
    return dict(rc=rc, result=res, calls=res.frames_done, call_off=off[:res.frames_done + 1], kind=kind[:n],
                frame=frame[:n], inputs=inp[:n], status=st[:n])


def stall_schedule(calls, max_prediction, seed, max_lag=None, stall_every=40, stall_len=None):
    """arrive_upto[c] for oracle_p2p_sched_run: jittered lags in [1, max_lag] (default max_prediction
    - 1) with, every ~stall_every calls, a network stall of stall_len calls (default max_prediction
    + 4) in which nothing arrives -- so sessions hit the prediction threshold and skip calls, then
    the burst arrives at once (a rollback as deep as the window).  Non-decreasing, <= c."""
    rng = np.random.default_rng(seed)
    max_lag = max_lag or max(1, max_prediction - 1)
    stall_len = stall_len or max_prediction + 4
    lag = rng.integers(1, max_lag + 1, calls)
    upto = np.arange(calls) - lag
    c = int(rng.integers(stall_every // 2, stall_every + 1))
    while c < calls:
        hold = upto[c - 1] if c > 0 else -1
        upto[c:c + stall_len] = np.minimum(upto[c:c + stall_len], hold)
        c += stall_len + int(rng.integers(stall_every // 2, stall_every + 1))
    upto = np.maximum.accumulate(np.maximum(upto, -1))
    return upto.astype(np.int32)


def peer_report(player, reporter, frame):
    """GGRS_PEER_REPORT: remote player `reporter`'s endpoint reports remote player `player`
    disconnected with last frame `frame` (a reports[] entry of p2p_sched_run / the device engine)."""
    return 16 | player | reporter << 2 | (frame + 1) << 5


def p2p_sched_run(inputs, arrive_upto, events=None, num_players=2, local_mask=0b01, input_delay=0,
                  max_prediction=8, predictor=0, sparse_saving=False, reports=None):
    """One peer's P2P session under an arrival schedule, with the prediction threshold and
    disconnects (oracle_p2p_sched_run): inputs[c] = local add_local_input of call c / remote input of
    frame c; arrive_upto[c] = newest remote frame delivered by call c; events[c] bit k = player k's
    Event::Disconnected at call c; reports[c] a peer's disconnect report (peer_report, 0 none);
    max_prediction 0 is lockstep mode.  Returns rc, result, per-call advanced / rb_frame / ck_trace,
    the final state and the ring; current_frame and skips derived from the counts."""
    inputs = np.ascontiguousarray(inputs, np.uint8).reshape(-1, num_players)
    calls = inputs.shape[0]
    upto = np.ascontiguousarray(arrive_upto, np.int32)
    assert upto.shape[0] >= calls
    ev = None if events is None else np.ascontiguousarray(events, np.uint8)
    rp = None if reports is None else np.ascontiguousarray(reports, np.int32)
    R, sb = max_prediction + 1, state_bytes(num_players)
    cfg = P2PCfg(num_players, max_prediction, input_delay, 1, local_mask, predictor, int(sparse_saving))
    res = P2PResult()
    out = dict(advanced=np.zeros(calls, np.uint8), rb_frame=np.zeros(calls, np.int32),
               ck_trace=np.zeros(calls, np.uint16), final_state=np.zeros(sb, np.uint8),
               ring_frames=np.zeros(R, np.int32), ring_cksums=np.zeros(R, np.uint16),
               ring_states=np.zeros((R, sb), np.uint8))
    L = lib()
    if not getattr(L, "_sched_bound", False):
        P = ctypes.POINTER
        u8p, u16p, i32p = P(ctypes.c_uint8), P(ctypes.c_uint16), P(ctypes.c_int32)
        L.oracle_p2p_sched_run.argtypes = [P(P2PCfg), ctypes.c_int32, u8p, i32p, u8p, i32p, u8p, i32p, u16p, u8p,
                                           i32p, u16p, u8p, P(P2PResult)]
        L.oracle_p2p_sched_run.restype = ctypes.c_int
        L._sched_bound = True
    rc = L.oracle_p2p_sched_run(
        ctypes.byref(cfg), calls, _ptr(inputs, ctypes.c_uint8), _ptr(upto, ctypes.c_int32), _ptr(ev, ctypes.c_uint8),
        _ptr(rp, ctypes.c_int32), _ptr(out["advanced"], ctypes.c_uint8), _ptr(out["rb_frame"], ctypes.c_int32),
        _ptr(out["ck_trace"], ctypes.c_uint16), _ptr(out["final_state"], ctypes.c_uint8),
        _ptr(out["ring_frames"], ctypes.c_int32), _ptr(out["ring_cksums"], ctypes.c_uint16),
        _ptr(out["ring_states"], ctypes.c_uint8), ctypes.byref(res))
    out["rc"] = rc
    out["result"] = res
    out["current_frame"] = int(res.n_advance - res.resim)
    out["skips"] = int(res.frames_done - out["current_frame"])
    return out


def handler_run(kind, frame, inputs, status=None, num_players=2, max_prediction=8):
    """Game::handle_requests over one lane's request stream (oracle_handler_run): dict with rc
    (0, or -(1 + k) at the request that would panic), the checksum of every Save in order, the
    final state and the ring."""
    kind = np.ascontiguousarray(kind, np.int32)
    frame = np.ascontiguousarray(frame, np.int32)
    n = kind.shape[0]
    inputs = np.ascontiguousarray(inputs, np.uint8).reshape(n, num_players)
    status = None if status is None else np.ascontiguousarray(status, np.uint8).reshape(n, num_players)
    R, sb = max_prediction + 1, state_bytes(num_players)
    out = dict(save_cks=np.zeros(max(1, int((kind == 0).sum())), np.uint16), final_state=np.zeros(sb, np.uint8),
               ring_frames=np.zeros(R, np.int32), ring_cksums=np.zeros(R, np.uint16),
               ring_states=np.zeros((R, sb), np.uint8))
    out["rc"] = lib().oracle_handler_run(num_players, max_prediction, n, _ptr(kind, ctypes.c_int32),
                                         _ptr(frame, ctypes.c_int32), _ptr(inputs, ctypes.c_uint8),
                                         _ptr(status, ctypes.c_uint8), _ptr(out["save_cks"], ctypes.c_uint16),
                                         _ptr(out["final_state"], ctypes.c_uint8),
                                         _ptr(out["ring_frames"], ctypes.c_int32),
                                         _ptr(out["ring_cksums"], ctypes.c_uint16),
                                         _ptr(out["ring_states"], ctypes.c_uint8))
    out["save_cks"] = out["save_cks"][:int((kind == 0).sum())]
    return out


def p2p_desync_pair_run(inputs, num_players=2, max_prediction=8, latency=2, local_masks=(0b01, 0b10),
                        predictor=0, interval=10, desync_peer=-1, desync_frame=-1, ev_cap=4096):
    """Both peers of one match with DesyncDetection::On{interval} (oracle_p2p_desync_pair_run):
    per peer and call the checksum report sent, and the DesyncDetected events raised as
    (peer, call, frame, local_checksum, remote_checksum), in call order."""
    inputs = np.ascontiguousarray(inputs, np.uint8).reshape(-1, num_players)
    frames = inputs.shape[0]
    masks = np.array(local_masks, np.int32)
    sent_frame = np.full((2, frames), -1, np.int32)
    sent_cs = np.zeros((2, frames), np.uint16)
    ev = {k: np.zeros(ev_cap, t) for k, t in (("peer", np.int32), ("call", np.int32), ("frame", np.int32),
                                              ("local", np.uint16), ("remote", np.uint16))}
    n_ev = ctypes.c_int32(0)
    trace = np.zeros((2, frames), np.uint16)
    rc = lib().oracle_p2p_desync_pair_run(
        num_players, max_prediction, latency, _ptr(masks, ctypes.c_int32), predictor, interval, frames,
        _ptr(inputs, ctypes.c_uint8), desync_peer, desync_frame, _ptr(sent_frame, ctypes.c_int32),
        _ptr(sent_cs, ctypes.c_uint16), ev_cap, _ptr(ev["peer"], ctypes.c_int32),
        _ptr(ev["call"], ctypes.c_int32), _ptr(ev["frame"], ctypes.c_int32),
        _ptr(ev["local"], ctypes.c_uint16), _ptr(ev["remote"], ctypes.c_uint16), ctypes.byref(n_ev),
        _ptr(trace, ctypes.c_uint16))
    n = min(n_ev.value, ev_cap)
    events = [(int(ev["peer"][i]), int(ev["call"][i]), int(ev["frame"][i]), int(ev["local"][i]),
               int(ev["remote"][i])) for i in range(n)]
    return dict(rc=rc, sent_frame=sent_frame, sent_cs=sent_cs, events=events, n_events=n_ev.value,
                cksum_trace=trace)


def particles_synctest_run(inputs, num_entities, num_players=2, max_prediction=17,
                           check_distance=16, session=0, corrupt_frame=-1, ring_states=True):
    """SyncTest over the config-5 particle world for one session (see particles.h for the game)."""
    inputs = np.ascontiguousarray(inputs, np.uint8).reshape(-1, num_players)
    frames = inputs.shape[0]
    R = max_prediction + 1
    sb = 4 + 100 * num_entities
    res = SyncTestResult()
    out = dict(ck_trace=np.zeros(frames, np.uint16), final_state=np.zeros(sb, np.uint8),
               ring_frames=np.zeros(R, np.int32), ring_cksums=np.zeros(R, np.uint16),
               ring_states=np.zeros((R, sb), np.uint8) if ring_states else None)
    rc = lib().oracle_particles_synctest_run(
        num_entities, num_players, max_prediction, check_distance, session, frames,
        _ptr(inputs, ctypes.c_uint8), corrupt_frame, _ptr(out["ck_trace"], ctypes.c_uint16),
        _ptr(out["final_state"], ctypes.c_uint8), _ptr(out["ring_frames"], ctypes.c_int32),
        _ptr(out["ring_cksums"], ctypes.c_uint16), _ptr(out["ring_states"], ctypes.c_uint8),
        ctypes.byref(res))
    out["rc"] = rc
    out["result"] = res
    return out


def sincos_digest(lo, hi, threads=8):
    return int(lib().oracle_sincos_digest(lo, hi, threads))


def sincos_range(lo, hi):
    n = hi - lo + 1
    s = np.zeros(n, np.uint32)
    c = np.zeros(n, np.uint32)
    lib().oracle_sincos_range(lo, hi, _ptr(s, ctypes.c_uint32), _ptr(c, ctypes.c_uint32))
    return s, c


def synctest_bench(threads, frames, warmup=1000, num_players=2, max_prediction=8,
                   check_distance=7, input_delay=2, model=MODEL_UNIFORM,
                   seed_base=0x6767525300000000):
    """CPU baseline: the reference SyncTest loop, one session per thread.

    Returns (resim_frames_total, wall_seconds, thread0_checksums)."""
    cfg = SyncTestCfg(num_players, max_prediction, check_distance, input_delay, 0, 0, 0, -1, 0)
    ck = np.zeros(frames, np.uint16)
    wall = ctypes.c_double(0)
    n = lib().oracle_synctest_bench(ctypes.byref(cfg), model, seed_base, threads, warmup, frames,
                                    _ptr(ck, ctypes.c_uint16), ctypes.byref(wall))
    if n < 0:
        raise RuntimeError("oracle bench session failed")
    return int(n), wall.value, ck


def branch_bench(num_players, window, alphabet, branches, remote_mask, sessions, rounds, threads,
                 model=MODEL_HELD, seed=0x6767525300000000):
    """CPU baseline of configs 3/4: B rollback replays of W frames per session per round plus the
    trunk confirmation, through the SyncLayer + ex_game handler (oracle_branch_bench), `sessions`
    sessions on each of `threads` threads.  Returns (logical resimulated frames, wall seconds,
    xor of every trunk checksum)."""
    wall = ctypes.c_double(0)
    dg = np.zeros(1, np.uint16)
    n = lib().oracle_branch_bench(num_players, window, alphabet, branches, remote_mask, sessions, rounds,
                                  threads, model, seed, ctypes.byref(wall), _ptr(dg, ctypes.c_uint16))
    if n < 0:
        raise ValueError("bad branch bench arguments")
    return int(n), wall.value, int(dg[0])


# ---------------------------------------------------------------- input wire codec (codec.c)
CODEC_OK, CODEC_E_BINCODE, CODEC_E_RLE, CODEC_E_DELTA, CODEC_E_CAP = 0, -1, -2, -3, -4


def _codec_bind(L):
    if getattr(L, "_codec_bound", False):
        return
    i64, i32 = ctypes.c_int64, ctypes.c_int32
    u8p = ctypes.POINTER(ctypes.c_uint8)
    i32p = ctypes.POINTER(ctypes.c_int32)
    L.oracle_codec_encode.argtypes = [u8p, i32, u8p, i32p, i32, u8p, i64]
    L.oracle_codec_encode.restype = i64
    L.oracle_codec_decode.argtypes = [u8p, i32, u8p, i64, u8p, i64, i32p, i32, i32p]
    L.oracle_codec_decode.restype = ctypes.c_int
    L.oracle_rle_encode.argtypes = [u8p, i64, u8p, i64]
    L.oracle_rle_encode.restype = i64
    L.oracle_rle_decode.argtypes = [u8p, i64, u8p, i64]
    L.oracle_rle_decode.restype = i64
    L.oracle_codec_bench.argtypes = [u8p, u8p, i32p, i64, i32, i32, i32, ctypes.POINTER(ctypes.c_double)]
    L.oracle_codec_bench.restype = i64
    L.oracle_codec_bench_mt.argtypes = [u8p, u8p, i32p, i64, i32, i32, i32, i32, ctypes.POINTER(ctypes.c_double)]
    L.oracle_codec_bench_mt.restype = i64
    L._codec_bound = True


def _u8(b):
    a = np.frombuffer(bytes(b), np.uint8) if not isinstance(b, np.ndarray) else np.ascontiguousarray(b, np.uint8)
    return a if a.size else np.zeros(1, np.uint8)


def codec_encode(reference, inputs):
    """compression::encode(reference, pending inputs) -> packet bytes (src/network/compression.rs:14-24)."""
    L = lib()
    _codec_bind(L)
    ref = _u8(reference)
    lens = np.array([len(x) for x in inputs] or [0], np.int32)
    flat = _u8(b"".join(bytes(x) for x in inputs))
    total = sum(len(x) for x in inputs)
    cap = 64 + 4 * len(inputs) + 2 * total
    out = np.zeros(cap, np.uint8)
    n = L.oracle_codec_encode(_ptr(ref, ctypes.c_uint8), len(reference), _ptr(flat, ctypes.c_uint8),
                              _ptr(lens, ctypes.c_int32), len(inputs), _ptr(out, ctypes.c_uint8), cap)
    if n < 0:
        raise RuntimeError(f"codec_encode: {n}")
    return out[:n].tobytes()


def codec_decode(reference, data, max_inputs=1 << 16):
    """compression::decode -> (0, [input bytes]) or (negative CODEC_E_*, None)."""
    L = lib()
    _codec_bind(L)
    ref = _u8(reference)
    d = _u8(data)
    cap = 1 << 24
    out = np.zeros(cap, np.uint8)
    lens = np.zeros(max_inputs, np.int32)
    n = ctypes.c_int32()
    rc = L.oracle_codec_decode(_ptr(ref, ctypes.c_uint8), len(reference), _ptr(d, ctypes.c_uint8), len(data),
                               _ptr(out, ctypes.c_uint8), cap, _ptr(lens, ctypes.c_int32), max_inputs,
                               ctypes.byref(n))
    if rc != 0:
        return rc, None
    res, p = [], 0
    for k in range(n.value):
        res.append(out[p:p + lens[k]].tobytes())
        p += lens[k]
    return 0, res


def codec_bench(ref, pending, count, passes=1, threads=1):
    """CPU baseline: encode + decode every packet one by one (oracle_codec_bench; threads > 1:
    oracle_codec_bench_mt, each thread its slice of the packets).  Returns (packets round-tripped,
    wall seconds)."""
    L = lib()
    _codec_bind(L)
    N, W, B = pending.shape
    ref = np.ascontiguousarray(ref, np.uint8)
    pending = np.ascontiguousarray(pending, np.uint8)
    count = np.ascontiguousarray(count, np.int32)
    wall = ctypes.c_double()
    if threads > 1:
        n = L.oracle_codec_bench_mt(_ptr(ref, ctypes.c_uint8), _ptr(pending, ctypes.c_uint8),
                                    _ptr(count, ctypes.c_int32), N, B, W, passes, threads, ctypes.byref(wall))
    else:
        n = L.oracle_codec_bench(_ptr(ref, ctypes.c_uint8), _ptr(pending, ctypes.c_uint8), _ptr(count, ctypes.c_int32),
                                 N, B, W, passes, ctypes.byref(wall))
    if n < 0:
        raise RuntimeError("codec round trip failed")
    return n, wall.value


def default_threads():
    """Threads for the batch entries: the CPU share a one-GPU job gets on the GPU box (its
    OMP_NUM_THREADS is 16 there), else this machine's CPUs."""
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(64, int(env) if env and env.isdigit() else (os.cpu_count() or 1)))


def synctest_batch(inputs, num_players=2, max_prediction=8, check_distance=2, input_delay=0, threads=None,
                   trace=True):
    """oracle_synctest_run for every lane of inputs[frames][lanes][P] (the engine's layout), on
    `threads` threads: dict of cksum [frames][lanes] (the display checksum after every call),
    final_states [lanes][sb], ring_frames / ring_cksums [lanes][R], status [lanes]."""
    inputs = np.ascontiguousarray(inputs, np.uint8)
    frames, lanes = inputs.shape[0], inputs.shape[1]
    R, sb = max_prediction + 1, state_bytes(num_players)
    cfg = SyncTestCfg(num_players, max_prediction, check_distance, input_delay, 0, 0, 1, -1, 0)
    out = dict(cksum=np.zeros((frames, lanes), np.uint16) if trace else None,
               final_states=np.zeros((lanes, sb), np.uint8), ring_frames=np.zeros((lanes, R), np.int32),
               ring_cksums=np.zeros((lanes, R), np.uint16), status=np.zeros(lanes, np.int32))
    L = lib()
    if not getattr(L, "_batch_bound", False):
        P = ctypes.POINTER
        u8p, u16p, i32p = P(ctypes.c_uint8), P(ctypes.c_uint16), P(ctypes.c_int32)
        L.oracle_synctest_batch.argtypes = [P(SyncTestCfg), ctypes.c_int32, ctypes.c_int64, u8p, ctypes.c_int32,
                                            u16p, u8p, i32p, u16p, i32p]
        L.oracle_synctest_batch.restype = ctypes.c_int
        L.oracle_p2p_replay_batch.argtypes = [ctypes.c_int32, ctypes.c_int64, u8p, i32p, ctypes.c_int32,
                                              ctypes.c_int32, u8p, ctypes.c_int32, u16p, u8p]
        L.oracle_p2p_replay_batch.restype = ctypes.c_int
        L._batch_bound = True
    L.oracle_synctest_batch(ctypes.byref(cfg), frames, lanes, _ptr(inputs, ctypes.c_uint8), threads or default_threads(),
                            _ptr(out["cksum"], ctypes.c_uint16), _ptr(out["final_states"], ctypes.c_uint8),
                            _ptr(out["ring_frames"], ctypes.c_int32), _ptr(out["ring_cksums"], ctypes.c_uint16),
                            _ptr(out["status"], ctypes.c_int32))
    return out


def p2p_replay_batch(start_states, start_index, load_frame, inputs, threads=None, states=False):
    """p2p_replay for many lanes at once: lane l from start_states[start_index[l]] (the cell of
    load_frame) over inputs[l][count][P]; returns (checksums [lanes][count], states
    [lanes][count][sb] or None)."""
    start_states = np.ascontiguousarray(start_states, np.uint8)
    sb = start_states.shape[-1]
    P = (sb - 36) // 20
    idx = np.ascontiguousarray(start_index, np.int32)
    inp = np.ascontiguousarray(inputs, np.uint8)
    lanes, count = inp.shape[0], inp.shape[1]
    cks = np.zeros((lanes, count), np.uint16)
    st = np.zeros((lanes, count, sb), np.uint8) if states else None
    L = lib()
    if not getattr(L, "_batch_bound", False):
        synctest_batch(np.zeros((1, 1, P), np.uint8), P, 2, 1, 0, threads=1)  # binds the batch entries
    rc = L.oracle_p2p_replay_batch(P, lanes, _ptr(start_states, ctypes.c_uint8), _ptr(idx, ctypes.c_int32), load_frame,
                                   count, _ptr(inp, ctypes.c_uint8), threads or default_threads(),
                                   _ptr(cks, ctypes.c_uint16), _ptr(st, ctypes.c_uint8))
    if rc != 0:
        raise ValueError("bad p2p replay batch arguments")
    return cks, st


def handler_bench(streams, num_players, max_prediction, tasks, threads=None):
    """oracle_handler_bench: `tasks` runs of oracle_handler_run over the request streams (a list of
    (kind, frame, inputs, status) per session; task k plays stream k % len(streams)) on `threads`
    threads.  Returns (streams run without error, wall seconds)."""
    M = len(streams)
    off = np.zeros(M + 1, np.int64)
    off[1:] = np.cumsum([len(st[0]) for st in streams])
    kind = np.ascontiguousarray(np.concatenate([st[0] for st in streams]), np.int32)
    frame = np.ascontiguousarray(np.concatenate([st[1] for st in streams]), np.int32)
    inp = np.ascontiguousarray(np.concatenate([st[2] for st in streams]), np.uint8)
    sta = np.ascontiguousarray(np.concatenate([st[3] for st in streams]), np.uint8)
    L = lib()
    P_ = ctypes.POINTER
    L.oracle_handler_bench.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, P_(ctypes.c_int64),
                                       P_(ctypes.c_int32), P_(ctypes.c_int32), P_(ctypes.c_uint8), P_(ctypes.c_uint8),
                                       ctypes.c_int64, ctypes.c_int32, P_(ctypes.c_double)]
    L.oracle_handler_bench.restype = ctypes.c_int64
    wall = ctypes.c_double()
    ok = L.oracle_handler_bench(num_players, max_prediction, M, _ptr(off, ctypes.c_int64), _ptr(kind, ctypes.c_int32),
                                _ptr(frame, ctypes.c_int32), _ptr(inp, ctypes.c_uint8), _ptr(sta, ctypes.c_uint8),
                                tasks, threads or default_threads(), ctypes.byref(wall))
    return int(ok), wall.value


def p2p_batch(inputs, arrive=None, num_players=2, local_mask=0b01, input_delay=0, max_prediction=8, latency=4,
              predictor=0, sparse_saving=False, threads=None):
    """p2p_run (arrive None, fixed latency) or p2p_sched_run (arrive[calls][lanes]) for every lane of
    inputs[calls][lanes][P] on `threads` threads: dict of final_states [lanes][sb], rollbacks,
    resim, current_frame, skips, rc [lanes]."""
    inputs = np.ascontiguousarray(inputs, np.uint8)
    calls, lanes = inputs.shape[0], inputs.shape[1]
    arr = None if arrive is None else np.ascontiguousarray(arrive, np.int32)
    if arr is not None:
        assert arr.shape[:2] == (calls, lanes)
        latency = 1
    cfg = P2PCfg(num_players, max_prediction, input_delay, latency, local_mask, predictor, int(sparse_saving))
    out = dict(final_states=np.zeros((lanes, state_bytes(num_players)), np.uint8),
               rollbacks=np.zeros(lanes, np.int64), resim=np.zeros(lanes, np.int64),
               current_frame=np.zeros(lanes, np.int32), skips=np.zeros(lanes, np.int32), rc=np.zeros(lanes, np.int32))
    L = lib()
    P_ = ctypes.POINTER
    u8p, i32p, i64p = P_(ctypes.c_uint8), P_(ctypes.c_int32), P_(ctypes.c_int64)
    L.oracle_p2p_batch.argtypes = [P_(P2PCfg), ctypes.c_int32, ctypes.c_int64, u8p, i32p, ctypes.c_int32, u8p, i64p,
                                   i64p, i32p, i32p, i32p]
    L.oracle_p2p_batch.restype = ctypes.c_int
    L.oracle_p2p_batch(ctypes.byref(cfg), calls, lanes, _ptr(inputs, ctypes.c_uint8), _ptr(arr, ctypes.c_int32),
                       threads or default_threads(), _ptr(out["final_states"], ctypes.c_uint8),
                       _ptr(out["rollbacks"], ctypes.c_int64), _ptr(out["resim"], ctypes.c_int64),
                       _ptr(out["current_frame"], ctypes.c_int32), _ptr(out["skips"], ctypes.c_int32),
                       _ptr(out["rc"], ctypes.c_int32))
    return out


def p2p_sched_desync_pair_run(inputs, arrive, num_players=2, max_prediction=8, local_masks=(0b01, 0b10),
                              predictor=0, interval=10, corrupt_peer=-1, corrupt_call=-1, desync_peer=-1,
                              desync_frame=-1, ev_cap=4096):
    """Both peers of one match under their own arrival schedules with DesyncDetection::On{interval}
    (oracle_p2p_sched_desync_pair_run): inputs[2][calls][P] each peer's local players' inputs per
    call, arrive[2][calls] the newest frame of the other peer each call polls.  Returns the rows a
    device engine of each peer needs (eff_inputs [2][calls][P], eff_arrive [2][calls]), per call the
    report sent (rep_frame / rep_cs), last_confirmed_frame at the comparison (lconf) and the last
    queued local frame (local_last), the DesyncDetected events (peer, call, frame, local, remote) in
    call order, and each peer's rc."""
    inputs = np.ascontiguousarray(inputs, np.uint8)
    calls = inputs.shape[1]
    arrive = np.ascontiguousarray(arrive, np.int32)
    masks = np.array(local_masks, np.int32)
    out = dict(eff_inputs=np.zeros((2, calls, num_players), np.uint8), eff_arrive=np.zeros((2, calls), np.int32),
               local_last=np.zeros((2, calls), np.int32), rep_frame=np.zeros((2, calls), np.int32),
               rep_cs=np.zeros((2, calls), np.uint16), lconf=np.zeros((2, calls), np.int32))
    ev = {k: np.zeros(ev_cap, t) for k, t in (("peer", np.int32), ("call", np.int32), ("frame", np.int32),
                                              ("local", np.uint16), ("remote", np.uint16))}
    n_ev = ctypes.c_int32(0)
    rc = np.zeros(2, np.int32)
    L = lib()
    P_ = ctypes.POINTER
    u8p, u16p, i32p, i32 = P_(ctypes.c_uint8), P_(ctypes.c_uint16), P_(ctypes.c_int32), ctypes.c_int32
    L.oracle_p2p_sched_desync_pair_run.argtypes = [i32, i32, i32, i32, i32p, i32, u8p, i32p, i32, i32, i32, i32,
                                                   u8p, i32p, i32p, i32p, u16p, i32p, i32, i32p, i32p, i32p, u16p,
                                                   u16p, i32p, i32p]
    L.oracle_p2p_sched_desync_pair_run.restype = ctypes.c_int
    r = L.oracle_p2p_sched_desync_pair_run(
        num_players, max_prediction, predictor, interval, _ptr(masks, ctypes.c_int32), calls,
        _ptr(inputs, ctypes.c_uint8), _ptr(arrive, ctypes.c_int32), corrupt_peer, corrupt_call, desync_peer,
        desync_frame, _ptr(out["eff_inputs"], ctypes.c_uint8), _ptr(out["eff_arrive"], ctypes.c_int32),
        _ptr(out["local_last"], ctypes.c_int32), _ptr(out["rep_frame"], ctypes.c_int32),
        _ptr(out["rep_cs"], ctypes.c_uint16), _ptr(out["lconf"], ctypes.c_int32), ev_cap,
        _ptr(ev["peer"], ctypes.c_int32), _ptr(ev["call"], ctypes.c_int32), _ptr(ev["frame"], ctypes.c_int32),
        _ptr(ev["local"], ctypes.c_uint16), _ptr(ev["remote"], ctypes.c_uint16), ctypes.byref(n_ev),
        _ptr(rc, ctypes.c_int32))
    if r != 0:
        raise ValueError("bad pair-run arguments")
    n = min(n_ev.value, ev_cap)
    out["events"] = [(int(ev["peer"][i]), int(ev["call"][i]), int(ev["frame"][i]), int(ev["local"][i]),
                      int(ev["remote"][i])) for i in range(n)]
    out["n_events"] = n_ev.value
    out["rc"] = rc
    return out
