"""GPU parity of the P2P engine under arrival schedules (ggrs_p2p_set_arrival_schedule / add_arrivals,
p2p_sched.hip) against the oracle's P2PSession stepped call by call under the same schedule
(oracle_p2p_sched_run): jittered remote arrivals, network stalls longer than max_prediction (calls
at the prediction threshold skip their AdvanceFrame, p2p_session.rs:393-423, then a burst as deep
as the window arrives), and disconnects (a rollback to the player's last frame + 1 and
InputStatus::Disconnected replays, :618-655, sync_layer.rs:280-293).  Every checked session's final
state, saved-state ring with its frame tags, rollback / resimulation counts, skipped calls, current
frame and error are bit-exact -- including the sessions where the reference would panic."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")  # loads torch's HIP runtime before the engine library

pytestmark = pytest.mark.gpu


def schedules(S, calls, mp, seed, local_mask, P, disconnect_every=5):
    """[calls][S] arrivals and events: per session its own network -- stalls with bursts (2 of 3
    sessions), plain jitter, or a fixed latency -- and a disconnect of one remote player in every
    `disconnect_every`-th session."""
    from oracle import oracle as o
    arrive = np.zeros((calls, S), np.int32)
    events = np.zeros((calls, S), np.uint8)
    remote = [k for k in range(P) if not (local_mask >> k) & 1]
    rng = np.random.default_rng(seed)
    for s in range(S):
        kind = s % 3
        if kind == 2:
            arrive[:, s] = np.maximum(np.arange(calls) - int(rng.integers(1, mp)), -1)
        else:
            arrive[:, s] = o.stall_schedule(calls, mp, seed * 1000 + s, stall_every=40 if kind == 0 else 10 ** 9)
        if disconnect_every and s % disconnect_every == 0:
            events[int(rng.integers(calls // 4, 3 * calls // 4)), s] = 1 << remote[s % len(remote)]
    return arrive, events


def check_sessions(eng, rows, arrive, events, sessions, calls, reports=None, **kw):
    from oracle import oracle as o
    from ggrs_amd._lib import GGRS_E_PRECONDITION
    frames, skipped, errors = eng.sessions()
    rb, rs = eng.stats()
    for s in sessions:
        out = o.p2p_sched_run(rows[:calls, s], arrive[:calls, s], events[:calls, s], num_players=eng.num_players,
                              local_mask=eng.local_mask, input_delay=eng.input_delay,
                              max_prediction=eng.max_prediction, predictor=eng.predictor,
                              reports=None if reports is None else reports[:calls, s], **kw)
        res = out["result"]
        if out["rc"] == -4:  # the reference panics at this call: the device stops the session there
            assert errors[s] == GGRS_E_PRECONDITION, (s, errors[s])
        else:
            assert out["rc"] == 0 and errors[s] == 0, (s, out["rc"], errors[s])
            assert frames[s] == out["current_frame"] and skipped[s] == out["skips"], (s, frames[s], out["current_frame"])
        assert bytes(eng.state(s)) == bytes(out["final_state"]), s
        fr, cks, states = eng.ring(s)
        assert (fr == out["ring_frames"]).all(), (s, fr, out["ring_frames"])
        assert (cks == out["ring_cksums"]).all(), s
        assert (states == out["ring_states"]).all(), s
        assert rb[s] == res.rollbacks and rs[s] == res.resim, (s, rb[s], res.rollbacks, rs[s], res.resim)


CASES = [
    # P, local players, delay, max_prediction, predictor, input model, sparse saving
    (2, (0,), 0, 8, 0, 0, False),
    (2, (1,), 2, 6, 0, 1, False),
    (4, (0, 2), 1, 7, 1, 0, False),
    (3, (0,), 0, 12, 0, 0, False),
    (2, (0,), 0, 8, 0, 0, True),
    (4, (1,), 1, 9, 0, 0, True),
    (2, (), 1, 8, 0, 0, False),
]


FORMS = ["chains", "flat"]


def set_form(monkeypatch, form):
    """chains: the time-aligned kernel (a session's replays on 16 lanes; the default for few
    sessions), flat: one thread per session (GGRS_SCHED_CHAINS=0; the many-session form)."""
    monkeypatch.setenv("GGRS_SCHED_CHAINS", "1" if form == "chains" else "0")


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("P,local,delay,mp,pred,model,sparse", CASES)
def test_p2p_arrival_schedules_match_oracle(oracle, monkeypatch, form, P, local, delay, mp, pred, model, sparse):
    set_form(monkeypatch, form)
    from ggrs_amd import P2PEngine
    S, calls = 200, 240
    mask = sum(1 << k for k in local)
    rows = np.stack([oracle.gen_inputs(oracle.session_seed(s, 0x5C4E), calls, P, model) for s in range(S)], axis=1)
    arrive, events = schedules(S, calls, mp, 11 + P, mask, P)
    eng = P2PEngine(S, num_players=P, local_players=local, input_delay=delay, max_prediction=mp, remote_latency=1,
                    predictor=pred, input_capacity=calls)
    if sparse:
        eng.set_sparse_saving(True)
    eng.set_arrival_schedule(True)
    eng.add_inputs(0, rows)
    eng.add_arrivals(0, arrive, events)
    done = 0
    for n in (1, 3, 60, 17, 159):
        eng.advance_frames(n)
        done += n
        if done in (4, 81):
            check_sessions(eng, rows, arrive, events, [0, 1, 5, 63, 64, 199], done, sparse_saving=sparse)
    assert done == calls
    check_sessions(eng, rows, arrive, events, range(0, S, 3), calls, sparse_saving=sparse)
    frames, skipped, errors = eng.sessions()
    assert skipped.sum() > 0  # stalls past max_prediction: calls at the prediction threshold
    rb, _ = eng.stats()
    assert rb.sum() > S


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("P,local,mp", [(2, (0,), 6), (2, (1,), 9), (3, (0,), 4)])
def test_p2p_predict_default_silent_start_matches_oracle(oracle, monkeypatch, form, P, local, mp):
    """PredictDefault sessions that receive nothing for their first 0 .. 2 max_prediction + 3 calls:
    while nothing is confirmed frames_ahead is current_frame (p2p_session.rs:399-405), so the session
    stops advancing at call max_prediction, not one call later.  Lets the control pass's fast form
    (which PredictDefault with nothing delivered may take) meet the NULL confirmed frame."""
    set_form(monkeypatch, form)
    from ggrs_amd import P2PEngine
    S, calls = 96, 120
    mask = sum(1 << k for k in local)
    rows = np.stack([oracle.gen_inputs(oracle.session_seed(s, 0xDEF), calls, P, 1) for s in range(S)], axis=1)
    arrive = np.empty((calls, S), np.int32)
    for s in range(S):
        silent = s % (2 * mp + 4)
        sched = oracle.stall_schedule(calls, mp, 77 + s, stall_every=10 ** 9)
        sched[:silent] = -1
        arrive[:, s] = np.maximum.accumulate(sched)
    events = np.zeros((calls, S), np.uint8)
    eng = P2PEngine(S, num_players=P, local_players=local, max_prediction=mp, remote_latency=1, predictor=1,
                    input_capacity=calls)
    eng.set_arrival_schedule(True)
    eng.add_inputs(0, rows)
    eng.add_arrivals(0, arrive, events)
    for n in (mp - 1, 2, 5, calls - mp - 6):
        eng.advance_frames(n)
    check_sessions(eng, rows, arrive, events, range(S), calls)
    frames, skipped, errors = eng.sessions()
    assert skipped.sum() > 0


def test_p2p_arrival_schedule_streamed_and_uniform(oracle):
    """Inputs and arrivals streamed through small rings in chunks; a uniform schedule (every
    session's remote input of frame g at call g + 4) equals the fixed-latency engine's states."""
    from ggrs_amd import P2PEngine
    S, calls, chunk, P = 130, 200, 20, 2
    rows = np.stack([oracle.gen_inputs(oracle.session_seed(s, 0x77), calls, P, 0) for s in range(S)], axis=1)
    arrive = np.repeat(np.maximum(np.arange(calls) - 4, -1)[:, None], S, axis=1).astype(np.int32)
    eng = P2PEngine(S, num_players=P, local_players=(0,), max_prediction=8, remote_latency=1, input_capacity=48)
    eng.set_arrival_schedule(True)
    ref = P2PEngine(S, num_players=P, local_players=(0,), max_prediction=8, remote_latency=4, input_capacity=48)
    for c0 in range(0, calls, chunk):
        eng.add_inputs(c0, rows[c0:c0 + chunk])
        eng.add_arrivals(c0, arrive[c0:c0 + chunk])
        eng.advance_frames(chunk)
        ref.add_inputs(c0, rows[c0:c0 + chunk])
        ref.advance_frames(chunk)
    frames, skipped, errors = eng.sessions()
    assert (frames == calls).all() and (skipped == 0).all() and (errors == 0).all()
    rb, rs = eng.stats()
    rb2, rs2 = ref.stats()
    assert (rb == rb2).all() and (rs == rs2).all()
    for s in (0, 64, 129):
        assert bytes(eng.state(s)) == bytes(ref.state(s))
        a, b = eng.ring(s), ref.ring(s)
        assert all((x == y).all() for x, y in zip(a, b))


def test_p2p_arrival_schedule_rejects(oracle):
    """Arrivals naming a frame after their call, and remote rows overwritten before they arrive,
    stop only the offending sessions (GGRS_E_INVALID / GGRS_E_PRECONDITION); API misuse raises."""
    from ggrs_amd import InvalidRequest, P2PEngine
    from ggrs_amd._lib import GGRS_E_INVALID, GGRS_E_PRECONDITION, GgrsError
    S, P = 70, 2
    eng = P2PEngine(S, num_players=P, local_players=(0,), max_prediction=8, remote_latency=1, input_capacity=32)
    with pytest.raises(GgrsError):
        eng.add_arrivals(0, np.zeros((1, S), np.int32))  # not in scheduled mode
    eng.set_arrival_schedule(True)
    eng.add_inputs(0, np.zeros((32, S, P), np.uint8))
    arrive = np.repeat(np.arange(16)[:, None] - 2, S, axis=1).astype(np.int32)
    arrive[3, 5] = 4  # frame 4 at call 3: later than the call
    eng.add_arrivals(0, arrive)
    with pytest.raises(InvalidRequest):
        eng.advance_frames(17)  # missing arrivals
    eng.advance_frames(16)
    frames, skipped, errors = eng.sessions()
    assert errors[5] == GGRS_E_INVALID and frames[5] == 3
    assert (np.delete(errors, 5) == 0).all() and (np.delete(frames, 5) == 16).all()
    # session 9 receives nothing for 16 calls: the rows of its frames 14, 15 are overwritten by
    # frames 46, 47 before they arrive (the prediction threshold stalls it meanwhile)
    late = np.repeat(np.arange(16, 32)[:, None] - 2, S, axis=1).astype(np.int32)
    late[:, 9] = 13
    eng.add_arrivals(16, late)
    eng.advance_frames(16)
    frames, skipped, errors = eng.sessions()
    assert skipped[9] > 0 and errors[9] == 0
    eng.add_inputs(32, np.zeros((16, S, P), np.uint8))
    eng.add_arrivals(32, np.repeat(np.arange(32, 48)[:, None] - 2, S, axis=1).astype(np.int32))
    eng.advance_frames(16)
    frames, skipped, errors = eng.sessions()
    assert errors[9] == GGRS_E_PRECONDITION
    assert errors[10] == 0 and frames[10] == 48 and skipped[10] == 0


@pytest.mark.parametrize("split", ["chains", "1", "0"])
@pytest.mark.parametrize("stalls,delay,local", [(False, 0, (0,)), (True, 0, (0,)), (False, 2, (1,))])
def test_p2p_synth_schedules_every_session(oracle, monkeypatch, stalls, delay, local, split):
    """The bench's schedules (synth.jitter_arrivals: jittered lags, optionally network stalls past
    max_prediction) for every one of 640 sessions, in launches that cross the kernel's stages at
    different calls -- the control pass's branch-free fast form (every player connected, the rows
    staged) decides nearly every call here -- state, ring, counts, skips and frames bit-exact; with
    the two-wave form (control pass of the next stage beside the step loop: the default when every
    CU holds one block, as here) and the one-wave form (GGRS_SCHED_SPLIT=0, the many-session form),
    and with the time-aligned form (a session's replays on 16 lanes, the default for few sessions)."""
    set_form(monkeypatch, "chains" if split == "chains" else "flat")
    monkeypatch.setenv("GGRS_SCHED_SPLIT", "1" if split == "chains" else split)
    from ggrs_amd import P2PEngine, synth
    S, calls, P, mp = 640, 200, 2, 8
    rows = synth.gen_inputs(0, S, calls, P, synth.MODEL_HELD)
    arrive = synth.jitter_arrivals(0, S, calls, mp, stalls=stalls)
    eng = P2PEngine(S, num_players=P, local_players=local, input_delay=delay, max_prediction=mp, remote_latency=1,
                    input_capacity=calls)
    eng.set_arrival_schedule(True)
    eng.add_inputs(0, rows)
    eng.add_arrivals(0, arrive)
    for n in (37, 64, 99):
        eng.advance_frames(n)
    events = np.zeros((calls, S), np.uint8)
    check_sessions(eng, rows, arrive, events, range(S), calls)
    frames, skipped, errors = eng.sessions()
    assert (errors == 0).all()
    assert (skipped.sum() > 0) == stalls


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("stalls", [False, True])
def test_p2p_bench_schedule_full_size_every_session(oracle, monkeypatch, form, stalls):
    """The bench's any-network configuration at full size (`bench.py --workload p2p --arrivals
    jitter|stall --sessions 4096 --max-prediction 9`: 4096 sessions, 64-call launches): EVERY
    session's final state, rollback count, current frame and skipped calls against the oracle's
    P2PSession under the same schedule (oracle_p2p_batch)."""
    from ggrs_amd import P2PEngine, synth
    from oracle import every_lane
    set_form(monkeypatch, form)
    S, calls, P, mp = 4096, 6 * 64, 2, 9
    rows = synth.gen_inputs(0, S, calls, P, synth.MODEL_HELD)
    arrive = synth.jitter_arrivals(0, S, calls, mp, stalls=stalls)
    eng = P2PEngine(S, num_players=P, local_players=(0,), max_prediction=mp, remote_latency=1, input_capacity=calls)
    eng.set_arrival_schedule(True)
    eng.add_inputs(0, rows)
    eng.add_arrivals(0, arrive)
    for _ in range(calls // 64):
        eng.advance_frames(64)
    r = every_lane.p2p(eng, rows, arrive, P=P, maxp=mp)
    assert r["rc_mismatched"] == r["final_state_mismatched"] == r["rollbacks_mismatched"] == 0, r
    assert r["frame_skips_mismatched"] == 0, r
    check_sessions(eng, rows, arrive, np.zeros((calls, S), np.uint8), (0, 1, S // 2, S - 1), calls)


@pytest.mark.parametrize("P,local,delay", [(2, (0,), 0), (2, (1,), 2), (4, (0, 2), 1), (3, (), 0)])
def test_p2p_lockstep_schedules_match_oracle(oracle, P, local, delay):
    """Lockstep mode under arrival schedules (max_prediction 0, p2p_session.rs:301-304, 393-397):
    no saves, no rollbacks, a call advances only when last_confirmed_frame == current_frame --
    jittered, stalled and fixed networks and disconnects; every session bit-exact against the
    oracle (state, frames, skipped calls, counts), in launches of uneven length."""
    from ggrs_amd import P2PEngine
    S, calls = 300, 180
    rows = np.stack([oracle.gen_inputs(oracle.session_seed(s, 77), calls, P, 1) for s in range(S)], axis=1)
    lmask = sum(1 << k for k in local)
    arrive, events = schedules(S, calls, 8, 13, lmask, P)
    eng = P2PEngine(S, num_players=P, local_players=local, input_delay=delay, max_prediction=0, remote_latency=1,
                    input_capacity=calls)
    eng.set_arrival_schedule(True)
    eng.add_inputs(0, rows)
    eng.add_arrivals(0, arrive, events)
    for n in (1, 30, 64, 85):
        eng.advance_frames(n)
    check_sessions(eng, rows, arrive, events, range(S), calls)
    rb, _ = eng.stats()
    assert (rb == 0).all()
    frames, skipped, errors = eng.sessions()
    assert skipped.sum() > 0 and frames.max() > 40


def peer_report_schedules(S, calls, mp, seed, P, local_mask):
    """Per session a network (schedules()) and peers' disconnect reports of several kinds: at the
    frame the call delivered (the local Event::Disconnected's frame), older ones (repeated rollbacks
    while the reporter runs; further back than the input queues hold: the reference panics), about a
    player already disconnected here at the reported frame, and a reported player's peer reporting
    its own reporter."""
    from oracle import oracle as o
    arrive, events = schedules(S, calls, mp, seed, local_mask, P, disconnect_every=0)
    remote = [k for k in range(P) if not (local_mask >> k) & 1]
    reports = np.zeros((calls, S), np.int32)
    rng = np.random.default_rng(seed + 1)
    for s in range(S):
        kind = s % 6
        k, r = (remote[0], remote[1]) if s % 2 == 0 else (remote[-1], remote[0])
        c = int(rng.integers(calls // 4, calls // 2))
        delivered = int(np.maximum.accumulate(arrive[:, s])[c])
        if kind == 0:
            reports[c, s] = o.peer_report(k, r, delivered)
            # the same endpoint later with an older frame: it keeps the newest (protocol.rs:576-584)
            reports[c + 4, s] = o.peer_report(k, r, max(delivered - 3, -1))
        elif kind == 1:
            reports[c, s] = o.peer_report(k, r, max(delivered - 1, -1))
            events[c + 3, s] |= 1 << r  # the reporter leaves: the repeated rollbacks stop
        elif kind == 2:
            reports[c, s] = o.peer_report(k, r, max(delivered - int(rng.integers(2, 12)), -1))
        elif kind == 3:
            events[c, s] |= 1 << k  # disconnected here first; a peer's report of the same frame changes nothing
            reports[c + 2, s] = o.peer_report(k, r, delivered)
        elif kind == 4:
            reports[c, s] = o.peer_report(k, r, delivered)
            reports[c + 5, s] = o.peer_report(r, k if k != r else remote[0], delivered)  # k's peer reports r
        # kind 5: no report
    return arrive, events, reports


@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("P,local,mp", [(4, (0,), 8), (3, (1,), 6), (4, (0, 3), 9)])
def test_p2p_peer_reported_disconnects_match_oracle(oracle, P, local, mp, sparse):
    """update_player_disconnects (p2p_session.rs:748-783) over the peers' reports, with P > 2
    (ggrs_p2p_add_peer_reports): every session's state, ring, counts, frames, skips and error --
    including the sessions whose report rolls back further than the reference's input queues hold
    (it panics there) -- bit-exact against the oracle."""
    from ggrs_amd import P2PEngine
    from ggrs_amd._lib import GGRS_E_PRECONDITION
    S, calls = 360, 160
    rows = np.stack([oracle.gen_inputs(oracle.session_seed(s, 91), calls, P, 1) for s in range(S)], axis=1)
    lmask = sum(1 << k for k in local)
    arrive, events, reports = peer_report_schedules(S, calls, mp, 29, P, lmask)
    eng = P2PEngine(S, num_players=P, local_players=local, max_prediction=mp, remote_latency=1, input_capacity=calls)
    eng.set_arrival_schedule(True)
    if sparse:
        eng.set_sparse_saving(True)
    eng.add_inputs(0, rows)
    eng.add_arrivals(0, arrive, events)
    eng.add_peer_reports(0, reports)
    for n in (37, 64, 59):
        eng.advance_frames(n)
    check_sessions(eng, rows, arrive, events, range(S), calls, reports=reports, sparse_saving=sparse)
    frames, skipped, errors = eng.sessions()
    assert (errors == GGRS_E_PRECONDITION).sum() > 0 and (errors == 0).sum() > S // 2


def test_p2p_peer_reports_rejected(oracle):
    from ggrs_amd import InvalidRequest, P2PEngine
    from ggrs_amd.p2p import peer_report
    S, calls, P = 8, 20, 3
    eng = P2PEngine(S, num_players=P, local_players=(0,), max_prediction=8, remote_latency=1, input_capacity=calls)
    eng.set_arrival_schedule(True)
    eng.add_inputs(0, np.zeros((calls, S, P), np.uint8))
    eng.add_arrivals(0, np.full((10, S), -1, np.int32))
    for bad in (peer_report(0, 2, 3), peer_report(1, 0, 3), peer_report(1, 1, 3), peer_report(1, 2, 6)):
        rep = np.zeros((10, S), np.int32)
        rep[5, 3] = bad
        with pytest.raises(InvalidRequest):
            eng.add_peer_reports(0, rep)
    with pytest.raises(InvalidRequest):  # calls whose arrivals are not added yet
        eng.add_peer_reports(5, np.zeros((10, S), np.int32))
    eng.add_peer_reports(0, np.zeros((10, S), np.int32))


@pytest.mark.parametrize("sparse,mp", [(False, 8), (True, 7), (False, 0)])
def test_p2p_display_trace_under_schedules(oracle, sparse, mp):
    """The display checksum after every call (the state after the call's last AdvanceFrame, replay
    or own; the previous one when it advanced nothing: ex_game.rs:115-127) under arrival schedules with
    stalls and disconnects, in rollback, sparse-saving and lockstep mode: every session's trace
    equals the oracle's up to where the reference would panic."""
    from ggrs_amd import P2PEngine
    S, calls, P = 320, 160, 3
    rows = np.stack([oracle.gen_inputs(oracle.session_seed(s, 55), calls, P, 1) for s in range(S)], axis=1)
    arrive, events = schedules(S, calls, max(mp, 4), 31, 0b001, P)
    eng = P2PEngine(S, num_players=P, local_players=(0,), max_prediction=mp, remote_latency=1, input_capacity=calls,
                    trace_capacity=calls)
    eng.set_arrival_schedule(True)
    if sparse:
        eng.set_sparse_saving(True)
    eng.add_inputs(0, rows)
    eng.add_arrivals(0, arrive, events)
    for n in (41, 64, 55):
        eng.advance_frames(n)
    tr = eng.trace(0, calls)
    for s in range(S):
        out = oracle.p2p_sched_run(rows[:, s], arrive[:, s], events[:, s], num_players=P, local_mask=0b001,
                                   max_prediction=mp, sparse_saving=sparse)
        done = out["result"].frames_done
        assert (tr[:done, s] == out["ck_trace"][:done]).all(), (s, int(np.argmax(tr[:done, s] != out["ck_trace"][:done])))
    check_sessions(eng, rows, arrive, events, range(0, S, 7), calls, sparse_saving=sparse)
