"""The oracle's scheduled P2P session in lockstep mode and under peers' disconnect reports
(oracle_p2p_sched_run with max_prediction 0 / reports[]), the checker of the matching GPU cases.
CPU only.

Lockstep (p2p_session.rs:301-304, 393-397) is pinned by oracle_p2p_run's lockstep mode at a fixed
latency and by its defining properties (no saves, no rollbacks, a call advances exactly when every
input of the current frame has arrived).  Peer reports (update_player_disconnects, :748-783) are
pinned by the equivalence the reference implies: a report of player k at its newest delivered frame
disconnects it exactly as the local Event::Disconnected does; a report of an older frame rolls back
further, and -- local_connect_status[k].last_frame staying newer -- again on every call until the
reporter's endpoint stops running or the frame leaves the prediction window (the reference panics in
load_frame, sync_layer.rs:231-237)."""
import numpy as np
import pytest

from oracle import oracle as o


def same_session(a, b):
    return (bytes(a["final_state"]) == bytes(b["final_state"]) and a["ring_frames"].tolist() == b["ring_frames"].tolist()
            and a["ring_cksums"].tolist() == b["ring_cksums"].tolist())


@pytest.mark.parametrize("latency,delay,P,local", [(1, 0, 2, 0b01), (4, 2, 2, 0b10), (3, 1, 3, 0b010)])
def test_lockstep_fixed_schedule_is_p2p_run(oracle, latency, delay, P, local):
    calls = 200
    inp = o.gen_inputs(o.session_seed(9), calls, P, 1)
    upto = (np.arange(calls) - latency).astype(np.int32)
    a = o.p2p_sched_run(inp, upto, num_players=P, local_mask=local, input_delay=delay, max_prediction=0)
    r = o.p2p_run(inp, num_players=P, local_mask=local, input_delay=delay, max_prediction=0, latency=latency)
    assert a["rc"] == 0
    assert bytes(a["final_state"]) == bytes(r["final_state"])
    assert a["result"].rollbacks == 0 and a["result"].n_save == 0 and a["result"].n_load == 0
    assert a["current_frame"] == int.from_bytes(r["final_state"][:4].tobytes(), "little")


def test_lockstep_jitter_advances_exactly_when_confirmed(oracle):
    """A call advances exactly when last_confirmed_frame == current_frame: every remote input of the
    current frame delivered and the local one queued by an earlier call (the call's own local input
    is registered after the confirmed frame is taken, p2p_session.rs:314-377, so at input delay 0 a
    session advances at most every other call); 240 calls keep the remote queue below its 128."""
    calls, P = 240, 2
    inp = o.gen_inputs(o.session_seed(4), calls, P, 1)
    upto = o.stall_schedule(calls, 8, 17, stall_every=60)
    a = o.p2p_sched_run(inp, upto, num_players=P, max_prediction=0)
    assert a["rc"] == 0 and a["result"].rollbacks == 0 and a["result"].n_save == 0
    cur, ll, dl = 0, -1, -1
    for c in range(calls):
        dl = max(dl, int(upto[c]))
        want = min(ll, dl) >= cur
        assert bool(a["advanced"][c]) == want, c
        if ll == -1 or cur == ll + 1:
            ll = cur
        cur += int(want)
    assert a["current_frame"] == cur and a["skips"] == calls - cur
    assert (a["ring_frames"] == -1).all()


@pytest.mark.parametrize("sparse", [False, True])
def test_report_at_delivered_frame_is_the_local_event(oracle, sparse):
    """P = 3, local player 0: player 2's endpoint reports player 1 disconnected at the frame this
    call delivered -- the same disconnect as the local Event::Disconnected of player 1."""
    calls, P, mp = 160, 3, 8
    inp = o.gen_inputs(o.session_seed(2), calls, P, 1)
    upto = o.jitter_schedule(calls, mp, 5)
    c0 = 70
    ev = np.zeros(calls, np.uint8)
    ev[c0] = 1 << 1
    rep = np.zeros(calls, np.int32)
    rep[c0] = o.peer_report(1, 2, int(np.maximum.accumulate(upto)[c0]))
    a = o.p2p_sched_run(inp, upto, ev, num_players=P, max_prediction=mp, sparse_saving=sparse)
    b = o.p2p_sched_run(inp, upto, num_players=P, max_prediction=mp, sparse_saving=sparse, reports=rep)
    assert a["rc"] == b["rc"] == 0
    assert same_session(a, b) and (a["ring_states"] == b["ring_states"]).all()
    assert a["result"].rollbacks == b["result"].rollbacks and a["result"].resim == b["result"].resim
    assert (a["rb_frame"] == b["rb_frame"]).all()


def older_report_run(n, reporter_leaves=True, calls=120):
    P, mp = 3, 8
    inp = o.gen_inputs(o.session_seed(6), calls, P, 1)
    upto = np.maximum(np.arange(calls) - 2, -1).astype(np.int32)
    rep = np.zeros(calls, np.int32)
    rep[50] = o.peer_report(1, 2, n)  # player 1 delivered up to 48 here
    ev = np.zeros(calls, np.uint8)
    if reporter_leaves:
        ev[53] = 1 << 2  # the reporter (player 2) disconnects 3 calls later
    return o.p2p_sched_run(inp, upto, ev, num_players=P, max_prediction=mp, reports=rep)


def test_older_report_rolls_back_every_call_until_the_reporter_stops(oracle):
    """A report older than the frames delivered: the session rolls back to its frame + 1 on every
    call while the reporter's endpoint runs; the reporter's own disconnect ends it.  Reported further
    back than the queues hold (last_confirmed - 1), the replay's InputQueue::input panics."""
    a = older_report_run(47)
    assert a["rc"] == 0
    assert [int(x) for x in a["rb_frame"][50:53]] == [48, 48, 48]
    assert (a["rb_frame"][54:] != 48).all()
    b = older_report_run(47, reporter_leaves=False)
    assert b["rc"] == -4 and 53 <= b["result"].frames_done < 60
    c = older_report_run(45)
    assert c["rc"] == -4 and c["result"].frames_done == 51


def test_queue_tail_precheck_is_the_restated_queues_assert(oracle):
    """The oracle's early "rolls back past the trimmed queues" test (ORACLE_SCHED_NO_TAIL_CHECK=1
    turns it off, leaving the restated InputQueue's assert to end the call) stops every run at the
    same call: it is the reference's panic condition, the one the device checks."""
    import json
    import os
    import subprocess
    import sys
    code = ("import json, numpy as np, sys; sys.path.insert(0, %r); from tests.test_oracle_sched_lockstep_reports "
            "import older_report_run; print(json.dumps([[int(r['rc']), int(r['result'].frames_done)] for r in "
            "(older_report_run(n, f) for n in range(40, 49) for f in (True, False))]))") % os.getcwd()
    out = {}
    for flag in ("0", "1"):
        env = dict(os.environ, ORACLE_SCHED_NO_TAIL_CHECK=flag)
        out[flag] = json.loads(subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                                              check=True, cwd=os.getcwd()).stdout)
    assert out["0"] == out["1"]
    assert any(rc == -4 for rc, _ in out["0"]) and any(rc == 0 for rc, _ in out["0"])


def test_report_validation(oracle):
    calls, P = 20, 3
    inp = o.gen_inputs(o.session_seed(1), calls, P, 1)
    upto = np.maximum(np.arange(calls) - 1, -1).astype(np.int32)
    for bad in (o.peer_report(0, 2, 3), o.peer_report(1, 0, 3), o.peer_report(1, 1, 3), o.peer_report(1, 2, 11)):
        rep = np.zeros(calls, np.int32)
        rep[10] = bad
        assert o.p2p_sched_run(inp, upto, num_players=P, max_prediction=8, reports=rep)["rc"] == -1
