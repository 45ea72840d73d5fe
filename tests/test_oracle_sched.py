"""The oracle's P2P session under an arrival schedule (oracle_p2p_sched_run), the checker of
tests/test_gpu_p2p_sched.py.  CPU only.

Pinned by the oracle's other P2P restatements, which share nothing with it but the game: a schedule
delivering frame c - D at call c is oracle_p2p_run at latency D (state, ring, rollbacks, resimulated
frames; every predictor and saving mode), and a jittered schedule gives the state and ring that
Game::handle_requests (oracle_handler_run) reaches over the request lists oracle_p2p_stream emits
for the same schedule (p2p_session.rs:265-426), with its rollback counts.  Stalls and disconnects,
which those restatements do not model, are checked by their defining properties: a call at the
prediction threshold advances nothing (p2p_session.rs:393-423), and a disconnected player's frames
past its last arrival are played as InputStatus::Disconnected (ex_game: input 4, sync_layer.rs:280-293)."""
import numpy as np
import pytest

from oracle import oracle as o

REQ_SAVE, REQ_LOAD, REQ_ADVANCE = 0, 1, 2


def same_session(a, b):
    return (bytes(a["final_state"]) == bytes(b["final_state"]) and a["ring_frames"].tolist() == b["ring_frames"].tolist()
            and a["ring_cksums"].tolist() == b["ring_cksums"].tolist())


@pytest.mark.parametrize("latency", [1, 3, 7])
@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("predictor", [0, 1])
def test_fixed_schedule_is_p2p_run(oracle, latency, sparse, predictor):
    inp = o.gen_inputs(o.session_seed(5), 300, 2, 1)
    upto = (np.arange(300) - latency).astype(np.int32)
    a = o.p2p_sched_run(inp, upto, max_prediction=8, predictor=predictor, sparse_saving=sparse)
    r = o.p2p_run(inp, latency=latency, max_prediction=8, predictor=predictor, sparse_saving=sparse)
    assert a["rc"] == 0 and r["rc"] == 0
    assert same_session(a, r)
    assert (a["ring_states"] == r["ring_states"]).all()
    assert a["result"].rollbacks == r["result"].rollbacks and a["result"].resim == r["result"].resim
    assert a["current_frame"] == 300 and a["skips"] == 0


@pytest.mark.parametrize("seed", [3, 4, 11])
@pytest.mark.parametrize("sparse", [False, True])
def test_jitter_schedule_is_the_request_stream(oracle, seed, sparse):
    inp = o.gen_inputs(o.session_seed(seed), 300, 2, 1)
    upto = o.jitter_schedule(300, 8, seed)
    a = o.p2p_sched_run(inp, upto, max_prediction=8, sparse_saving=sparse)
    s = o.p2p_stream(inp, upto, max_prediction=8, sparse_saving=sparse)
    assert a["rc"] == 0 and s["rc"] == 0 and s["calls"] == 300
    h = o.handler_run(s["kind"], s["frame"], s["inputs"], s["status"], 2, 8)
    assert h["rc"] == 0 and same_session(a, h)
    assert a["result"].rollbacks == s["result"].rollbacks and a["result"].resim == s["result"].resim
    # the per-call rollback frames are the stream's Load frames
    loads = [int(s["frame"][s["call_off"][c]:s["call_off"][c + 1]][s["kind"][s["call_off"][c]:s["call_off"][c + 1]]
                             == REQ_LOAD][0]) if (s["kind"][s["call_off"][c]:s["call_off"][c + 1]] == REQ_LOAD).any()
             else -1 for c in range(300)]
    assert [int(x) for x in a["rb_frame"]] == loads


def test_stalls_skip_at_the_prediction_threshold(oracle):
    calls, mp = 400, 8
    inp = o.gen_inputs(o.session_seed(21), calls, 2, 1)
    upto = o.stall_schedule(calls, mp, 7)
    a = o.p2p_sched_run(inp, upto, max_prediction=mp)
    assert a["rc"] == 0
    assert a["skips"] > 0 and a["current_frame"] + a["skips"] == calls
    adv = a["advanced"].astype(bool)
    # a call advances only while the session is less than max_prediction frames past the newest frame
    # every player has confirmed (the remote player: its newest arrival; the local one is never behind)
    frame = 0
    for c in range(calls):
        confirmed = min(int(upto[c]), frame)  # (the local input of every frame up to `frame` is queued)
        assert adv[c] == (frame - confirmed < mp), c
        frame += int(adv[c])
    # after the stall the burst arrives: the rollbacks reach max_prediction frames deep
    rb = [c - int(f) for c, f in enumerate(a["rb_frame"]) if f >= 0]
    assert max(rb) >= mp - 1


@pytest.mark.parametrize("at", [37, 120])
def test_disconnect_plays_input_4_past_the_last_arrival(oracle, at):
    """Player 1 (remote) disconnects at call `at`, everything up to frame `at` - 3 having arrived: the
    final state is the one of a session whose player-1 inputs past that frame are 4 and arrive
    without delay."""
    calls, mp, lag = 200, 8, 3
    inp = o.gen_inputs(o.session_seed(at), calls, 2, 0)
    upto = np.maximum(np.arange(calls) - lag, -1).astype(np.int32)
    ev = np.zeros(calls, np.uint8)
    ev[at] = 0b10
    a = o.p2p_sched_run(inp, upto, ev, max_prediction=mp)
    assert a["rc"] == 0 and a["current_frame"] == calls
    last = int(upto[at])
    ref_in = inp.copy()
    ref_in[last + 1:, 1] = 4
    b = o.p2p_sched_run(ref_in, np.arange(calls, dtype=np.int32), max_prediction=mp)
    assert bytes(a["final_state"]) == bytes(b["final_state"])
