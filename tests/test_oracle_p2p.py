"""The C oracle's P2P session (oracle_p2p_run: P2PSession::advance_frame, p2p_session.rs:265-426,
with a deterministic network) pinned by known answers derived from the reference's code and by
the reference's own P2P test properties (tests/test_p2p_session.rs:69-110: the game state's frame
after call i is i + 1; :114-155: two peers fed the same inputs never desync).  CPU only."""
import numpy as np
import pytest

from oracle import oracle as o

REQ_SAVE, REQ_LOAD, REQ_ADVANCE = o.REQ_SAVE, o.REQ_LOAD, o.REQ_ADVANCE


def calls(out, frames):
    """Split the request trace into per-call lists."""
    res, k = [], 0
    for f in range(frames):
        n = int(out["req_len"][f])
        res.append(out["req_trace"][k:k + n].tolist())
        k += n
    return res


def test_constant_default_input_never_rolls_back(oracle):
    # the remote queue predicts the default input before anything arrived (input_queue.rs:139-161)
    inp = np.zeros((100, 2), np.uint8)
    out = o.p2p_run(inp, latency=3, max_prediction=8, req_cap=1000)
    assert out["rc"] == 0 and out["result"].rollbacks == 0
    per = calls(out, 100)
    assert per[0] == [REQ_SAVE, REQ_SAVE, REQ_ADVANCE]   # first-frame save (:305-308) + save (:337)
    assert all(c == [REQ_SAVE, REQ_ADVANCE] for c in per[1:])
    # tests/test_p2p_session.rs:105: frame after call i is i + 1
    assert int.from_bytes(out["final_state"][:4].tobytes(), "little") == 100


@pytest.mark.parametrize("latency", [1, 3, 7])
def test_constant_input_rolls_back_once(oracle, latency):
    """The remote player holds input 5 from frame 0: frames 0..D-1 were predicted with the default
    input, so frame 0's arrival at call D is the only misprediction: one rollback loading frame 0
    and replaying D frames; afterwards repeat-last predicts 5 correctly."""
    inp = np.full((60, 2), 5, np.uint8)
    out = o.p2p_run(inp, latency=latency, max_prediction=8, req_cap=1000)
    res = out["result"]
    assert res.rollbacks == 1 and res.resim == latency
    assert list(np.nonzero(out["rb_frame"] >= 0)[0]) == [latency] and out["rb_frame"][latency] == 0
    per = calls(out, 60)
    want = [REQ_LOAD] + [REQ_ADVANCE] + [REQ_SAVE, REQ_ADVANCE] * (latency - 1) + [REQ_SAVE, REQ_ADVANCE]
    assert per[latency] == want


def test_predict_default_rolls_back_on_every_nonzero_arrival(oracle):
    inp = np.zeros((50, 2), np.uint8)
    inp[10, 1] = 3      # remote player deviates from the default on frame 10 only
    inp[20:, 1] = 7     # and holds 7 from frame 20
    D = 2
    rep = o.p2p_run(inp, latency=D, max_prediction=8, predictor=0)
    dft = o.p2p_run(inp, latency=D, max_prediction=8, predictor=1)
    # repeat-last: wrong on 10 (predicted 0), on 11 (predicted 3 again), on 20 -> 3 rollbacks
    assert list(np.nonzero(rep["rb_frame"] >= 0)[0]) == [10 + D, 11 + D, 20 + D]
    # default predictor: wrong on 10 and on every frame >= 20
    assert list(np.nonzero(dft["rb_frame"] >= 0)[0]) == [10 + D] + list(range(20 + D, 50))
    # the same confirmed history: saved states of frames <= 49 - D agree, predicted ones differ
    for slot, fr in enumerate(rep["ring_frames"]):
        assert dft["ring_frames"][slot] == fr
        same = (rep["ring_states"][slot] == dft["ring_states"][slot]).all()
        assert same == (fr <= 49 - D + 1), fr


def test_rollback_loads_the_arriving_frame(oracle):
    inp = o.gen_inputs(o.session_seed(3), 400, 3, o.MODEL_UNIFORM)
    for D in (1, 4, 6):
        out = o.p2p_run(inp, num_players=3, local_mask=0b001, latency=D, max_prediction=7, req_cap=20000)
        rb = out["rb_frame"]
        f = np.nonzero(rb >= 0)[0]
        assert (rb[f] == f - D).all()
        res = out["result"]
        assert res.resim == D * res.rollbacks
        assert res.n_advance == 400 + res.resim
        assert res.n_load == res.rollbacks
        # saves: the first-frame save, one per call, and count-1 per rollback (adjust_gamestate :698)
        assert res.n_save == 1 + 400 + (D - 1) * res.rollbacks


def test_ring_holds_the_last_frames(oracle):
    inp = o.gen_inputs(o.session_seed(1), 123, 2, o.MODEL_HELD)
    out = o.p2p_run(inp, latency=4, max_prediction=8)
    R = 9
    assert sorted(out["ring_frames"].tolist()) == list(range(123 - R, 123))
    for slot, fr in enumerate(out["ring_frames"]):
        assert fr % R == slot
        assert o.fletcher16(out["ring_states"][slot].tobytes()) == out["ring_cksums"][slot]


@pytest.mark.parametrize("delay", [0, 2])
def test_two_peers_agree_on_confirmed_frames(oracle, delay):
    """Peer A (player 0 local) and peer B (player 1 local) on the same inputs: every frame both
    peers hold confirmed (<= f - D) has the same saved state -- the no-desync property of
    test_desyncs_detected (tests/test_p2p_session.rs:114-155).  With an input delay d the
    remote player's frame g is the local player's call g - d, so B is fed A's inputs shifted."""
    D, frames, mp = 3, 200, 8
    inp = o.gen_inputs(o.session_seed(9), frames, 2, o.MODEL_HELD)
    a_rows = inp.copy()
    b_rows = inp.copy()
    if delay:
        # what each peer's queue holds on frame g for the LOCAL player is call g - delay's input;
        # the remote peer (delay 0 in this network model) must send exactly that for frame g
        a_rows[:, 1] = np.concatenate([np.zeros(delay, np.uint8), inp[:-delay, 1]])
        b_rows[:, 0] = np.concatenate([np.zeros(delay, np.uint8), inp[:-delay, 0]])
    a = o.p2p_run(a_rows, local_mask=0b01, input_delay=delay, latency=D, max_prediction=mp)
    b = o.p2p_run(b_rows, local_mask=0b10, input_delay=delay, latency=D, max_prediction=mp)
    last_confirmed = frames - 1 - D
    for slot in range(mp + 1):
        fa, fb = a["ring_frames"][slot], b["ring_frames"][slot]
        assert fa == fb
        if fa <= last_confirmed:
            assert (a["ring_states"][slot] == b["ring_states"][slot]).all(), fa
            assert a["ring_cksums"][slot] == b["ring_cksums"][slot]


def test_invalid_configs(oracle):
    inp = np.zeros((5, 2), np.uint8)
    assert o.p2p_run(inp, latency=8, max_prediction=8)["rc"] == -1   # prediction threshold
    assert o.p2p_run(inp, latency=0, max_prediction=8)["rc"] == -1
    assert o.p2p_run(inp, local_mask=0b100)["rc"] == -1


@pytest.mark.parametrize("latency,mp,model", [(4, 8, 1), (2, 8, 0), (7, 8, 1), (3, 12, 0)])
def test_sparse_saving_same_game_fewer_saves(latency, mp, model):
    """Sparse saving (p2p_session.rs:666-702, :819-843) changes which states are saved and how far
    rollbacks replay, never the simulated game: identical display checksums and final state, fewer
    SaveGameState requests, at least as many resimulated frames; the restated assertion that the
    confirmed state is never lost (:837-842) holds throughout (an oracle assert would abort)."""
    from oracle import oracle as O
    inp = O.gen_inputs(O.session_seed(3, 9), 500, 2, model)
    dense = O.p2p_run(inp, latency=latency, max_prediction=mp, req_cap=1 << 16)
    sparse = O.p2p_run(inp, latency=latency, max_prediction=mp, req_cap=1 << 16, sparse_saving=True)
    assert dense["rc"] == 0 and sparse["rc"] == 0
    assert (dense["ck_trace"] == sparse["ck_trace"]).all()
    assert bytes(dense["final_state"]) == bytes(sparse["final_state"])
    assert sparse["result"].n_save < dense["result"].n_save
    assert sparse["result"].resim >= dense["result"].resim


@pytest.mark.parametrize("delay,latency", [(0, 1), (0, 3), (1, 2), (2, 5)])
def test_lockstep_mode(oracle, delay, latency):
    """max_prediction 0 = lockstep (builder.rs:134-147): no SaveGameState or LoadGameState ever
    (p2p_session.rs:301-310), an AdvanceFrame only once the current frame is confirmed from every
    player (:393-407), so every input it carries is Confirmed.  The schedule: nothing before the
    first remote input arrives (call `latency`); then with input delay 0 the local input of the
    current frame only enters during the call (after confirmed_frame was taken), so the session
    advances every other call; with a delay it is queued ahead and every call advances."""
    calls = 80
    inp = o.gen_inputs(o.session_seed(21), calls, 2, 1)
    r = o.p2p_run(inp, max_prediction=0, latency=latency, input_delay=delay, req_cap=4 * calls)
    assert r["rc"] == 0 and r["result"].frames_done == calls
    assert r["result"].n_save == 0 and r["result"].n_load == 0 and r["result"].rollbacks == 0
    per = calls_of(r, calls)
    adv = [len(c) for c in per]
    assert set(adv) <= {0, 1} and all(k == [REQ_ADVANCE] for k in per if k)
    assert adv[:latency] == [0] * latency
    steady = adv[latency + 2:]
    if delay == 0:  # alternating: advance, wait, advance, ...
        assert all(steady[i] != steady[i + 1] for i in range(len(steady) - 1))
    else:
        assert all(steady)
    frame = int.from_bytes(r["final_state"][:4].tobytes(), "little")
    assert frame == sum(adv)
    # every AdvanceFrame carries confirmed inputs only
    s = o.p2p_stream(inp, (np.arange(calls) - latency).astype(np.int32), max_prediction=0, input_delay=delay)
    assert s["rc"] == 0 and (s["status"] == 0).all() and (s["kind"] == REQ_ADVANCE).all()
    h = o.handler_run(s["kind"], s["frame"], s["inputs"], s["status"], 2, 1)
    assert bytes(h["final_state"]) == bytes(r["final_state"])


def calls_of(out, frames):
    return calls(out, frames)


def test_branch_bench_trunk_is_the_confirmed_chain(oracle):
    """oracle_branch_bench (the configs 3/4 CPU baseline) keeps every session's trunk on the
    confirmed inputs: the xor of its trunk checksums is the chain State::advance gives, and its
    frame count is rounds x sessions x (B W + 1)."""
    P, W, S, R, T = 4, 8, 3, 10, 2
    seed = 0x6767525300000000
    want = 0
    for t in range(T):
        for s in range(S):
            inp = o.gen_inputs(seed + t * S + s, R + 1, P, o.MODEL_HELD)
            st = o.state_new(P)
            for f in range(R):
                st = o.state_advance(st, inp[f])
                want ^= o.fletcher16(bytes(st))
    n, wall, dg = o.branch_bench(P, W, 16, 16, 0b1110, S, R, T, seed=seed)
    assert dg == want and n == T * S * R * (16 * W + 1)
    n3, _, _ = o.branch_bench(2, 4, 16, 16 ** 4, 0b10, 1, 1, 1)
    assert n3 == 16 ** 4 * 4 + 1
    with pytest.raises(ValueError):
        o.branch_bench(2, 4, 16, 100, 0b10, 1, 1, 1)  # not a power of the alphabet
