"""GPU parity of the request-level boundary (ggrs_handle_requests / BoxGameHandler): an ordered
GgrsRequest list (src/lib.rs:171-195) executed on every lane exactly as ex_game's
Game::handle_requests (examples/ex_game/ex_game.rs:79-127) would."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def synctest_requests(f, cd, P, lane_inputs, delay):
    """The request list SyncTestSession::advance_frame emits at frame f (sync_test_session.rs:85-150)."""
    from ggrs_amd import AdvanceFrame, LoadGameState, SaveGameState

    def inp(g):
        return lane_inputs[g - delay] if g >= delay else np.zeros_like(lane_inputs[0])
    reqs = []
    if cd > 0 and f > cd:
        reqs.append(LoadGameState(f - cd))
        for i in range(cd):
            g = f - cd + i
            if i > 0:
                reqs.append(SaveGameState(g))
            reqs.append(AdvanceFrame(inp(g)))
    if cd > 0:
        reqs.append(SaveGameState(f))
    reqs.append(AdvanceFrame(inp(f)))
    return reqs


def test_handler_replays_synctest_stream(oracle):
    from ggrs_amd import BoxGameHandler, Engine
    P, maxp, cd, d, F, lanes = 2, 8, 7, 2, 60, 96
    inputs = np.stack([oracle.gen_inputs(oracle.session_seed(l, 123), F, P) for l in range(lanes)], axis=1)
    eng = Engine(lanes, P, maxp, cd, d, trace_capacity=F)
    h = BoxGameHandler(eng)
    for f in range(F):
        saves = h.handle_requests(synctest_requests(f, cd, P, inputs, d))
        assert f in saves or cd == 0
        if f == F - 1:  # the batched read equals one read per saved frame
            for fr, ck in saves.items():
                assert (eng.save_checksums(fr) == ck).all()
    for lane in (0, 50, 95):
        r = oracle.synctest_run(inputs[:, lane, :], P, maxp, cd, d)
        assert bytes(eng.state(lane)) == bytes(r["final_state"])
        fr, ck, st = eng.ring(lane)
        assert fr.tolist() == r["ring_frames"].tolist()
        assert ck.tolist() == r["ring_cksums"].tolist()
        assert eng.trace(F - 10, 10)[:, lane].tolist() == r["cksum"][F - 10:].tolist()


def test_disconnected_status_spins(oracle):
    from ggrs_amd import AdvanceFrame, BoxGameHandler, Engine, SaveGameState
    P, lanes = 4, 64
    eng = Engine(lanes, P, 8, 2, 0)
    h = BoxGameHandler(eng)
    rng = np.random.default_rng(1)
    state = [oracle.state_new(P) for _ in range(lanes)]
    for f in range(30):
        inp = rng.integers(0, 16, (lanes, P)).astype(np.uint8)
        st = np.where(rng.random((lanes, P)) < 0.25, 2, rng.integers(0, 2, (lanes, P))).astype(np.uint8)
        h.handle_requests([AdvanceFrame(inp, st)])
        state = [oracle.state_advance(state[l], inp[l], st[l]) for l in range(lanes)]
    for lane in range(0, lanes, 9):
        assert bytes(eng.state(lane)) == bytes(state[lane])
    cks = h.handle_requests([SaveGameState(30)])[30]
    for lane in range(0, lanes, 9):
        assert int(cks[lane]) == oracle.fletcher16(bytes(state[lane]))


def test_request_preconditions(oracle):
    from ggrs_amd import AdvanceFrame, BoxGameHandler, Engine, LoadGameState, PreconditionError, SaveGameState
    eng = Engine(4, 2, 8, 2, 0)
    h = BoxGameHandler(eng)
    z = np.zeros((4, 2), np.uint8)
    with pytest.raises(PreconditionError, match="save frame"):
        h.handle_requests([SaveGameState(3)])          # ex_game.rs:104 assert_eq!(frame)
    with pytest.raises(PreconditionError, match="no saved state"):
        h.handle_requests([LoadGameState(0)])          # nothing saved yet
    h.handle_requests([SaveGameState(0), AdvanceFrame(z), SaveGameState(1), AdvanceFrame(z)])
    h.handle_requests([LoadGameState(0), AdvanceFrame(z)])
    assert eng.current_frame() == 1
    with pytest.raises(PreconditionError, match="no saved cell"):
        eng.save_checksums_frames([0, 5])               # frame 5 was never saved
    assert eng.save_checksums_frames([1, 0]).shape == (2, 4)
    ref = oracle.state_advance(oracle.state_new(2), [0, 0])
    assert bytes(eng.state(2)) == bytes(ref)
