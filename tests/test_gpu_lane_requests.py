"""GPU parity of per-lane request lists (ggrs_handle_requests_lanes, ggrs_lane_batch_run): every
lane is its own GGRS session with its own Vec<GgrsRequest> per call (src/lib.rs:171-195).

The lists come from the oracle's P2PSession (oracle/ggrs_oracle.c oracle_p2p_stream, a restatement
of p2p_session.rs:265-426) under a jittery network -- remote inputs arrive in bursts, so each
session rolls back to its own first_incorrect frame with its own replay count
(adjust_gamestate, :658-714) -- and sessions start at different calls, so lanes sit at different
frames in one batch.  Expected results: the oracle's request handler (oracle_handler_run,
Game::handle_requests ex_game.rs:79-127 over its own SavedStates ring) run on each lane's stream:
every Save's checksum, the final state and the ring, bit-exact.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REQ_SAVE, REQ_LOAD, REQ_ADVANCE = 0, 1, 2


def p2p_lane_streams(O, lanes, calls, P=2, maxp=8, sparse=False, seed=0, local_mask=0b01, max_lag=None):
    """Per lane: the oracle P2P session's request stream, with the call index each request
    belongs to (lane l's session starts at call l % 7: empty lists before)."""
    out = []
    for l in range(lanes):
        start = l % 7
        n = calls - start
        inp = O.gen_inputs(O.session_seed(l, 0x5EED0000 + seed), n, P, 1)
        up = O.jitter_schedule(n, maxp, seed * 1000 + l, max_lag)
        s = O.p2p_stream(inp, up, num_players=P, local_mask=local_mask, max_prediction=maxp, sparse_saving=sparse)
        assert s["rc"] == 0 and s["calls"] == n
        call_of = np.full(len(s["kind"]), -1, np.int64)
        for c in range(n):
            call_of[s["call_off"][c]:s["call_off"][c + 1]] = c + start
        s["call_of"] = call_of
        s["start"] = start
        out.append(s)
    return out


def expected(O, streams, P, maxp, status_override=None):
    exp = []
    for l, s in enumerate(streams):
        st = s["status"] if status_override is None else status_override[l]
        h = O.handler_run(s["kind"], s["frame"], s["inputs"], st, P, maxp)
        assert h["rc"] == 0
        exp.append(h)
    return exp


def call_lists(streams, c):
    """CSR arrays of call c over all lanes: reqs [n][2], offsets, inputs / status rows, and the
    per-lane index range of the requests in each stream."""
    reqs, offsets, inputs, status, spans = [], [0], [], [], []
    for s in streams:
        idx = np.nonzero(s["call_of"] == c)[0]
        spans.append(idx)
        k, f = s["kind"][idx], s["frame"][idx]
        reqs.append(np.stack([k, f], axis=1))
        adv = idx[k == REQ_ADVANCE]
        inputs.append(s["inputs"][adv])
        status.append(s["st_use"][adv] if "st_use" in s else s["status"][adv])
        offsets.append(offsets[-1] + len(idx))
    return (np.concatenate(reqs).astype(np.int32), np.array(offsets, np.int32), np.concatenate(inputs),
            np.concatenate(status), spans)


def check_final(eng, exp, lanes):
    for l in lanes:
        assert bytes(eng.state(l)) == bytes(exp[l]["final_state"]), f"lane {l} final state"
        fr, ck, st = eng.ring(l)
        assert fr.tolist() == exp[l]["ring_frames"].tolist(), f"lane {l} ring frames"
        for s in range(len(fr)):
            if fr[s] >= 0:
                assert int(ck[s]) == int(exp[l]["ring_cksums"][s]) and bytes(st[s]) == bytes(exp[l]["ring_states"][s])


def run_generic(eng, streams, exp, calls, with_status=True):
    L = len(streams)
    got = [[] for _ in range(L)]
    for c in range(calls):
        reqs, off, inp, st, spans = call_lists(streams, c)
        cks, res = eng.handle_requests_lanes(reqs, off, inp, st if with_status else None)
        assert (res >= 0).all()
        k = 0
        for l in range(L):
            n = int((reqs[off[l]:off[l + 1], 0] == REQ_SAVE).sum())
            got[l].extend(cks[k:k + n].tolist())
            k += n
    for l in range(L):
        assert got[l] == exp[l]["save_cks"].tolist(), f"lane {l}: save checksums differ"
    return got


@pytest.mark.parametrize("sparse,server", [(False, True), (True, True), (False, False)])
def test_p2p_lists_300_sessions_generic(oracle, sparse, server):
    """300 P2P sessions, differing first_incorrect per call, through ggrs_handle_requests_lanes."""
    from ggrs_amd import Engine
    L, calls, P, maxp = 300, 90, 2, 8
    streams = p2p_lane_streams(oracle, L, calls, P, maxp, sparse=sparse, seed=1 + sparse)
    loads = [int((s["kind"] == REQ_LOAD).sum()) for s in streams]
    assert sum(loads) > 200  # plenty of rollbacks
    # rollbacks of differing depth: session frame at a call = its call number (input delay 0)
    depth = {int(s["call_of"][i]) - s["start"] - int(s["frame"][i])
             for s in streams for i in np.nonzero(s["kind"] == REQ_LOAD)[0]}
    assert len(depth) >= 4
    exp = expected(oracle, streams, P, maxp)
    eng = Engine(L, P, maxp, 0, 0)
    eng.set_lane_server(server)
    run_generic(eng, streams, exp, calls)
    check_final(eng, exp, range(L))
    fr = eng.lane_frames()
    assert fr.tolist() == [int(np.frombuffer(bytes(e["final_state"][:4]), np.int32)[0]) for e in exp]


@pytest.mark.parametrize("server,L", [(True, 257), (False, 257), (True, 320), (False, 320)])
def test_p2p_lists_batch_form(oracle, server, L):
    """The same lists pre-encoded per lane into the engine's mapped batch (ggrs_lane_batch_run),
    through the persistent lane server or one launch per batch; L = 320 (a multiple of 8) takes the
    wide staging and write-back (8-byte host words per thread), 257 the per-lane form."""
    import time
    from ggrs_amd import Engine, encode_lane_lists
    calls, P, maxp = 80, 2, 8
    streams = p2p_lane_streams(oracle, L, calls, P, maxp, seed=7)
    exp = expected(oracle, streams, P, maxp)
    eng = Engine(L, P, maxp, 0, 0)
    eng.set_lane_server(server)
    batch = eng.lane_batch(2, 2, 2 * maxp + 2, 2 * maxp + 2)
    got = [[] for _ in range(L)]
    for c in range(calls):
        lists = []
        for s in streams:
            idx = np.nonzero(s["call_of"] == c)[0]
            lists.append([(int(s["kind"][i]), int(s["frame"][i]), s["inputs"][i], s["status"][i]) for i in idx])
        enc = encode_lane_lists(lists, P)
        W, LD, A, S = enc["shape"]
        batch.tokens[:W] = enc["tokens"]
        batch.load_frames[:LD] = enc["load_frames"]
        batch.inputs[:A] = enc["inputs"]
        batch.status[:A] = enc["status"]
        if c == 40:
            time.sleep(0.4)  # the host went idle: the server is restarted (its lanes' states kept)
        assert batch.run(W, LD, A, S, status=True) == 0
        for l, x in enumerate(lists):
            n = sum(1 for r in x if r[0] == REQ_SAVE)
            got[l].extend(batch.checksums[:n, l].tolist())
        assert (batch.lane_result >= 0).all()
    for l in range(L):
        assert got[l] == exp[l]["save_cks"].tolist(), f"lane {l}"
    check_final(eng, exp, range(0, L, 16))


@pytest.mark.parametrize("P,local_mask,L", [(4, 0b0011, 130), (3, 0b001, 130), (1, 0b0, 130), (4, 0b0011, 136),
                                           (3, 0b001, 136), (1, 0b0, 264)])
def test_disconnected_status_and_player_counts(oracle, P, local_mask, L):
    """InputStatus::Disconnected players spin (input 4, ex_game.rs:277-281), any player count, in
    the per-lane (L = 130) and wide (L % 8 == 0) staging forms."""
    from ggrs_amd import Engine
    calls, maxp = 60, 7
    streams = p2p_lane_streams(oracle, L, calls, P, maxp, seed=11 + P, local_mask=local_mask)
    rng = np.random.default_rng(P)
    over = []
    for s in streams:
        st = s["status"].copy()
        st[rng.random(st.shape) < 0.1] = 2  # GGRS_STATUS_DISCONNECTED
        s["st_use"] = st
        over.append(st)
    exp = expected(oracle, streams, P, maxp, status_override=over)
    eng = Engine(L, P, maxp, 0, 0)
    run_generic(eng, streams, exp, calls)
    check_final(eng, exp, (0, 1, 63, 64, 129))


def synctest_lists(inputs, f, cd, delay):
    """SyncTestSession::advance_frame's list at frame f (sync_test_session.rs:85-150), with the
    inputs each AdvanceFrame carries (input delay: frames below it hold the default input)."""
    def inp(g):
        return inputs[g - delay] if g >= delay else np.zeros(inputs.shape[1], np.uint8)
    reqs = []
    if cd > 0 and f > cd:
        reqs.append((REQ_LOAD, f - cd, None))
        for i in range(cd):
            if i > 0:
                reqs.append((REQ_SAVE, f - cd + i, None))
            reqs.append((REQ_ADVANCE, 0, inp(f - cd + i)))
    if cd > 0:
        reqs.append((REQ_SAVE, f, None))
    reqs.append((REQ_ADVANCE, 0, inp(f)))
    return reqs


def test_synctest_lists_lanes_at_different_frames(oracle):
    """SyncTest sessions that joined at different calls: one batch holds lanes at different frames;
    final states equal the oracle SyncTestSession run (which pins the lists themselves)."""
    from ggrs_amd import Engine
    L, calls, P, maxp, cd, delay = 96, 70, 2, 8, 7, 2
    ins = [oracle.gen_inputs(oracle.session_seed(l, 99), calls, P, 0) for l in range(L)]
    eng = Engine(L, P, maxp, 0, 0)
    for c in range(calls):
        reqs, off, adv = [], [0], []
        for l in range(L):
            f = c - (l % 5)
            if f >= 0:
                for k, fr, i in synctest_lists(ins[l], f, cd, delay):
                    reqs.append((k, fr))
                    if i is not None:
                        adv.append(i)
            off.append(len(reqs))
        eng.handle_requests_lanes(np.array(reqs, np.int32), np.array(off, np.int32), np.stack(adv))
    for l in (0, 1, 2, 3, 4, 50, 95):
        n = calls - (l % 5)
        r = oracle.synctest_run(ins[l][:n], P, maxp, cd, delay)
        assert bytes(eng.state(l)) == bytes(r["final_state"]), f"lane {l}"
        fr, ck, st = eng.ring(l)
        assert fr.tolist() == r["ring_frames"].tolist()
        assert ck.tolist() == r["ring_cksums"].tolist()


@pytest.mark.parametrize("L,server", [(70, True), (72, True), (72, False)])
def test_validation_fails_lanes_not_the_batch(oracle, L, server):
    """A Load of a frame the lane's cell does not hold (sync_layer.rs:248) and a Save of a frame
    other than the state's (ex_game.rs:104) fail only their lanes, which are left untouched (the
    server reports the batch's failure count with its done word)."""
    from ggrs_amd import Engine, LanesFailed
    calls, P, maxp = 30, 2, 8
    streams = p2p_lane_streams(oracle, L, calls, P, maxp, seed=21)
    eng = Engine(L, P, maxp, 0, 0)
    eng.set_lane_server(server)
    for c in range(20):
        reqs, off, inp, st, _ = call_lists(streams, c)
        eng.handle_requests_lanes(reqs, off, inp, st)
    before = {l: bytes(eng.state(l)) for l in (5, 7, 9)}
    ring_before = eng.ring(5)
    fr = eng.lane_frames()
    # lane 5: Load of a frame older than its ring holds; lane 7: Save of the wrong frame;
    # lane 9: Load(NULL_FRAME)
    reqs, off = [], [0]
    adv = []
    for l in range(L):
        if l == 5:
            reqs += [(REQ_SAVE, int(fr[l])), (REQ_LOAD, int(fr[l]) - 20), (REQ_ADVANCE, 0)]
            adv.append([1, 2])
        elif l == 7:
            reqs += [(REQ_SAVE, int(fr[l]) + 3), (REQ_ADVANCE, 0)]
            adv.append([1, 2])
        elif l == 9:
            reqs += [(REQ_LOAD, -1)]
        else:
            reqs += [(REQ_SAVE, int(fr[l])), (REQ_ADVANCE, 0)]
            adv.append([3, 4])
        off.append(len(reqs))
    with pytest.raises(LanesFailed) as ei:
        eng.handle_requests_lanes(np.array(reqs, np.int32), np.array(off, np.int32), np.array(adv, np.uint8))
    res = ei.value.lane_result
    assert ei.value.lanes.tolist() == [5, 7, 9]
    assert res[5] == -2 and res[7] == -1 and res[9] == -1
    for l in (5, 7, 9):
        assert bytes(eng.state(l)) == before[l]
    r5 = eng.ring(5)
    assert r5[0].tolist() == ring_before[0].tolist() and r5[1].tolist() == ring_before[1].tolist()
    new = eng.lane_frames()
    ok = np.ones(L, bool)
    ok[[5, 7, 9]] = False
    assert (new[ok] == fr[ok] + 1).all() and (new[~ok] == fr[~ok]).all()


def test_lane_mode_excludes_lane_uniform_calls(oracle):
    from ggrs_amd import Engine, GgrsError
    eng = Engine(8, 2, 8, 0, 0)
    reqs = np.array([(REQ_SAVE, 0), (REQ_ADVANCE, 0)] * 8, np.int32)
    eng.handle_requests_lanes(reqs, np.arange(0, 17, 2, dtype=np.int32), np.zeros((8, 2), np.uint8))
    with pytest.raises(GgrsError):
        eng.current_frame()
    with pytest.raises(GgrsError):
        eng.synctest_advance_frames(1)
    with pytest.raises(GgrsError):
        eng.handle_requests([(REQ_SAVE, 1)])
    assert eng.lane_frames().tolist() == [1] * 8


def test_lane_handler_mirror(oracle):
    """LaneBoxGameHandler: GgrsRequest objects per lane, checksums per lane back."""
    from ggrs_amd import AdvanceFrame, Engine, LaneBoxGameHandler, LoadGameState, SaveGameState
    L, calls, P, maxp = 40, 40, 2, 8
    streams = p2p_lane_streams(oracle, L, calls, P, maxp, seed=31)
    exp = expected(oracle, streams, P, maxp)
    h = LaneBoxGameHandler(Engine(L, P, maxp, 0, 0))
    got = [[] for _ in range(L)]
    for c in range(calls):
        lists = []
        for s in streams:
            x = []
            for i in np.nonzero(s["call_of"] == c)[0]:
                k = int(s["kind"][i])
                x.append(SaveGameState(int(s["frame"][i])) if k == REQ_SAVE else
                         LoadGameState(int(s["frame"][i])) if k == REQ_LOAD else
                         AdvanceFrame(s["inputs"][i], s["status"][i]))
            lists.append(x)
        for l, cks in enumerate(h.handle_requests(lists)):
            got[l].extend(cks.tolist())
    for l in range(L):
        assert got[l] == exp[l]["save_cks"].tolist()


@pytest.mark.parametrize("L,server", [(72, True), (72, False), (70, True)])
def test_batch_form_failure_count(oracle, L, server):
    """ggrs_lane_batch_run's failure count: the server's done word carries the batch's failed
    sessions (the host scans lane results only then); failed lanes keep their state, the rest run."""
    from ggrs_amd import Engine, encode_lane_lists
    P, maxp = 2, 8
    eng = Engine(L, P, maxp, 0, 0)
    eng.set_lane_server(server)
    batch = eng.lane_batch(1, 1, 2, 2)
    inp, st = np.array([1, 2], np.uint8), np.zeros(2, np.uint8)
    ok = [(REQ_SAVE, 0, None, None), (REQ_ADVANCE, 0, inp, st)]
    for c in range(3):
        enc = encode_lane_lists([[(k, c if k == REQ_SAVE else f, i, s) for k, f, i, s in ok]] * L, P)
        batch.tokens[:1], batch.inputs[:1] = enc["tokens"], enc["inputs"]
        assert batch.run(1, 0, 1, 1) == 0
        assert (batch.lane_result == c + 1).all()
    bad = {3: [(REQ_LOAD, 7, None, None)], L - 1: [(REQ_SAVE, 3, None, None), (REQ_LOAD, -1, None, None)]}
    lists = [bad.get(l, [(REQ_SAVE, 3, None, None), (REQ_ADVANCE, 0, inp, st)]) for l in range(L)]
    enc = encode_lane_lists(lists, P)
    W, LD, A, S = enc["shape"]
    batch.tokens[:W], batch.load_frames[:LD], batch.inputs[:A] = enc["tokens"], enc["load_frames"], enc["inputs"]
    assert batch.run(W, LD, A, S) == 2
    res = batch.lane_result.copy()
    assert res[3] == -1 and res[L - 1] == -2
    good = np.ones(L, bool)
    good[[3, L - 1]] = False
    assert (res[good] == 4).all()
    fr = eng.lane_frames()
    assert fr[3] == 3 and fr[L - 1] == 3 and (fr[good] == 4).all()


def test_lane_batch_shape_beyond_lds_is_rejected(oracle):
    """A batch shape whose lane block would need more LDS than a workgroup gets is GGRS_E_INVALID
    at map time (not a failed launch); the largest shapes that fit still map."""
    import ctypes
    from ggrs_amd import Engine, GgrsError
    eng = Engine(64, 2, 63, 0, 0)

    def lds(shape):
        need, lim = ctypes.c_int64(), ctypes.c_int64()
        assert eng._L.ggrs_lane_batch_lds(eng._h, *shape, ctypes.byref(need), ctypes.byref(lim)) == 0
        return need.value, lim.value

    big, small = (32, 8, 128, 256), (8, 2, 32, 32)
    # LaneLds at 2 players, ring 64: 184,832 bytes + 64 static for the big shape, over any
    # CDNA workgroup's LDS (160 KiB on gfx950); the small one well under it
    need, lim = lds(big)
    assert need == 184896 and need > lim, (need, lim)
    assert lds(small)[0] < lim
    with pytest.raises(GgrsError):
        eng.lane_batch(*big)
    b = eng.lane_batch(*small)
    b.tokens[:1] = 0xFFFFFFFF  # every lane's list empty
    assert b.run(1, 0, 0, 0) == 0
    assert (b.lane_result == 0).all()


def test_synchronize_stops_idle_server(oracle):
    """ggrs_synchronize ends an idle lane server at once (not after its 1 s idle watchdog) and the
    next batch restarts it with the lanes' states intact."""
    import time
    from ggrs_amd import Engine, encode_lane_lists
    L, calls, P, maxp = 64, 30, 2, 8
    streams = p2p_lane_streams(oracle, L, calls, P, maxp, seed=41)
    exp = expected(oracle, streams, P, maxp)
    eng = Engine(L, P, maxp, 0, 0)
    batch = eng.lane_batch(2, 2, 2 * maxp + 2, 2 * maxp + 2)
    got = [[] for _ in range(L)]
    for c in range(calls):
        lists = []
        for s in streams:
            idx = np.nonzero(s["call_of"] == c)[0]
            lists.append([(int(s["kind"][i]), int(s["frame"][i]), s["inputs"][i], s["status"][i]) for i in idx])
        enc = encode_lane_lists(lists, P)
        W, LD, A, S = enc["shape"]
        batch.tokens[:W], batch.load_frames[:LD] = enc["tokens"], enc["load_frames"]
        batch.inputs[:A], batch.status[:A] = enc["inputs"], enc["status"]
        assert batch.run(W, LD, A, S, status=True) == 0
        for l, x in enumerate(lists):
            got[l].extend(batch.checksums[:sum(1 for r in x if r[0] == REQ_SAVE), l].tolist())
        if c in (5, 17):
            t0 = time.perf_counter()
            eng.synchronize()
            assert time.perf_counter() - t0 < 0.3
    for l in range(L):
        assert got[l] == exp[l]["save_cks"].tolist(), f"lane {l}"
    check_final(eng, exp, range(0, L, 7))


def call_list_tuples(streams, c):
    """Per lane: call c's requests [(kind, frame)], and its AdvanceFrame input / status rows."""
    out = []
    for s in streams:
        idx = np.nonzero(s["call_of"] == c)[0]
        k = s["kind"][idx]
        adv = idx[k == REQ_ADVANCE]
        out.append(([(int(s["kind"][i]), int(s["frame"][i])) for i in idx], s["inputs"][adv], s["status"][adv]))
    return out


@pytest.mark.parametrize("server", [True, False])
def test_two_lane_groups_submit_wait(oracle, server):
    """A handler serving its sessions as two lane groups (two engines): group A's batch is on the
    device (ggrs_lane_batch_submit) while group B's lists are encoded (ggrs_lane_encode, the
    shared C encoder, with every Save frame checked against the lane's frame) and submitted; then
    both are collected (ggrs_lane_batch_wait).  Every Save's checksum, final state and ring equal
    the oracle handler's."""
    from ggrs_amd import Engine
    G, calls, P, maxp = 136, 60, 2, 8
    streams = p2p_lane_streams(oracle, 2 * G, calls, P, maxp, seed=23)
    exp = expected(oracle, streams, P, maxp)
    groups = [streams[:G], streams[G:]]
    engs = [Engine(G, P, maxp, 0, 0) for _ in range(2)]
    batches = []
    for e in engs:
        e.set_lane_server(server)
        batches.append(e.lane_batch(2, 2, 2 * maxp + 2, 2 * maxp + 2))
    frames = [np.zeros(G, np.int32) for _ in range(2)]
    got = [[] for _ in range(2 * G)]
    for c in range(calls):
        per = [call_list_tuples(g, c) for g in groups]
        for gi in range(2):
            b = batches[gi]
            for l, (reqs, inp, st) in enumerate(per[gi]):
                assert b.encode(l, reqs, inp, st, int(frames[gi][l])) == -1
            b.submit(status=True)
        for gi in range(2):
            b = batches[gi]
            assert b.wait() == 0
            assert (b.lane_result >= 0).all()
            frames[gi][:] = b.lane_result
            for l, (reqs, _, _) in enumerate(per[gi]):
                n = sum(1 for k, _ in reqs if k == REQ_SAVE)
                got[gi * G + l].extend(b.checksums[:n, l].tolist())
    for l in range(2 * G):
        assert got[l] == exp[l]["save_cks"].tolist(), f"lane {l}"
    check_final(engs[0], exp[:G], range(0, G, 9))
    check_final(engs[1], exp[G:], range(0, G, 9))


def test_encoder_rejects_a_bad_save_frame_on_device(oracle):
    """A Save of a frame other than the one the list reaches (ex_game.rs:104) is rejected by the
    encoder: that lane runs an empty list (state untouched), the others run."""
    from ggrs_amd import Engine
    L, P, maxp = 72, 2, 8
    eng = Engine(L, P, maxp, 0, 0)
    b = eng.lane_batch(1, 1, 2, 2)
    bad_lane = 5
    for l in range(L):
        reqs = [(REQ_SAVE, 0 if l != bad_lane else 3), (REQ_ADVANCE, 0)]
        r = b.encode(l, reqs, np.full((1, P), 1, np.uint8), None, 0)
        assert r == (0 if l == bad_lane else -1)
    b.submit()
    assert b.wait() == 0
    fr = eng.lane_frames()
    assert fr[bad_lane] == 0 and (np.delete(fr, bad_lane) == 1).all()


def test_csr_growth_invalidates_batch_views(oracle):
    """a CSR call whose list needs a larger batch re-maps (and frees) the lane batch;
    views of the old mapping are invalidated instead of writing into freed pinned memory, and a
    fresh batch runs a short list afterwards."""
    from ggrs_amd import Engine, GgrsError
    L, P, maxp = 16, 1, 8
    eng = Engine(L, P, maxp, 0, 0)
    old = eng.lane_batch(2, 1, 4, 4)
    # 100 x (Save f, Advance) per lane: 13 token words, 100 advances -- larger than the mapping
    n = 100
    reqs = np.array([(REQ_SAVE, f // 2) if f % 2 == 0 else (REQ_ADVANCE, 0) for f in range(2 * n)] * L, np.int32)
    off = np.arange(0, (L + 1) * 2 * n, 2 * n, dtype=np.int32)
    inp = np.ones((n * L, P), np.uint8)
    cks, res = eng.handle_requests_lanes(reqs, off, inp)
    assert (res == n).all()
    assert not old.valid and old.tokens is None
    with pytest.raises(GgrsError):
        old.run()
    b = eng.lane_batch(1, 1, 1, 1)
    for l in range(L):
        assert b.encode(l, [(REQ_SAVE, n), (REQ_ADVANCE, 0)], np.ones((1, P), np.uint8), None, n) == -1
    assert b.run(1, 0, 1, 1) == 0
    assert (eng.lane_frames() == n + 1).all()


@pytest.mark.parametrize("deferred", [False, True])
def test_batched_handler_cells(oracle, deferred):
    """ggrs_amd.handler.BatchedHandler (the Rust crate's BatchedBoxGame mirrored) over the engine's
    lane batch and lane server: every SaveGameState's checksum reaches its GameStateCell in request
    order -- at once, or (deferred, P2P sessions) on the next call -- and equals the oracle
    handler's (Game::handle_requests, ex_game.rs:79-127)."""
    from ggrs_amd import Engine
    from ggrs_amd.handler import BatchedHandler, GameStateCell
    L, calls, P, maxp = 128, 60, 2, 8
    streams = p2p_lane_streams(oracle, L, calls, P, maxp, seed=41)
    exp = expected(oracle, streams, P, maxp)
    eng = Engine(L, P, maxp, 0, 0)
    h = BatchedHandler(L, P, lambda shape: eng.lane_batch(*shape), deferred=deferred)
    cells = [[] for _ in range(L)]  # every saved cell of lane l, in request order
    prev = []
    for c in range(calls):
        lists, saved = [], []
        for l, s in enumerate(streams):
            x = []
            for i in np.nonzero(s["call_of"] == c)[0]:
                k, f = int(s["kind"][i]), int(s["frame"][i])
                if k == REQ_ADVANCE:
                    x.append(("advance", s["inputs"][i], s["status"][i]))
                else:
                    cell = GameStateCell()  # one cell object per request: it holds that save's value
                    x.append(("save" if k == REQ_SAVE else "load", cell, f))
                    if k == REQ_SAVE:
                        saved.append(cell)
                        cells[l].append(cell)
            lists.append(x)
        assert h.handle_requests(lists) == []
        assert all((cell.checksum is None) == deferred for cell in saved)
        assert all(cell.checksum is not None for cell in prev)  # the previous call's, collected
        prev = saved
    assert h.flush() == []
    for l in range(L):
        assert [cell.checksum for cell in cells[l]] == exp[l]["save_cks"].tolist(), f"lane {l}"
    check_final(eng, exp, range(0, L, 9))
