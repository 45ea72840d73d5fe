"""GPU parity of the fused SyncTest program (ggrs_synctest_advance_frames) against the oracle.

Bit-exact, no tolerance: per-frame display checksums, final states, the saved-state ring
(frames, checksums, state bytes) and mismatch reports must equal the CPU restatement of
SyncTestSession + ex_game (oracle/ggrs_oracle.c, pinned by tests/golden/golden.json).
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))
CASES = {c["name"]: c for c in GOLDEN["synctest"]}


def lane_inputs(O, base_seed, lanes, frames, players, model):
    return np.stack([O.gen_inputs(O.session_seed(l, base_seed), frames, players, model)
                     for l in range(lanes)], axis=1)  # [frames][lanes][P]


# PIPELINED (auto: the batched v5 kernel at check_distance 8 where it packs more sessions per wave,
# else v4; sequential where a session's chains do not fit a wave), SEQUENTIAL
PATHS = [0, 1]
# every kernel at check_distance 8: auto (v5), SEQUENTIAL, PIPELINED_CHAINS (v4)
PATHS_CD8 = [0, 1, 2]


def make_engine(lanes, P, maxp, cd, d, frames, trace=True, path=0):
    from ggrs_amd import Engine
    eng = Engine(lanes, P, maxp, cd, d, input_capacity=frames + d + cd + 2,
                 trace_capacity=frames if trace else 0)
    eng.set_synctest_path(path)
    return eng


def run_chunks(eng, inputs, chunks):
    eng.add_local_inputs(0, inputs)
    done = 0
    for n in chunks:
        eng.synctest_advance_frames(n)
        done += n
    eng.synchronize()
    return done


def check_lane(O, eng, inputs, lane, P, maxp, cd, d, frames, trace=None):
    r = O.synctest_run(inputs[:, lane, :], P, maxp, cd, d)
    assert r["result"].status == 0
    if trace is not None:
        assert (trace[:, lane] == r["cksum"]).all(), f"lane {lane} trace differs at frame " \
            f"{int(np.argmax(trace[:, lane] != r['cksum']))}"
    assert bytes(eng.state(lane)) == bytes(r["final_state"]), f"lane {lane} final state"
    fr, ck, st = eng.ring(lane)
    assert fr.tolist() == r["ring_frames"].tolist()
    for s in range(len(fr)):
        if fr[s] >= 0:
            assert int(ck[s]) == int(r["ring_cksums"][s]) and bytes(st[s]) == bytes(r["ring_states"][s])


@pytest.mark.parametrize("path", PATHS_CD8)
@pytest.mark.parametrize("name", sorted(CASES))
def test_golden_cases(oracle, name, path):
    c = CASES[name]
    P, maxp, cd, d, F = c["num_players"], c["max_prediction"], c["check_distance"], c["input_delay"], c["frames"]
    lanes = 130  # three waves, the last partial
    inputs = lane_inputs(oracle, c["seed"] + 1000, lanes, F, P, c["input_model"])
    inputs[:, 0, :] = oracle.gen_inputs(c["seed"], F, P, c["input_model"])  # lane 0 = the golden session
    eng = make_engine(lanes, P, maxp, cd, d, F, path=path)
    run_chunks(eng, inputs, [1, 2, cd + 1, F - cd - 4])
    assert eng.current_frame() == F
    tr = eng.trace(0, F)
    assert tr[:, 0].tolist() == c["checksums"]
    assert bytes(eng.state(0)).hex() == c["final_state"]
    fr, ck, st = eng.ring(0)
    for s, g in enumerate(c["ring"]):
        assert fr[s] == g["frame"]
        if g["state"] is not None:
            assert bytes(st[s]).hex() == g["state"] and int(ck[s]) == g["checksum"]
    for lane in (1, 63, 64, 129):
        check_lane(oracle, eng, inputs, lane, P, maxp, cd, d, F, tr)
    st, _, _ = eng.mismatches()
    assert (st == 0).all()


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("cd", [7, 8])
@pytest.mark.parametrize("chunks", [[300], [1] * 20 + [280], [7, 13, 280], [150, 150], [9, 3, 5, 283]])
def test_chunking_is_invisible(oracle, chunks, path, cd):
    """Launch boundaries anywhere (cd 8: inside the batched kernel's 8-step batch grid too)."""
    P, maxp, d, F, lanes = 2, cd + 1, 2, 300, 64
    inputs = lane_inputs(oracle, 77, lanes, F, P, 0)
    eng = make_engine(lanes, P, maxp, cd, d, F, path=path)
    run_chunks(eng, inputs, chunks)
    tr = eng.trace(0, F)
    for lane in (0, 31, 63):
        check_lane(oracle, eng, inputs, lane, P, maxp, cd, d, F, tr)


def test_streamed_inputs_small_queue(oracle):
    """Inputs added a few frames at a time into the default 128-frame queue (InputQueue length)."""
    from ggrs_amd import Engine
    P, maxp, cd, d, F, lanes = 2, 8, 7, 2, 1000, 96
    inputs = lane_inputs(oracle, 5, lanes, F, P, 1)
    eng = Engine(lanes, P, maxp, cd, d, trace_capacity=64)
    f = 0
    while f < F:
        n = min(100, F - f)
        eng.add_local_inputs(f, inputs[f:f + n])
        # frames whose (delayed) input is queued can run; the rest wait for the next batch
        runnable = min(f + n + d, F) - eng.current_frame()
        eng.synctest_advance_frames(runnable)
        f += n
    assert eng.current_frame() == F
    tr = eng.trace(F - 64, 64)
    for lane in (0, 95):
        r = oracle.synctest_run(inputs[:, lane, :], P, maxp, cd, d)
        assert (tr[:, lane] == r["cksum"][F - 64:]).all()
        assert bytes(eng.state(lane)) == bytes(r["final_state"])


@pytest.mark.parametrize("path,chunk,call,cd", [(0, 120, 40, 7), (1, 120, 40, 7), (0, 16, 40, 7),
                                                (0, 16, 48, 7), (0, 7, 9, 7), (1, 7, 9, 7),
                                                (0, 120, 110, 7),
                                                (0, 120, 40, 8), (0, 16, 49, 8), (0, 7, 10, 8),
                                                (0, 13, 57, 8), (0, 120, 110, 8), (2, 16, 49, 8)])
def test_mismatch_detection_matches_reference(oracle, path, chunk, call, cd):
    """A non-deterministic simulation on one lane: the SyncTest must report
    MismatchedChecksum{current_frame, mismatched_frames} exactly as the reference session
    (pipelined launches detect it and are replayed on the sequential kernel from a checkpoint;
    chunk 16 puts the failure in a later launch, call 48 on a launch's first chain)."""
    from ggrs_amd import MismatchedChecksum, SessionBuilder
    P, maxp, d, F, lanes, bad_lane = 2, cd + 1, 2, 120, 70, 66
    inputs = lane_inputs(oracle, 9, lanes, F, P, 0)
    sess = (SessionBuilder().with_num_players(P).with_max_prediction_window(maxp)
            .with_check_distance(cd).with_input_delay(d).with_num_lanes(lanes)
            .with_input_capacity(F + 16).start_synctest_session())
    sess.engine.set_synctest_path(path)
    sess.engine.corrupt_on_load(bad_lane, call)
    sess.add_local_inputs(inputs)
    with pytest.raises(MismatchedChecksum) as ei:
        done = 0
        while done < F:
            n = min(chunk, F - done)
            sess.advance_frames(n, check=False)
            done += n
        sess.raise_on_mismatch()
    r = oracle.synctest_run(inputs[:, bad_lane, :], P, maxp, cd, d, corrupt_frame=call)
    assert r["result"].status == 1
    assert ei.value.current_frame == r["result"].mismatch_frame == call + 1
    mask = int(r["result"].mismatch_mask)
    assert ei.value.mismatched_frames == [call + 1 - cd + k for k in range(64) if mask >> k & 1]
    assert list(ei.value.lanes) == [bad_lane]
    st, mf, mm = sess.engine.mismatches()
    assert st[bad_lane] == 1 and mf[bad_lane] == call + 1 and int(mm[bad_lane]) == mask
    # the halted lane keeps the state the reference session had when it returned Err
    assert bytes(sess.engine.state(bad_lane)) == bytes(r["final_state"])
    fr, ck, sts = sess.engine.ring(bad_lane)
    for s in range(len(fr)):
        assert int(ck[s]) == int(r["ring_cksums"][s]) and bytes(sts[s]) == bytes(r["ring_states"][s])
    # every other lane ran to the end
    assert (st[np.arange(lanes) != bad_lane] == 0).all()
    check_lane(oracle, sess.engine, inputs, bad_lane - 1, P, maxp, cd, d, F)


@pytest.mark.parametrize("lanes,bad_lane,call,cd", [(16384, 16383, 30, 7), (16384, 0, 30, 7), (12000, 6001, 77, 7),
                                                    (40000, 39999, 31, 8), (40000, 17, 77, 8)])
def test_mismatch_restore_when_grid_exceeds_residency(oracle, lanes, bad_lane, call, cd):
    """A mismatch in a launch whose grid has more blocks than fit the chip at once: blocks
    scheduled after the failing one must still take their launch checkpoint (they used
    to skip it and be restored from a stale shadow).  Every lane other than the corrupted one ends
    in the oracle's state; the corrupted lane halts exactly as the reference's session."""
    from ggrs_amd import MismatchedChecksum, SessionBuilder
    P, maxp, d, F = 2, cd + 1, 0, 120
    rng = np.random.default_rng(lanes + call)
    inputs = rng.integers(0, 16, (F, lanes, P), dtype=np.uint8)
    sess = (SessionBuilder().with_num_players(P).with_max_prediction_window(maxp).with_check_distance(cd)
            .with_input_delay(d).with_num_lanes(lanes).with_input_capacity(F + 16).start_synctest_session())
    sess.engine.corrupt_on_load(bad_lane, call)
    sess.add_local_inputs(inputs)
    sess.advance_frames(cd + 1, check=False)  # warm-up launch
    sess.advance_frames(F - cd - 1, check=False)  # one pipelined launch that fails
    with pytest.raises(MismatchedChecksum) as ei:
        sess.raise_on_mismatch()
    assert list(ei.value.lanes) == [bad_lane]
    r = oracle.synctest_run(inputs[:, bad_lane, :], P, maxp, cd, d, corrupt_frame=call)
    assert ei.value.current_frame == r["result"].mismatch_frame
    assert bytes(sess.engine.state(bad_lane)) == bytes(r["final_state"])
    for lane in sorted({0, 1, lanes // 2, lanes - 1, (bad_lane + 1) % lanes} - {bad_lane}):
        check_lane(oracle, sess.engine, inputs, lane, P, maxp, cd, d, F)


@pytest.mark.parametrize("path", PATHS_CD8)
def test_full_size_config2(oracle, path):
    """Config 2 at full size: 4096 sessions, 8-frame rollback every frame (SyncTest cd 8,
    max_prediction 9), held-key inputs.  EVERY lane bit-exact against the oracle's SyncTestSession
    (oracle_synctest_batch): the display checksum after every frame, the final state and the
    saved-state ring's frames and checksums; sampled lanes' ring state bytes too."""
    from ggrs_amd import synth
    P, maxp, cd, d, F, lanes = 2, 9, 8, 0, 400, 4096
    inputs = synth.gen_inputs(0, lanes, F, P, synth.MODEL_HELD)
    eng = make_engine(lanes, P, maxp, cd, d, F, path=path)
    run_chunks(eng, inputs, [F])
    ref = oracle.synctest_batch(inputs, P, maxp, cd, d)
    assert (ref["status"] == 0).all()
    tr = eng.trace(0, F)
    bad = np.nonzero((tr != ref["cksum"]).any(axis=0))[0]
    assert bad.size == 0, f"{bad.size} lanes' traces differ, first {bad[:8].tolist()}"
    states = eng.states()
    bad = np.nonzero((states != ref["final_states"]).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} lanes' final states differ, first {bad[:8].tolist()}"
    ring_frames = ref["ring_frames"][0]
    assert (ref["ring_frames"] == ring_frames).all()  # SyncTest lanes step in lockstep
    held = [(slot, int(f)) for slot, f in enumerate(ring_frames) if f >= 0]
    cks = eng.save_checksums_frames([f for _, f in held])
    for i, (slot, f) in enumerate(held):
        assert (cks[i] == ref["ring_cksums"][:, slot]).all(), f"ring checksum of frame {f}"
    for lane in (0, 4095):
        check_lane(oracle, eng, inputs, lane, P, maxp, cd, d, F, tr)
    st, _, _ = eng.mismatches()
    assert (st == 0).all()


@pytest.mark.parametrize("path", PATHS_CD8)
@pytest.mark.parametrize("lanes,P", [(67, 2), (37, 4), (10, 3), (13, 1)])
def test_ragged_last_block_every_lane(oracle, path, lanes, P):
    """Lane counts that leave the last workgroup partly empty (idle lanes there map past the
    last session): every lane's trace and final state bit-exact, across an input restage."""
    maxp, cd, d, F = 9, 8, 1, 300
    inputs = lane_inputs(oracle, 11, lanes, F, P, 0)
    eng = make_engine(lanes, P, maxp, cd, d, F, path=path)
    run_chunks(eng, inputs, [F])
    tr = eng.trace(0, F)
    for lane in range(lanes):
        check_lane(oracle, eng, inputs, lane, P, maxp, cd, d, F, tr)


@pytest.mark.parametrize("path", PATHS)
def test_max_ring_and_four_players(oracle, path):
    P, maxp, cd, d, F, lanes = 4, 63, 62, 0, 200, 64
    inputs = lane_inputs(oracle, 3, lanes, F, P, 0)
    eng = make_engine(lanes, P, maxp, cd, d, F, path=path)
    run_chunks(eng, inputs, [F])
    tr = eng.trace(0, F)
    for lane in (0, 63):
        check_lane(oracle, eng, inputs, lane, P, maxp, cd, d, F, tr)


def test_missing_input_is_invalid_request(oracle):
    from ggrs_amd import Engine, InvalidRequest
    eng = Engine(8, 2, 8, 2, 0)
    eng.add_local_inputs(0, np.zeros((5, 8, 2), np.uint8))
    eng.synctest_advance_frames(5)
    with pytest.raises(InvalidRequest, match="Missing local input"):
        eng.synctest_advance_frames(1)
    with pytest.raises(InvalidRequest, match="sequentially"):
        eng.add_local_inputs(7, np.zeros((1, 8, 2), np.uint8))
    with pytest.raises(InvalidRequest, match="queue full"):
        eng.add_local_inputs(5, np.zeros((200, 8, 2), np.uint8))


def test_per_frame_api(oracle):
    """add_local_input(handle, lanes) + advance_frame(), one frame at a time, as ex_game_synctest."""
    from ggrs_amd import SessionBuilder
    P, F, lanes = 2, 40, 16
    inputs = lane_inputs(oracle, 11, lanes, F, P, 0)
    sess = (SessionBuilder().with_num_players(P).with_check_distance(7).with_input_delay(2)
            .with_max_prediction_window(8).with_num_lanes(lanes).start_synctest_session())
    for f in range(F):
        for p in range(P):
            sess.add_local_input(p, inputs[f, :, p])
        sess.advance_frame()
    for lane in (0, 15):
        r = oracle.synctest_run(inputs[:, lane, :], P, 8, 7, 2)
        assert bytes(sess.engine.state(lane)) == bytes(r["final_state"])


def test_advance_frame_reports_mismatch_before_missing_input(oracle):
    """SyncTestSession::advance_frame returns MismatchedChecksum (sync_test_session.rs:89-102)
    before it checks for missing local input (:108-113): a lane that halted in an unchecked launch
    is reported by the next advance_frame even when that call has no inputs; the call after it
    (mismatch already reported) raises the missing-input InvalidRequest."""
    from ggrs_amd import InvalidRequest, MismatchedChecksum, SessionBuilder
    P, maxp, cd, F, lanes = 2, 8, 7, 40, 64
    inputs = lane_inputs(oracle, 4, lanes, F, P, 0)
    sess = (SessionBuilder().with_num_players(P).with_max_prediction_window(maxp).with_check_distance(cd)
            .with_num_lanes(lanes).with_input_capacity(F + 16).start_synctest_session())
    sess.engine.corrupt_on_load(5, 20)
    sess.add_local_inputs(inputs)
    sess.advance_frames(F, check=False)
    with pytest.raises(MismatchedChecksum) as ei:
        sess.advance_frame()  # no pending local input
    assert list(ei.value.lanes) == [5]
    with pytest.raises(InvalidRequest):
        sess.advance_frame()
