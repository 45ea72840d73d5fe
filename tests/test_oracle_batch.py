"""The oracle's multi-threaded batch entries (oracle_synctest_batch, oracle_p2p_batch,
oracle_p2p_replay_batch: the every-lane checkers of the full-size GPU tests and of bench.py's
parity leg) equal the single-session restatements they run per lane, lane for lane."""
import numpy as np


def test_synctest_batch_equals_single_runs(oracle):
    from ggrs_amd import synth
    P, maxp, cd, d, F, lanes = 2, 9, 8, 1, 90, 37
    inputs = synth.gen_inputs(3, lanes, F, P, synth.MODEL_HELD)
    out = oracle.synctest_batch(inputs, P, maxp, cd, d, threads=5)
    for lane in range(lanes):
        r = oracle.synctest_run(inputs[:, lane, :], P, maxp, cd, d)
        assert (out["cksum"][:, lane] == r["cksum"]).all()
        assert bytes(out["final_states"][lane]) == bytes(r["final_state"])
        assert out["ring_frames"][lane].tolist() == r["ring_frames"].tolist()
        assert out["ring_cksums"][lane].tolist() == r["ring_cksums"].tolist()
        assert out["status"][lane] == 0


def test_p2p_batch_equals_single_runs(oracle):
    from ggrs_amd import synth
    P, maxp, calls, lanes = 2, 9, 150, 23
    rows = synth.gen_inputs(5, lanes, calls, P, synth.MODEL_HELD)
    fixed = oracle.p2p_batch(rows, num_players=P, max_prediction=maxp, latency=6, threads=4)
    arrive = synth.jitter_arrivals(0, lanes, calls, maxp, stalls=True)
    sched = oracle.p2p_batch(rows, arrive, num_players=P, max_prediction=maxp, threads=3)
    for s in range(lanes):
        r = oracle.p2p_run(rows[:, s], num_players=P, max_prediction=maxp, latency=6)
        assert fixed["rc"][s] == 0 and bytes(fixed["final_states"][s]) == bytes(r["final_state"])
        assert fixed["rollbacks"][s] == r["result"].rollbacks and fixed["resim"][s] == r["result"].resim
        q = oracle.p2p_sched_run(rows[:, s], arrive[:, s], num_players=P, max_prediction=maxp)
        assert sched["rc"][s] == q["rc"] == 0 and bytes(sched["final_states"][s]) == bytes(q["final_state"])
        assert sched["rollbacks"][s] == q["result"].rollbacks
        assert sched["current_frame"][s] == q["current_frame"] and sched["skips"][s] == q["skips"]
    assert sched["skips"].sum() > 0  # the stalls hit the prediction threshold


def test_p2p_replay_batch_equals_single_replays(oracle):
    P, W, lanes = 3, 5, 17
    rng = np.random.default_rng(1)
    starts = [oracle.state_new(P)]
    for f in range(4):
        starts.append(oracle.state_advance(starts[-1], rng.integers(0, 16, P, dtype=np.uint8)))
    start = np.stack([np.frombuffer(bytes(starts[-1]), np.uint8)] * 2)
    idx = rng.integers(0, 2, lanes).astype(np.int32)
    inp = rng.integers(0, 16, (lanes, W, P), dtype=np.uint8)
    cks, st = oracle.p2p_replay_batch(start, idx, 4, inp, threads=4, states=True)
    for lane in range(lanes):
        states, ck1, _ = oracle.p2p_replay(starts[-1], 4, inp[lane])
        assert cks[lane].tolist() == [int(c) for c in ck1]
        for k in range(W):
            assert bytes(st[lane, k]) == bytes(states[k])
