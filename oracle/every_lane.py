"""Every-lane checks of a full-size run against the oracle's batch entries.  TEST INFRASTRUCTURE
ONLY: used by tests/ and bench.py's parity leg, as the checker, never by the product.

Each function runs the oracle's restatement for every lane of an engine (oracle_synctest_batch,
oracle_p2p_batch, oracle_p2p_replay_batch on the job's CPU share) and returns a dict whose
"*_mismatched" entries count the lanes that differ (all 0 when the engine is bit-exact) plus the
number of lanes compared."""
import numpy as np

from . import oracle as O


def synctest(eng, inputs, P, maxp, cd, delay, trace_first=None, trace_n=0):
    """SyncTestSession (sync_test_session.rs:173-217) on every lane of `inputs[frames][lanes][P]`:
    final state, the saved ring's checksums and, when trace_n > 0, the display checksums of
    frames trace_first .. trace_first + trace_n - 1."""
    ref = O.synctest_batch(inputs, P, maxp, cd, delay, trace=trace_n > 0)
    out = {"lanes": int(inputs.shape[1]), "status_mismatched": int((ref["status"] != 0).sum())}
    out["final_state_mismatched"] = int((eng.states() != ref["final_states"]).any(axis=1).sum())
    held = [(slot, int(f)) for slot, f in enumerate(ref["ring_frames"][0]) if f >= 0]
    bad_ring = ~(ref["ring_frames"] == ref["ring_frames"][0]).all(axis=1)
    cks = eng.save_checksums_frames([f for _, f in held])
    for i, (slot, _) in enumerate(held):
        bad_ring |= cks[i] != ref["ring_cksums"][:, slot]
    out["ring_checksum_mismatched"] = int(bad_ring.sum())
    if trace_n:
        tr = eng.trace(trace_first, trace_n)
        out["trace_mismatched"] = int((tr != ref["cksum"][trace_first:trace_first + trace_n]).any(axis=0).sum())
    return out


def p2p(eng, rows, arrive=None, P=2, local_mask=0b01, maxp=8, latency=4, sparse=False):
    """One peer's P2PSession (p2p_session.rs:304-339, 658-714) on every session: final state and
    rollback count, and under an arrival schedule the current frame and skipped calls."""
    ref = O.p2p_batch(rows, arrive, num_players=P, local_mask=local_mask, max_prediction=maxp, latency=latency,
                      sparse_saving=sparse)
    S = rows.shape[1]
    out = {"lanes": int(S), "rc_mismatched": int((ref["rc"] != 0).sum())}
    out["final_state_mismatched"] = int((eng.states() != ref["final_states"]).any(axis=1).sum())
    rb, _ = eng.stats()
    out["rollbacks_mismatched"] = int((rb != ref["rollbacks"]).sum())
    if arrive is not None:
        fr, sk, er = eng.sessions()
        out["frame_skips_mismatched"] = int(((fr != ref["current_frame"]) | (sk != ref["skips"]) | (er != 0)).sum())
    return out


def branch_inputs_all(eng, truth, f_c, W):
    """The inputs every lane of a branch engine plays from trunk frame f_c: [lanes][W][P] (the
    host restatement of the device generator: the first remote player enumerates the branch's
    base-alphabet digits, further remote players repeat their last confirmed input)."""
    S, B, P, A = eng.num_sessions, eng.branches, eng.num_players, eng.alphabet
    lane = np.arange(S * B)
    sess, br = lane // B, lane % B
    last = truth[f_c - 1] if f_c > 0 else np.zeros((S, P), np.uint8)
    E, v = 0, 1
    while v < B:
        v *= A
        E += 1
    first_remote = next(q for q in range(P) if eng.remote_mask >> q & 1)
    out = np.empty((S * B, W, P), np.uint8)
    for k in range(W):
        for q in range(P):
            if not eng.remote_mask >> q & 1:
                out[:, k, q] = truth[f_c + k, sess, q]
            elif q == first_remote and B > 1:
                out[:, k, q] = (br // A ** min(k, E - 1)) % A
            else:
                out[:, k, q] = last[sess, q]
    return out


def branch(eng, truth, states=True):
    """After n rounds (trunk frame n): every lane's last speculated window (the cells of frames
    n .. n + W - 1) against adjust_gamestate's replay (p2p_session.rs:658-714) from the confirmed
    trunk of frame n - 1 with that lane's inputs; every session's report checksum against
    fletcher16 of the oracle's trunk; every survival bit against "assumed the confirmed inputs"."""
    S, B, P, W = eng.num_sessions, eng.branches, eng.num_players, eng.window
    n = eng.trunk_frame()
    zero = np.frombuffer(bytes(O.state_new(P)), np.uint8)[None]
    _, tst = O.p2p_replay_batch(zero, np.zeros(S, np.int32), 0, np.ascontiguousarray(truth[:n].transpose(1, 0, 2)),
                                states=True)
    start = tst[:, n - 2] if n >= 2 else np.repeat(zero, S, axis=0)
    ins = branch_inputs_all(eng, truth, n - 1, W)
    sess = (np.arange(S * B) // B).astype(np.int32)
    cks, sts = O.p2p_replay_batch(start, sess, n - 1, ins, states=states)
    bad = np.zeros(S * B, bool)
    for k in range(W):
        ck, st = eng.cells(n + k, states=states)
        bad |= ck != cks[:, k]
        if states:
            bad |= (st != sts[:, k]).any(axis=1)
    ck, _ = eng.report()
    want = np.array([O.fletcher16(bytes(tst[s, n - 1])) for s in range(S)], np.uint16)
    surv = (ins[:, 0, :] == truth[n - 1, sess]).all(axis=1)
    return {"lanes": int(S * B), "cells_mismatched": int(bad.sum()), "first_bad_lane": int(np.argmax(bad)) if bad.any() else -1,
            "report_mismatched": int((ck != want).sum()), "survivors_mismatched": int((eng.survivors() != surv).sum()),
            "desyncs": int((eng.desync() >= 0).sum()), "trunk_states": tst[:, n - 1]}
