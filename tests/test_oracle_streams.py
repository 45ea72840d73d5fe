"""The oracle's per-lane request streams (oracle_p2p_stream) and request handler
(oracle_handler_run), the checkers of tests/test_gpu_lane_requests.py.  CPU only.

Pinned by: the P2P session restatement it shares with oracle_p2p_run (a delivery schedule of one
frame per call at latency D must reproduce oracle_p2p_run exactly), the reference's list grammar
(p2p_session.rs:304-339,658-714: [Save 0] [Load first_incorrect (Save?, Advance)*] Save current
Advance), and SyncTestSession's own request stream (a handler run over the lists of
sync_test_session.rs:85-150 must end in oracle_synctest_run's state and ring)."""
import numpy as np
import pytest

from oracle import oracle as o

REQ_SAVE, REQ_LOAD, REQ_ADVANCE = 0, 1, 2


@pytest.mark.parametrize("latency,sparse", [(1, False), (4, False), (7, False), (3, True)])
def test_fixed_latency_schedule_is_p2p_run(oracle, latency, sparse):
    inp = o.gen_inputs(o.session_seed(5), 400, 2, 1)
    upto = (np.arange(400) - latency).astype(np.int32)
    s = o.p2p_stream(inp, upto, max_prediction=8, sparse_saving=sparse)
    r = o.p2p_run(inp, latency=latency, max_prediction=8, sparse_saving=sparse)
    assert s["rc"] == 0 and r["rc"] == 0
    assert s["result"].rollbacks == r["result"].rollbacks and s["result"].resim == r["result"].resim
    h = o.handler_run(s["kind"], s["frame"], s["inputs"], s["status"], 2, 8)
    assert h["rc"] == 0
    assert bytes(h["final_state"]) == bytes(r["final_state"])
    assert h["ring_frames"].tolist() == r["ring_frames"].tolist()
    assert h["ring_cksums"].tolist() == r["ring_cksums"].tolist()


def test_jitter_lists_follow_the_reference_grammar(oracle):
    maxp = 8
    inp = o.gen_inputs(o.session_seed(9), 500, 2, 1)
    s = o.p2p_stream(inp, o.jitter_schedule(500, maxp, 3), max_prediction=maxp)
    assert s["rc"] == 0 and s["calls"] == 500
    depths = set()
    for f in range(500):
        k = s["kind"][s["call_off"][f]:s["call_off"][f + 1]].tolist()
        fr = s["frame"][s["call_off"][f]:s["call_off"][f + 1]].tolist()
        if f == 0:
            assert k[:1] == [REQ_SAVE] and fr[0] == 0  # :305-308
            k, fr = k[1:], fr[1:]
        if k[0] == REQ_LOAD:
            load = fr[0]
            assert f - maxp <= load < f  # sync_layer.rs:231-248
            depths.add(f - load)
            n = f - load
            # (Save?, Advance) x n: every replayed frame but the loaded one is saved (:698-702)
            body = k[1:1 + 2 * n - 1]
            assert body == [REQ_ADVANCE] + [REQ_SAVE, REQ_ADVANCE] * (n - 1)
            k, fr = k[2 * n:], fr[2 * n:]
        assert k == [REQ_SAVE, REQ_ADVANCE] and fr[0] == f  # :337, :393-423
    assert len(depths) >= 4  # bursts give rollbacks of differing depth
    h = o.handler_run(s["kind"], s["frame"], s["inputs"], s["status"], 2, maxp)
    assert h["rc"] == 0 and len(h["save_cks"]) == int((s["kind"] == REQ_SAVE).sum())


def synctest_stream(inputs, frames, cd, delay):
    kind, frame, adv = [], [], []

    def inp(g):
        return inputs[g - delay] if g >= delay else np.zeros(inputs.shape[1], np.uint8)
    for f in range(frames):
        if cd > 0 and f > cd:
            kind.append(REQ_LOAD)
            frame.append(f - cd)
            adv.append(np.zeros(inputs.shape[1], np.uint8))
            for i in range(cd):
                if i > 0:
                    kind.append(REQ_SAVE)
                    frame.append(f - cd + i)
                    adv.append(np.zeros(inputs.shape[1], np.uint8))
                kind.append(REQ_ADVANCE)
                frame.append(0)
                adv.append(inp(f - cd + i))
        if cd > 0:
            kind.append(REQ_SAVE)
            frame.append(f)
            adv.append(np.zeros(inputs.shape[1], np.uint8))
        kind.append(REQ_ADVANCE)
        frame.append(0)
        adv.append(inp(f))
    return np.array(kind, np.int32), np.array(frame, np.int32), np.stack(adv)


@pytest.mark.parametrize("P,cd,delay", [(2, 7, 2), (4, 3, 0), (1, 2, 1)])
def test_handler_over_synctest_stream_is_synctest_run(oracle, P, cd, delay):
    frames, maxp = 200, 8
    inputs = o.gen_inputs(o.session_seed(17), frames, P, 0)
    k, f, a = synctest_stream(inputs, frames, cd, delay)
    h = o.handler_run(k, f, a, None, P, maxp)
    r = o.synctest_run(inputs, P, maxp, cd, delay)
    assert h["rc"] == 0 and r["result"].status == 0
    assert bytes(h["final_state"]) == bytes(r["final_state"])
    assert h["ring_frames"].tolist() == r["ring_frames"].tolist()
    assert h["ring_cksums"].tolist() == r["ring_cksums"].tolist()


def test_handler_rejects_what_the_reference_panics_on(oracle):
    z = np.zeros((4, 2), np.uint8)
    # Save of a frame other than the state's (ex_game.rs:104)
    assert o.handler_run([REQ_SAVE], [1], z[:1])["rc"] == -1
    # Load of a frame no cell holds (sync_layer.rs:248)
    assert o.handler_run([REQ_SAVE, REQ_ADVANCE, REQ_LOAD], [0, 0, 1], z[:3])["rc"] == -3
    # a valid Load
    assert o.handler_run([REQ_SAVE, REQ_ADVANCE, REQ_LOAD, REQ_ADVANCE], [0, 0, 0, 0], z)["rc"] == 0
