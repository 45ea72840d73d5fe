"""CPU tests of the oracle's P2P desync detection (oracle_p2p_desync_pair_run): the restatement of
DesyncDetection::On{interval} (src/sessions/p2p_session.rs:281-291, :904-975) and the remote
endpoint's checksum reports (src/network/protocol.rs:27, :663-698), pinned by the reference's own
tests/test_p2p_session.rs::test_desyncs_detected (:113-210) restated on the ex_game state."""
import numpy as np
import pytest

from oracle import oracle as O


def inputs(frames, seed=5):
    return O.gen_inputs(O.session_seed(0, seed), frames, 2, 0)


@pytest.mark.parametrize("latency", [1, 2, 4])
def test_desyncs_detected_restated(latency):
    """test_p2p_session.rs:113-210: interval 100, 110 clean frames, then one peer's state goes
    wrong; after 100 more frames each peer holds exactly one DesyncDetected, at frame 200, with
    the other's checksums swapped."""
    r = O.p2p_desync_pair_run(inputs(210), latency=latency, interval=100, desync_peer=0, desync_frame=110)
    assert r["rc"] == 0
    ev = r["events"]
    assert len(ev) == 2, ev
    by_peer = {e[0]: e for e in ev}
    assert set(by_peer) == {0, 1}
    _, _, f0, l0, r0 = by_peer[0]
    _, _, f1, l1, r1 = by_peer[1]
    assert f0 == f1 == 200
    assert l0 != r0 and l1 != r1
    assert (r0, l0) == (l1, r1)


def test_no_desync_no_events_and_identical_reports():
    r = O.p2p_desync_pair_run(inputs(400), latency=3, interval=10)
    assert r["rc"] == 0 and r["events"] == []
    for k in (0, 1):
        sent = [(c, int(f)) for c, f in enumerate(r["sent_frame"][k]) if f >= 0]
        # frame_to_send = interval, 2*interval, ... goes out once confirmed and saved:
        # frame F at call F + latency + 1 (last_confirmed_frame = call - 1 - latency)
        assert sent == [(F + 3 + 1, F) for F in range(10, 400 - 4, 10)]
    assert (r["sent_cs"][0] == r["sent_cs"][1]).all()


@pytest.mark.parametrize("interval,latency,desync_frame", [(10, 3, 57), (7, 2, 0), (1, 1, 33), (16, 5, 100)])
def test_later_reports_desync(interval, latency, desync_frame):
    """A deterministic desync from frame X on one peer: exactly the report frames whose checksums
    differ between the peers raise DesyncDetected, on both peers, at call F + 2*latency + 1 (the
    report arrives latency calls after it was sent at F + latency + 1, and F <
    last_confirmed_frame already holds), the first of them being the first report frame > X
    (a ship pushed against a wall can later heal the difference, so not every later frame)."""
    frames = 300
    r = O.p2p_desync_pair_run(inputs(frames), latency=latency, interval=interval, desync_peer=1,
                              desync_frame=desync_frame)
    assert r["rc"] == 0
    sent = [{int(f): int(c) for f, c in zip(r["sent_frame"][k], r["sent_cs"][k]) if f >= 0} for k in (0, 1)]
    differ = [F for F in sorted(sent[0]) if sent[0][F] != sent[1].get(F, sent[0][F])
              and F + 2 * latency + 1 < frames]
    assert differ and differ[0] == (desync_frame // interval + 1) * interval
    for k in (0, 1):
        ev = [e for e in r["events"] if e[0] == k]
        assert [e[2] for e in ev] == differ
        assert all(e[1] == e[2] + 2 * latency + 1 for e in ev)
        assert all((e[3], e[4]) == (sent[k][e[2]], sent[1 - k][e[2]]) for e in ev)


def test_desync_detection_off():
    r = O.p2p_desync_pair_run(inputs(200), latency=2, interval=0, desync_peer=0, desync_frame=10)
    assert r["rc"] == 0 and r["events"] == [] and (r["sent_frame"] < 0).all()
