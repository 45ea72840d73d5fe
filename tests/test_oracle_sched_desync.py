"""CPU checks of desync detection under arrival schedules (no GPU): the two-peer oracle run
(oracle_p2p_sched_desync_pair_run) equals the fixed-latency pair run (oracle_p2p_desync_pair_run,
pinned by the reference's test_desyncs_detected) when both networks deliver at a fixed lag, and
the host-side bookkeeping (ggrs_amd.desync.SchedDesyncDetector: pending reports, local history,
comparison, p2p_session.rs:904-975, protocol.rs:663-682) fed the oracle's own per-call report rows
raises exactly the oracle's DesyncDetected events under jittered and stalled networks."""
import numpy as np
import pytest

from ggrs_amd import synth
from ggrs_amd.desync import SchedDesyncDetector


def pair_inputs(calls, P, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 16, (2, calls, P)).astype(np.uint8)


def pair_arrivals(calls, mp, seed, stalls):
    return np.stack([synth.jitter_arrivals(0, 1, calls, mp, stalls=stalls, seed=seed + k)[:, 0] for k in (0, 1)])


@pytest.mark.parametrize("L,interval,desync_frame", [(2, 10, 150), (1, 1, 40), (4, 7, 95)])
def test_uniform_schedules_equal_fixed_latency_pair(oracle, L, interval, desync_frame):
    calls, P = 300, 2
    inp = pair_inputs(calls, P, L)
    arr = np.stack([np.maximum(np.arange(calls) - L, -1)] * 2).astype(np.int32)
    full = np.zeros((calls, P), np.uint8)
    full[:, 0], full[:, 1] = inp[0, :, 0], inp[1, :, 1]
    a = oracle.p2p_desync_pair_run(full, P, 8, L, (1, 2), 0, interval, desync_peer=1, desync_frame=desync_frame)
    b = oracle.p2p_sched_desync_pair_run(inp, arr, P, 8, (1, 2), 0, interval, desync_peer=1,
                                         desync_frame=desync_frame)
    assert a["rc"] == 0 and (b["rc"] == 0).all() and a["events"]
    assert a["events"] == b["events"]
    assert (a["sent_frame"] == b["rep_frame"]).all() and (a["sent_cs"] == b["rep_cs"]).all()


class _RowsEngine:
    """An engine stand-in that serves one peer's oracle report rows (one session)."""

    def __init__(self, out, k):
        self.out, self.k, self.num_sessions, self.n = out, k, 1, 0

    def set_desync_detection(self, interval):
        pass

    def calls(self):
        return self.n

    def reports(self, first, n):
        sl = slice(first, first + n)
        return dict(frame=self.out["rep_frame"][self.k, sl, None], checksum=self.out["rep_cs"][self.k, sl, None],
                    last_confirmed=self.out["lconf"][self.k, sl, None],
                    local_last=self.out["local_last"][self.k, sl, None])


@pytest.mark.parametrize("stalls,interval,corrupt", [(False, 10, (0, 60)), (True, 7, (1, 100)), (True, 1, (0, 30)),
                                                     (False, 3, (-1, -1))])
def test_detector_bookkeeping_matches_oracle(oracle, stalls, interval, corrupt):
    calls, P, mp = 240, 2, 8
    inp = pair_inputs(calls, P, interval)
    arr = pair_arrivals(calls, mp, 5 + interval, stalls)
    out = oracle.p2p_sched_desync_pair_run(inp, arr, P, mp, (1, 2), 0, interval, corrupt_peer=corrupt[0],
                                           corrupt_call=corrupt[1])
    assert (out["rc"] == 0).all()
    engs = [_RowsEngine(out, k) for k in (0, 1)]
    dets = [SchedDesyncDetector(e, interval, addr=1 - k) for k, e in enumerate(engs)]
    for k in (0, 1):
        dets[k].note_arrivals(0, out["eff_arrive"][k][:, None])
    events = [[], []]
    for n in (17, 40, 99, calls - 156):  # chunks: exchange after each, then poll
        for e in engs:
            e.n += n
        for k in (0, 1):
            dets[1 - k].receive(*dets[k].outgoing())
        for k in (0, 1):
            events[k] += dets[k].poll()
    for k in (0, 1):
        got = [(ev.call, ev.frame, ev.local_checksum, ev.remote_checksum) for ev in events[k]]
        want = [(c, f, l, r) for (p, c, f, l, r) in out["events"] if p == k]
        assert got == want
    assert (len(out["events"]) > 0) == (corrupt[0] >= 0)
    for d in dets:  # the replayed calls' arrival rows and the delivered remote rows are dropped
        assert not d.arrive and len(d.remote) == d.remote_in - d.remote_base <= calls
        assert d.remote_base == int(d.next_remote.min())
