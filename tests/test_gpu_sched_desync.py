"""GPU parity of desync detection under arrival schedules (ggrs_p2p_set_desync_detection with
ggrs_p2p_set_arrival_schedule, ggrs_p2p_read_reports + ggrs_amd.desync.SchedDesyncDetector)
against the oracle's two-peer run under the same networks (oracle_p2p_sched_desync_pair_run:
check_checksum_send_interval + compare_local_checksums_against_peers per session,
p2p_session.rs:281-291, 904-975, protocol.rs:663-698).  Both machines of every match run as two
P2P engines (peer A: player 0 local, peer B: player 1 local), each session under its own jittered
network with stalls past max_prediction; in some matches one peer's input is corrupted in flight.
Every call's report (frame, checksum), the last_confirmed_frame it compared against and its last
queued frame are the oracle's, bit for bit, and so are the DesyncDetected events (frame, session,
both checksums, call) -- in the time-aligned and the one-thread-per-session kernel."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")  # loads torch's HIP runtime before the engine library

pytestmark = pytest.mark.gpu


def build_matches(oracle, S, calls, mp, interval, seed, corrupt_every=3):
    """Per session: both peers' inputs and networks, the oracle's pair run; returns the engine rows
    [2][calls][S][P], arrivals [2][calls][S] and the oracle outputs per session."""
    from ggrs_amd import synth
    P = 2
    rows = np.zeros((2, calls, S, P), np.uint8)
    arr = np.zeros((2, calls, S), np.int32)
    refs = []
    rng = np.random.default_rng(seed)
    for s in range(S):
        inp = np.stack([synth.gen_inputs(2 * s + k, 1, calls, P, synth.MODEL_HELD, base=seed)[:, 0] for k in (0, 1)])
        a = np.stack([synth.jitter_arrivals(s, 1, calls, mp, stalls=(s + k) % 2 == 0, seed=seed + k)[:, 0]
                      for k in (0, 1)])
        cp, cc = (-1, -1)
        if s % corrupt_every == 1:
            cp, cc = int(rng.integers(0, 2)), int(rng.integers(calls // 5, 3 * calls // 5))
        out = oracle.p2p_sched_desync_pair_run(inp, a, P, mp, (1, 2), 0, interval, corrupt_peer=cp, corrupt_call=cc)
        rows[:, :, s, :] = out["eff_inputs"]
        arr[:, :, s] = out["eff_arrive"]
        refs.append(out)
    return rows, arr, refs


def check_reports(eng, k, refs, calls):
    rep = eng.reports(0, calls)
    frames, skipped, errors = eng.sessions()
    for s, out in enumerate(refs):
        assert out["rc"][k] == 0 and errors[s] == 0, (s, k)
        assert (rep["frame"][:, s] == out["rep_frame"][k]).all(), (s, k)
        assert (rep["checksum"][:, s] == out["rep_cs"][k]).all(), (s, k)
        assert (rep["last_confirmed"][:, s] == out["lconf"][k]).all(), (s, k)
        assert (rep["local_last"][:, s] == out["local_last"][k]).all(), (s, k)


@pytest.mark.parametrize("form", ["chains", "flat"])
@pytest.mark.parametrize("interval,mp,chunks", [(7, 8, (17, 64, 99, 60)), (1, 6, (120, 120)), (25, 9, (240,))])
def test_sched_desync_pair_matches_oracle(oracle, monkeypatch, form, interval, mp, chunks):
    from ggrs_amd import P2PEngine
    from ggrs_amd.desync import SchedDesyncDetector
    monkeypatch.setenv("GGRS_SCHED_CHAINS", "1" if form == "chains" else "0")
    S, calls = 96, 240
    rows, arr, refs = build_matches(oracle, S, calls, mp, interval, 0x5EED + interval)
    engs, dets = [], []
    for k in (0, 1):
        e = P2PEngine(S, num_players=2, local_players=(k,), max_prediction=mp, remote_latency=1, input_capacity=calls)
        d = SchedDesyncDetector(e, interval, addr=1 - k)  # (before or after the schedule: either order)
        e.set_arrival_schedule(True)
        e.add_inputs(0, rows[k])
        e.add_arrivals(0, arr[k])
        d.note_arrivals(0, arr[k])
        engs.append(e)
        dets.append(d)
    events = [[], []]
    for n in chunks:
        for e in engs:
            e.advance_frames(n)
        for k in (0, 1):
            dets[1 - k].receive(*dets[k].outgoing())
        for k in (0, 1):
            events[k] += dets[k].poll()
    for k in (0, 1):
        check_reports(engs[k], k, refs, calls)
        got = sorted((ev.session, ev.call, ev.frame, ev.local_checksum, ev.remote_checksum) for ev in events[k])
        want = sorted((s, c, f, l, r) for s, out in enumerate(refs) for (p, c, f, l, r) in out["events"] if p == k)
        assert got == want
        assert all(ev.addr == 1 - k for ev in events[k])
    assert sum(len(out["events"]) for out in refs) > 0
    assert all(s % 3 == 1 for s, out in enumerate(refs) if out["events"])  # only the corrupted matches desync


def _sched_peer_rank(rank, port, args, out):
    import os
    import torch.distributed as dist
    from ggrs_amd import P2PEngine, exchange
    from ggrs_amd.desync import SchedDesyncDetector
    from oracle import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        S, calls, mp, interval, chunk, seed = args
        rows, arr, refs = build_matches(oracle, S, calls, mp, interval, seed)
        eng = P2PEngine(S, num_players=2, local_players=(rank,), max_prediction=mp, remote_latency=1,
                        input_capacity=calls)
        eng.set_arrival_schedule(True)
        det = SchedDesyncDetector(eng, interval, addr=exchange.peer_of(rank, 2))
        eng.add_inputs(0, rows[rank])
        eng.add_arrivals(0, arr[rank])
        det.note_arrivals(0, arr[rank])
        events, done = [], 0
        while done < calls:
            n = min(chunk, calls - done)
            eng.advance_frames(n)
            exchange.exchange_sched_reports(det)
            events += det.poll()
            done += n
        got = sorted((ev.session, ev.call, ev.frame, ev.local_checksum, ev.remote_checksum) for ev in events)
        want = sorted((s, c, f, l, r) for s, o in enumerate(refs) for (p, c, f, l, r) in o["events"] if p == rank)
        out[rank] = 1 if (got == want and len(want) > 0) else 2
    finally:
        dist.destroy_process_group()


def test_sched_peers_in_two_processes(oracle):
    """The two machines of every match in two processes (one engine each on the same GPU), their
    per-session report rows crossing a gloo process group (exchange.exchange_sched_reports): each
    process's DesyncDetected events are the oracle's."""
    import socket
    import torch.multiprocessing as mp_
    args = (64, 200, 8, 10, 45, 0xD5)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp_.get_context("spawn")
    out = ctx.Array("i", 2)
    procs = [ctx.Process(target=_sched_peer_rank, args=(r, port, args, out)) for r in (0, 1)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs)
    assert list(out) == [1, 1]
