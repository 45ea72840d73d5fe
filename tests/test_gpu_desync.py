"""GPU parity of P2P desync detection (ggrs_p2p_set_desync_detection / local_checksums /
compare_checksums + ggrs_amd/desync.py) against the oracle's two-peer run
(oracle_p2p_desync_pair_run: check_checksum_send_interval + compare_local_checksums_against_peers,
p2p_session.rs:904-975, protocol.rs:663-698): both machines of every match run on the GPU as two
P2P engines (peer A: player 0 local, peer B: player 1 local); the reports each peer sends and the
DesyncDetected events each raises (frame, session, checksums, call) are exactly the oracle's."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")  # loads torch's HIP runtime before the engine library

pytestmark = pytest.mark.gpu


def stream(S, frames, P, seed_base=0x6464):
    from oracle import oracle as o
    return np.stack([o.gen_inputs(o.session_seed(s, seed_base), frames, P, 0) for s in range(S)], axis=1)


def run_pair(S, frames, D, mp, interval, chunk, desync=None):
    from ggrs_amd import P2PEngine
    from ggrs_amd.desync import DesyncDetector, exchange
    rows = stream(S, frames, 2)
    engs = [P2PEngine(S, num_players=2, local_players=(k,), max_prediction=mp, remote_latency=D,
                      input_capacity=frames + 16)
            for k in (0, 1)]
    dets = [DesyncDetector(e, interval, addr=1 - k) for k, e in enumerate(engs)]
    if desync is not None:
        sess, frame = desync
        engs[1].debug_desync(sess, frame)
    for e in engs:
        e.add_inputs(0, rows)
    events = [[], []]
    done = 0
    while done < frames:
        n = min(chunk, frames - done)
        for e in engs:
            e.advance_frames(n)
        exchange(dets[0], dets[1])
        for k in (0, 1):
            events[k] += dets[k].poll()
        done += n
    return rows, engs, events


@pytest.mark.parametrize("interval,D,chunk", [(10, 2, 37), (1, 1, 16), (7, 3, 64), (100, 4, 105)])
def test_desync_events_match_oracle(oracle, interval, D, chunk):
    S, frames, mp = 200, 320, 8
    bad, X = 77, 123
    rows, engs, events = run_pair(S, frames, D, mp, interval, chunk, desync=(bad, X))
    ref = oracle.p2p_desync_pair_run(rows[:, bad], latency=D, max_prediction=mp, interval=interval,
                                     desync_peer=1, desync_frame=X)
    assert ref["rc"] == 0 and ref["events"]
    for k in (0, 1):
        got = [(ev.call, ev.frame, ev.local_checksum, ev.remote_checksum) for ev in events[k]]
        want = [(c, f, l, r) for (p, c, f, l, r) in ref["events"] if p == k]
        assert all(ev.session == bad and ev.addr == 1 - k for ev in events[k])
        assert got == want
    # every other session: both peers' reports identical (spot-check one frame) and no events
    last = ((frames - 2 - D) // interval) * interval
    a, b = engs[0].local_checksums(last), engs[1].local_checksums(last)
    differ = np.nonzero(a != b)[0].tolist()
    assert set(differ) <= {bad}


def test_reports_equal_oracle_and_no_events_without_desync(oracle):
    S, frames, D, mp, interval = 64, 200, 3, 8, 10
    rows, engs, events = run_pair(S, frames, D, mp, interval, 50)
    assert events == [[], []]
    for s in (0, 31, 63):
        ref = oracle.p2p_desync_pair_run(rows[:, s], latency=D, max_prediction=mp, interval=interval)
        sent = {int(f): int(c) for f, c in zip(ref["sent_frame"][0], ref["sent_cs"][0]) if f >= 0}
        newest = frames - 2 - D
        for F, cs in sent.items():
            if F > newest - 32 * interval:  # still in the 32-report history
                assert int(engs[0].local_checksums(F)[s]) == cs
                assert int(engs[1].local_checksums(F)[s]) == cs


def test_history_bounds_are_preconditions():
    from ggrs_amd import P2PEngine, PreconditionError
    e = P2PEngine(8, num_players=2, local_players=(0,), max_prediction=8, remote_latency=2, input_capacity=320)
    e.set_desync_detection(5)
    e.add_inputs(0, np.zeros((300, 8, 2), np.uint8))
    e.advance_frames(300)
    with pytest.raises(PreconditionError):
        e.local_checksums(7)          # not a report frame
    with pytest.raises(PreconditionError):
        e.local_checksums(300)        # not reported yet
    with pytest.raises(PreconditionError):
        e.local_checksums(5)          # left the 32-report history
    e.local_checksums(290)            # newest report: frame 295 (call 298); 290 still held
    with pytest.raises(Exception):
        e.set_desync_detection(10)    # configuration: before the first call only


def _peer_rank(rank, port, args, out):
    import os
    import torch.distributed as dist
    from ggrs_amd import P2PEngine, exchange
    from ggrs_amd.desync import DesyncDetector
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        S, frames, D, mp, interval, chunk, bad, X = args
        rows = stream(S, frames, 2)
        eng = P2PEngine(S, num_players=2, local_players=(rank,), max_prediction=mp, remote_latency=D,
                        input_capacity=frames + 16)
        det = DesyncDetector(eng, interval, addr=exchange.peer_of(rank, 2))
        if rank == 1:
            eng.debug_desync(bad, X)
        eng.add_inputs(0, rows)
        events, done = [], 0
        while done < frames:
            n = min(chunk, frames - done)
            eng.advance_frames(n)
            exchange.exchange_p2p_reports(det)
            events += det.poll()
            done += n
        for k, ev in enumerate(events[:60]):
            out[rank * 300 + 5 * k: rank * 300 + 5 * k + 5] = [ev.call, ev.frame, ev.local_checksum,
                                                               ev.remote_checksum, ev.session]
        out[600 + rank] = len(events)
    finally:
        dist.destroy_process_group()


def test_peers_in_two_processes_over_process_group(oracle):
    """The two machines of every match in two processes (one P2P engine each on the same GPU),
    their checksum reports crossing a gloo process group (exchange.exchange_p2p_reports, the path
    the multi-GPU bench takes over RCCL): the DesyncDetected events are the oracle's."""
    import socket
    import torch.multiprocessing as mp_
    S, frames, D, mp, interval, chunk, bad, X = 96, 240, 2, 8, 10, 40, 17, 91
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp_.get_context("spawn")
    out = ctx.Array("i", 602)
    procs = [ctx.Process(target=_peer_rank, args=(r, port, (S, frames, D, mp, interval, chunk, bad, X), out))
             for r in (0, 1)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs)
    rows = stream(S, frames, 2)
    ref = oracle.p2p_desync_pair_run(rows[:, bad], latency=D, max_prediction=mp, interval=interval,
                                     desync_peer=1, desync_frame=X)
    for k in (0, 1):
        n = out[600 + k]
        got = [tuple(out[k * 300 + 5 * i: k * 300 + 5 * i + 5]) for i in range(min(n, 60))]
        want = [(c, f, l, r, bad) for (p, c, f, l, r) in ref["events"] if p == k]
        assert n == len(want) and got == want[:60]
