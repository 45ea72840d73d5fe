"""Multi-rank exchange of confirmation reports over gloo on CPU (world size 2 and 4): the
all-gather returns every rank's report in rank order, peers are paired across the world, and a
differing session checksum between peer replicas becomes DesyncDetected (p2p_session.rs:904-937)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ggrs_amd import exchange

S, L = 37, 37 * 16


def fake_report(rank, frame, corrupt_session=None):
    ck_bytes, words, total = exchange.report_layout(S, L)
    # every replica of a session computes the same checksum, so peers (rank, rank + w/2) agree
    ck = np.random.default_rng(1000 * frame).integers(0, 65535, S).astype(np.uint16)
    if corrupt_session is not None:
        ck[corrupt_session] ^= 0x5A5A
    bits = np.random.default_rng(rank).integers(0, 2 ** 63, words, dtype=np.uint64)
    buf = np.zeros(total, np.uint8)
    buf[:2 * S] = ck.view(np.uint8)
    buf[ck_bytes:] = bits.view(np.uint8)
    return buf


def worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        for frame in range(3):
            corrupt = 5 if (frame == 2 and rank == 0) else None
            local = torch.from_numpy(fake_report(rank, frame, corrupt))
            g = exchange.allgather_reports(local)
            assert g.shape == (world, local.numel())
            for r in range(world):
                want = fake_report(r, frame, 5 if (frame == 2 and r == 0) else None)
                assert (g[r].numpy() == want).all()
            ev = exchange.desyncs_against_peer(g, rank, world, frame, S, L)
            pr = exchange.peer_of(rank, world)
            if frame == 2 and (rank == 0 or pr == 0):
                assert [e.session for e in ev] == [5] and ev[0].addr == pr
                assert ev[0].local_checksum != ev[0].remote_checksum
            else:
                assert ev == []
        out[rank] = 1
    finally:
        dist.destroy_process_group()


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 4])
def test_allgather_and_desync_gloo(world):
    ctx = mp.get_context("spawn")
    out = ctx.Array("i", world)
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert list(out) == [1] * world


def test_split_report_roundtrip():
    buf = fake_report(0, 1)
    ck, bits = exchange.split_report(buf, S, L)
    assert ck.size == S and bits.size == (L + 63) // 64


class FakeP2PEngine:
    """The parts of P2PEngine a DesyncDetector reads: checksum reports per frame (a deterministic
    function of frame and session, the same on both peers except one corrupted session)."""

    max_prediction = 8

    def __init__(self, sessions, latency, corrupt=None):
        self.num_sessions, self.remote_latency, self.frame, self.corrupt = sessions, latency, 0, corrupt

    def set_desync_detection(self, interval):
        self.interval = interval

    def current_frame(self):
        return self.frame

    def calls(self):
        return self.frame

    def local_checksums(self, frame, out=None):
        ck = np.random.default_rng(77 + frame).integers(0, 65536, self.num_sessions).astype(np.uint16)
        if self.corrupt is not None and frame >= self.corrupt[1]:
            ck[self.corrupt[0]] ^= 0x8001
        if out is not None:
            out.copy_(torch.from_numpy(ck.view(np.int16)))
            return out
        return ck

    def compare_checksums(self, frame, remote):
        remote = remote.cpu().numpy().view(np.uint16) if hasattr(remote, "cpu") else np.asarray(remote, np.uint16)
        return np.nonzero(self.local_checksums(frame) != remote)[0]


def p2p_worker(rank, world, port, out):
    from ggrs_amd.desync import DesyncDetector
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        interval, latency = 10, 3
        # rank 0's session 4 desyncs from frame 40 on; its peer sees the same event
        eng = FakeP2PEngine(23, latency, corrupt=(4, 40) if rank == 0 else None)
        det = DesyncDetector(eng, interval, addr=exchange.peer_of(rank, world))
        events = []
        for _ in range(8):  # 8 batches of 16 calls, one collective per batch
            eng.frame += 16
            exchange.exchange_p2p_reports(det)
            events += det.poll()
        pr = exchange.peer_of(rank, world)
        if rank == 0 or pr == 0:
            assert {e.session for e in events} == {4}
            assert min(e.frame for e in events) == 40
            assert all(e.addr == pr and e.local_checksum != e.remote_checksum for e in events)
        else:
            assert events == []
        out[rank] = 1
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_p2p_reports_between_peers_gloo(world):
    """P2P checksum reports travel between the two peers of each match through the process group;
    a session whose checksums diverge raises DesyncDetected on both peers, no other rank sees one."""
    ctx = mp.get_context("spawn")
    out = ctx.Array("i", world)
    port = free_port()
    procs = [ctx.Process(target=p2p_worker, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert list(out) == [1] * world


class FakeBranchEngine:
    """The parts of BranchEngine a ReportExchange drives: round_to_tensor / trunk_frame and the
    report shape.  Reports are a deterministic function of (frame, rank):
    session checksums agree between peer replicas except a corrupted session from `corrupt`
    on; survival words differ per rank.  `log` records the call order."""

    def __init__(self, rank, corrupt=None):
        self.num_sessions, self.num_lanes = S, L
        self.report_bytes = exchange.report_layout(S, L)[2]
        self.rank, self.frame, self.corrupt, self.log = rank, 0, corrupt, []

    def trunk_frame(self):
        return self.frame

    def expected(self, rank, frame):
        c = None
        if self.corrupt is not None and rank == self.corrupt[2] and frame >= self.corrupt[1]:
            c = self.corrupt[0]
        return fake_report(rank, frame, c)

    def round_to_tensor(self, t):
        self.log.append(("round", self.frame))
        t.copy_(torch.from_numpy(self.expected(self.rank, self.frame)))
        self.frame += 1


def report_exchange_worker(rank, world, port, out, batch=1):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank 0's session 7 desyncs from round 5 on: rank 0 and its peer count it every round
        eng = FakeBranchEngine(rank, corrupt=(7, 5, 0))
        ex = exchange.ReportExchange(eng, peers=True, keep_history=True, batch=batch)
        rounds = 9
        for _ in range(rounds):
            ex.step()
        ex.drain()
        # one fused round call per round, in order
        assert eng.log == [("round", r) for r in range(rounds)]
        # every round's gathered reports, in round order, hold every rank's report
        assert [f for f, _ in ex.history] == list(range(rounds))
        for f, g in ex.history:
            for r in range(world):
                assert (g[r].numpy() == eng.expected(r, f)).all(), (f, r)
        pr = exchange.peer_of(rank, world)
        involved = rank == 0 or pr == 0
        assert int(ex.desync_count) == ((rounds - 5) if involved else 0)
        assert int(ex.first_desync_round) == (5 if involved else -1)
        out[rank] = 1
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,batch", [(2, 1), (4, 1), (2, 4), (4, 3), (2, 9), (2, 16)])
def test_report_exchange_stream_ordered_gloo(world, batch):
    """ReportExchange (configs 3/4 across GPUs): double-buffered async all-gathers, one per batch
    of rounds (9 rounds: full batches, a partial last batch, or one partial batch), results
    consumed a batch later; contents, ordering and peer desync counts."""
    ctx = mp.get_context("spawn")
    out = ctx.Array("i", world)
    port = free_port()
    procs = [ctx.Process(target=report_exchange_worker, args=(r, world, port, out, batch)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert list(out) == [1] * world


def test_peer_of_needs_an_even_world():
    assert exchange.peer_of(1, 4) == 3 and exchange.peer_of(3, 4) == 1
    with pytest.raises(ValueError):
        exchange.peer_of(0, 3)
