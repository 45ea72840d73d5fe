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
