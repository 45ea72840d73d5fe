"""The stream-ordered report exchange of configs 3/4 (exchange.ReportExchange) on the GPU with a
one-rank RCCL group: the engine runs on torch's current stream, every round's report is
all-gathered asynchronously behind its confirm, and the gathered reports equal the reports of an
identical engine run round by round without any exchange (ggrs_branch_confirm's report,
p2p_session.rs:939-975's ChecksumReport restated)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_report_exchange_world1_nccl(oracle):
    import torch.distributed as dist
    from ggrs_amd import BranchEngine, exchange, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(free_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        S, B, P, W, rounds = 64, 16, 4, 8, 12
        truth = synth.gen_inputs(0, S, rounds + W + 1, P, synth.MODEL_HELD)
        engs = []
        for _ in range(2):
            e = BranchEngine(S, num_players=P, remote_mask=0b1110, window=W, branches=B, alphabet=16,
                             input_capacity=rounds + W + 3)
            e.add_inputs(0, truth)
            engs.append(e)
        ex = exchange.ReportExchange(engs[0], peers=False, keep_history=True)
        for _ in range(rounds):
            ex.step()
        ex.drain()
        torch.cuda.synchronize()
        want = []
        frames = []
        for _ in range(rounds):
            engs[1].speculate()
            frames.append(engs[1].trunk_frame())
            engs[1].confirm()
            ck, bits = engs[1].report()
            want.append((ck.copy(), bits.copy()))
        assert [f for f, _ in ex.history] == frames
        for (f, g), (ck, bits) in zip(ex.history, want):
            got_ck, got_bits = exchange.split_report(g[0].cpu().numpy(), S, engs[0].num_lanes)
            assert (got_ck == ck).all() and (got_bits == bits).all(), f
        assert bytes(engs[0].trunk(0)) == bytes(engs[1].trunk(0))
        assert int(ex.desync_count.item()) == 0
    finally:
        dist.destroy_process_group()


def test_compare_peer_kernel():
    """ggrs_branch_compare_peer: sessions whose checksum differs between this rank's row and its
    peer's row of an all-gathered block are counted; the first frame with any is kept."""
    from ggrs_amd import BranchEngine, synth
    S, B, P, W = 300, 1, 2, 4
    e = BranchEngine(S, num_players=P, remote_mask=0b10, window=W, branches=B, alphabet=16, input_capacity=16)
    e.add_inputs(0, synth.gen_inputs(0, S, W + 2, P, synth.MODEL_HELD))
    buf = torch.zeros(e.report_bytes, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the engine runs on its own stream here
    e.round_to_tensor(buf)
    e.synchronize()
    ck, _ = e.report()
    assert (buf[:2 * S].cpu().numpy().view(np.uint16) == ck).all()  # the kernel's own report copy
    g = torch.stack([buf, buf, buf.clone()])  # world 3: rank 0 vs peer 2
    g[2, 2 * 3] ^= 1      # session 3
    g[2, 2 * 299 + 1] ^= 0x80  # session 299
    g[1, 2 * 5] ^= 1      # row 1 is neither rank nor peer
    count = torch.zeros((), dtype=torch.int64, device="cuda")
    first = torch.full((), -1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    e.compare_peer(g, 0, 2, 7, count, first)
    e.compare_peer(g, 0, 1, 9, count, first)
    e.synchronize()
    assert int(count) == 3 and int(first) == 7


@pytest.mark.parametrize("batch,fused", [(4, False), (5, False), (4, True), (5, True), (1, True)])
def test_report_exchange_batched_world1_nccl(oracle, batch, fused):
    """One all-gather per batch of rounds (12 rounds: full batches and a partial last one), the
    rounds launched one by one or a batch per launch: the gathered reports still equal every
    round's report of an exchange-free engine."""
    import torch.distributed as dist
    from ggrs_amd import BranchEngine, exchange, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(free_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        S, B, P, W, rounds = 64, 16, 4, 8, 12
        truth = synth.gen_inputs(3, S, rounds + W + 1, P, synth.MODEL_HELD)
        engs = []
        for _ in range(2):
            e = BranchEngine(S, num_players=P, remote_mask=0b1110, window=W, branches=B, alphabet=16,
                             input_capacity=rounds + W + 3)
            e.add_inputs(0, truth)
            engs.append(e)
        ex = exchange.ReportExchange(engs[0], peers=False, keep_history=True, batch=batch)
        if fused:  # whole batches as one launch each (ggrs_branch_rounds_reports), in uneven pieces
            for n in (3, 1, 8):
                ex.run(n)
        else:
            for _ in range(rounds):
                ex.step()
        ex.drain()
        torch.cuda.synchronize()
        assert [f for f, _ in ex.history] == list(range(rounds))
        for f, g in ex.history:
            engs[1].speculate()
            engs[1].confirm()
            ck, bits = engs[1].report()
            got_ck, got_bits = exchange.split_report(g[0].cpu().numpy(), S, engs[0].num_lanes)
            assert (got_ck == ck).all() and (got_bits == bits).all(), f
    finally:
        dist.destroy_process_group()


def test_compare_peer_rows_kernel():
    """ggrs_branch_compare_peer_rows: a [world][rows][report] block compared row by row in one
    launch; the count sums every row, the first frame is the earliest row with a difference."""
    from ggrs_amd import BranchEngine, synth
    S, B, P, W, rows = 300, 1, 2, 4, 5
    e = BranchEngine(S, num_players=P, remote_mask=0b10, window=W, branches=B, alphabet=16, input_capacity=16)
    e.add_inputs(0, synth.gen_inputs(0, S, W + 2, P, synth.MODEL_HELD))
    buf = torch.zeros(e.report_bytes, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    e.round_to_tensor(buf)
    e.synchronize()
    g = buf.repeat(2, rows, 1).contiguous()  # [world 2][rows][report]
    g[1, 3, 2 * 10] ^= 1     # row 3: session 10
    g[1, 4, 2 * 11] ^= 4     # row 4: sessions 11 and 299
    g[1, 4, 2 * 299 + 1] ^= 1
    g[1, 1, 2 * 42] ^= 1     # row 1: session 42
    count = torch.zeros((), dtype=torch.int64, device="cuda")
    first = torch.full((), -1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    e.compare_peer_rows(g, rows, 0, 1, 20, count, first)
    e.synchronize()
    assert int(count) == 4 and int(first) == 21
    count.zero_()
    first.fill_(-1)
    torch.cuda.synchronize()
    e.compare_peer_rows(g, 3, 0, 1, 30, count, first)  # rows 0..2 of 5 per rank
    e.synchronize()
    assert int(count) == 1 and int(first) == 31


def test_report_exchange_null_stream_world1_nccl(oracle):
    """The engine bound to torch's current stream when that is the null stream (handle 0) and NO
    dedicated exchange stream: ggrs_branch_set_stream(NULL) is HIP's null stream (ABI 3), so the
    fused rounds that write each batch's reports are ordered before the RCCL all-gather that reads
    them; the gathered reports equal an exchange-free engine's every round (protocol.rs:692-698:
    the report sent is the saved cell's)."""
    import torch.distributed as dist
    from ggrs_amd import BranchEngine, exchange, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(free_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert torch.cuda.current_stream().cuda_stream == 0
        S, B, P, W, rounds = 512, 16, 4, 8, 24
        truth = synth.gen_inputs(5, S, rounds + W + 1, P, synth.MODEL_HELD)
        engs = []
        for _ in range(2):
            e = BranchEngine(S, num_players=P, remote_mask=0b1110, window=W, branches=B, alphabet=16,
                             input_capacity=rounds + W + 3)
            e.add_inputs(0, truth)
            engs.append(e)
        ex = exchange.ReportExchange(engs[0], peers=False, keep_history=True, batch=4, dedicated_stream=False)
        assert ex.stream is None
        for n in (4, 3, 5, 8, 4):
            ex.run(n)
        ex.drain()
        torch.cuda.synchronize()
        assert [f for f, _ in ex.history] == list(range(rounds))
        for f, g in ex.history:
            engs[1].speculate()
            engs[1].confirm()
            ck, bits = engs[1].report()
            got_ck, got_bits = exchange.split_report(g[0].cpu().numpy(), S, engs[0].num_lanes)
            assert (got_ck == ck).all() and (got_bits == bits).all(), f
        engs[0].use_own_stream()
        engs[0].synchronize()
        assert bytes(engs[0].trunk(0)) == bytes(engs[1].trunk(0))
    finally:
        dist.destroy_process_group()
