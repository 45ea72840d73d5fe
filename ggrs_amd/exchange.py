"""Cross-GPU exchange of confirmation reports: one all-gather per confirmation.

A branch engine's report per confirmed frame is [S] u16 session checksums (padded to 8 bytes) +
ceil(L/64) u64 survival words (ggrs_branch_confirm).  Every rank contributes its report and
receives all of them: over RCCL (backend "nccl") the gather is all_gather_into_tensor on device
buffers, over gloo (CPU tests) a list all_gather.  This replaces GGRS's per-peer ChecksumReport
messages (src/network/protocol.rs:692-698 send, :663-682 receive) and the comparison in
P2PSession::compare_local_checksums_against_peers (src/sessions/p2p_session.rs:904-937): with
peer replicas (rank r and rank r + world/2 simulating the same sessions, like the two machines of
a match), a differing checksum is a DesyncDetected event (src/lib.rs:158-167).
"""
from dataclasses import dataclass

import numpy as np


@dataclass
class DesyncDetected:
    """GgrsEvent::DesyncDetected (src/lib.rs:158-167); addr is the peer's rank."""
    frame: int
    session: int
    local_checksum: int
    remote_checksum: int
    addr: int


def report_layout(num_sessions, num_lanes):
    ck_bytes = (2 * num_sessions + 7) & ~7
    words = (num_lanes + 63) // 64
    return ck_bytes, words, ck_bytes + 8 * words


def split_report(buf, num_sessions, num_lanes):
    """(checksums[S] u16, survival words u64) from one report's bytes (numpy uint8)."""
    ck_bytes, words, total = report_layout(num_sessions, num_lanes)
    b = np.ascontiguousarray(buf, np.uint8).reshape(-1)[:total]
    return b[:2 * num_sessions].view(np.uint16), b[ck_bytes:ck_bytes + 8 * words].view(np.uint64)


def allgather_reports(local, group=None):
    """All-gather one report tensor (uint8, 1-D) from every rank -> [world, nbytes] tensor."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":
        out = torch.empty((world, local.numel()), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out.view(-1), local.contiguous(), group=group)
        return out
    parts = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(parts, local.contiguous(), group=group)
    return torch.stack(parts)


def peer_of(rank, world):
    """The rank simulating the same sessions as `rank` (the other machine of each match): ranks r
    and r + world/2 pair up, an involution only for an even world size."""
    if world % 2 != 0:
        raise ValueError(f"peer replicas need an even world size, got {world}")
    return (rank + world // 2) % world


def desyncs_against_peer(gathered, rank, world, frame, num_sessions, num_lanes):
    """Compare this rank's session checksums with its peer replica's (p2p_session.rs:904-937)."""
    if world < 2:
        return []
    peer = peer_of(rank, world)
    g = gathered.cpu().numpy() if hasattr(gathered, "cpu") else np.asarray(gathered)
    mine, _ = split_report(g[rank], num_sessions, num_lanes)
    theirs, _ = split_report(g[peer], num_sessions, num_lanes)
    bad = np.nonzero(mine != theirs)[0]
    return [DesyncDetected(frame, int(s), int(mine[s]), int(theirs[s]), peer) for s in bad]



def exchange_p2p_reports(detector, group=None):
    """Checksum reports of a P2P engine's sessions between the two peers of every match, over the
    process group: rank r and rank peer_of(r) run the same sessions as the two machines of each
    match (a desync.DesyncDetector on each).  Every rank runs the same calls, so each sends the same
    number of reports for the same frames; they are stacked into one [k][2S] byte tensor,
    all-gathered (RCCL on device tensors, gloo on CPU tensors), and the peer's rows are
    delivered with DesyncDetector.receive -- the ChecksumReport messages of protocol.rs:692-698
    (send) and :663-682 (receive), one collective per batch of calls.  Returns the number of
    reports sent."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    peer = peer_of(rank, world)  # ValueError for an odd world size
    nccl = dist.get_backend(group) == "nccl"
    device = torch.device("cuda", torch.cuda.current_device()) if nccl else None
    out = detector.outgoing(device=device)
    if not out:
        return 0
    # as bytes: neither gloo nor RCCL reduce or gather 16-bit integers
    if nccl:
        local = torch.stack([r for _, _, r in out]).view(torch.uint8)
        gathered = torch.empty((world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(gathered.view(-1), local.contiguous().view(-1), group=group)
    else:
        local = torch.from_numpy(np.stack([np.asarray(r, np.uint16).view(np.uint8) for _, _, r in out]))
        parts = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(parts, local.contiguous(), group=group)
        gathered = torch.stack(parts)
    theirs = gathered[peer]
    for k, (call, frame, _) in enumerate(out):
        row = theirs[k]
        detector.receive(call, frame, row.view(torch.int16) if nccl else row.numpy().view(np.uint16))
    return len(out)


def exchange_sched_reports(detector, group=None):
    """The same for P2P engines under arrival schedules (desync.SchedDesyncDetector): each rank's
    report rows of the calls run since the last exchange -- per call and session the report frame,
    checksum and the local players' last queued frame (the report travels with those inputs) -- are
    all-gathered over the process group as one int32 block, and the peer's rows go to
    SchedDesyncDetector.receive.  Every rank runs the same calls.  Returns the number of calls."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    peer = peer_of(rank, world)
    first, rows = detector.outgoing()
    if rows is None:
        return 0
    block = np.stack([rows["frame"], rows["checksum"].astype(np.int32), rows["local_last"]], axis=1)
    local = torch.from_numpy(np.ascontiguousarray(block, np.int32))
    if dist.get_backend(group) == "nccl":
        local = local.cuda()
    parts = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(parts, local, group=group)
    theirs = parts[peer].cpu().numpy()
    detector.receive(first, dict(frame=theirs[:, 0], checksum=theirs[:, 1].astype(np.uint16),
                                 local_last=theirs[:, 2]))
    return theirs.shape[0]


class ReportExchange:
    """Stream-ordered exchange of branch-engine reports (configs 3/4 across GPUs): one all-gather
    per batch of `batch` confirmations (default 1: one per confirmation) with no host
    synchronisation in the round loop.

    The engine runs on the caller's current stream (BranchEngine.set_stream), so per round r:
      round(r) -> row r % batch of report buffer (r // batch) % 2  -- one launch (speculate +
                                              confirm, ggrs_branch_round), the kernel writing the
                                              report into the buffer
    and after the batch's last round:
      wait for the previous batch's all-gather -- a device-side stream wait (work.wait()), after
                                              which its peer comparison is queued on the device
                                              (ggrs_branch_compare_peer_rows, one small kernel)
      all-gather of this batch's buffer      -- async on the collective's stream, which orders
                                              itself after the current stream
    so a batch's all-gather overlaps the next batch's kernels, and a buffer is never overwritten
    before its all-gather has read it (the next batch writing into it is queued after the current
    stream has waited for that all-gather).  The reference sends its checksum reports every
    `DesyncDetection::On { interval }` frames (p2p_session.rs:939-962); `batch` plays that role
    for the collective, amortising its latency (~20 us per all-gather on one MI355X) over rounds.
    With `peers` (rank r and rank r + world/2 run the same sessions, the two machines of each match)
    every round's session checksums are compared with the peer replica's on the device
    (compare_local_checksums_against_peers, p2p_session.rs:904-937): `desync_count` counts
    DesyncDetected events (src/lib.rs:158-167), `first_desync_round` the earliest round with one.
    Works over RCCL (device tensors) and gloo (CPU tensors, for tests; gloo's wait blocks the
    host, and the comparison runs as torch ops on the host)."""

    def __init__(self, engine, group=None, peers=False, keep_history=False, device=None, batch=1,
                 dedicated_stream=True):
        import torch
        import torch.distributed as dist
        if batch < 1:
            raise ValueError(f"batch must be >= 1, got {batch}")
        self.eng = engine
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.nccl = dist.get_backend(group) == "nccl"
        self.peer = peer_of(self.rank, self.world) if peers and self.world >= 2 else None
        dev = device if device is not None else (torch.device("cuda", torch.cuda.current_device())
                                                 if self.nccl else torch.device("cpu"))
        n = engine.report_bytes
        self.S = engine.num_sessions
        self.batch = batch
        self.bufs = [torch.zeros((batch, n), dtype=torch.uint8, device=dev) for _ in range(2)]
        self.gathered = [torch.zeros((self.world, batch, n), dtype=torch.uint8, device=dev) for _ in range(2)]
        self.work = [None, None]
        self.frame_of = [None, None]   # frame of the batch's first round
        self.rows_of = [0, 0]          # rounds in the batch
        self.round = 0
        self.desync_count = torch.zeros((), dtype=torch.int64, device=dev)
        self.first_desync_round = torch.full((), -1, dtype=torch.int64, device=dev)
        self.history = [] if keep_history else None
        # With dedicated_stream one stream of the exchange's own carries the engine's rounds, the
        # all-gathers' stream waits, the history copies and the comparisons (it starts behind the
        # caller's work so far); without it all of that runs on the caller's current stream, which
        # may be the null stream (handle 0: ggrs_branch_set_stream binds the engine to HIP's null
        # stream, ABI 3).  Either way the rounds that write a report are stream-ordered before the
        # all-gather that reads it (RCCL's stream waits for the current stream).
        self.stream = None
        if self.nccl:
            if dedicated_stream:
                self.stream = torch.cuda.Stream(device=dev)
                self.stream.wait_stream(torch.cuda.current_stream(dev))
                engine.set_stream(self.stream.cuda_stream)
            else:
                engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)

    def _on_stream(self):
        import contextlib
        import torch
        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()

    def _finish(self, k):
        """Wait (device-side) for the all-gather in slot k and queue its comparison."""
        import torch
        w = self.work[k]
        if w is None:
            return
        w.wait()
        self.work[k] = None
        g = self.gathered[k]
        rows = self.rows_of[k]
        if self.history is not None:
            for j in range(rows):
                self.history.append((self.frame_of[k] + j, g[:, j].clone()))
        if self.peer is None:
            return
        if self.nccl:
            self.eng.compare_peer_rows(g, rows, self.rank, self.peer, self.frame_of[k], self.desync_count,
                                       self.first_desync_round)
            return
        ck = 2 * self.S
        for j in range(rows):
            mine = g[self.rank, j, :ck].view(torch.int16)
            theirs = g[self.peer, j, :ck].view(torch.int16)
            n = (mine != theirs).sum()
            first = torch.where((n > 0) & (self.first_desync_round < 0),
                                torch.full_like(self.first_desync_round, self.frame_of[k] + j),
                                self.first_desync_round)
            self.desync_count += n
            self.first_desync_round.copy_(first)

    def _start(self, k, rows):
        import torch.distributed as dist
        self.rows_of[k] = rows
        if self.nccl:
            self.work[k] = dist.all_gather_into_tensor(self.gathered[k].view(-1), self.bufs[k].view(-1),
                                                       group=self.group, async_op=True)
        else:  # gloo: CPU tensors
            parts = list(self.gathered[k].unbind(0))
            self.work[k] = dist.all_gather(parts, self.bufs[k], group=self.group, async_op=True)

    def step(self):
        """One round: the fused round kernel; after a batch's last round, finish the previous
        batch's all-gather and start this one's."""
        with self._on_stream():
            self._step()

    def _step(self):
        k = (self.round // self.batch) % 2
        j = self.round % self.batch
        if j == 0:
            self.frame_of[k] = self.eng.trunk_frame()
        self.eng.round_to_tensor(self.bufs[k][j])
        self.round += 1
        if j + 1 == self.batch:
            self._finish(1 - k)
            self._start(k, self.batch)

    def run(self, n_rounds):
        """n rounds, a batch's rounds as ONE fused launch (ggrs_branch_rounds_reports: every
        round's report written into its row of the batch buffer by the kernel) followed by the
        batch's all-gather -- the same reports, exchanges and comparisons as n step() calls.  Over
        gloo (host tensors) it is n step() calls."""
        if not self.nccl or not hasattr(self.eng, "rounds_to_tensor"):
            for _ in range(n_rounds):
                self.step()
            return
        with self._on_stream():
            self._run(n_rounds)

    def _run(self, n_rounds):
        while n_rounds > 0:
            k = (self.round // self.batch) % 2
            j = self.round % self.batch
            m = min(self.batch - j, n_rounds)
            if j == 0:
                self.frame_of[k] = self.eng.trunk_frame()
            self.eng.rounds_to_tensor(self.bufs[k][j:], m)
            self.round += m
            n_rounds -= m
            if j + m == self.batch:
                self._finish(1 - k)
                self._start(k, self.batch)

    def drain(self):
        """Start the gather of a partial last batch, finish every all-gather (device-side wait) --
        call before reading results.  The caller's current stream is then ordered after all of it."""
        import torch
        with self._on_stream():
            k = (self.round // self.batch) % 2
            j = self.round % self.batch
            if j:
                self._finish(1 - k)
                self._start(k, j)
            self._finish(k)
            self._finish(1 - k)
        if self.stream is not None:
            torch.cuda.current_stream(self.stream.device).wait_stream(self.stream)
