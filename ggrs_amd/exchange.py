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


class ReportExchange:
    """Stream-ordered exchange of branch-engine reports (configs 3/4 across GPUs), one all-gather
    per confirmation with no host synchronisation in the round loop.

    The engine runs on the caller's current stream (BranchEngine.set_stream), so per round r:
      round(r) -> report buffer r % 2      -- one launch (speculate + confirm, ggrs_branch_round),
                                              the kernel writing the report into the buffer
      wait for all-gather(r-1)             -- a device-side stream wait (work.wait()), after which
                                              its peer comparison is queued on the device
                                              (ggrs_branch_compare_peer, one small kernel)
      all-gather(r) of that buffer         -- async on the collective's stream, which orders itself
                                              after the current stream
    so round r-1's all-gather overlaps round r's kernel (it only needs round r-1's report), and the
    double-buffered report of round r-1 is never overwritten before its all-gather has read it
    (round r+1 writes it after the current stream has waited for that all-gather).
    With `peers` (rank r and rank r + world/2 run the same sessions, the two machines of each match)
    every round's session checksums are compared with the peer replica's on the device
    (compare_local_checksums_against_peers, p2p_session.rs:904-937): `desync_count` counts
    DesyncDetected events (src/lib.rs:158-167), `first_desync_round` the earliest round with one.
    Works over RCCL (device tensors) and gloo (CPU tensors, for tests; gloo's wait blocks the
    host, and the comparison runs as torch ops on the host)."""

    def __init__(self, engine, group=None, peers=False, keep_history=False, device=None):
        import torch
        import torch.distributed as dist
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
        self.bufs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.gathered = [torch.zeros((self.world, n), dtype=torch.uint8, device=dev) for _ in range(2)]
        self.work = [None, None]
        self.frame_of = [None, None]
        self.round = 0
        self.desync_count = torch.zeros((), dtype=torch.int64, device=dev)
        self.first_desync_round = torch.full((), -1, dtype=torch.int64, device=dev)
        self.history = [] if keep_history else None
        if self.nccl:
            engine.set_stream(torch.cuda.current_stream().cuda_stream)

    def _finish(self, k):
        """Wait (device-side) for the all-gather in slot k and queue its comparison."""
        import torch
        w = self.work[k]
        if w is None:
            return
        w.wait()
        self.work[k] = None
        g = self.gathered[k]
        if self.history is not None:
            self.history.append((self.frame_of[k], g.clone()))
        if self.peer is None:
            return
        if self.nccl:
            self.eng.compare_peer(g, self.rank, self.peer, self.frame_of[k], self.desync_count,
                                  self.first_desync_round)
            return
        ck = 2 * self.S
        mine = g[self.rank, :ck].view(torch.int16)
        theirs = g[self.peer, :ck].view(torch.int16)
        n = (mine != theirs).sum()
        first = torch.where((n > 0) & (self.first_desync_round < 0),
                            torch.full_like(self.first_desync_round, self.frame_of[k]), self.first_desync_round)
        self.desync_count += n
        self.first_desync_round.copy_(first)

    def step(self):
        """One round: the fused round kernel, finish the previous all-gather, start this one."""
        import torch.distributed as dist
        k = self.round % 2
        frame = self.eng.trunk_frame()
        self.eng.round_to_tensor(self.bufs[k])
        self._finish(1 - k)
        if self.nccl:
            self.work[k] = dist.all_gather_into_tensor(self.gathered[k].view(-1), self.bufs[k], group=self.group,
                                                       async_op=True)
        else:  # gloo: CPU tensors
            parts = list(self.gathered[k].unbind(0))
            self.work[k] = dist.all_gather(parts, self.bufs[k], group=self.group, async_op=True)
        self.frame_of[k] = frame
        self.round += 1

    def drain(self):
        """Finish the last all-gather (device-side wait) -- call before reading results."""
        self._finish(self.round % 2)
        self._finish(1 - self.round % 2)
