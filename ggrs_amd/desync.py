"""P2P desync detection for every session of a P2PEngine: the host-side bookkeeping of
DesyncDetection::On{interval} around the device-resident checksum history.

Reference semantics restated (caspark/ggrs 0.10.2):
  * P2PSession::advance_frame runs check_checksum_send_interval, then
    compare_local_checksums_against_peers, before any rollback of the call
    (src/sessions/p2p_session.rs:281-291);
  * check_checksum_send_interval (:939-975): frame_to_send = interval, 2 interval, ... once
    <= last_confirmed_frame and last_saved_frame; the saved cell's checksum is sent to every remote
    and kept in local_checksum_history, pruned to MAX_CHECKSUM_HISTORY_SIZE = 32 reports
    (src/network/protocol.rs:27).  The device records it (ggrs_p2p_set_desync_detection); in the
    engine's network model that is call frame_to_send + remote_latency + 1;
  * UdpProtocol::on_checksum_report (protocol.rs:663-682) keeps received reports in
    pending_checksums, pruned to frames >= frame - 31 interval once 32 are pending;
  * compare_local_checksums_against_peers (:904-937): every pending report with
    frame < last_confirmed_frame whose frame is in the local history is compared (on the device,
    ggrs_p2p_compare_checksums), raising GgrsEvent::DesyncDetected per differing session, and is
    removed; the others stay pending.
Reports travel between peers like inputs: what a peer sends in call g is received at the start of
call g + remote_latency.  Pending reports are visited in frame order (the reference iterates a
HashMap, whose order is unspecified).
"""
from dataclasses import dataclass

MAX_CHECKSUM_HISTORY_SIZE = 32  # src/network/protocol.rs:27


@dataclass
class DesyncDetected:
    """GgrsEvent::DesyncDetected (src/lib.rs:158-167) for one session; `call` is the advance_frame
    call that raised it, `addr` the remote peer."""
    frame: int
    session: int
    local_checksum: int
    remote_checksum: int
    addr: object
    call: int


class DesyncDetector:
    """One peer's desync detection against one remote peer, for all sessions of `engine`."""

    def __init__(self, engine, interval, addr=None):
        self.engine = engine
        self.interval = interval
        self.addr = addr
        self.latency = engine.remote_latency
        engine.set_desync_detection(interval)
        self.local_history = []   # report frames held in the device history, oldest first
        self.pending = {}         # frame -> remote report ([S] u16 numpy or device tensor)
        self.arrivals = {}        # call -> [(frame, report)] received at the start of that call
        self.processed = 0        # calls whose desync steps have been replayed on the host
        self.sent = 0             # calls whose outgoing reports have been handed out

    def _send_frame(self, call):
        """frame_to_send that goes out in `call`, or None."""
        if self.engine.max_prediction == 0:  # lockstep mode saves nothing, so it never reports
            return None
        fts = call - 1 - self.latency
        return fts if self.interval > 0 and fts >= self.interval and fts % self.interval == 0 else None

    def outgoing(self, device=None):
        """Reports sent in the calls run since the last outgoing(): [(call, frame, report)], each
        report [S] u16 numpy, or an int16 torch tensor on `device` (the bits of the u16 values)."""
        out = []
        current = self.engine.calls()
        for call in range(self.sent, current):
            fts = self._send_frame(call)
            if fts is not None:
                if device is None:
                    rep = self.engine.local_checksums(fts)
                else:
                    import torch
                    rep = self.engine.local_checksums(
                        fts, out=torch.empty(self.engine.num_sessions, dtype=torch.int16, device=device))
                out.append((call, fts, rep))
        self.sent = current
        return out

    def receive(self, sent_call, frame, report):
        """The remote's report of `frame`, sent in its call `sent_call`: received at the start of
        call sent_call + latency."""
        self.arrivals.setdefault(sent_call + self.latency, []).append((frame, report))

    def _on_checksum_report(self, frame, report):
        if len(self.pending) >= MAX_CHECKSUM_HISTORY_SIZE:
            oldest = frame - (MAX_CHECKSUM_HISTORY_SIZE - 1) * self.interval
            self.pending = {f: r for f, r in self.pending.items() if f >= oldest}
        self.pending[frame] = report

    def poll(self):
        """Replay the desync steps of every call run so far (arrivals, send, compare) and return
        the DesyncDetected events they raise, in call order."""
        events = []
        current = self.engine.calls()
        for call in range(self.processed, current):
            for frame, report in self.arrivals.pop(call, []):          # poll_remote_clients
                self._on_checksum_report(frame, report)
            fts = self._send_frame(call)                               # check_checksum_send_interval
            if fts is not None:
                self.local_history.append(fts)
                if len(self.local_history) > MAX_CHECKSUM_HISTORY_SIZE:
                    oldest = fts - (MAX_CHECKSUM_HISTORY_SIZE - 1) * self.interval
                    self.local_history = [f for f in self.local_history if f >= oldest]
            last_confirmed = call - 1 - self.latency                   # compare_local_checksums...
            checked = []
            for frame in sorted(self.pending):
                if frame >= last_confirmed or frame not in self.local_history:
                    continue
                report = self.pending[frame]
                sessions = self.engine.compare_checksums(frame, report)
                if len(sessions):
                    local = self.engine.local_checksums(frame)
                    remote = report.cpu().numpy() if hasattr(report, "cpu") else report
                    for s in sessions:
                        events.append(DesyncDetected(frame, int(s), int(local[s]) & 0xFFFF,
                                                     int(remote[s]) & 0xFFFF, self.addr, call))
                checked.append(frame)
            for frame in checked:
                del self.pending[frame]
        self.processed = current
        return events


def exchange(a, b):
    """Deliver each detector's outgoing reports to the other (the two peers of one match)."""
    for call, frame, report in a.outgoing():
        b.receive(call, frame, report)
    for call, frame, report in b.outgoing():
        a.receive(call, frame, report)


class SchedDesyncDetector:
    """Desync detection for every session of a P2PEngine under arrival schedules
    (ggrs_p2p_set_arrival_schedule): each session sends its checksum reports at its own calls, for
    its own frames (check_checksum_send_interval on the device, ggrs_p2p_read_reports), and this
    class keeps the rest of the reference's bookkeeping per session:
      * a report the remote peer sent in its call g travels with the inputs it sent in that call
        (its last queued frame, `local_last`), so it is received at the first local call c > g whose
        poll delivers that frame (the arrival rows handed to the engine, `note_arrivals`);
      * UdpProtocol::on_checksum_report (protocol.rs:663-682) keeps it in pending_checksums;
      * the local report of a call enters local_checksum_history (pruned to 32 reports);
      * compare_local_checksums_against_peers (p2p_session.rs:904-937) compares every pending report
        older than the call's last_confirmed_frame that is in the history, raises DesyncDetected when
        they differ, and drops it -- pending reports are visited in frame order.
    """

    def __init__(self, engine, interval, addr=None):
        import numpy as np
        self.np = np
        self.engine = engine
        self.interval = interval
        self.addr = addr
        engine.set_desync_detection(interval)
        S = engine.num_sessions
        self.local = [dict() for _ in range(S)]     # local_checksum_history per session
        self.pending = [dict() for _ in range(S)]   # remote pending_checksums per session
        self.arrive = {}                            # call -> [S] newest remote frame delivered
        self.remote = []                            # remote report rows: (call, frame[S], cs[S], local_last[S])
        self.remote_base = 0                        # the call of self.remote[0] (earlier rows are delivered)
        self.remote_in = 0                          # remote rows received so far
        self.next_remote = np.zeros(S, np.int64)    # per session: remote rows delivered so far
        self.processed = 0
        self.sent = 0

    def note_arrivals(self, first_call, arrive_upto):
        """The arrival rows given to the engine (ggrs_p2p_add_arrivals), for the report delivery."""
        for k, row in enumerate(self.np.asarray(arrive_upto)):
            self.arrive[first_call + k] = self.np.asarray(row, self.np.int32)

    def outgoing(self):
        """The report rows of the calls run since the last outgoing(): (first_call, engine.reports)."""
        current = self.engine.calls()
        first, n = self.sent, current - self.sent
        self.sent = current
        return first, self.engine.reports(first, n) if n > 0 else None

    def receive(self, first_call, rows):
        """The remote peer's outgoing() rows (its calls first_call ..)."""
        if rows is None:
            return
        assert first_call == self.remote_in, "remote report rows must be received in order"
        for k in range(rows["frame"].shape[0]):
            self.remote.append((first_call + k, rows["frame"][k], rows["checksum"][k], rows["local_last"][k]))
        self.remote_in += rows["frame"].shape[0]

    def _on_checksum_report(self, s, frame, cs):
        pend = self.pending[s]
        if len(pend) >= MAX_CHECKSUM_HISTORY_SIZE:
            oldest = frame - (MAX_CHECKSUM_HISTORY_SIZE - 1) * self.interval
            self.pending[s] = pend = {f: c for f, c in pend.items() if f >= oldest}
        pend[frame] = cs

    def poll(self):
        """Replay the desync steps of every call run so far (report arrivals, the local report, the
        comparison) and return the DesyncDetected events they raise, in call order."""
        np = self.np
        events = []
        current = self.engine.calls()
        if current <= self.processed:
            return events
        first = self.processed
        own = self.engine.reports(first, current - first)
        for c in range(first, current):
            arrive = self.arrive[c]
            # poll_remote_clients: remote reports whose inputs this call's poll delivers, in order
            for s in range(len(self.local)):
                g = int(self.next_remote[s])
                while g < self.remote_in and g < c:
                    _, fr, cs, ll = self.remote[g - self.remote_base]
                    if ll[s] > arrive[s]:
                        break
                    if fr[s] >= 0:
                        self._on_checksum_report(s, int(fr[s]), int(cs[s]))
                    g += 1
                self.next_remote[s] = g
            row = c - first
            fr, cs, lc = own["frame"][row], own["checksum"][row], own["last_confirmed"][row]
            for s in np.nonzero(fr >= 0)[0]:           # check_checksum_send_interval
                hist = self.local[s]
                hist[int(fr[s])] = int(cs[s])
                if len(hist) > MAX_CHECKSUM_HISTORY_SIZE:
                    oldest = int(fr[s]) - (MAX_CHECKSUM_HISTORY_SIZE - 1) * self.interval
                    self.local[s] = {f: v for f, v in hist.items() if f >= oldest}
            for s in range(len(self.local)):           # compare_local_checksums_against_peers
                pend = self.pending[s]
                if not pend:
                    continue
                hist = self.local[s]
                checked = []
                for frame in sorted(pend):
                    if frame >= lc[s] or frame not in hist:
                        continue
                    if hist[frame] != pend[frame]:
                        events.append(DesyncDetected(frame, s, hist[frame], pend[frame], self.addr, c))
                    checked.append(frame)
                for frame in checked:
                    del pend[frame]
        self.processed = current
        # drop what no later call reads: the arrival rows of the calls replayed, the remote rows
        # every session has taken
        for c in range(first, current):
            del self.arrive[c]
        done = int(self.next_remote.min()) if len(self.local) else self.remote_in
        if done > self.remote_base:
            del self.remote[:done - self.remote_base]
            self.remote_base = done
        return events
