"""The request handler of many sessions over one engine's lane batch: the Python mirror of the Rust
crate's `BatchedBoxGame` (rust/ggrs-mi355x/src/lib.rs), which replaces `Game::handle_requests`
(examples/ex_game/ex_game.rs:79-127) for every session at once.

GGRS hands a handler one ordered `Vec<GgrsRequest>` per session per `advance_frame` (src/lib.rs:
171-195).  Here a request is a tuple:
    ("save", cell, frame)         GgrsRequest::SaveGameState  -> cell.save(frame, None, checksum)
    ("load", cell, frame)         GgrsRequest::LoadGameState  (the state stays in the HBM ring)
    ("advance", inputs, status)   GgrsRequest::AdvanceFrame   (inputs / status: P bytes each)
and a cell is anything with GGRS's `save(frame, data, checksum)` (`GameStateCell` below mirrors
sync_layer.rs:14-101).  The state never leaves the device: every save hands GGRS
`cell.save(frame, None, Some(checksum))` -- `data = None` is legal (CHANGELOG.md:121) and GGRS only
reads a cell's frame() and checksum() (sync_layer.rs:72-78).

Two delivery modes:
  synchronous (default)  handle_requests returns with every checksum in its cell: what a
                         SyncTestSession needs, since checksums_consistent reads the cells the
                         previous call saved (sync_test_session.rs:173-190).
  deferred               for P2PSessions: handle_requests encodes and submits the batch, saves
                         every cell as `save(frame, None, None)` at once and returns; the device
                         round trip then overlaps the caller's session logic, and the NEXT call
                         (or flush()) waits for the batch and fills `Some(checksum)` into those
                         cells, in request order.  Safe because a P2PSession reads a cell's
                         checksum only for confirmed frames at its desync interval and, while it is
                         None, skips it and retries on a later call
                         (check_checksum_send_interval, p2p_session.rs:939-963); a confirmed
                         frame is never re-saved, so the value it then sends is the same.  A cell
                         re-saved by the next call (a rollback replaying its frame) first gets its
                         earlier checksum and then None again with the new save, as GGRS's own
                         order of saves would leave it.  Lanes the device rejects are reported by
                         the call that collects their batch.

The device work is any object with the LaneBatch interface (session.LaneBatch over an engine;
tests substitute a host model): encode(lane, reqs, inputs, status, lane_frame) -> -1 or the index
of a rejected Save, submit(token_words, load_slots, adv_rows, save_rows, status=True), wait() ->
number of failed lanes, views `checksums` [S][L] and `lane_result` [L], and `shape`.
"""
import numpy as np

from ._lib import NULL_FRAME, REQ_ADVANCE, REQ_LOAD, REQ_SAVE

_KIND = {"save": REQ_SAVE, "load": REQ_LOAD, "advance": REQ_ADVANCE}


class GameStateCell:
    """sync_layer.rs:14-101: frame, data, checksum; save() asserts frame != NULL_FRAME (:20)."""

    def __init__(self):
        self.frame = NULL_FRAME
        self.data = None
        self.checksum = None

    def save(self, frame, data, checksum):
        assert frame != NULL_FRAME
        self.frame, self.data, self.checksum = frame, data, checksum


def lane_shape(reqs):
    """(token words, Loads, AdvanceFrames, SaveGameStates) one list needs (ggrs_lane_shape)."""
    kinds = [k for k, _ in reqs]
    return (-(-len(reqs) // 16), kinds.count(REQ_LOAD), kinds.count(REQ_ADVANCE), kinds.count(REQ_SAVE))


class BatchedHandler:
    """handle_requests for L sessions (one engine lane each) through a lane batch.

    map_batch(shape) -> a LaneBatch of at least that shape (called when a call's lists need a larger
    one; every earlier batch has been collected by then)."""

    def __init__(self, num_lanes, num_players, map_batch, deferred=False):
        self.L, self.P = num_lanes, num_players
        self.map_batch = map_batch
        self.deferred = deferred
        self.batch = None
        self.lane_frames = np.zeros(num_lanes, np.int32)  # every lane's frame after its last list
        self._pending = None  # the submitted, uncollected batch: [(lane, [(cell, frame), ...])]

    @staticmethod
    def _abi_list(lst, P):
        reqs, inputs, status = [], [], []
        for r in lst:
            kind = _KIND[r[0]]
            if kind == REQ_ADVANCE:
                reqs.append((kind, 0))
                inputs.append(np.asarray(r[1], np.uint8).reshape(P))
                status.append(np.zeros(P, np.uint8) if r[2] is None else np.asarray(r[2], np.uint8).reshape(P))
            else:
                reqs.append((kind, int(r[2])))
        inp = np.stack(inputs) if inputs else None
        st = np.stack(status) if status else None
        return reqs, inp, st

    def handle_requests(self, lists):
        """lists[l] = session l's request list.  Returns the failed lanes as [(lane, index of the
        first rejected request)] -- those lanes did not run (where the reference panics).  In
        deferred mode the list also holds the lanes the device rejected in the previous call's
        batch, which this call collected."""
        if len(lists) != self.L:
            raise ValueError(f"{len(lists)} request lists for {self.L} lanes")
        failed = self.flush()  # deferred: the previous batch's checksums into their cells
        abi = [self._abi_list(lst, self.P) for lst in lists]
        need = np.max([lane_shape(r) for r, _, _ in abi], axis=0) if abi else np.zeros(4, int)
        need = tuple(max(1, int(x)) for x in need)
        if self.batch is None or any(n > h for n, h in zip(need, self.batch.shape)):
            self.batch = self.map_batch(tuple(max(n, h) for n, h in zip(need, self.batch.shape))
                                        if self.batch is not None else need)
        b = self.batch
        rejected = set()
        saves = []
        for lane, (lst, (reqs, inp, st)) in enumerate(zip(lists, abi)):
            bad = b.encode(lane, reqs, inp, st, int(self.lane_frames[lane]))
            if bad >= 0:
                failed.append((lane, bad))
                rejected.add(lane)
                continue
            saves.append((lane, [(r[1], r[2]) for r in lst if r[0] == "save"]))
        b.submit(*need, status=True)  # only the rows this call's lists use cross PCIe
        self._pending = (saves, rejected)
        if self.deferred:
            for _, cells in saves:
                for cell, frame in cells:
                    cell.save(frame, None, None)
            return failed
        return failed + self.flush()

    def flush(self):
        """Collect the submitted batch, if any: wait for it, every Save's checksum into its cell in
        request order, every lane's frame.  Returns the lanes the device rejected."""
        if self._pending is None:
            return []
        saves, rejected = self._pending
        self._pending = None
        b = self.batch
        b.wait()
        failed = []
        res = b.lane_result
        for lane, cells in saves:
            r = int(res[lane])
            if r < 0:
                failed.append((lane, -r - 1))
                continue
            self.lane_frames[lane] = r
            for si, (cell, frame) in enumerate(cells):
                cell.save(frame, None, int(b.checksums[si, lane]))
        return failed
