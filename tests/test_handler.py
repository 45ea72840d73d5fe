"""The request handler's delivery of SaveGameState checksums (ggrs_amd/handler.py, the Python mirror
of rust/ggrs-mi355x BatchedBoxGame), synchronous and deferred, on the CPU with
a host model of the lane batch: every Save's checksum reaches its GameStateCell in request order;
in deferred mode a call's cells hold `None` until the next call collects the batch, a cell re-saved
by that call ends with its newer save, and lanes the device rejects are reported by the collecting
call.  The P2P request lists come from the oracle's P2PSession (oracle_p2p_stream, p2p_session.rs:
265-426), so rollbacks of differing depth re-save cells across calls."""
import numpy as np
import pytest

from ggrs_amd._lib import REQ_ADVANCE, REQ_LOAD, REQ_SAVE
from ggrs_amd.handler import BatchedHandler, GameStateCell


class HostBatch:
    """The LaneBatch interface executed on the host: a lane's state is its frame (a Load sets it to
    the loaded cell's frame if the lane's ring holds it, else the lane fails with -(1 + k) as
    ggrs_lane_batch_run does); a Save's checksum is a function of (lane, frame, the batch's
    number), so a re-save in a later batch gives a different value."""

    def __init__(self, L, shape, ring_len):
        self.L, self.shape, self.R = L, shape, ring_len
        W, LD, A, S = shape
        self.checksums = np.zeros((S, L), np.uint16)
        self.lane_result = np.zeros(L, np.int32)
        self.lists = [[] for _ in range(L)]
        self.frame = np.zeros(L, np.int64)
        self.ring = [dict() for _ in range(L)]  # slot -> frame saved there
        self.batches = 0
        self.waits = 0
        self.submitted = False

    @staticmethod
    def ck(lane, frame, batch):
        return (lane * 7919 + frame * 104729 + batch * 31) & 0xFFFF

    def encode(self, lane, reqs, inputs, status, lane_frame):
        f = lane_frame
        for k, (kind, fr) in enumerate(reqs):  # the Save-frame check of ggrs_lane_encode
            if kind == REQ_LOAD:
                f = fr
            elif kind == REQ_ADVANCE:
                f += 1
            elif fr != f:
                self.lists[lane] = []
                return k
        self.lists[lane] = list(reqs)
        return -1

    def submit(self, W, LD, A, S, status=False):
        assert not self.submitted, "a batch is already on the device"
        self.submitted = True
        self.batches += 1
        for lane, reqs in enumerate(self.lists):
            f, si, res = int(self.frame[lane]), 0, None
            for k, (kind, fr) in enumerate(reqs):
                if kind == REQ_LOAD:
                    if self.ring[lane].get(fr % self.R) != fr:
                        res = -(1 + k)
                        break
                    f = fr
                elif kind == REQ_ADVANCE:
                    f += 1
                else:
                    self.ring[lane][fr % self.R] = fr
                    self.checksums[si, lane] = self.ck(lane, fr, self.batches)
                    si += 1
            if res is None:
                self.frame[lane] = f
                res = f
            self.lane_result[lane] = res

    def wait(self):
        assert self.submitted
        self.submitted = False
        self.waits += 1
        return int((self.lane_result < 0).sum())


def p2p_calls(L, calls, P=2, maxp=8):
    """Per lane, the request lists of `calls` P2PSession::advance_frame calls (kinds and frames),
    remote inputs arriving in jittered bursts so sessions roll back by differing depths."""
    from oracle import oracle as O
    O.build()
    out = []
    for lane in range(L):
        inputs = O.gen_inputs(O.session_seed(lane, 0x777), calls, P, O.MODEL_HELD)
        s = O.p2p_stream(inputs, O.jitter_schedule(calls, maxp, seed=500 + lane), num_players=P,
                         max_prediction=maxp)
        assert s["rc"] == 0 and s["calls"] == calls
        out.append(s)
    return out


def lists_for_call(streams, c, cells):
    """GgrsRequest lists of call c for every lane, with SaveGameState / LoadGameState carrying the
    lane's ring cell of that frame (SavedStates::get_cell, sync_layer.rs:144-166)."""
    out = []
    for lane, s in enumerate(streams):
        a, b = int(s["call_off"][c]), int(s["call_off"][c + 1])
        lst = []
        for kind, fr in zip(s["kind"][a:b], s["frame"][a:b]):
            if kind == REQ_ADVANCE:
                lst.append(("advance", np.zeros(2, np.uint8), None))
            else:
                lst.append(("save" if kind == REQ_SAVE else "load", cells[lane][int(fr) % len(cells[lane])], int(fr)))
        out.append(lst)
    return out


@pytest.fixture(scope="module")
def streams():
    return p2p_calls(6, 40)


def mapper(L, R, batches):
    """map_batch for the host model: a larger mapping keeps the lanes' device state (frames, rings)
    and the batch count, as re-mapping an engine's batch does."""
    def map_batch(shape):
        b = HostBatch(L, shape, R)
        if batches:
            b.frame, b.ring, b.batches = batches[-1].frame, batches[-1].ring, batches[-1].batches
        batches.append(b)
        return b
    return map_batch


def run(streams, deferred, calls=40, R=9):
    L = len(streams)
    cells = [[GameStateCell() for _ in range(R)] for _ in range(L)]
    batches = []
    map_batch = mapper(L, R, batches)

    h = BatchedHandler(L, 2, map_batch, deferred=deferred)
    history = []
    for c in range(calls):
        lists = lists_for_call(streams, c, cells)
        failed = h.handle_requests(lists)
        assert failed == []
        saved = [(lane, r[1], r[2]) for lane, lst in enumerate(lists) for r in lst if r[0] == "save"]
        history.append(saved)
        for lane, cell, frame in saved:
            assert cell.frame == frame
            if deferred:
                assert cell.checksum is None  # handed back by the next call
            else:
                assert cell.checksum == HostBatch.ck(lane, frame, batches[-1].batches)
        if deferred and c > 0:
            # the previous call's cells now hold their batch's checksums, unless this call re-saved them
            now = {id(cell) for _, cell, _ in saved}
            for lane, cell, frame in history[-2]:
                if id(cell) not in now:
                    assert cell.frame == frame and cell.checksum == HostBatch.ck(lane, frame, batches[-1].batches - 1)
    assert h.flush() == []
    return cells, batches


def test_sync_and_deferred_deliver_the_same_checksums(streams):
    cs, bs = run(streams, deferred=False)
    cd, bd = run(streams, deferred=True)
    assert bs[-1].batches == bd[-1].batches == 40
    for lane in range(len(streams)):
        for a, b in zip(cs[lane], cd[lane]):
            assert (a.frame, a.checksum) == (b.frame, b.checksum)
            assert a.data is None and b.data is None


def test_deferred_waits_only_at_the_next_call(streams):
    L = len(streams)
    cells = [[GameStateCell() for _ in range(9)] for _ in range(L)]
    made = []

    def map_batch(shape):
        made.append(HostBatch(L, (max(shape[0], 4), max(shape[1], 1), max(shape[2], 16), max(shape[3], 16)), 9))
        return made[-1]

    h = BatchedHandler(L, 2, map_batch, deferred=True)
    h.handle_requests(lists_for_call(streams, 0, cells))
    b = made[0]
    assert b.submitted and b.waits == 0  # returned with the batch on the "device"
    h.handle_requests(lists_for_call(streams, 1, cells))
    assert b.waits == 1 and b.submitted
    h.flush()
    assert b.waits == 2 and not b.submitted
    assert h.flush() == [] and b.waits == 2


def test_deferred_reports_device_rejections_on_the_collecting_call():
    """A lane whose Load names a frame its ring does not hold fails on the device (sync_layer.rs:248):
    in deferred mode the call that collects the batch reports it, and its cells get no checksum."""
    L, R = 2, 4
    cells = [[GameStateCell() for _ in range(R)] for _ in range(L)]
    h = BatchedHandler(L, 2, mapper(L, R, []), deferred=True)
    adv = ("advance", np.zeros(2, np.uint8), None)
    first = [[("save", cells[l][0], 0), adv] for l in range(L)]
    assert h.handle_requests(first) == []
    bad = [[("save", cells[0][1], 1), adv],                              # lane 0: fine
           [("load", cells[1][3], 3), adv, ("save", cells[1][0], 4), adv]]  # lane 1: frame 3 never saved
    assert h.handle_requests(bad) == []            # nothing known yet: the batch is on the "device"
    assert cells[0][0].checksum == HostBatch.ck(0, 0, 1)  # call 1's cells were filled
    assert cells[1][0].frame == 4 and cells[1][0].checksum is None
    assert h.flush() == [(1, 0)]                   # lane 1 rejected at request 0
    assert cells[0][1].checksum == HostBatch.ck(0, 1, 2)
    assert cells[1][0].checksum is None
    assert list(h.lane_frames) == [2, 1]


def test_encoder_rejection_is_reported_at_once():
    """A SaveGameState of a frame other than the one the list reaches is rejected while encoding
    (ex_game.rs:104): reported by the same call in both modes; the lane's cells are not touched."""
    for deferred in (False, True):
        L = 2
        cells = [[GameStateCell() for _ in range(4)] for _ in range(L)]
        h = BatchedHandler(L, 2, mapper(L, 4, []), deferred=deferred)
        adv = ("advance", np.zeros(2, np.uint8), None)
        lists = [[("save", cells[0][0], 0), adv], [("save", cells[1][1], 5), adv]]
        assert h.handle_requests(lists) == [(1, 0)]
        assert cells[1][1].frame == -1 and cells[1][1].checksum is None
        h.flush()
