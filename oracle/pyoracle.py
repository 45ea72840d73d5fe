"""Independent pure-Python restatement of the GGRS SyncTest hot path.  TEST INFRASTRUCTURE ONLY.

Second, independently written restatement of the same reference code the C oracle
(oracle/ggrs_oracle.c) restates; it exists to pin that oracle and to generate the committed
fixtures in tests/golden/ (tests/golden/make_golden.py).  Only tests/ may import it.

f32 arithmetic uses numpy float32 scalars (IEEE single, round-to-nearest, no contraction);
sinf/cosf/fmodf come from this image's glibc libm through ctypes -- the functions Rust's
f32::sin/cos/% call on the reference's CPU path.  numpy's own sin/cos are NOT glibc and are never
used.  Sources restated (caspark/ggrs 0.10.2):
  examples/ex_game/ex_game.rs:10-55 (constants, fletcher16), :236-333 (State, new, advance)
  src/sessions/sync_test_session.rs:61-217, src/sync_layer.rs:144-375, src/input_queue.rs:39-266
The input queue is modelled by its observable behaviour in a SyncTest (every input confirmed,
delay d replays the default input for frames < d; src/input_queue.rs:233-265, :340-353) and the
session's request generation is restated statement by statement.
"""
import ctypes
import struct

import numpy as np

_libm = ctypes.CDLL("libm.so.6")
for _fn in ("sinf", "cosf"):
    getattr(_libm, _fn).restype = ctypes.c_float
    getattr(_libm, _fn).argtypes = [ctypes.c_float]
_libm.fmodf.restype = ctypes.c_float
_libm.fmodf.argtypes = [ctypes.c_float, ctypes.c_float]

f32 = np.float32
NULL_FRAME = -1


def sinf(x):
    return f32(_libm.sinf(float(x)))


def cosf(x):
    return f32(_libm.cosf(float(x)))


def fmodf(a, b):
    return f32(_libm.fmodf(float(a), float(b)))


FPS = 60
WINDOW_HEIGHT = f32(800.0)
WINDOW_WIDTH = f32(600.0)
MOVEMENT_SPEED = f32(15.0) / f32(FPS)
ROTATION_SPEED = f32(2.5) / f32(FPS)
MAX_SPEED = f32(7.0)
FRICTION = f32(0.98)
PI = f32(np.pi)
TWO_PI = f32(2.0) * PI


class State:
    """ex_game.rs:236-243 -- frame, positions[(x, y)], velocities[(vx, vy)], rotations[rot]."""

    def __init__(self, frame, pos, vel, rot):
        self.frame = int(frame)
        self.pos = [list(p) for p in pos]
        self.vel = [list(v) for v in vel]
        self.rot = list(rot)

    def clone(self):
        return State(self.frame, self.pos, self.vel, self.rot)

    @staticmethod
    def new(num_players):  # ex_game.rs:246-269
        r = WINDOW_WIDTH / f32(4.0)
        pos, vel, rots = [], [], []
        with np.errstate(all="ignore"):
            for i in range(num_players):
                rot = f32(i) / f32(num_players) * f32(2.0) * PI
                x = WINDOW_WIDTH / f32(2.0) + r * cosf(rot)
                y = WINDOW_HEIGHT / f32(2.0) + r * sinf(rot)
                pos.append([x, y])
                vel.append([f32(0.0), f32(0.0)])
                rots.append(fmodf(rot + PI, f32(2.0) * PI))
        return State(0, pos, vel, rots)

    def advance(self, inputs):  # ex_game.rs:271-333; inputs = [(inp, status)], status 2 = Disconnected
        self.frame += 1
        with np.errstate(all="ignore"):
            for i in range(len(self.rot)):
                inp, status = inputs[i]
                inp = 4 if status == 2 else inp
                old_x, old_y = self.pos[i]
                old_vx, old_vy = self.vel[i]
                rot = self.rot[i]
                vx = old_vx * FRICTION
                vy = old_vy * FRICTION
                if inp & 1 and not inp & 2:
                    vx = vx + MOVEMENT_SPEED * cosf(rot)
                    vy = vy + MOVEMENT_SPEED * sinf(rot)
                if not inp & 1 and inp & 2:
                    vx = vx - MOVEMENT_SPEED * cosf(rot)
                    vy = vy - MOVEMENT_SPEED * sinf(rot)
                if inp & 4 and not inp & 8:
                    rot = rem_euclid(rot - ROTATION_SPEED, TWO_PI)
                if not inp & 4 and inp & 8:
                    rot = rem_euclid(rot + ROTATION_SPEED, TWO_PI)
                mag = f32(np.sqrt(vx * vx + vy * vy))
                if mag > MAX_SPEED:
                    vx = (vx * MAX_SPEED) / mag
                    vy = (vy * MAX_SPEED) / mag
                x = old_x + vx
                y = old_y + vy
                x = f32(min(max(x, f32(0.0)), WINDOW_WIDTH))
                y = f32(min(max(y, f32(0.0)), WINDOW_HEIGHT))
                self.pos[i] = [x, y]
                self.vel[i] = [vx, vy]
                self.rot[i] = rot

    def bincode(self):
        """bincode 1.x fixint little-endian encoding of the serde-derived State (36 + 20P bytes)."""
        p = len(self.rot)
        b = struct.pack("<iQ", self.frame, p)
        b += struct.pack("<Q", p) + b"".join(struct.pack("<ff", *xy) for xy in self.pos)
        b += struct.pack("<Q", p) + b"".join(struct.pack("<ff", *v) for v in self.vel)
        b += struct.pack("<Q", p) + b"".join(struct.pack("<f", r) for r in self.rot)
        return b


def rem_euclid(a, b):
    r = fmodf(a, b)
    return r + abs(b) if r < f32(0.0) else r


def fletcher16(data):  # ex_game.rs:45-55
    s1 = s2 = 0
    for d in data:
        s1 = (s1 + d) % 255
        s2 = (s2 + s1) % 255
    return (s2 << 8) | s1


class SyncTest:
    """SyncTestSession + SyncLayer + the ex_game request handler, restated.

    Returns per call the request kinds ('S', 'L', 'A') so the reference's structural tests
    (tests/test_synctest_session.rs:14-65) can be replayed against it.
    """

    def __init__(self, num_players, max_prediction, check_distance, input_delay, checksum_fn=None):
        if check_distance >= max_prediction:  # builder.rs:347-351
            raise ValueError("InvalidRequest: Check distance too big.")
        self.P, self.maxp, self.cd, self.delay = num_players, max_prediction, check_distance, input_delay
        self.current = 0
        self.cells = [[NULL_FRAME, None, None] for _ in range(max_prediction + 1)]  # frame, state, cksum
        self.queue = {}  # frame -> tuple(inputs); every synctest input is confirmed
        self.hist = {}
        self.game = State.new(num_players)
        self.last_checksum = None
        self.checksum_fn = checksum_fn or (lambda st: fletcher16(st.bincode()))

    def _inputs(self, frame):
        return [(self.queue[frame][p], 0) for p in range(self.P)]

    def _cell(self, frame):
        return self.cells[frame % len(self.cells)]

    def _consistent(self, fc):  # sync_test_session.rs:173-190
        oldest = self.current - self.cd
        self.hist = {k: v for k, v in self.hist.items() if k >= oldest}
        cell = self._cell(fc)
        if cell[0] != fc:
            return True
        if fc in self.hist:
            return self.hist[fc] == cell[2]
        self.hist[fc] = cell[2]
        return True

    def advance_frame(self, local_inputs):
        """One add_local_input for every player + advance_frame + handle_requests."""
        reqs = []
        cur = self.current
        if self.cd > 0 and cur > self.cd:
            mism = [f for f in range(cur - self.cd, cur + 1) if not self._consistent(f)]
            if mism:
                return ("MismatchedChecksum", cur, mism)
            frame_to = cur - self.cd
            assert frame_to >= cur - self.maxp and self._cell(frame_to)[0] == frame_to
            reqs.append(("L", frame_to))
            self.current = frame_to
            for i in range(cur - frame_to):
                inp = self._inputs(self.current)
                if i > 0:
                    reqs.append(("S", self.current))
                self.current += 1
                reqs.append(("A", inp))
        # add_local_input with input delay: the queue fills frames < delay with the default input
        if cur == 0:
            for f in range(self.delay):
                self.queue[f] = tuple([0] * self.P)
        self.queue[cur + self.delay] = tuple(local_inputs)
        if self.cd > 0:
            reqs.append(("S", self.current))
        reqs.append(("A", self._inputs(self.current)))
        self.current += 1
        for r in reqs:  # Game::handle_requests (ex_game.rs:79-99)
            if r[0] == "L":
                self.game = self._cell(r[1])[1].clone()
            elif r[0] == "S":
                assert self.game.frame == r[1]
                c = self._cell(r[1])
                c[0], c[1], c[2] = r[1], self.game.clone(), self.checksum_fn(self.game)
            else:
                self.game.advance(r[1])
                self.last_checksum = fletcher16(self.game.bincode())
        return "".join(r[0] for r in reqs)
