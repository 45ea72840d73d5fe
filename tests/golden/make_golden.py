"""Generate tests/golden/*.json from the independent pure-Python restatement (oracle/pyoracle.py).

The reference (Rust) cannot run in this image, and it holds no numeric golden vectors of its own
(SURVEY.md section 4 / 8c), so the fixtures are produced by the Python restatement, which shares
no code with the C oracle it pins (oracle/ggrs_oracle.c) nor with the HIP engine.  Inputs come
from the splitmix64 generator spelled out below (same definition as oracle_gen_inputs).
sinf/cosf values and the [0, 2*pi] digest come straight from this image's glibc libm.

    python tests/golden/make_golden.py        # rewrites the fixtures (about a minute)
"""
import ctypes
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import pyoracle as Py  # noqa: E402

M64 = (1 << 64) - 1


def splitmix64(state):
    state = (state + 0x9E3779B97F4A7C15) & M64
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return state, z ^ (z >> 31)


def gen_inputs(seed, frames, players, model):
    """model 0: uniform [0,15]; model 1: held key (keep previous unless ((r>>8)&7)==0)."""
    st, prev, out = seed, [0] * players, []
    for _ in range(frames):
        row = []
        for p in range(players):
            st, r = splitmix64(st)
            v = r & 15
            if model == 1 and ((r >> 8) & 7) != 0:
                v = prev[p]
            prev[p] = v
            row.append(v)
        out.append(row)
    return out


SYNCTEST_CASES = [
    # name, players, max_prediction, check_distance, input_delay, frames, model, seed
    ("p2_cd7_d2", 2, 8, 7, 2, 2000, 0, 0x6767525300000000),      # config 1 (ex_game_synctest)
    ("p2_cd8_held", 2, 9, 8, 0, 600, 1, 0x6767525300000001),     # config 2 semantics
    ("p4_cd7_d1", 4, 8, 7, 1, 400, 0, 0x6767525300000002),
    ("p1_cd2_d0", 1, 8, 2, 0, 400, 0, 0x6767525300000003),
    ("p3_cd5_d3", 3, 6, 5, 3, 300, 1, 0x6767525300000004),
    ("p2_cd0", 2, 8, 0, 0, 200, 0, 0x6767525300000005),
    ("p2_cd1", 2, 8, 1, 0, 200, 0, 0x6767525300000006),
]


def synctest_fixture(name, P, maxp, cd, d, frames, model, seed):
    inputs = gen_inputs(seed, frames, P, model)
    s = Py.SyncTest(P, maxp, cd, d)
    cks, reqs = [], []
    for f in range(frames):
        r = s.advance_frame(inputs[f])
        assert isinstance(r, str), r
        reqs.append(r)
        cks.append(s.last_checksum)
    ring = []
    for frame, st, ck in s.cells:
        ring.append({"frame": frame, "checksum": ck, "state": st.bincode().hex() if st else None})
    return {
        "name": name, "num_players": P, "max_prediction": maxp, "check_distance": cd,
        "input_delay": d, "frames": frames, "input_model": model, "seed": seed,
        "checksums": cks, "requests_first": reqs[: cd + 3], "requests_last": reqs[-1],
        "request_counts": [len(r) for r in reqs],
        "final_state": s.game.bincode().hex(), "ring": ring,
    }


def f2h(x):
    return struct.unpack("<I", struct.pack("<f", x))[0]


def main():
    libm = ctypes.CDLL("libm.so.6")
    for fn in ("sinf", "cosf"):
        getattr(libm, fn).restype = ctypes.c_float
        getattr(libm, fn).argtypes = [ctypes.c_float]

    out = {"state_new": {str(p): Py.State.new(p).bincode().hex() for p in range(1, 5)}}

    # Fletcher-16 KATs on byte strings (ex_game.rs:45-55)
    st = 12345
    kats = []
    for n in (0, 1, 2, 5, 76, 116, 255, 1000):
        b = bytearray()
        for _ in range(n):
            st, r = splitmix64(st)
            b.append(r & 0xFF)
        kats.append({"bytes": bytes(b).hex(), "fletcher16": Py.fletcher16(b)})
    kats.append({"bytes": (b"\xff" * 300).hex(), "fletcher16": Py.fletcher16(b"\xff" * 300)})
    out["fletcher16"] = kats

    # single advance steps from State::new with every input value, both statuses
    steps = []
    for p in (1, 2, 4):
        for inp in range(16):
            s = Py.State.new(p)
            ins = [((inp + 3 * i) % 16, 0) for i in range(p)]
            s.advance(ins)
            steps.append({"players": p, "inputs": [i for i, _ in ins], "status": [0] * p,
                          "after": s.bincode().hex()})
        s = Py.State.new(p)
        ins = [(1, 2 if i == 0 else 0) for i in range(p)]  # player 0 disconnected -> spins
        s.advance(ins)
        steps.append({"players": p, "inputs": [1] * p, "status": [2] + [0] * (p - 1),
                      "after": s.bincode().hex()})
    out["advance_steps"] = steps

    # glibc sinf/cosf samples, including inputs where glibc is not correctly rounded
    hexes = ["0x1.d12ed2p-12", "0x1.1e377ap-11", "0x1.1475bap+4", "0x1.52e6cp+6", "-0x1.d0f4aap+6"]
    pts = [0.0, 1e-30, 0.5, 0.78539818, 1.0, 1.5707964, 3.1415927, 4.712389, 6.2831855,
           6.2831850, 2.0943951, 119.99999, 120.0, 1000.5, 1e20, -3.0] + [float.fromhex(h) for h in hexes]
    out["sincos"] = [{"x": f2h(x), "sin": f2h(libm.sinf(x)), "cos": f2h(libm.cosf(x))} for x in pts]

    # order-independent digest of libm sinf/cosf over every f32 in [0, 2*pi] (0x00000000 ..
    # 0x40c90fdb = TWO_PI), computed by libm itself through the oracle's threaded loop
    from oracle import oracle as O
    O.build()
    out["sincos_digest_0_2pi"] = {"lo": 0, "hi": 0x40C90FDB, "digest": O.sincos_digest(0, 0x40C90FDB)}

    out["synctest"] = [synctest_fixture(*c) for c in SYNCTEST_CASES]
    path = os.path.join(HERE, "golden.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=0)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
