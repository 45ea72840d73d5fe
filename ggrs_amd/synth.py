"""Synthetic input streams for benchmarks and large parity runs.

Session s draws from splitmix64 seeded with (base + s), one draw r per (frame, player) in that
order; model 0 ("uniform") plays r & 15, model 1 ("held key") keeps the player's previous input
unless ((r >> 8) & 7) == 0, then plays r & 15.  Vectorised over sessions with numpy uint64
arithmetic (wrapping mod 2^64, like the C definition tests check it against).
"""
import numpy as np

SEED_BASE = 0x6767525300000000
MODEL_UNIFORM, MODEL_HELD = 0, 1
_G = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def gen_inputs(first_session, sessions, frames, players, model=MODEL_UNIFORM, base=SEED_BASE):
    """[frames][sessions][players] u8 inputs for sessions first_session .. first_session+sessions-1."""
    st = (np.uint64(base) + np.arange(first_session, first_session + sessions, dtype=np.uint64))
    prev = np.zeros((sessions, players), np.uint8)
    out = np.empty((frames, sessions, players), np.uint8)
    with np.errstate(over="ignore"):
        for f in range(frames):
            for p in range(players):
                st = st + _G
                z = st
                z = (z ^ (z >> np.uint64(30))) * _M1
                z = (z ^ (z >> np.uint64(27))) * _M2
                r = z ^ (z >> np.uint64(31))
                v = (r & np.uint64(15)).astype(np.uint8)
                if model == MODEL_HELD:
                    keep = ((r >> np.uint64(8)) & np.uint64(7)) != 0
                    v = np.where(keep, prev[:, p], v)
                prev[:, p] = v
                out[f, :, p] = v
    return out


def jitter_arrivals(first_session, sessions, calls, max_prediction, stalls=False, seed=0x5C4E,
                    stall_every=48, stall_len=None):
    """[calls][sessions] int32 remote-arrival schedules (ggrs_p2p_add_arrivals): per session and call
    a lag drawn uniformly from [1, max_prediction - 1], made non-decreasing, so the remote inputs
    come in bursts of differing size and sessions roll back to differing depths; with `stalls`,
    every session also loses its network for stall_len calls (default max_prediction + 4) once per
    stall_every calls at its own phase, so it reaches the prediction threshold and skips calls
    (p2p_session.rs:393-423) before the burst arrives.  Deterministic in (seed, first_session)."""
    rng = np.random.default_rng([seed, first_session])
    c = np.arange(calls, dtype=np.int32)[:, None]
    upto = c - rng.integers(1, max(2, max_prediction), size=(calls, sessions), dtype=np.int32)
    if stalls:
        stall_len = stall_len or max_prediction + 4
        phase = rng.integers(0, stall_every, size=sessions, dtype=np.int32)[None, :]
        upto[(c + phase) % stall_every < stall_len] = -1
    np.maximum(upto, -1, out=upto)
    return np.maximum.accumulate(upto, axis=0)
