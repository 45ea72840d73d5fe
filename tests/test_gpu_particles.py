"""GPU parity of the config-5 particle world SyncTest (ggrs_particle_*): final states, saved cells
(bytes + checksums) and mismatch reports bit-exact against the oracle's restatement."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def inputs_for(O, sessions, frames, P, first=0):
    return np.stack([O.gen_inputs(O.session_seed(first + s), frames, P, 1) for s in range(sessions)], axis=1)


@pytest.mark.parametrize("N,P,maxp,cd,frames,chunks", [
    (64, 2, 17, 16, 60, [1, 20, 39]),
    (1024, 3, 8, 7, 30, [30]),
    (260, 1, 4, 2, 25, [5, 5, 15]),
    (32, 4, 8, 0, 12, [12]),
    (10000, 2, 17, 16, 22, [22]),  # the config-5 entity count (1 MB states)
])
@pytest.mark.parametrize("ept", ["1", "2", "4"])  # entities per thread (GGRS_PW_EPT)
def test_particles_match_oracle(oracle, monkeypatch, ept, N, P, maxp, cd, frames, chunks):
    from ggrs_amd import ParticleEngine
    monkeypatch.setenv("GGRS_PW_EPT", ept)
    S = 5
    inp = inputs_for(oracle, S, frames, P)
    eng = ParticleEngine(S, N, P, maxp, cd, input_capacity=frames + cd + 2)
    eng.add_local_inputs(inp)
    for n in chunks:
        eng.synctest_advance_frames(n)
    eng.synchronize()
    assert eng.current_frame() == frames
    for s in (0, S - 1):
        r = oracle.particles_synctest_run(inp[:, s, :], N, P, maxp, cd, session=s)
        assert r["result"].status == 0
        assert bytes(eng.state(s)) == bytes(r["final_state"]), f"session {s} final state"
        for fr, ck, st in zip(r["ring_frames"], r["ring_cksums"], r["ring_states"]):
            if fr >= 0:
                gck, gst = eng.saved(s, int(fr))
                assert gck == int(ck) and bytes(gst) == bytes(st), (s, int(fr))
    st, _, _ = eng.mismatches()
    assert (st == 0).all()


@pytest.mark.parametrize("ept", ["1", "2", "4"])
def test_particles_mismatch(oracle, monkeypatch, ept):
    from ggrs_amd import ParticleEngine
    monkeypatch.setenv("GGRS_PW_EPT", ept)
    S, N, P, maxp, cd, frames, call = 3, 128, 2, 9, 8, 40, 20
    inp = inputs_for(oracle, S, frames, P)
    eng = ParticleEngine(S, N, P, maxp, cd, input_capacity=frames + cd + 2)
    eng.corrupt_on_load(1, call)
    eng.add_local_inputs(inp)
    eng.synctest_advance_frames(frames)
    st, mf, mm = eng.mismatches()
    r = oracle.particles_synctest_run(inp[:, 1, :], N, P, maxp, cd, session=1, corrupt_frame=call)
    assert r["result"].status == 1
    assert st.tolist() == [0, 1, 0]
    assert mf[1] == r["result"].mismatch_frame == call + 1
    assert int(mm[1]) == int(r["result"].mismatch_mask)
    assert bytes(eng.state(1)) == bytes(r["final_state"])


@pytest.mark.parametrize("ept", ["1", "4"])
def test_particles_state_between_launches(oracle, monkeypatch, ept):
    """The post-call state of a replay call is materialised on read (Advance of the saved cell):
    reading it between launches, in warm-up and in steady state, must equal the oracle's state
    after that many frames, and must not disturb the following launches."""
    from ggrs_amd import ParticleEngine
    monkeypatch.setenv("GGRS_PW_EPT", ept)
    S, N, P, maxp, cd = 3, 300, 2, 6, 5
    chunks = [2, 4, 1, 7, 9]  # ends at frames 2 (warm-up), 6 (first replay), 7, 14, 23
    frames = sum(chunks)
    inp = inputs_for(oracle, S, frames, P)
    eng = ParticleEngine(S, N, P, maxp, cd, input_capacity=frames + cd + 2)
    eng.add_local_inputs(inp)
    done = 0
    for n in chunks:
        eng.synctest_advance_frames(n)
        done += n
        for s in (0, S - 1):
            r = oracle.particles_synctest_run(inp[:done, s, :], N, P, maxp, cd, session=s, ring_states=False)
            assert bytes(eng.state(s)) == bytes(r["final_state"]), (s, done)
    st, _, _ = eng.mismatches()
    assert (st == 0).all()
