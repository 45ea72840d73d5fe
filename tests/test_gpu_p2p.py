"""GPU parity of the device P2P rollback decision (ggrs_p2p_*) against the oracle's P2P session
(oracle_p2p_run: P2PSession::advance_frame, p2p_session.rs:265-426) on the same inputs: every
session's display-checksum trace, final state, saved-state ring and rollback/resimulation counts
are bit-exact."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")  # loads torch's HIP runtime before the engine library

pytestmark = pytest.mark.gpu


def stream(S, frames, P, model, seed_base=0x5050):
    from oracle import oracle as o
    return np.stack([o.gen_inputs(o.session_seed(s, seed_base), frames, P, model) for s in range(S)], axis=1)


def check_against_oracle(eng, rows, sessions, frames, trace=True):
    from oracle import oracle as o
    rb, rs = eng.stats()
    tr = eng.trace(0, frames) if trace else None
    for s in sessions:
        out = o.p2p_run(rows[:, s], num_players=eng.num_players, local_mask=eng.local_mask,
                        input_delay=eng.input_delay, max_prediction=eng.max_prediction,
                        latency=eng.remote_latency, predictor=eng.predictor,
                        sparse_saving=getattr(eng, "sparse_saving", False))
        assert out["rc"] == 0
        res = out["result"]
        if tr is not None:
            assert (tr[:, s] == out["ck_trace"]).all(), s
        assert bytes(eng.state(s)) == bytes(out["final_state"]), s
        frames_r, cks, states = eng.ring(s)
        assert (frames_r == out["ring_frames"]).all(), s
        assert (cks == out["ring_cksums"]).all(), s
        assert (states == out["ring_states"]).all(), s
        assert rb[s] == res.rollbacks and rs[s] == res.resim, (s, rb[s], res.rollbacks)


CASES = [
    # P, local players, delay, max_prediction, latency, predictor, input model
    (2, (0,), 0, 8, 4, 0, 1),
    (2, (1,), 2, 8, 7, 0, 0),
    (3, (0,), 0, 7, 1, 0, 0),
    (4, (0, 2), 1, 8, 3, 1, 1),
    (4, (0,), 0, 12, 6, 0, 1),
    (1, (), 0, 8, 2, 0, 1),
    (2, (), 1, 8, 3, 0, 0),
]


@pytest.mark.parametrize("form", ["default", "flat", "lockstep", "unstaged"])
@pytest.mark.parametrize("P,local,delay,mp,D,pred,model", CASES)
def test_p2p_matches_oracle(oracle, P, local, delay, mp, D, pred, model, form):
    """Every kernel form: per-session step sequences with the block's rings in LDS (default, where
    they fit 28 KB) or in HBM ("flat"), calls in lockstep with input rows staged in LDS, and in
    lockstep reading rows from global memory."""
    from ggrs_amd import P2PEngine
    S, frames = 300, 160
    rows = stream(S, frames, P, model)
    eng = P2PEngine(S, num_players=P, local_players=local, input_delay=delay, max_prediction=mp,
                    remote_latency=D, predictor=pred, trace_capacity=frames)
    eng.set_kernel_form(form)
    eng.add_inputs(0, rows)
    # chunks of several sizes: state, queues and stats carry across launches
    for n in (1, 2, 5, 40, 112):
        eng.advance_frames(n)
    assert eng.current_frame() == frames
    check_against_oracle(eng, rows, [0, 1, 63, 64, 150, 299], frames)


@pytest.mark.parametrize("form", ["default", "flat_queues", "canonical", "chains"])
@pytest.mark.parametrize("P,local,delay,mp,D,pred,model", CASES)
def test_p2p_plain_launches_match_oracle(oracle, P, local, delay, mp, D, pred, model, form):
    """Launches without trace, desync history or debug flip: the flat kernel's plain
    specialisation stepping the queues, the canonical flat kernel (rollback decision read off the
    inputs), the chains form, and the default's choice among them (chains at 300 sessions): final
    states, rings, rollback counts and queue states bit-exact with the oracle."""
    from ggrs_amd import P2PEngine
    S, frames = 300, 160
    rows = stream(S, frames, P, model, seed_base=0x7070)
    eng = P2PEngine(S, num_players=P, local_players=local, input_delay=delay, max_prediction=mp,
                    remote_latency=D, predictor=pred)
    eng.set_kernel_form(form)
    eng.add_inputs(0, rows)
    for n in (3, 45, 112):
        eng.advance_frames(n)
    check_against_oracle(eng, rows, [0, 1, 63, 64, 150, 299], frames, trace=False)


def test_p2p_all_sessions_streamed(oracle):
    """Inputs streamed through a small input ring; every session checked."""
    from ggrs_amd import P2PEngine
    S, frames, chunk = 129, 200, 25
    rows = stream(S, frames, 2, 1, seed_base=77)
    eng = P2PEngine(S, num_players=2, local_players=(0,), input_delay=1, max_prediction=8,
                    remote_latency=5, input_capacity=40, trace_capacity=frames)
    for f0 in range(0, frames, chunk):
        eng.add_inputs(f0, rows[f0:f0 + chunk])
        eng.advance_frames(chunk)
    check_against_oracle(eng, rows, range(S), frames)


def test_p2p_input_checks(oracle):
    from ggrs_amd import InvalidRequest, P2PEngine
    eng = P2PEngine(10, num_players=2, remote_latency=3, input_capacity=20)
    with pytest.raises(InvalidRequest):
        eng.advance_frames(1)                      # Missing local input
    eng.add_inputs(0, np.zeros((10, 10, 2), np.uint8))
    with pytest.raises(InvalidRequest):
        eng.add_inputs(5, np.zeros((1, 10, 2), np.uint8))  # out of order
    with pytest.raises(InvalidRequest):
        eng.add_inputs(10, np.zeros((15, 10, 2), np.uint8))  # ring full
    eng.advance_frames(10)
    eng.add_inputs(10, np.zeros((15, 10, 2), np.uint8))
    eng.advance_frames(15)
    assert eng.current_frame() == 25
    rb, rs = eng.stats()
    assert (rb == 0).all() and (rs == 0).all()



SPARSE_CASES = [
    # P, local players, delay, max_prediction, latency, predictor, input model
    (2, (0,), 0, 8, 4, 0, 1),
    (2, (1,), 2, 8, 7, 0, 0),
    (4, (0, 2), 1, 8, 3, 1, 1),
    (3, (0,), 0, 12, 2, 0, 0),
]


@pytest.mark.parametrize("form", ["default", "flat", "lockstep"])
@pytest.mark.parametrize("P,local,delay,mp,D,pred,model", SPARSE_CASES)
def test_p2p_sparse_saving_matches_oracle(oracle, P, local, delay, mp, D, pred, model, form):
    """Sparse saving (builder.rs:160-169): rollbacks from the last save, saves only at
    min_confirmed or when the last save would leave the window; every session bit-exact with the
    oracle's P2PSession including which frames the ring cells hold."""
    from ggrs_amd import P2PEngine
    S, frames = 300, 200
    rows = stream(S, frames, P, model)
    eng = P2PEngine(S, num_players=P, local_players=local, input_delay=delay, max_prediction=mp,
                    remote_latency=D, predictor=pred, trace_capacity=frames)
    eng.set_sparse_saving(True)
    eng.set_kernel_form(form)
    eng.add_inputs(0, rows)
    for n in (1, 3, 17, 79, 100):
        eng.advance_frames(n)
    check_against_oracle(eng, rows, [0, 1, 63, 64, 150, 299], frames)


@pytest.mark.parametrize("form", ["default", "flat_queues", "mixed"])
@pytest.mark.parametrize("P,local,delay,mp,D,pred,model", SPARSE_CASES)
def test_p2p_sparse_plain_launches_match_oracle(oracle, P, local, delay, mp, D, pred, model, form):
    """Sparse saving in launches without trace/debug: the canonical sparse kernel (default), the
    queue-stepping flat kernel's plain sparse specialisation, and the two alternating launch by
    launch ("mixed": each continues from the other's queues, last save and ring tags): states,
    rings with their frame tags, and rollback / resimulation counts bit-exact."""
    from ggrs_amd import P2PEngine
    S, frames = 300, 200
    rows = stream(S, frames, P, model, seed_base=0x3131)
    eng = P2PEngine(S, num_players=P, local_players=local, input_delay=delay, max_prediction=mp,
                    remote_latency=D, predictor=pred)
    eng.set_sparse_saving(True)
    eng.add_inputs(0, rows)
    for k, n in enumerate((2, 61, 5, 1, 131)):
        if form == "mixed":
            eng.set_kernel_form(("canonical", "flat_queues")[k % 2])
        elif form != "default":
            eng.set_kernel_form(form)
        eng.advance_frames(n)
    check_against_oracle(eng, rows, [0, 1, 63, 64, 150, 299], frames, trace=False)


@pytest.mark.parametrize("P,local,delay,D", [(2, (0,), 0, 3), (2, (1,), 2, 1), (4, (0, 2), 1, 4), (3, (0,), 0, 2),
                                             (2, (), 1, 2)])
def test_lockstep_mode_matches_oracle(oracle, P, local, delay, D):
    """max_prediction 0 = lockstep mode (builder.rs:134-147): calls advance only with every
    player's input of the current frame confirmed, never save, load or resimulate
    (p2p_session.rs:301-310,393-407).  Display-checksum trace per call, final state, empty ring and
    the session frame equal the oracle P2PSession's, across launches of several sizes."""
    from ggrs_amd import P2PEngine
    S, frames = 300, 160
    rows = stream(S, frames, P, 1, seed_base=0x10C5)
    eng = P2PEngine(S, num_players=P, local_players=local, input_delay=delay, max_prediction=0,
                    remote_latency=D, trace_capacity=frames)
    eng.set_sparse_saving(True)  # ignored in lockstep mode, as the reference does (:187-197)
    eng.add_inputs(0, rows)
    for n in (1, 2, 5, 40, 112):
        eng.advance_frames(n)
    assert eng.calls() == frames
    ref = oracle.p2p_run(rows[:, 0], num_players=P, local_mask=eng.local_mask, input_delay=delay,
                         max_prediction=0, latency=D)
    assert eng.current_frame() == int.from_bytes(ref["final_state"][:4].tobytes(), "little") < frames
    check_against_oracle(eng, rows, [0, 1, 63, 64, 150, 299], frames)


def test_full_size_p2p_bench_config(oracle):
    """The P2P bench configuration at full size: 65,536 sessions, 2 players (1 remote, inputs 4
    frames late), max_prediction 8, held-key inputs, 64-call launches on the default (LDS-ring,
    plain) kernel; sampled sessions' final state, ring and rollback counts bit-exact."""
    from ggrs_amd import P2PEngine, synth
    S, frames, P = 65536, 128, 2
    rows = synth.gen_inputs(9, S, frames, P, synth.MODEL_HELD)
    eng = P2PEngine(S, num_players=P, local_players=(0,), input_delay=0, max_prediction=8, remote_latency=4,
                    input_capacity=frames + 6)
    eng.add_inputs(0, rows)
    for _ in range(frames // 64):
        eng.advance_frames(64)
    rng = np.random.default_rng(2)
    sessions = sorted(set([0, 1, 63, 64, S // 2, S - 1] + rng.integers(0, S, 8).tolist()))
    check_against_oracle(eng, rows, sessions, frames, trace=False)
    rb, _ = eng.stats()
    assert rb.sum() > S  # rollbacks happen throughout
    # EVERY session's final state and rollback count (oracle_p2p_batch)
    from oracle import every_lane
    r = every_lane.p2p(eng, rows, P=P, maxp=8, latency=4)
    assert r["rc_mismatched"] == r["final_state_mismatched"] == r["rollbacks_mismatched"] == 0, r


@pytest.mark.parametrize("form", ["default", "flat", "chains"])
def test_config2_p2p_shape(oracle, form):
    """BASELINE config 2 in its P2P form: 4096 sessions, 2 players, the remote
    player's inputs 8 frames late, max_prediction 9, repeat-last prediction
    (input_queue.rs:128-161), held-key inputs, 64-call launches -- the shape `bench.py --workload
    p2p --sessions 4096 --latency 8 --max-prediction 9` measures.  Sampled sessions' final state,
    ring, trace and rollback/resimulation counts bit-exact against the oracle's P2PSession."""
    from ggrs_amd import P2PEngine, synth
    S, frames, P = 4096, 192, 2
    rows = synth.gen_inputs(0, S, frames, P, synth.MODEL_HELD)
    eng = P2PEngine(S, num_players=P, local_players=(0,), input_delay=0, max_prediction=9, remote_latency=8,
                    input_capacity=frames + 10)
    eng.set_kernel_form(form)
    eng.add_inputs(0, rows)
    for _ in range(frames // 64):
        eng.advance_frames(64)
    rng = np.random.default_rng(4)
    sessions = sorted(set([0, 1, 63, 64, 2047, S - 1] + rng.integers(0, S, 10).tolist()))
    check_against_oracle(eng, rows, sessions, frames, trace=False)
    rb, rs = eng.stats()
    assert rb.sum() > 0 and rs.sum() >= 8 * rb.sum() - 8 * S  # rollbacks of up to 8 frames
    from oracle import every_lane
    r = every_lane.p2p(eng, rows, P=P, maxp=9, latency=8)  # every session
    assert r["rc_mismatched"] == r["final_state_mismatched"] == r["rollbacks_mismatched"] == 0, r


@pytest.mark.parametrize("P,local,delay,mp,D,pred,model", CASES)
def test_p2p_chains_form_matches_oracle(oracle, P, local, delay, mp, D, pred, model):
    """The chains form (every call as the chain of D + 1 advances from the confirmed state,
    pipelined over (D + 1) x players lanes per session) in launches of uneven length -- the first
    D calls on the flattened form, launches shorter than D, a launch split for its LDS rows --
    then alternating with the flattened form: states, rings, rollback and resimulation counts
    bit-exact against the oracle's P2PSession after every launch."""
    from ggrs_amd import P2PEngine
    S, frames = 300, 170
    rows = stream(S, frames, P, model, seed_base=0x6060)
    eng = P2PEngine(S, num_players=P, local_players=local, input_delay=delay, max_prediction=mp,
                    remote_latency=D, predictor=pred, input_capacity=frames + 8)
    eng.add_inputs(0, rows)
    done = 0
    for k, (n, form) in enumerate([(2, "chains"), (1, "chains"), (9, "chains"), (40, "chains"), (3, "flat"),
                                   (1, "chains"), (50, "chains"), (20, "flat"), (44, "chains")]):
        eng.set_kernel_form(form)
        eng.advance_frames(n)
        done += n
        if k in (3, 6, 8):
            check_against_oracle(eng, rows[:done], [0, 1, 63, 64, 150, 299], done, trace=False)
    assert done == frames


CHAINS8_CASES = [
    # P, local players, delay, max_prediction, latency 8, predictor, input model
    (2, (0,), 0, 9, 8, 0, 1),
    (2, (1,), 2, 9, 8, 1, 0),
    (2, (), 1, 10, 8, 0, 0),
]


@pytest.mark.parametrize("P,local,delay,mp,D,pred,model", CHAINS8_CASES)
def test_p2p_chains_latency8_matches_oracle(oracle, P, local, delay, mp, D, pred, model):
    """The chains form's compile-time latency-8 kernel (config 2's P2P shape: DPP rotation, decoded
    input records, sin/cos one step ahead) in launches of uneven length -- shorter than a batch,
    not a multiple of 8, one split for its LDS budget (300 calls) -- with a partial last block
    (301 sessions), PredictDefault, input delay and no local player: bit-exact against the
    oracle's P2PSession after every checked launch."""
    from ggrs_amd import P2PEngine
    S, frames = 301, 398
    rows = stream(S, frames, P, model, seed_base=0x7171)
    eng = P2PEngine(S, num_players=P, local_players=local, input_delay=delay, max_prediction=mp,
                    remote_latency=D, predictor=pred, input_capacity=frames + 8)
    eng.add_inputs(0, rows)
    done = 0
    for k, (n, form) in enumerate([(2, "chains"), (7, "chains"), (9, "chains"), (300, "chains"), (3, "flat"),
                                   (13, "chains"), (64, "chains")]):
        eng.set_kernel_form(form)
        eng.advance_frames(n)
        done += n
        if k in (2, 3, 6):
            check_against_oracle(eng, rows[:done], [0, 1, 3, 4, 150, 299, 300], done, trace=False)
    assert done == frames


def test_p2p_chains_form_rejects_non_plain(oracle):
    """Forcing the chains form where it does not apply is an error, not a silent fallback."""
    from ggrs_amd import P2PEngine
    from ggrs_amd._lib import GgrsError
    eng = P2PEngine(8, num_players=2, local_players=(0,), max_prediction=8, remote_latency=4, trace_capacity=16)
    eng.add_inputs(0, stream(8, 16, 2, 1))
    eng.set_kernel_form("chains")
    with pytest.raises(GgrsError):
        eng.advance_frames(8)


@pytest.mark.parametrize("P,local,delay,mp,D,form", [(2, (0,), 0, 8, 3, "canonical"), (2, (1,), 1, 7, 5, "canonical"),
                                                     (4, (0, 2), 0, 8, 4, "canonical"), (2, (0,), 0, 8, 3, "default")])
def test_p2p_single_call_launches_match_oracle(oracle, P, local, delay, mp, D, form):
    """advance_frames(1) per tick on the canonical flat kernel with remote_latency >= 2 and uniform
    inputs (a misprediction at almost every call): a rollback in a launch's first calls re-saves
    frames before the launch's first frame (adjust_gamestate saves every replayed frame but the
    loaded one, p2p_session.rs:696-706), and those cells must reach HBM -- the next launch loads
    them.  State, whole ring and stats bit-exact with the oracle after every launch."""
    from ggrs_amd import P2PEngine
    S, frames = 130, 36
    rows = stream(S, frames, P, 0, seed_base=0x5151)
    eng = P2PEngine(S, num_players=P, local_players=local, input_delay=delay, max_prediction=mp,
                    remote_latency=D, input_capacity=frames + 8)
    eng.set_kernel_form(form)
    eng.add_inputs(0, rows)
    for done in range(1, frames + 1):
        eng.advance_frames(1)
        if done >= D:
            check_against_oracle(eng, rows[:done], [0, 64, 129], done, trace=False)
    rb, _ = eng.stats()
    assert (rb > frames // 2).all()  # uniform inputs: rollbacks at most calls


def test_p2p_forms_interleave_with_equal_queues(oracle):
    """Every plain form leaves the InputQueue state the others continue from: launches alternate
    between the queue-stepping flat kernel, the canonical flat kernel and the chains form, with
    the device queue words equal to the queue-stepping kernel's after each launch."""
    from ggrs_amd import P2PEngine
    S, frames, P = 200, 150, 2
    rows = stream(S, frames, P, 1, seed_base=0x8181)
    engs = {}
    for k in ("flat_queues", "mixed"):
        e = P2PEngine(S, num_players=P, local_players=(1,), input_delay=1, max_prediction=8, remote_latency=3,
                      input_capacity=frames + 8)
        e.add_inputs(0, rows)
        engs[k] = e
    engs["flat_queues"].set_kernel_form("flat_queues")
    for k, n in enumerate((5, 17, 1, 30, 2, 40, 55)):
        engs["mixed"].set_kernel_form(("canonical", "chains", "flat_queues")[k % 3])
        for e in engs.values():
            e.advance_frames(n)
        qa, qb = engs["flat_queues"].queues(), engs["mixed"].queues()
        assert (qa == qb).all(), k
    check_against_oracle(engs["mixed"], rows, [0, 1, 63, 64, 150, 199], frames, trace=False)
