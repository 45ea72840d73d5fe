"""GPU parity of the speculative branch rollback (ggrs_branch_*): every lane's replay equals the
oracle's P2PSession::adjust_gamestate (p2p_session.rs:658-714 + the save at :337) run with that
branch's inputs; the trunk equals the confirmed-input replay; survival bits equal "assumed the
confirmed inputs"; the report checksum is fletcher16 of the confirmed state.  Bit-exact."""
import numpy as np
import pytest

# torch (plumbing for device buffers / RCCL) must load its bundled HIP runtime before the engine
# library: both link libamdhip64.so.7, and whichever loads first serves the process.  bench.py
# imports torch first for the same reason.
torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def branch_inputs(eng, truth, f_c, lane, W):
    """[W][P] inputs lane `lane` plays from trunk frame f_c (host restatement of the generator)."""
    s, b = divmod(lane, eng.branches)
    last = truth[f_c - 1, s] if f_c > 0 else np.zeros(eng.num_players, np.uint8)
    rows = []
    for k in range(W):
        assumed = eng.assumed_remote(b, k, last)
        rows.append([truth[f_c + k, s, q] if a is None else a for q, a in enumerate(assumed)])
    return np.array(rows, np.uint8)


def check_every_lane(oracle, eng, truth):
    """Every lane's last speculated window, every report checksum and survival bit, no desync
    (oracle/every_lane.py: oracle_p2p_replay_batch from the oracle's confirmed trunk)."""
    from oracle import every_lane
    r = every_lane.branch(eng, truth)
    assert r["cells_mismatched"] == 0, (r["cells_mismatched"], r["first_bad_lane"])
    assert r["report_mismatched"] == 0 and r["survivors_mismatched"] == 0 and r["desyncs"] == 0
    for s in (0, eng.num_sessions - 1):
        assert bytes(eng.trunk(s)) == bytes(r["trunk_states"][s])


def run_rounds(oracle, eng, truth, rounds, lanes_to_check):
    S, P, W = eng.num_sessions, eng.num_players, eng.window
    trunks = {s: oracle.state_new(P) for s in set(l // eng.branches for l in lanes_to_check) | {0}}
    for r in range(rounds):
        f_c = eng.trunk_frame()
        assert f_c == r
        eng.speculate()
        eng.synchronize()
        for lane in lanes_to_check:
            s = lane // eng.branches
            states, cks, _ = oracle.p2p_replay(trunks[s], f_c, branch_inputs(eng, truth, f_c, lane, W))
            for k in range(W):
                ck, st = eng.lane_state(lane, f_c + k + 1)
                assert ck == int(cks[k]) and bytes(st) == bytes(states[k]), (lane, r, k)
        eng.confirm()
        ck, bits = eng.report()
        surv = eng.survivors()
        for s in trunks:
            trunks[s] = oracle.state_advance(trunks[s], truth[f_c, s])
            assert bytes(eng.trunk(s)) == bytes(trunks[s])
            assert int(ck[s]) == oracle.fletcher16(bytes(trunks[s]))
        for lane in lanes_to_check:
            s, b = divmod(lane, eng.branches)
            want = branch_inputs(eng, truth, f_c, lane, 1)[0]
            assert surv[lane] == bool((want == truth[f_c, s]).all()), (lane, r)
    assert (eng.desync() == -1).all()


def test_config3_enumeration(oracle):
    """Config 3: 1 session x 16^4 branches over a 4-frame window, 2 players (1 remote)."""
    from ggrs_amd import BranchEngine, synth
    eng = BranchEngine(1, num_players=2, remote_mask=0b10, window=4, branches=16 ** 4, alphabet=16)
    rounds = 6
    truth = synth.gen_inputs(0, 1, rounds + 8, 2, synth.MODEL_HELD)
    eng.add_inputs(0, truth)
    rng = np.random.default_rng(3)
    lanes = sorted(set([0, 1, 15, 16, 255, 4096, 65535] + rng.integers(0, 65536, 10).tolist()))
    run_rounds(oracle, eng, truth, rounds, lanes)
    # exactly the 16^3 branches whose digit 0 matched the confirmed input survive each round
    surv = eng.survivors()
    assert surv.sum() == 16 ** 3


@pytest.mark.parametrize("branches,window,P,mask", [(1, 8, 4, 0b1110), (16, 8, 4, 0b0010), (16, 3, 2, 0b01),
                                                    (256, 5, 3, 0b110)])
def test_generators_many_sessions(oracle, branches, window, P, mask):
    from ggrs_amd import BranchEngine, synth
    S = 300
    eng = BranchEngine(S, num_players=P, remote_mask=mask, window=window, branches=branches, alphabet=16)
    rounds = 5
    truth = synth.gen_inputs(7, S, rounds + window + 2, P, synth.MODEL_HELD)
    eng.add_inputs(0, truth)
    L = S * branches
    lanes = sorted(set([0, 1, branches, L - 1, L // 2, 63, 64]))
    run_rounds(oracle, eng, truth, rounds, lanes)


@pytest.mark.parametrize("launches", ["fused", "per_round"])
@pytest.mark.parametrize("S,B,A", [(200, 16, 16), (150, 27, 3), (7, 729, 3), (300, 1, 16)])
def test_native_rounds_equal_single_rounds(oracle, launches, S, B, A):
    """rounds(n) (one fused launch, or back-to-back native launches) leaves every trunk, report,
    ring and survivor set exactly as n single speculate + confirm calls; the survival bits feed the
    next round's desync check.  Branch counts 27 and 729 put a session's lanes across blocks."""
    from ggrs_amd import BranchEngine, synth
    W, n = 6, 9
    truth = synth.gen_inputs(11, S, 2 * n + W + 2, 4, synth.MODEL_HELD)
    engs = [BranchEngine(S, num_players=4, remote_mask=0b0110, window=W, branches=B, alphabet=A) for _ in (0, 1)]
    for e in engs:
        e.add_inputs(0, truth)
    engs[0].set_round_launches(launches == "per_round")
    engs[0].rounds(3)  # two calls: the second starts from a previous confirm
    engs[0].rounds(n - 3)
    for _ in range(n):
        engs[1].speculate()
        engs[1].confirm()
    for lane in (0, 1, B - 1, B, S * B // 2, S * B - 1):
        for f in range(n + 1, n + W):
            a0, a1 = engs[0].lane_state(lane, f), engs[1].lane_state(lane, f)
            assert a0[0] == a1[0] and bytes(a0[1]) == bytes(a1[1]), (lane, f)
    for e in engs:
        e.synchronize()
    assert engs[0].trunk_frame() == engs[1].trunk_frame() == n
    for s in (0, 1, S - 1):
        assert bytes(engs[0].trunk(s)) == bytes(engs[1].trunk(s))
    a, b = engs[0].report(), engs[1].report()
    assert (a[0] == b[0]).all() and (a[1] == b[1]).all()
    assert (engs[0].desync() == -1).all() and (engs[1].desync() == -1).all()
    st = oracle.state_new(4)
    for f in range(n):
        st = oracle.state_advance(st, truth[f, 0])
    assert bytes(engs[0].trunk(0)) == bytes(st)


def test_report_to_device_buffer(oracle):
    """confirm() can copy the report into a caller-owned device buffer (the all-gather input)."""
    from ggrs_amd import BranchEngine, synth
    eng = BranchEngine(100, num_players=2, remote_mask=0b10, window=4, branches=16, alphabet=16)
    truth = synth.gen_inputs(0, 100, 20, 2)
    eng.add_inputs(0, truth)
    buf = torch.zeros(eng.report_bytes, dtype=torch.uint8, device="cuda")
    eng.speculate()
    eng.confirm(buf.data_ptr())
    eng.synchronize()
    host = buf.cpu().numpy()
    ck, bits = eng.report()
    assert (host[:200].view(np.uint16) == ck).all()
    assert (host[eng.report_ck_bytes:].view(np.uint64) == bits).all()


def test_full_size_config4(oracle):
    """Config 4 at full per-GPU size: 8192 four-player sessions x 16 branches = 131,072 lanes,
    window 8.  Single rounds checked lane by lane against the oracle's adjust_gamestate replay on
    sampled lanes each round; then EVERY lane of the single-round engine and of the fused rounds
    launch (the bench path) against the oracle (check_every_lane)."""
    from ggrs_amd import BranchEngine, synth
    S, B, P, mask, W, rounds = 8192, 16, 4, 0b1110, 8, 3
    truth = synth.gen_inputs(5, S, 2 * rounds + W + 2, P, synth.MODEL_HELD)
    eng = BranchEngine(S, num_players=P, remote_mask=mask, window=W, branches=B, alphabet=16)
    eng.add_inputs(0, truth)
    L = S * B
    rng = np.random.default_rng(4)
    lanes = sorted(set([0, 1, 15, 16, L // 2, L - 17, L - 1] + rng.integers(0, L, 9).tolist()))
    run_rounds(oracle, eng, truth, rounds, lanes)
    check_every_lane(oracle, eng, truth)
    fused = BranchEngine(S, num_players=P, remote_mask=mask, window=W, branches=B, alphabet=16)
    fused.add_inputs(0, truth)
    fused.rounds(rounds)
    fused.synchronize()
    check_every_lane(oracle, fused, truth)


@pytest.mark.parametrize("S,B,A,P,mask,W", [(1, 16 ** 4, 16, 2, 0b10, 4), (200, 16, 16, 2, 0b01, 6),
                                           (7, 729, 3, 4, 0b0100, 6), (40, 9, 3, 3, 0b001, 2),
                                           (5, 16, 16, 2, 0b10, 1), (33, 64, 4, 4, 0b1000, 5)])
def test_prefix_rounds_equal_full_rounds(oracle, S, B, A, P, mask, W):
    """Prefix-shared rounds (one remote player, enumerated: every lane advances only that player,
    the local players' window and the depth-k representatives' cells shared) leave every lane's
    cell -- resolved to its representative -- every trunk, report, survivor set and desync record
    exactly as the full replay and as per-round speculate + confirm; sampled lanes equal the oracle's
    adjust_gamestate replay."""
    from ggrs_amd import BranchEngine, synth
    n = 7
    truth = synth.gen_inputs(13, S, 2 * n + W + 3, P, synth.MODEL_HELD)
    engs = {f: BranchEngine(S, num_players=P, remote_mask=mask, window=W, branches=B, alphabet=A)
            for f in ("fused", "full", "per_round")}
    for f, e in engs.items():
        e.add_inputs(0, truth)
        e.set_round_form(f)
        e.rounds(2)   # the second launch starts from a previous confirm (survivor check)
        e.rounds(n - 2)
        e.synchronize()
    L = S * B
    rng = np.random.default_rng(5)
    lanes = sorted(set([0, 1, A - 1, A, B - 1, B % L, L // 2, L - 1] + rng.integers(0, L, 12).tolist()))
    ref = engs["per_round"]
    for f, e in engs.items():
        assert e.trunk_frame() == n
        a, b = e.report(), ref.report()
        assert (a[0] == b[0]).all() and (a[1] == b[1]).all(), f
        assert (e.desync() == -1).all(), f
        for s in (0, S // 2, S - 1):
            assert bytes(e.trunk(s)) == bytes(ref.trunk(s)), (f, s)
        for lane in lanes:
            for fr in range(n - 1, n + W):
                x, y = e.lane_state(lane, fr), ref.lane_state(lane, fr)
                assert x[0] == y[0] and bytes(x[1]) == bytes(y[1]), (f, lane, fr)
    # against the oracle: the last round's replay from trunk frame n - 1
    fused = engs["fused"]
    for lane in lanes[:6]:
        s = lane // B
        st = oracle.state_new(P)
        for fr in range(n - 1):
            st = oracle.state_advance(st, truth[fr, s])
        states, cks, _ = oracle.p2p_replay(st, n - 1, branch_inputs(fused, truth, n - 1, lane, W))
        for k in range(W):
            ck, got = fused.lane_state(lane, n + k)
            assert ck == int(cks[k]) and bytes(got) == bytes(states[k]), (lane, k)


@pytest.mark.parametrize("splits", [(3, 1, 3), (4, 2, 8), (1, 1, 1, 5)])
def test_prefix_pipe_ramp_forms(splits):
    """The pipelined prefix kernel at W = 4 (compile-time W: a launch of n >= W - 1 rounds steps
    only the stages that hold a round in its ramp and drain, shorter launches take the guarded
    form): launches of n = W - 1 exactly, fewer and more rounds leave every trunk, report and
    sampled cell as per-round speculate + confirm."""
    from ggrs_amd import BranchEngine, synth
    S, B, A, P, mask, W = 3, 16 ** 3, 16, 2, 0b10, 4
    n = sum(splits)
    truth = synth.gen_inputs(21, S, 2 * n + W + 3, P, synth.MODEL_HELD)
    engs = {f: BranchEngine(S, num_players=P, remote_mask=mask, window=W, branches=B, alphabet=A)
            for f in ("fused", "per_round")}
    for f, e in engs.items():
        e.add_inputs(0, truth)
        e.set_round_form(f)
        for k in splits:
            e.rounds(k)
        e.synchronize()
    a, b = engs["fused"], engs["per_round"]
    assert a.trunk_frame() == b.trunk_frame() == n
    ra, rb = a.report(), b.report()
    assert (ra[0] == rb[0]).all() and (ra[1] == rb[1]).all()
    assert (a.desync() == b.desync()).all()
    for s in range(S):
        assert bytes(a.trunk(s)) == bytes(b.trunk(s)), s
    rng = np.random.default_rng(9)
    L = S * B
    for lane in sorted(set([0, 1, A, B - 1, L - 1] + rng.integers(0, L, 16).tolist())):
        for fr in range(n - 1, n + W):
            x, y = a.lane_state(lane, fr), b.lane_state(lane, fr)
            assert x[0] == y[0] and bytes(x[1]) == bytes(y[1]), (lane, fr)


def test_config3_fused_rounds_full_size(oracle):
    """Config 3 through the bench's path (fused prefix-shared rounds): 16 rounds, then EVERY one of
    the 65,536 lanes' last window (4 cells each, depth-4 cells included) against the oracle's
    replay, the trunk, the report and the 16^3 survivors."""
    from ggrs_amd import BranchEngine, synth
    eng = BranchEngine(1, num_players=2, remote_mask=0b10, window=4, branches=16 ** 4, alphabet=16)
    n = 16
    truth = synth.gen_inputs(0, 1, n + 8, 2, synth.MODEL_HELD)
    eng.add_inputs(0, truth)
    eng.rounds(n)
    eng.synchronize()
    check_every_lane(oracle, eng, truth)
    assert eng.survivors().sum() == 16 ** 3


def test_prefix_rounds_chunked_launches_and_reports(oracle):
    """More rounds than one prefix launch's LDS holds input rows for (ns_max sessions per block x
    (n + W - 1) rows > 32 KiB: launch_rounds splits them into chunks), with every round's report
    written to a device buffer (ggrs_branch_rounds_reports, the per-round copy offsets of each
    chunk): reports, trunks, desync records and sampled cells equal per-round speculate + confirm
    (ADVICE r3)."""
    import torch
    from ggrs_amd import BranchEngine, synth
    S, B, A, P, mask, W, n = 300, 4, 4, 2, 0b10, 5, 130
    truth = synth.gen_inputs(17, S, n + W + 3, P, synth.MODEL_HELD)
    engs, bufs = {}, {}
    for f in ("fused", "per_round"):
        e = BranchEngine(S, num_players=P, remote_mask=mask, window=W, branches=B, alphabet=A,
                         input_capacity=n + W + 4)
        e.add_inputs(0, truth)
        e.set_round_form(f)
        bufs[f] = torch.zeros((n, e.report_bytes), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        if f == "fused":
            e.rounds_to_tensor(bufs[f], n)
        else:  # separate speculate / confirm launches, each confirm copying its report
            for r in range(n):
                e.speculate()
                e.confirm(bufs[f][r].data_ptr())
        e.synchronize()
        engs[f] = e
    a, b = engs["fused"], engs["per_round"]
    assert a.trunk_frame() == b.trunk_frame() == n
    assert torch.equal(bufs["fused"], bufs["per_round"])
    assert (a.desync() == -1).all() and (b.desync() == -1).all()
    ra, rb = a.report(), b.report()
    assert (ra[0] == rb[0]).all() and (ra[1] == rb[1]).all()
    assert bytes(bufs["fused"][-1, :2 * S].cpu().numpy()) == ra[0].tobytes()
    for s in (0, 1, S // 2, S - 1):
        assert bytes(a.trunk(s)) == bytes(b.trunk(s)), s
    st = oracle.state_new(P)
    for fr in range(n):
        st = oracle.state_advance(st, truth[fr, 0])
    assert bytes(a.trunk(0)) == bytes(st)
    rng = np.random.default_rng(11)
    L = S * B
    for lane in sorted(set([0, 1, A, B - 1, L - 1] + rng.integers(0, L, 12).tolist())):
        for fr in range(n - 1, n + W):
            x, y = a.lane_state(lane, fr), b.lane_state(lane, fr)
            assert x[0] == y[0] and bytes(x[1]) == bytes(y[1]), (lane, fr)
