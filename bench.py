#!/usr/bin/env python3
"""bench.py -- resimulated session-frames/s of the batched SyncTest rollback program on MI355X.

Workload (BASELINE.json configs[1]): ex_game state x 4096 independent
sessions per GPU, an 8-frame rollback every frame (SyncTestSession with check_distance 8,
max_prediction 9), 2 players, held-key synthetic inputs.  One step = one fused launch running
`--frames-per-step` SyncTest frames on every session: per frame and session 1 LoadGameState,
8 resimulated AdvanceFrames (the metric's unit), 8 SaveGameStates with fused Fletcher-16, the
checksum comparisons, and the new frame's AdvanceFrame.

Multi-GPU: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) this process is one
rank; run plainly with `--gpus N > 1` it first starts the N ranks itself (one torch.distributed.run
child on 127.0.0.1, launched before anything imports torch or touches the GPU) and forwards rank
0's line.  Sessions are sharded across ranks with no data-path collective (SyncTest has no
exchange step), so scaling is weak and `value` is the sum of all ranks' resimulated
session-frames over the max-over-ranks wall time; the line's `dist` records the process group's
observed world size, backend and every rank's own figures.  GGRS_BENCH_BACKEND=gloo rehearses N
ranks on fewer GPUs (ranks share devices).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames-per-step F]
    python bench.py --config 3|4 ...   # speculative branch rollback

Configs 3 and 4 (branch engine): a step is one round -- speculate (every (session, branch) lane
replays the window from its session's confirmed trunk with the branch generator's remote inputs)
then confirm (the trunk replays the confirmed frame; survival bits and checksums form the report)
and, with more than one rank, the RCCL all-gather of the reports.  Resimulated session-frames per
round = lanes x window + sessions.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# the process's CPU set before anything binds a thread: the requests workload binds the handler's
# OpenMP workers (OMP_PROC_BIND), which pins the main thread too, and threads it creates inherit that
# mask -- the CPU baselines restore it for theirs
PROCESS_AFFINITY = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else None


def unbind_main_thread():
    if PROCESS_AFFINITY is not None:
        os.sched_setaffinity(0, PROCESS_AFFINITY)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def bytes_per_synctest_call(P, cd):
    """Algorithmic HBM bytes one lane moves per SyncTest frame (DESIGN.md "Roofline"): load one
    state, cd saves of state + u16 checksum, the first-seen checksum, 2 u16 reads per comparison
    (cd - 1 of them), one input byte per player for each of the cd + 1 advances."""
    S = 4 + 20 * P
    return S + cd * (S + 2) + 2 + 4 * (cd - 1) + (cd + 1) * P


def pmc_traffic(workload):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary, if one exists for this
    workload (profiles/pmc_<workload>.json written by tools/profile_pmc.py), else None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as fh:
            return float(json.load(fh)["hbm_bytes_per_launch"])
    except Exception:
        return None


def pmc_valu(workload):
    """VALU utilisation of the step kernel from the same committed profile summary (rocprofv3
    SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, SQ_INSTS_VALU / SQ_WAVES), or None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
        if d.get("valu_active_frac_of_wave_cycles") is None:
            return None
        return {"issue_frac": None if d.get("valu_issue_frac") is None else round(d["valu_issue_frac"], 4),
                "wave_issue_frac": None if d.get("valu_wave_issue_frac") is None else round(d["valu_wave_issue_frac"], 4),
                "active_frac_of_wave_cycles": round(d["valu_active_frac_of_wave_cycles"], 4),
                "insts_per_wave": round(d["valu_insts_per_wave"], 1),
                "wait_frac_of_wave_cycles": round(d["wait_any_frac"], 4), "profile": d.get("tag")}
    except Exception:
        return None


class FenceFreeEvents:
    """HIP timing events without the system-scope release fence (hipEventDisableSystemFence), from
    the HIP runtime this process already loaded (torch's and libggrs_amd's), recorded on torch's
    current stream.  A default event's fence flushes the caches: three per codec step cost the
    stream ~10 us of a 63 us step and added ~2 us to each kernel's measured duration."""
    DISABLE_SYSTEM_FENCE = 0x20000000

    def __init__(self, torch):
        import ctypes
        self.torch, self.ct = torch, ctypes
        path = None
        with open("/proc/self/maps") as f:
            for ln in f:
                if "libamdhip64.so" in ln:
                    path = ln.split()[-1]
                    break
        if path is None:
            raise RuntimeError("the HIP runtime is not loaded")
        self.hip = ctypes.CDLL(path)

    def record(self):
        ct = self.ct
        e = ct.c_void_p()
        if self.hip.hipEventCreateWithFlags(ct.byref(e), ct.c_uint(self.DISABLE_SYSTEM_FENCE)) != 0:
            raise RuntimeError("hipEventCreateWithFlags failed")
        if self.hip.hipEventRecord(e, ct.c_void_p(self.torch.cuda.current_stream().cuda_stream)) != 0:
            raise RuntimeError("hipEventRecord failed")
        return e

    def elapsed_ms(self, a, b):
        ms = self.ct.c_float()
        if self.hip.hipEventElapsedTime(self.ct.byref(ms), a, b) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return ms.value

    def destroy(self, *evs):
        for e in evs:
            self.hip.hipEventDestroy(e)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_launch_cmd(argv, n, port, python=None):
    """The child command `bench.py --gpus N` runs when it is not itself a rank: one
    torch.distributed.run that starts N ranks of this script on this node (the driver's own
    multi-GPU invocation), rendezvous on 127.0.0.1."""
    return [python or sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def launch_ranks(argv, n, env=None, python=None):
    """Run N ranks of this bench as ONE child process tree and forward rank 0's JSON line.

    The parent never imports torch or touches the GPU (a process that has initialised the GPU must
    not exec another program); it starts `torch.distributed.run` as a child, lets the ranks'
    stderr through, sends any non-JSON stdout to stderr, prints the last JSON line with the
    launch recorded in it, and returns the child's exit status (non-zero when any rank failed or
    no line was printed)."""
    import subprocess
    env = dict(os.environ if env is None else env)
    env.pop("WORLD_SIZE", None)
    cmd = rank_launch_cmd(argv, n, free_port(), python)
    print("launching: " + " ".join(cmd), file=sys.stderr)
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, env=env, text=True)
    line = None
    for ln in proc.stdout.splitlines():
        try:
            obj = json.loads(ln)
        except ValueError:
            obj = None
        if isinstance(obj, dict) and "metric" in obj:
            line = obj
        elif ln.strip():
            print(ln, file=sys.stderr)
    if proc.returncode != 0:
        print(f"bench: a rank failed (torch.distributed.run exit {proc.returncode})", file=sys.stderr)
        return proc.returncode
    if line is None:
        print("bench: rank 0 printed no JSON line", file=sys.stderr)
        return 1
    line["launch"] = {"launcher": "bench.py -> torch.distributed.run", "ranks_spawned": n}
    print(json.dumps(line))
    sys.stdout.flush()
    return 0


def rank_timings(dist, torch, elapsed, units):
    """Max-over-ranks wall time plus every rank's own figures: (max elapsed, total units, rows).
    One all-gather of (elapsed, units) per rank; gloo groups gather on the host."""
    if dist is None:
        return elapsed, units, [{"rank": 0, "elapsed_s": round(elapsed, 6), "value": round(units / elapsed, 1)}]
    dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
    t = torch.tensor([elapsed, float(units)], dtype=torch.float64, device=dev)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    rows = [o.tolist() for o in out]
    per = [{"rank": r, "elapsed_s": round(e, 6), "value": round(u / e, 1)} for r, (e, u) in enumerate(rows)]
    return max(e for e, _ in rows), sum(u for _, u in rows), per


def dist_info(dist, per_rank):
    """What the line records about the process group it was measured in."""
    if dist is None:
        return {"world_size": 1, "backend": None, "per_rank": per_rank}
    return {"world_size": dist.get_world_size(), "backend": dist.get_backend(), "per_rank": per_rank}


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and rank == 0:
        print(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using {world} rank(s)", file=sys.stderr)
    import torch  # before the engine: torch's bundled HIP runtime must serve the process
    dist = None
    # GGRS_BENCH_DIST=1 forms the process group at one rank too (the multi-rank code path measured
    # on one GPU: a one-rank RCCL all-gather per round)
    if world > 1 or os.environ.get("GGRS_BENCH_DIST") == "1":
        import torch.distributed as dist
        gloo = os.environ.get("GGRS_BENCH_BACKEND") == "gloo"
        if gloo:
            # rehearsal of N ranks on fewer GPUs: ranks share devices, collectives over gloo
            local_rank = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local_rank)
        # RCCL (and gloo) print connection banners to stdout while the group forms; the driver
        # reads rank 0's stdout as the ONE JSON line, so they go to stderr
        import ctypes
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            if gloo:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
            dist.barrier()
            ctypes.CDLL(None).fflush(None)
        finally:
            os.dup2(saved, 1)
            os.close(saved)
    return world, rank, local_rank, torch, dist


BRANCH_CONFIGS = {
    # sessions per GPU, branches, players, remote mask, window
    3: dict(sessions=1, branches=16 ** 4, players=2, remote_mask=0b10, window=4,
            text="config3: 1 session x 65,536 branches (16^4 remote-input sequences over a 4-frame "
                 "window), 2 players, speculate + confirm per round"),
    4: dict(sessions=8192, branches=16, players=4, remote_mask=0b1110, window=8,
            text="config4: 4-player P2P, 8192 sessions x 16 branches = 131,072 lanes per GPU, "
                 "window 8, RCCL all-gather of checksums + survival bits per confirmation"),
}


class _StubReportEngine:
    """A CPU stand-in for BranchEngine's report interface (launch-selftest only): the exchange leg's
    collective path and record shape checked without a GPU.  Round r's report is a deterministic
    function of (session group, r), so peer replicas agree and the desync count must be 0."""

    def __init__(self, group, S=64, L=1024):
        import numpy as np
        self.np = np
        self.group, self.num_sessions, self.num_lanes = group, S, L
        self.report_bytes = ((2 * S + 7) & ~7) + 8 * ((L + 63) // 64)
        self.r = 0

    def trunk_frame(self):
        return self.r

    def round_to_tensor(self, t):
        import torch
        v = (self.np.arange(self.report_bytes, dtype=self.np.uint32) * 7 + self.r * 13 + self.group) & 0xFF
        t.copy_(torch.from_numpy(v.astype(self.np.uint8)))
        self.r += 1

    def rounds(self, n):
        self.r += n

    def synchronize(self):
        pass


def exchange_leg(torch, dist, make_engine, rounds, batch, gpu):
    """The config-4 report exchange across the ranks of the current process group (SURVEY.md 8e,
    the analogue of the ChecksumReport send/receive, p2p_session.rs:904-975 and
    protocol.rs:692-698): `rounds` rounds with one stream-ordered all-gather of `batch` rounds'
    reports (exchange.ReportExchange, peers on when the world size is even: rank r and r + world/2
    run the same sessions and compare checksums on the device), then the same rounds with no
    exchange, then the all-gather alone on the same buffers.  Max over ranks of each span.
    Returns the line's `exchange` record."""
    from ggrs_amd import exchange
    world, rank = dist.get_world_size(), dist.get_rank()
    peers = world >= 2 and world % 2 == 0
    group = rank % (world // 2) if peers else rank
    eng = make_engine(group)

    def sync():
        eng.synchronize()
        if gpu:
            torch.cuda.synchronize()
        dist.barrier()

    def span(fn):
        sync()
        t0 = time.perf_counter()
        fn()
        sync()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda" if gpu else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    ex = exchange.ReportExchange(eng, peers=peers, batch=batch)
    ex.run(batch)  # warm-up batch (the communicator's first collective included)
    ex.drain()

    def with_exchange():
        ex.run(rounds)
        ex.drain()
    t_ex = span(with_exchange)

    def without():
        for _ in range(rounds // batch):
            eng.rounds(batch)
        if rounds % batch:
            eng.rounds(rounds % batch)
    t_plain = span(without)
    n_ag = max(1, rounds // batch)
    buf, out = ex.bufs[0], ex.gathered[0]

    def gathers():
        for _ in range(n_ag):
            if gpu:
                dist.all_gather_into_tensor(out.view(-1), buf.view(-1))
            else:
                dist.all_gather(list(out.unbind(0)), buf)
    stream = ex.stream if ex.stream is not None else None
    if stream is not None:
        with torch.cuda.stream(stream):
            t_ag = span(gathers)
    else:
        t_ag = span(gathers)
    cnt = ex.desync_count.detach().clone().to("cuda" if gpu else "cpu").reshape(1)
    dist.all_reduce(cnt)
    gathered_bytes = world * batch * eng.report_bytes
    return {
        "what": "config-4 batched ReportExchange after the timed region (not in value): per rank "
                f"{eng.num_sessions} sessions x {eng.num_lanes // eng.num_sessions} branches, one "
                f"all-gather of {batch} rounds' reports (checksums + survival bits)"
                + (", peer ranks r and r + world/2 compare checksums" if peers else ""),
        "world_size": world, "backend": dist.get_backend(), "peers": peers,
        "engine": type(eng).__name__,
        "rounds": rounds, "batch": batch, "allgathers": n_ag,
        "us_per_round_with_allgather": round(t_ex / rounds * 1e6, 3),
        "us_per_round_without_allgather": round(t_plain / rounds * 1e6, 3),
        "report_bytes_per_round_per_rank": eng.report_bytes,
        "gathered_bytes_per_allgather": gathered_bytes,
        "us_per_allgather_alone": round(t_ag / n_ag * 1e6, 3),
        "allgather_bytes_per_s": round(gathered_bytes * n_ag / t_ag, 1),
        "desyncs": int(cnt.item()),
    }


def branch_exchange_engine(torch, local_rank, rounds):
    """The config-4 branch engine of rank group g (the sessions it shards), for exchange_leg."""
    from ggrs_amd import BranchEngine, synth
    c = BRANCH_CONFIGS[4]
    S, B, P, W = c["sessions"], c["branches"], c["players"], c["window"]

    def make(group):
        truth = synth.gen_inputs(group * S, S, rounds + W + 2, P, synth.MODEL_HELD)
        eng = BranchEngine(S, num_players=P, remote_mask=c["remote_mask"], window=W, branches=B, alphabet=16,
                           input_capacity=rounds + W + 4, device=local_rank)
        eng.add_inputs(0, truth)
        return eng
    return make


def run_branch(args):
    world, rank, local_rank, torch, dist = setup_dist(args)
    from ggrs_amd import BranchEngine, exchange, synth
    c = BRANCH_CONFIGS[args.config]
    S, B, P, W = c["sessions"], c["branches"], c["players"], c["window"]
    rps = args.rounds_per_step  # one step = rps rounds (a round lasts microseconds)
    rounds = (args.warmup + args.steps) * rps
    group = rank % (world // 2) if (args.peers and world >= 2) else rank
    truth = synth.gen_inputs(group * S, S, rounds + W + 1, P, synth.MODEL_HELD)
    eng = BranchEngine(S, num_players=P, remote_mask=c["remote_mask"], window=W, branches=B,
                       alphabet=16, input_capacity=rounds + W + 3, device=local_rank)
    eng.add_inputs(0, truth)
    L = eng.num_lanes
    # more than one rank: every round's report is all-gathered, stream-ordered behind the confirm
    # on the device (exchange.ReportExchange: no host synchronisation in the round loop, round r's
    # all-gather overlapping round r+1's speculation); one rank: rounds run fused in one launch
    ex = exchange.ReportExchange(eng, peers=args.peers, batch=args.exchange_batch) if dist is not None else None

    def sync_all():
        eng.synchronize()
        if dist is not None:
            torch.cuda.synchronize()
            dist.barrier()

    for _ in range(args.warmup * rps):
        if ex is not None:
            ex.run(1)
        else:
            eng.speculate()
            eng.confirm()
    if ex is not None:
        ex.drain()
    sync_all()
    eng.timing_reset()
    t0 = time.perf_counter()
    if ex is None:
        for _ in range(args.steps):
            eng.rounds(rps)  # one GPU: no exchange between rounds, one fused launch per step
    else:
        ex.run(args.steps * rps)  # a batch of rounds per launch and per all-gather
        ex.drain()
    eng.timing_stop()  # the end event right behind the last launch, no wait inside the span
    sync_all()
    t1 = time.perf_counter()
    kernel_ms, launches = eng.timing_read()
    elapsed = t1 - t0
    n_desync = int(ex.desync_count.item()) if ex is not None else 0
    resim_round = L * W + S
    general = None
    if args.config == 3 and ex is None:
        # the same rounds without player separability (round form "full": every lane replays every
        # player of its window and saves every logical cell, what a game whose players interact needs;
        # GGRS's Config::State contract gives no separability) -- beside the headline, not in it
        g_eng = BranchEngine(S, num_players=P, remote_mask=c["remote_mask"], window=W, branches=B,
                             alphabet=16, input_capacity=rounds + W + 3, device=local_rank)
        g_eng.add_inputs(0, truth)
        g_eng.set_round_form("full")
        for _ in range(args.warmup):
            g_eng.rounds(rps)
        g_eng.synchronize()
        g_eng.timing_reset()
        tg0 = time.perf_counter()
        for _ in range(args.steps):
            g_eng.rounds(rps)
        g_eng.timing_stop()
        g_eng.synchronize()
        tg = time.perf_counter() - tg0
        g_ms, g_launches = g_eng.timing_read()
        general = {"general_form_frames_per_s": round(resim_round * rps * args.steps / tg, 1),
                   "us_per_round": round(tg / (rps * args.steps) * 1e6, 3),
                   "kernel_us_per_round": round(g_ms * 1e3 / (rps * args.steps), 3),
                   "kernel": "rounds_kernel (fused rounds, every lane all players, every logical save)"}
        g_eng.close()
    elapsed, total, per_rank = rank_timings(dist, torch, elapsed, resim_round * rps * args.steps)
    value = total / elapsed
    Sp = 4 + 20 * P
    bytes_round = L * (Sp + W * (Sp + 2) + W * P) + S * (2 * Sp + 2 + P) + 8 * ((L + 63) // 64)
    avg_round_s = kernel_ms / 1e3 / max(launches, 1) * 2  # speculate + confirm launches per round
    achieved = bytes_round / avg_round_s / 1e9
    parity = None
    if rank == 0:
        try:
            from oracle import oracle as O
            O.build()
            from oracle import every_lane
            # EVERY lane's last speculated window (cells and states), every report checksum and
            # survival bit against the oracle's replay (oracle_p2p_replay_batch)
            r = every_lane.branch(eng, truth)
            parity = {k: v for k, v in r.items() if k != "trunk_states"}
            parity["session0_trunk_bit_exact"] = bytes(eng.trunk(0)) == bytes(r["trunk_states"][0])
            parity["desyncs"] += n_desync
            parity["every_lane_bit_exact"] = (all(v == 0 for k, v in parity.items() if k.endswith("_mismatched"))
                                              and parity["session0_trunk_bit_exact"])
        except Exception as exc:
            parity = {"error": repr(exc)}
        cpu_baseline = None
        if world == 1 and not args.no_cpu_baseline:
            cpu_baseline = branch_cpu_baseline(args, c)
        # distinct speculated states per round: branches sharing their first k digits share the
        # state after k + 1 frames (config 3: 16 + 256 + 4096 + 65536 of the 4 x 65536 logical)
        A = 16
        E = 0
        while A ** E < B:
            E += 1
        distinct = S * sum(min(A ** min(k + 1, E), B) for k in range(W)) + S
        # the prefix-shared kernel saves only the distinct cells: its algorithmic bytes are those
        # saves, the trunk replay and the survival bits (the logical figure stays beside it)
        prefix_kernel = bin(c["remote_mask"]).count("1") == 1 and B > 1  # the engine's dispatch rule
        bytes_prefix = (distinct - S) * (Sp + 2) + S * (2 * Sp + 2 + P) + 8 * ((L + 63) // 64)
        bytes_kernel = bytes_prefix if prefix_kernel else bytes_round
        achieved = bytes_kernel / avg_round_s / 1e9
        line = {
            "metric": "resimulated session-frames/sec (node)", "value": round(value, 1),
            "unit": "session-frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": c["text"], "sessions_per_gpu": S, "branches": B, "lanes_per_gpu": L,
                       "players": P, "window": W, "peers": bool(args.peers),
                       "logical_frames_per_round": resim_round, "prefix_distinct_frames_per_round": distinct,
                       "prefix_distinct_frames_per_s": round(distinct * rps * args.steps * world / elapsed, 1),
                       "rounds_per_step": rps,
                       "parallelism": f"sessions sharded over {world} GPU(s)" + (
                           (", one stream-ordered RCCL all-gather of the reports per round" if args.exchange_batch == 1
                            else f", {args.exchange_batch} rounds per launch and per stream-ordered RCCL all-gather"
                                 " of their reports")
                           if dist is not None else ""),
                       "exchange_batch": args.exchange_batch if dist is not None else None},
            "dist": dist_info(dist, per_rank),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": pmc_traffic(f"config{args.config}"),
                         "algorithmic_bytes_per_round": bytes_kernel,
                         "algorithmic_bytes_per_round_logical": bytes_round,
                         "bytes_basis": "prefix-distinct saves" if prefix_kernel else "every logical save",
                         "avg_kernel_ms_per_round": round(avg_round_s * 1e3, 4)},
            "cpu_baseline": cpu_baseline, "parity": parity,
        }
        if general is not None:
            line["general_form"] = general
            line["config"]["general_form_frames_per_s"] = general["general_form_frames_per_s"]
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def run_particles(args):
    """Config 5: SyncTest (check_distance 16, max_prediction 17) on 1 MB particle-world states;
    one step = one SyncTest frame on every session (1 load + 16 resimulated advances with 16 saves
    + the new advance), so every Load/Save streams through HBM."""
    world, rank, local_rank, torch, dist = setup_dist(args)
    from ggrs_amd import ParticleEngine, synth
    S = args.sessions or 8192
    N, P, maxp, cd = 10000, 2, 17, 16
    warm = max(args.warmup, cd + 2)
    frames = warm + args.steps
    inputs = synth.gen_inputs(rank * S, S, frames, P, synth.MODEL_HELD)
    eng = ParticleEngine(S, N, P, maxp, cd, input_capacity=frames + cd + 2, device=local_rank,
                         first_session_id=rank * S)
    eng.add_local_inputs(inputs)
    for _ in range(warm):
        eng.synctest_advance_frames(1)
    eng.synchronize()
    if dist is not None:
        dist.barrier()
    eng.timing_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.synctest_advance_frames(1)
    eng.timing_stop()  # the end event right behind the last launch, no wait inside the span
    eng.synchronize()
    if dist is not None:
        dist.barrier()
    t1 = time.perf_counter()
    kernel_ms, launches = eng.timing_read()
    elapsed = t1 - t0
    elapsed, total, per_rank = rank_timings(dist, torch, elapsed, S * cd * args.steps)
    st, _, _ = eng.mismatches()
    value = total / elapsed
    Sb = 4 + 100 * N
    bytes_launch = S * (Sb + cd * (Sb + 2) + 2 + 4 * (cd - 1) + (cd + 1) * P)
    avg_s = kernel_ms / 1e3 / max(launches, 1)
    achieved = bytes_launch / avg_s / 1e9
    parity = None
    if rank == 0:
        try:
            from oracle import oracle as O
            O.build()
            r = O.particles_synctest_run(inputs[:, 0, :], N, P, maxp, cd, session=0, ring_states=False)
            parity = {"session0_final_state_bit_exact": bytes(eng.state(0)) == bytes(r["final_state"]),
                      "session0_ring_checksums": all(
                          eng.saved(0, int(fr), with_state=False)[0] == int(ck)
                          for fr, ck in zip(r["ring_frames"], r["ring_cksums"]) if fr >= 0)}
        except Exception as exc:
            parity = {"error": repr(exc)}
        cpu_baseline = None
        if world == 1 and not args.no_cpu_baseline:
            cpu_baseline = particles_cpu_baseline(args, synth, N, P, maxp, cd)
        line = {
            "metric": "resimulated session-frames/sec (node)", "value": round(value, 1),
            "unit": "session-frames/s", "n_gpus": world, "steps": args.steps, "warmup": warm,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "config5: particle world, 10k entities x 100 B (~1 MB) per session, "
                                   "SyncTest check_distance 16 / max_prediction 17 (ring 17 x 1 MB)",
                       "sessions_per_gpu": S, "entities": N, "players": P, "check_distance": cd,
                       "hbm_ring_gb_per_gpu": round(S * Sb * (maxp + 1) / 1e9, 2),
                       "parallelism": f"sessions sharded over {world} GPU(s)"},
            "dist": dist_info(dist, per_rank),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": pmc_traffic(f"config5_s{S}"),
                         "algorithmic_bytes_per_launch": bytes_launch,
                         "avg_launch_ms": round(avg_s * 1e3, 4)},
            "cpu_baseline": cpu_baseline, "halted_lanes": int((st != 0).sum()), "parity": parity,
        }
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def run_p2p(args):
    """P2P rollback decision on the device (ggrs_p2p_*): S sessions of one peer, 2 players (one
    remote, inputs arrive --latency frames late, default 4), --max-prediction (default 8),
    repeat-last prediction, held-key inputs.  One step = 64 advance_frame calls on every session:
    poll, misprediction check, rollback + resimulation where the session's prediction failed, save,
    advance.  BASELINE config 2's P2P form: --sessions 4096 --latency 8 --max-prediction 9."""
    world, rank, local_rank, torch, dist = setup_dist(args)
    from ggrs_amd import P2PEngine, synth
    S = args.sessions or 65536
    P, D, maxp, calls = 2, args.latency, args.max_prediction, args.p2p_calls
    sched = args.arrivals != "fixed"
    if sched and (maxp < 2 or args.peers or args.p2p_form != "default"):
        raise SystemExit("--arrivals jitter/stall: rollback mode (--max-prediction >= 2), no --peers, default form")
    if not sched and not (1 <= D <= maxp - 1 or (maxp == 0 and D >= 1)):
        raise SystemExit(f"--latency {D} must be in 1..--max-prediction - 1 = {maxp - 1} (1.. in lockstep mode): "
                         "the engine's contract (include/ggrs_amd.h, ggrs_p2p_config_t.remote_latency), else the "
                         "prediction threshold stalls the session (p2p_session.rs:393-423)")
    frames = (args.warmup + args.steps) * calls
    # --peers: rank r and rank r + world/2 are the two machines of the same matches (local player
    # 0 on one, 1 on the other, the same inputs); their checksum reports (desync detection,
    # interval 32) cross the process group once per step (exchange.exchange_p2p_reports)
    peers = bool(args.peers) and dist is not None and world >= 2 and world % 2 == 0
    pair = rank % (world // 2) if peers else rank
    local = (1,) if peers and rank >= world // 2 else (0,)
    rows = synth.gen_inputs(pair * S, S, frames, P, synth.MODEL_HELD)
    eng = P2PEngine(S, num_players=P, local_players=local, input_delay=0, max_prediction=maxp,
                    remote_latency=1 if sched else D, input_capacity=frames + D + 2, device=local_rank)
    eng.set_kernel_form(args.p2p_form)
    if args.sparse:
        eng.set_sparse_saving(True)  # builder.rs:160-169
    arrive = None
    if sched:  # every session its own network (p2p_sched.hip): jittered lags, optionally stalls
        arrive = synth.jitter_arrivals(pair * S, S, frames, maxp, stalls=args.arrivals == "stall")
        eng.set_arrival_schedule(True)
        eng.add_arrivals(0, arrive)
    det, events = None, []
    if peers:
        from ggrs_amd import exchange
        from ggrs_amd.desync import DesyncDetector
        det = DesyncDetector(eng, 32, addr=exchange.peer_of(rank, world))
    eng.add_inputs(0, rows)
    eng.synchronize()

    def step():
        eng.advance_frames(calls)
        if det is not None:
            exchange.exchange_p2p_reports(det)
            events.extend(det.poll())

    for _ in range(args.warmup):
        step()
    eng.synchronize()
    rb0, rs0 = eng.stats()
    if dist is not None:
        dist.barrier()
    eng.timing_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.timing_stop()  # the end event right behind the last launch, no wait inside the span
    eng.synchronize()
    if dist is not None:
        dist.barrier()
    t1 = time.perf_counter()
    kernel_ms, launches = eng.timing_read()
    elapsed = t1 - t0
    n_desync = len(events)
    session_calls = S * calls * args.steps
    elapsed, total, per_rank = rank_timings(dist, torch, elapsed, session_calls)
    if dist is not None:
        c = torch.tensor([n_desync], dtype=torch.int64, device="cpu" if dist.get_backend() == "gloo" else "cuda")
        dist.all_reduce(c)
        n_desync = int(c.item())
    rb1, rs1 = eng.stats()
    resim = int((rs1 - rs0).sum())
    rollbacks = int((rb1 - rb0).sum())
    value = total / elapsed
    F = 5 * P + 1
    skipped = errors = None
    if sched:
        fr1, sk1, er1 = eng.sessions()
        skipped, errors = int(sk1.sum()), int((er1 != 0).sum())
    # HBM bytes per launch: the state in/out, every save (state + checksum), every rollback load,
    # the queue words in/out and the input rows each call reads (arrival + its own, + replays)
    # (sparse saving: about one save per call, at min_confirmed, and replays save nothing)
    # every replayed frame but the first is saved (p2p_session.rs:690-711)
    replay_saves = 0 if args.sparse else (resim - rollbacks) // args.steps * (4 * F + 2)
    bytes_launch = (2 * 4 * F * S + (session_calls // args.steps) * (4 * F + 2) * 1
                    + (rollbacks // args.steps) * 4 * F + replay_saves
                    + 2 * 16 * P * S + (session_calls // args.steps) * 2 * 2 + (resim // args.steps) * 2 * 2)
    if sched:  # + per call its arrival word, the queue word of the frame that arrives and of the
        # local input (read-modify-write), each save's frame tag; the session words in and out
        per_call = session_calls // args.steps
        bytes_launch += per_call * (4 + 2 * 8) + (per_call + (resim - rollbacks) // args.steps) * 4 + 2 * 4 * (9 + 5 * P) * S
    avg_s = kernel_ms / 1e3 / max(launches, 1)
    achieved = bytes_launch / avg_s / 1e9
    parity = cpu_baseline = None
    if rank == 0:
        try:
            from oracle import oracle as O
            O.build()
            from oracle import every_lane
            # EVERY session against the oracle's P2PSession (oracle_p2p_batch): final state, rollbacks,
            # and under a schedule the current frame and skipped calls
            parity = every_lane.p2p(eng, rows, arrive, P=P, local_mask=eng.local_mask, maxp=maxp, latency=D,
                                    sparse=bool(args.sparse))
            parity["every_session_bit_exact"] = all(v == 0 for k, v in parity.items() if k.endswith("_mismatched"))
            if peers:
                parity["peers_desync_events"] = n_desync
            if world == 1 and not args.no_cpu_baseline:
                cpu_baseline = (p2p_sched_cpu_baseline(args, O, synth, P, maxp) if sched
                                else p2p_cpu_baseline(args, O, synth, P, D, maxp))
        except Exception as exc:
            parity = {"error": repr(exc)}
        line = {
            "metric": "P2P session-frames/sec (node)", "value": round(value, 1),
            "unit": "session-frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"p2p: {S} sessions per GPU, 2 players (1 remote, " + (
                                       f"inputs {D} frames late" if not sched else
                                       "per-session jittered arrivals, lag 1..max_prediction-1"
                                       + (", network stalls of max_prediction + 4 calls every 48" if args.arrivals == "stall" else ""))
                                   + f"), max_prediction {maxp}, held-key inputs, {calls} calls per step",
                       "arrivals": args.arrivals,
                       "sessions_per_gpu": S, "peers": peers, "sparse_saving": bool(args.sparse),
                       "parallelism": f"sessions sharded over {world} GPU(s)"
                                      + (f", peer ranks exchange checksum reports over {dist.get_backend()}" if peers else "")},
            "dist": dist_info(dist, per_rank),
            "rollbacks_per_session_frame": round(rollbacks / session_calls, 5),
            # the replayed AdvanceFrames the sessions actually executed (p2p_session.rs:690-711)
            "resimulated_session_frames_per_s": round(resim * world / elapsed, 1),
            "resimulated_per_session_frame": round(resim / session_calls, 5),
            "advances_per_sec": round((session_calls + resim) * world / elapsed, 1),
            "skipped_calls": skipped, "sessions_in_error": errors,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": pmc_traffic(f"p2p_s{S}" + (f"_{args.arrivals}_m{maxp}" if sched else
                                                               ("" if (D, maxp) == (4, 8) else f"_d{D}_m{maxp}"))
                                               + ("_sparse" if args.sparse else "")),
                         "algorithmic_bytes_per_launch": bytes_launch,
                         "avg_launch_ms": round(avg_s * 1e3, 4)},
            "cpu_baseline": cpu_baseline, "parity": parity,
        }
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def run_codec(args):
    """Input wire codec, batched (ggrs_codec_*; src/network/compression.rs): one step = encode and
    decode N packets, each a reference input plus W pending inputs of B bytes (config 4 flavour:
    per GPU 1,048,576 endpoint packets of the 8-frame prediction window, 2 local players x 1 byte,
    held-key inputs).  Metric: packets round-tripped per second."""
    world, rank, local_rank, torch, dist = setup_dist(args)
    import numpy as np
    from ggrs_amd import codec
    N, W, B = args.sessions or 1 << 20, 8, 2
    rng = np.random.default_rng(1234 + rank)
    ref = rng.integers(0, 16, (N, B), dtype=np.uint8)
    held = np.repeat(ref[:, None, :], W, axis=1)
    flip = rng.random((N, W, B)) < 1.0 / 8.0  # a new key 1 frame in 8 (SURVEY.md 8d input model)
    pend = np.where(flip, rng.integers(0, 16, (N, W, B), dtype=np.uint8), held).astype(np.uint8)
    count = np.full(N, W, np.int32)
    dev = torch.device("cuda", local_rank)
    d_ref, d_pend, d_cnt = (torch.from_numpy(x).to(dev) for x in (ref, pend, count))
    stride = codec.max_packet_bytes(B, W)
    chunked = args.codec_layout == "chunked"  # each 256-packet block's packets back to back
    dec_buf = torch.empty((N, W, B), dtype=torch.uint8, device=dev)  # decoded inputs, reused per step
    hev = FenceFreeEvents(torch)
    evs = []

    def step(timed):
        e = [hev.record()] if timed else None
        out, ln = codec.encode(d_ref, d_pend, d_cnt, stride, chunked=chunked)
        if timed:
            e.append(hev.record())
        dec, cnt, st = codec.decode(d_ref, out, ln, W, chunked=chunked, out=dec_buf)
        if timed:
            e.append(hev.record())
            evs.append(e)
        return out, ln, dec, cnt, st

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    # the kernels' durations: fence-free HIP events around encode and decode of every 4th timed step
    # (even without the fence an event costs the stream ~1.7 us, 8 % of a step carrying three)
    for i in range(args.steps):
        res = step(i % 4 == 0)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed, total, per_rank = rank_timings(dist, torch, elapsed, N * args.steps)
    enc_ms = sum(hev.elapsed_ms(e[0], e[1]) for e in evs) / len(evs)
    dec_ms = sum(hev.elapsed_ms(e[1], e[2]) for e in evs) / len(evs)
    for e in evs:
        hev.destroy(*e)
    out, ln, dec, cnt, st = res
    ln_h = ln.cpu().numpy()
    pkt_bytes = int(ln_h.sum())
    ok = bool((st == 0).all().item()) and bool((cnt == d_cnt).all().item()) and bool((dec == d_pend).all().item())
    value = total / elapsed
    # algorithmic HBM bytes: encode reads ref + pending + count, writes packets + lengths; decode
    # reads ref + packets + lengths, writes inputs + count + status
    enc_bytes = N * (B + W * B + 4) + pkt_bytes + 4 * N
    dec_bytes = N * (B + 4) + pkt_bytes + N * (W * B + 8)
    dom = "decode" if dec_ms >= enc_ms else "encode"
    dom_bytes, dom_ms = (dec_bytes, dec_ms) if dom == "decode" else (enc_bytes, enc_ms)
    achieved = dom_bytes / (dom_ms / 1e3) / 1e9
    parity = cpu_baseline = None
    if rank == 0:
        try:
            from oracle import oracle as O
            O.build()
            flat = out.cpu().numpy().reshape(-1)
            off = codec.chunk_offsets(ln_h, stride) if chunked else np.arange(N, dtype=np.int64) * stride
            same = all(flat[off[p]:off[p] + ln_h[p]].tobytes() ==
                       O.codec_encode(ref[p].tobytes(), [pend[p, k].tobytes() for k in range(W)])
                       for p in (0, 1, N // 2, N - 1))
            parity = {"round_trip_all_packets": ok, "packets_0_1_mid_last_bytes_equal_oracle": bool(same)}
            if world == 1 and not args.no_cpu_baseline:
                sample = min(N, 1 << 18)
                T = cpu_threads(args)
                n1, w1 = O.codec_bench(ref[:sample], pend[:sample], count[:sample], 1)
                passes = max(1, int(10.0 * T / max(w1, 1e-3)))  # about 10 s on T threads
                n, wall = O.codec_bench(ref[:sample], pend[:sample], count[:sample], passes, threads=T)
                cpu_baseline = {"value": round(n / wall, 1), "unit": "packets/s", "cores": T, "kind": "port",
                                "sample": f"{passes} passes x {sample} packets (W {W}, B {B}) on {T} threads, each "
                                          f"its slice, encode + decode one packet at a time (oracle/codec.c)",
                                "wall_s": round(wall, 3), "cpu": cpu_model(),
                                "single_thread": {"value": round(n1 / w1, 1), "cores": 1, "wall_s": round(w1, 3)}}
        except Exception as exc:
            parity = {"error": repr(exc)}
        line = {
            "metric": "input packets encoded+decoded/sec (node)", "value": round(value, 1), "unit": "packets/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"codec: {N} endpoint packets per GPU, {W} pending inputs x {B} bytes, "
                                   f"held-key inputs; encode + decode per step",
                       "packets_per_gpu": N, "pending": W, "input_bytes": B, "layout": args.codec_layout,
                       "mean_packet_bytes": round(pkt_bytes / N, 2),
                       "parallelism": f"packets sharded over {world} GPU(s)"},
            "dist": dist_info(dist, per_rank),
            "kernel_ms": {"encode": round(enc_ms, 4), "decode": round(dec_ms, 4), "event_steps": len(evs)},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": pmc_traffic(f"codec_{dom}_n{N}" + ("" if chunked else "_strided")),
                         "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_ms": round(dom_ms, 4)},
            "cpu_baseline": cpu_baseline, "parity": parity,
        }
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def cpu_threads(args):
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return args.cpu_threads or min(16, avail)


def branch_cpu_baseline(args, c):
    """Configs 3/4 on the host: every branch a rollback replay through the SyncLayer + ex_game
    handler restatement (oracle_branch_bench, ggrs_oracle.c), T threads with their own sessions."""
    from oracle import oracle as O
    O.build()
    T = cpu_threads(args)
    if c["sessions"] == 1:  # config 3: one 65,536-branch session per thread
        sessions, rounds = 1, 12
    else:                   # config 4: 16-branch sessions
        sessions, rounds = 512, 48
    n, wall, _ = O.branch_bench(c["players"], c["window"], 16, c["branches"], c["remote_mask"], sessions, rounds, T)
    return {"value": round(n / wall, 1), "unit": "session-frames/s", "cores": T, "kind": "port",
            "sample": f"{T} threads x {sessions} session(s) x {rounds} rounds of {c['branches']} branch rollbacks "
                      f"(W={c['window']}, P={c['players']}) + trunk confirm, SyncLayer + ex_game handler "
                      "restatement (oracle/ggrs_oracle.c oracle_branch_bench)",
            "wall_s": round(wall, 3)}


def particles_cpu_baseline(args, synth, N, P, maxp, cd):
    """Config 5 on the host: the particle-world SyncTest restatement (oracle_particles_synctest_run,
    1 MB states cloned per save, checksummed per save and advance), one session per thread."""
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np
    from oracle import oracle as O
    O.build()
    T = cpu_threads(args)
    frames = 3 * cd
    rows = synth.gen_inputs(0, T, frames, P, synth.MODEL_HELD)
    per = [np.ascontiguousarray(rows[:, t]) for t in range(T)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(T) as ex:
        res = list(ex.map(lambda a: O.particles_synctest_run(a, N, P, maxp, cd, ring_states=False), per))
    wall = time.perf_counter() - t0
    resim = T * (frames - cd - 1) * cd  # calls f > cd each replay cd frames (sync_test_session.rs:192-217)
    return {"value": round(resim / wall, 2), "unit": "session-frames/s", "cores": T, "kind": "port",
            "sample": f"{T} threads x {frames} SyncTest frames of one {N}-entity session each (cd {cd}, "
                      "the first cd + 1 frames without rollback), C restatement oracle_particles_synctest_run",
            "wall_s": round(wall, 3), "all_ok": all(r["rc"] == 0 for r in res)}


def requests_cpu_baseline(args, synth, P, maxp, cd):
    """The request boundary on the host: ex_game's handler restatement (oracle_handler_run: Save =
    clone + bincode + fletcher16, Load = clone, Advance = State::advance + checksum) over one
    session's SyncTest request lists per thread -- what the Rust handler does per session without
    this engine."""
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np
    from oracle import oracle as O
    O.build()
    unbind_main_thread()
    T = cpu_threads(args)
    frames = 300_000
    inputs = np.stack([O.gen_inputs(synth.SEED_BASE + t, frames, P, O.MODEL_HELD) for t in range(T)], 1)
    # the request stream of SyncTestSession::advance_frame (sync_test_session.rs:85-150), delay 0
    # one input row per request (read by the Advances only); calls f <= cd: [Save f, Advance f],
    # calls f > cd: [Load f-cd, Advance, (Save, Advance) x (cd-1), Save f, Advance]: request 2i is
    # the Load / Save of frame g = f-cd+i, request 2i+1 the Advance of frame g
    head = np.repeat(np.arange(cd + 1), 2)
    g = np.arange(cd + 1, frames)[:, None] - cd + np.arange(cd + 1)[None, :]
    even = np.zeros(cd + 1, np.int32)
    even[0] = 1
    kinds = np.concatenate([np.tile([0, 2], cd + 1),
                            np.stack([np.broadcast_to(even, g.shape), np.full(g.shape, 2)], -1).ravel()]).astype(np.int32)
    fr = np.concatenate([np.stack([np.arange(cd + 1), np.zeros(cd + 1, int)], -1).ravel(),
                         np.stack([g, np.zeros_like(g)], -1).ravel()]).astype(np.int32)
    idx = np.concatenate([head, np.repeat(g.ravel(), 2)]).astype(np.int64)
    streams = [np.ascontiguousarray(inputs[idx, t]) for t in range(T)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(T) as ex:
        res = list(ex.map(lambda a: O.handler_run(kinds, fr, a, None, P, maxp)["rc"], streams))
    wall = time.perf_counter() - t0
    resim = T * (frames - cd - 1) * cd
    return {"value": round(resim / wall, 1), "unit": "session-frames/s", "cores": T, "kind": "port",
            "sample": f"{T} threads x one session's {frames} SyncTest request lists (cd {cd}) through the "
                      "ex_game handler restatement (oracle_handler_run)",
            "wall_s": round(wall, 3), "all_ok": all(r == 0 for r in res)}


def requests_p2p_cpu_baseline(args, fx):
    """The request boundary with P2P lists on the host: ex_game's handler restatement
    (oracle_handler_run: Save = clone + bincode + fletcher16, Load = clone, Advance = State::advance)
    over the same committed fixture's lists, one session's whole stream per task on T threads --
    what the Rust handler does per session without this engine.  Units: advance_frame calls."""
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np
    from ggrs_amd._lib import REQ_ADVANCE
    from oracle import oracle as O
    O.build()
    unbind_main_thread()
    T = cpu_threads(args)
    M, C, P, maxp = fx["M"], fx["C"], fx["P"], fx["maxp"]
    streams = []
    for m in range(M):
        a, b = int(fx["req_off"][m, 0]), int(fx["req_off"][m, C])
        kind = np.ascontiguousarray(fx["kind"][a:b].astype(np.int32))
        inp = np.zeros((b - a, P), np.uint8)
        st = np.zeros((b - a, P), np.uint8)
        adv = np.nonzero(kind == REQ_ADVANCE)[0]
        a0 = int(fx["adv_off"][m, 0])
        inp[adv] = fx["inputs"][a0:a0 + len(adv)]
        st[adv] = fx["status"][a0:a0 + len(adv)]
        streams.append((kind, np.ascontiguousarray(fx["frame"][a:b]), inp, st))
    ok, one = O.handler_bench(streams, P, maxp, M, 1)  # every stream once, one thread: the size of a task
    tasks = max(T, int(10.0 * T * M / max(one, 1e-6)))  # about 10 s of wall time on T threads
    ok, wall = O.handler_bench(streams, P, maxp, tasks, T)
    res = [0 if ok == tasks else -1]  # (every stream ran without a rejected request)
    return {"value": round(tasks * C / wall, 1), "unit": "session-frames/s", "cores": T, "kind": "port",
            "sample": f"{T} threads x {tasks} session streams of {C} advance_frame calls each (the committed P2P "
                      f"fixture's {M} sessions' request lists) through the ex_game handler restatement "
                      "(oracle_handler_run)",
            "wall_s": round(wall, 3), "cpu": cpu_model(), "all_ok": all(r == 0 for r in res)}


def read_host_profile(drv, T, n_calls, lanes_per_group, G):
    """handler_profile_read after a profiled run: per call and per thread (mean over threads), the
    time spinning / handing back / encoding, and per lane the counters of each pass."""
    import ctypes

    import numpy as np
    nc = 5
    w = 5 + 2 * nc
    buf = np.zeros((max(T, 1), w), np.float64)
    drv.handler_profile_read.restype = ctypes.c_int32
    drv.handler_profile_read.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    n = drv.handler_profile_read(ctypes.c_void_p(buf.ctypes.data), buf.shape[0])
    buf = buf[:n]
    names = ["cycles", "instructions", "cache_references", "cache_misses", "l1d_read_misses"]
    lanes_call = lanes_per_group * G  # every lane encoded once per call, its share on each thread
    out = {"threads": int(n), "calls": int(n_calls),
           "us_per_call_per_thread": {"spin": round(float(buf[:, 0].mean()) / n_calls * 1e6, 3),
                                      "handback": round(float(buf[:, 1].mean()) / n_calls * 1e6, 3),
                                      "encode": round(float(buf[:, 2].mean()) / n_calls * 1e6, 3)},
           "ns_per_lane": {"handback": round(float(buf[:, 1].sum()) / (n_calls * lanes_call) * 1e9, 2),
                           "encode": round(float(buf[:, 2].sum()) / (n_calls * lanes_call) * 1e9, 2)},
           "counters_open": int(buf[:, 4 + 2 * nc].min()) if n else 0}
    k = out["counters_open"]
    if k:
        for j, part in ((5, "handback"), (5 + nc, "encode")):
            tot = buf[:, j - 2:j - 2 + nc].sum(axis=0)
            out[f"{part}_per_lane"] = {names[i]: round(float(tot[i]) / (n_calls * lanes_call), 3) for i in range(k)}
            if k >= 2 and tot[0] > 0:
                out[f"{part}_per_lane"]["ipc"] = round(float(tot[1] / tot[0]), 3)
    return out


def p2p_cpu_baseline(args, O, synth, P, D, maxp):
    """The oracle's P2P session (C restatement of p2p_session.rs:265-426 + ex_game) on T host
    threads, one session per thread (ctypes drops the GIL for the call)."""
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np
    T = cpu_threads(args)
    frames = 2_000_000
    per = [O.gen_inputs(synth.SEED_BASE + t, frames, P, O.MODEL_HELD) for t in range(T)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(T) as ex:
        res = list(ex.map(lambda a: O.p2p_run(a, num_players=P, local_mask=0b01, max_prediction=maxp,
                                              latency=D, sparse_saving=bool(args.sparse))["rc"], per))
    wall = time.perf_counter() - t0
    return {"value": round(T * frames / wall, 1), "unit": "session-frames/s", "cores": T, "kind": "port",
            "sample": f"{T} threads x {frames} P2P advance_frame calls (1 session/thread, same game, "
                      f"latency {D}, held-key inputs{', sparse saving' if args.sparse else ''}), C restatement "
                      f"oracle/ggrs_oracle.c oracle_p2p_run",
            "wall_s": round(wall, 3), "all_ok": all(r == 0 for r in res)}


def p2p_sched_cpu_baseline(args, O, synth, P, maxp):
    """The oracle's P2P session under the same arrival-schedule model (oracle_p2p_sched_run: the
    InputQueue / SyncLayer / P2PSession restatement stepped call by call) on T host threads, one
    session per thread."""
    from concurrent.futures import ThreadPoolExecutor
    T = cpu_threads(args)
    calls = 1_000_000
    per = [(O.gen_inputs(synth.SEED_BASE + t, calls, P, O.MODEL_HELD),
            synth.jitter_arrivals(t, 1, calls, maxp, stalls=args.arrivals == "stall")[:, 0].copy()) for t in range(T)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(T) as ex:
        res = list(ex.map(lambda a: O.p2p_sched_run(a[0], a[1], num_players=P, local_mask=0b01, max_prediction=maxp,
                                                    sparse_saving=bool(args.sparse))["rc"], per))
    wall = time.perf_counter() - t0
    return {"value": round(T * calls / wall, 1), "unit": "session-frames/s", "cores": T, "kind": "port",
            "sample": f"{T} threads x {calls} P2P advance_frame calls (1 session/thread, {args.arrivals} arrivals, "
                      f"max_prediction {maxp}, held-key inputs{', sparse saving' if args.sparse else ''}), "
                      "C restatement oracle/ggrs_oracle.c oracle_p2p_sched_run",
            "wall_s": round(wall, 3), "all_ok": all(r == 0 for r in res)}


def synctest_tokens(f, cd):
    """The request kinds of SyncTestSession::advance_frame at frame f (sync_test_session.rs:85-150)
    as lane-batch tokens: [Load f-cd, Advance, (Save, Advance) x (cd-1)] when f > cd, then Save f,
    Advance.  Returns (token words, n_tokens, loads, advances, saves)."""
    from ggrs_amd._lib import TOK_ADVANCE, TOK_END, TOK_LOAD, TOK_SAVE, TOKENS_PER_WORD
    toks = []
    if f > cd:
        toks += [TOK_LOAD, TOK_ADVANCE] + [TOK_SAVE, TOK_ADVANCE] * (cd - 1)
    toks += [TOK_SAVE, TOK_ADVANCE]
    n = len(toks)
    W = -(-n // TOKENS_PER_WORD)
    toks += [TOK_END] * (W * TOKENS_PER_WORD - n)
    words = [sum(t << (2 * i) for i, t in enumerate(toks[w * TOKENS_PER_WORD:(w + 1) * TOKENS_PER_WORD]))
             for w in range(W)]
    return words, n, int(f > cd), toks.count(TOK_ADVANCE), toks.count(TOK_SAVE)


def load_p2p_fixture():
    """bench_native/fixtures/p2p_lists.npz (bench_native/make_p2p_fixture.py): M P2P sessions'
    request lists per call, generated once by the oracle's P2PSession stream and committed."""
    import numpy as np
    with np.load(os.path.join(ROOT, "bench_native", "fixtures", "p2p_lists.npz")) as z:
        d = {k: z[k] for k in z.files}
    M, C = int(d["sessions"]), int(d["calls"])
    reqs = np.stack([d["kind"].astype(np.int32), d["frame"]], axis=1)
    # per (session, call): its list length, AdvanceFrames and SaveGameStates, and the batch shape
    n_req = np.diff(d["req_off"], axis=1)
    n_adv = np.diff(d["adv_off"], axis=1)
    is_load = np.concatenate([[0], np.cumsum(d["kind"] == 1)])
    is_save = np.concatenate([[0], np.cumsum(d["kind"] == 0)])
    n_load = np.diff(is_load[d["req_off"]], axis=1)
    n_save = np.diff(is_save[d["req_off"]], axis=1)
    shape = np.array([-(-int(n_req.max()) // 16), int(n_load.max()), int(n_adv.max()), int(n_save.max())], np.int32)
    return dict(M=M, C=C, P=int(d["players"]), maxp=int(d["max_prediction"]), reqs=np.ascontiguousarray(reqs),
                req_off=np.ascontiguousarray(d["req_off"]), adv_off=np.ascontiguousarray(d["adv_off"]),
                inputs=np.ascontiguousarray(d["inputs"]), status=np.ascontiguousarray(d["status"]),
                kind=d["kind"], frame=d["frame"], n_adv=n_adv, shape=shape)


def run_requests(args):
    """The request-level drop-in boundary (what the Rust request handler of INTEGRATION.md calls
    once per advance_frame of every session), every Save's checksum handed back to host memory.
      --req-form native  (default) SyncTest sessions (config 2: cd 8): every lane's list of
                         SyncTestSession::advance_frame (sync_test_session.rs:85-150: Load f-cd,
                         cd x (Save, Advance) with the first Save skipped, Save f, Advance) encoded
                         into the engines' mapped batches by a C request handler
                         (bench_native/handler_driver.c: request kinds, Load frames and input rows,
                         ggrs_lane_batch_submit / _wait, every Save's checksum read back), the batches
                         served by the persistent lane servers
      --req-form p2p     every lane its own P2PSession's lists (rollbacks of differing depth,
                         p2p_session.rs:265-426) from the committed oracle fixture
                         (bench_native/fixtures/p2p_lists.npz), each lane encoded by ggrs_lane_encode
                         (the Rust crate's encoder) with its Save frames checked
      --req-form batch   the SyncTest encoding written from Python (numpy) per call
      --req-form lanes   ggrs_handle_requests_lanes: the GgrsRequest lists themselves (CSR)
      --req-form lockstep  ggrs_handle_requests: one list for every lane (lockstep sessions)
    --req-groups G (native, p2p; default 2): the sessions served as G lane groups (G engines): each
    group's batch is on the device while the host hands back and encodes the others';
    --req-threads T (native; default 1): host threads, thread t serving groups t*G/T .. (a game
    server runs its sessions' GGRS instances on several cores; each group is its own engine);
    --session-us T: host time per group and call spent in the modelled GGRS session logic (spin).
    One step = `calls` such calls; inputs are resident in host memory before the timed region."""
    world, rank, local_rank, torch, dist = setup_dist(args)
    import ctypes

    import numpy as np
    from ggrs_amd import Engine, synth
    from ggrs_amd._lib import REQ_ADVANCE, REQ_LOAD, REQ_SAVE
    L, P, maxp, cd, calls = args.lanes, 2, 9, 8, 64
    form = args.req_form
    G = args.req_groups if form in ("native", "p2p") else 1
    if L % G:
        raise SystemExit(f"--lanes {L} is not a multiple of --req-groups {G}")
    if G > 4 and not args.no_lane_server:
        print(f"note: --req-groups {G}: at most 4 lane servers run on a device (GPU_MAX_HW_QUEUES); the other "
              "groups' batches run as one launch each", file=sys.stderr)
    T = args.req_threads if form in ("native", "p2p") else 1
    if args.req_deferred and form != "p2p":
        raise SystemExit("--req-deferred is for P2P lists only: a SyncTestSession reads the previous call's "
                         "checksums (sync_test_session.rs:173-190)")
    if T < 1 or (form == "native" and G % T):
        raise SystemExit(f"--req-groups {G} is not a multiple of --req-threads {T}")
    sink = np.zeros(1, np.uint64)
    phases = np.zeros(4)
    drv = None
    fx = None
    if form in ("native", "p2p"):
        from ggrs_amd import build as gbuild
        drv = ctypes.CDLL(gbuild.build_driver())
        drv.handler_last_error.restype = ctypes.c_char_p
    if form == "p2p":
        fx = load_p2p_fixture()
        P, maxp = fx["P"], fx["maxp"]
        if (args.warmup + args.steps) * calls > fx["C"]:
            raise SystemExit(f"the P2P fixture holds {fx['C']} calls; --warmup + --steps must cover at most "
                             f"{fx['C'] // calls} steps of {calls} calls")
    frames = cd + 1 + (args.warmup + args.steps) * calls
    inputs = synth.gen_inputs(rank * L, L, frames, P, synth.MODEL_HELD) if form != "p2p" else None  # [frames][L][P]
    engs = [Engine(L // G, P, maxp, cd if form == "lockstep" else 0, 0, device=local_rank, trace_capacity=0)
            for _ in range(G)]
    eng = engs[0]
    for e in engs:
        if args.no_lane_server:
            e.set_lane_server(False)  # one lane_requests_kernel launch per call (per-launch profiles)
    handles = (ctypes.c_void_p * G)(*[e._h.value for e in engs])
    dbl = ctypes.POINTER(ctypes.c_double)
    u64 = ctypes.POINTER(ctypes.c_uint64)
    lane_frames = np.zeros(L, np.int32)

    def engine_of(lane):
        return engs[lane // (L // G)], lane % (L // G)

    if form == "native":
        inputs = np.ascontiguousarray(inputs)
        drv.handler_drive_synctest_groups.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p] + \
            [ctypes.c_int32] * 5 + [ctypes.c_double, u64, dbl, dbl]
        drv.handler_drive_synctest_threads.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                                       ctypes.c_void_p] + [ctypes.c_int32] * 5 + \
            [ctypes.c_double, u64, dbl, dbl]

        def run_calls(f, n):
            s, sec = ctypes.c_uint64(), ctypes.c_double()
            ph = (ctypes.c_double * 4)()
            if T > 1:
                rc = drv.handler_drive_synctest_threads(handles, G, T, ctypes.c_void_p(inputs.ctypes.data), L, P, cd,
                                                        f, n, args.session_us, ctypes.byref(s), ctypes.byref(sec), ph)
                ph = [x / T for x in ph]  # thread-seconds -> per-call wall shares
            else:
                rc = drv.handler_drive_synctest_groups(handles, G, ctypes.c_void_p(inputs.ctypes.data), L, P, cd, f,
                                                       n, args.session_us, ctypes.byref(s), ctypes.byref(sec), ph)
            assert rc == 0, rc
            phases[:] = list(ph)  # of the last batch of calls (the timed one)
            sink[0] += s.value
    elif form == "p2p":
        vp = ctypes.c_void_p
        drv.handler_drive_p2p_groups.argtypes = [vp, ctypes.c_int32] + [ctypes.c_int32] * 4 + [vp] * 7 + \
            [ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_int32, u64, dbl, dbl]

        def run_calls(c, n):
            s, sec = ctypes.c_uint64(), ctypes.c_double()
            ph = (ctypes.c_double * 4)()
            ptr = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
            rc = drv.handler_drive_p2p_groups(handles, G, L, P, fx["M"], fx["C"], ptr(fx["reqs"]), ptr(fx["req_off"]),
                                              ptr(fx["adv_off"]), ptr(fx["inputs"]), ptr(fx["status"]),
                                              ptr(fx["shape"]), ptr(lane_frames), c, n, args.session_us,
                                              int(args.req_deferred), T, ctypes.byref(s), ctypes.byref(sec), ph)
            assert rc == 0, (rc, drv.handler_last_error() or eng._L.ggrs_last_error())
            phases[:] = list(ph)
            sink[0] += s.value
    elif form == "batch":
        batch = eng.lane_batch(2, 1, cd + 1, cd + 1)
        steady = np.array(synctest_tokens(cd + 1, cd)[0], np.uint32)[:, None].repeat(L, axis=1)

        def call(f):
            words, n, nl, na, ns = synctest_tokens(f, cd)
            if f > cd:
                batch.tokens[:2] = steady
                batch.load_frames[0].fill(f - cd)
                batch.inputs[:na] = inputs[f - cd:f + 1]
            else:
                batch.tokens[:len(words)] = np.array(words, np.uint32)[:, None]
                batch.inputs[:1] = inputs[f:f + 1]
            nf = batch.run(len(words), nl, na, ns)
            assert nf == 0
            sink[0] += int(batch.checksums[ns - 1, 0])  # the checksums are back in host memory
    else:
        def lists(f):
            reqs, adv = [], []
            if f > cd:
                reqs.append((REQ_LOAD, f - cd))
                for i in range(cd):
                    if i > 0:
                        reqs.append((REQ_SAVE, f - cd + i))
                    reqs.append((REQ_ADVANCE, 0))
                    adv.append(f - cd + i)
            reqs.append((REQ_SAVE, f))
            reqs.append((REQ_ADVANCE, 0))
            adv.append(f)
            return reqs, adv
        if form == "lanes":
            def call(f):
                reqs, adv = lists(f)
                r = np.array(reqs * L, np.int32)
                off = np.arange(0, (L + 1) * len(reqs), len(reqs), dtype=np.int32)
                inp = np.ascontiguousarray(inputs[adv].transpose(1, 0, 2)).reshape(-1, P)
                cks, _ = eng.handle_requests_lanes(r, off, inp)
                sink[0] += int(cks[-1])
        else:
            def call(f):
                reqs, adv = lists(f)
                eng.handle_requests(reqs, np.ascontiguousarray(inputs[adv]))

    if drv is None:
        def run_calls(f, n):
            for k in range(n):
                call(f + k)
    # warm-up calls, then the timed ones (SyncTest lists: the first cd + 1 frames carry no rollback)
    f = (0 if form == "p2p" else cd + 1) + args.warmup * calls
    host_profile = None
    if form == "p2p" and args.req_profile and args.warmup >= 2:
        # the encoder's profile over warm-up steps 2.. (instrumented: not the timed region)
        run_calls(0, calls)
        os.environ["GGRS_DRIVER_PROFILE"] = "1"
        try:
            run_calls(calls, f - calls)
        finally:
            os.environ.pop("GGRS_DRIVER_PROFILE", None)
        host_profile = read_host_profile(drv, T, f - calls, L // G, G)
    else:
        run_calls(0, f)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    run_calls(f, args.steps * calls)  # every call returns with its results in host memory: synchronised
    f_timed = f
    f += args.steps * calls
    for e in engs:
        e.synchronize()  # stops the idle lane server (a device-wide barrier would wait out its watchdog)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    n_calls = args.steps * calls
    if form == "p2p":
        # session-frames: every call of every lane; resimulated: the AdvanceFrames of the rollbacks
        m_of = np.arange(L) % fx["M"]
        resim = int(np.maximum(fx["n_adv"][m_of][:, f_timed:f] - 1, 0).sum())
        units = L * n_calls
    else:
        resim = L * cd * n_calls
        units = resim
    elapsed, total, per_rank = rank_timings(dist, torch, elapsed, units)
    _, total_resim, _ = rank_timings(dist, torch, elapsed, resim) if form == "p2p" else (None, total, None)
    value = total / elapsed
    parity = None
    if rank == 0:
        try:
            from oracle import oracle as O
            O.build()
            if form == "p2p":
                ok = {}
                for lane in (0, L - 1):
                    m = lane % fx["M"]
                    a, b = int(fx["req_off"][m, 0]), int(fx["req_off"][m, f])
                    kind = fx["kind"][a:b].astype(np.int32)
                    inp = np.zeros((b - a, P), np.uint8)
                    st = np.zeros((b - a, P), np.uint8)
                    adv = np.nonzero(kind == REQ_ADVANCE)[0]
                    a0 = int(fx["adv_off"][m, 0])
                    inp[adv] = fx["inputs"][a0:a0 + len(adv)]
                    st[adv] = fx["status"][a0:a0 + len(adv)]
                    r = O.handler_run(kind, fx["frame"][a:b], inp, st, P, maxp)
                    e, li = engine_of(lane)
                    ok[f"lane{lane}_final_state_bit_exact"] = r["rc"] == 0 and bytes(e.state(li)) == bytes(
                        r["final_state"])
                parity = ok
            else:
                e_last, l_last = engine_of(L - 1)
                r = O.synctest_run(inputs[:f, 0, :], P, maxp, cd, 0)
                parity = {"lane0_final_state_bit_exact": bytes(eng.state(0)) == bytes(r["final_state"]),
                          "lane_last_final_state_bit_exact": bytes(e_last.state(l_last)) == bytes(
                              O.synctest_run(inputs[:f, L - 1, :], P, maxp, cd, 0)["final_state"])}
        except Exception as exc:
            parity = {"error": repr(exc)}
        cpu_baseline = None
        if world == 1 and not args.no_cpu_baseline:
            cpu_baseline = (requests_p2p_cpu_baseline(args, fx) if form == "p2p" else
                            requests_cpu_baseline(args, synth, P, maxp, cd))
        # the device work of one call is the SyncTest frame's Load + cd x (Advance, Save) per lane:
        # its algorithmic HBM bytes over the call's wall time (PCIe round trip and host handler
        # included -- the call is latency-bound, so this is far below the HBM roofline)
        call_s = elapsed / n_calls
        per_call = L * bytes_per_synctest_call(P, cd)
        roofline = {"bound": "hbm", "achieved": round(per_call / call_s / 1e9, 3), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(per_call / call_s / 1e9 / HBM_PEAK_GBS, 6),
                    "traffic": pmc_traffic(f"requests_l{L}"), "algorithmic_bytes_per_call": per_call,
                    "note": "per call: one PCIe round trip (lists + inputs in, checksums out) around a "
                            "microsecond-scale kernel; latency-bound by construction"} if form != "p2p" else None
        wl = (f"requests: {L} SyncTest sessions per GPU (cd {cd}, 2 players), each call every session's request "
              f"list of one advance_frame (form {form})" if form != "p2p" else
              f"requests: {L} P2P sessions per GPU (2 players, max_prediction {maxp}, remote inputs arriving in "
              f"jittered bursts), each lane its own session's list per call from the committed oracle fixture "
              f"({fx['M']} distinct sessions tiled over the lanes), encoded per lane by ggrs_lane_encode")
        line = {
            "metric": ("resimulated session-frames/sec (node), request-level boundary" if form != "p2p"
                       else "P2P session-frames/sec (node), request-level boundary"),
            "value": round(value, 1), "unit": "session-frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": wl + f", {calls} calls per step, lists and inputs from host memory, checksums "
                                        "back to host memory each call",
                       "sessions_per_gpu": L, "req_form": form, "lane_groups": G, "host_threads": T,
                       "deferred_handback": bool(args.req_deferred),
                       "session_us_per_group_call":
                           args.session_us, "lane_server": not args.no_lane_server,
                       "us_per_call": round(elapsed / n_calls * 1e6, 2),
                       **({("us_per_call_encode_handback_submit_wait_session" if form == "p2p" else
                            "us_per_call_host_encode_device_handback_session"): [round(x / n_calls * 1e6, 2)
                                                                                 for x in phases]}
                          if drv is not None else {}),
                       "parallelism": f"sessions sharded over {world} GPU(s)"},
            "dist": dist_info(dist, per_rank),
            "roofline": roofline, "cpu_baseline": cpu_baseline, "parity": parity,
            "note": "latency-bound by construction (one PCIe round trip per call and lane group); the fused "
                    "ggrs_synctest_advance_frames path is the default bench"}
        if form == "p2p":
            line["resimulated_session_frames_per_s"] = round(total_resim / elapsed, 1)
            line["resimulated_per_session_frame"] = round(resim / units, 4)
            # the bound: each call is a host encode + hand-back of every lane's list and one PCIe
            # round trip per lane group; the device's own work per call (the lists' advances, saves,
            # loads) is microseconds of HBM traffic, so the HBM figure is a floor, and the call's
            # critical path is the host's -- achieved against the measured device round trip
            m_of = np.arange(L) % fx["M"]
            adv_c = int(fx["n_adv"][m_of][:, f_timed:f].sum()) / n_calls
            Sp = 4 + 20 * P
            dev_bytes = adv_c * (2 * Sp + P) + L * 2 * Sp  # per call: every advance's state in/out + inputs,
            call_us = elapsed / n_calls * 1e6             # each lane's state loaded and stored once
            wait_us = phases[2] / n_calls * 1e6
            submit_us = phases[1] / n_calls * 1e6
            line["roofline"] = {
                "bound": "hbm", "achieved": round(dev_bytes / (call_us * 1e-6) / 1e9, 3), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(dev_bytes / (call_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 6), "traffic": None,
                "algorithmic_bytes_per_call": int(dev_bytes),
                "latency_bound": {"unit": "us", "us_per_call": round(call_us, 2),
                                  "device_round_trip_us_per_call": round(wait_us + submit_us, 2),
                                  "host_encode_handback_us_per_call": round(phases[0] / n_calls * 1e6, 2),
                                  "frac_of_call_on_device_round_trip": round((wait_us + submit_us) / call_us, 4)},
                "note": "host-bound: the call is the host encode + hand-back of every lane's list plus the lane "
                        "groups' PCIe round trips; the device work per call is microseconds of HBM"}
            if host_profile is not None:
                line["host_profile"] = host_profile
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def run_launch_selftest(args):
    """The launcher's own check, on the CPU: every rank joins a gloo group, the ranks' (RANK,
    LOCAL_RANK, WORLD_SIZE) are all-gathered and rank 0 prints them as the one JSON line.  Rank
    --selftest-fail-rank exits with status 3 before joining (exit-status propagation)."""
    rank = int(os.environ.get("RANK", "0"))
    if rank == args.selftest_fail_rank:
        sys.exit(3)
    import torch
    import torch.distributed as dist
    if "WORLD_SIZE" not in os.environ:  # one rank, in process
        os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    dist.init_process_group("gloo")
    me =torch.tensor([rank, int(os.environ.get("LOCAL_RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))])
    out = [torch.empty_like(me) for _ in range(dist.get_world_size())]
    dist.all_gather(out, me)
    xleg = exchange_leg(torch, dist, lambda g: _StubReportEngine(g), 24, 8, False)
    if rank == 0:
        print(json.dumps({"metric": "launch-selftest", "value": dist.get_world_size(), "n_gpus": dist.get_world_size(),
                          "ranks": [o.tolist() for o in out],
                          "master_addr": os.environ.get("MASTER_ADDR"), "exchange": xleg}))
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames-per-step", type=int, default=512)
    ap.add_argument("--lanes", type=int, default=4096, help="sessions per GPU (config 2: 4096)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cores available)")
    ap.add_argument("--cpu-frames", type=int, default=3000000,
                    help="SyncTest frames per CPU thread (default: ~10 s of host work)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--path", choices=["pipelined", "sequential", "chains", "batched"], default="pipelined",
                    help="SyncTest kernel (DESIGN.md section 3)")
    ap.add_argument("--config", type=int, choices=[2, 3, 4, 5], default=2,
                    help="BASELINE.json config: 2 = SyncTest (default), 3/4 = branch rollback, "
                         "5 = 1 MB particle-world SyncTest")
    ap.add_argument("--no-lane-server", action="store_true", help="requests: a launch per call")
    ap.add_argument("--rounds-per-step", type=int, default=16, help="configs 3/4: rounds per step")
    ap.add_argument("--sessions", type=int, default=0, help="config 5: sessions per GPU (0 = 8192)")
    ap.add_argument("--exchange-batch", type=int, default=0,
                    help="configs 3/4 across ranks: rounds per report all-gather (1 = one per confirmation; "
                         "0 = --rounds-per-step, one all-gather per step)")
    ap.add_argument("--no-exchange-leg", action="store_true",
                    help="config 2 across ranks: skip the config-4 report all-gather leg (the line's exchange key)")
    ap.add_argument("--exchange-rounds", type=int, default=256,
                    help="config 2 across ranks: rounds of the exchange leg (gloo: at most 32)")
    ap.add_argument("--exchange-leg-batch", type=int, default=16,
                    help="config 2 across ranks: rounds per all-gather in the exchange leg")
    ap.add_argument("--peers", action="store_true",
                    help="configs 3/4 and p2p: rank r and r + world/2 run the same sessions (the two "
                         "machines of a match) and compare checksums exchanged over the process group")
    ap.add_argument("--p2p-form", choices=["default", "flat", "lockstep", "unstaged", "chains", "flat_queues", "canonical"],
                    default="default",
                    help="p2p: kernel form (DESIGN.md section 3)")
    ap.add_argument("--sparse", action="store_true", help="p2p: sparse saving (SURVEY.md 8f row 4)")
    ap.add_argument("--arrivals", choices=["fixed", "jitter", "stall"], default="fixed",
                    help="p2p: the network -- every remote input --latency frames late (fixed), or per-session "
                         "arrival schedules (ggrs_p2p_add_arrivals): jittered lags, plus network stalls")
    ap.add_argument("--latency", type=int, default=4, help="p2p: frames the remote player's inputs arrive late")
    ap.add_argument("--max-prediction", type=int, default=8, help="p2p: max_prediction (builder.rs:130-147)")
    ap.add_argument("--p2p-calls", type=int, default=64,
                    help="p2p: advance_frame calls per session per step (one launch; default 64)")
    ap.add_argument("--req-form", choices=["native", "p2p", "batch", "lanes", "lockstep"], default="native",
                    help="requests: the boundary form (run_requests docstring)")
    ap.add_argument("--codec-layout", choices=["chunked", "strided"], default="chunked",
                    help="codec: packet layout (chunked: each 256-packet block's packets back to back)")
    ap.add_argument("--req-groups", type=int, default=2,
                    help="requests (native, p2p): lane groups (engines) whose batches overlap the host's work; at most 4 with the lane server (one persistent server per hardware queue)")
    ap.add_argument("--req-threads", type=int, default=1,
                    help="requests: host threads -- native: serving the lane groups (G a multiple of it); "
                         "p2p: encoding and handing back each group's lanes")
    ap.add_argument("--req-deferred", action="store_true",
                    help="requests (p2p): deferred checksum hand-back (handle_requests_deferred): the session "
                         "logic (--session-us) overlaps the batch on the device")
    ap.add_argument("--req-profile", action="store_true",
                    help="requests (p2p): profile the host encoder over the warm-up calls after the first step "
                         "(per thread: spin / hand-back / encode time, and user-space cache counters where the "
                         "kernel allows them) -- reported as host_profile, outside the timed region")
    ap.add_argument("--session-us", type=float, default=0.0,
                    help="requests: modelled GGRS session-logic host time per lane group and call (us)")
    ap.add_argument("--workload", choices=["synctest", "p2p", "codec", "requests", "launch-selftest"],
                    default="synctest",
                    help="p2p: the device P2P rollback decision (SURVEY.md 8f), --sessions per GPU; "
                         "launch-selftest: the rank launcher alone (CPU, gloo; tests/test_bench_launch.py)")
    ap.add_argument("--selftest-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.exchange_batch <= 0:
        args.exchange_batch = args.rounds_per_step
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `bench.py --gpus N` run plainly: start the N ranks here (before anything touches the GPU)
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    if args.workload == "launch-selftest":
        return run_launch_selftest(args)
    if args.workload == "p2p":
        return run_p2p(args)
    if args.workload == "codec":
        return run_codec(args)
    if args.workload == "requests":
        # the host handler's worker threads meet at barriers twice per lane group and call: spin
        # there (before torch loads libgomp, which reads this once)
        os.environ.setdefault("OMP_WAIT_POLICY", "active")
        # one worker per physical core, bound: unbound, the workers of a job whose affinity spans the
        # machine (a CPU quota, not a cpuset) share SMT siblings and migrate -- the P2P encoder then
        # takes 204 cycles per lane at IPC 1.7 instead of 83 at IPC 4.1 for the same 342
        # instructions (profiles/r06_reqp2p/plateau_threads_binding.txt)
        if args.req_form == "p2p" and args.req_threads > 1:
            os.environ.setdefault("OMP_PROC_BIND", "close")
            os.environ.setdefault("OMP_PLACES", "cores")
        return run_requests(args)
    if args.config == 5:
        return run_particles(args)
    if args.config != 2:
        return run_branch(args)

    world, rank, local_rank, torch, dist = setup_dist(args)
    from ggrs_amd import Engine
    from ggrs_amd import synth

    P, maxp, cd, delay = 2, 9, 8, 0
    lanes, fps = args.lanes, args.frames_per_step
    total_frames = (args.warmup + args.steps) * fps
    assert args.warmup * fps > cd, "warm-up must cover the first check_distance frames"
    trace_cap = min(256, total_frames)

    inputs = synth.gen_inputs(rank * lanes, lanes, total_frames, P, synth.MODEL_HELD)
    eng = Engine(lanes, P, maxp, cd, delay, input_capacity=total_frames + cd + delay + 2,
                 device=local_rank, trace_capacity=trace_cap)
    eng.set_synctest_path({"pipelined": 0, "sequential": 1, "chains": 2, "batched": 3}[args.path])
    eng.add_local_inputs(0, inputs)  # resident in HBM before anything is timed
    eng.synchronize()

    def barrier():
        eng.synchronize()
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        eng.synctest_advance_frames(fps)
    barrier()
    eng.timing_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.synctest_advance_frames(fps)
    eng.timing_stop()  # the end event right behind the last launch, no wait inside the span
    barrier()
    t1 = time.perf_counter()
    kernel_ms, launches = eng.timing_read()
    elapsed = t1 - t0
    elapsed, total_resim, per_rank = rank_timings(dist, torch, elapsed, lanes * cd * fps * args.steps)

    status, _, _ = eng.mismatches()
    halted = int((status != 0).sum())  # a halted lane would stop resimulating: must be none
    value = total_resim / elapsed

    # roofline of the one kernel that runs in the timed region (synctest_kernel<2>)
    per_call = bytes_per_synctest_call(P, cd)
    bytes_per_launch = lanes * fps * per_call
    avg_launch_s = kernel_ms / 1e3 / max(launches, 1)
    achieved = bytes_per_launch / avg_launch_s / 1e9
    workload = f"config2_l{lanes}_f{fps}"
    roofline = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": pmc_traffic(workload),
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "avg_launch_ms": round(avg_launch_s * 1e3, 4),
                # SURVEY.md 8(d)'s per-resimulated-frame figure (S + 2) + S / cd + P (53.5 B at cd 8,
                # two players) instead of this program's per-call count above (57.5 B per frame)
                "frac_survey_bytes": round(lanes * fps * cd * ((4 + 20 * P + 2) + (4 + 20 * P) / cd + P)
                                           / avg_launch_s / 1e9 / HBM_PEAK_GBS, 6),
                "valu": pmc_valu(workload),
                "note": "issue/latency-bound step kernel (f32 step + f64 glibc sincosf, one wave per "
                        "SIMD); the 2 MB ring fits L2/MALL, so HBM traffic is below the algorithmic bytes"}

    parity = None
    cpu_baseline = None
    if rank == 0:
        try:
            from oracle import oracle as O  # checker + CPU baseline only
            O.build()
            from oracle import every_lane
            # EVERY lane against the oracle's SyncTestSession (oracle_synctest_batch on the job's
            # CPU share): final state, ring checksums, the trace's last trace_cap frames
            parity = every_lane.synctest(eng, inputs, P, maxp, cd, delay, trace_first=total_frames - trace_cap,
                                         trace_n=trace_cap)
            parity["every_lane_bit_exact"] = all(v == 0 for k, v in parity.items() if k.endswith("_mismatched"))
            if world == 1 and not args.no_cpu_baseline:
                threads = cpu_threads(args)
                frames = max(args.cpu_frames, total_frames)
                n, wall, ck0 = O.synctest_bench(threads, frames, warmup=0, num_players=P,
                                                max_prediction=maxp, check_distance=cd,
                                                input_delay=delay, model=O.MODEL_HELD,
                                                seed_base=synth.SEED_BASE)
                gpu_tr = eng.trace(total_frames - trace_cap, trace_cap)[:, 0]
                # the same loop on one thread beside the multi-thread run
                frames1 = max(args.cpu_frames // 3, total_frames)
                n1, wall1, _ = O.synctest_bench(1, frames1, warmup=0, num_players=P, max_prediction=maxp,
                                                check_distance=cd, input_delay=delay, model=O.MODEL_HELD,
                                                seed_base=synth.SEED_BASE)
                # config 1's own semantics (the reference's ex_game SyncTest: check_distance 7,
                # input delay 2, max_prediction 8, uniform inputs) on the same threads
                frames_c1 = max(args.cpu_frames // 2, total_frames)
                n_c1, wall_c1, _ = O.synctest_bench(threads, frames_c1, warmup=0, num_players=2, max_prediction=8,
                                                    check_distance=7, input_delay=2, model=O.MODEL_UNIFORM,
                                                    seed_base=synth.SEED_BASE)
                cpu_baseline = {
                    "value": round(n / wall, 1), "unit": "session-frames/s", "cores": threads,
                    "kind": "port",
                    "sample": f"{threads} threads x {frames} SyncTest frames (1 session/thread, "
                              f"cd {cd}, 2 players, held-key inputs), C restatement of the "
                              f"reference loop (oracle/ggrs_oracle.c)",
                    "wall_s": round(wall, 3), "cpu": cpu_model(),
                    "thread0_matches_gpu_lane0": bool((ck0[total_frames - trace_cap:total_frames] == gpu_tr).all()),
                    "single_thread": {"value": round(n1 / wall1, 1), "cores": 1, "frames": frames1,
                                      "wall_s": round(wall1, 3)},
                    "config1_semantics": {"value": round(n_c1 / wall_c1, 1), "cores": threads, "frames": frames_c1,
                                          "wall_s": round(wall_c1, 3),
                                          "sample": "check_distance 7, input delay 2, max_prediction 8, uniform "
                                                    "inputs, 2 players (the reference's ex_game SyncTest)"},
                }
        except Exception as exc:  # the oracle is optional on the measurement path
            parity = {"error": repr(exc)}

    xleg = None
    if dist is not None and not args.no_exchange_leg:
        # the one collective the north star names, measured beside (not inside) the headline:
        # the config-4 report all-gather across this run's ranks
        gpu = dist.get_backend() != "gloo"
        n = args.exchange_rounds if gpu else min(args.exchange_rounds, 32)
        xleg = exchange_leg(torch, dist, branch_exchange_engine(torch, local_rank, 2 * n + 32), n,
                            args.exchange_leg_batch, gpu)

    if rank == 0:
        line = {
            "metric": "resimulated session-frames/sec (node)",
            "value": round(value, 1),
            "unit": "session-frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": "config2: ex_game x 4096 sessions/GPU, SyncTest 8-frame rollback "
                                   "every frame (check_distance 8, max_prediction 9), 2 players, "
                                   "held-key inputs",
                       "sessions_per_gpu": lanes, "global_sessions": lanes * world,
                       "frames_per_step": fps, "players": P, "check_distance": cd,
                       "max_prediction": maxp, "kernel_path": args.path,
                       "parallelism": f"sessions sharded over {world} GPU(s)"},
            "dist": dist_info(dist, per_rank),
            "roofline": roofline,
            "cpu_baseline": cpu_baseline,
            "halted_lanes": halted,
            "parity": parity,
        }
        if xleg is not None:
            line["exchange"] = xleg
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
