"""bench.py --gpus N starts its N ranks itself: the parent spawns one
torch.distributed.run child before anything imports torch, forwards rank 0's JSON line and
propagates a failing rank's exit status.  CPU only (gloo)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _run(*extra, env_extra=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "launch-selftest", *extra],
                          capture_output=True, text=True, env=env, timeout=240)


def test_launch_cmd_shape():
    cmd = bench.rank_launch_cmd(["--gpus", "4", "--config", "4"], 4, 29999, python="py")
    assert cmd[:3] == ["py", "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert "--master-port=29999" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--config", "4"]
    assert cmd[-5].endswith("bench.py")


def test_parent_does_not_import_torch_before_launch():
    # the launcher path runs before any torch import: bench.py imports nothing heavy at module level
    src = open(os.path.join(ROOT, "bench.py")).read()
    head = src[:src.index("def ")]
    assert "import torch" not in head


@pytest.mark.parametrize("n", [2, 3])
def test_spawns_n_ranks_and_forwards_one_line(n):
    r = _run("--gpus", str(n))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["value"] == n
    assert sorted(tuple(x) for x in d["ranks"]) == [(k, k, n) for k in range(n)]
    assert d["master_addr"] == "127.0.0.1"
    assert d["launch"] == {"launcher": "bench.py -> torch.distributed.run", "ranks_spawned": n}


def test_failing_rank_propagates_nonzero_exit():
    r = _run("--gpus", "2", "--selftest-fail-rank", "1")
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.strip()]


def test_single_rank_runs_in_process():
    r = _run("--gpus", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]  # gloo's banner aside
    d = json.loads(lines[-1])
    assert d["n_gpus"] == 1 and "launch" not in d


EXCHANGE_KEYS = {"what", "world_size", "backend", "peers", "engine", "rounds", "batch", "allgathers",
                 "us_per_round_with_allgather", "us_per_round_without_allgather", "report_bytes_per_round_per_rank",
                 "gathered_bytes_per_allgather", "us_per_allgather_alone", "allgather_bytes_per_s", "desyncs"}


@pytest.mark.parametrize("n", [2, 3])
def test_exchange_leg_record(n):
    """The `exchange` key a multi-rank bench line carries: bench.exchange_leg
    runs the batched ReportExchange across the ranks (here over gloo with a CPU report engine, on
    the GPU box the config-4 BranchEngine over RCCL) and records the world size the process group
    saw, per-round times with and without the all-gather, gathered bytes and the desync count."""
    r = _run("--gpus", str(n))
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][0])
    x = d["exchange"]
    assert set(x) == EXCHANGE_KEYS
    assert x["world_size"] == n and x["backend"] == "gloo"
    assert x["peers"] == (n % 2 == 0)
    assert x["rounds"] == 24 and x["batch"] == 8 and x["allgathers"] == 3
    assert x["gathered_bytes_per_allgather"] == n * 8 * x["report_bytes_per_round_per_rank"]
    assert x["desyncs"] == 0
    for k in ("us_per_round_with_allgather", "us_per_round_without_allgather", "us_per_allgather_alone",
              "allgather_bytes_per_s"):
        assert x[k] > 0
