"""Generate bench_native/fixtures/p2p_lists.npz: the request lists M P2P sessions emit per call
(the oracle's P2PSession restatement, oracle_p2p_stream: p2p_session.rs:265-426 under a jittery
network, so each session rolls back to its own first_incorrect frame with its own replay count),
for bench.py --workload requests --req-form p2p.  The bench replays the committed lists; the oracle
is not run at bench time.  Run from the repo root:  python bench_native/make_p2p_fixture.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

M, C, P, MAXP = 64, 1600, 2, 8


def main():
    O.build()
    kinds, frames, inputs, status = [], [], [], []
    req_off = np.zeros((M, C + 1), np.int64)
    adv_off = np.zeros((M, C + 1), np.int64)
    n_req = n_adv = 0
    for m in range(M):
        inp = O.gen_inputs(O.session_seed(m, 0xB3AC0000), C, P, O.MODEL_HELD)
        s = O.p2p_stream(inp, O.jitter_schedule(C, MAXP, seed=1000 + m), num_players=P, max_prediction=MAXP)
        assert s["rc"] == 0 and s["calls"] == C
        off = s["call_off"]
        k = s["kind"]
        adv_before = np.concatenate([[0], np.cumsum(k == 2)])
        req_off[m] = n_req + off
        adv_off[m] = n_adv + adv_before[off]
        kinds.append(k.astype(np.uint8))
        frames.append(s["frame"].astype(np.int32))
        inputs.append(s["inputs"][k == 2])
        status.append(s["status"][k == 2])
        n_req += len(k)
        n_adv += int((k == 2).sum())
    out = os.path.join(ROOT, "bench_native", "fixtures", "p2p_lists.npz")
    np.savez_compressed(out, kind=np.concatenate(kinds), frame=np.concatenate(frames),
                        inputs=np.concatenate(inputs), status=np.concatenate(status), req_off=req_off,
                        adv_off=adv_off, sessions=M, calls=C, players=P, max_prediction=MAXP,
                        seed_base=0xB3AC0000)
    print(out, n_req, "requests", n_adv, "advances", os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
