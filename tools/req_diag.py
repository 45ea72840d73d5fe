"""Where a request-boundary call's time goes (bench --workload requests, batch form): host writes
into the mapped batch, the run call (launch + kernel + wait), and the run call on an unchanged
batch.  Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402  (one HIP runtime: torch's)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from ggrs_amd import Engine, synth  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
SERVER = (sys.argv[2] != "0") if len(sys.argv) > 2 else True
P, cd, maxp, calls = 2, 8, 9, 2000
inputs = synth.gen_inputs(0, L, calls + cd + 1, P, synth.MODEL_HELD)
eng = Engine(L, P, maxp, 0, 0)
eng.set_lane_server(SERVER)
batch = eng.lane_batch(2, 1, cd + 1, cd + 1)
steady = np.array(bench.synctest_tokens(cd + 1, cd)[0], np.uint32)[:, None].repeat(L, axis=1)
for f in range(cd + 1):
    words, n, nl, na, ns = bench.synctest_tokens(f, cd)
    batch.tokens[:len(words)] = np.array(words, np.uint32)[:, None]
    batch.inputs[:1] = inputs[f:f + 1]
    batch.run(len(words), nl, na, ns)
tw = tr = 0.0
f = cd + 1
eng.timing_reset()
for _ in range(calls):
    t0 = time.perf_counter()
    batch.tokens[:2] = steady
    batch.load_frames[0].fill(f - cd)
    batch.inputs[:cd + 1] = inputs[f - cd:f + 1]
    t1 = time.perf_counter()
    batch.run(2, 1, cd + 1, cd)
    t2 = time.perf_counter()
    tw += t1 - t0
    tr += t2 - t1
    f += 1
span_ms, launches = eng.timing_read()
# the run call alone, same batch each time (frames do not advance: Load f-cd again is valid
# while the cell holds it, so re-run the last call's list on a saved copy is not possible --
# instead time a list of only Save + Advance)
batch.tokens[0] = np.uint32(bench.synctest_tokens(0, cd)[0][0])
t0 = time.perf_counter()
n_small = 2000
for _ in range(n_small):
    batch.run(1, 0, 1, 1)
t_small = (time.perf_counter() - t0) / n_small
x = torch.zeros(1, device="cuda")
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(2000):
    x.add_(1)
    torch.cuda.synchronize()
t_floor = (time.perf_counter() - t0) / 2000
print(json.dumps({"lanes": L, "server": SERVER, "us_torch_launch_sync_floor": round(t_floor * 1e6, 2), "us_write": round(tw / calls * 1e6, 2), "us_run": round(tr / calls * 1e6, 2),
                  "us_span_per_launch": round(span_ms * 1e3 / max(launches, 1), 2),
                  "us_run_save_advance_only": round(t_small * 1e6, 2)}))
