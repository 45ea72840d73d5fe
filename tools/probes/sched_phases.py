"""Phase clocks of the scheduled P2P kernel (timing probe, experiment library only):
GGRS_AMD_EXP_LIB=libggrs_amd_stamps.so python tools/probes/sched_phases.py [sessions] [max_prediction]
The stamps build writes per block (lanes 0-3 of its first session's resim counter) the cycles spent
staging, in the control pass, in the step loop, and in the whole stage loop of the last launch."""
import sys
import numpy as np
import torch  # noqa: F401  (HIP runtime first)
from ggrs_amd import P2PEngine, synth

S = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
maxp = int(sys.argv[2]) if len(sys.argv) > 2 else 8
calls, launches = 64, 4
frames = calls * launches
rows = synth.gen_inputs(0, S, frames, 2, synth.MODEL_HELD)
eng = P2PEngine(S, num_players=2, local_players=(0,), max_prediction=maxp, remote_latency=1, input_capacity=frames + 4)
eng.set_arrival_schedule(True)
eng.add_arrivals(0, synth.jitter_arrivals(0, S, frames, maxp))
eng.add_inputs(0, rows)
for _ in range(launches):
    eng.advance_frames(calls)
eng.synchronize()
rb, rs = eng.stats()
import os
seg = "stamps3" in os.environ.get("GGRS_AMD_EXP_LIB", "")
blocks = np.asarray(rs).reshape(-1, 64)[:, :8].astype(np.float64)
names = (["staging", "control", "call start", "decisions + local input", "inputs + save", "advance", "step loop", "iterations"]
         if seg else ["staging", "control", "step loop", "stage loop total"])
for k, n in enumerate(names):
    col = blocks[:, k]
    print(f"{n:18s} mean {col.mean():10.0f} cycles  max {col.max():10.0f}  (last launch, per block)")
