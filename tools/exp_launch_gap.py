"""Timing experiment: config-2 step time with and without the per-launch HIP event pair.

Run once per library (GGRS_AMD_EXP_LIB selects tools/exp_build.sh's variant); prints the wall
time per 512-frame step over K back-to-back launches.  Not a parity check.
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from ggrs_amd import Engine, synth  # noqa: E402

lanes, fps, P, K, W = 4096, 512, 2, 40, 3
inputs = synth.gen_inputs(0, lanes, (K + W) * fps, P, synth.MODEL_HELD)
eng = Engine(lanes, P, 9, 8, 0, input_capacity=(K + W) * fps + 12, device=0, trace_capacity=256)
eng.add_local_inputs(0, inputs)
for _ in range(W):
    eng.synctest_advance_frames(fps)
eng.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    eng.synctest_advance_frames(fps)
eng.synchronize()
dt = (time.perf_counter() - t0) / K
print(f"lib={os.environ.get('GGRS_AMD_EXP_LIB', 'default')} ms_per_step={dt * 1e3:.4f} "
      f"value={lanes * 8 * fps / dt:.4e}")
