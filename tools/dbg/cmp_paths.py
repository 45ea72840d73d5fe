"""Debug: run one SyncTest configuration on two kernel paths and report the first differing
trace frame / lanes (tools only)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from ggrs_amd import Engine, synth

def run(path, inputs, P, maxp, cd, d, chunks):
    F, L = inputs.shape[0], inputs.shape[1]
    eng = Engine(L, P, maxp, cd, d, input_capacity=F + d + cd + 2, trace_capacity=F)
    eng.set_synctest_path(path)
    eng.add_local_inputs(0, inputs)
    for n in chunks:
        eng.synctest_advance_frames(n)
    eng.synchronize()
    return eng.trace(0, F)

P, maxp, cd, d, F, L = 2, 9, 8, 0, 600, 64
inputs = synth.gen_inputs(0, L, F, P, synth.MODEL_HELD)
for chunks in ([1, 2, 9, 588], [600], [12, 588]):
    a = run(2, inputs, P, maxp, cd, d, chunks)
    b = run(3, inputs, P, maxp, cd, d, chunks)
    diff = np.argwhere(a != b)
    print(chunks, "differences:", len(diff), "first:", diff[:5].tolist())
