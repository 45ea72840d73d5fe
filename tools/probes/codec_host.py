"""Where the codec bench step's time goes beyond its two kernels: host time per step() call, step
time with and without the per-step timing events, and one step captured in a graph and replayed.
Run on the GPU box from the repo root: python tools/probes/codec_host.py"""
import time

import numpy as np
import torch

from ggrs_amd import codec

N, W, B, K = 1 << 20, 8, 2, 200
rng = np.random.default_rng(1234)
ref = rng.integers(0, 16, (N, B), dtype=np.uint8)
held = np.repeat(ref[:, None, :], W, axis=1)
flip = rng.random((N, W, B)) < 1.0 / 8.0
pend = np.where(flip, rng.integers(0, 16, (N, W, B), dtype=np.uint8), held).astype(np.uint8)
dev = torch.device("cuda", 0)
d_ref, d_pend = torch.from_numpy(ref).to(dev), torch.from_numpy(pend).to(dev)
d_cnt = torch.full((N,), W, dtype=torch.int32, device=dev)
stride = codec.max_packet_bytes(B, W)
dec_buf = torch.empty((N, W, B), dtype=torch.uint8, device=dev)


def step(ev=None):
    if ev:
        ev[0].record()
    out, ln = codec.encode(d_ref, d_pend, d_cnt, stride, chunked=True)
    if ev:
        ev[1].record()
    codec.decode(d_ref, out, ln, W, chunked=True, out=dec_buf)
    if ev:
        ev[2].record()


def timed(fn, label):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    host = 0.0
    t0 = time.perf_counter()
    for _ in range(K):
        h0 = time.perf_counter()
        fn()
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{label}: {dt / K * 1e6:.1f} us/step, host {host / K * 1e6:.1f} us/step, {N * K / dt:.3e} packets/s", flush=True)


timed(step, "plain")
timed(lambda: step([torch.cuda.Event(enable_timing=True) for _ in range(3)]), "events")
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    step()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    step()
timed(g.replay, "graph")
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2):
    for _ in range(10):
        step()
K //= 10
timed(g2.replay, "graph x10 (per 10 steps)")

# events created through the HIP runtime with release-scope flags, recorded on torch's stream
import ctypes
hip = ctypes.CDLL("libamdhip64.so")
K = 200
for flags, name in ((0, "default"), (0x40000000, "ReleaseToDevice"), (0x20000000, "DisableSystemFence")):
    evs = []

    def hstep():
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        e = [ctypes.c_void_p() for _ in range(3)]
        for x in e:
            assert hip.hipEventCreateWithFlags(ctypes.byref(x), ctypes.c_uint(flags)) == 0
        hip.hipEventRecord(e[0], st)
        out, ln = codec.encode(d_ref, d_pend, d_cnt, stride, chunked=True)
        hip.hipEventRecord(e[1], st)
        codec.decode(d_ref, out, ln, W, chunked=True, out=dec_buf)
        hip.hipEventRecord(e[2], st)
        evs.append(e)

    timed(hstep, f"hip events {name}")
    ms = ctypes.c_float()
    enc = dec = 0.0
    for e in evs:
        hip.hipEventElapsedTime(ctypes.byref(ms), e[0], e[1]); enc += ms.value
        hip.hipEventElapsedTime(ctypes.byref(ms), e[1], e[2]); dec += ms.value
        for x in e:
            hip.hipEventDestroy(x)
    print(f"   encode {enc / len(evs) * 1e3:.1f} us, decode {dec / len(evs) * 1e3:.1f} us", flush=True)
