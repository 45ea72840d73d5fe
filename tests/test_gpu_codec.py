"""GPU parity of the batched input wire codec (ggrs_codec_encode / ggrs_codec_decode) against the
CPU restatement of src/network/compression.rs (oracle/codec.c): encoded packets byte-identical,
decode results and error codes identical, on random packets, ex_game-like input windows, the
reference's own test vector (compression.rs:216-231) and hostile bytes (:205-213)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")  # loads torch's HIP runtime before the engine library

pytestmark = pytest.mark.gpu


def batch(rng, N, W, B, held=False):
    ref = rng.integers(0, 256, (N, B), dtype=np.uint8)
    if held:  # ex_game-like: keys held over frames -> long zero runs in the XOR delta
        pend = np.repeat(rng.integers(0, 16, (N, 1, B), dtype=np.uint8), W, axis=1)
        flip = rng.random((N, W, B)) < 0.15
        pend = np.where(flip, rng.integers(0, 16, (N, W, B), dtype=np.uint8), pend).astype(np.uint8)
    else:
        pend = rng.integers(0, 256, (N, W, B), dtype=np.uint8)
        pend[rng.random((N, W, B)) < 0.3] = 0
        pend[rng.random((N, W, B)) < 0.1] = 255
    count = rng.integers(0, W + 1, N).astype(np.int32)
    return ref, pend, count


def gpu(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.fixture(params=["default", "staged", "direct"])
def kernels(request):
    """Every kernel form: default (lane-cooperative where W*B <= 64 and rows are whole dwords),
    thread-per-packet LDS-staged, and direct."""
    from ggrs_amd import codec
    codec.set_kernels(request.param)
    yield request.param
    codec.set_kernels("default")


# W*B: 8, 32 (lane-cooperative segments of 8 / 32 lanes), 132, 128 (thread-per-packet staged), 7
# (direct); then 16 (the bench shape), 64, 4, 12 (segments of 16 / 64 / 4 / 16 lanes)
@pytest.mark.parametrize("N,W,B,held", [(5000, 8, 1, True), (3000, 16, 2, False), (2000, 33, 4, False),
                                         (1000, 128, 1, True), (257, 1, 7, False), (4000, 8, 2, True),
                                         (3000, 16, 4, True), (2000, 4, 1, False), (2000, 12, 1, True),
                                         (999, 3, 4, False), (1500, 64, 1, True)])
def test_encode_matches_oracle_and_round_trips(oracle, kernels, N, W, B, held):
    from ggrs_amd import codec
    rng = np.random.default_rng(N + W + B)
    ref, pend, count = batch(rng, N, W, B, held)
    out, ln = codec.encode(gpu(ref), gpu(pend), gpu(count))
    out, ln = out.cpu().numpy(), ln.cpu().numpy()
    for p in range(N):
        want = oracle.codec_encode(ref[p].tobytes(), [pend[p, k].tobytes() for k in range(count[p])])
        assert ln[p] == len(want), p
        assert out[p, :ln[p]].tobytes() == want, p
    dec, cnt, st = codec.decode(gpu(ref), gpu(out), gpu(ln), max_inputs=W)
    dec, cnt, st = dec.cpu().numpy(), cnt.cpu().numpy(), st.cpu().numpy()
    assert (st == 0).all() and (cnt == count).all()
    for p in range(N):
        assert (dec[p, :count[p]] == pend[p, :count[p]]).all(), p


def test_reference_vector():
    from ggrs_amd import codec
    ref = np.array([[0, 0, 0, 1]], np.uint8)
    pend = np.array([[[0, 0, 1, 0], [0, 0, 1, 1], [0, 1, 0, 0], [0, 1, 0, 1], [0, 1, 1, 0]]], np.uint8)
    out, ln = codec.encode(gpu(ref), gpu(pend), gpu(np.array([5], np.int32)))
    dec, cnt, st = codec.decode(gpu(ref), out, ln, max_inputs=5)
    assert int(st[0]) == 0 and int(cnt[0]) == 5
    assert (dec.cpu().numpy() == pend).all()


@pytest.mark.parametrize("mode", ["mutated", "random", "truncated"])
def test_hostile_packets_match_oracle(oracle, kernels, mode):
    """Every packet the reference rejects is rejected with the same error class; every packet it
    accepts decodes identically (or is UNSUPPORTED when its inputs are not all B bytes)."""
    from ggrs_amd import codec
    rng = np.random.default_rng({"mutated": 1, "random": 2, "truncated": 3}[mode])
    N, W, B = 4000, 16, 2
    ref, pend, count = batch(rng, N, W, B)
    out, ln = codec.encode(gpu(ref), gpu(pend), gpu(count))
    pk, ln = out.cpu().numpy().copy(), ln.cpu().numpy().copy()
    if mode == "mutated":
        for p in range(N):
            for _ in range(int(rng.integers(1, 4))):
                pk[p, int(rng.integers(0, max(ln[p], 1)))] = rng.integers(0, 256)
    elif mode == "random":
        pk[:] = rng.integers(0, 256, pk.shape, dtype=np.uint8)
        ln = rng.integers(0, pk.shape[1] + 1, N).astype(np.int32)
        framed = (rng.random(N) < 0.7) & (ln >= 9)  # valid bincode framing, random runs inside
        pk[framed, 0] = 0
        for p in np.nonzero(framed)[0]:
            pk[p, 1:9] = np.frombuffer(int(ln[p] - 9).to_bytes(8, "little"), np.uint8)
    else:  # cut packets short and shrink the bincode length to match: runs end mid-way
        ln = (ln * rng.random(N)).astype(np.int32)
        for p in np.nonzero(ln >= 9)[0]:
            pk[p, 1:9] = np.frombuffer(int(ln[p] - 9).to_bytes(8, "little"), np.uint8)
    dec, cnt, st = codec.decode(gpu(ref), gpu(pk), gpu(ln), max_inputs=W)
    dec, cnt, st = dec.cpu().numpy(), cnt.cpu().numpy(), st.cpu().numpy()
    seen = set()
    for p in range(N):
        rc, want = oracle.codec_decode(ref[p].tobytes(), pk[p, :ln[p]].tobytes())
        seen.add(rc)
        if rc < 0:
            assert st[p] == rc, (p, st[p], rc)
        elif st[p] == 0:
            assert [dec[p, k].tobytes() for k in range(cnt[p])] == want, p
        else:
            assert st[p] in (codec.UNSUPPORTED, codec.E_CAP), (p, st[p])
            assert st[p] != codec.UNSUPPORTED or any(len(x) != B for x in want)
            assert st[p] != codec.E_CAP or len(want) > W
    assert len(seen) >= 2


@pytest.mark.parametrize("W,B", [(16, 2), (8, 1), (33, 4), (3, 7)])
def test_decode_writes_whole_rows(kernels, W, B):
    """Every kernel form writes each output row whole into a dirty buffer: the decoded inputs, zero
    past count, and an all-zero row for a rejected packet (the ABI's out needs no clearing)."""
    from ggrs_amd import codec
    rng = np.random.default_rng(W * 10 + B)
    N = 1000
    ref, pend, count = batch(rng, N, W, B)
    out, ln = codec.encode(gpu(ref), gpu(pend), gpu(count))
    ln = ln.cpu().numpy().copy()
    bad = rng.random(N) < 0.2
    ln[bad] = -1  # rejected: E_INVALID
    dirty = torch.full((N, W, B), 0xAB, dtype=torch.uint8, device="cuda")
    dec, cnt, st = codec.decode(gpu(ref), out, gpu(ln), max_inputs=W, out=dirty)
    assert dec.data_ptr() == dirty.data_ptr()
    dec, cnt, st = dec.cpu().numpy(), cnt.cpu().numpy(), st.cpu().numpy()
    for p in range(N):
        if bad[p]:
            assert st[p] != 0 and cnt[p] == 0 and (dec[p] == 0).all(), p
        else:
            assert st[p] == 0 and cnt[p] == count[p], p
            assert (dec[p, :count[p]] == pend[p, :count[p]]).all(), p
            assert (dec[p, count[p]:] == 0).all(), p


@pytest.mark.parametrize("W,B", [(8, 2), (16, 4), (33, 4), (1, 7)])
def test_encode_errors(oracle, kernels, W, B):
    """count outside 0..W -> E_INVALID; a stride too small for the packet -> E_CAP; every other
    packet of the batch still matches the oracle."""
    from ggrs_amd import codec
    rng = np.random.default_rng(W * 31 + B)
    N = 600
    ref, pend, count = batch(rng, N, W, B, False)
    count[::7] = -1
    count[3::11] = W + 1
    stride = 12 if (W * B) % 4 == 0 else 13  # a few bytes of runs fit, longer packets do not
    out, ln = codec.encode(gpu(ref), gpu(pend), gpu(count), stride=stride)
    out, ln = out.cpu().numpy(), ln.cpu().numpy()
    for p in range(N):
        if count[p] < 0 or count[p] > W:
            assert ln[p] == codec.E_INVALID, p
            continue
        want = oracle.codec_encode(ref[p].tobytes(), [pend[p, k].tobytes() for k in range(count[p])])
        if len(want) > stride:
            assert ln[p] == codec.E_CAP, p
        else:
            assert ln[p] == len(want) and out[p, :ln[p]].tobytes() == want, p


@pytest.mark.parametrize("N,W,B,held", [(5000, 8, 1, True), (3000, 16, 2, False), (4000, 8, 2, True),
                                         (3000, 8, 4, True), (2000, 12, 1, True), (777, 4, 1, False)])
def test_chunked_layout_matches_oracle(oracle, N, W, B, held):
    """The chunked layout (each 256-packet block's packets back to back, dword-padded): every
    packet's bytes at its chunk offset equal the oracle's encoding, and the chunked decode returns
    what the strided decode returns."""
    from ggrs_amd import codec
    rng = np.random.default_rng(N * 3 + W + B)
    ref, pend, count = batch(rng, N, W, B, held)
    out, ln = codec.encode(gpu(ref), gpu(pend), gpu(count), chunked=True)
    stride = out.shape[1]
    flat, lh = out.cpu().numpy().reshape(-1), ln.cpu().numpy()
    off = codec.chunk_offsets(lh, stride)
    for p in range(N):
        want = oracle.codec_encode(ref[p].tobytes(), [pend[p, k].tobytes() for k in range(count[p])])
        assert lh[p] == len(want), p
        assert flat[off[p]:off[p] + lh[p]].tobytes() == want, p
        pad = (-int(lh[p])) % 4
        assert not flat[off[p] + lh[p]:off[p] + lh[p] + pad].any(), p  # padding is zero
    dec, cnt, st = codec.decode(gpu(ref), out, ln, max_inputs=W, chunked=True)
    dec, cnt, st = dec.cpu().numpy(), cnt.cpu().numpy(), st.cpu().numpy()
    assert (st == 0).all() and (cnt == count).all()
    for p in range(N):
        assert (dec[p, :count[p]] == pend[p, :count[p]]).all(), p


@pytest.mark.parametrize("mode", ["mutated", "random", "truncated"])
@pytest.mark.parametrize("W,B", [(16, 2), (8, 1), (16, 4)])
def test_chunked_decode_hostile_lengths_match_strided(oracle, mode, W, B):
    """Lengths outside [1, stride] take no bytes in the chunked layout and give the strided decode's
    error codes; hostile packets at their chunk offsets -- mutated bytes, random runs inside valid
    bincode framing, packets cut short -- decode as the strided form of the same bytes (the chunked
    decode stages the block's packets in LDS from their packed offsets, the strided one whole rows)."""
    from ggrs_amd import codec
    rng = np.random.default_rng(77 + W + B + {"mutated": 0, "random": 1000, "truncated": 2000}[mode])
    N = 3000
    ref, pend, count = batch(rng, N, W, B)
    out, ln = codec.encode(gpu(ref), gpu(pend), gpu(count))  # strided
    pk, lh = out.cpu().numpy().copy(), ln.cpu().numpy().copy()
    stride = pk.shape[1]
    if mode == "mutated":
        for p in range(N):
            if rng.random() < 0.3:
                pk[p, int(rng.integers(0, max(lh[p], 1)))] = rng.integers(0, 256)
    elif mode == "random":
        pk[:] = rng.integers(0, 256, pk.shape, dtype=np.uint8)
        pk[:, 9:][rng.random((N, stride - 9)) < 0.5] &= 0x7F  # short varints: runs that parse
        lh = rng.integers(1, stride + 1, N).astype(np.int32)
        framed = (rng.random(N) < 0.8) & (lh >= 9)
        pk[framed, 0] = 0
        for p in np.nonzero(framed)[0]:
            pk[p, 1:9] = np.frombuffer(int(lh[p] - 9).to_bytes(8, "little"), np.uint8)
    else:
        lh = (lh * rng.random(N)).astype(np.int32)
        for p in np.nonzero(lh >= 9)[0]:
            pk[p, 1:9] = np.frombuffer(int(lh[p] - 9).to_bytes(8, "little"), np.uint8)
    bad = rng.random(N) < 0.1
    lh[bad] = rng.choice([-5, 0, stride + 4, 10 ** 6], int(bad.sum())).astype(np.int32)
    # the same packets in the chunked layout
    off = codec.chunk_offsets(lh, stride)
    flat = np.zeros(N * stride, np.uint8)
    for p in range(N):
        if 1 <= lh[p] <= stride:
            flat[off[p]:off[p] + lh[p]] = pk[p, :lh[p]]
    a = codec.decode(gpu(ref), gpu(pk), gpu(lh), max_inputs=W)
    b = codec.decode(gpu(ref), gpu(flat.reshape(N, stride)), gpu(lh), max_inputs=W, chunked=True)
    for x, y in zip(a, b):
        assert (x.cpu().numpy() == y.cpu().numpy()).all()
    assert (b[2].cpu().numpy()[bad] != 0).all()
