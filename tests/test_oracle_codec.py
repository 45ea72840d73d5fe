"""CPU tests of the input wire codec restatements (oracle/codec.c and the independent
oracle/pycodec.py), pinned by the reference's own tests in src/network/compression.rs:188-232:
test_encode_decode (:216-231), the encode_decode_round_trip property (:195-203) incl. its
recorded regression case (proptest-regressions/network/compression.txt: reference = [],
inputs = [[], []]) and decode_arbitrary_input_never_panics (:205-213)."""
import numpy as np
from hypothesis import example, given, settings, strategies as st

from oracle import oracle as O
from oracle import pycodec as PC

small_bytes = st.binary(min_size=0, max_size=32)


def test_encode_decode_reference_example():
    ref = bytes([0, 0, 0, 1])
    pend = [bytes(x) for x in ([0, 0, 1, 0], [0, 0, 1, 1], [0, 1, 0, 0], [0, 1, 0, 1], [0, 1, 1, 0])]
    enc = O.codec_encode(ref, pend)
    assert enc == PC.encode(ref, pend)
    assert O.codec_decode(ref, enc) == (0, pend)
    assert PC.decode(ref, enc) == pend


def test_regression_empty_reference_two_empty_inputs():
    enc = O.codec_encode(b"", [b"", b""])
    assert enc == PC.encode(b"", [b"", b""])
    # input_sizes = Some([0, 0]): tag 1, two sizes, no payload
    assert enc == bytes([1]) + (2).to_bytes(8, "little") + bytes(8) + (0).to_bytes(8, "little")
    assert O.codec_decode(b"", enc) == (0, [b"", b""])


@settings(max_examples=400, deadline=None)
@given(small_bytes, st.lists(small_bytes, min_size=0, max_size=32))
def test_round_trip_property(reference, inputs):
    enc = O.codec_encode(reference, inputs)
    assert enc == PC.encode(reference, inputs)
    assert O.codec_decode(reference, enc) == (0, inputs)
    assert PC.decode(reference, enc) == inputs


@settings(max_examples=400, deadline=None)
@given(st.binary(min_size=0, max_size=2048), st.binary(min_size=0, max_size=2048))
def test_decode_arbitrary_input_never_fails_hard(reference, data):
    rc, out = O.codec_decode(reference, data)
    try:
        want = PC.decode(reference, data)
        assert rc == 0 and out == want
    except PC.CodecError:
        assert rc < 0 and out is None


def test_rle_runs():
    buf = bytes([0] * 100 + [255] * 3 + [7, 8, 0, 9] + [255])
    enc = PC.rle_encode(buf)
    assert PC.rle_decode(enc) == buf
    # 100 zeros -> one compressed run (100 << 2 | 1 = 401 = varint 0x91 0x03)
    assert enc[:2] == bytes([0x91, 0x03])


def test_fixed_size_ex_game_stream():
    """ex_game inputs: one u8 per local player; a window of held keys compresses to a few bytes."""
    rng = np.random.default_rng(1)
    ref = bytes([3])
    pend = [bytes([3])] * 6 + [bytes([int(rng.integers(0, 16))]) for _ in range(4)]
    enc = O.codec_encode(ref, pend)
    assert enc[0] == 0 and O.codec_decode(ref, enc) == (0, pend)


CODEC_E_CAP = -4   # oracle/codec.c: decoded inputs exceed the caller's buffers
MAX_INPUTS = 1 << 16


@settings(max_examples=400, deadline=None)
# regression: tag byte zeroed -> fixed-size decode of a stream whose RLE yields > 2^16 inputs
@example(b"\x00", [b"\x00", b"N\x97~\xf9\x06\x0f0F\x00", b"\xf2\x9d ", b"\x88\xca\xce3\xea\xc6", b"\x00", b"e",
                   b"\x8d-\xd2Xi\xdd\x88\xd8\xfer", b"R\xe6Q\xc8\xbc", b"", b"", b"", b"", b""], [(0, 0)])
@given(small_bytes, st.lists(small_bytes, min_size=1, max_size=16), st.lists(st.tuples(st.integers(0, 4096), st.integers(0, 255)), min_size=1, max_size=4))
def test_mutated_packets_agree(reference, inputs, muts):
    """Valid packets with a few bytes overwritten reach the RLE and delta checks; both
    restatements accept or reject identically."""
    enc = bytearray(O.codec_encode(reference, inputs))
    for pos, val in muts:
        enc[pos % len(enc)] = val
    enc = bytes(enc)
    rc, out = O.codec_decode(reference, enc, max_inputs=MAX_INPUTS)
    try:
        want = PC.decode(reference, enc)
        if rc == CODEC_E_CAP:  # valid, but more inputs than the checker's output buffers hold
            assert len(want) > MAX_INPUTS
        else:
            assert rc == 0 and out == want
    except PC.CodecError:
        assert rc < 0 and rc != CODEC_E_CAP
