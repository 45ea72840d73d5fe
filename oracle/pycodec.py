"""Independent pure-Python restatement of GGRS's input wire codec (TEST INFRASTRUCTURE; cross-checks
oracle/codec.c).  src/network/compression.rs:14-182 (delta_encode / delta_decode), bitfield-rle
0.2.1's run format (LEB128 header: odd -> (h >> 2) bytes of 0x00/0xFF by bit 1, even -> (h >> 1)
literal bytes), bincode 1.3 fixint framing of EncodedInputSequence."""
import struct

MAX_DECODED = 1 << 24


class CodecError(Exception):
    pass


def _varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


def rle_encode(buf):
    out, i, n = bytearray(), 0, len(buf)
    while i < n:
        j = i
        if buf[i] in (0x00, 0xFF):
            while j < n and buf[j] == buf[i]:
                j += 1
            out += _varint(((j - i) << 2) | (2 if buf[i] == 0xFF else 0) | 1)
        else:
            while j < n and buf[j] not in (0x00, 0xFF):
                j += 1
            out += _varint((j - i) << 1) + bytes(buf[i:j])
        i = j
    return bytes(out)


def rle_decode(buf):
    out, pos = bytearray(), 0
    while pos < len(buf):
        h, shift = 0, 0
        while True:
            if pos >= len(buf) or shift >= 64:
                raise CodecError("rle: truncated varint")
            b = buf[pos]
            pos += 1
            h |= (b & 0x7F) << shift
            shift += 7
            if not b & 0x80:
                break
        h &= (1 << 64) - 1
        ln = h >> 2 if h & 1 else h >> 1
        if len(out) + ln > MAX_DECODED:
            raise CodecError("rle: too long")
        if h & 1:
            out += (b"\xff" if h & 2 else b"\x00") * ln
        else:
            if len(buf) - pos < ln:
                raise CodecError("rle: truncated literal")
            out += buf[pos:pos + ln]
            pos += ln
    return bytes(out)


def encode(reference, inputs):
    sizes = None
    if not (all(len(x) == len(reference) for x in inputs) and len(reference) > 0):
        sizes, base = [], len(reference)
        for x in inputs:
            sizes.append(len(x) - base)
            base = len(x)
    enc, base = bytearray(), reference
    for x in inputs:
        enc += bytes(a ^ b for a, b in zip(base, x))
        if len(x) > len(base):
            enc += x[len(base):]
        base = x
    rle = rle_encode(bytes(enc))
    out = bytearray()
    if sizes is None:
        out.append(0)
    else:
        out.append(1)
        out += struct.pack("<Q", len(sizes)) + b"".join(struct.pack("<i", s) for s in sizes)
    out += struct.pack("<Q", len(rle)) + rle
    return bytes(out)


def decode(reference, data):
    """-> list of inputs; raises CodecError for every input the reference rejects."""
    pos = 0
    if len(data) < 1 or data[0] > 1:
        raise CodecError("bincode: tag")
    tag, pos = data[0], 1
    sizes_rel = None
    if tag == 1:
        if len(data) - pos < 8:
            raise CodecError("bincode: short")
        (n,) = struct.unpack_from("<Q", data, pos)
        pos += 8
        if n > (len(data) - pos) // 4:
            raise CodecError("bincode: short")
        sizes_rel = list(struct.unpack_from(f"<{n}i", data, pos))
        pos += 4 * n
    if len(data) - pos < 8:
        raise CodecError("bincode: short")
    (m,) = struct.unpack_from("<Q", data, pos)
    pos += 8
    if m > len(data) - pos:
        raise CodecError("bincode: short")
    enc = rle_decode(data[pos:pos + m])
    if sizes_rel is not None:
        sizes, base = [], len(reference)
        for r in sizes_rel:
            sz = ((base + r + 2 ** 31) % 2 ** 32) - 2 ** 31   # i32 arithmetic
            if sz < 0:
                raise CodecError("delta: negative size")
            sizes.append(sz)
            base = sz
    else:
        if len(reference) == 0:
            raise CodecError("delta: empty reference")
        sizes = [len(reference)] * (len(enc) // len(reference))
    if sum(sizes) != len(enc):
        raise CodecError("delta: size mismatch")
    out, pos, base = [], 0, reference
    for sz in sizes:
        chunk = bytearray(enc[pos:pos + sz])
        for i in range(min(sz, len(base))):
            chunk[i] ^= base[i]
        out.append(bytes(chunk))
        base = out[-1]
        pos += sz
    return out
