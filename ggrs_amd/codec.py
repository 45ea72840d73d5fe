"""Batched input wire codec over the C ABI (include/ggrs_amd.h, ggrs_codec_*): GGRS's
compression::encode / decode (src/network/compression.rs:14-182) for many packets per launch on
the GPU.  Buffers are torch tensors on the engine's device (torch is only the allocator); there
is no CPU path.

    enc = encode(ref, pending, count)            # ref [N][B] u8, pending [N][W][B] u8, count [N]
    packets, lengths = enc                       # [N][stride] u8, [N] i32 (length or error code)
    out, count, status = decode(ref, packets, lengths, max_inputs=W)
"""
import ctypes

from . import _lib

OK, E_BINCODE, E_RLE, E_DELTA, E_CAP, E_INVALID, UNSUPPORTED = 0, -1, -2, -3, -4, -5, -6

_bound = False


def _bind(L):
    global _bound
    if _bound:
        return
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    L.ggrs_codec_encode.argtypes = [vp, vp, vp, i64, i32, i32, vp, i32, vp, vp]
    L.ggrs_codec_decode.argtypes = [vp, vp, vp, i64, i32, i32, i32, vp, vp, vp, vp]
    L.ggrs_codec_encode_chunked.argtypes = [vp, vp, vp, i64, i32, i32, vp, i32, vp, vp]
    L.ggrs_codec_decode_chunked.argtypes = [vp, vp, vp, i64, i32, i32, i32, vp, vp, vp, vp]
    L.ggrs_codec_max_packet_bytes.argtypes = [i32, i32]
    L.ggrs_codec_max_packet_bytes.restype = i32
    L.ggrs_codec_set_direct.argtypes = [i32]
    _bound = True


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream(t):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def max_packet_bytes(input_bytes, max_inputs):
    L = _lib.lib()
    _bind(L)
    return L.ggrs_codec_max_packet_bytes(input_bytes, max_inputs)


def encode(ref, pending, count, stride=None, chunked=False):
    """ref [N][B], pending [N][W][B] (uint8, cuda), count [N] int32 -> (packets [N][stride] u8,
    lengths [N] int32: packet bytes, or a negative GGRS_CODEC_E_* code).  chunked: the packets of
    each block of 256 back to back, dword-padded (chunk_offsets locates them)."""
    import torch
    L = _lib.lib()
    _bind(L)
    N, W, B = pending.shape
    if ref.shape != (N, B) or count.shape != (N,):
        raise _lib.InvalidRequest(-1, "ref must be [N][B], count [N]")
    ref, pending = ref.contiguous(), pending.contiguous()
    count = count.to(torch.int32).contiguous()
    stride = stride or max_packet_bytes(B, W)
    out = torch.empty((N, stride), dtype=torch.uint8, device=pending.device)
    out_len = torch.empty(N, dtype=torch.int32, device=pending.device)
    fn = L.ggrs_codec_encode_chunked if chunked else L.ggrs_codec_encode
    _lib.check(fn(_p(ref), _p(pending), _p(count), N, B, W, _p(out), stride, _p(out_len), _stream(pending)))
    return out, out_len


def decode(ref, packets, lengths, max_inputs, chunked=False, out=None):
    """ref [N][B], packets [N][stride] u8, lengths [N] int32 -> (inputs [N][max_inputs][B] u8,
    count [N] int32, status [N] int32: 0 or a GGRS_CODEC_* code).  `out` (optional): a contiguous
    u8 tensor [N][max_inputs][B] on the packets' device to decode into; every row is written whole
    (slots past count and failed packets' rows are zero), so it needs no clearing."""
    import torch
    L = _lib.lib()
    _bind(L)
    N, B = ref.shape
    stride = packets.shape[1]
    ref, packets = ref.contiguous(), packets.contiguous()
    lengths = lengths.to(torch.int32).contiguous()
    if out is None:
        out = torch.empty((N, max_inputs, B), dtype=torch.uint8, device=packets.device)
    elif (tuple(out.shape) != (N, max_inputs, B) or out.dtype != torch.uint8 or not out.is_contiguous()
          or out.device != packets.device):
        raise ValueError(f"out must be a contiguous uint8 tensor of shape {(N, max_inputs, B)} on {packets.device}")
    cnt = torch.empty(N, dtype=torch.int32, device=packets.device)
    st = torch.empty(N, dtype=torch.int32, device=packets.device)
    fn = L.ggrs_codec_decode_chunked if chunked else L.ggrs_codec_decode
    _lib.check(fn(_p(ref), _p(packets), _p(lengths), N, stride, B, max_inputs, _p(out), _p(cnt), _p(st),
                  _stream(packets)))
    return out, cnt, st


def chunk_offsets(lengths, stride):
    """Byte offset of every packet in the chunked layout (numpy int64 [N]): block b = i // 256
    starts at 256 * b * stride; inside it the packets' lengths padded to 4 bytes, back to back (a
    length outside [1, stride] takes none)."""
    import numpy as np
    n = np.asarray(lengths, np.int64)
    cb = np.where((n >= 1) & (n <= stride), (n + 3) & ~3, 0)
    N = len(n)
    out = np.zeros(N, np.int64)
    for b0 in range(0, N, 256):
        c = cb[b0:b0 + 256]
        out[b0:b0 + 256] = 256 * (b0 // 256) * stride + np.concatenate([[0], np.cumsum(c)[:-1]])
    return out


KERNEL_FORMS = {"default": 0, "direct": 1, "staged": 2}


def set_direct(on):
    """Force the direct (unstaged) thread-per-packet kernels; False restores the default."""
    set_kernels("direct" if on else "default")


def set_kernels(form):
    """Kernel form for later calls: "default" (lane-cooperative where W*B <= 64, else LDS-staged),
    "direct" or "staged" (thread-per-packet forms)."""
    L = _lib.lib()
    _bind(L)
    _lib.check(L.ggrs_codec_set_direct(KERNEL_FORMS[form]))
