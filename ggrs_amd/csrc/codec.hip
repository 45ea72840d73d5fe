// codec.hip -- GGRS's input wire codec, batched: many packets encoded / decoded per launch, one
// thread per packet.
//
// Reference: src/network/compression.rs (encode :14-24, delta_encode :26-81, decode :83-95,
// delta_decode :97-182), called by UdpProtocol::send_pending_output (protocol.rs:450-480: the
// pending inputs against the last acked input) and on_input (:580-642: against the input before
// the packet's start frame).  Wire format per packet: bincode 1.3 fixint
// EncodedInputSequence { input_sizes: Option<Vec<i32>>, encoded_bytes: Vec<u8> } where
// encoded_bytes is bitfield-rle 0.2.1 over the XOR delta of each input against the previous one
// (the first against the reference).  Run format: LEB128 header h; h odd -> (h >> 2) bytes of
// 0xFF (h & 2) or 0x00; h even -> (h >> 1) literal bytes follow.  Encoder run choice: maximal runs
// of 0x00 / 0xFF are compressed, maximal stretches of other bytes literal (oracle/codec.c).
//
// The batched form covers what a GGRS peer sends: every input B bytes, the size of the non-empty
// reference (input_sizes = None).  Decode accepts every packet the reference accepts whose inputs
// are all B bytes (input_sizes None, or Some with every size B); a packet the reference rejects
// gets that error code, one it would decode into other sizes gets GGRS_CODEC_UNSUPPORTED.
//
// Layouts (device memory, row per packet):
//   encode in : ref [N][B], pending [N][W][B], count [N] (<= W)
//   encode out: packet bytes [N][stride], length [N] (GGRS_CODEC_E_CAP if stride is too small)
//   decode in : ref [N][B], packets [N][stride], length [N]
//   decode out: inputs [N][W][B], count [N], status [N]
#include <hip/hip_runtime.h>

#include <type_traits>

#include "common.h"

using namespace ggrs;

namespace {

constexpr int64_t kMaxDecoded = 1 << 24;  // oracle/codec.c CODEC_MAX_DECODED
int g_codec_mode = 0;  // ggrs_codec_set_direct: 0 default, 1 direct, 2 staged thread-per-packet

struct EncodeParams {
  const uint8_t* ref;
  const uint8_t* pending;
  const int32_t* count;
  uint8_t* out;
  int32_t* out_len;
  int64_t N;
  int32_t B, W, stride;
};

__device__ inline int varint_len(uint64_t v) {
  int n = 1;
  while (v >= 0x80) { v >>= 7; n++; }
  return n;
}

// Byte i of the XOR-delta stream of packet p: input k = i / B against input k-1 (or the reference).
struct DeltaStream {
  const uint8_t* ref;
  const uint8_t* in;
  int32_t B;
  __device__ inline uint8_t at(int64_t i) const {
    const int64_t k = i / B, b = i - k * B;
    const uint8_t base = k == 0 ? ref[b] : in[(k - 1) * B + b];
    return base ^ in[i];
  }
};

// One pass of bitfield-rle over the delta stream: emit == false only measures.
template <bool kEmit>
__device__ inline int64_t rle_pass(const DeltaStream& x, int64_t L, uint8_t* out) {
  int64_t pos = 0, i = 0;
  auto put_varint = [&](uint64_t v) {
    do {
      uint8_t b = v & 0x7f;
      v >>= 7;
      if (kEmit) out[pos] = b | (v ? 0x80 : 0);
      pos++;
    } while (v);
  };
  while (i < L) {
    const uint8_t c = x.at(i);
    int64_t j = i + 1;
    if (c == 0x00 || c == 0xFF) {
      while (j < L && x.at(j) == c) j++;
      put_varint(((uint64_t)(j - i) << 2) | (c == 0xFF ? 2u : 0u) | 1u);
    } else {
      while (j < L) {
        const uint8_t d = x.at(j);
        if (d == 0x00 || d == 0xFF) break;
        j++;
      }
      put_varint((uint64_t)(j - i) << 1);
      if (kEmit)
        for (int64_t k = i; k < j; k++) out[pos + (k - i)] = x.at(k);
      pos += j - i;
    }
    i = j;
  }
  return pos;
}

__global__ __launch_bounds__(256) void encode_kernel(EncodeParams p) {
  const int64_t pk = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (pk >= p.N) return;
  const int32_t n = p.count[pk];
  if (n < 0 || n > p.W) {
    p.out_len[pk] = GGRS_CODEC_E_INVALID;
    return;
  }
  const DeltaStream x{p.ref + pk * p.B, p.pending + pk * (int64_t)p.W * p.B, p.B};
  const int64_t L = (int64_t)n * p.B;
  const int64_t rle = rle_pass<false>(x, L, nullptr);
  const int64_t total = 1 + 8 + rle;
  if (total > p.stride) {
    p.out_len[pk] = GGRS_CODEC_E_CAP;
    return;
  }
  uint8_t* o = p.out + pk * (int64_t)p.stride;
  o[0] = 0;  // input_sizes: None (every input is the reference's size, compression.rs:27-35)
  for (int b = 0; b < 8; b++) o[1 + b] = (uint8_t)((uint64_t)rle >> (8 * b));
  rle_pass<true>(x, L, o + 9);
  p.out_len[pk] = (int32_t)total;
}

struct DecodeParams {
  const uint8_t* ref;
  const uint8_t* packets;
  const int32_t* len;
  uint8_t* out;
  int32_t* count;
  int32_t* status;
  int64_t N;
  int32_t B, W, stride;
};

__device__ inline bool get_varint(const uint8_t* in, int64_t n, int64_t& pos, uint64_t& v) {
  uint64_t r = 0;
  for (int shift = 0; shift < 64; shift += 7) {
    if (pos >= n) return false;
    const uint8_t b = in[pos++];
    r |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) {
      v = r;
      return true;
    }
  }
  return false;
}

__global__ __launch_bounds__(256) void decode_kernel(DecodeParams p) {
  const int64_t pk = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (pk >= p.N) return;
  uint8_t* const orow = p.out + pk * (int64_t)p.W * p.B;
  auto fail = [&](int32_t code) {
    for (int64_t b = 0; b < (int64_t)p.W * p.B; b++) orow[b] = 0;  // every form writes whole rows
    p.status[pk] = code;
    p.count[pk] = 0;
  };
  const int64_t len = p.len[pk];
  if (len < 0 || len > p.stride) return fail(GGRS_CODEC_E_INVALID);
  const uint8_t* d = p.packets + pk * (int64_t)p.stride;
  const int32_t B = p.B;
  // bincode::deserialize (compression.rs:88)
  int64_t pos = 0;
  if (len < 1 || d[0] > 1) return fail(GGRS_CODEC_E_BINCODE);
  const uint8_t tag = d[pos++];
  uint64_t n_sizes = 0;
  int64_t sizes_at = 0;
  if (tag == 1) {
    if (len - pos < 8) return fail(GGRS_CODEC_E_BINCODE);
    for (int b = 0; b < 8; b++) n_sizes |= (uint64_t)d[pos + b] << (8 * b);
    pos += 8;
    if (n_sizes > (uint64_t)(len - pos) / 4) return fail(GGRS_CODEC_E_BINCODE);
    sizes_at = pos;
    pos += 4 * (int64_t)n_sizes;
  }
  if (len - pos < 8) return fail(GGRS_CODEC_E_BINCODE);
  uint64_t m = 0;
  for (int b = 0; b < 8; b++) m |= (uint64_t)d[pos + b] << (8 * b);
  pos += 8;
  if (m > (uint64_t)(len - pos)) return fail(GGRS_CODEC_E_BINCODE);
  const uint8_t* rle = d + pos;
  // bitfield_rle::decode, measuring pass (:91)
  int64_t xl = 0;
  {
    int64_t q = 0;
    while (q < (int64_t)m) {
      uint64_t h;
      if (!get_varint(rle, (int64_t)m, q, h)) return fail(GGRS_CODEC_E_RLE);
      const uint64_t rl = (h & 1) ? h >> 2 : h >> 1;
      if (rl > (uint64_t)kMaxDecoded || (uint64_t)xl + rl > (uint64_t)kMaxDecoded) return fail(GGRS_CODEC_E_RLE);
      if (!(h & 1)) {
        if ((uint64_t)((int64_t)m - q) < rl) return fail(GGRS_CODEC_E_RLE);
        q += (int64_t)rl;
      }
      xl += (int64_t)rl;
    }
  }
  // delta_decode size checks (:103-154)
  int64_t count;
  bool all_b = true;
  if (tag == 1) {
    count = (int64_t)n_sizes;
    int64_t bs = B, sum = 0;
    for (int64_t k = 0; k < count; k++) {
      uint32_t u = 0;
      for (int b = 0; b < 4; b++) u |= (uint32_t)d[sizes_at + 4 * k + b] << (8 * b);
      const int64_t sz = (int64_t)(int32_t)((uint32_t)bs + u);  // i32 arithmetic (:118)
      if (sz < 0) return fail(GGRS_CODEC_E_DELTA);
      all_b &= sz == B;
      bs = sz;
      sum += sz;
      if (sum > xl) return fail(GGRS_CODEC_E_DELTA);
    }
    if (sum != xl) return fail(GGRS_CODEC_E_DELTA);
  } else {
    count = xl / B;
    if (count * B != xl) return fail(GGRS_CODEC_E_DELTA);
  }
  if (!all_b) return fail(GGRS_CODEC_UNSUPPORTED);
  if (count > p.W) return fail(GGRS_CODEC_E_CAP);
  // second pass: runs -> XOR against the previous decoded input (or the reference)
  uint8_t* o = p.out + pk * (int64_t)p.W * B;
  const uint8_t* r = p.ref + pk * B;
  int64_t q = 0, i = 0;
  auto emit = [&](uint8_t xb) {
    const int64_t k = i / B, b = i - k * B;
    const uint8_t base = k == 0 ? r[b] : o[(k - 1) * B + b];
    o[i++] = xb ^ base;
  };
  while (q < (int64_t)m) {
    uint64_t h;
    get_varint(rle, (int64_t)m, q, h);
    const int64_t rl = (int64_t)((h & 1) ? h >> 2 : h >> 1);
    if (h & 1) {
      const uint8_t fill = (h & 2) ? 0xFF : 0x00;
      for (int64_t k = 0; k < rl; k++) emit(fill);
    } else {
      for (int64_t k = 0; k < rl; k++) emit(rle[q + k]);
      q += rl;
    }
  }
  for (int64_t b = i; b < (int64_t)p.W * B; b++) o[b] = 0;  // the slots past count
  p.count[pk] = (int32_t)count;
  p.status[pk] = GGRS_CODEC_OK;
}

// ------------------------------------------------------------------------------------------
// LDS-staged forms (the default when rows are whole dwords): a workgroup's packets are contiguous
// in memory, so the whole block moves between HBM and LDS with coalesced dword loads and stores,
// and each thread's byte-serial RLE works out of LDS instead of issuing byte accesses to global
// memory.  LDS rows are padded to an odd number of dwords so that threads stepping through their
// own rows in lockstep spread over the banks.
__host__ __device__ inline int odd_dword_pitch(int bytes) {
  int dw = (bytes + 3) / 4;
  if ((dw & 1) == 0) dw += 1;
  return dw * 4;
}

// rows x row_bytes contiguous bytes at src (dword aligned, row_bytes % 4 == 0) -> LDS rows of
// `pitch` bytes, and back.
__device__ inline void block_to_lds(uint8_t* lds, int pitch, const uint8_t* src, int rows, int row_bytes) {
  const int dpr = row_bytes / 4, total = rows * dpr;
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
  for (int q = threadIdx.x; q < total; q += blockDim.x) {
    const int r = q / dpr, c = q - r * dpr;
    reinterpret_cast<uint32_t*>(lds + r * pitch)[c] = s32[q];
  }
}
__device__ inline void lds_to_block(uint8_t* dst, const uint8_t* lds, int pitch, int rows, int row_bytes) {
  const int dpr = row_bytes / 4, total = rows * dpr;
  uint32_t* d32 = reinterpret_cast<uint32_t*>(dst);
  for (int q = threadIdx.x; q < total; q += blockDim.x) {
    const int r = q / dpr, c = q - r * dpr;
    d32[q] = reinterpret_cast<const uint32_t*>(lds + r * pitch)[c];
  }
}

__global__ __launch_bounds__(256) void encode_lds_kernel(EncodeParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int T = blockDim.x, B = p.B, W = p.W, stride = p.stride;
  const int in_pitch = odd_dword_pitch(W * B), out_pitch = odd_dword_pitch(stride);
  uint8_t* l_in = smem;                                  // [T][in_pitch]
  uint8_t* l_out = l_in + T * in_pitch;                  // [T][out_pitch]
  uint8_t* l_ref = l_out + T * out_pitch;                // [T][B]
  const int64_t pk0 = (int64_t)blockIdx.x * T;
  const int np = (int)((p.N - pk0) < T ? (p.N - pk0) : T);
  block_to_lds(l_in, in_pitch, p.pending + pk0 * W * B, np, W * B);
  for (int q = threadIdx.x; q < np * B; q += T) l_ref[q] = p.ref[pk0 * B + q];
  __syncthreads();
  const int t = threadIdx.x;
  if (t < np) {
    const int32_t n = p.count[pk0 + t];
    uint8_t* o = l_out + t * out_pitch;
    const uint8_t* in = l_in + t * in_pitch;
    const uint8_t* rf = l_ref + t * B;
    int32_t total = GGRS_CODEC_E_INVALID;
    if (n >= 0 && n <= W) {
      const int L = n * B;
      auto x = [&](int i) -> uint8_t { return (i < B ? rf[i] : in[i - B]) ^ in[i]; };
      // pass 1: RLE length
      int rle = 0;
      for (int i = 0; i < L;) {
        const uint8_t c = x(i);
        int j = i + 1;
        if (c == 0x00 || c == 0xFF) {
          while (j < L && x(j) == c) j++;
          rle += varint_len(((uint64_t)(j - i) << 2) | 1u);
        } else {
          while (j < L) {
            const uint8_t d = x(j);
            if (d == 0x00 || d == 0xFF) break;
            j++;
          }
          rle += varint_len((uint64_t)(j - i) << 1) + (j - i);
        }
        i = j;
      }
      total = 9 + rle;
      if (total > stride) {
        total = GGRS_CODEC_E_CAP;
      } else {
        o[0] = 0;
        for (int b = 0; b < 8; b++) o[1 + b] = (uint8_t)((uint64_t)rle >> (8 * b));
        int pos = 9;
        auto put_varint = [&](uint64_t v) {
          do {
            const uint8_t b = v & 0x7f;
            v >>= 7;
            o[pos++] = b | (v ? 0x80 : 0);
          } while (v);
        };
        for (int i = 0; i < L;) {
          const uint8_t c = x(i);
          int j = i + 1;
          if (c == 0x00 || c == 0xFF) {
            while (j < L && x(j) == c) j++;
            put_varint(((uint64_t)(j - i) << 2) | (c == 0xFF ? 2u : 0u) | 1u);
          } else {
            while (j < L) {
              const uint8_t d = x(j);
              if (d == 0x00 || d == 0xFF) break;
              j++;
            }
            put_varint((uint64_t)(j - i) << 1);
            for (int k = i; k < j; k++) o[pos++] = x(k);
          }
          i = j;
        }
        for (; pos < stride; pos++) o[pos] = 0;  // the row is stored whole
      }
    }
    if (total < 0)
      for (int b = 0; b < stride; b++) o[b] = 0;
    p.out_len[pk0 + t] = total;
  }
  __syncthreads();
  lds_to_block(p.out + pk0 * stride, l_out, out_pitch, np, stride);
}

__global__ __launch_bounds__(256) void decode_lds_kernel(DecodeParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int T = blockDim.x, B = p.B, W = p.W, stride = p.stride;
  const int in_pitch = odd_dword_pitch(stride), out_pitch = odd_dword_pitch(W * B);
  uint8_t* l_in = smem;                                  // [T][in_pitch] packets
  uint8_t* l_out = l_in + T * in_pitch;                  // [T][out_pitch] decoded inputs
  uint8_t* l_ref = l_out + T * out_pitch;                // [T][B]
  const int64_t pk0 = (int64_t)blockIdx.x * T;
  const int np = (int)((p.N - pk0) < T ? (p.N - pk0) : T);
  block_to_lds(l_in, in_pitch, p.packets + pk0 * stride, np, stride);
  for (int q = threadIdx.x; q < np * B; q += T) l_ref[q] = p.ref[pk0 * B + q];
  __syncthreads();
  const int t = threadIdx.x;
  if (t < np) {
    const int64_t pk = pk0 + t;
    const uint8_t* d = l_in + t * in_pitch;
    uint8_t* o = l_out + t * out_pitch;
    const uint8_t* rf = l_ref + t * B;
    int32_t status = GGRS_CODEC_OK, count = 0;
    const int64_t len = p.len[pk];
    // the same checks, in the same order, as decode_kernel (compression.rs:83-182)
    do {
      if (len < 0 || len > stride) { status = GGRS_CODEC_E_INVALID; break; }
      int64_t pos = 0;
      if (len < 1 || d[0] > 1) { status = GGRS_CODEC_E_BINCODE; break; }
      const uint8_t tag = d[pos++];
      uint64_t n_sizes = 0;
      int64_t sizes_at = 0;
      if (tag == 1) {
        if (len - pos < 8) { status = GGRS_CODEC_E_BINCODE; break; }
        for (int b = 0; b < 8; b++) n_sizes |= (uint64_t)d[pos + b] << (8 * b);
        pos += 8;
        if (n_sizes > (uint64_t)(len - pos) / 4) { status = GGRS_CODEC_E_BINCODE; break; }
        sizes_at = pos;
        pos += 4 * (int64_t)n_sizes;
      }
      if (len - pos < 8) { status = GGRS_CODEC_E_BINCODE; break; }
      uint64_t m = 0;
      for (int b = 0; b < 8; b++) m |= (uint64_t)d[pos + b] << (8 * b);
      pos += 8;
      if (m > (uint64_t)(len - pos)) { status = GGRS_CODEC_E_BINCODE; break; }
      const uint8_t* rle = d + pos;
      int64_t xl = 0;
      {
        int64_t q = 0;
        bool bad = false;
        while (q < (int64_t)m) {
          uint64_t h;
          if (!get_varint(rle, (int64_t)m, q, h)) { bad = true; break; }
          const uint64_t rl = (h & 1) ? h >> 2 : h >> 1;
          if (rl > (uint64_t)kMaxDecoded || (uint64_t)xl + rl > (uint64_t)kMaxDecoded) { bad = true; break; }
          if (!(h & 1)) {
            if ((uint64_t)((int64_t)m - q) < rl) { bad = true; break; }
            q += (int64_t)rl;
          }
          xl += (int64_t)rl;
        }
        if (bad) { status = GGRS_CODEC_E_RLE; break; }
      }
      int64_t cnt;
      bool all_b = true;
      if (tag == 1) {
        cnt = (int64_t)n_sizes;
        int64_t bs = B, sum = 0;
        bool bad = false;
        for (int64_t k = 0; k < cnt; k++) {
          uint32_t u = 0;
          for (int b = 0; b < 4; b++) u |= (uint32_t)d[sizes_at + 4 * k + b] << (8 * b);
          const int64_t sz = (int64_t)(int32_t)((uint32_t)bs + u);
          if (sz < 0) { bad = true; break; }
          all_b &= sz == B;
          bs = sz;
          sum += sz;
          if (sum > xl) { bad = true; break; }
        }
        if (bad || sum != xl) { status = GGRS_CODEC_E_DELTA; break; }
      } else {
        cnt = xl / B;
        if (cnt * B != xl) { status = GGRS_CODEC_E_DELTA; break; }
      }
      if (!all_b) { status = GGRS_CODEC_UNSUPPORTED; break; }
      if (cnt > W) { status = GGRS_CODEC_E_CAP; break; }
      int64_t q = 0;
      int i = 0;
      auto emit = [&](uint8_t xb) {
        const uint8_t base = i < B ? rf[i] : o[i - B];
        o[i] = xb ^ base;
        i++;
      };
      while (q < (int64_t)m) {
        uint64_t h;
        get_varint(rle, (int64_t)m, q, h);
        const int64_t rl = (int64_t)((h & 1) ? h >> 2 : h >> 1);
        if (h & 1) {
          const uint8_t fill = (h & 2) ? 0xFF : 0x00;
          for (int64_t k = 0; k < rl; k++) emit(fill);
        } else {
          for (int64_t k = 0; k < rl; k++) emit(rle[q + k]);
          q += rl;
        }
      }
      count = (int32_t)cnt;
    } while (false);
    for (int b = status == GGRS_CODEC_OK ? count * B : 0; b < W * B; b++) o[b] = 0;
    p.count[pk] = status == GGRS_CODEC_OK ? count : 0;
    p.status[pk] = status;
  }
  __syncthreads();
  lds_to_block(p.out + pk0 * (int64_t)W * B, l_out, out_pitch, np, W * B);
}

// ------------------------------------------------------------------------------------------
// Run-level forms (the default for input_bytes 1, 2 or 4 and W*B <= 64 whole dwords): still one
// thread per packet, but the delta stream lives in registers as NDW dwords and the RLE works
// run by run instead of byte by byte:
//   encode: the XOR delta is formed a dword at a time (v_alignbyte for the B-byte shift), bytes
//           equal to 0x00 / 0xFF become two 64-bit masks (SWAR zero-byte test), run starts are
//           the class changes of those masks, and each run is one header plus, for a literal
//           stretch, a byte copy out of an LDS scratch row;
//   decode: the packet is validated by the same checks in the same order as the other forms,
//           the runs are expanded into an LDS scratch row, and the delta chain (input k XOR input
//           k-1) is a prefix XOR of stride B done on whole dwords in registers.
// Rows move between HBM and LDS whole (block_to_lds / lds_to_block), as in the staged forms.

// one bit per byte of v that is zero (bit k for byte k)
__device__ inline uint32_t zero_byte_bits(uint32_t v) {
  const uint32_t t = ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v) & 0x80808080u;
  return ((t >> 7) * 0x00204081u) >> 21 & 0xFu;
}

__device__ inline uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t shift) {
  return __builtin_amdgcn_alignbyte(hi, lo, shift);
}

// bincode + bitfield-rle validation of one packet (compression.rs:83-154), the checks of
// decode_kernel in the same order.  On GGRS_CODEC_OK: *cnt inputs, the RLE stream at d + *rle_at
// with *m bytes.
__device__ inline int32_t validate_packet(const uint8_t* d, int64_t len, int stride, int B, int W, int64_t* cnt_out,
                                          uint64_t* m_out, int64_t* rle_at) {
  if (len < 0 || len > stride) return GGRS_CODEC_E_INVALID;
  int64_t pos = 0;
  if (len < 1 || d[0] > 1) return GGRS_CODEC_E_BINCODE;
  const uint8_t tag = d[pos++];
  uint64_t n_sizes = 0;
  int64_t sizes_at = 0;
  if (tag == 1) {
    if (len - pos < 8) return GGRS_CODEC_E_BINCODE;
    for (int b = 0; b < 8; b++) n_sizes |= (uint64_t)d[pos + b] << (8 * b);
    pos += 8;
    if (n_sizes > (uint64_t)(len - pos) / 4) return GGRS_CODEC_E_BINCODE;
    sizes_at = pos;
    pos += 4 * (int64_t)n_sizes;
  }
  if (len - pos < 8) return GGRS_CODEC_E_BINCODE;
  uint64_t m = 0;
  for (int b = 0; b < 8; b++) m |= (uint64_t)d[pos + b] << (8 * b);
  pos += 8;
  if (m > (uint64_t)(len - pos)) return GGRS_CODEC_E_BINCODE;
  const uint8_t* rle = d + pos;
  int64_t xl = 0;
  for (int64_t q = 0; q < (int64_t)m;) {
    uint64_t h;
    if (!get_varint(rle, (int64_t)m, q, h)) return GGRS_CODEC_E_RLE;
    const uint64_t rl = (h & 1) ? h >> 2 : h >> 1;
    if (rl > (uint64_t)kMaxDecoded || (uint64_t)xl + rl > (uint64_t)kMaxDecoded) return GGRS_CODEC_E_RLE;
    if (!(h & 1)) {
      if ((uint64_t)((int64_t)m - q) < rl) return GGRS_CODEC_E_RLE;
      q += (int64_t)rl;
    }
    xl += (int64_t)rl;
  }
  int64_t cnt;
  bool all_b = true;
  if (tag == 1) {
    cnt = (int64_t)n_sizes;
    int64_t bs = B, sum = 0;
    for (int64_t k = 0; k < cnt; k++) {
      uint32_t u = 0;
      for (int b = 0; b < 4; b++) u |= (uint32_t)d[sizes_at + 4 * k + b] << (8 * b);
      const int64_t sz = (int64_t)(int32_t)((uint32_t)bs + u);
      if (sz < 0) return GGRS_CODEC_E_DELTA;
      all_b &= sz == B;
      bs = sz;
      sum += sz;
      if (sum > xl) return GGRS_CODEC_E_DELTA;
    }
    if (sum != xl) return GGRS_CODEC_E_DELTA;
  } else {
    cnt = xl / B;
    if (cnt * B != xl) return GGRS_CODEC_E_DELTA;
  }
  if (!all_b) return GGRS_CODEC_UNSUPPORTED;
  if (cnt > W) return GGRS_CODEC_E_CAP;
  *cnt_out = cnt;
  *m_out = m;
  *rle_at = pos;
  return GGRS_CODEC_OK;
}

// row pitches of the run-level forms: rows long enough for any run layout of <= 4*NDW bytes
// (alternating one-byte runs: 9 + 3 * 4 * NDW), so a packet too long for the stride is measured
// in its own row and then reported as GGRS_CODEC_E_CAP
__host__ __device__ inline int swar_out_pitch(int stride, int ndw) {
  return odd_dword_pitch(stride > 9 + 12 * ndw ? stride : 9 + 12 * ndw);
}

// the chunked encode compacts its packets in place of the output rows when a row fits in 16 dwords
__host__ __device__ constexpr bool encode_in_place(int ndw) { return (9 + 12 * ndw + 3) / 4 <= 16; }

// Chunked packet layout (ggrs_codec_encode_chunked / _decode_chunked): the packets of the 256-packet
// block b lie back to back from byte b * 256 * stride, each padded to whole dwords (a packet whose
// length is outside [1, stride] -- an error code -- takes no bytes), so a block's packets are one
// contiguous run of exactly their bytes: encode writes and decode reads the packets' own bytes with
// coalesced dword copies, instead of whole stride-byte rows (a received datagram buffer holds the
// packets back to back as well).  The byte offsets follow from the lengths by a block-wide scan.
__device__ inline int chunk_bytes(int64_t len, int stride) {
  return (len >= 1 && len <= stride) ? (int)((len + 3) & ~3ll) : 0;
}
// exclusive prefix sum over the block (blockDim.x <= 1024, a multiple of 64); *total = the sum
__device__ inline int block_excl_scan(int v, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  int base = 0, tot = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); w++) {
    const int sw = wsum[w];
    base += w < wid ? sw : 0;
    tot += sw;
  }
  *total = tot;
  return base + x - v;
}

template <int B, int NDW, bool kChunked>
__global__ __launch_bounds__(256) void encode_swar_kernel(EncodeParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int T = blockDim.x, W = p.W, WB = W * B, stride = p.stride;
  const int out_pitch = swar_out_pitch(stride, NDW), x_pitch = odd_dword_pitch(4 * NDW);
  uint8_t* l_out = smem;                    // [T][out_pitch]
  uint8_t* l_x = l_out + T * out_pitch;     // [T][x_pitch] delta bytes, for literal copies
  uint8_t* l_chunk = l_x + T * x_pitch;     // kChunked, NDW > 4: [T * stride] the block's packets back to back
  const int64_t pk0 = (int64_t)blockIdx.x * T;
  const int np = (int)((p.N - pk0) < T ? (p.N - pk0) : T);
  for (int q = threadIdx.x; q < np * out_pitch / 4; q += T) reinterpret_cast<uint32_t*>(l_out)[q] = 0;
  const int t = threadIdx.x;
  const int64_t pk = pk0 + t;
  uint32_t cw[NDW], xw[NDW];
  int32_t n = 0;
  int32_t code = 0;  // the packet's length or error code
  uint32_t rw = 0;
  if (t < np) {
    n = p.count[pk];
    const uint32_t* src = reinterpret_cast<const uint32_t*>(p.pending + pk * WB);
#pragma unroll
    for (int k = 0; k < NDW; k++) cw[k] = 4 * k < WB ? src[k] : 0u;
#pragma unroll
    for (int b = 0; b < B; b++) rw |= (uint32_t)p.ref[pk * B + b] << (8 * b);
  }
  // delta stream: input k XOR input k-1 (the first against the reference), a dword at a time
#pragma unroll
  for (int k = 0; k < NDW; k++) {
    uint32_t prev;
    if constexpr (B == 4) prev = k == 0 ? rw : cw[k - 1];
    else prev = alignbyte(cw[k], k == 0 ? rw << (8 * (4 - B)) : cw[k - 1], 4 - B);
    xw[k] = cw[k] ^ prev;
  }
  __syncthreads();  // output rows zeroed
  if (t < np) {
    if (n < 0 || n > W) {
      code = GGRS_CODEC_E_INVALID;
    } else {
      const int L = n * B;
      // byte-class masks, one bit per delta byte: 32-bit when the stream has at most 32 bytes
      using Mk = typename std::conditional<(4 * NDW <= 32), uint32_t, uint64_t>::type;
      constexpr int kMb = 8 * (int)sizeof(Mk);
      auto ctzm = [](Mk v) -> int {
        if constexpr (sizeof(Mk) == 4) return (int)__builtin_ctz(v);
        else return (int)__builtin_ctzll(v);
      };
      Mk zm = 0, fm = 0;
      uint32_t* xrow = reinterpret_cast<uint32_t*>(l_x + t * x_pitch);
#pragma unroll
      for (int k = 0; k < NDW; k++) {
        zm |= (Mk)zero_byte_bits(xw[k]) << (4 * k);
        fm |= (Mk)zero_byte_bits(~xw[k]) << (4 * k);
        xrow[k] = xw[k];
      }
      const Mk valid = L >= kMb ? ~(Mk)0 : (((Mk)1 << L) - 1);
      zm &= valid;
      fm &= valid;
      // a run starts where the class (0x00 / 0xFF / literal) changes
      Mk starts = ((zm ^ (zm << 1)) | (fm ^ (fm << 1)) | (Mk)1) & valid;
      uint8_t* o = l_out + t * out_pitch;
      const uint8_t* xb = l_x + t * x_pitch;
      int pos = 9;
      while (starts) {
        const int i = ctzm(starts);
        starts &= starts - 1;
        const int nx = starts ? ctzm(starts) : L;
        const uint32_t len = (uint32_t)(nx - i);
        const bool fill = ((zm | fm) >> i) & 1;
        const uint32_t h = fill ? (len << 2) | (uint32_t)((fm >> i) & 1) << 1 | 1u : len << 1;  // < 2^14
        if constexpr (4 * NDW <= 31) {  // runs of <= 31 bytes: every header is one LEB128 byte
          o[pos++] = (uint8_t)h;
        } else {
          o[pos++] = (uint8_t)((h & 0x7fu) | (h >= 0x80u ? 0x80u : 0u));
          if (h >= 0x80u) o[pos++] = (uint8_t)(h >> 7);
        }
        if (!fill) {  // (a literal run has >= 1 byte; most have exactly one: no loop for them)
          o[pos++] = xb[i];
          for (int q = i + 1; q < nx; q++) o[pos++] = xb[q];
        }
      }
      const int rle = pos - 9;
      code = pos > stride ? GGRS_CODEC_E_CAP : pos;
      if (code > 0) {
        // input_sizes: None (byte 0), then the u64 length of encoded_bytes (bytes 1..8): the row
        // was zeroed and rle < 2^24, so one dword store (the row starts dword-aligned)
        *reinterpret_cast<uint32_t*>(o) = (uint32_t)rle << 8;
      } else {
        for (int q = 0; q < pos; q++) o[q] = 0;  // an error row is stored as zeros
      }
    }
    p.out_len[pk] = code;
  }
  if constexpr (kChunked && encode_in_place(NDW)) {
    // the block's packets compacted in place of the output rows (a packet's chunk offset is at most
    // its row's): no staging area, so twice the blocks per CU.  A row has at most kRowDw dwords.
    constexpr int kRowDw = (9 + 12 * NDW + 3) / 4;
    int* wsum = reinterpret_cast<int*>(l_x);  // the delta rows, no longer read after this barrier
    __syncthreads();
    int total;
    const int cb = t < np ? chunk_bytes(code, stride) : 0;
    const int off = block_excl_scan(cb, wsum, &total);  // (its barrier also orders the row writes)
    const uint32_t* row = reinterpret_cast<const uint32_t*>(l_out + t * out_pitch);
    uint32_t rr[kRowDw];
#pragma unroll
    for (int k = 0; k < kRowDw; k++) rr[k] = 4 * k < cb ? row[k] : 0u;
    __syncthreads();
    uint32_t* dst = reinterpret_cast<uint32_t*>(l_out + off);
#pragma unroll
    for (int k = 0; k < kRowDw; k++)
      if (4 * k < cb) dst[k] = rr[k];
    __syncthreads();
    uint32_t* out32 = reinterpret_cast<uint32_t*>(p.out + pk0 * stride);
    const uint32_t* c32 = reinterpret_cast<const uint32_t*>(l_out);
    for (int q = t; q < total / 4; q += T) out32[q] = c32[q];
  } else if constexpr (kChunked) {
    __shared__ int wsum[4];
    int total;
    const int cb = t < np ? chunk_bytes(code, stride) : 0;
    const int off = block_excl_scan(cb, wsum, &total);  // (its barrier also orders the row writes)
    const uint32_t* row = reinterpret_cast<const uint32_t*>(l_out + t * out_pitch);
    uint32_t* dst = reinterpret_cast<uint32_t*>(l_chunk + off);
    for (int k = 0; k < cb / 4; k++) dst[k] = row[k];
    __syncthreads();
    uint32_t* out32 = reinterpret_cast<uint32_t*>(p.out + pk0 * stride);
    const uint32_t* c32 = reinterpret_cast<const uint32_t*>(l_chunk);
    for (int q = t; q < total / 4; q += T) out32[q] = c32[q];
  } else {
    __syncthreads();
    lds_to_block(p.out + pk0 * stride, l_out, out_pitch, np, stride);
  }
}

template <int B, int NDW, bool kChunked>
__global__ __launch_bounds__(256) void decode_swar_kernel(DecodeParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int T = blockDim.x, W = p.W, WB = W * B, stride = p.stride;
  const int in_pitch = odd_dword_pitch(stride), x_pitch = odd_dword_pitch(4 * NDW);
  uint8_t* l_in = smem;                     // [T][in_pitch] packets
  uint8_t* l_x = l_in + T * in_pitch;       // [T][x_pitch] expanded runs, then (in place) the decoded inputs
  const int64_t pk0 = (int64_t)blockIdx.x * T;
  const int np = (int)((p.N - pk0) < T ? (p.N - pk0) : T);
  const int t = threadIdx.x;
  // the packet's length and reference input, read first: their memory latency beside the packet
  // copy's instead of after it
  int64_t len = 0;
  uint32_t rw = 0;
  if (t < np) {
    len = p.len[pk0 + t];
    const uint8_t* rp = p.ref + (pk0 + t) * B;  // (byte loads: the caller's pointer may be unaligned)
#pragma unroll
    for (int b = 0; b < B; b++) rw |= (uint32_t)rp[b] << (8 * b);
  }
  int d_off = t * in_pitch;
  if constexpr (kChunked) {  // the block's packets back to back: one coalesced copy of their bytes
    __shared__ int wsum[4];
    int total;
    const int cb = t < np ? chunk_bytes(len, stride) : 0;
    d_off = block_excl_scan(cb, wsum, &total);
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(p.packets + pk0 * stride);
    for (int q = t; q < total / 4; q += T) reinterpret_cast<uint32_t*>(l_in)[q] = s32[q];
  } else {
    block_to_lds(l_in, in_pitch, p.packets + pk0 * stride, np, stride);
  }
  __syncthreads();
  if (t < np) {
    const int64_t pk = pk0 + t;
    const uint8_t* d = l_in + d_off;
    constexpr int kCap = 4 * NDW;  // scratch bytes: any valid packet expands to <= W * B of them
    uint8_t* xb = l_x + t * x_pitch;
    uint32_t* xr32 = reinterpret_cast<uint32_t*>(xb);
#pragma unroll
    for (int k = 0; k < NDW; k++) xr32[k] = 0;  // 0x00 runs need no writes
    int64_t cnt = 0;
    int32_t status = GGRS_CODEC_OK;
    // one bit per scratch byte inside a 0xFF run (32-bit when the scratch row has at most 32 bytes)
    using Mf = typename std::conditional<(kCap <= 32), uint32_t, uint64_t>::type;
    constexpr int kFb = 8 * (int)sizeof(Mf);
    Mf ffm = 0;
    if (len < 0 || len > stride || len < 1 || d[0] != 0) {
      // a length outside the row, or input_sizes = Some(..) (or a bad tag): the general checks
      // (validate_packet, the same order as decode_kernel), then the runs are expanded
      int64_t rle_at = 0;
      uint64_t m = 0;
      status = validate_packet(d, len, stride, B, W, &cnt, &m, &rle_at);
      if (status == GGRS_CODEC_OK) {
        const uint8_t* rle = d + rle_at;
        int at = 0;
        for (int64_t q = 0; q < (int64_t)m;) {
          uint64_t h;
          get_varint(rle, (int64_t)m, q, h);
          const int rl = (int)((h & 1) ? h >> 2 : h >> 1);
          if (h & 1) {
            if (h & 2)
              for (int k = 0; k < rl; k++) xb[at + k] = 0xFF;
          } else {
            for (int k = 0; k < rl; k++) xb[at + k] = rle[q + k];
            q += rl;
          }
          at += rl;
        }
      }
    } else {
      // input_sizes = None, the packet GGRS sends: the checks of decode_kernel in the same order,
      // with the runs expanded during the measuring pass (bytes past kCap are never kept: such a
      // packet fails with E_CAP or E_DELTA below)
      const uint32_t* dw = reinterpret_cast<const uint32_t*>(d);
      if (len - 1 < 8) {
        status = GGRS_CODEC_E_BINCODE;
      } else {
        const uint32_t w0 = dw[0], w1 = dw[1], w2 = dw[2];
        const uint64_t m = (uint64_t)alignbyte(w1, w0, 1) | (uint64_t)alignbyte(w2, w1, 1) << 32;
        if (m > (uint64_t)(len - 9)) {
          status = GGRS_CODEC_E_BINCODE;
        } else {
          const uint8_t* rle = d + 9;
          const int mm = (int)m;  // <= len - 9 < stride
          int q = 0, xl = 0;      // xl <= kMaxDecoded
          // one-byte headers (every run of <= 31 fill / 63 literal bytes), the loop left only through
          // its condition (a break per error costs every iteration exec-mask bookkeeping); a multi-byte
          // header sends the packet to the general loop below, from the start
          bool multi = false;
          while (q < mm) {
            const uint32_t h = rle[q];
            const bool one = h < 0x80u, lit = !(h & 1u);
            const int rl = (int)(lit ? (h >> 1) & 0x3fu : (h >> 2) & 0x1fu);
            const bool over = one && lit && mm - (q + 1) < rl;
            if (one && !over) {
              const bool fits = xl + rl <= kCap;
              if (lit) {
                if (fits && rl > 0) {  // (most literal runs are one byte: no loop for them)
                  xb[xl] = rle[q + 1];
                  for (int k = 1; k < rl; k++) xb[xl + k] = rle[q + 1 + k];
                }
              } else if ((h & 2) && fits && rl > 0) {
                ffm |= (((Mf)1 << rl) - 1) << xl;  // 0xFF bytes, expanded below (rl <= 31, xl + rl <= kCap)
              }
            }
            if (over) status = GGRS_CODEC_E_RLE;
            multi |= !one;
            xl += rl;
            q = (!one || over) ? mm : q + 1 + (lit ? rl : 0);
          }
          if (multi) {
            q = 0;
            xl = 0;
            ffm = 0;
          }
          while (multi && q < mm) {
            uint32_t h = rle[q];
            int rl;
            if (h < 0x80u) {
              q++;
              rl = (int)((h & 1) ? h >> 2 : h >> 1);
              if (xl + rl > kMaxDecoded) { status = GGRS_CODEC_E_RLE; break; }
            } else {
              int64_t q64 = q;
              uint64_t h64;
              if (!get_varint(rle, mm, q64, h64)) { status = GGRS_CODEC_E_RLE; break; }
              const uint64_t rl64 = (h64 & 1) ? h64 >> 2 : h64 >> 1;
              if (rl64 > (uint64_t)kMaxDecoded || (uint64_t)xl + rl64 > (uint64_t)kMaxDecoded) { status = GGRS_CODEC_E_RLE; break; }
              q = (int)q64;
              h = (uint32_t)h64;
              rl = (int)rl64;
            }
            const bool fits = xl + rl <= kCap;
            if (!(h & 1)) {
              if (mm - q < rl) { status = GGRS_CODEC_E_RLE; break; }
              if (fits)
                for (int k = 0; k < rl; k++) xb[xl + k] = rle[q + k];
              q += rl;
            } else if ((h & 2) && fits && rl > 0) {
              ffm |= (rl >= kFb ? ~(Mf)0 : ((Mf)1 << rl) - 1) << xl;  // 0xFF bytes, expanded below
            }
            xl += rl;
          }
          if (status == GGRS_CODEC_OK) {
            cnt = xl / B;
            if (cnt * B != xl) status = GGRS_CODEC_E_DELTA;
            else if (cnt > W) status = GGRS_CODEC_E_CAP;
          }
        }
      }
    }
    uint32_t* orow = xr32;  // dword k of the output replaces dword k of the runs, in order
    if (status == GGRS_CODEC_OK) {
      const int xl = (int)cnt * B;
      const uint32_t refpat = B == 1 ? rw * 0x01010101u : (B == 2 ? rw * 0x00010001u : rw);
      const uint32_t* xr = xr32;
      uint32_t carry = 0;  // the previous dword's last input, repeated
#pragma unroll
      for (int k = 0; k < NDW; k++) {
        if (4 * k >= WB) break;
        const int live_bytes = xl - 4 * k;
        const uint32_t keep = live_bytes >= 4 ? 0xFFFFFFFFu : (live_bytes <= 0 ? 0u : (1u << (8 * live_bytes)) - 1u);
        const uint32_t ffb = (uint32_t)(ffm >> (4 * k)) & 0xFu;
        uint32_t y = (xr[k] | (((ffb * 0x00204081u) & 0x01010101u) * 0xFFu)) & keep;
        // prefix XOR of stride B inside the dword, then the carry from the dwords before
        if constexpr (B == 1) {
          y ^= y << 8;
          y ^= y << 16;
        } else if constexpr (B == 2) {
          y ^= y << 16;
        }
        y ^= carry;
        carry = B == 1 ? (y >> 24) * 0x01010101u : (B == 2 ? (y >> 16) * 0x00010001u : y);
        orow[k] = (y ^ refpat) & keep;
      }
      p.count[pk] = (int32_t)cnt;
    } else {
      for (int k = 0; k < WB / 4; k++) orow[k] = 0;
      p.count[pk] = 0;
    }
    p.status[pk] = status;
  }
  __syncthreads();
  lds_to_block(p.out + pk0 * (int64_t)WB, l_x, x_pitch, np, WB);
}

size_t encode_swar_bytes(int ndw, int stride, bool chunked = false) {
  return (size_t)256 * (swar_out_pitch(stride, ndw) + odd_dword_pitch(4 * ndw) +
                        (chunked && !encode_in_place(ndw) ? stride : 0));
}
size_t decode_swar_bytes(int ndw, int B, int W, int stride) {
  return (size_t)256 * (odd_dword_pitch(stride) + odd_dword_pitch(4 * ndw));
}
// dwords of the run-level forms' register stream (a power of two >= W*B/4), or 0 when they do
// not apply
int swar_ndw(int B, int W, int stride) {
  const int WB = W * B;
  if ((B != 1 && B != 2 && B != 4) || WB <= 0 || WB > 64 || WB % 4 || stride % 4) return 0;
  int n = 1;
  while (4 * n < WB) n <<= 1;
  return n;
}

template <int B, bool C>
void launch_encode_swar(int ndw, int64_t grid, size_t lds, hipStream_t s, const EncodeParams& p) {
  switch (ndw) {
    case 1: encode_swar_kernel<B, 1, C><<<grid, 256, lds, s>>>(p); break;
    case 2: encode_swar_kernel<B, 2, C><<<grid, 256, lds, s>>>(p); break;
    case 4: encode_swar_kernel<B, 4, C><<<grid, 256, lds, s>>>(p); break;
    case 8: encode_swar_kernel<B, 8, C><<<grid, 256, lds, s>>>(p); break;
    default: encode_swar_kernel<B, 16, C><<<grid, 256, lds, s>>>(p); break;
  }
}
template <int B, bool C>
void launch_decode_swar(int ndw, int64_t grid, size_t lds, hipStream_t s, const DecodeParams& p) {
  switch (ndw) {
    case 1: decode_swar_kernel<B, 1, C><<<grid, 256, lds, s>>>(p); break;
    case 2: decode_swar_kernel<B, 2, C><<<grid, 256, lds, s>>>(p); break;
    case 4: decode_swar_kernel<B, 4, C><<<grid, 256, lds, s>>>(p); break;
    case 8: decode_swar_kernel<B, 8, C><<<grid, 256, lds, s>>>(p); break;
    default: decode_swar_kernel<B, 16, C><<<grid, 256, lds, s>>>(p); break;
  }
}
template <bool C>
void encode_swar_any(int B, int ndw, int64_t grid, size_t lds, hipStream_t s, const EncodeParams& p) {
  if (B == 1) launch_encode_swar<1, C>(ndw, grid, lds, s, p);
  else if (B == 2) launch_encode_swar<2, C>(ndw, grid, lds, s, p);
  else launch_encode_swar<4, C>(ndw, grid, lds, s, p);
}
template <bool C>
void decode_swar_any(int B, int ndw, int64_t grid, size_t lds, hipStream_t s, const DecodeParams& p) {
  if (B == 1) launch_decode_swar<1, C>(ndw, grid, lds, s, p);
  else if (B == 2) launch_decode_swar<2, C>(ndw, grid, lds, s, p);
  else launch_decode_swar<4, C>(ndw, grid, lds, s, p);
}

// LDS bytes for a block of T threads, or 0 when the staged form does not apply
size_t encode_lds_bytes(int T, int B, int W, int stride) {
  if ((W * B) % 4 || stride % 4 || W * B == 0) return 0;
  return (size_t)T * (odd_dword_pitch(W * B) + odd_dword_pitch(stride) + B);
}
size_t decode_lds_bytes(int T, int B, int W, int stride) {
  if ((W * B) % 4 || stride % 4 || W * B == 0) return 0;
  return (size_t)T * (odd_dword_pitch(stride) + odd_dword_pitch(W * B) + B);
}
bool aligned4(const void* a) { return ((uintptr_t)a & 3) == 0; }
constexpr size_t kLdsBudget = 64 * 1024;

}  // namespace

extern "C" {

int ggrs_codec_encode(const uint8_t* ref, const uint8_t* pending, const int32_t* count, int64_t n_packets,
                      int32_t input_bytes, int32_t max_inputs, uint8_t* out, int32_t out_stride, int32_t* out_len,
                      void* stream) {
  if (n_packets < 0 || input_bytes < 1 || max_inputs < 0 || out_stride < 9)
    return set_error(GGRS_E_INVALID, "codec: need n_packets >= 0, input_bytes >= 1, max_inputs >= 0, stride >= 9");
  if (n_packets == 0) return GGRS_OK;
  if (!ref || !pending || !count || !out || !out_len) return set_error(GGRS_E_INVALID, "null argument");
  EncodeParams p{ref, pending, count, out, out_len, n_packets, input_bytes, max_inputs, out_stride};
  const int ndw = swar_ndw(input_bytes, max_inputs, out_stride);
  const bool al = aligned4(pending) && aligned4(out);
  if (g_codec_mode == 0 && ndw && al && encode_swar_bytes(ndw, out_stride) <= kLdsBudget) {
    const size_t lds = encode_swar_bytes(ndw, out_stride);
    encode_swar_any<false>(input_bytes, ndw, grid_of(n_packets, 256), lds, (hipStream_t)stream, p);
    HIP_TRY(hipGetLastError());
    return GGRS_OK;
  }
  const size_t lds = encode_lds_bytes(256, input_bytes, max_inputs, out_stride);
  if (lds && lds <= kLdsBudget && al && g_codec_mode != 1)
    encode_lds_kernel<<<grid_of(n_packets, 256), 256, lds, (hipStream_t)stream>>>(p);
  else
    encode_kernel<<<grid_of(n_packets, 256), 256, 0, (hipStream_t)stream>>>(p);
  HIP_TRY(hipGetLastError());
  return GGRS_OK;
}

int ggrs_codec_decode(const uint8_t* ref, const uint8_t* packets, const int32_t* packet_len, int64_t n_packets,
                      int32_t packet_stride, int32_t input_bytes, int32_t max_inputs, uint8_t* out, int32_t* count,
                      int32_t* status, void* stream) {
  if (n_packets < 0 || input_bytes < 1 || max_inputs < 0 || packet_stride < 0)
    return set_error(GGRS_E_INVALID, "codec: need n_packets >= 0, input_bytes >= 1, max_inputs >= 0");
  if (n_packets == 0) return GGRS_OK;
  if (!ref || !packets || !packet_len || !out || !count || !status) return set_error(GGRS_E_INVALID, "null argument");
  DecodeParams p{ref, packets, packet_len, out, count, status, n_packets, input_bytes, max_inputs, packet_stride};
  const int ndw = swar_ndw(input_bytes, max_inputs, packet_stride);
  const bool al = aligned4(packets) && aligned4(out);
  if (g_codec_mode == 0 && ndw && al && decode_swar_bytes(ndw, input_bytes, max_inputs, packet_stride) <= kLdsBudget) {
    const size_t lds = decode_swar_bytes(ndw, input_bytes, max_inputs, packet_stride);
    decode_swar_any<false>(input_bytes, ndw, grid_of(n_packets, 256), lds, (hipStream_t)stream, p);
    HIP_TRY(hipGetLastError());
    return GGRS_OK;
  }
  const size_t lds = decode_lds_bytes(256, input_bytes, max_inputs, packet_stride);
  if (lds && lds <= kLdsBudget && al && g_codec_mode != 1)
    decode_lds_kernel<<<grid_of(n_packets, 256), 256, lds, (hipStream_t)stream>>>(p);
  else
    decode_kernel<<<grid_of(n_packets, 256), 256, 0, (hipStream_t)stream>>>(p);
  HIP_TRY(hipGetLastError());
  return GGRS_OK;
}

int ggrs_codec_encode_chunked(const uint8_t* ref, const uint8_t* pending, const int32_t* count, int64_t n_packets,
                              int32_t input_bytes, int32_t max_inputs, uint8_t* out, int32_t out_stride,
                              int32_t* out_len, void* stream) {
  if (n_packets < 0 || input_bytes < 1 || max_inputs < 0 || out_stride < 9)
    return set_error(GGRS_E_INVALID, "codec: need n_packets >= 0, input_bytes >= 1, max_inputs >= 0, stride >= 9");
  if (n_packets == 0) return GGRS_OK;
  if (!ref || !pending || !count || !out || !out_len) return set_error(GGRS_E_INVALID, "null argument");
  const int ndw = swar_ndw(input_bytes, max_inputs, out_stride);
  if (!ndw || !aligned4(pending) || !aligned4(out) || encode_swar_bytes(ndw, out_stride, true) > kLdsBudget)
    return set_error(GGRS_E_INVALID, "codec: the chunked layout needs 1-, 2- or 4-byte inputs, W * B <= 64 and "
                                     "multiple of 4, a stride multiple of 4 and dword-aligned buffers");
  EncodeParams p{ref, pending, count, out, out_len, n_packets, input_bytes, max_inputs, out_stride};
  encode_swar_any<true>(input_bytes, ndw, grid_of(n_packets, 256), encode_swar_bytes(ndw, out_stride, true),
                        (hipStream_t)stream, p);
  HIP_TRY(hipGetLastError());
  return GGRS_OK;
}

int ggrs_codec_decode_chunked(const uint8_t* ref, const uint8_t* packets, const int32_t* packet_len, int64_t n_packets,
                              int32_t packet_stride, int32_t input_bytes, int32_t max_inputs, uint8_t* out,
                              int32_t* count, int32_t* status, void* stream) {
  if (n_packets < 0 || input_bytes < 1 || max_inputs < 0 || packet_stride < 0)
    return set_error(GGRS_E_INVALID, "codec: need n_packets >= 0, input_bytes >= 1, max_inputs >= 0");
  if (n_packets == 0) return GGRS_OK;
  if (!ref || !packets || !packet_len || !out || !count || !status) return set_error(GGRS_E_INVALID, "null argument");
  const int ndw = swar_ndw(input_bytes, max_inputs, packet_stride);
  const size_t lds = ndw ? decode_swar_bytes(ndw, input_bytes, max_inputs, packet_stride) : 0;
  if (!ndw || !aligned4(packets) || !aligned4(out) || lds > kLdsBudget)
    return set_error(GGRS_E_INVALID, "codec: the chunked layout needs 1-, 2- or 4-byte inputs, W * B <= 64 and "
                                     "multiple of 4, a stride multiple of 4 and dword-aligned buffers");
  DecodeParams p{ref, packets, packet_len, out, count, status, n_packets, input_bytes, max_inputs, packet_stride};
  decode_swar_any<true>(input_bytes, ndw, grid_of(n_packets, 256), lds, (hipStream_t)stream, p);
  HIP_TRY(hipGetLastError());
  return GGRS_OK;
}

int32_t ggrs_codec_max_packet_bytes(int32_t input_bytes, int32_t max_inputs) {
  // tag + u64 length + worst-case runs: alternating 1-byte literal / 1-byte compressed runs
  // (3 bytes per 2 input bytes) plus one varint header per run; rounded up to 16 bytes so rows
  // stay dword aligned (the LDS-staged kernels move whole dwords)
  const int64_t L = (int64_t)input_bytes * max_inputs;
  const int64_t v = (1 + 8 + L + (L + 1) / 2 + 10 + 15) / 16 * 16;
  return v > 0x7fffffff ? -1 : (int32_t)v;
}

int ggrs_codec_set_direct(int32_t mode) {
  if (mode < 0 || mode > 2) return set_error(GGRS_E_INVALID, "codec mode %d (0 default, 1 direct, 2 staged)", mode);
  g_codec_mode = mode;
  return GGRS_OK;
}

}  // extern "C"
