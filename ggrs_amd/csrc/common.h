// common.h -- helpers shared by the engine translation units (engine.hip, branch.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ggrs_amd.h"
#include "box_game.h"

#pragma clang fp contract(off)

namespace ggrs {

// Sets the calling thread's ggrs_last_error() message and returns `code` (defined in engine.hip).
int set_error(int code, const char* fmt, ...);

#define HIP_TRY(expr)                                                                            \
  do {                                                                                           \
    hipError_t e_ = (expr);                                                                      \
    if (e_ != hipSuccess) return ::ggrs::set_error(GGRS_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

constexpr int kWave = 64;

// Device time of a span of fused launches (ggrs_*_timing_reset .. _read): one HIP event pair on
// the engine's stream brackets the whole span, so the timed path records no per-launch events
// (a pair per launch cost ~7.8 us of a 0.26 ms SyncTest launch).
struct SpanTimer {
  hipEvent_t begin = nullptr, end = nullptr;
  bool collecting = false, open = false, stopped = false;
  int32_t launches = 0;
  int create() {
    HIP_TRY(hipEventCreate(&begin));
    HIP_TRY(hipEventCreate(&end));
    return GGRS_OK;
  }
  void destroy() {
    if (begin) (void)hipEventDestroy(begin);
    if (end) (void)hipEventDestroy(end);
    begin = end = nullptr;
  }
  // before enqueueing a fused launch: the span's first one records the begin event
  int before(hipStream_t s) {
    if (collecting && !open) {
      HIP_TRY(hipEventRecord(begin, s));
      open = true;
    }
    return GGRS_OK;
  }
  void count(int32_t n = 1) {
    if (collecting) launches += n;
  }
  int reset(hipStream_t s) {
    HIP_TRY(hipStreamSynchronize(s));
    collecting = true;
    open = false;
    stopped = false;
    launches = 0;
    return GGRS_OK;
  }
  // the span's end event right behind the last launch, without waiting (read then reports it)
  int stop(hipStream_t s) {
    if (open && !stopped) {
      HIP_TRY(hipEventRecord(end, s));
      stopped = true;
    }
    collecting = false;
    return GGRS_OK;
  }
  // span milliseconds (launch gaps included) and fused launches; stops collecting
  int read(hipStream_t s, float* ms, int32_t* n) {
    *ms = 0.0f;
    if (open) {
      if (!stopped) HIP_TRY(hipEventRecord(end, s));
      HIP_TRY(hipEventSynchronize(end));
      HIP_TRY(hipEventElapsedTime(ms, begin, end));
    } else {
      HIP_TRY(hipStreamSynchronize(s));
    }
    *n = launches;
    collecting = open = stopped = false;
    launches = 0;
    return GGRS_OK;
  }
};

// Cache-policy operand of the raw buffer store builtins on gfx950: sc1, a write-through store.
// Used for saves a launch does not read back from L2 soon, so they drain to memory while the
// kernel runs rather than in the end-of-kernel write-back of every dirtied L2 line.
constexpr int kStoreWriteThrough = 16;

// XCD-aware block order.  The dispatcher deals workgroup i to XCD i % 8 (MI355X: 8 XCDs, each
// with its own L2), so neighbouring blocks -- whose sessions share 64-byte lines of every SoA
// row (ring fields, checksums, input rows) -- would sit on different XCDs: each XCD fetches the
// shared line, and partial-line writes from several L2s reach HBM separately.  xcd_block maps
// workgroup i to the logical block that gives XCD x a contiguous range of logical blocks
// (q = n / 8 each, the first n % 8 XCDs one more): a bijection of [0, n).
constexpr int kXcds = 8;
__device__ inline int64_t xcd_block(int64_t i, int64_t n) {
  const int64_t q = n / kXcds, r = n % kXcds, x = i % kXcds, k = i / kXcds;
  return x * q + (x < r ? x : r) + k;
}

inline int padded_players(int p) { return p <= 1 ? 1 : (p == 2 ? 2 : 4); }
inline int64_t grid_of(int64_t n, int64_t block) { return (n + block - 1) / block; }

template <int P>
struct InputWord;
template <>
struct InputWord<1> { using T = uint8_t; };
template <>
struct InputWord<2> { using T = uint16_t; };
template <>
struct InputWord<3> { using T = uint32_t; };
template <>
struct InputWord<4> { using T = uint32_t; };

// the Pp-byte input record of one lane/session (players packed little-endian)
template <int P>
__device__ inline uint32_t load_inputs(const uint8_t* base, int64_t idx) {
  using T = typename InputWord<P>::T;
  return (uint32_t)reinterpret_cast<const T*>(base)[idx];
}

template <int P>
__device__ inline void load_state(BoxState<P>& s, const uint32_t* base, int64_t L) {
#pragma unroll
  for (int k = 0; k < state_fields(P); k++) s.w[k] = base[k * L];
}
template <int P>
__device__ inline void store_state(const BoxState<P>& s, uint32_t* base, int64_t L) {
#pragma unroll
  for (int k = 0; k < state_fields(P); k++) base[k * L] = s.w[k];
}

// exact fmod for |a| < 2|b| (Sterbenz), library fmodf otherwise
__device__ inline float fmod_exact(float a, float b) {
  float aa = __builtin_fabsf(a), ab = __builtin_fabsf(b);
  if (aa < ab) return a;
  if (aa < 2.0f * ab) return __builtin_copysignf(aa - ab, a);
  return fmodf(a, b);
}

// bincode encoding of a SoA state record (i32 frame, u64 P, u64 P + (x, y)*P, u64 P + (vx, vy)*P,
// u64 P + rot*P): the bytes ex_game.rs:105 hands to fletcher16.
inline void serialize_state_bytes(const uint32_t* w, int P, uint8_t* out) {
  uint8_t* o = out;
  auto u32 = [&](uint32_t v) { __builtin_memcpy(o, &v, 4); o += 4; };
  auto u64 = [&](uint64_t v) { __builtin_memcpy(o, &v, 8); o += 8; };
  u32(w[0]);
  u64((uint64_t)P);
  u64((uint64_t)P);
  for (int k = 1; k <= 2 * P; k++) u32(w[k]);
  u64((uint64_t)P);
  for (int k = 2 * P + 1; k <= 4 * P; k++) u32(w[k]);
  u64((uint64_t)P);
  for (int k = 4 * P + 1; k <= 5 * P; k++) u32(w[k]);
}

namespace {

// State::new(P) for every lane (ex_game.rs:246-269)
template <int P>
__global__ __launch_bounds__(256) void init_states_kernel(uint32_t* cur, int64_t L) {
  const int64_t lane = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= L) return;
  BoxState<P> s;
  s.w[0] = 0;
  const float r = kWindowWidth / 4.0f;
#pragma unroll
  for (int i = 0; i < P; i++) {
    float rot = (float)i / (float)P * 2.0f * kPi;
    s.set(fld_x(P, i), kWindowWidth / 2.0f + r * glibc_cosf(rot));
    s.set(fld_y(P, i), kWindowHeight / 2.0f + r * glibc_sinf(rot));
    s.set(fld_vx(P, i), 0.0f);
    s.set(fld_vy(P, i), 0.0f);
    s.set(fld_rot(P, i), fmod_exact(rot + kPi, 2.0f * kPi));
  }
  store_state<P>(s, cur + lane, L);
}

// Repack [n][L][P] user inputs into a [C][L][Pp] queue at queue frames q0.. (wrapping).
__global__ void pack_inputs_kernel(const uint8_t* src, uint8_t* dst, int64_t L, int32_t P,
                                   int32_t Pp, int32_t n, int32_t q0, int32_t cap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)n * L) return;
  const int64_t fr = i / L, lane = i % L;
  const int64_t q = ((int64_t)q0 + fr) % cap;
  for (int k = 0; k < Pp; k++) dst[(q * L + lane) * Pp + k] = k < P ? src[i * P + k] : 0;
}

template <typename F>
inline void dispatch_players(int p, F&& f) {
  switch (p) {
    case 1: f(std::integral_constant<int, 1>()); break;
    case 2: f(std::integral_constant<int, 2>()); break;
    case 3: f(std::integral_constant<int, 3>()); break;
    default: f(std::integral_constant<int, 4>()); break;
  }
}

// A pointer held in vector registers: the kernel's uniform values exceed the scalar register file
// (102 SGPRs) and the compiler spills them to VGPR lanes, reloading each with a v_readlane at every
// use; the buffers touched only at a launch's start and end and by rare paths live in VGPRs instead
// (an empty asm statement: it emits no instruction).
template <typename T>
__device__ inline T* in_vgpr_ptr(T* ptr) {
  uint64_t u = reinterpret_cast<uint64_t>(ptr);
  asm volatile("" : "+v"(u));
  return reinterpret_cast<T*>(u);
}
__device__ inline int32_t in_vgpr_i32(int32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}

}  // namespace

}  // namespace ggrs
