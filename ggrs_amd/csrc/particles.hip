// particles.hip -- the SyncTest rollback program (SyncTestSession::advance_frame,
// src/sessions/sync_test_session.rs:85-150, same bookkeeping as synctest_kernel in engine.hip) on
// the config-5 particle world (particles.h): ~1 MB states, so every Load/Save is an HBM stream.
//
// One workgroup per session.  Each thread owns units of E consecutive entities (E = 1, 2 or 4;
// E-dword loads/stores per field) and keeps a unit in registers across one call's replay: Load
// (1 read of the unit), cd x (Save, Advance), Save of the current frame, the new frame's Advance.
// HBM per call and session = S (load) + cd * S (saves), S = 4 + 100 N bytes -- per resimulated
// frame S * (1 + 1/cd); the post-call state is not stored (it is Advance(saved cell f, input f),
// materialised when the host reads it).  The Fletcher-16 of every saved frame is reduced mod 255
// per entity in registers, accumulated per lane in LDS and summed over the workgroup once per call.
//
// HBM layout: a state record is [ceil(N/256) tiles][25 fields][256 entities] u32 (tile-major,
// field-major inside a tile, entity fastest), so one block-step's saves of 256 entities are one
// contiguous 25 KB run rather than 25 runs 40 KB apart; ring [R][L][rec], cur [L][rec], frame
// counters [R][L] / [L] i32, ring_ck / first_ck [R][L] u16, inputs [C][L] u32 (P input bytes per frame).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "common.h"
#include "particles.h"

#pragma clang fp contract(off)

using namespace ggrs;
using namespace ggrs::particles;

namespace {

constexpr int kBlock = 256;
constexpr int kMaxCd = 62;

constexpr int kTile = 256;  // entities per tile of the record layout

// u32 words of one (padded) state record, and the word of (field k, entity e) inside it
__host__ __device__ inline size_t pw_rec(int32_t N) { return (size_t)((N + kTile - 1) / kTile) * kFields * kTile; }
__host__ __device__ inline size_t pw_idx(int32_t k, int32_t e) {
  return (size_t)(e / kTile) * kFields * kTile + (size_t)k * kTile + (size_t)(e % kTile);
}

struct PWParams {
  int64_t L;
  int32_t N, R, cd, f0, n, cap, P;
  int32_t corrupt_lane, corrupt_frame;
  int32_t nt_saves;
  uint32_t* cur;
  int32_t* cur_frame;
  uint32_t* ring;
  int32_t* ring_frame;
  uint16_t* ring_ck;
  uint16_t* first_ck;
  const uint32_t* inputs;
  int32_t* lane_status;
  int32_t* mis_frame;
  uint64_t* mis_mask;
};

__global__ void pw_init_kernel(uint32_t* cur, int32_t* cur_frame, int64_t L, int32_t N, int64_t first_session) {
  const int64_t s = blockIdx.y;
  for (int32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < N; e += gridDim.x * blockDim.x) {
    uint32_t* base = cur + (size_t)s * pw_rec(N) + pw_idx(0, e);
    const float r = kWindowWidth / 4.0f;
    const float rot = (float)e / (float)N * 2.0f * kPi;
    base[0] = __builtin_bit_cast(uint32_t, kWindowWidth / 2.0f + r * glibc_cosf(rot));
    base[kTile] = __builtin_bit_cast(uint32_t, kWindowHeight / 2.0f + r * glibc_sinf(rot));
    base[2 * kTile] = 0u;
    base[3 * kTile] = 0u;
    base[4 * kTile] = __builtin_bit_cast(uint32_t, fmod_exact(rot + kPi, 2.0f * kPi));
    for (int k = 0; k < 20; k++)
      base[(5 + k) * kTile] = initial_payload((uint64_t)(first_session + s), (uint64_t)e, k);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) cur_frame[s] = 0;
}

// A thread owns E consecutive entities (E = 1, 2, 4; unit q = entities E*q .. E*q+E-1, inside one
// tile): one E-dword access per field.
template <int E>
using uvec = uint32_t __attribute__((ext_vector_type(E)));

template <int E>
__device__ inline void load_unit(uint32_t (&w)[E][kFields], const uint32_t* rec, int32_t q) {
  const uint32_t* base = rec + pw_idx(0, E * q);
#pragma unroll
  for (int k = 0; k < kFields; k++) {
    if constexpr (E == 1) {
      w[0][k] = base[k * kTile];
    } else {
      const uvec<E> v = *reinterpret_cast<const uvec<E>*>(base + k * kTile);
#pragma unroll
      for (int j = 0; j < E; j++) w[j][k] = v[j];
    }
  }
}
// Nt: ring saves are write-once-per-call streams far larger than any cache (non-temporal stores)
template <int E, bool Nt>
__device__ inline void store_unit(const uint32_t (&w)[E][kFields], uint32_t* rec, int32_t q) {
  uint32_t* base = rec + pw_idx(0, E * q);
#pragma unroll
  for (int k = 0; k < kFields; k++) {
    if constexpr (E == 1) {
      uint32_t* d = base + k * kTile;
      if constexpr (Nt) __builtin_nontemporal_store(w[0][k], d);
      else *d = w[0][k];
    } else {
      uvec<E> v;
#pragma unroll
      for (int j = 0; j < E; j++) v[j] = w[j][k];
      uvec<E>* d = reinterpret_cast<uvec<E>*>(base + k * kTile);
      if constexpr (Nt) __builtin_nontemporal_store(v, d);
      else *d = v;
    }
  }
}
template <int E, bool Lean>
__device__ inline void advance_unit(uint32_t (&w)[E][kFields], uint32_t in_word, int32_t P, int32_t e0) {
#pragma unroll
  for (int j = 0; j < E; j++) advance_entity<Lean>(w[j], (in_word >> (8 * ((e0 + j) % P))) & 0xffu);
}
// Fletcher partials of one unit (fletcher_entity_mod), added to the lane's own LDS slots of the
// saved frame (ds_add, no cross-lane traffic in the replay loop).
template <int E>
__device__ inline void fletcher_unit(uint32_t* slot_s1, uint32_t* slot_s2, const uint32_t (&w)[E][kFields],
                                     const uint32_t (&ce)[E]) {
  uint32_t s1d = 0, s2d = 0;
#pragma unroll
  for (int j = 0; j < E; j++) fletcher_entity_mod(s1d, s2d, w[j], ce[j]);
  atomicAdd(slot_s1, s1d);
  atomicAdd(slot_s2, s2d);
}

// checksum of one frame from the block's sums of doubled per-entity remainders (t1d, t2d: even,
// < 510 N) plus the frame counter at byte offset 0 (sum1 += A_f, sum2 += n A_f - B_f)
__device__ inline uint16_t finish_checksum(uint32_t t1d, uint32_t t2d, int32_t frame, int32_t N) {
  const uint64_t n = 4 + (uint64_t)kEntityBytes * N;
  const uint32_t fw = (uint32_t)frame;
  const uint32_t a = __builtin_amdgcn_udot4(fw, 0x01010101u, 0u, false);
  const uint32_t b = __builtin_amdgcn_udot4(fw, 0x03020100u, 0u, false);  // <= 1530
  const uint64_t t1 = (uint64_t)(t1d >> 1) + a;
  const uint64_t t2 = (uint64_t)(t2d >> 1) + n * a + 1530u - b;  // + 6 * 255 keeps it >= 0
  return (uint16_t)(((t2 % 255u) << 8) | (t1 % 255u));
}

constexpr int kWaves = kBlock / 64;

// dynamic LDS of pw_synctest_kernel: per lane and saved frame of a call, two u32 Fletcher sums
inline size_t pw_lds_bytes(int32_t cd) { return (size_t)(cd + 1) * 2 * kBlock * sizeof(uint32_t); }

// One call's replay of one unit (E entities) from its loaded frame g0: Save(g) + Fletcher
// (skipped for i = 0 on a replay: that cell was just loaded), Advance.  Only `on` lanes (owning
// a unit) do anything; slots = the lane's LDS column, [frame i][s1, s2] with stride kBlock.
template <int E, bool Lean>
__device__ inline void replay_unit(uint32_t (&w)[E][kFields], const PWParams& p, int64_t s, int32_t g0,
                                   int32_t steps, bool save_first, uint32_t in_cur, int32_t q, uint32_t* slots) {
  const size_t rec = pw_rec(p.N);
  const int32_t e0 = E * q;
  uint32_t ce[E];
#pragma unroll
  for (int j = 0; j < E; j++) ce[j] = (uint32_t)(((int64_t)kEntityBytes * (p.N - (e0 + j))) % 255);
  for (int32_t i = 0; i <= steps; ++i) {
    const int32_t g = g0 + i;  // frame the unit holds
    if (p.cd > 0 && (i > 0 || save_first)) {  // SaveGameState(g): the replay's saves, then save current
      uint32_t* dst = p.ring + ((size_t)(g % p.R) * p.L + s) * rec;
      if (p.nt_saves) store_unit<E, true>(w, dst, q);
      else store_unit<E, false>(w, dst, q);
      fletcher_unit<E>(slots + (2 * i) * kBlock, slots + (2 * i + 1) * kBlock, w, ce);
    }
    advance_unit<E, Lean>(w, i < steps ? p.inputs[(int64_t)(g % p.cap) * p.L + s] : in_cur, p.P, e0);
  }
}

template <int E>
__global__ __launch_bounds__(kBlock) void pw_synctest_kernel(PWParams p) {
  // per lane, per saved frame i of a call: sums of the doubled Fletcher remainders (s1, s2) of
  // the lane's units, [cd + 1][2][kBlock] u32 (dynamic: pw_lds_bytes)
  extern __shared__ uint32_t lds_slots[];
  __shared__ uint32_t lds_tot[kMaxCd + 1][2];
  __shared__ int32_t lds_stop;
  const int64_t s = blockIdx.x;
  if (p.lane_status[s] != GGRS_LANE_RUNNING) return;
  const int32_t N = p.N, R = p.R, nq = N / E, cd = p.cd;
  const int64_t L = p.L;
  const int wave = threadIdx.x >> 6;
  const size_t rec = pw_rec(N);  // u32 per session state (padded to whole tiles)
  uint32_t* cur = p.cur + (size_t)s * rec;
  for (int32_t f = p.f0; f < p.f0 + p.n; ++f) {
    const bool replay = cd > 0 && f > cd;
    if (replay && f >= cd + 2) {  // checksums_consistent over f-cd .. f (sync_test_session.rs:173-190)
      if (threadIdx.x == 0) {
        uint64_t mism = 0;
        for (int32_t fc = f - cd; fc <= f - 2; ++fc) {
          const int64_t o = (int64_t)(fc % R) * L + s;
          if (p.ring_ck[o] != p.first_ck[o]) mism |= 1ull << (fc - (f - cd));
        }
        lds_stop = mism != 0;
        if (mism) {
          p.lane_status[s] = GGRS_LANE_MISMATCH;
          p.mis_frame[s] = f;
          p.mis_mask[s] = mism;
        }
      }
      __syncthreads();
      if (lds_stop) {
        // Err(MismatchedChecksum): the session stops before the rollback, holding the state of
        // call f-1's final AdvanceFrame -- the advance of the frame-(f-1) cell it saved.
        const uint32_t in_prev = p.inputs[(int64_t)((f - 1) % p.cap) * L + s];
        for (int32_t q = threadIdx.x; q < nq; q += kBlock) {
          uint32_t w[E][kFields];
          load_unit<E>(w, p.ring + ((size_t)((f - 1) % R) * L + s) * rec, q);
          advance_unit<E, false>(w, in_prev, p.P, E * q);
          store_unit<E, false>(w, cur, q);
        }
        return;
      }
    }
    uint32_t* slots = lds_slots + threadIdx.x;  // this lane's column: only it touches it until the sums
    for (int k = 0; k < 2 * (cd + 1); k++) slots[k * kBlock] = 0;
    const uint32_t in_cur = p.inputs[(int64_t)(f % p.cap) * L + s];
    const int32_t g0 = replay ? f - cd : f;
    for (int32_t q = threadIdx.x; q < nq; q += kBlock) {
      uint32_t w[E][kFields];
      if (replay) {  // LoadGameState(f - cd)
        load_unit<E>(w, p.ring + ((size_t)(g0 % R) * L + s) * rec, q);
        if (s == p.corrupt_lane && f == p.corrupt_frame && q == 0) w[0][0] ^= 1u;
      } else {
        load_unit<E>(w, cur, q);  // the handler's current state (warm-up calls)
      }
      const int32_t steps = replay ? cd : 0;
      // one domain test per loaded unit: the lean step keeps rot in [+0, 2pi], so the whole
      // replay runs in the form the loaded rotations allow
      bool dom = true;
#pragma unroll
      for (int j = 0; j < E; j++) dom = dom && w[j][4] <= kTwoPiBits;
      if (__builtin_expect(dom, 1)) replay_unit<E, true>(w, p, s, g0, steps, !replay, in_cur, q, slots);
      else replay_unit<E, false>(w, p, s, g0, steps, !replay, in_cur, q, slots);
      // the game state after the call.  A replay call's result is Advance(ring cell f, input f),
      // both of which stay in place until the next call: the next call reloads from the ring, and
      // the host materialises `cur` on demand (pw_materialize_kernel), so only warm-up calls,
      // whose successor reads `cur`, store it.
      if (!replay) store_unit<E, false>(w, cur, q);
    }
    __syncthreads();
    // block sums of the saved frames' slots: wave v sums frames i = v, v + kWaves, ...
    const int i_lo = replay ? 1 : 0, i_hi = replay ? cd : 0;
    if (cd > 0) {
      for (int i = i_lo + wave; i <= i_hi; i += kWaves) {
        uint32_t t1 = 0, t2 = 0;
        for (int l = threadIdx.x & 63; l < kBlock; l += 64) {
          t1 += lds_slots[(2 * i) * kBlock + l];
          t2 += lds_slots[(2 * i + 1) * kBlock + l];
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
          t1 += (uint32_t)__shfl_xor((int)t1, m, 64);
          t2 += (uint32_t)__shfl_xor((int)t2, m, 64);
        }
        if ((threadIdx.x & 63) == 0) {
          lds_tot[i][0] = t1;
          lds_tot[i][1] = t2;
        }
      }
    }
    __syncthreads();
    if (cd > 0 && threadIdx.x == 0) {
      for (int i = i_lo; i <= i_hi; i++) {
        const int32_t g = g0 + i;
        const uint16_t ck = finish_checksum(lds_tot[i][0], lds_tot[i][1], g, N);
        p.ring_ck[(int64_t)(g % R) * L + s] = ck;
        p.ring_frame[(int64_t)(g % R) * L + s] = g;
        if (g == f) p.first_ck[(int64_t)(f % R) * L + s] = ck;  // first sighting of frame f
      }
    }
    if (threadIdx.x == 0) p.cur_frame[s] = f + 1;
    __syncthreads();
  }
}

// The handler's current state after a replay call f: Advance(ring cell f, input f) -- what the
// call computed last and did not store (pw_synctest_kernel).  Halted sessions keep the state the
// mismatch path stored.
__global__ __launch_bounds__(kBlock) void pw_materialize_kernel(PWParams p, int32_t f) {
  const int64_t s = blockIdx.x;
  if (p.lane_status[s] != GGRS_LANE_RUNNING) return;
  const size_t rec = pw_rec(p.N);
  const uint32_t in = p.inputs[(int64_t)(f % p.cap) * p.L + s];
  for (int32_t q = threadIdx.x; q < p.N; q += kBlock) {
    uint32_t w[1][kFields];
    load_unit<1>(w, p.ring + ((size_t)(f % p.R) * p.L + s) * rec, q);
    advance_unit<1, false>(w, in, p.P, q);
    store_unit<1, false>(w, p.cur + (size_t)s * rec, q);
  }
}

}  // namespace

struct ggrs_particle_engine {
  ggrs_particle_config_t cfg{};
  int R = 2, cap = 128;
  hipStream_t stream = nullptr;
  uint32_t* cur = nullptr;
  int32_t* cur_frame = nullptr;
  uint32_t* ring = nullptr;
  int32_t* ring_frame = nullptr;
  uint16_t* ring_ck = nullptr;
  uint16_t* first_ck = nullptr;
  uint32_t* inputs = nullptr;
  int32_t* lane_status = nullptr;
  int32_t* mis_frame = nullptr;
  uint64_t* mis_mask = nullptr;
  uint8_t* staging = nullptr;
  size_t staging_bytes = 0;
  int32_t current_frame = 0, next_input_frame = 0;
  int32_t corrupt_lane = -1, corrupt_frame = -1;
  int32_t nt_saves = 1;  // GGRS_PW_STORE=plain selects plain stores for the ring saves
  int32_t ept = 1;       // entities per thread (1, 2, 4); GGRS_PW_EPT selects (1: 4 waves/SIMD, no scratch)
  bool cur_stale = false;  // the last call was a replay: `cur` is materialised on read
  SpanTimer timer;
};

namespace {

__global__ void pw_pack_inputs(const uint8_t* src, uint32_t* dst, int64_t L, int32_t P, int32_t n, int32_t q0, int32_t cap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)n * L) return;
  const int64_t fr = i / L, s = i % L;
  uint32_t w = 0;
  for (int k = 0; k < P; k++) w |= (uint32_t)src[i * P + k] << (8 * k);
  dst[(((int64_t)q0 + fr) % cap) * L + s] = w;
}

}  // namespace

extern "C" {

int ggrs_particle_engine_destroy(ggrs_particle_engine_t* e) {
  if (!e) return GGRS_OK;
  (void)hipSetDevice(e->cfg.device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  void* bufs[] = {e->cur, e->cur_frame, e->ring, e->ring_frame, e->ring_ck, e->first_ck, e->inputs,
                  e->lane_status, e->mis_frame, e->mis_mask, e->staging};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  e->timer.destroy();
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
  return GGRS_OK;
}

int ggrs_particle_engine_create(const ggrs_particle_config_t* cfg, ggrs_particle_engine_t** out) {
  if (!cfg || !out) return set_error(GGRS_E_INVALID, "null argument");
  *out = nullptr;
  const ggrs_particle_config_t c = *cfg;
  if (c.num_sessions < 1) return set_error(GGRS_E_INVALID, "num_sessions must be >= 1");
  if (c.num_entities < 4 || c.num_entities % 4 != 0 || c.num_entities > 160000)
    return set_error(GGRS_E_INVALID, "num_entities must be a multiple of 4 in 4..160000");
  if (c.num_players < 1 || c.num_players > 4) return set_error(GGRS_E_INVALID, "num_players must be in 1..4");
  if (c.check_distance < 0 || c.check_distance > kMaxCd)
    return set_error(GGRS_E_INVALID, "check_distance must be in 0..%d", kMaxCd);
  if (c.check_distance >= c.max_prediction)
    return set_error(GGRS_E_INVALID, "Check distance too big. (check_distance must be < max_prediction)");
  if (c.max_prediction > 63) return set_error(GGRS_E_INVALID, "max_prediction must be <= 63");
  ggrs_particle_engine* e = new ggrs_particle_engine();
  e->cfg = c;
  e->R = c.max_prediction + 1;
  e->cap = c.input_capacity ? c.input_capacity : 128;
  if (const char* sp = getenv("GGRS_PW_STORE")) e->nt_saves = strcmp(sp, "plain") != 0;
  if (const char* se = getenv("GGRS_PW_EPT")) {
    const int v = atoi(se);
    if (v == 1 || v == 2 || v == 4) e->ept = v;
  }
  e->cfg.input_capacity = e->cap;
  if (e->cap < c.check_distance + 2) {
    delete e;
    return set_error(GGRS_E_INVALID, "input_capacity must be >= check_distance + 2");
  }
  auto fail = [&](int rc) {
    std::string msg = ggrs_last_error();
    ggrs_particle_engine_destroy(e);
    set_error(rc, "%s", msg.c_str());
    return rc;
  };
#define CTRY(expr)                                                                      \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) return fail(set_error(GGRS_E_HIP, "%s: %s", #expr, hipGetErrorString(e_))); \
  } while (0)
  const int64_t L = c.num_sessions;
  const size_t rec = pw_rec(c.num_entities);
  CTRY(hipSetDevice(c.device));
  CTRY(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
  if (e->timer.create()) return fail(GGRS_E_HIP);
  if (pw_lds_bytes(c.check_distance) > 65536) {  // large check distances: past the default 64 KB
    const int lds = (int)pw_lds_bytes(c.check_distance);
    CTRY(hipFuncSetAttribute((const void*)pw_synctest_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CTRY(hipFuncSetAttribute((const void*)pw_synctest_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CTRY(hipFuncSetAttribute((const void*)pw_synctest_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  }
  CTRY(hipMalloc(&e->cur, 4 * rec * L));
  CTRY(hipMalloc(&e->cur_frame, 4 * L));
  CTRY(hipMalloc(&e->ring, 4 * rec * L * e->R));
  CTRY(hipMalloc(&e->ring_frame, 4 * (size_t)L * e->R));
  CTRY(hipMalloc(&e->ring_ck, 2 * (size_t)L * e->R));
  CTRY(hipMalloc(&e->first_ck, 2 * (size_t)L * e->R));
  CTRY(hipMalloc(&e->inputs, 4 * (size_t)L * e->cap));
  CTRY(hipMalloc(&e->lane_status, 4 * L));
  CTRY(hipMalloc(&e->mis_frame, 4 * L));
  CTRY(hipMalloc(&e->mis_mask, 8 * L));
  CTRY(hipMemsetAsync(e->ring_frame, 0xff, 4 * (size_t)L * e->R, e->stream));
  CTRY(hipMemsetAsync(e->ring_ck, 0, 2 * (size_t)L * e->R, e->stream));
  CTRY(hipMemsetAsync(e->first_ck, 0, 2 * (size_t)L * e->R, e->stream));
  CTRY(hipMemsetAsync(e->inputs, 0, 4 * (size_t)L * e->cap, e->stream));
  CTRY(hipMemsetAsync(e->lane_status, 0, 4 * L, e->stream));
  CTRY(hipMemsetAsync(e->mis_frame, 0xff, 4 * L, e->stream));
  CTRY(hipMemsetAsync(e->mis_mask, 0, 8 * L, e->stream));
  {
    dim3 grid((unsigned)std::min<int64_t>(64, (c.num_entities + 255) / 256), (unsigned)L);
    pw_init_kernel<<<grid, 256, 0, e->stream>>>(e->cur, e->cur_frame, L, c.num_entities, c.first_session_id);
    CTRY(hipGetLastError());
  }
  CTRY(hipStreamSynchronize(e->stream));
#undef CTRY
  *out = e;
  return GGRS_OK;
}

int ggrs_particle_add_local_inputs(ggrs_particle_engine_t* e, int32_t first_frame, int32_t n, const uint8_t* inputs) {
  if (!e || (!inputs && n > 0)) return set_error(GGRS_E_INVALID, "null argument");
  if (n < 0) return set_error(GGRS_E_INVALID, "n_frames must be >= 0");
  if (first_frame != e->next_input_frame)
    return set_error(GGRS_E_INVALID, "inputs must be added sequentially (expected frame %d, got %d)",
                     e->next_input_frame, first_frame);
  if (n == 0) return GGRS_OK;
  const int64_t oldest_needed = (int64_t)e->current_frame - e->cfg.check_distance;
  if ((int64_t)first_frame + n - 1 - oldest_needed >= e->cap)
    return set_error(GGRS_E_INVALID, "input queue full (capacity %d)", e->cap);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t L = e->cfg.num_sessions;
  const size_t bytes = (size_t)n * L * e->cfg.num_players;
  if (bytes > e->staging_bytes) {
    if (e->staging) HIP_TRY(hipFree(e->staging));
    e->staging = nullptr;
    e->staging_bytes = 0;
    HIP_TRY(hipMalloc(&e->staging, bytes));
    e->staging_bytes = bytes;
  }
  HIP_TRY(hipMemcpyAsync(e->staging, inputs, bytes, hipMemcpyHostToDevice, e->stream));
  pw_pack_inputs<<<grid_of((int64_t)n * L, 256), 256, 0, e->stream>>>(e->staging, e->inputs, L, e->cfg.num_players, n,
                                                                       first_frame % e->cap, e->cap);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->next_input_frame = first_frame + n;
  return GGRS_OK;
}

int ggrs_particle_synctest_advance_frames(ggrs_particle_engine_t* e, int32_t n) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (n < 0) return set_error(GGRS_E_INVALID, "n_frames must be >= 0");
  if (n == 0) return GGRS_OK;
  if ((int64_t)e->current_frame + n - 1 >= e->next_input_frame)
    return set_error(GGRS_E_INVALID, "Missing local input while calling advance_frame(): frame %d not added",
                     e->current_frame + n - 1);
  HIP_TRY(hipSetDevice(e->cfg.device));
  PWParams p;
  p.L = e->cfg.num_sessions;
  p.N = e->cfg.num_entities;
  p.R = e->R;
  p.cd = e->cfg.check_distance;
  p.f0 = e->current_frame;
  p.n = n;
  p.cap = e->cap;
  p.P = e->cfg.num_players;
  p.corrupt_lane = e->corrupt_lane;
  p.corrupt_frame = e->corrupt_frame;
  p.nt_saves = e->nt_saves;
  p.cur = e->cur;
  p.cur_frame = e->cur_frame;
  p.ring = e->ring;
  p.ring_frame = e->ring_frame;
  p.ring_ck = e->ring_ck;
  p.first_ck = e->first_ck;
  p.inputs = e->inputs;
  p.lane_status = e->lane_status;
  p.mis_frame = e->mis_frame;
  p.mis_mask = e->mis_mask;
  if (int rc = e->timer.before(e->stream)) return rc;
  const size_t lds = pw_lds_bytes(p.cd);
  if (e->ept == 1) pw_synctest_kernel<1><<<p.L, kBlock, lds, e->stream>>>(p);
  else if (e->ept == 2) pw_synctest_kernel<2><<<p.L, kBlock, lds, e->stream>>>(p);
  else pw_synctest_kernel<4><<<p.L, kBlock, lds, e->stream>>>(p);
  HIP_TRY(hipGetLastError());
  e->timer.count();
  e->current_frame += n;
  e->cur_stale = p.cd > 0 && e->current_frame - 1 > p.cd;  // the last call was a replay
  return GGRS_OK;
}

int ggrs_particle_synchronize(ggrs_particle_engine_t* e) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

int ggrs_particle_current_frame(const ggrs_particle_engine_t* e, int32_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  *out = e->current_frame;
  return GGRS_OK;
}

int ggrs_particle_read_mismatches(ggrs_particle_engine_t* e, int32_t* st, int32_t* mf, uint64_t* mm) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  const size_t L = e->cfg.num_sessions;
  if (st) HIP_TRY(hipMemcpyAsync(st, e->lane_status, 4 * L, hipMemcpyDeviceToHost, e->stream));
  if (mf) HIP_TRY(hipMemcpyAsync(mf, e->mis_frame, 4 * L, hipMemcpyDeviceToHost, e->stream));
  if (mm) HIP_TRY(hipMemcpyAsync(mm, e->mis_mask, 8 * L, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

// declared layout bytes of a tiled record: frame, then per entity 25 little-endian words
static void pw_serialize(const std::vector<uint32_t>& soa, int32_t frame, int32_t N, uint8_t* out) {
  memcpy(out, &frame, 4);
  for (int32_t e2 = 0; e2 < N; e2++)
    for (int k = 0; k < kFields; k++) memcpy(out + 4 + (size_t)kEntityBytes * e2 + 4 * k, &soa[pw_idx(k, e2)], 4);
}

int ggrs_particle_read_state(ggrs_particle_engine_t* e, int32_t session, uint8_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  if (session < 0 || session >= e->cfg.num_sessions) return set_error(GGRS_E_INVALID, "session out of range");
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int32_t N = e->cfg.num_entities;
  const size_t rec = pw_rec(N);
  if (e->cur_stale) {  // the handler's state after the last (replay) call, for every running session
    PWParams p{};
    p.L = e->cfg.num_sessions;
    p.N = N;
    p.R = e->R;
    p.cap = e->cap;
    p.P = e->cfg.num_players;
    p.cur = e->cur;
    p.ring = e->ring;
    p.inputs = e->inputs;
    p.lane_status = e->lane_status;
    pw_materialize_kernel<<<p.L, kBlock, 0, e->stream>>>(p, e->current_frame - 1);
    HIP_TRY(hipGetLastError());
    e->cur_stale = false;
  }
  std::vector<uint32_t> soa(rec);
  int32_t frame = 0;
  HIP_TRY(hipMemcpyAsync(soa.data(), e->cur + rec * session, 4 * rec, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipMemcpyAsync(&frame, e->cur_frame + session, 4, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  pw_serialize(soa, frame, N, out);
  return GGRS_OK;
}

int ggrs_particle_read_saved(ggrs_particle_engine_t* e, int32_t session, int32_t frame, uint16_t* checksum, uint8_t* out) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (session < 0 || session >= e->cfg.num_sessions) return set_error(GGRS_E_INVALID, "session out of range");
  if (frame < 0) return set_error(GGRS_E_INVALID, "negative frame");
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int32_t N = e->cfg.num_entities;
  const size_t rec = pw_rec(N);
  const int slot = frame % e->R;
  int32_t tag = -1;
  uint16_t ck = 0;
  HIP_TRY(hipMemcpyAsync(&tag, e->ring_frame + (size_t)slot * e->cfg.num_sessions + session, 4, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipMemcpyAsync(&ck, e->ring_ck + (size_t)slot * e->cfg.num_sessions + session, 2, hipMemcpyDeviceToHost, e->stream));
  std::vector<uint32_t> soa(out ? rec : 0);
  if (out)
    HIP_TRY(hipMemcpyAsync(soa.data(), e->ring + ((size_t)slot * e->cfg.num_sessions + session) * rec, 4 * rec,
                           hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (tag != frame) return set_error(GGRS_E_PRECONDITION, "no saved cell for frame %d (slot holds %d)", frame, tag);
  if (checksum) *checksum = ck;
  if (out) pw_serialize(soa, frame, N, out);
  return GGRS_OK;
}

int ggrs_particle_debug_corrupt_on_load(ggrs_particle_engine_t* e, int32_t session, int32_t frame) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  e->corrupt_lane = session;
  e->corrupt_frame = frame;
  return GGRS_OK;
}

int ggrs_particle_timing_reset(ggrs_particle_engine_t* e) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  return e->timer.reset(e->stream);
}

int ggrs_particle_timing_stop(ggrs_particle_engine_t* e) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  return e->timer.stop(e->stream);
}

int ggrs_particle_timing_read(ggrs_particle_engine_t* e, float* total_ms, int32_t* launches) {
  if (!e || !total_ms || !launches) return set_error(GGRS_E_INVALID, "null argument");
  HIP_TRY(hipSetDevice(e->cfg.device));
  return e->timer.read(e->stream, total_ms, launches);
}

}  // extern "C"
