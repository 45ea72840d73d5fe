// Config 5 "particle world": the large-state stress game SURVEY.md 8d defines (not in the
// reference).  A session's state is one frame counter and N entities of 100 bytes each:
//   ship   x, y, vx, vy, rot  (f32)  -- stepped exactly like one ex_game player
//                                      (State::advance body, examples/ex_game/ex_game.rs:276-331)
//   payload p[0..19]          (u32)  -- integer state updated exactly every frame
// Initial state (frame 0): ship e as State::new places player e of N (ex_game.rs:246-269);
//   payload p[k] = low 32 bits of mix64((session << 40) ^ (e << 8) ^ k).
// Advance(inputs in[0..P-1]): frame += 1; entity e plays input in[e % P] through the ship step;
//   payload p'[k] = p[k] * 0x9E3779B1 + (p[(k + 1) % 20] >> 7) + input  (old values, u32 wrap).
// Declared byte layout (little endian) for the checksum: frame (4 bytes), then for each entity
//   x, y, vx, vy, rot, p[0..19] -- n = 4 + 100 N bytes; checksum = ex_game's fletcher16
//   (ex_game.rs:45-55) over those bytes, evaluated in closed form with 64-bit sums.
// The CPU restatement is oracle/ggrs_oracle.c (particle_*).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "box_game.h"

#pragma clang fp contract(off)

namespace ggrs {
namespace particles {

constexpr int kFields = 25;        // 5 ship floats + 20 payload words per entity
constexpr int kEntityBytes = 100;  // 4 * kFields
constexpr uint32_t kPayloadMul = 0x9E3779B1u;

__host__ __device__ inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__host__ __device__ inline uint32_t initial_payload(uint64_t session, uint64_t e, int k) {
  return (uint32_t)mix64((session << 40) ^ (e << 8) ^ (uint64_t)k);
}

// One entity's frame step.  w[0..4] ship bits, w[5..24] payload.  Lean = the caller has checked
// that rot is in [+0, 2pi] (box_game.h advance_player_lean, which keeps it there); otherwise the
// general form.
template <bool Lean>
__device__ inline void advance_entity(uint32_t (&w)[kFields], uint32_t input) {
  float x = __builtin_bit_cast(float, w[0]), y = __builtin_bit_cast(float, w[1]);
  float vx = __builtin_bit_cast(float, w[2]), vy = __builtin_bit_cast(float, w[3]);
  float rot = __builtin_bit_cast(float, w[4]);
  if constexpr (Lean) advance_player_lean(x, y, vx, vy, rot, input);
  else advance_player_general(x, y, vx, vy, rot, input);
  w[0] = __builtin_bit_cast(uint32_t, x);
  w[1] = __builtin_bit_cast(uint32_t, y);
  w[2] = __builtin_bit_cast(uint32_t, vx);
  w[3] = __builtin_bit_cast(uint32_t, vy);
  w[4] = __builtin_bit_cast(uint32_t, rot);
  const uint32_t p0 = w[5];
#pragma unroll
  for (int k = 0; k < 20; k++) {
    const uint32_t next = k < 19 ? w[5 + k + 1] : p0;
    w[5 + k] = w[5 + k] * kPayloadMul + (next >> 7) + input;
  }
}

// Fletcher-16 partial sums of one entity record at byte offset o in an n-byte stream:
//   s1 += sum of bytes, s2 += sum_j (n - o - j) d_j  split as (n - o) * sum(bytes) - sum_j j d_j.
// Over a record: sum_j j d_j = sum_k (4k * A(w_k) + B(w_k)), A = dot4(w, 1111), B = dot4(w, 0123).
struct FletcherAcc {
  uint32_t s1;     // byte sum (<= 2^32 per thread: 255 * 100 * entities-per-thread)
  uint64_t s2pos;  // sum (n - o_e) * A_e
  uint32_t s2neg;  // sum of the in-record weights
};

// The in-record weight of byte b of word k is 4k + b <= 99, so both sums are one accumulating
// dot4 per word: A += dot4(w_k, 1111), J += dot4(w_k, [4k, 4k+1, 4k+2, 4k+3]).
__device__ inline void fletcher_entity(FletcherAcc& acc, const uint32_t (&w)[kFields], uint64_t n_minus_o) {
  uint32_t a = 0, j = 0;
#pragma unroll
  for (int k = 0; k < kFields; k++) {
    a = __builtin_amdgcn_udot4(w[k], 0x01010101u, a, false);
    j = __builtin_amdgcn_udot4(w[k], 0x03020100u + 0x04040404u * (uint32_t)k, j, false);
  }
  acc.s1 += a;
  acc.s2pos += n_minus_o * (uint64_t)a;
  acc.s2neg += j;
}

}  // namespace particles
}  // namespace ggrs
