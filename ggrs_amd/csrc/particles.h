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

// Fletcher-16 contribution of one entity record at byte offset o_e = 4 + 100 e of the n-byte
// stream (n = 4 + 100 N), reduced mod 255 (fletcher16's sums are mod 255, a ring homomorphism):
//   sum1 part  A_e = sum of the record's bytes,
//   sum2 part  sum_j (n - o_e - j) d_j = (n - o_e) A_e - J_e,  J_e = sum_j j d_j in the record,
// with c_e = (n - o_e) mod 255 = 100 (N - e) mod 255 precomputed per entity.  The in-record weight
// of byte b of word k is 4k + b <= 99, so doubled weights (<= 198) still fit v_dot4's u8 lanes:
// A2 = 2 A_e and J2 = 2 J_e are one accumulating dot4 per word each.  Then
//   x2 = c_e A2 + 2K - J2  (K = 255 * 4951 >= max J_e keeps it >= 0; x2 < 2^24),
// and the doubled remainders 2 (x mod 255) come from one 24-bit multiply-high each
// (as box_game.h fletcher_from_doubled).  Adds s1d = 2 (A_e mod 255), s2d = 2 (x mod 255), each < 510.
constexpr uint32_t kJ2Bias = 2u * 255u * 4951u;

// (24-bit multiply-adds written with __umul24 / __mul24, not inline asm: the inline-asm form
// gave wrong checksums under LLVM's max-ilp scheduler -- profiles/r04r, r04v -- and this unit is
// HBM-bound, so the compiler's choice of instructions costs nothing measurable)
__device__ inline uint32_t mad_u24(uint32_t a, uint32_t b, uint32_t c) { return __umul24(a, b) + c; }
__device__ inline uint32_t rem255_doubled(uint32_t x2) {  // 2 (x mod 255) for x2 = 2x < 2^24
  const uint32_t q = mulhi_u24(x2, 0x808081u);
  return (uint32_t)(__mul24((int32_t)q, -510) + (int32_t)x2);
}
__device__ inline void fletcher_entity_mod(uint32_t& s1d, uint32_t& s2d, const uint32_t (&w)[kFields], uint32_t c_e) {
  uint32_t a2 = 0, j2 = 0;
#pragma unroll
  for (int k = 0; k < kFields; k++) {
    a2 = __builtin_amdgcn_udot4(w[k], 0x02020202u, a2, false);
    j2 = __builtin_amdgcn_udot4(w[k], 0x06040200u + 0x08080808u * (uint32_t)k, j2, false);
  }
  s1d += rem255_doubled(a2);
  s2d += rem255_doubled(mad_u24(c_e, a2, kJ2Bias) - j2);
}

}  // namespace particles
}  // namespace ggrs
