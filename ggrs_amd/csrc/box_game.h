// ex_game box-game state, step and fused Fletcher-16, for one lane per (session, branch).
//
// Reference: examples/ex_game/ex_game.rs
//   constants              :10-26
//   fletcher16             :45-55   (over bincode::serialize(&State), :105-106 and :121-122)
//   State                  :236-243 (frame, num_players, positions, velocities, rotations)
//   State::new             :246-269
//   State::advance         :271-333
// Bit-exactness rules: separately rounded f32 ops in the reference's order
// (compile with -ffp-contract=off; Rust never contracts), correctly rounded f32 sqrt and division
// (hipcc's default), f32 denormals kept (hipcc's default), glibc's own sinf/cosf algorithm
// (glibc_sincosf.h), exact fmodf for rem_euclid.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "glibc_sincosf.h"

#pragma clang fp contract(off)

namespace ggrs {

constexpr float kWindowHeight = 800.0f;
constexpr float kWindowWidth = 600.0f;
constexpr float kMovementSpeed = 15.0f / 60.0f;  // 15.0 / FPS as f32
constexpr float kRotationSpeed = 2.5f / 60.0f;   // 2.5 / FPS as f32 (0x1.555556p-5)
constexpr float kMaxSpeed = 7.0f;
constexpr float kFriction = 0.98f;
constexpr float kPi = 3.14159265358979323846f;   // std::f32::consts::PI
constexpr float kTwoPi = 2.0f * kPi;             // 2.0 * PI evaluated in f32
constexpr uint32_t kInputUp = 1u, kInputDown = 2u, kInputLeft = 4u, kInputRight = 8u;

// Number of 32-bit fields of the SoA state: frame + (x, y, vx, vy, rot) per player.
__host__ __device__ constexpr int state_fields(int p) { return 1 + 5 * p; }
// bincode size of State (fixint LE): i32 + u64 + 3 * (u64 len) + 20 * P.
__host__ __device__ constexpr int bincode_bytes(int p) { return 36 + 20 * p; }

// SoA field index, in bincode order: frame, (x_i, y_i)*, (vx_i, vy_i)*, rot_i*.
__host__ __device__ constexpr int fld_frame() { return 0; }
__host__ __device__ constexpr int fld_x(int p, int i) { return 1 + 2 * i; }
__host__ __device__ constexpr int fld_y(int p, int i) { return 2 + 2 * i; }
__host__ __device__ constexpr int fld_vx(int p, int i) { return 1 + 2 * p + 2 * i; }
__host__ __device__ constexpr int fld_vy(int p, int i) { return 2 + 2 * p + 2 * i; }
__host__ __device__ constexpr int fld_rot(int p, int i) { return 1 + 4 * p + i; }
// byte offset of SoA field k inside the bincode encoding
__host__ __device__ constexpr int fld_offset(int p, int k) {
  return k == 0 ? 0 : (k <= 2 * p ? 20 + 4 * (k - 1) : (k <= 4 * p ? 28 + 4 * (k - 1) : 36 + 4 * (k - 1)));
}

template <int P>
struct BoxState {
  uint32_t w[state_fields(P)];  // raw bits; w[0] is the i32 frame
  __device__ __host__ float f(int k) const { return __builtin_bit_cast(float, w[k]); }
  __device__ __host__ void set(int k, float v) { w[k] = __builtin_bit_cast(uint32_t, v); }
};

// f32::rem_euclid: r = a % b (fmodf, exact); if r < 0 { r + |b| } else { r }.
// The fast path is exact fmod for |a| < 2|b| (Sterbenz), which covers rot +- ROTATION_SPEED for
// every rot in [0, 2*pi]; anything else takes the library fmodf (exact as well).
__device__ inline float rem_euclid(float a, float b) {
  float aa = __builtin_fabsf(a), ab = __builtin_fabsf(b);
  float r;
  if (aa < ab) r = a;
  else if (aa < 2.0f * ab) r = __builtin_copysignf(aa - ab, a);
  else r = fmodf(a, b);
  return r < 0.0f ? r + ab : r;
}

// One player of State::advance (ex_game.rs:276-331).  `input` is Input.inp, already mapped to 4
// for InputStatus::Disconnected by the caller (ex_game.rs:277-281).  General form: any rot.
__device__ inline void advance_player_general(float& x, float& y, float& vx, float& vy, float& rot,
                                              uint32_t input) {
  float vel_x = vx * kFriction;
  float vel_y = vy * kFriction;
  const bool up = (input & kInputUp) != 0, down = (input & kInputDown) != 0;
  const bool left = (input & kInputLeft) != 0, right = (input & kInputRight) != 0;
  if (up != down) {  // thrust (up && !down) or brake (!up && down), both with the OLD rot
    float s, c;
    if (__builtin_fabsf(rot) < 120.0f) {
      glibc_sincosf_small(rot, &s, &c);
    } else {
      s = glibc_sinf(rot);
      c = glibc_cosf(rot);
    }
    const float dx = kMovementSpeed * c, dy = kMovementSpeed * s;
    if (up) {
      vel_x = vel_x + dx;
      vel_y = vel_y + dy;
    } else {
      vel_x = vel_x - dx;
      vel_y = vel_y - dy;
    }
  }
  if (left && !right) rot = rem_euclid(rot - kRotationSpeed, kTwoPi);
  if (!left && right) rot = rem_euclid(rot + kRotationSpeed, kTwoPi);
  const float magnitude = __builtin_sqrtf(vel_x * vel_x + vel_y * vel_y);
  if (magnitude > kMaxSpeed) {
    vel_x = (vel_x * kMaxSpeed) / magnitude;
    vel_y = (vel_y * kMaxSpeed) / magnitude;
  }
  float nx = x + vel_x, ny = y + vel_y;
  nx = __builtin_fmaxf(nx, 0.0f);
  nx = __builtin_fminf(nx, kWindowWidth);
  ny = __builtin_fmaxf(ny, 0.0f);
  ny = __builtin_fminf(ny, kWindowHeight);
  x = nx;
  y = ny;
  vx = vel_x;
  vy = vel_y;
}

// The same step, branch-free, for +0 <= rot <= 2*pi -- the only rotations a state can hold
// (State::new starts there, rem_euclid keeps it there).  Every value is computed with the same
// IEEE ops as the general form and the branches become selects:
//   * sin/cos of the old rot: glibc_sincosf_domain (one reduction + both polynomials);
//   * thrust/brake: both vel +- d are formed, the input picks one (or neither);
//   * rotation: a = rot -+ ROTATION_SPEED lies in [-0.042, 2*pi + 0.042], so rem_euclid is the
//     Sterbenz step (|a| < 2|b|) plus the negative fix-up, never fmodf; no rotation keeps rot.
// Only the speed clamp (two correctly rounded divisions) stays a branch.
__device__ inline void advance_player_domain(float& x, float& y, float& vx, float& vy, float& rot,
                                             uint32_t input) {
  float vel_x = vx * kFriction;
  float vel_y = vy * kFriction;
  const bool up = (input & kInputUp) != 0, down = (input & kInputDown) != 0;
  const bool left = (input & kInputLeft) != 0, right = (input & kInputRight) != 0;
  float s, c;
  glibc_sincosf_domain(rot, &s, &c);
  const float dx = kMovementSpeed * c, dy = kMovementSpeed * s;
  const bool thrust = up && !down, brake = down && !up;
  const float tx = vel_x + dx, ty = vel_y + dy, bx = vel_x - dx, by = vel_y - dy;
  vel_x = thrust ? tx : (brake ? bx : vel_x);
  vel_y = thrust ? ty : (brake ? by : vel_y);
  const bool ccw = left && !right, cw = right && !left;
  const float a = ccw ? rot - kRotationSpeed : rot + kRotationSpeed;
  const float aa = __builtin_fabsf(a);
  float r = aa < kTwoPi ? a : __builtin_copysignf(aa - kTwoPi, a);
  r = r < 0.0f ? r + kTwoPi : r;
  rot = (ccw || cw) ? r : rot;
  const float magnitude = __builtin_sqrtf(vel_x * vel_x + vel_y * vel_y);
  if (magnitude > kMaxSpeed) {
    vel_x = (vel_x * kMaxSpeed) / magnitude;
    vel_y = (vel_y * kMaxSpeed) / magnitude;
  }
  float nx = x + vel_x, ny = y + vel_y;
  nx = __builtin_fmaxf(nx, 0.0f);
  nx = __builtin_fminf(nx, kWindowWidth);
  ny = __builtin_fmaxf(ny, 0.0f);
  ny = __builtin_fminf(ny, kWindowHeight);
  x = nx;
  y = ny;
  vx = vel_x;
  vy = vel_y;
}

// Correctly rounded sqrtf for the speed clamp, where s > 49: hipcc's own correctly rounded
// expansion (raw v_sqrt_f32, then the neighbour residual test) without its small-input scaling
// (s < 2^-96) and zero/inf/NaN class fix-up, neither of which applies to s > 49.
__device__ inline float sqrt_rn_above_49(float s) {
  const float m = __builtin_amdgcn_sqrtf(s);
  const uint32_t mb = __builtin_bit_cast(uint32_t, m);
  const float dn = __builtin_bit_cast(float, mb - 1u), up = __builtin_bit_cast(float, mb + 1u);
  const float rd = __builtin_fmaf(-dn, m, s);
  const float ru = __builtin_fmaf(-up, m, s);
  const float r = rd <= 0.0f ? dn : m;
  return ru > 0.0f ? up : r;
}

// Correctly rounded f32 division a / m for the speed clamp, through binary64: a reciprocal of m
// refined by two Newton steps (relative error < 2^-51) times a, rounded once to f32.  For f32
// operands the exact quotient lies at least 2^-49 (relative) away from every f32 rounding
// boundary (midpoint), so a binary64 value within 2^-50.5 of it rounds to the same f32 as the
// exact quotient: RN32(q64) == RN32(a / m).  Checked against hipcc's correctly rounded division
// on the GPU (tests/test_gpu_sincosf.py).  m is finite, > 7 here.
__device__ inline double rcp_f64_refined(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  return __builtin_fma(r, e, r);
}

// advance_player_domain with fewer instructions and the same IEEE results (v4 SyncTest kernel):
//   * thrust / brake / neither add d / -d / -0.0f: x - d == x + (-d) exactly and x + (-0) == x
//     for every x, signed zeros included, so one add replaces two adds and a select;
//   * the clamp test |v| > 7 is sqrtf(s) > 7 <=> s > 49, true for every f32 s (exhaustive host
//     KAT, tests/native/step_kat_host.c), so the square root is only taken inside the clamp, and
//     the clamp's two divisions share one refined binary64 reciprocal (rcp_f64_refined);
//   * max(min(.)) clamps become v_med3_f32: equal for every non-NaN input without -0, and a
//     position sum is never -0 (x >= +0, and x + v == 0 only as +0) nor NaN.
//   * the turn's rem_euclid on [-RS, 2pi + RS] is one add or subtract of 2pi chosen by two
//     compares (every rot in the domain, both directions: tests/native/remeuclid_kat_host.c).
typedef float ggrs_f2 __attribute__((ext_vector_type(2)));
struct NoHook {
  __device__ void operator()(float) const {}
};
// advance_player_lean with sin/cos of the old rot supplied by the caller, and a hook that sees the
// new rot before the speed clamp (the v5 kernel computes the NEXT step's sin/cos there: work that
// does not depend on this step's velocity chain, in the same basic block as it).
template <typename Hook = NoHook>
__device__ inline void advance_player_lean_sc(float& x, float& y, float& vx, float& vy, float& rot,
                                              uint32_t input, float s, float c, Hook&& hook = Hook()) {
  // the x/y pairs go through packed f32 ops (v_pk_mul_f32 / v_pk_add_f32: two IEEE f32 ops each,
  // the same roundings as the scalar ops)
  ggrs_f2 vel = ggrs_f2{vx, vy} * kFriction;
  const ggrs_f2 d = ggrs_f2{c, s} * kMovementSpeed;
  const uint32_t ud = input & (kInputUp | kInputDown), lr = input & (kInputLeft | kInputRight);
  const bool thrust = ud == kInputUp, brake = ud == kInputDown;
  vel = vel + ggrs_f2{thrust ? d.x : (brake ? -d.x : -0.0f), thrust ? d.y : (brake ? -d.y : -0.0f)};
  const bool ccw = lr == kInputLeft, turn = ccw || lr == kInputRight;
  const float a = rot + (ccw ? -kRotationSpeed : kRotationSpeed);
  // rem_euclid(a, 2pi) for a in [-RS, 2pi + RS] (host KAT over every rot in the domain,
  // tests/native/remeuclid_kat_host.c), as one add of +2pi / -2pi / +0: a - 2pi == a + (-2pi),
  // and a + 0 == a since a is never -0
  const float r = a + (a < 0.0f ? kTwoPi : (a >= kTwoPi ? -kTwoPi : 0.0f));
  rot = turn ? r : rot;
  hook(rot);
  const ggrs_f2 sq = vel * vel;
  const float mag2 = sq.x + sq.y;
  // the clamp is rare (a few % of player steps): a wave-uniform test skips it with one branch on
  // VCC instead of an exec-mask save / restore around it on every step
  const bool clamp = mag2 > kMaxSpeed * kMaxSpeed;
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(clamp) != 0, 0)) {
    if (clamp) {
      const float magnitude = sqrt_rn_above_49(mag2);
      const double rr = rcp_f64_refined((double)magnitude);
      vel.x = (float)((double)(vel.x * kMaxSpeed) * rr);
      vel.y = (float)((double)(vel.y * kMaxSpeed) * rr);
    }
  }
  const ggrs_f2 pos = ggrs_f2{x, y} + vel;
  x = __builtin_amdgcn_fmed3f(pos.x, 0.0f, kWindowWidth);
  y = __builtin_amdgcn_fmed3f(pos.y, 0.0f, kWindowHeight);
  vx = vel.x;
  vy = vel.y;
}

// One player's input decoded for advance_player_rec: everything the step derives from Input.inp
// (ex_game.rs:283-309), computed once per (frame, session, player) when the input is staged and
// shared by every chain that replays the frame (the v5 SyncTest kernel replays each frame 9 times).
//   delta: the turn's f32 addend (-RS, +RS) or +0.0 without a turn;
//   thr:   the wrap threshold, 2pi with a turn, +inf without (a non-turning rot of exactly 2pi must
//          stay 2pi: ex_game only applies rem_euclid when it turns);
//   sgn:   0 (thrust), 0x80000000 (brake: the increment's sign flips), or 0x80000000 (neither:
//          the increment is -0.0, see below);
//   keep:  0xffffffff with thrust or brake, 0 without.
struct InputRec {
  uint32_t delta, thr, sgn, keep;
};
__host__ __device__ inline InputRec make_input_rec(uint32_t input) {
  const uint32_t ud = input & (kInputUp | kInputDown), lr = input & (kInputLeft | kInputRight);
  const bool thrust = ud == kInputUp, brake = ud == kInputDown;
  const bool ccw = lr == kInputLeft, cw = lr == kInputRight;
  InputRec r;
  r.delta = ccw ? __builtin_bit_cast(uint32_t, -kRotationSpeed) : (cw ? __builtin_bit_cast(uint32_t, kRotationSpeed) : 0u);
  r.thr = (ccw || cw) ? __builtin_bit_cast(uint32_t, kTwoPi) : 0x7f800000u;
  r.sgn = thrust ? 0u : 0x80000000u;
  r.keep = (thrust || brake) ? 0xffffffffu : 0u;
  return r;
}

// advance_player_lean_sc from a staged InputRec, with the same IEEE results:
//   * velocity increment (thrust ? d : brake ? -d : -0.0f) as bit operations:
//     keep ? d ^ sgn : sgn, i.e. v_bfi(keep, d ^ sgn, sgn) -- with sgn = 0x80000000 and keep = 0
//     the increment is -0.0 exactly as the select form;
//   * turn: a = rot + delta (rot + 0.0 == rot: rot is never -0 in the domain), then
//     r = a + (a < 0 ? 2pi : (a >= thr ? -2pi : +0)): without a turn a = rot <= 2pi < thr = inf
//     and r = rot + 0 == rot; with a turn it is the one-add rem_euclid of advance_player_lean_sc.
template <typename Hook = NoHook>
__device__ inline void advance_player_rec(float& x, float& y, float& vx, float& vy, float& rot, const InputRec& in,
                                          float s, float c, Hook&& hook = Hook()) {
  ggrs_f2 vel = ggrs_f2{vx, vy} * kFriction;
  const ggrs_f2 d = ggrs_f2{c, s} * kMovementSpeed;
  // (elements copied out first: __builtin_bit_cast of an ext_vector element lvalue read element 0
  // for both -- seen with this image's hipcc, caught by the device KAT)
  const float dx = d.x, dy = d.y;
  const uint32_t ix = ((__builtin_bit_cast(uint32_t, dx) ^ in.sgn) & in.keep) | (in.sgn & ~in.keep);
  const uint32_t iy = ((__builtin_bit_cast(uint32_t, dy) ^ in.sgn) & in.keep) | (in.sgn & ~in.keep);
  vel = vel + ggrs_f2{__builtin_bit_cast(float, ix), __builtin_bit_cast(float, iy)};
  const float a = rot + __builtin_bit_cast(float, in.delta);
  rot = a + (a < 0.0f ? kTwoPi : (a >= __builtin_bit_cast(float, in.thr) ? -kTwoPi : 0.0f));
  hook(rot);
  const ggrs_f2 sq = vel * vel;
  const float mag2 = sq.x + sq.y;
  const bool clamp = mag2 > kMaxSpeed * kMaxSpeed;
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(clamp) != 0, 0)) {
    if (clamp) {
      const float magnitude = sqrt_rn_above_49(mag2);
      const double rr = rcp_f64_refined((double)magnitude);
      vel.x = (float)((double)(vel.x * kMaxSpeed) * rr);
      vel.y = (float)((double)(vel.y * kMaxSpeed) * rr);
    }
  }
  const ggrs_f2 pos = ggrs_f2{x, y} + vel;
  x = __builtin_amdgcn_fmed3f(pos.x, 0.0f, kWindowWidth);
  y = __builtin_amdgcn_fmed3f(pos.y, 0.0f, kWindowHeight);
  vx = vel.x;
  vy = vel.y;
}

// advance_player_rec from glibc_sincosf_domain_raw's unsigned values and quadrant signs: the
// velocity increment keep ? (d ^ q ^ sgn) : sgn of advance_player_rec (d = MOVEMENT_SPEED times the
// signed sin/cos) with d = MOVEMENT_SPEED x the raw value, whose sign q is applied as a bit flip
// after the multiplication (RN(k * -v) == -RN(k * v) exactly): (d & keep) ^ (sgn ^ (q & keep)).
template <typename Hook = NoHook>
__device__ inline void advance_player_rec_q(float& x, float& y, float& vx, float& vy, float& rot, const InputRec& in,
                                            float sr, float cr, uint32_t qs, uint32_t qc, Hook&& hook = Hook()) {
  ggrs_f2 vel = ggrs_f2{vx, vy} * kFriction;
  const ggrs_f2 d = ggrs_f2{cr, sr} * kMovementSpeed;
  const float dx = d.x, dy = d.y;
  const uint32_t wx = in.sgn ^ (qc & in.keep), wy = in.sgn ^ (qs & in.keep);
  const uint32_t ix = (__builtin_bit_cast(uint32_t, dx) & in.keep) ^ wx;
  const uint32_t iy = (__builtin_bit_cast(uint32_t, dy) & in.keep) ^ wy;
  vel = vel + ggrs_f2{__builtin_bit_cast(float, ix), __builtin_bit_cast(float, iy)};
  const float a = rot + __builtin_bit_cast(float, in.delta);
  rot = a + (a < 0.0f ? kTwoPi : (a >= __builtin_bit_cast(float, in.thr) ? -kTwoPi : 0.0f));
  hook(rot);
  const ggrs_f2 sq = vel * vel;
  const float mag2 = sq.x + sq.y;
  const bool clamp = mag2 > kMaxSpeed * kMaxSpeed;
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(clamp) != 0, 0)) {
    if (clamp) {
      const float magnitude = sqrt_rn_above_49(mag2);
      const double rr = rcp_f64_refined((double)magnitude);
      vel.x = (float)((double)(vel.x * kMaxSpeed) * rr);
      vel.y = (float)((double)(vel.y * kMaxSpeed) * rr);
    }
  }
  const ggrs_f2 pos = ggrs_f2{x, y} + vel;
  x = __builtin_amdgcn_fmed3f(pos.x, 0.0f, kWindowWidth);
  y = __builtin_amdgcn_fmed3f(pos.y, 0.0f, kWindowHeight);
  vx = vel.x;
  vy = vel.y;
}

__device__ inline void advance_player_lean(float& x, float& y, float& vx, float& vy, float& rot,
                                           uint32_t input) {
  float s, c;
  glibc_sincosf_domain(rot, &s, &c);
  advance_player_lean_sc(x, y, vx, vy, rot, input, s, c);
}

// N independent player steps (advance_player_lean each, the same IEEE ops in the same order per
// player) with ONE speed-clamp branch: every player's step up to the clamp test, then the rare
// clamp block for the players that need it, then every position update.  One clamp branch per
// player step would cut the N step chains into N basic blocks, which the scheduler cannot
// interleave; with one, a wave alone on its SIMD issues the N chains side by side.
// v[i] = {x, y, vx, vy, rot} bits of player step i, in[i] its input.
template <int N>
__device__ inline void advance_players_lean(uint32_t (&v)[N][5], const uint32_t (&in)[N],
                                            const SincosConsts& K = sincos_consts_vgpr()) {
  ggrs_f2 vel[N];
  float mag2[N];
  bool any = false;
#pragma unroll
  for (int i = 0; i < N; i++) {
    float rot = __builtin_bit_cast(float, v[i][4]);
    float s, c;
    glibc_sincosf_domain_k(rot, &s, &c, K);
    ggrs_f2 ve = ggrs_f2{__builtin_bit_cast(float, v[i][2]), __builtin_bit_cast(float, v[i][3])} * kFriction;
    const ggrs_f2 d = ggrs_f2{c, s} * kMovementSpeed;
    const uint32_t ud = in[i] & (kInputUp | kInputDown), lr = in[i] & (kInputLeft | kInputRight);
    const bool thrust = ud == kInputUp, brake = ud == kInputDown;
    ve = ve + ggrs_f2{thrust ? d.x : (brake ? -d.x : -0.0f), thrust ? d.y : (brake ? -d.y : -0.0f)};
    const bool ccw = lr == kInputLeft, turn = ccw || lr == kInputRight;
    const float a = rot + (ccw ? -kRotationSpeed : kRotationSpeed);
    const float r = a + (a < 0.0f ? kTwoPi : (a >= kTwoPi ? -kTwoPi : 0.0f));
    v[i][4] = __builtin_bit_cast(uint32_t, turn ? r : rot);
    const ggrs_f2 sq = ve * ve;
    mag2[i] = sq.x + sq.y;
    any = any || mag2[i] > kMaxSpeed * kMaxSpeed;
    vel[i] = ve;
  }
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(any) != 0, 0)) {
#pragma unroll
    for (int i = 0; i < N; i++) {
      if (mag2[i] > kMaxSpeed * kMaxSpeed) {
        const float magnitude = sqrt_rn_above_49(mag2[i]);
        const double rr = rcp_f64_refined((double)magnitude);
        vel[i].x = (float)((double)(vel[i].x * kMaxSpeed) * rr);
        vel[i].y = (float)((double)(vel[i].y * kMaxSpeed) * rr);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < N; i++) {
    const ggrs_f2 pos = ggrs_f2{__builtin_bit_cast(float, v[i][0]), __builtin_bit_cast(float, v[i][1])} + vel[i];
    v[i][0] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_fmed3f(pos.x, 0.0f, kWindowWidth));
    v[i][1] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_fmed3f(pos.y, 0.0f, kWindowHeight));
    const float vx = vel[i].x, vy = vel[i].y;
    v[i][2] = __builtin_bit_cast(uint32_t, vx);
    v[i][3] = __builtin_bit_cast(uint32_t, vy);
  }
}

// advance_players_lean from decoded inputs (InputRec, make_input_rec) and the raw sin/cos with its
// quadrant signs folded into the increment (advance_player_rec_q's arithmetic): the same IEEE ops.
template <int N>
__device__ inline void advance_players_rec(uint32_t (&v)[N][5], const InputRec (&in)[N],
                                           const SincosConsts& K = sincos_consts_vgpr()) {
  ggrs_f2 vel[N];
  float mag2[N];
  bool any = false;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const float rot = __builtin_bit_cast(float, v[i][4]);
    float sr, cr;
    uint32_t qs, qc;
    glibc_sincosf_domain_raw_k(rot, &sr, &cr, &qs, &qc, K);
    ggrs_f2 ve = ggrs_f2{__builtin_bit_cast(float, v[i][2]), __builtin_bit_cast(float, v[i][3])} * kFriction;
    const ggrs_f2 d = ggrs_f2{cr, sr} * kMovementSpeed;
    const float dx = d.x, dy = d.y;
    const uint32_t wx = in[i].sgn ^ (qc & in[i].keep), wy = in[i].sgn ^ (qs & in[i].keep);
    const uint32_t ix = (__builtin_bit_cast(uint32_t, dx) & in[i].keep) ^ wx;
    const uint32_t iy = (__builtin_bit_cast(uint32_t, dy) & in[i].keep) ^ wy;
    ve = ve + ggrs_f2{__builtin_bit_cast(float, ix), __builtin_bit_cast(float, iy)};
    const float a = rot + __builtin_bit_cast(float, in[i].delta);
    v[i][4] = __builtin_bit_cast(uint32_t, a + (a < 0.0f ? kTwoPi : (a >= __builtin_bit_cast(float, in[i].thr) ? -kTwoPi : 0.0f)));
    const ggrs_f2 sq = ve * ve;
    mag2[i] = sq.x + sq.y;
    any = any || mag2[i] > kMaxSpeed * kMaxSpeed;
    vel[i] = ve;
  }
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(any) != 0, 0)) {
#pragma unroll
    for (int i = 0; i < N; i++) {
      if (mag2[i] > kMaxSpeed * kMaxSpeed) {
        const float magnitude = sqrt_rn_above_49(mag2[i]);
        const double rr = rcp_f64_refined((double)magnitude);
        vel[i].x = (float)((double)(vel[i].x * kMaxSpeed) * rr);
        vel[i].y = (float)((double)(vel[i].y * kMaxSpeed) * rr);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < N; i++) {
    const ggrs_f2 pos = ggrs_f2{__builtin_bit_cast(float, v[i][0]), __builtin_bit_cast(float, v[i][1])} + vel[i];
    v[i][0] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_fmed3f(pos.x, 0.0f, kWindowWidth));
    v[i][1] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_fmed3f(pos.y, 0.0f, kWindowHeight));
    const float vx = vel[i].x, vy = vel[i].y;
    v[i][2] = __builtin_bit_cast(uint32_t, vx);
    v[i][3] = __builtin_bit_cast(uint32_t, vy);
  }
}

// Dispatch (every kernel): the lean branch-free form when every active lane's rot is in the
// domain (always, for states this engine produced), else the general form for the whole wave.
// advance_player_domain stays as the KAT reference of the lean form.
__device__ inline void advance_player(float& x, float& y, float& vx, float& vy, float& rot, uint32_t input) {
  const bool in_domain = __builtin_bit_cast(uint32_t, rot) <= kTwoPiBits;
  if (__builtin_expect(__all(in_domain), 1)) advance_player_lean(x, y, vx, vy, rot, input);
  else advance_player_general(x, y, vx, vy, rot, input);
}

// State::advance for all players.  `inputs` packs player i's Input.inp in byte i; a set bit i of
// `disconnected` marks InputStatus::Disconnected (the player spins: input 4).
template <int P>
__device__ inline void advance_state(BoxState<P>& s, uint32_t inputs, uint32_t disconnected) {
  s.w[0] = (uint32_t)((int32_t)s.w[0] + 1);
#pragma unroll
  for (int i = 0; i < P; i++) {
    uint32_t in = (disconnected >> i) & 1u ? 4u : (inputs >> (8 * i)) & 0xffu;
    float x = s.f(fld_x(P, i)), y = s.f(fld_y(P, i)), vx = s.f(fld_vx(P, i)), vy = s.f(fld_vy(P, i));
    float rot = s.f(fld_rot(P, i));
    advance_player(x, y, vx, vy, rot, in);
    s.set(fld_x(P, i), x);
    s.set(fld_y(P, i), y);
    s.set(fld_vx(P, i), vx);
    s.set(fld_vy(P, i), vy);
    s.set(fld_rot(P, i), rot);
  }
}

// State::advance through advance_player_lean only: for callers that have checked once that every
// state they step lies in the lean form's rotation domain (states this engine produced always do).
// (The players as one advance_players_rec call -- one clamp branch for all of them -- measured 1 %
// faster on the P2P flat kernel and 3 % slower on config 4's rounds kernel, 173 -> 242 VGPRs:
// not adopted, profiles/r03y.)
template <int P>
__device__ inline void advance_state_lean(BoxState<P>& s, uint32_t inputs) {
  s.w[0] = (uint32_t)((int32_t)s.w[0] + 1);
#pragma unroll
  for (int i = 0; i < P; i++) {
    float x = s.f(fld_x(P, i)), y = s.f(fld_y(P, i)), vx = s.f(fld_vx(P, i)), vy = s.f(fld_vy(P, i));
    float rot = s.f(fld_rot(P, i));
    advance_player_lean(x, y, vx, vy, rot, (inputs >> (8 * i)) & 0xffu);
    s.set(fld_x(P, i), x);
    s.set(fld_y(P, i), y);
    s.set(fld_vx(P, i), vx);
    s.set(fld_vy(P, i), vy);
    s.set(fld_rot(P, i), rot);
  }
}

// The same with the players' steps side by side (advance_players_lean: one clamp branch) and the
// sin/cos constants the caller hoisted into vector registers (sincos_consts_vgpr): for step loops
// whose many uniform values would otherwise spill the constants' scalar registers.
template <int P>
__device__ inline void advance_state_lean_k(BoxState<P>& st, uint32_t inputs, const SincosConsts& K) {
  uint32_t v[P][5], pin[P];
#pragma unroll
  for (int k = 0; k < P; k++) {
    v[k][0] = st.w[fld_x(P, k)];
    v[k][1] = st.w[fld_y(P, k)];
    v[k][2] = st.w[fld_vx(P, k)];
    v[k][3] = st.w[fld_vy(P, k)];
    v[k][4] = st.w[fld_rot(P, k)];
    pin[k] = (inputs >> (8 * k)) & 0xffu;
  }
  advance_players_lean<P>(v, pin, K);
  st.w[0] = (uint32_t)((int32_t)st.w[0] + 1);
#pragma unroll
  for (int k = 0; k < P; k++) {
    st.w[fld_x(P, k)] = v[k][0];
    st.w[fld_y(P, k)] = v[k][1];
    st.w[fld_vx(P, k)] = v[k][2];
    st.w[fld_vy(P, k)] = v[k][3];
    st.w[fld_rot(P, k)] = v[k][4];
  }
}

template <int P>
__device__ inline bool rot_in_domain(const BoxState<P>& s) {
  bool ok = true;
#pragma unroll
  for (int i = 0; i < P; i++) ok = ok && s.w[fld_rot(P, i)] <= kTwoPiBits;
  return ok;
}

// ---------------------------------------------------------------------------------------------
// Fletcher-16 of the bincode encoding, without materialising the bytes.
// fletcher16 reduces mod 255 after every byte; since x -> x mod 255 is a ring homomorphism,
//   sum1 = sum_j d_j (mod 255),  sum2 = sum_j (n - j) d_j (mod 255)  over the n = 36+20P bytes.
// A 32-bit field at byte offset o contributes dot4(w, [1,1,1,1]) to sum1 and
// dot4(w, [n-o, n-o-1, n-o-2, n-o-3]) to sum2 (weights <= 116 fit a byte): two v_dot4_u32_u8.
// The u64 length prefixes (= P) are constants folded into kSum1Const / kSum2Const.
__host__ __device__ constexpr uint32_t weights_at(int n, int o) {
  return (uint32_t)(n - o) | ((uint32_t)(n - o - 1) << 8) | ((uint32_t)(n - o - 2) << 16) |
         ((uint32_t)(n - o - 3) << 24);
}
template <int P>
struct Fletcher {
  static constexpr int n = bincode_bytes(P);
  // num_players u64 at 4, positions len at 12, velocities len at 20+8P, rotations len at 28+16P:
  // each has low byte P and seven zero bytes.
  static constexpr uint32_t kSum1Const = 4u * P;
  static constexpr uint32_t kSum2Const =
      (uint32_t)P * ((n - 4) + (n - 12) + (n - (20 + 8 * P)) + (n - (28 + 16 * P)));
};

__device__ inline uint32_t dot4_u8(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_udot4(a, b, c, false);
}

// Fletcher-16 from DOUBLED sums d1 = 2*sum1, d2 = 2*sum2 (< 2^22; accumulated with doubled byte
// weights, all <= 2*116 = 232 so they still fit v_dot4's u8 lanes).  Doubling lets the mod-255
// run on full-rate instructions: q = floor(x/255) = (2x * 0x808081) >> 32 for x < 2^31/127
// (0x808081 * 255 = 2^31 + 127), one v_mul_hi_u32_u24; 2r = 2x - 510 q, one multiply-add (exact:
// q < 2^22 / 255 < 2^14); then (r2 << 8) | r1 = (2 r2 << 7) | (2 r1 >> 1).  Replaces four
// quarter-rate 32-bit multiplies.
//
// No inline asm (round 5): these multiply-adds were `v_mad_i32_i24` inline asm until round 4, and
// the same construct in particles.h gave wrong checksums under LLVM's max-ilp scheduler.  The
// cause (hipcc -S of particles.hip at 9732acd^ with and without the asm): gfx950
// needs 3 wait states between a v_dot* that writes a VGPR and another VALU instruction reading it
// (the compiler inserts `s_nop 2` / `s_nop 1` before its own readers), but LLVM's hazard recognizer
// does not treat an inline-asm statement as a VALU reader, so max-ilp placed
//     v_dot4_u32_u8 v27, v26, s85, v27        ; last step of the a2 dot4 chain
//     v_mad_u32_u24 v32, v59, v27, v84         ; inline asm: reads v27 0 wait states later
// and the asm read a stale accumulator.  Builtins keep every consumer visible to the hazard
// recognizer (tools/asm_hazards.py checks every unit's ISA for the pattern).
__device__ inline uint32_t mulhi_u24(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)(a & 0xffffffu) * (uint64_t)(b & 0xffffffu)) >> 32);
}
// 2x - 510 q (q < 2^14), two exact forms: kMad24 a signed 24-bit multiply-add; else v_dot2c_i32_i16
// over the 16-bit lanes (q, 0) x (-510, 0).  Which one is faster depends on the kernel around it
// (profiles/r05ac, r05ad: the dot form's readers need the three DOT wait states, the mad form the
// integer multiply pipe): config 3's prefix kernel 24.3 us per launch with the mad against 26.4
// with the dot, config 4's rounds kernel 300 against 290 us, configs 2 / P2P within 1 %; the
// prefix kernel takes kMad24, the rest the dot form.
typedef short ggrs_short2 __attribute__((ext_vector_type(2)));
template <bool kMad24>
__device__ inline uint32_t sub510_small(uint32_t x2, uint32_t q) {
  if constexpr (kMad24) {
    return (uint32_t)((int32_t)x2 + __mul24((int32_t)q, -510));
  } else {
    const ggrs_short2 m = {(short)-510, (short)0};
    return (uint32_t)__builtin_amdgcn_sdot2(__builtin_bit_cast(ggrs_short2, q), m, (int32_t)x2, false);
  }
}
template <bool kMad24 = false>
__device__ inline uint32_t fletcher_from_doubled(uint32_t d1, uint32_t d2) {
  const uint32_t q1 = mulhi_u24(d1, 0x808081u), q2 = mulhi_u24(d2, 0x808081u);
  const uint32_t r1 = sub510_small<kMad24>(d1, q1), r2 = sub510_small<kMad24>(d2, q2);
  return (r2 << 7) | (r1 >> 1);
}

// Doubled sums (byte weights <= 2 * 116 = 232 still fit v_dot4's u8 lanes; d2 <= 2 * 255 * n(n+1)/2
// < 2^22 at P = 4), reduced by fletcher_from_doubled's full-rate 24-bit multiplies instead of two
// `% 255` (a quarter-rate v_mul_hi_u32 each).
template <int P>
__device__ inline uint16_t fletcher16_state(const BoxState<P>& s) {
  constexpr int n = Fletcher<P>::n;
  constexpr int F = state_fields(P);
  // two independent accumulator pairs halve the dependent v_dot4 chain
  uint32_t a1 = 2u * Fletcher<P>::kSum1Const, a2 = 2u * Fletcher<P>::kSum2Const, b1 = 0, b2 = 0;
#pragma unroll
  for (int k = 0; k < F; k += 2) {
    a1 = dot4_u8(s.w[k], 0x02020202u, a1);
    a2 = dot4_u8(s.w[k], 2u * weights_at(n, fld_offset(P, k)), a2);
    if (k + 1 < F) {
      b1 = dot4_u8(s.w[k + 1], 0x02020202u, b1);
      b2 = dot4_u8(s.w[k + 1], 2u * weights_at(n, fld_offset(P, k + 1)), b2);
    }
  }
  return (uint16_t)fletcher_from_doubled(a1 + b1, a2 + b2);
}

// Host mirror of the same closed form (used by the C ABI's host-side helpers/tests).
template <int P>
inline uint16_t fletcher16_state_host(const uint32_t* w) {
  constexpr int n = Fletcher<P>::n;
  uint64_t s1 = Fletcher<P>::kSum1Const, s2 = Fletcher<P>::kSum2Const;
  for (int k = 0; k < state_fields(P); k++) {
    uint32_t wt = weights_at(n, fld_offset(P, k));
    for (int b = 0; b < 4; b++) {
      uint32_t byte = (w[k] >> (8 * b)) & 0xff;
      s1 += byte;
      s2 += byte * ((wt >> (8 * b)) & 0xff);
    }
  }
  return (uint16_t)(((s2 % 255u) << 8) | (s1 % 255u));
}

}  // namespace ggrs
