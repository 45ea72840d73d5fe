// glibc 2.35 sinf/cosf, restated for gfx950 device code (and host, for the CPU KAT).
//
// Why this exists: the reference's box game (`examples/ex_game/ex_game.rs:294-300`) calls Rust
// `f32::cos`/`f32::sin`, which lower to the platform libm `cosf`/`sinf`.  On the reference's CPU
// path (this image: glibc 2.35, x86-64) those are NOT correctly rounded (SURVEY.md finding 2), so a
// device kernel is bit-exact with the reference only if it evaluates glibc's own algorithm.
//
// Algorithm (glibc sysdeps/ieee754/flt-32 s_sinf.c / s_cosf.c / sincosf.h / sincosf_data.c, the
// ARM "optimized-routines" single-precision sin/cos), evaluated entirely in binary64:
//   |y| <  2^-12 : sinf(y) = y,  cosf(y) = 1
//   |y| <  pi/4  : odd/even polynomial in x = (double)y
//   |y| <  120   : reduce_fast: n = round(x * 2/pi) via the 2^24-scaled int trick, x -= n*pi/2
//   otherwise    : reduce_large: 32x96-bit fixed-point multiply by a 192-bit table of 4/pi
// then sin/cos polynomials chosen by quadrant n; the table swaps the cosine polynomial's sign for
// quadrants with bit 1 set.  x86-64 glibc builds the non-TOINT_INTRINSICS variant.  Every product
// and sum below is an explicitly chosen binary64 op (fma exactly where the FMA build fuses, see
// below), so the file must be compiled with -ffp-contract=off (the pragma enforces it locally).
//
// Verified exhaustively against this image's /lib/x86_64-linux-gnu/libm.so.6 on ALL 2^32 f32
// inputs (sin, cos and the fused form; tests/test_sincosf_kat.py, CPU) and on the device over
// every f32 in [0, 2*pi] (tests/test_gpu_sincosf.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace ggrs {

// quadrant sign of the reduced argument: sign[n & 3] = {1, -1, -1, 1}
__host__ __device__ inline double quadrant_sign(int n) { return ((n + 1) & 2) ? -1.0 : 1.0; }

__host__ __device__ inline uint32_t f32_bits(float f) { return __builtin_bit_cast(uint32_t, f); }
__host__ __device__ inline uint32_t abstop12(float f) { return (f32_bits(f) >> 20) & 0x7ff; }

// __sincosf_table[0] coefficients ([1] has c0..c4 negated and identical s1..s3); hpi_inv is
// 2/pi * 2^24 (the non-TOINT_INTRINSICS form), hpi = pi/2, pi63 = pi * 2^-63.
#define GGRS_SC_C0 0x1p0
#define GGRS_SC_C1 -0x1.ffffffd0c621cp-2
#define GGRS_SC_C2 0x1.55553e1068f19p-5
#define GGRS_SC_C3 -0x1.6c087e89a359dp-10
#define GGRS_SC_C4 0x1.99343027bf8c3p-16
#define GGRS_SC_S1 -0x1.555545995a603p-3
#define GGRS_SC_S2 0x1.1107605230bc4p-7
#define GGRS_SC_S3 -0x1.994eb3774cf24p-13
#define GGRS_SC_HPI_INV 0x1.45F306DC9C883p+23
#define GGRS_SC_HPI 0x1.921FB54442D18p0
#define GGRS_SC_PI63 0x1.921FB54442D18p-62

// Which variant: this image's libm.so.6 dispatches sinf/cosf through an IFUNC to the build
// compiled with -mfma -mavx2 (`__sinf_fma`), in which gcc contracted every `a + b*c` of the C
// source into one fused multiply-add (and the reduction `x - n*hpi` into one fnmadd).  On
// [0, 2*pi] the FMA and SSE2 builds agree bit for bit; on the rest of
// |x| < 120 only the FMA form matches the library the reference links (34 of 2^32 inputs differ), so the
// FMA form is restated here with explicit fma (one v_fma_f64 each on gfx950).

// The sine and cosine polynomials of sinf_poly (sincosf.h) for table[0].  table[1] negates the
// cosine coefficients; fma(a,-b,-c) == -fma(a,b,c) exactly, so table[1]'s cosine is -cos_poly.
__host__ __device__ inline double sin_poly(double x, double x2) {
  double x3 = x * x2;
  double s1 = __builtin_fma(x2, GGRS_SC_S3, GGRS_SC_S2);
  double x7 = x3 * x2;
  double s = __builtin_fma(x3, GGRS_SC_S1, x);
  return __builtin_fma(x7, s1, s);
}
__host__ __device__ inline double cos_poly(double x2) {
  double x4 = x2 * x2;
  double c2 = __builtin_fma(x2, GGRS_SC_C4, GGRS_SC_C3);
  double c1 = __builtin_fma(x2, GGRS_SC_C1, GGRS_SC_C0);
  double x6 = x4 * x2;
  double c = __builtin_fma(x4, GGRS_SC_C2, c1);
  return __builtin_fma(x6, c2, c);
}

// sinf_poly(x, x2, p, n) of sincosf.h: n even -> sine polynomial, odd -> cosine polynomial;
// `neg_cos` selects __sincosf_table[1].
__host__ __device__ inline float sinf_poly(double x, double x2, bool neg_cos, int n) {
  if ((n & 1) == 0) return (float)sin_poly(x, x2);
  double c = cos_poly(x2);
  return (float)(neg_cos ? -c : c);
}

// reduce_fast of sincosf.h (valid for |x| < 120); FMA build: x - n*hpi is one fnmadd.
__host__ __device__ inline double reduce_fast(double x, int* np) {
  double r = x * GGRS_SC_HPI_INV;
  int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return __builtin_fma(-(double)n, GGRS_SC_HPI, x);
}

// reduce_large of sincosf.h: 4/pi to 192 bits (__inv_pio4 of sincosf_data.c).
__host__ __device__ inline double reduce_large(uint32_t xi, int* np) {
  // __inv_pio4[i] = bits [8i, 8i+32) of the 4/pi binary expansion
  const uint32_t inv_pio4[24] = {
      0xa2u,       0xa2f9u,     0xa2f983u,   0xa2f9836eu, 0xf9836e4eu, 0x836e4e44u,
      0x6e4e4415u, 0x4e441529u, 0x441529fcu, 0x1529fc27u, 0x29fc2757u, 0xfc2757d1u,
      0x2757d1f5u, 0x57d1f534u, 0xd1f534ddu, 0xf534ddc0u, 0x34ddc0dbu, 0xddc0db62u,
      0xc0db6295u, 0xdb629599u, 0x6295993cu, 0x95993c43u, 0x993c4390u, 0x3c439041u};
  const uint32_t* arr = &inv_pio4[(xi >> 26) & 15];
  int shift = (xi >> 23) & 7;
  xi = (xi & 0xffffff) | 0x800000;
  xi <<= shift;
  uint64_t res0 = (uint64_t)(uint32_t)(xi * arr[0]);
  uint64_t res1 = (uint64_t)xi * arr[4];
  uint64_t res2 = (uint64_t)xi * arr[8];
  res0 = (res2 >> 32) | (res0 << 32);
  res0 += res1;
  uint64_t n = (res0 + (1ULL << 61)) >> 62;
  res0 -= n << 62;
  double x = (double)(int64_t)res0;
  *np = (int)n;
  return x * GGRS_SC_PI63;
}

// sinf(y) exactly as glibc 2.35 (finite y; NaN/Inf return NaN like __math_invalidf).
__host__ __device__ inline float glibc_sinf(float y) {
  double x = y;
  int n;
  if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {  // |y| < pi/4
    double s = x * x;
    if (abstop12(y) < abstop12(0x1p-12f)) return y;
    return sinf_poly(x, s, false, 0);
  } else if (abstop12(y) < abstop12(120.0f)) {
    x = reduce_fast(x, &n);
    double s = quadrant_sign(n);
    return sinf_poly(x * s, x * x, (n & 2) != 0, n);
  } else if (abstop12(y) < abstop12(__builtin_inff())) {
    uint32_t xi = f32_bits(y);
    int sign = xi >> 31;
    x = reduce_large(xi, &n);
    double s = quadrant_sign(n + sign);
    return sinf_poly(x * s, x * x, ((n + sign) & 2) != 0, n);
  }
  return __builtin_nanf("");
}

// cosf(y) exactly as glibc 2.35.
__host__ __device__ inline float glibc_cosf(float y) {
  double x = y;
  int n;
  if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
    double x2 = x * x;
    if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
    return sinf_poly(x, x2, false, 1);
  } else if (abstop12(y) < abstop12(120.0f)) {
    x = reduce_fast(x, &n);
    double s = quadrant_sign(n);
    return sinf_poly(x * s, x * x, (n & 2) != 0, n ^ 1);
  } else if (abstop12(y) < abstop12(__builtin_inff())) {
    uint32_t xi = f32_bits(y);
    int sign = xi >> 31;
    x = reduce_large(xi, &n);
    double s = quadrant_sign(n + sign);
    return sinf_poly(x * s, x * x, ((n + sign) & 2) != 0, n ^ 1);
  }
  return __builtin_nanf("");
}

// Fused sin+cos of one argument: the SAME two results as glibc_sinf(y)/glibc_cosf(y) (both
// reduce identically), sharing the reduction and both polynomials.  With S = sin_poly(x),
// C = cos_poly(x) of the reduced x, quadrant q = n & 3 gives (sin, cos) =
// (S, C), (C, -S), (-S, -C), (-C, S): every op in the polynomials is sign-symmetric under
// round-to-nearest, so the sign flips of glibc's sign[]/table[1] are exact negations.
// Valid for finite |y| < 120, which covers every reachable ship rotation (rot stays in
// [0, 2*pi] by rem_euclid, ex_game.rs:303-309).
__host__ __device__ inline void glibc_sincosf_small(float y, float* sinp, float* cosp) {
  double x = y;
  if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
    if (abstop12(y) < abstop12(0x1p-12f)) {
      *sinp = y;
      *cosp = 1.0f;
      return;
    }
    double x2 = x * x;
    *sinp = (float)sin_poly(x, x2);
    *cosp = (float)cos_poly(x2);
    return;
  }
  int n;
  x = reduce_fast(x, &n);
  double x2 = x * x;
  float S = (float)sin_poly(x, x2);
  float C = (float)cos_poly(x2);
  float sv = (n & 1) ? C : S;
  float cv = (n & 1) ? -S : C;
  bool flip = (n & 2) != 0;
  *sinp = flip ? -sv : sv;
  *cosp = flip ? -cv : cv;
}

// Branch-free sin+cos for the ship-rotation domain +0 <= y <= 2*pi (bit patterns
// 0x00000000 .. 0x40c90fdb), the only values rot takes (ex_game.rs:303-309 keeps it there by
// rem_euclid; State::new starts it there).  On that domain glibc's small-argument paths agree
// with the reduction path: for y < 0.75 (the |y| < pi/4 test of abstop12) reduce_fast yields
// n = 0 and x - 0*hpi = x exactly, and the |y| < 2^-12 shortcut (sin = y, cos = 1) is what the
// polynomials round to there.  Verified against libm on every f32 of the domain
// (tests/native/sincosf_kat_host.cpp, bad_domain).
//
// The reduction without integer conversions: reduce_fast's n = ((int32_t)(x * hpi_inv) +
// 2^23) >> 24 is floor(x * hpi_inv * 2^-24 + 1/2) for x >= 0 (floor((floor(r) + k) / m) =
// floor((r + k) / m) for integers k, m), and on this domain it equals round-to-nearest of the
// exact product x * (hpi_inv * 2^-24): fma(x, hpi_inv * 2^-24, 1.5 * 2^52) leaves n in the low
// mantissa bits (n <= 4, so the low dword IS n) and subtracting 1.5 * 2^52 gives (double)n
// exactly.  Checked on every f32 of the domain (n and the reduced x both identical: the host KAT
// below compares the whole function with libm).  On gfx950 this replaces v_mul_f64 +
// v_cvt_i32_f64 + v_add_u32 + v_ashrrev + v_cvt_f64_i32 (the two conversions cost ~40 cycles of
// dependent latency each, tools/microbench/vdep.hip) with v_fma_f64 + v_add_f64.
__host__ __device__ inline void glibc_sincosf_domain(float y, float* sinp, float* cosp) {
  const double xin = (double)y;
  const double t = __builtin_fma(xin, GGRS_SC_HPI_INV * 0x1p-24, 0x1.8p52);
  const uint32_t n = (uint32_t)__builtin_bit_cast(uint64_t, t);
  const double x = __builtin_fma(-(t - 0x1.8p52), GGRS_SC_HPI, xin);
  const double x2 = x * x;
  const float S = (float)sin_poly(x, x2);
  const float C = (float)cos_poly(x2);
  const float sv = (n & 1) ? C : S;
  const float cv = (n & 1) ? -S : C;
  const bool flip = (n & 2) != 0;
  *sinp = flip ? -sv : sv;
  *cosp = flip ? -cv : cv;
}
constexpr uint32_t kTwoPiBits = 0x40c90fdbu;  // bits of (float)(2*pi)

// glibc_sincosf_domain with its binary64 constants held in (vector) registers chosen by the
// caller: the same operations in the same order, so the same results.  A loop that runs several
// sin/cos per iteration beside many uniform values otherwise keeps these ten 64-bit constants in
// scalar registers, where they spill to VGPR lanes and come back through v_readlane each use.
struct SincosConsts {
  double hpi_inv24, magic, hpi, s1, s2, s3, c1, c2, c3, c4;
};
__host__ __device__ inline double in_vgpr(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(x));
#endif
  return x;
}
__host__ __device__ inline SincosConsts sincos_consts_vgpr() {
  return SincosConsts{in_vgpr(GGRS_SC_HPI_INV * 0x1p-24), in_vgpr(0x1.8p52), in_vgpr(GGRS_SC_HPI),
                      in_vgpr(GGRS_SC_S1),  in_vgpr(GGRS_SC_S2), in_vgpr(GGRS_SC_S3),
                      in_vgpr(GGRS_SC_C1),  in_vgpr(GGRS_SC_C2), in_vgpr(GGRS_SC_C3), in_vgpr(GGRS_SC_C4)};
}
__host__ __device__ inline void glibc_sincosf_domain_k(float y, float* sinp, float* cosp, const SincosConsts& K) {
  const double xin = (double)y;
  const double t = __builtin_fma(xin, K.hpi_inv24, K.magic);
  const uint32_t n = (uint32_t)__builtin_bit_cast(uint64_t, t);
  const double x = __builtin_fma(-(t - K.magic), K.hpi, xin);
  const double x2 = x * x;
  // sin_poly / cos_poly with the constants from K (the same fma / mul tree)
  const double x3 = x * x2;
  const double s1 = __builtin_fma(x2, K.s3, K.s2);
  const double x7 = x3 * x2;
  const double ss = __builtin_fma(x3, K.s1, x);
  const float S = (float)__builtin_fma(x7, s1, ss);
  const double x4 = x2 * x2;
  const double c2 = __builtin_fma(x2, K.c4, K.c3);
  const double c1 = __builtin_fma(x2, K.c1, GGRS_SC_C0);
  const double x6 = x4 * x2;
  const double cc = __builtin_fma(x4, K.c2, c1);
  const float C = (float)__builtin_fma(x6, c2, cc);
  const float sv = (n & 1) ? C : S;
  const float cv = (n & 1) ? -S : C;
  const bool flip = (n & 2) != 0;
  *sinp = flip ? -sv : sv;
  *cosp = flip ? -cv : cv;
}

// glibc_sincosf_domain's two polynomial values before the quadrant's swap and signs are applied,
// for callers that fold the signs into later bit operations: with S, C the polynomials and n the
// quadrant, sin = sr ^ qs and cos = cr ^ qc as bits, where sr = n odd ? C : S, cr = n odd ? S : C,
// qs = bit 1 of n at bit 31, qc = (bit 0 ^ bit 1) of n at bit 31 (the four quadrants' (sin, cos):
// (S, C), (C, -S), (-S, -C), (-C, S)).  The swap is a bit-field select on a mask from n's bit 0.
// The constants come from K (glibc_sincosf_domain_k's operations, in the same order).
__host__ __device__ inline void glibc_sincosf_domain_raw_k(float y, float* sr, float* cr, uint32_t* qs, uint32_t* qc,
                                                           const SincosConsts& K) {
  const double xin = (double)y;
  const double t = __builtin_fma(xin, K.hpi_inv24, K.magic);
  const uint32_t n = (uint32_t)__builtin_bit_cast(uint64_t, t);
  const double x = __builtin_fma(-(t - K.magic), K.hpi, xin);
  const double x2 = x * x;
  const double x3 = x * x2;
  const double s1 = __builtin_fma(x2, K.s3, K.s2);
  const double x7 = x3 * x2;
  const double ss = __builtin_fma(x3, K.s1, x);
  const uint32_t S = __builtin_bit_cast(uint32_t, (float)__builtin_fma(x7, s1, ss));
  const double x4 = x2 * x2;
  const double c2 = __builtin_fma(x2, K.c4, K.c3);
  const double c1 = __builtin_fma(x2, K.c1, GGRS_SC_C0);
  const double x6 = x4 * x2;
  const double cc = __builtin_fma(x4, K.c2, c1);
  const uint32_t C = __builtin_bit_cast(uint32_t, (float)__builtin_fma(x6, c2, cc));
  // the swap as xor-selects: gfx950 codegen is one v_bfe_i32 (all ones in odd quadrants) and two
  // v_bitop3_b32 -- the instruction count of the round-4 inline asm (v_bfe_i32 + two v_bfi_b32),
  // with every consumer visible to the compiler's hazard recognizer (box_game.h,
  // fletcher_from_doubled, says why that matters)
  const uint32_t m = 0u - (n & 1u);  // all ones in odd quadrants
  const uint32_t sc = S ^ C;
  *sr = __builtin_bit_cast(float, S ^ (sc & m));
  *cr = __builtin_bit_cast(float, C ^ (sc & m));
  const uint32_t l30 = n << 30, l31 = n << 31;
  *qs = l30 & 0x80000000u;
  *qc = (l30 ^ l31) & 0x80000000u;
}
// the constants as literals (folded into the instructions or scalar registers)
constexpr SincosConsts kSincosLiteral{GGRS_SC_HPI_INV * 0x1p-24, 0x1.8p52, GGRS_SC_HPI, GGRS_SC_S1, GGRS_SC_S2,
                                      GGRS_SC_S3, GGRS_SC_C1, GGRS_SC_C2, GGRS_SC_C3, GGRS_SC_C4};
__host__ __device__ inline void glibc_sincosf_domain_raw(float y, float* sr, float* cr, uint32_t* qs, uint32_t* qc) {
  glibc_sincosf_domain_raw_k(y, sr, cr, qs, qc, kSincosLiteral);
}

}  // namespace ggrs
