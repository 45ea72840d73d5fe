// Device-side KAT of the product sincosf restatement (ggrs_amd/csrc/glibc_sincosf.h): the same
// order-independent digest oracle_sincos_digest computes from glibc libm, evaluated on the GPU.
// Test infrastructure, compiled by tests/test_gpu_sincosf.py.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "glibc_sincosf.h"
#include "box_game.h"

__device__ inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// fused != 0: the fused sincos used by the step kernel; else separate glibc_sinf / glibc_cosf.
__global__ void digest_kernel(uint32_t lo, uint32_t hi, int fused, unsigned long long* acc) {
  uint64_t local = 0;
  for (uint64_t u = (uint64_t)lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u <= hi;
       u += (uint64_t)gridDim.x * blockDim.x) {
    float f = __builtin_bit_cast(float, (uint32_t)u);
    float s, c;
    if (fused) ggrs::glibc_sincosf_small(f, &s, &c);
    else { s = ggrs::glibc_sinf(f); c = ggrs::glibc_cosf(f); }
    local += mix64((u << 32) | __builtin_bit_cast(uint32_t, s)) +
             mix64(((u << 32) | __builtin_bit_cast(uint32_t, c)) ^ 0xC05C05C05C05C05Cull);
  }
  for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(acc, (unsigned long long)local);
}

// values of sin/cos bits for an explicit list of inputs (spot checks against libm)
__global__ void values_kernel(const uint32_t* x, int n, uint32_t* s, uint32_t* c) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float f = __builtin_bit_cast(float, x[i]);
  s[i] = __builtin_bit_cast(uint32_t, ggrs::glibc_sinf(f));
  c[i] = __builtin_bit_cast(uint32_t, ggrs::glibc_cosf(f));
}

extern "C" int kat_digest(uint32_t lo, uint32_t hi, int fused, uint64_t* out) {
  unsigned long long* d;
  if (hipMalloc(&d, 8) != hipSuccess) return -1;
  if (hipMemset(d, 0, 8) != hipSuccess) return -1;
  digest_kernel<<<256 * 32, 256>>>(lo, hi, fused, d);
  if (hipGetLastError() != hipSuccess) return -2;
  if (hipMemcpy(out, d, 8, hipMemcpyDeviceToHost) != hipSuccess) return -3;
  (void)hipFree(d);
  return 0;
}

extern "C" int kat_values(const uint32_t* x, int n, uint32_t* s, uint32_t* c) {
  uint32_t *dx, *ds, *dc;
  if (hipMalloc(&dx, 4 * n) || hipMalloc(&ds, 4 * n) || hipMalloc(&dc, 4 * n)) return -1;
  if (hipMemcpy(dx, x, 4 * n, hipMemcpyHostToDevice)) return -1;
  values_kernel<<<(n + 255) / 256, 256>>>(dx, n, ds, dc);
  if (hipMemcpy(s, ds, 4 * n, hipMemcpyDeviceToHost) || hipMemcpy(c, dc, 4 * n, hipMemcpyDeviceToHost)) return -3;
  (void)hipFree(dx); (void)hipFree(ds); (void)hipFree(dc);
  return 0;
}

// sqrt_rn_above_49 (the v4 step's clamp square root) against hipcc's correctly rounded sqrtf on
// every f32 above 49 up to +inf: counts bitwise differences.
__global__ void sqrt49_kernel(unsigned long long* bad) {
  const uint32_t lo = 0x42440001u, hi = 0x7f800000u;  // next float after 49.0f .. +inf
  unsigned long long local = 0;
  for (uint64_t u = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u <= hi;
       u += (uint64_t)gridDim.x * blockDim.x) {
    const float s = __builtin_bit_cast(float, (uint32_t)u);
    local += __builtin_bit_cast(uint32_t, ggrs::sqrt_rn_above_49(s)) != __builtin_bit_cast(uint32_t, __builtin_sqrtf(s));
  }
  for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(bad, local);
}

__device__ inline uint64_t splitmix(uint64_t& st) {
  uint64_t z = (st += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// advance_player_lean vs advance_player_domain (the v3 step) on random in-domain player states
// and all 16 inputs: positions in [0, 600] x [0, 800] (edges included), velocities up to |v| ~ 13
// (both sides of the clamp, plus zero, -0 and subnormals), rotations anywhere in [0, 2*pi].
__global__ void lean_step_kernel(uint64_t seed, int iters, unsigned long long* bad) {
  uint64_t st = seed ^ ((uint64_t)(blockIdx.x * blockDim.x + threadIdx.x) << 20);
  unsigned long long local = 0;
  for (int it = 0; it < iters; it++) {
    const uint64_t a = splitmix(st), b = splitmix(st);
    float x = (float)(a & 0xffff) * (600.0f / 65535.0f);
    float y = (float)((a >> 16) & 0xffff) * (800.0f / 65535.0f);
    float vx = ((float)((a >> 32) & 0xffff) - 32768.0f) * (13.0f / 32768.0f);
    float vy = ((float)((a >> 48) & 0xffff) - 32768.0f) * (13.0f / 32768.0f);
    const uint32_t kind = (uint32_t)(b >> 60);
    if (kind == 0) vx = 0.0f;
    if (kind == 1) vy = -0.0f;
    if (kind == 2) vx = __builtin_bit_cast(float, (uint32_t)(b & 0x807fffffu));  // subnormal / zero
    if (kind == 3) x = 0.0f;
    if (kind == 4) y = 800.0f;
    const float rot = __builtin_bit_cast(float, (uint32_t)((b & 0xffffffffu) % (ggrs::kTwoPiBits + 1u)));
    for (uint32_t in = 0; in < 16; in++) {
      float x1 = x, y1 = y, vx1 = vx, vy1 = vy, r1 = rot;
      float x2 = x, y2 = y, vx2 = vx, vy2 = vy, r2 = rot;
      float x3 = x, y3 = y, vx3 = vx, vy3 = vy, r3 = rot;
      ggrs::advance_player_domain(x1, y1, vx1, vy1, r1, in);
      ggrs::advance_player_lean(x2, y2, vx2, vy2, r2, in);
      {  // the staged-record form of the v5 SyncTest kernel
        float s, c;
        ggrs::glibc_sincosf_domain(r3, &s, &c);
        ggrs::advance_player_rec(x3, y3, vx3, vy3, r3, ggrs::make_input_rec(in), s, c);
      }
      local += (__builtin_bit_cast(uint32_t, x1) != __builtin_bit_cast(uint32_t, x2)) |
               (__builtin_bit_cast(uint32_t, y1) != __builtin_bit_cast(uint32_t, y2)) |
               (__builtin_bit_cast(uint32_t, vx1) != __builtin_bit_cast(uint32_t, vx2)) |
               (__builtin_bit_cast(uint32_t, vy1) != __builtin_bit_cast(uint32_t, vy2)) |
               (__builtin_bit_cast(uint32_t, r1) != __builtin_bit_cast(uint32_t, r2));
      local += ((__builtin_bit_cast(uint32_t, x1) != __builtin_bit_cast(uint32_t, x3)) |
                (__builtin_bit_cast(uint32_t, y1) != __builtin_bit_cast(uint32_t, y3)) |
                (__builtin_bit_cast(uint32_t, vx1) != __builtin_bit_cast(uint32_t, vx3)) |
                (__builtin_bit_cast(uint32_t, vy1) != __builtin_bit_cast(uint32_t, vy3)) |
                (__builtin_bit_cast(uint32_t, r1) != __builtin_bit_cast(uint32_t, r3))) << 20;
    }
  }
  for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(bad, local);
}

// The clamp division through rcp_f64_refined against hipcc's correctly rounded f32 division:
// every f32 divisor m in (7, 16] (the clamp's magnitudes: sqrt of s in (49, 256]) against `iters`
// random numerators each -- uniform bit patterns of |a| < 2^8 (every exponent down to
// subnormals and zero, both signs) -- counting bitwise differences.
__global__ void div_kernel(uint64_t seed, int iters, unsigned long long* bad) {
  const uint32_t lo = 0x40e00001u, hi = 0x41800000u;  // next float after 7.0f .. 16.0f
  unsigned long long local = 0;
  for (uint64_t u = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u <= hi;
       u += (uint64_t)gridDim.x * blockDim.x) {
    const float m = __builtin_bit_cast(float, (uint32_t)u);
    const double r = ggrs::rcp_f64_refined((double)m);
    uint64_t st = seed ^ (u * 0x9E3779B97F4A7C15ull);
    for (int it = 0; it < iters; it++) {
      uint64_t z = (st += 0x9E3779B97F4A7C15ull);
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      z ^= z >> 31;
      const uint32_t bits = (uint32_t)z % 0x43800000u | ((uint32_t)(z >> 32) & 0x80000000u);
      const float a = __builtin_bit_cast(float, bits);
      const float q1 = (float)((double)a * r), q2 = a / m;
      local += __builtin_bit_cast(uint32_t, q1) != __builtin_bit_cast(uint32_t, q2);
    }
  }
  for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(bad, local);
}

static int run_count(int which, uint64_t seed, int iters, uint64_t* out) {
  unsigned long long* d;
  if (hipMalloc(&d, 8) != hipSuccess) return -1;
  if (hipMemset(d, 0, 8) != hipSuccess) return -1;
  if (which == 0) sqrt49_kernel<<<256 * 32, 256>>>(d);
  else if (which == 1) lean_step_kernel<<<256 * 8, 256>>>(seed, iters, d);
  else div_kernel<<<256 * 8, 256>>>(seed, iters, d);
  if (hipGetLastError() != hipSuccess) return -2;
  if (hipMemcpy(out, d, 8, hipMemcpyDeviceToHost) != hipSuccess) return -3;
  (void)hipFree(d);
  return 0;
}

extern "C" int kat_sqrt49(uint64_t* bad) { return run_count(0, 0, 0, bad); }
extern "C" int kat_lean_step(uint64_t seed, int iters, uint64_t* bad) { return run_count(1, seed, iters, bad); }
extern "C" int kat_clamp_div(uint64_t seed, int iters, uint64_t* bad) { return run_count(2, seed, iters, bad); }
