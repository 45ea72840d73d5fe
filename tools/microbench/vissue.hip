// VALU issue cost per instruction class on one MI355X SIMD, with 1 and 2 waves per SIMD:
// each wave runs ITER x 8 independent instances of one instruction (8 accumulators, no
// dependency between consecutive instructions), the kernel time gives cycles per instruction
// per SIMD.  Build: hipcc --offload-arch=gfx950 -O3 -o vissue vissue.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int ITER = 4096;

#define BODY8(ASM, T, C)                                                            \
  T a0 = (T)(threadIdx.x + 1), a1 = a0 + (T)1, a2 = a0 + (T)2, a3 = a0 + (T)3,      \
    a4 = a0 + (T)4, a5 = a0 + (T)5, a6 = a0 + (T)6, a7 = a0 + (T)7;                 \
  T b = (T)seed;                                                                    \
  for (int i = 0; i < ITER; i++) {                                                  \
    asm volatile(ASM : "+" C(a0) : C(b));                                           \
    asm volatile(ASM : "+" C(a1) : C(b));                                           \
    asm volatile(ASM : "+" C(a2) : C(b));                                           \
    asm volatile(ASM : "+" C(a3) : C(b));                                           \
    asm volatile(ASM : "+" C(a4) : C(b));                                           \
    asm volatile(ASM : "+" C(a5) : C(b));                                           \
    asm volatile(ASM : "+" C(a6) : C(b));                                           \
    asm volatile(ASM : "+" C(a7) : C(b));                                           \
  }                                                                                 \
  out[blockIdx.x * blockDim.x + threadIdx.x] = (double)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);

#define KERNEL(NAME, ASM, T, C) \
  __global__ __launch_bounds__(64) void NAME(double* out, int seed) { BODY8(ASM, T, C) }

KERNEL(k_add_f32, "v_add_f32 %0, %0, %1", float, "v")
KERNEL(k_fma_f32, "v_fma_f32 %0, %0, %1, %1", float, "v")
KERNEL(k_mul_f64, "v_mul_f64 %0, %0, %1", double, "v")
KERNEL(k_fma_f64, "v_fma_f64 %0, %0, %1, %1", double, "v")
KERNEL(k_add_u32, "v_add_u32 %0, %0, %1", unsigned, "v")
KERNEL(k_and_b32, "v_and_b32 %0, %0, %1", unsigned, "v")
KERNEL(k_dot4, "v_dot4_u32_u8 %0, %0, %1, %0", unsigned, "v")
KERNEL(k_mulhi24, "v_mul_hi_u32_u24 %0, %0, %1", unsigned, "v")
KERNEL(k_med3, "v_med3_f32 %0, %0, %1, %1", float, "v")
__global__ __launch_bounds__(64) void k_cvt_f64_f32(double* out, int seed) {
  double a[8];
  float b = seed + threadIdx.x;
  for (int k = 0; k < 8; k++) a[k] = 0;
  for (int i = 0; i < ITER; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      double t;
      asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(t) : "v"(b));
      asm volatile("" : "+v"(a[k]) : "v"(t));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a[0] + a[7];
}
KERNEL(k_sqrt_f32, "v_sqrt_f32 %0, %0", float, "v")
KERNEL(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc", unsigned, "v")
KERNEL(k_dpp_add, "v_add_u32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf", unsigned, "v")
__global__ __launch_bounds__(64) void k_salu(double* out, int seed) {
  unsigned a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3, a4 = seed + 4, a5 = seed + 5, a6 = seed + 6,
           a7 = seed + 7, b = seed * 3;
  for (int i = 0; i < ITER; i++) {
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(a0) : "s"(b));
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(a1) : "s"(b));
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(a2) : "s"(b));
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(a3) : "s"(b));
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(a4) : "s"(b));
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(a5) : "s"(b));
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(a6) : "s"(b));
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(a7) : "s"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// the same instruction counts, with the VALU op mix interleaved with scalar ops: VALU add, SALU
__global__ __launch_bounds__(64) void k_mix_valu_salu(double* out, int seed) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  unsigned s0 = seed, s1 = seed + 1;
  float b = seed;
  for (int i = 0; i < ITER; i++) {
    asm volatile("v_add_f32 %0, %0, %1" : "+v"(a0) : "v"(b));
    asm volatile("s_add_u32 %0, %0, 3" : "+s"(s0));
    asm volatile("v_add_f32 %0, %0, %1" : "+v"(a1) : "v"(b));
    asm volatile("s_add_u32 %0, %0, 5" : "+s"(s1));
    asm volatile("v_add_f32 %0, %0, %1" : "+v"(a2) : "v"(b));
    asm volatile("s_add_u32 %0, %0, 3" : "+s"(s0));
    asm volatile("v_add_f32 %0, %0, %1" : "+v"(a3) : "v"(b));
    asm volatile("s_add_u32 %0, %0, 5" : "+s"(s1));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + s0 + s1;
}

typedef void (*K)(double*, int);
struct Case { const char* name; K k; int per_iter; };

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  Case cases[] = {{"v_add_f32", k_add_f32, 8}, {"v_fma_f32", k_fma_f32, 8}, {"v_mul_f64", k_mul_f64, 8},
                  {"v_fma_f64", k_fma_f64, 8}, {"v_add_u32", k_add_u32, 8}, {"v_and_b32", k_and_b32, 8},
                  {"v_dot4_u32_u8", k_dot4, 8}, {"v_mul_hi_u32_u24", k_mulhi24, 8}, {"v_med3_f32", k_med3, 8},
                  {"v_cvt_f64_f32", k_cvt_f64_f32, 8}, {"v_sqrt_f32", k_sqrt_f32, 8},
                  {"v_cndmask_b32", k_cndmask, 8}, {"v_add_u32_dpp", k_dpp_add, 8}, {"s_add_u32", k_salu, 8},
                  {"mix 4 VALU + 4 SALU", k_mix_valu_salu, 8}};
  double* out;
  hipMalloc(&out, sizeof(double) * 64 * 8192);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int clk_khz = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs %d, clock %.0f MHz (nominal)\n", cus, clk_khz / 1e3);
  for (auto& c : cases) {
    for (int wps = 1; wps <= 4; wps *= 2) {
      const int blocks = cus * 4 * wps;
      printf("%s wps %d ...\n", c.name, wps);
      hipLaunchKernelGGL(c.k, dim3(blocks), dim3(64), 0, 0, out, 3);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int r = 0; r < 5; r++) hipLaunchKernelGGL(c.k, dim3(blocks), dim3(64), 0, 0, out, 3);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double cycles = ms / 5 * 1e-3 * 2.4e9;  // at 2.4 GHz
      const double per = cycles / ((double)ITER * c.per_iter * wps);
      printf("%-22s waves/SIMD %d: %.2f cycles per instruction per SIMD (%.3f ms)\n", c.name, wps, per, ms / 5);
    }
  }
  return 0;
}
