// Dependent-chain cost per VALU instruction on one MI355X SIMD, one wave per SIMD: k independent
// chains interleaved (k = 1: every instruction waits for the previous one's result).  Build:
// hipcc --offload-arch=gfx950 -O3 -o vdep vdep.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 4096;

#define CH1(ASM, C, T) \
  for (int i = 0; i < ITER; i++) { _Pragma("unroll") for (int u = 0; u < 8; u++) asm volatile(ASM : "+" C(a[0]) : C(b)); }
#define CHK(K, ASM, C)                                                                \
  for (int i = 0; i < ITER; i++) {                                                    \
    _Pragma("unroll") for (int u = 0; u < 8 / K; u++) {                               \
      _Pragma("unroll") for (int k = 0; k < K; k++) asm volatile(ASM : "+" C(a[k]) : C(b)); \
    }                                                                                 \
  }

#define KERNEL(NAME, K, ASM, T, C)                                                    \
  __global__ __launch_bounds__(64) void NAME(double* out, int seed) {                 \
    T a[8];                                                                           \
    _Pragma("unroll") for (int k = 0; k < 8; k++) a[k] = (T)(threadIdx.x + k + 1);     \
    T b = (T)seed;                                                                    \
    CHK(K, ASM, C)                                                                    \
    double s = 0;                                                                     \
    _Pragma("unroll") for (int k = 0; k < 8; k++) s += (double)a[k];                  \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                   \
  }

KERNEL(f64_1, 1, "v_fma_f64 %0, %0, %1, %1", double, "v")
KERNEL(f64_2, 2, "v_fma_f64 %0, %0, %1, %1", double, "v")
KERNEL(f64_4, 4, "v_fma_f64 %0, %0, %1, %1", double, "v")
KERNEL(f64_8, 8, "v_fma_f64 %0, %0, %1, %1", double, "v")
KERNEL(mul64_1, 1, "v_mul_f64 %0, %0, %1", double, "v")
KERNEL(f32_1, 1, "v_fma_f32 %0, %0, %1, %1", float, "v")
KERNEL(f32_2, 2, "v_fma_f32 %0, %0, %1, %1", float, "v")
KERNEL(add32_1, 1, "v_add_f32 %0, %0, %1", float, "v")
KERNEL(add32_2, 2, "v_add_f32 %0, %0, %1", float, "v")
KERNEL(dot4_1, 1, "v_dot4_u32_u8 %0, %1, %1, %0", unsigned, "v")
KERNEL(u32_1, 1, "v_add_u32 %0, %0, %1", unsigned, "v")
KERNEL(pk_1, 1, "v_pk_add_f32 %0, %0, %1", double, "v")

// cvt round trip f32 -> f64 -> f32, dependent
__global__ __launch_bounds__(64) void cvt_1(double* out, int seed) {
  float a = (float)threadIdx.x + 1.0f;
  double d;
  for (int i = 0; i < ITER; i++) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d) : "v"(a));
      asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(a) : "v"(d));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

KERNEL(dpp_1, 1, "v_mov_b32_dpp %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf", unsigned, "v")

// v_add_f32 -> v_cmp (VCC) -> s_cbranch_vccnz (never taken): the VALU -> branch round trip
__global__ __launch_bounds__(64) void cmpbr_1(double* out, int seed) {
  float a = (float)threadIdx.x + 1.0f, b = (float)seed;
  for (int i = 0; i < ITER; i++) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      asm volatile("v_add_f32 %0, %0, %1\n\tv_cmp_lt_f32 vcc, 1e30, %0\n\ts_cbranch_vccnz 0f\n0:" : "+v"(a) : "v"(b) : "vcc");
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

// f32 -> f64 -> *c -> i32 -> f64 -> fma: the reduction head of glibc_sincosf_domain, dependent
__global__ __launch_bounds__(64) void red_1(double* out, int seed) {
  float a = (float)threadIdx.x + 1.0f;
  double d, e;
  int n;
  for (int i = 0; i < ITER; i++) {
#pragma unroll
    for (int u = 0; u < 2; u++) {
      asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d) : "v"(a));
      asm volatile("v_mul_f64 %0, %1, %1" : "=v"(e) : "v"(d));
      asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(n) : "v"(e));
      asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(e) : "v"(n));
      asm volatile("v_fma_f64 %0, %1, %1, %0" : "+v"(d) : "v"(e));
      asm volatile("v_mul_f64 %0, %0, %0" : "+v"(d));
      asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(d));
      asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(a) : "v"(d));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

// single-wave issue cost of INDEPENDENT instructions: 8 chains, 64 instructions per loop iteration
// (loop overhead 1/64 of the figure)
#define WIDE(NAME, ASM, T, C)                                                         \
  __global__ __launch_bounds__(64) void NAME(double* out, int seed) {                 \
    T a[8];                                                                           \
    _Pragma("unroll") for (int k = 0; k < 8; k++) a[k] = (T)(threadIdx.x + k + 1);     \
    T b = (T)seed;                                                                    \
    for (int i = 0; i < ITER / 8; i++) {                                              \
      _Pragma("unroll") for (int u = 0; u < 8; u++) {                                 \
        _Pragma("unroll") for (int k = 0; k < 8; k++) asm volatile(ASM : "+" C(a[k]) : C(b)); \
      }                                                                               \
    }                                                                                 \
    double s = 0;                                                                     \
    _Pragma("unroll") for (int k = 0; k < 8; k++) s += (double)a[k];                  \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                   \
  }
WIDE(w_f64fma, "v_fma_f64 %0, %0, %1, %1", double, "v")
WIDE(w_f64mul, "v_mul_f64 %0, %0, %1", double, "v")
WIDE(w_f32fma, "v_fma_f32 %0, %0, %1, %1", float, "v")
WIDE(w_f32add, "v_add_f32 %0, %0, %1", float, "v")
WIDE(w_pkmul, "v_pk_mul_f32 %0, %0, %1", double, "v")
WIDE(w_dot4, "v_dot4_u32_u8 %0, %1, %1, %0", unsigned, "v")
WIDE(w_u32add, "v_add_u32 %0, %0, %1", unsigned, "v")




typedef void (*Kf)(double*, int);
struct Case { const char* name; Kf k; };

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  Case cases[] = {{"v_fma_f64 1 chain", f64_1}, {"v_fma_f64 2 chains", f64_2}, {"v_fma_f64 4 chains", f64_4},
                  {"v_fma_f64 8 chains", f64_8}, {"v_mul_f64 1 chain", mul64_1}, {"v_fma_f32 1 chain", f32_1},
                  {"v_fma_f32 2 chains", f32_2}, {"v_add_f32 1 chain", add32_1}, {"v_add_f32 2 chains", add32_2},
                  {"v_dot4 1 chain", dot4_1}, {"v_add_u32 1 chain", u32_1}, {"v_pk_add_f32 1 chain", pk_1},
                  {"cvt f32<->f64 1 chain", cvt_1}, {"dpp row_shr 1 chain", dpp_1},
                  {"add+cmp+cbranch 1 chain (per 3)", cmpbr_1},
                  {"sincos head 1 chain (per 8)", red_1},
                  {"INDEPENDENT v_fma_f64 x8", w_f64fma}, {"INDEPENDENT v_mul_f64 x8", w_f64mul},
                  {"INDEPENDENT v_fma_f32 x8", w_f32fma}, {"INDEPENDENT v_add_f32 x8", w_f32add},
                  {"INDEPENDENT v_pk_mul_f32 x8", w_pkmul}, {"INDEPENDENT v_dot4 x8", w_dot4},
                  {"INDEPENDENT v_add_u32 x8", w_u32add}};
  double* out;
  hipMalloc(&out, sizeof(double) * 64 * 8192);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (auto& c : cases) {
    const int blocks = cus * 4;
    hipLaunchKernelGGL(c.k, dim3(blocks), dim3(64), 0, 0, out, 3);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(c.k, dim3(blocks), dim3(64), 0, 0, out, 3);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double cycles = ms / 5 * 1e-3 * 2.4e9;
    printf("%-24s %.2f cycles per instruction (one wave per SIMD)\n", c.name, cycles / ((double)ITER * 8));
  }
  return 0;
}
