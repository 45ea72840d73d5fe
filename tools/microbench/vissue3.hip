// Integer multiply classes and accumulate forms (see vissue.hip).
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 4096;

#define BODY8(PRE, ASM, T, C)                                                       \
  T a0 = (T)(threadIdx.x + 1), a1 = a0 + (T)1, a2 = a0 + (T)2, a3 = a0 + (T)3,      \
    a4 = a0 + (T)4, a5 = a0 + (T)5, a6 = a0 + (T)6, a7 = a0 + (T)7;                 \
  T b = (T)seed;                                                                    \
  asm volatile(PRE);                                                                \
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

#define KERNEL(NAME, PRE, ASM, T, C) \
  __global__ __launch_bounds__(64) void NAME(double* out, int seed) { BODY8(PRE, ASM, T, C) }

KERNEL(k_mul_lo, "", "v_mul_lo_u32 %0, %0, %1", unsigned, "v")
KERNEL(k_mul_hi, "", "v_mul_hi_u32 %0, %0, %1", unsigned, "v")
KERNEL(k_mul_u24, "", "v_mul_u32_u24 %0, %0, %1", unsigned, "v")
KERNEL(k_mad_u24, "", "v_mad_u32_u24 %0, %0, %1, %1", unsigned, "v")
KERNEL(k_dot4_acc, "", "v_dot4_u32_u8 %0, %1, %1, %0", unsigned, "v")
KERNEL(k_lshl_add, "", "v_lshl_add_u32 %0, %0, 3, %1", unsigned, "v")
KERNEL(k_lshr, "", "v_lshrrev_b32 %0, 7, %0", unsigned, "v")

typedef void (*K)(double*, int);
struct Case { const char* name; K k; int per_iter; };

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  Case cases[] = {{"v_mul_lo_u32", k_mul_lo, 8}, {"v_mul_hi_u32", k_mul_hi, 8}, {"v_mul_u32_u24", k_mul_u24, 8},
                  {"v_mad_u32_u24", k_mad_u24, 8}, {"v_dot4 acc (dst=src2)", k_dot4_acc, 8},
                  {"v_lshl_add_u32", k_lshl_add, 8}, {"v_lshrrev_b32 (const)", k_lshr, 8}};
  double* out;
  (void)hipMalloc(&out, sizeof(double) * 64 * 8192);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (auto& c : cases) {
    for (int wps = 1; wps <= 2; wps *= 2) {
      const int blocks = cus * 4 * wps;
      hipLaunchKernelGGL(c.k, dim3(blocks), dim3(64), 0, 0, out, 3);
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0);
      for (int r = 0; r < 5; r++) hipLaunchKernelGGL(c.k, dim3(blocks), dim3(64), 0, 0, out, 3);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double cycles = ms / 5 * 1e-3 * 2.4e9;
      printf("%-22s waves/SIMD %d: %.2f cycles per instruction per SIMD\n", c.name, wps,
             cycles / ((double)ITER * c.per_iter * wps));
    }
  }
  return 0;
}
