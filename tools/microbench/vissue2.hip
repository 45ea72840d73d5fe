// Select / compare cost variants and more VALU classes (see vissue.hip).
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

KERNEL(k_cnd_vcc_init, "s_mov_b64 vcc, -1", "v_cndmask_b32 %0, %0, %1, vcc", unsigned, "v")
KERNEL(k_cnd_sgpr, "s_mov_b64 s[20:21], -1", "v_cndmask_b32_e64 %0, %0, %1, s[20:21]", unsigned, "v")
KERNEL(k_cmp_cnd, "", "v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc", unsigned, "v")
KERNEL(k_cmp_cnd_sgpr, "", "v_cmp_gt_u32_e64 s[20:21], %0, %1\n v_cndmask_b32_e64 %0, %0, %1, s[20:21]", unsigned, "v")
KERNEL(k_mul_f32, "", "v_mul_f32 %0, %0, %1", float, "v")
KERNEL(k_fmac_f32, "", "v_fmac_f32 %0, %1, %1", float, "v")
KERNEL(k_xor, "", "v_xor_b32 %0, %0, %1", unsigned, "v")
KERNEL(k_bfi, "", "v_bfi_b32 %0, %0, %1, %1", unsigned, "v")
KERNEL(k_lshl_or, "", "v_lshl_or_b32 %0, %0, 3, %1", unsigned, "v")
KERNEL(k_add3, "", "v_add3_u32 %0, %0, %1, %1", unsigned, "v")
KERNEL(k_cmp_only, "", "v_cmp_gt_u32 vcc, %0, %1", unsigned, "v")
KERNEL(k_rcp_f64, "", "v_rcp_f64 %0, %0", double, "v")
KERNEL(k_pk_fma, "", "v_pk_fma_f32 %0, %0, %1, %1", double, "v")
KERNEL(k_pk_add, "", "v_pk_add_f32 %0, %0, %1", double, "v")
KERNEL(k_mad_i24, "", "v_mad_i32_i24 %0, %0, %1, %1", unsigned, "v")
KERNEL(k_bpermute, "", "ds_bpermute_b32 %0, %1, %0\n s_waitcnt lgkmcnt(0)", unsigned, "v")

typedef void (*K)(double*, int);
struct Case { const char* name; K k; int per_iter; };

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  Case cases[] = {{"cndmask vcc (init)", k_cnd_vcc_init, 8}, {"cndmask sgpr pair", k_cnd_sgpr, 8},
                  {"cmp vcc + cndmask", k_cmp_cnd, 16}, {"cmp sgpr + cndmask", k_cmp_cnd_sgpr, 16},
                  {"v_mul_f32", k_mul_f32, 8}, {"v_fmac_f32", k_fmac_f32, 8}, {"v_xor_b32", k_xor, 8},
                  {"v_bfi_b32", k_bfi, 8}, {"v_lshl_or_b32", k_lshl_or, 8}, {"v_add3_u32", k_add3, 8},
                  {"v_cmp_gt_u32 vcc", k_cmp_only, 8}, {"v_rcp_f64", k_rcp_f64, 8},
                  {"v_pk_fma_f32", k_pk_fma, 8}, {"v_pk_add_f32", k_pk_add, 8}, {"v_mad_i32_i24", k_mad_i24, 8},
                  {"ds_bpermute + wait", k_bpermute, 8}};
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
