// Device-side KAT of the product sincosf restatement (ggrs_amd/csrc/glibc_sincosf.h): the same
// order-independent digest oracle_sincos_digest computes from glibc libm, evaluated on the GPU.
// Test infrastructure, compiled by tests/test_gpu_sincosf.py.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "glibc_sincosf.h"

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
