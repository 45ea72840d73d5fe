// Probe (tools only): can the host write a fine-grained device allocation directly (a host-mapped
// VRAM window), which would let a lane batch be published into device memory?  Prints what
// hipPointerGetAttributes reports and whether a host write to the pointer reaches the device.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void read_back(const int* p, int* out) { out[0] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }

int main() {
  int* d = nullptr;
  hipError_t e = hipExtMallocWithFlags((void**)&d, 4096, hipDeviceMallocFinegrained);
  printf("hipExtMallocWithFlags(fine-grained): %s ptr %p\n", hipGetErrorString(e), (void*)d);
  if (e != hipSuccess) return 0;
  hipPointerAttribute_t a{};
  e = hipPointerGetAttributes(&a, d);
  printf("attributes: %s type %d device %d devicePointer %p hostPointer %p isManaged %d\n", hipGetErrorString(e),
         (int)a.type, a.device, a.devicePointer, a.hostPointer, (int)a.isManaged);
  void* hp = nullptr;
  e = hipHostGetDevicePointer(&hp, d, 0);
  printf("hipHostGetDevicePointer on it: %s\n", hipGetErrorString(e));
  int v = 0x1234;
  e = hipMemcpy(d, &v, 4, hipMemcpyHostToDevice);
  int* out = nullptr;
  hipMalloc(&out, 4);
  read_back<<<1, 1>>>(d, out);
  int r = 0;
  hipMemcpy(&r, out, 4, hipMemcpyDeviceToHost);
  printf("device read after memcpy: 0x%x\n", r);
  if (a.hostPointer) {
    ((volatile int*)a.hostPointer)[0] = 0x5678;
    read_back<<<1, 1>>>(d, out);
    hipMemcpy(&r, out, 4, hipMemcpyDeviceToHost);
    printf("device read after a host store through hostPointer: 0x%x\n", r);
  }
  return 0;
}
