// server_probe.hip -- measures the host<->persistent-kernel round trip the lane server relies on
// (ggrs_amd/csrc/requests.hip) and checks that results written by the kernel are complete when the
// host sees a block's done flag.  Variants of the kernel's publish step:
//   0: __threadfence_system() per thread, then a release store of the done flag
//   1: wait for the block's stores (vmcnt(0)), barrier, relaxed system-scope done store
//   2: as 1, with every result store a relaxed system-scope atomic store
// Each batch a block also writes `dirty` KB of device memory (the ring saves of a real batch).
// usage: server_probe <variant> <blocks> <batches> <dirty_kb>
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                       \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

struct alignas(16) Ctl {
  int32_t epoch, quit, a, b;
  int32_t hb_polls, hb_seen, hb_started, hb_stage;  // heartbeat written by block 0
};

__global__ __launch_bounds__(64) void probe(int variant, Ctl* ctl, int32_t* done, int32_t* out, uint32_t* dev,
                                            int dirty_words, long long idle) {
  __shared__ int32_t s_e;
  const int wl = threadIdx.x;
  int32_t last = 0;
  for (;;) {
    if (wl == 0) {
      const long long t0 = wall_clock64();
      int32_t e = -1;
      int32_t polls = 0;
      if (blockIdx.x == 0) __hip_atomic_store(&ctl->hb_started, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      for (;;) {
        if (blockIdx.x == 0 && (++polls & 1023) == 0)
          __hip_atomic_store(&ctl->hb_polls, polls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 c = *(const volatile u32x4*)ctl;
        if ((int32_t)c.y) break;
        if ((int32_t)c.x != last) {
          e = (int32_t)c.x;
          if (blockIdx.x == 0) __hip_atomic_store(&ctl->hb_seen, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        if (wall_clock64() - t0 > idle) break;
        __builtin_amdgcn_s_sleep(2);
      }
      s_e = e;
    }
    __syncthreads();
    const int32_t e = s_e;
    __syncthreads();
    if (e < 0) break;
    if (blockIdx.x == 0 && wl == 0) __hip_atomic_store(&ctl->hb_stage, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* d = dev + (size_t)blockIdx.x * dirty_words;
    for (int i = wl; i < dirty_words; i += 64) d[i] = (uint32_t)(e + i);
    const int idx = blockIdx.x * 64 + wl;
    if (variant == 2) __hip_atomic_store(&out[idx], e * 1000 + wl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else out[idx] = e * 1000 + wl;
    if (blockIdx.x == 0 && wl == 0) __hip_atomic_store(&ctl->hb_stage, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (variant == 0) {
      __threadfence_system();
      __syncthreads();
      if (wl == 0) __hip_atomic_store(&done[blockIdx.x], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      __builtin_amdgcn_s_waitcnt(0x0F70);
      __syncthreads();
      if (wl == 0) __hip_atomic_store(&done[blockIdx.x], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (blockIdx.x == 0 && wl == 0) __hip_atomic_store(&ctl->hb_stage, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    last = e;
  }
}

int main(int argc, char** argv) {
  const int variant = argc > 1 ? atoi(argv[1]) : 0;
  const int blocks = argc > 2 ? atoi(argv[2]) : 64;
  const int batches = argc > 3 ? atoi(argv[3]) : 20000;
  const int dirty_kb = argc > 4 ? atoi(argv[4]) : 16;
  const int dirty_words = dirty_kb * 256;
  uint8_t* mem;
  const size_t bytes = sizeof(Ctl) + 4 * (size_t)blocks + 4 * (size_t)blocks * 64;
  CK(hipHostMalloc((void**)&mem, bytes, hipHostMallocMapped | hipHostMallocCoherent));
  memset(mem, 0, bytes);
  Ctl* ctl = (Ctl*)mem;
  int32_t* done = (int32_t*)(mem + sizeof(Ctl));
  int32_t* out = done + blocks;
  void *dctl, *ddone, *dout;
  CK(hipHostGetDevicePointer(&dctl, ctl, 0));
  CK(hipHostGetDevicePointer(&ddone, done, 0));
  CK(hipHostGetDevicePointer(&dout, out, 0));
  uint32_t* dev;
  CK(hipMalloc(&dev, 4 * (size_t)blocks * (dirty_words > 0 ? dirty_words : 1)));
  int rate = 0;
  CK(hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  probe<<<blocks, 64, 0, s>>>(variant, (Ctl*)dctl, (int32_t*)ddone, (int32_t*)dout, dev, dirty_words,
                              (long long)rate * 1000);
  CK(hipGetLastError());
  if (getenv("PROBE_DELAY_MS")) {
    const int ms = atoi(getenv("PROBE_DELAY_MS"));
    auto t = std::chrono::steady_clock::now();
    while (std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count() < ms) {}
  }
  long bad = 0;
  auto t0 = std::chrono::steady_clock::now();
  for (int ep = 1; ep <= batches; ep++) {
    __atomic_store_n(&ctl->epoch, ep, __ATOMIC_RELEASE);
    for (int b = 0; b < blocks; b++) {
      long spins = 0;
      while (__atomic_load_n(&done[b], __ATOMIC_ACQUIRE) != ep) {
        _mm_pause();
        if (++spins > 10000000L) {
          fprintf(stderr, "timeout at batch %d block %d: started %d polls %d seen %d done0 %d stage %d out0 %d\n", ep, b,
                  __atomic_load_n(&ctl->hb_started, __ATOMIC_ACQUIRE), __atomic_load_n(&ctl->hb_polls, __ATOMIC_ACQUIRE),
                  __atomic_load_n(&ctl->hb_seen, __ATOMIC_ACQUIRE), __atomic_load_n(&done[0], __ATOMIC_ACQUIRE),
                  __atomic_load_n(&ctl->hb_stage, __ATOMIC_ACQUIRE), __atomic_load_n(&out[0], __ATOMIC_ACQUIRE));
          __atomic_store_n(&ctl->quit, 1, __ATOMIC_RELEASE);
          return 2;
        }
      }
    }
    for (int i = 0; i < blocks * 64; i++)
      if (__atomic_load_n(&out[i], __ATOMIC_RELAXED) != ep * 1000 + (i & 63)) bad++;
  }
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / batches;
  __atomic_store_n(&ctl->quit, 1, __ATOMIC_RELEASE);
  CK(hipStreamSynchronize(s));
  printf("{\"variant\": %d, \"blocks\": %d, \"dirty_kb_per_block\": %d, \"us_per_batch\": %.2f, \"stale_results\": %ld}\n",
         variant, blocks, dirty_kb, us, bad);
  return 0;
}
