#include <hip/hip_runtime.h>
#include <cstdio>
#include "box_game.h"
__global__ void k(float* out) {
  const int in = threadIdx.x & 15;
  float x = 300.f, y = 400.f, vx = 1.f, vy = -2.f, rot = 0.5f;
  float x2 = x, y2 = y, vx2 = vx, vy2 = vy, r2 = rot;
  ggrs::advance_player_lean(x, y, vx, vy, rot, in);
  float s, c;
  ggrs::glibc_sincosf_domain(r2, &s, &c);
  const ggrs::InputRec rr = ggrs::make_input_rec(in);
  ggrs::advance_player_rec(x2, y2, vx2, vy2, r2, rr, s, c);
  float* o = out + threadIdx.x * 16;
  o[0] = x; o[1] = y; o[2] = vx; o[3] = vy; o[4] = rot;
  o[5] = x2; o[6] = y2; o[7] = vx2; o[8] = vy2; o[9] = r2;
  o[10] = __builtin_bit_cast(float, rr.delta); o[11] = __builtin_bit_cast(float, rr.thr);
  o[12] = __builtin_bit_cast(float, rr.sgn); o[13] = __builtin_bit_cast(float, rr.keep);
}
int main() {
  float* d; (void)hipMalloc(&d, 64 * 16 * 4);
  k<<<1, 64>>>(d);
  float h[64 * 16];
  (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int i = 0; i < 16; i++) {
    float* o = h + i * 16;
    printf("in %2d lean %g %g %g %g %g | rec %g %g %g %g %g | d %08x thr %08x sgn %08x keep %08x\n", i, o[0], o[1], o[2], o[3], o[4],
           o[5], o[6], o[7], o[8], o[9], *(unsigned*)&o[10], *(unsigned*)&o[11], *(unsigned*)&o[12], *(unsigned*)&o[13]);
  }
}
