/* Host KAT behind advance_player_lean's turn (ggrs_amd/csrc/box_game.h): for EVERY f32 rotation
 * rot in the lean step's domain [+0, 2pi] (bits 0 .. 0x40C90FDB) and both turn directions, the
 * branch-light form
 *     a = rot -/+ ROTATION_SPEED;  r = a < 0 ? a + 2pi : (a >= 2pi ? a - 2pi : a)
 * and its one-add form r = a + (a < 0 ? 2pi : (a >= 2pi ? -2pi : +0)) (what box_game.h runs)
 * equal the reference's f32::rem_euclid(a, 2pi) (ex_game.rs:300-306; Rust: r = a % b, then
 * r < 0 ? r + |b| : r, with % = fmodf), bit for bit.  Test infrastructure, compiled and run by
 * tests/test_step_kat.py.  Prints "bad <count>". */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int nthreads = 8;
static uint64_t bad[64];
static const uint32_t kTwoPiBits = 0x40C90FDBu;

static uint32_t bits(float f) {
  uint32_t b;
  memcpy(&b, &f, 4);
  return b;
}

static float rem_euclid_ref(float a, float b) {
  float r = fmodf(a, b);
  return r < 0.0f ? r + fabsf(b) : r;
}

static void* work(void* arg) {
  const int id = (int)(intptr_t)arg;
  const volatile float two_pi_v = 2.0f * 3.14159265358979323846f;
  const volatile float rs_v = 2.5f / 60.0f;
  const float two_pi = two_pi_v, rs = rs_v;
  const uint64_t n_all = (uint64_t)kTwoPiBits + 1;
  const uint64_t span = n_all / (uint64_t)nthreads;
  const uint64_t lo = span * (uint64_t)id, hi = id == nthreads - 1 ? n_all : lo + span;
  uint64_t n = 0;
  for (uint64_t u = lo; u < hi; u++) {
    const uint32_t b = (uint32_t)u;
    float rot;
    memcpy(&rot, &b, 4);
    for (int dir = 0; dir < 2; dir++) {
      const float a = dir ? rot + rs : rot - rs;
      const float mine = a < 0.0f ? a + two_pi : (a >= two_pi ? a - two_pi : a);
      const volatile float zero = 0.0f;
      const float one_add = a + (a < 0.0f ? two_pi : (a >= two_pi ? -two_pi : zero));
      const uint32_t ref = bits(rem_euclid_ref(a, two_pi));
      n += (bits(mine) != ref) + (bits(one_add) != ref);
    }
  }
  bad[id] = n;
  return NULL;
}

int main(int argc, char** argv) {
  if (argc > 1) nthreads = atoi(argv[1]);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  if (bits(2.0f * 3.14159265358979323846f) != kTwoPiBits) {
    printf("bad constant\n");
    return 1;
  }
  pthread_t th[64];
  for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, work, (void*)(intptr_t)i);
  uint64_t total = 0;
  for (int i = 0; i < nthreads; i++) {
    pthread_join(th[i], NULL);
    total += bad[i];
  }
  printf("bad %llu\n", (unsigned long long)total);
  return total != 0;
}
