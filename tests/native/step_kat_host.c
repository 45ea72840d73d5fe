/* Host KAT behind advance_player_lean's clamp test (ggrs_amd/csrc/box_game.h): for EVERY f32 s,
 * sqrtf(s) > 7.0f (the reference's `magnitude > MAX_SPEED`, ex_game.rs:313-317, with correctly
 * rounded sqrtf) has the same truth value as s > 49.0f.  Test infrastructure, compiled and run by
 * tests/test_step_kat.py.  Prints "bad <count>". */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int nthreads = 8;
static uint64_t bad[64];

static void* work(void* arg) {
  const int id = (int)(intptr_t)arg;
  const uint64_t span = (1ull << 32) / (uint64_t)nthreads;
  const uint64_t lo = span * (uint64_t)id, hi = id == nthreads - 1 ? (1ull << 32) : lo + span;
  uint64_t n = 0;
  for (uint64_t u = lo; u < hi; u++) {
    const uint32_t b = (uint32_t)u;
    float s;
    memcpy(&s, &b, 4);
    n += (sqrtf(s) > 7.0f) != (s > 49.0f);
  }
  bad[id] = n;
  return NULL;
}

int main(int argc, char** argv) {
  if (argc > 1) nthreads = atoi(argv[1]);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
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
