/* Host sanitizer driver for the oracle (TEST INFRASTRUCTURE): built with
 * -fsanitize=address,undefined by tests/test_oracle_sanitized.py, runs the SyncTest, P2P replay and
 * particle-world restatements on seeded inputs and prints digests the test compares with the
 * normally built oracle. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  int32_t num_players, max_prediction, check_distance, input_delay;
  int32_t predictor, random_checksums;
  uint64_t rng_seed;
  int32_t corrupt_frame, pad_;
} Cfg;
typedef struct {
  int32_t status, frames_done, mismatch_frame;
  uint64_t mismatch_mask;
  int64_t n_load, n_save, n_advance, n_resim;
} Res;

int oracle_synctest_run(const Cfg*, int32_t, const uint8_t*, uint16_t*, uint8_t*, int64_t, int32_t*, uint8_t*,
                        int32_t*, uint16_t*, uint8_t*, Res*);
void oracle_gen_inputs(uint64_t, int64_t, int64_t, int, uint8_t*);
int oracle_particles_synctest_run(int32_t, int32_t, int32_t, int32_t, uint64_t, int32_t, const uint8_t*, int32_t,
                                  uint16_t*, uint8_t*, int32_t*, uint16_t*, uint8_t*, Res*);
int oracle_p2p_replay(int32_t, const uint8_t*, int32_t, int32_t, int32_t, const uint8_t*, const uint8_t*, uint8_t*,
                      uint16_t*, uint8_t*);
void oracle_state_new_bytes(int32_t, uint8_t*);
uint16_t oracle_fletcher16(const uint8_t*, size_t);

int main(void) {
  const int cases[][6] = {{2, 8, 7, 2, 400, 0}, {4, 9, 8, 0, 300, 1}, {1, 4, 2, 1, 200, 0}, {3, 63, 62, 0, 150, 1}};
  for (int c = 0; c < 4; c++) {
    const int* k = cases[c];
    int32_t P = k[0], frames = k[4];
    uint8_t* in = malloc((size_t)frames * P);
    oracle_gen_inputs(0x6767525300000000ull + c, frames, P, k[5], in);
    Cfg cfg = {P, k[1], k[2], k[3], 0, 0, 1, c == 1 ? 77 : -1, 0};
    uint16_t* ck = malloc(2 * (size_t)frames);
    uint8_t fin[116];
    Res r;
    oracle_synctest_run(&cfg, frames, in, ck, NULL, 0, NULL, fin, NULL, NULL, NULL, &r);
    printf("synctest %d status %d frames %d last %u final %u\n", c, r.status, r.frames_done,
           ck[r.frames_done ? r.frames_done - 1 : 0], oracle_fletcher16(fin, 36 + 20 * (size_t)P));
    free(ck);
    free(in);
  }
  {
    int32_t N = 64, P = 2, frames = 40;
    uint8_t* in = malloc((size_t)frames * P);
    oracle_gen_inputs(9, frames, P, 1, in);
    uint8_t* fin = malloc(4 + 100 * (size_t)N);
    uint16_t ck[40];
    Res r;
    oracle_particles_synctest_run(N, P, 17, 16, 3, frames, in, -1, ck, fin, NULL, NULL, NULL, &r);
    printf("particles status %d last %u final %u\n", r.status, ck[frames - 1], oracle_fletcher16(fin, 4 + 100 * (size_t)N));
    free(in);
    free(fin);
  }
  {
    uint8_t st[76], states[8 * 76], fin[76];
    uint16_t cks[8];
    uint8_t in[16];
    for (int i = 0; i < 16; i++) in[i] = (uint8_t)(i * 5 % 16);
    oracle_state_new_bytes(2, st);
    oracle_p2p_replay(2, st, 0, 8, 8, in, NULL, states, cks, fin);
    printf("p2p last %u\n", cks[7]);
  }
  return 0;
}
