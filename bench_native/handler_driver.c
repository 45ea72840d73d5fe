/* handler_driver.c -- the request handler's per-call host work, in C, for bench.py's request-boundary
 * workload (bench --workload requests).  What the Rust request handler of INTEGRATION.md does for L
 * GGRS sessions per advance_frame: encode every session's request list into the engine's mapped
 * lane batch (request kinds, Load frames, the AdvanceFrame input rows), run it through the C ABI
 * (ggrs_lane_batch_run) and hand every SaveGameState's checksum back (GameStateCell::save,
 * sync_layer.rs:18-24) -- here summed into a sink so the reads happen.  The lists are
 * SyncTestSession::advance_frame's (sync_test_session.rs:85-150): Load f-cd, Advance,
 * (Save, Advance) x (cd-1), Save f, Advance.  Bench infrastructure, not part of the engine. */
#include <stdint.h>
#include <string.h>
#include <time.h>

#include "ggrs_amd.h"

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* 2-bit request kinds of the SyncTest list at frame f, least significant first */
static int synctest_tokens(int32_t f, int32_t cd, uint32_t* words, int* nl, int* na, int* ns) {
  int k = 0;
  uint32_t w[4] = {0, 0, 0, 0};
#define PUT(t) (w[k >> 4] |= (uint32_t)(t) << (2 * (k & 15)), k++)
  *nl = *na = *ns = 0;
  if (f > cd) {
    PUT(GGRS_TOK_LOAD), ++*nl;
    PUT(GGRS_TOK_ADVANCE), ++*na;
    for (int i = 1; i < cd; i++) PUT(GGRS_TOK_SAVE), ++*ns, PUT(GGRS_TOK_ADVANCE), ++*na;
  }
  PUT(GGRS_TOK_SAVE), ++*ns;
  PUT(GGRS_TOK_ADVANCE), ++*na;
#undef PUT
  const int W = (k + GGRS_TOKENS_PER_WORD - 1) / GGRS_TOKENS_PER_WORD;
  for (int j = k; j < W * GGRS_TOKENS_PER_WORD; j++) w[j >> 4] |= (uint32_t)GGRS_TOK_END << (2 * (j & 15));
  for (int j = 0; j < W; j++) words[j] = w[j];
  return W;
}

/* Runs calls f_begin .. f_begin+n_calls-1 for every lane.  inputs: [frames][L][P] user inputs
 * (input delay 0), resident in host memory.  Returns 0, or the failing ABI code; *seconds = wall
 * time of the calls, *sink = sum of every Save checksum handed back; phases (may be NULL) gets the
 * seconds spent encoding, in ggrs_lane_batch_run, and handing checksums back. */
int handler_drive_synctest(ggrs_engine_t* eng, const uint8_t* inputs, int32_t L, int32_t P, int32_t cd,
                           int32_t f_begin, int32_t n_calls, uint64_t* sink, double* seconds, double* phases) {
  double t_enc = 0, t_run = 0, t_back = 0;
  ggrs_lane_batch_t b;
  int rc = ggrs_lane_batch_map(eng, 2, 1, cd + 1, cd + 1, &b);
  if (rc) return rc;
  uint64_t acc = 0;
  const double t0 = now_s();
  for (int32_t f = f_begin; f < f_begin + n_calls; f++) {
    const double ta = now_s();
    uint32_t words[4];
    int nl, na, ns;
    const int W = synctest_tokens(f, cd, words, &nl, &na, &ns);
    for (int j = 0; j < W; j++)
      for (int32_t l = 0; l < L; l++) b.tokens[(size_t)j * L + l] = words[j];
    if (nl)
      for (int32_t l = 0; l < L; l++) b.load_frames[l] = f - cd;
    const int32_t first = f - (na - 1); /* the frames the list's AdvanceFrames replay, in order */
    memcpy(b.inputs, inputs + (size_t)first * L * P, (size_t)na * L * P);
    ggrs_lane_batch_t run = b;
    run.token_words = W;
    run.load_slots = nl;
    run.adv_rows = na;
    run.save_rows = ns;
    int32_t failed = 0;
    const double tb = now_s();
    rc = ggrs_lane_batch_run(eng, &run, 0, &failed);
    if (rc) return rc;
    const double tc = now_s();
    for (int k = 0; k < ns; k++) {  /* row sums in 32 bits: one vectorised pass over the row */
      const uint16_t* row = b.checksums + (size_t)k * L;
      uint32_t s = 0;
      for (int32_t l = 0; l < L; l++) s += row[l];
      acc += s;
    }
    const double td = now_s();
    t_enc += tb - ta;
    t_run += tc - tb;
    t_back += td - tc;
  }
  *seconds = now_s() - t0;
  if (phases) {
    phases[0] = t_enc;
    phases[1] = t_run;
    phases[2] = t_back;
  }
  *sink = acc;
  return 0;
}
