/* handler_driver.c -- the request handler's per-call host work, in C, for bench.py's request-boundary
 * workload (bench --workload requests).  What the Rust request handler of INTEGRATION.md does for L
 * GGRS sessions per advance_frame: encode every session's request list into the engine's mapped
 * lane batch (request kinds, Load frames, the AdvanceFrame input rows), run it through the C ABI
 * and hand every SaveGameState's checksum back (GameStateCell::save, sync_layer.rs:18-24) -- here
 * summed into a sink so the reads happen.  Bench infrastructure, not part of the engine.
 *
 * Lane groups: the sessions are served as G engines of L/G lanes each.  Per call, group g waits for
 * its previous batch (ggrs_lane_batch_wait), hands its checksums back, spends the modelled session
 * time (the GGRS session logic that produces the next lists), encodes its next lists and submits
 * them (ggrs_lane_batch_submit) -- while the other groups' batches are on the device.  G = 1 is the
 * plain synchronous handler.
 *
 * Two list sources:
 *   synctest  SyncTestSession::advance_frame's lists (sync_test_session.rs:85-150): Load f-cd,
 *             Advance, (Save, Advance) x (cd-1), Save f, Advance -- the same kinds for every lane,
 *             written as token rows;
 *   p2p       every lane its own P2PSession's lists (p2p_session.rs:265-426, rollbacks of differing
 *             depth) from a fixture the oracle generated (bench_native/make_p2p_fixture.py), each
 *             lane encoded by ggrs_lane_encode, the encoder the Rust crate uses. */
#include <linux/perf_event.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ioctl.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include "ggrs_amd.h"
#include <omp.h>
#include <stdatomic.h>

/* the rejection message of a failed encode on an OpenMP worker: ggrs_last_error() is thread-local
 * in the engine, so the worker's message is copied here for the calling thread (handler_last_error) */
static char g_drv_error[512];
const char* handler_last_error(void) { return g_drv_error; }

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* ---- the P2P encoder's profile (GGRS_DRIVER_PROFILE=1; bench.py --req-profile): per host thread
 * the time spent waiting for the step's release / the workers (spin), handing checksums back and
 * encoding lists -- the two as separate passes over the thread's lanes -- and, where the kernel
 * lets a process count its own events (perf_event_open, user space only), cycles, instructions,
 * cache references / misses and L1D read misses of each pass, read as one group per pass. */
#define PROF_MAX_T 64
#define PROF_NC 5
typedef struct {
  double t_spin, t_hb, t_enc;
  uint64_t c_hb[PROF_NC], c_enc[PROF_NC];
  int64_t lanes;
  int32_t counters;  /* the events that opened (0: none) */
} thread_prof_t;
static thread_prof_t g_prof[PROF_MAX_T];
static int32_t g_prof_threads;

static int prof_open(uint32_t type, uint64_t config, int group) {
  struct perf_event_attr a;
  memset(&a, 0, sizeof a);
  a.size = sizeof a;
  a.type = type;
  a.config = config;
  a.disabled = group < 0;
  a.exclude_kernel = 1;
  a.exclude_hv = 1;
  a.read_format = PERF_FORMAT_GROUP;
  return (int)syscall(SYS_perf_event_open, &a, 0, -1, group, 0);
}
/* this thread's counter group: its leader's fd, or -1 */
static int prof_group(int32_t* n_open) {
  const uint64_t l1d_miss = PERF_COUNT_HW_CACHE_L1D | (PERF_COUNT_HW_CACHE_OP_READ << 8) |
                            ((uint64_t)PERF_COUNT_HW_CACHE_RESULT_MISS << 16);
  const int lead = prof_open(PERF_TYPE_HARDWARE, PERF_COUNT_HW_CPU_CYCLES, -1);
  *n_open = 0;
  if (lead < 0) return -1;
  *n_open = 1;
  const struct { uint32_t t; uint64_t c; } ev[PROF_NC - 1] = {{PERF_TYPE_HARDWARE, PERF_COUNT_HW_INSTRUCTIONS},
                                                             {PERF_TYPE_HARDWARE, PERF_COUNT_HW_CACHE_REFERENCES},
                                                             {PERF_TYPE_HARDWARE, PERF_COUNT_HW_CACHE_MISSES},
                                                             {PERF_TYPE_HW_CACHE, l1d_miss}};
  for (int i = 0; i < PROF_NC - 1; i++) {
    if (prof_open(ev[i].t, ev[i].c, lead) < 0) break;
    ++*n_open;
  }
  ioctl(lead, PERF_EVENT_IOC_ENABLE, PERF_IOC_FLAG_GROUP);
  return lead;
}
static void prof_read(int fd, int32_t n, uint64_t* v) {
  uint64_t buf[1 + PROF_NC];
  memset(v, 0, sizeof(uint64_t) * PROF_NC);
  if (fd < 0 || read(fd, buf, sizeof(uint64_t) * (1 + (size_t)n)) <= 0) return;
  for (int i = 0; i < n && i < PROF_NC; i++) v[i] = buf[1 + i];
}
/* out[t][3 + 2 PROF_NC + 2]: t_spin, t_hb, t_enc (s), the handback counters, the encode counters,
 * lanes encoded, counters open; returns the threads profiled */
int32_t handler_profile_read(double* out, int32_t max_threads) {
  const int32_t n = g_prof_threads < max_threads ? g_prof_threads : max_threads;
  for (int32_t t = 0; t < n; t++) {
    double* o = out + (size_t)t * (5 + 2 * PROF_NC);
    o[0] = g_prof[t].t_spin;
    o[1] = g_prof[t].t_hb;
    o[2] = g_prof[t].t_enc;
    for (int i = 0; i < PROF_NC; i++) {
      o[3 + i] = (double)g_prof[t].c_hb[i];
      o[3 + PROF_NC + i] = (double)g_prof[t].c_enc[i];
    }
    o[3 + 2 * PROF_NC] = (double)g_prof[t].lanes;
    o[4 + 2 * PROF_NC] = g_prof[t].counters;
  }
  return n;
}

static void spin_us(double us) {
  if (us <= 0) return;
  const double end = now_s() + us * 1e-6;
  while (now_s() < end) {
  }
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

#define MAX_GROUPS 8

typedef struct {
  ggrs_lane_batch_t b, run;
  int pending;
  int32_t base; /* first lane of the group in the global lane numbering */
  int32_t lanes;
  int32_t saves; /* SaveGameStates per lane of the pending batch (synctest) */
} group_t;

/* SyncTest lists.  inputs: [frames][L][P] user inputs (input delay 0), resident in host memory.
 * Runs calls f_begin .. f_begin+n_calls-1 for every lane of every group.  Returns 0, or the failing
 * ABI code; *seconds = wall time of the calls, *sink = sum of every Save checksum handed back;
 * phases (may be NULL): seconds spent encoding, waiting for the device (submit + wait), handing
 * checksums back, and in the modelled session logic. */
/* groups of lanes lane0 .. lane0 + L - 1 of input rows L_all lanes wide */
static int drive_groups(ggrs_engine_t** engs, int32_t G, const uint8_t* inputs, int32_t L, int32_t L_all, int32_t lane0,
                        int32_t P, int32_t cd, int32_t f_begin, int32_t n_calls, double session_us, uint64_t* sink,
                        double* seconds, double* phases) {
  if (G < 1 || G > MAX_GROUPS || L % G) return GGRS_E_INVALID;
  group_t g[MAX_GROUPS];
  const int32_t Lg = L / G;
  for (int q = 0; q < G; q++) {
    int rc = ggrs_lane_batch_map(engs[q], 2, 1, cd + 1, cd + 1, &g[q].b);
    if (rc) return rc;
    g[q].pending = 0;
    g[q].base = lane0 + q * Lg;
    g[q].lanes = Lg;
  }
  double t_enc = 0, t_dev = 0, t_back = 0, t_sess = 0;
  uint64_t acc = 0;
  const double t0 = now_s();
  for (int32_t f = f_begin; f <= f_begin + n_calls; f++) {
    for (int q = 0; q < G; q++) {
      group_t* gq = &g[q];
      if (gq->pending) {
        const double ta = now_s();
        int32_t failed = 0;
        int rc = ggrs_lane_batch_wait(engs[q], &failed);
        if (rc) return rc;
        const double tb = now_s();
        for (int k = 0; k < gq->saves; k++) { /* row sums in 32 bits: one vectorised pass per row */
          const uint16_t* row = gq->b.checksums + (size_t)k * Lg;
          uint32_t s = 0;
          for (int32_t l = 0; l < Lg; l++) s += row[l];
          acc += s;
        }
        const double tc = now_s();
        spin_us(session_us); /* the GGRS session logic producing this group's next lists */
        t_dev += tb - ta;
        t_back += tc - tb;
        t_sess += now_s() - tc;
        gq->pending = 0;
      }
      if (f == f_begin + n_calls) continue; /* drained */
      const double ta = now_s();
      uint32_t words[4];
      int nl, na, ns;
      const int W = synctest_tokens(f, cd, words, &nl, &na, &ns);
      for (int j = 0; j < W; j++)
        for (int32_t l = 0; l < Lg; l++) gq->b.tokens[(size_t)j * Lg + l] = words[j];
      if (nl)
        for (int32_t l = 0; l < Lg; l++) gq->b.load_frames[l] = f - cd;
      const int32_t first = f - (na - 1); /* the frames the list's AdvanceFrames replay, in order */
      for (int a = 0; a < na; a++)
        memcpy(gq->b.inputs + (size_t)a * Lg * P, inputs + ((size_t)(first + a) * L_all + gq->base) * P, (size_t)Lg * P);
      gq->run = gq->b;
      gq->run.token_words = W;
      gq->run.load_slots = nl;
      gq->run.adv_rows = na;
      gq->run.save_rows = ns;
      gq->saves = ns;
      const double tb = now_s();
      int rc = ggrs_lane_batch_submit(engs[q], &gq->run, 0);
      if (rc) return rc;
      gq->pending = 1;
      t_enc += tb - ta;
      t_dev += now_s() - tb;
    }
  }
  *seconds = now_s() - t0;
  if (phases) {
    phases[0] = t_enc;
    phases[1] = t_dev;
    phases[2] = t_back;
    phases[3] = t_sess;
  }
  *sink = acc;
  return 0;
}

int handler_drive_synctest_groups(ggrs_engine_t** engs, int32_t G, const uint8_t* inputs, int32_t L, int32_t P,
                                  int32_t cd, int32_t f_begin, int32_t n_calls, double session_us, uint64_t* sink,
                                  double* seconds, double* phases) {
  return drive_groups(engs, G, inputs, L, L, 0, P, cd, f_begin, n_calls, session_us, sink, seconds, phases);
}

/* Host threads: T threads, thread t serving groups t, t + T, ... through the loop above (a game
 * server runs its sessions' GGRS instances on several cores; each engine is one lane group and the
 * library keeps no state shared between engines).  The threads start together; *seconds is the
 * slowest thread's wall time, *sink and phases sum over threads (phases: thread-seconds). */
#include <pthread.h>

typedef struct {
  ggrs_engine_t* engs[MAX_GROUPS];
  int32_t G;
  const uint8_t* inputs;
  int32_t L, L_all, lane0, P, cd, f_begin, n_calls;
  double session_us;
  uint64_t sink;
  double seconds, phases[4];
  int rc;
  pthread_barrier_t* start;
} thread_job_t;

static void* drive_thread(void* arg) {
  thread_job_t* j = (thread_job_t*)arg;
  pthread_barrier_wait(j->start);
  j->rc = drive_groups(j->engs, j->G, j->inputs, j->L, j->L_all, j->lane0, j->P, j->cd, j->f_begin, j->n_calls,
                       j->session_us, &j->sink, &j->seconds, j->phases);
  return NULL;
}

int handler_drive_synctest_threads(ggrs_engine_t** engs, int32_t G, int32_t T, const uint8_t* inputs, int32_t L,
                                   int32_t P, int32_t cd, int32_t f_begin, int32_t n_calls, double session_us,
                                   uint64_t* sink, double* seconds, double* phases) {
  if (T < 1 || T > G || G % T || G > MAX_GROUPS || L % G) return GGRS_E_INVALID;
  thread_job_t jobs[MAX_GROUPS];
  pthread_t th[MAX_GROUPS];
  pthread_barrier_t start;
  pthread_barrier_init(&start, NULL, (unsigned)T);
  const int32_t per = G / T, Lg = L / G;
  for (int t = 0; t < T; t++) {
    thread_job_t* j = &jobs[t];
    memset(j, 0, sizeof *j);
    for (int q = 0; q < per; q++) j->engs[q] = engs[t * per + q];
    j->G = per;
    j->inputs = inputs;  /* the thread's groups: lanes t*per*Lg .. of rows L lanes wide */
    j->L = per * Lg;
    j->L_all = L;
    j->lane0 = t * per * Lg;
    j->P = P;
    j->cd = cd;
    j->f_begin = f_begin;
    j->n_calls = n_calls;
    j->session_us = session_us;
    j->start = &start;
    if (pthread_create(&th[t], NULL, drive_thread, j)) return GGRS_E_STATE;
  }
  int rc = 0;
  double worst = 0;
  uint64_t acc = 0;
  double ph[4] = {0, 0, 0, 0};
  for (int t = 0; t < T; t++) {
    pthread_join(th[t], NULL);
    if (jobs[t].rc && !rc) rc = jobs[t].rc;
    if (jobs[t].seconds > worst) worst = jobs[t].seconds;
    acc += jobs[t].sink;
    for (int k = 0; k < 4; k++) ph[k] += jobs[t].phases[k];
  }
  pthread_barrier_destroy(&start);
  *seconds = worst;
  *sink = acc;
  if (phases)
    for (int k = 0; k < 4; k++) phases[k] = ph[k];
  return rc;
}

/* The single-engine form kept for bench.py --req-groups 1 (one synchronous batch per call). */
int handler_drive_synctest(ggrs_engine_t* eng, const uint8_t* inputs, int32_t L, int32_t P, int32_t cd,
                           int32_t f_begin, int32_t n_calls, uint64_t* sink, double* seconds, double* phases) {
  double ph[4];
  int rc = handler_drive_synctest_groups(&eng, 1, inputs, L, P, cd, f_begin, n_calls, 0.0, sink, seconds, ph);
  if (phases) {
    phases[0] = ph[0];
    phases[1] = ph[1];
    phases[2] = ph[2];
  }
  return rc;
}

/* P2P lists from the fixture: M sessions' streams, lane l (global) plays session l % M.
 *   reqs     [N] ggrs_request_t of every session's calls, back to back
 *   req_off  [M][C + 1] start of session m's call c in reqs
 *   adv_off  [M][C + 1] start of its AdvanceFrame rows in inputs / status
 *   inputs, status [N_adv][P]
 * Calls c_begin .. c_begin+n_calls-1.  lane_frames [L] in/out: every lane's frame (the encoder's
 * Save-frame check); shape[4]: the batch shape to map (the fixture's largest list).
 * deferred: the handler's deferred hand-back (rust/ggrs-mi355x handle_requests_deferred): a call
 * submits its batch and returns, the modelled session logic runs while the batch is on the device,
 * and the next call collects it (checksums into the cells) before encoding its own lists;
 * synchronous: the session logic runs after the call's checksums are back.  threads > 1: the lanes
 * of a group are encoded and handed back by that many host threads (OpenMP). */
int handler_drive_p2p_groups(ggrs_engine_t** engs, int32_t G, int32_t L, int32_t P, int32_t M, int32_t C,
                             const ggrs_request_t* reqs, const int64_t* req_off, const int64_t* adv_off,
                             const uint8_t* inputs, const uint8_t* status, const int32_t* shape, int32_t* lane_frames,
                             int32_t c_begin, int32_t n_calls, double session_us, int32_t deferred, int32_t threads,
                             uint64_t* sink, double* seconds, double* phases) {
  if (G < 1 || G > MAX_GROUPS || L % G || c_begin < 0 || c_begin + n_calls > C || threads < 1) return GGRS_E_INVALID;
  group_t g[MAX_GROUPS];
  const int32_t Lg = L / G;
  for (int q = 0; q < G; q++) {
    int rc = ggrs_lane_batch_map(engs[q], shape[0], shape[1] > 0 ? shape[1] : 1, shape[2] > 0 ? shape[2] : 1,
                                 shape[3] > 0 ? shape[3] : 1, &g[q].b);
    if (rc) return rc;
    g[q].pending = 0;
    g[q].base = q * Lg;
    g[q].lanes = Lg;
  }
  /* phases (the master thread's clock): encode + hand-back of a group's lanes (the threads' shares
   * between two barriers), submit, wait, session logic; the barriers themselves are in the first */
  double t_work = 0, t_submit = 0, t_wait = 0, t_sess = 0;
  uint64_t acc = 0;
  int32_t prev_call[MAX_GROUPS];
  /* err: the first failure; written under `omp critical` by workers and by the master, so atomic.
   * step_err: its value when the master released step e -- every thread of the step reads that
   * one (ordered by the release/acquire chain on `ready`), so no two threads of a step disagree
   * on whether to hand back or encode */
  _Atomic int err = 0;
  int step_err = 0;
  const double t0 = now_s();
  /* One parallel region for the whole run: the threads persist across calls (a fork/join per group
   * and call cost more than the encoding itself).  Step e = (call, group): the
   * master collects the group's previous batch and releases the step (ready = e), every thread
   * hands back the checksums of its share of the lanes and encodes their next lists (one pass over
   * each lane) and counts itself done, the master submits once all have.  A release flag and an
   * arrival counter instead of two full barriers per step. */
  _Atomic int64_t ready = -1, done = 0;
  const int64_t n_steps = (int64_t)(n_calls + 1) * G;
  const char* prof_env = getenv("GGRS_DRIVER_PROFILE");
  const int prof = prof_env && prof_env[0] == '1';
  if (prof) {
    memset(g_prof, 0, sizeof g_prof);
    g_prof_threads = threads < PROF_MAX_T ? threads : PROF_MAX_T;
  }
#pragma omp parallel num_threads(threads) reduction(+ : acc) if (threads > 1)
  {
    const int tid = omp_get_thread_num(), nt = omp_get_num_threads();
    thread_prof_t* tp = prof && tid < PROF_MAX_T ? &g_prof[tid] : NULL;
    int32_t n_open = 0;
    const int pfd = tp ? prof_group(&n_open) : -1;
    if (tp) tp->counters = n_open;
    uint64_t c0[PROF_NC], c1[PROF_NC], c2[PROF_NC];
    for (int64_t e = 0; e < n_steps; e++) {
      const int32_t c = c_begin + (int32_t)(e / G);
      const int q = (int)(e % G);
      group_t* gq = &g[q];
      if (tid == 0) {
        if (gq->pending && !atomic_load_explicit(&err, memory_order_relaxed)) {
          const double ta = now_s();
          int32_t failed = 0;
          int rc = ggrs_lane_batch_wait(engs[q], &failed);
          if (rc) atomic_store_explicit(&err, rc, memory_order_relaxed);
          t_wait += now_s() - ta;
          if (!deferred) spin_us(session_us); /* the session logic after the checksums are back */
        }
        step_err = atomic_load_explicit(&err, memory_order_relaxed);
        atomic_store_explicit(&ready, e, memory_order_release);
      } else {
        const double ts = tp ? now_s() : 0;
        while (atomic_load_explicit(&ready, memory_order_acquire) < e) __builtin_ia32_pause();
        if (tp) tp->t_spin += now_s() - ts;
      }
      const double tw = now_s();
      const int32_t l0 = (int32_t)((int64_t)Lg * tid / nt), l1 = (int32_t)((int64_t)Lg * (tid + 1) / nt);
      const int handback = gq->pending && !step_err, encode = c < c_begin + n_calls && !step_err;
      const int32_t pc = prev_call[q];
      /* profiling: the hand-back and the encode as two passes, each timed and counted */
      const int passes = tp ? 2 : 1;
      for (int pass = 0; pass < passes; pass++) {
      const int do_hb = handback && (!tp || pass == 0), do_enc = encode && (!tp || pass == 1);
      double tp0 = 0;
      if (tp) {
        prof_read(pfd, n_open, pass == 0 ? c0 : c1);
        tp0 = now_s();
      }
      for (int32_t l = l0; l < l1; l++) {
        const int32_t lane = gq->base + l, m = lane % M;
        if (do_hb) { /* every Save's checksum of the lane's previous list */
          const int64_t a = req_off[(int64_t)m * (C + 1) + pc], b = req_off[(int64_t)m * (C + 1) + pc + 1];
          int si = 0;
          for (int64_t k = a; k < b; k++)
            if (reqs[k].kind == GGRS_REQ_SAVE) acc += gq->b.checksums[(size_t)si++ * Lg + l];
          lane_frames[lane] = gq->b.lane_result[l];
        }
        if (do_enc) {
          const int64_t a = req_off[(int64_t)m * (C + 1) + c], b = req_off[(int64_t)m * (C + 1) + c + 1];
          const int64_t ad = adv_off[(int64_t)m * (C + 1) + c];
          int32_t bad = -1;
          int rc = ggrs_lane_encode(&gq->b, Lg, P, l, reqs + a, (int32_t)(b - a), inputs + ad * P, status + ad * P,
                                    lane_frames[lane], &bad);
          if (rc) {
#pragma omp critical
            { /* the fixture's lists are valid: any rejection is an error here */
              if (!atomic_load_explicit(&err, memory_order_relaxed)) {
                strncpy(g_drv_error, ggrs_last_error(), sizeof g_drv_error - 1);
                g_drv_error[sizeof g_drv_error - 1] = 0;
                atomic_store_explicit(&err, rc, memory_order_relaxed);
              }
            }
          }
        }
      }
      if (tp) {
        const double dt = now_s() - tp0;
        prof_read(pfd, n_open, pass == 0 ? c2 : c0);
        if (pass == 0) {
          tp->t_hb += dt;
          for (int i = 0; i < PROF_NC; i++) tp->c_hb[i] += c2[i] - c0[i];
        } else {
          tp->t_enc += dt;
          for (int i = 0; i < PROF_NC; i++) tp->c_enc[i] += c0[i] - c1[i];
          if (encode) tp->lanes += l1 - l0;
        }
      }
      }
      if (tid != 0) {
        atomic_fetch_add_explicit(&done, 1, memory_order_release);
      } else {
        const int64_t want = (e + 1) * (nt - 1);
        const double ts = tp ? now_s() : 0;
        while (atomic_load_explicit(&done, memory_order_acquire) < want) __builtin_ia32_pause();
        if (tp) tp->t_spin += now_s() - ts;
        t_work += now_s() - tw;
        gq->pending = 0;
        if (encode && !atomic_load_explicit(&err, memory_order_relaxed)) {
          gq->run = gq->b;
          const double tb = now_s();
          int rc = ggrs_lane_batch_submit(engs[q], &gq->run, GGRS_BATCH_STATUS);
          if (rc) atomic_store_explicit(&err, rc, memory_order_relaxed);
          gq->pending = rc == 0;
          prev_call[q] = c;
          t_submit += now_s() - tb;
          if (deferred) { /* the call has returned: the session logic overlaps the batch on the device */
            const double td = now_s();
            spin_us(session_us);
            t_sess += now_s() - td;
          }
        }
      }
    }
    if (pfd >= 0) close(pfd);
  }
  if (atomic_load_explicit(&err, memory_order_relaxed)) return atomic_load_explicit(&err, memory_order_relaxed);
  *seconds = now_s() - t0;
  if (phases) { /* encode + hand-back (barriers included), submit, wait, session logic */
    phases[0] = t_work;
    phases[1] = t_submit;
    phases[2] = t_wait;
    phases[3] = t_sess;
  }
  *sink = acc;
  return 0;
}
