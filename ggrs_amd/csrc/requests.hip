// requests.hip -- per-lane request lists: every lane is its own GGRS session and fulfils its own
// ordered Vec<GgrsRequest> (src/lib.rs:171-195) in one launch.
//
// Reference: the user's request handler Game::handle_requests (examples/ex_game/ex_game.rs:79-127)
// for the lists P2PSession::advance_frame (src/sessions/p2p_session.rs:265-426: save of frame 0,
// adjust_gamestate's Load first_incorrect + (Save, Advance) replay :658-714, sparse saving's
// check_last_saved_state :819-843, save current :337, advance :393-423) and
// SyncTestSession::advance_frame (sync_test_session.rs:85-150) emit.  Lanes' lists differ: a
// session rolls back to its own first_incorrect with its own replay count.
//
// Encoding (include/ggrs_amd.h, ggrs_lane_batch_t): per lane the request kinds in 2-bit tokens,
// position-major words [W][L] (a wavefront reads one coalesced row per 16 requests), the Load
// frames [LD][L], one input row [A][L][P] per AdvanceFrame, checksums out [S][L].  Save frames are
// implicit (a save stores the state's own frame, which ex_game.rs:104 asserts it is); a Load names
// its frame, validated against the cell's tag -- the frame field of the lane's ring cell (ring
// cells start as NULL_FRAME), i.e. GameStateCell.frame (sync_layer.rs:72-78, 248).
//
// The kernel: one thread per lane, one 64-lane wavefront per block.  The batch lives in pinned
// host memory mapped into the device; every row the lane needs is staged into LDS up front (all
// loads in flight at once: one PCIe round trip instead of one per request), the list is validated
// against the lane's cell tags (also in LDS), then executed with the state in registers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "common.h"
#include "engine.h"

#pragma clang fp contract(off)

using namespace ggrs;

namespace {

struct LaneBatchParams {
  int64_t L;
  int32_t R, W, LD, A, S, use_status, trace_cap;
  const uint32_t* tokens;      // [W][L]
  const int32_t* load_frames;  // [LD][L]
  const uint8_t* inputs;       // [A][L][P]
  const uint8_t* status;       // [A][L][P]
  uint16_t* cks;               // [S][L]
  int32_t* result;             // [L]
  uint32_t* cur;
  uint32_t* ring;
  uint16_t* ring_ck;
  uint16_t* trace;
};

// P bytes of one lane's row, packed little-endian (player i in byte i)
template <int P>
__device__ inline uint32_t row_bytes(const uint8_t* row, int64_t lane) {
  if constexpr (P == 1) return row[lane];
  if constexpr (P == 2) return reinterpret_cast<const uint16_t*>(row)[lane];
  if constexpr (P == 4) return reinterpret_cast<const uint32_t*>(row)[lane];
  const uint8_t* b = row + lane * 3;
  return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16);
}

// LDS: tokens [W][64] u32 | load frames [LD][64] i32 | cell tags [R][64] i32 | inputs [A][64] u32
// | status [A][64] u32 (when used)
__host__ __device__ inline size_t lane_batch_lds_bytes(int W, int LD, int R, int A, int use_status) {
  return (size_t)kWave * 4 * ((size_t)W + LD + R + (size_t)A * (use_status ? 2 : 1));
}

template <int P>
__global__ __launch_bounds__(kWave) void lane_requests_kernel(LaneBatchParams p) {
  extern __shared__ uint32_t lds[];
  const int wl = threadIdx.x;
  const int64_t L = p.L;
  const int64_t lane = (int64_t)blockIdx.x * kWave + wl;
  const bool valid = lane < L;
  const int64_t ln = valid ? lane : 0;
  const int R = p.R;
  constexpr int F = state_fields(P);
  uint32_t* l_tok = lds;
  int32_t* l_load = (int32_t*)(l_tok + p.W * kWave);
  int32_t* l_tag = l_load + p.LD * kWave;
  uint32_t* l_in = (uint32_t*)(l_tag + R * kWave);
  uint32_t* l_st = l_in + p.A * kWave;
  // stage every row of this lane's batch (host memory: issue them all before waiting on any) and
  // the lane's cell tags (the frame field of each ring cell)
  for (int w = 0; w < p.W; w++) l_tok[w * kWave + wl] = p.tokens[(int64_t)w * L + ln];
  for (int k = 0; k < p.LD; k++) l_load[k * kWave + wl] = p.load_frames[(int64_t)k * L + ln];
  for (int a = 0; a < p.A; a++) l_in[a * kWave + wl] = row_bytes<P>(p.inputs + (int64_t)a * L * P, ln);
  if (p.use_status)
    for (int a = 0; a < p.A; a++) l_st[a * kWave + wl] = row_bytes<P>(p.status + (int64_t)a * L * P, ln);
  for (int s = 0; s < R; s++) l_tag[s * kWave + wl] = (int32_t)p.ring[(int64_t)s * F * L + ln];
  BoxState<P> st;
  load_state<P>(st, p.cur + ln, L);
  if (!valid) return;  // no barrier follows: every lane only reads its own LDS column

  const int n_tok = p.W * GGRS_TOKENS_PER_WORD;
  auto token = [&](int k) -> uint32_t { return (l_tok[(k >> 4) * kWave + wl] >> (2 * (k & 15))) & 3u; };
  // (1) validation: walk the list with the lane's frame and cell tags; nothing is written
  int32_t frame = (int32_t)st.w[0];
  int32_t err = -1;
  {
    int na = 0, ns = 0, nl = 0;
    int32_t slot = frame % R;
    for (int k = 0; k < n_tok; k++) {
      const uint32_t t = token(k);
      if (t == GGRS_TOK_END) break;
      if (t == GGRS_TOK_SAVE) {
        if (ns == p.S) { err = k; break; }
        l_tag[slot * kWave + wl] = frame;
        ++ns;
      } else if (t == GGRS_TOK_LOAD) {
        if (nl == p.LD) { err = k; break; }
        const int32_t f = l_load[nl * kWave + wl];
        if (f < 0 || l_tag[(f % R) * kWave + wl] != f) { err = k; break; }  // sync_layer.rs:248
        frame = f;
        slot = f % R;
        ++nl;
      } else {
        if (na == p.A) { err = k; break; }
        ++frame;
        slot = slot + 1 == R ? 0 : slot + 1;
        ++na;
      }
    }
  }
  if (err >= 0) {  // the lane does not run (a reference session would have panicked here)
    p.result[lane] = -(1 + err);
    return;
  }
  // (2) execution: Game::handle_requests, requests strictly in order (ex_game.rs:79-99)
  int na = 0, ns = 0, nl = 0;
  int32_t slot = (int32_t)st.w[0] % R;
  for (int k = 0; k < n_tok; k++) {
    const uint32_t t = token(k);
    if (t == GGRS_TOK_END) break;
    if (t == GGRS_TOK_SAVE) {  // save_game_state (:103-108): state + fletcher16 into the cell
      store_state<P>(st, p.ring + (int64_t)slot * F * L + lane, L);
      const uint16_t ck = fletcher16_state<P>(st);
      p.ring_ck[(int64_t)slot * L + lane] = ck;
      p.cks[(int64_t)ns * L + lane] = ck;
      ++ns;
    } else if (t == GGRS_TOK_LOAD) {  // load_game_state (:111-113)
      const int32_t f = l_load[nl * kWave + wl];
      slot = f % R;
      load_state<P>(st, p.ring + (int64_t)slot * F * L + lane, L);
      ++nl;
    } else {  // advance_frame (:115-127); Disconnected players spin (input 4, :277-281)
      uint32_t disc = 0;
      if (p.use_status) {
        const uint32_t sb = l_st[na * kWave + wl];
#pragma unroll
        for (int i = 0; i < P; i++)
          if (((sb >> (8 * i)) & 0xffu) == GGRS_STATUS_DISCONNECTED) disc |= 1u << i;
      }
      advance_state<P>(st, l_in[na * kWave + wl], disc);
      if (p.trace) p.trace[(int64_t)(((int32_t)st.w[0] - 1) % p.trace_cap) * L + lane] = fletcher16_state<P>(st);
      slot = slot + 1 == R ? 0 : slot + 1;
      ++na;
    }
  }
  store_state<P>(st, p.cur + lane, L);
  p.result[lane] = (int32_t)st.w[0];
}

int map_batch(ggrs_engine* e, int32_t W, int32_t LD, int32_t A, int32_t S) {
  LaneBatchHost& b = e->batch;
  if (b.base && W <= b.words && LD <= b.loads && A <= b.adv && S <= b.saves) return GGRS_OK;
  W = std::max(W, b.words);
  LD = std::max(LD, b.loads);
  A = std::max(A, b.adv);
  S = std::max(S, b.saves);
  const size_t L = (size_t)e->cfg.num_lanes, P = (size_t)e->cfg.num_players;
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  LaneBatchHost n;
  n.words = W;
  n.loads = LD;
  n.adv = A;
  n.saves = S;
  size_t o = 0;
  n.off_tokens = o; o += up(4 * L * (size_t)W);
  n.off_loads = o; o += up(4 * L * (size_t)LD);
  n.off_inputs = o; o += up(L * P * (size_t)A);
  n.off_status = o; o += up(L * P * (size_t)A);
  n.off_cks = o; o += up(2 * L * (size_t)S);
  n.off_result = o; o += up(4 * L);
  n.bytes = o;
  // pinned, mapped into the device's address space: the kernel reads the rows and writes the
  // results in place
  HIP_TRY(hipHostMalloc((void**)&n.base, n.bytes, hipHostMallocMapped));
  std::memset(n.base, 0, n.bytes);
  if (b.base) {
    HIP_TRY(hipStreamSynchronize(e->stream));
    HIP_TRY(hipHostFree(b.base));
  }
  b = n;
  return GGRS_OK;
}

void fill_batch_view(const ggrs_engine* e, ggrs_lane_batch_t* out) {
  const LaneBatchHost& b = e->batch;
  out->token_words = b.words;
  out->load_slots = b.loads;
  out->adv_rows = b.adv;
  out->save_rows = b.saves;
  out->tokens = (uint32_t*)(b.base + b.off_tokens);
  out->load_frames = (int32_t*)(b.base + b.off_loads);
  out->inputs = b.base + b.off_inputs;
  out->status = b.base + b.off_status;
  out->checksums = (uint16_t*)(b.base + b.off_cks);
  out->lane_result = (int32_t*)(b.base + b.off_result);
}

template <typename T>
T* device_view(T* host) {
  void* d = nullptr;
  return hipHostGetDevicePointer(&d, (void*)host, 0) == hipSuccess ? (T*)d : nullptr;
}

// Launch over the engine's mapped batch with the given counts; waits for completion.
int run_batch(ggrs_engine* e, int32_t W, int32_t LD, int32_t A, int32_t S, int use_status) {
  ggrs_lane_batch_t v;
  fill_batch_view(e, &v);
  LaneBatchParams p;
  p.L = e->cfg.num_lanes;
  p.R = e->R;
  p.W = W;
  p.LD = LD;
  p.A = A;
  p.S = S;
  p.use_status = use_status;
  p.trace_cap = e->cfg.trace_capacity;
  p.tokens = device_view(v.tokens);
  p.load_frames = device_view(v.load_frames);
  p.inputs = device_view(v.inputs);
  p.status = device_view(v.status);
  p.cks = device_view(v.checksums);
  p.result = device_view(v.lane_result);
  if (!p.tokens || !p.load_frames || !p.inputs || !p.status || !p.cks || !p.result)
    return set_error(GGRS_E_HIP, "hipHostGetDevicePointer failed for the lane batch");
  p.cur = e->cur;
  p.ring = e->ring;
  p.ring_ck = e->ring_ck;
  p.trace = e->trace;
  const size_t lds = lane_batch_lds_bytes(W, LD, e->R, A, use_status);
  const int64_t grid = grid_of(p.L, kWave);
  e->mode = kModeLaneRequests;
  int rc = launch_timed(e, [&] {
    switch (e->cfg.num_players) {
      case 1: lane_requests_kernel<1><<<grid, kWave, lds, e->stream>>>(p); break;
      case 2: lane_requests_kernel<2><<<grid, kWave, lds, e->stream>>>(p); break;
      case 3: lane_requests_kernel<3><<<grid, kWave, lds, e->stream>>>(p); break;
      default: lane_requests_kernel<4><<<grid, kWave, lds, e->stream>>>(p); break;
    }
  });
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

int check_mode(const ggrs_engine* e) {
  if (e->mode == kModeSyncTest || e->mode == kModeLockstepRequests)
    return set_error(GGRS_E_STATE, "engine already driven by a lane-uniform program");
  return GGRS_OK;
}

int check_shape(int32_t W, int32_t LD, int32_t A, int32_t S) {
  if (W < 0 || W > GGRS_BATCH_MAX_WORDS || LD < 0 || LD > GGRS_BATCH_MAX_LOADS || A < 0 || A > GGRS_BATCH_MAX_ADV ||
      S < 0 || S > GGRS_BATCH_MAX_SAVES)
    return set_error(GGRS_E_INVALID, "lane batch shape (%d words, %d loads, %d advances, %d saves) outside "
                                     "the limits (%d, %d, %d, %d)", W, LD, A, S, GGRS_BATCH_MAX_WORDS,
                     GGRS_BATCH_MAX_LOADS, GGRS_BATCH_MAX_ADV, GGRS_BATCH_MAX_SAVES);
  return GGRS_OK;
}

// failed lanes of the last run: count, and the first one's message
int report_failures(const ggrs_engine* e, const int32_t* result, int32_t* n_failed) {
  const int64_t L = e->cfg.num_lanes;
  int32_t n = 0;
  int64_t first = -1;
  for (int64_t l = 0; l < L; l++)
    if (result[l] < 0) {
      if (first < 0) first = l;
      ++n;
    }
  if (n_failed) *n_failed = n;
  if (n == 0) return GGRS_OK;
  return set_error(GGRS_E_PRECONDITION,
                   "%d lane(s) failed validation and did not run; lane %lld at request %d (a Load of a frame "
                   "its cell does not hold, sync_layer.rs:248 / ex_game.rs:112, a Save of a frame other than "
                   "the state's, ex_game.rs:104, or more requests than the batch holds)",
                   n, (long long)first, -result[first] - 1);
}

}  // namespace

extern "C" {

int ggrs_lane_batch_map(ggrs_engine_t* e, int32_t W, int32_t LD, int32_t A, int32_t S, ggrs_lane_batch_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  int rc = check_shape(W, LD, A, S);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(e->cfg.device));
  rc = map_batch(e, W, LD, A, S);
  if (rc) return rc;
  fill_batch_view(e, out);
  return GGRS_OK;
}

int ggrs_lane_batch_run(ggrs_engine_t* e, const ggrs_lane_batch_t* b, int32_t flags, int32_t* n_failed) {
  if (!e || !b) return set_error(GGRS_E_INVALID, "null argument");
  if (n_failed) *n_failed = 0;
  int rc = check_mode(e);
  if (rc) return rc;
  const LaneBatchHost& h = e->batch;
  ggrs_lane_batch_t v;
  if (!h.base) return set_error(GGRS_E_STATE, "no lane batch mapped (ggrs_lane_batch_map)");
  fill_batch_view(e, &v);
  if (b->tokens != v.tokens || b->load_frames != v.load_frames || b->inputs != v.inputs || b->status != v.status ||
      b->checksums != v.checksums || b->lane_result != v.lane_result)
    return set_error(GGRS_E_INVALID, "batch pointers are not this engine's current mapping");
  if (b->token_words < 0 || b->token_words > h.words || b->load_slots < 0 || b->load_slots > h.loads ||
      b->adv_rows < 0 || b->adv_rows > h.adv || b->save_rows < 0 || b->save_rows > h.saves)
    return set_error(GGRS_E_INVALID, "batch counts exceed the mapped shape");
  HIP_TRY(hipSetDevice(e->cfg.device));
  e->lane_frame.clear();  // the lanes' frames moved on the device only
  rc = run_batch(e, b->token_words, b->load_slots, b->adv_rows, b->save_rows, (flags & GGRS_BATCH_STATUS) != 0);
  if (rc) return rc;
  return report_failures(e, v.lane_result, n_failed);
}

int ggrs_handle_requests_lanes(ggrs_engine_t* e, const ggrs_request_t* reqs, const int32_t* offsets,
                               const uint8_t* inputs, const uint8_t* status, uint16_t* save_checksums,
                               int32_t* lane_result) {
  if (!e || !offsets) return set_error(GGRS_E_INVALID, "null argument");
  int rc = check_mode(e);
  if (rc) return rc;
  const int64_t L = e->cfg.num_lanes;
  const int P = e->cfg.num_players;
  if (offsets[0] != 0) return set_error(GGRS_E_INVALID, "offsets[0] must be 0");
  for (int64_t l = 0; l < L; l++)
    if (offsets[l + 1] < offsets[l]) return set_error(GGRS_E_INVALID, "offsets must be non-decreasing (lane %lld)", (long long)l);
  if (offsets[L] > 0 && !reqs) return set_error(GGRS_E_INVALID, "null request list");
  // the shape: the longest list, the most loads / advances / saves of any lane
  int32_t max_tok = 0, max_ld = 0, max_adv = 0, max_sv = 0;
  int64_t n_adv_total = 0;
  for (int64_t l = 0; l < L; l++) {
    int32_t nl = 0, na = 0, ns = 0;
    for (int32_t r = offsets[l]; r < offsets[l + 1]; r++) {
      const int32_t k = reqs[r].kind;
      if (k == GGRS_REQ_SAVE) ++ns;
      else if (k == GGRS_REQ_LOAD) ++nl;
      else if (k == GGRS_REQ_ADVANCE) ++na;
      else return set_error(GGRS_E_INVALID, "lane %lld request %d: unknown kind %d", (long long)l, r - offsets[l], k);
    }
    max_tok = std::max(max_tok, offsets[l + 1] - offsets[l]);
    max_ld = std::max(max_ld, nl);
    max_adv = std::max(max_adv, na);
    max_sv = std::max(max_sv, ns);
    n_adv_total += na;
  }
  if (n_adv_total > 0 && !inputs) return set_error(GGRS_E_INVALID, "inputs required for AdvanceFrame requests");
  const int32_t W = (max_tok + GGRS_TOKENS_PER_WORD - 1) / GGRS_TOKENS_PER_WORD;
  rc = check_shape(W, max_ld, max_adv, max_sv);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(e->cfg.device));
  rc = map_batch(e, W, max_ld, max_adv, max_sv);
  if (rc) return rc;
  // every lane's frame at the start of its list: the Save frames are checked on the host
  if ((int64_t)e->lane_frame.size() != L) {
    e->lane_frame.assign(L, 0);
    std::vector<int32_t> fr(L);
    HIP_TRY(hipMemcpyAsync(fr.data(), e->cur, 4 * L, hipMemcpyDeviceToHost, e->stream));  // frame field row
    HIP_TRY(hipStreamSynchronize(e->stream));
    e->lane_frame = fr;
  }
  ggrs_lane_batch_t v;
  fill_batch_view(e, &v);
  std::vector<int32_t> host_err(L, -1);
  int64_t adv_at = 0;
  for (int64_t l = 0; l < L; l++) {
    uint32_t word = 0;
    int32_t nl = 0, na = 0, k = 0;
    int32_t frame = e->lane_frame[l];
    for (int32_t r = offsets[l]; r < offsets[l + 1]; r++, k++) {
      const int32_t kind = reqs[r].kind;
      uint32_t tok;
      if (kind == GGRS_REQ_SAVE) {
        if (reqs[r].frame != frame && host_err[l] < 0) host_err[l] = k;  // ex_game.rs:104
        tok = GGRS_TOK_SAVE;
      } else if (kind == GGRS_REQ_LOAD) {
        v.load_frames[(int64_t)nl * L + l] = reqs[r].frame;
        frame = reqs[r].frame;
        tok = GGRS_TOK_LOAD;
        ++nl;
      } else {
        const uint8_t* src = inputs + adv_at * P;
        std::memcpy(v.inputs + ((int64_t)na * L + l) * P, src, P);
        if (status) std::memcpy(v.status + ((int64_t)na * L + l) * P, status + adv_at * P, P);
        ++frame;
        ++adv_at;
        tok = GGRS_TOK_ADVANCE;
        ++na;
      }
      word |= tok << (2 * (k & 15));
      if ((k & 15) == 15) {
        v.tokens[(int64_t)(k >> 4) * L + l] = word;
        word = 0;
      }
    }
    // END after the list, then every remaining word all END
    for (int32_t kk = k; kk < W * GGRS_TOKENS_PER_WORD; kk++) {
      word |= (uint32_t)GGRS_TOK_END << (2 * (kk & 15));
      if ((kk & 15) == 15) {
        v.tokens[(int64_t)(kk >> 4) * L + l] = word;
        word = 0;
      }
    }
    if (host_err[l] >= 0) {  // the lane does not run: an empty list
      for (int32_t w = 0; w < W; w++) v.tokens[(int64_t)w * L + l] = 0xffffffffu;
    }
  }
  rc = run_batch(e, W, max_ld, max_adv, max_sv, status != nullptr);
  if (rc) return rc;
  // results: per-Save checksums in request order, lane results, the lanes' new frames
  int64_t sv_at = 0;
  for (int64_t l = 0; l < L; l++) {
    int32_t res = v.lane_result[l];
    if (host_err[l] >= 0) res = -(1 + host_err[l]);
    int32_t ns = 0;
    for (int32_t r = offsets[l]; r < offsets[l + 1]; r++) {
      if (reqs[r].kind != GGRS_REQ_SAVE) continue;
      if (save_checksums) save_checksums[sv_at] = res >= 0 ? v.checksums[(int64_t)ns * L + l] : 0;
      ++sv_at;
      ++ns;
    }
    if (res >= 0) e->lane_frame[l] = res;
    if (lane_result) lane_result[l] = res;
    v.lane_result[l] = res;
  }
  int32_t n_failed = 0;
  return report_failures(e, v.lane_result, &n_failed);
}

int ggrs_read_lane_frames(ggrs_engine_t* e, int32_t* frames) {
  if (!e || !frames) return set_error(GGRS_E_INVALID, "null argument");
  HIP_TRY(hipSetDevice(e->cfg.device));
  int rc = ggrs_synchronize(e);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(frames, e->cur, 4 * (size_t)e->cfg.num_lanes, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

}  // extern "C"
