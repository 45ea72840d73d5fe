// p2p_sched.hip -- P2PSession::advance_frame (src/sessions/p2p_session.rs:265-426) for S sessions of
// one peer under a real network: every session's remote inputs arrive on its own schedule
// (ggrs_p2p_add_arrivals: the newest remote frame each call's poll_remote_clients delivered, and
// Event::Disconnected bits), so each session rolls back to its own earliest misprediction with its
// own depth, stops advancing at the prediction threshold, and rolls back to a disconnected
// player's last frame + 1 and replays it with InputStatus::Disconnected.  The fixed-latency kernels
// of p2p.hip (remote input of frame g at exactly call g + D for every session) stay the fast paths
// for that uniform network; this is the general one.  Checked against oracle_p2p_sched_run
// (oracle/ggrs_oracle.c), which steps the restated InputQueue / SyncLayer / P2PSession.
//
// One thread per session, each its own step sequence (as p2p_flat_kernel): an iteration is one
// AdvanceFrame of the lane's current work -- a replayed frame, or its call's own frame -- or a call
// that does not advance; the call start (poll, disconnect events, first save, rollback decision)
// runs in the iteration that begins the call.
//
// Per-session device state (between launches, HBM):
//   cur   [F][S] u32        the game state after the last call (the handler's State)
//   ring  [S][R][C] u32     saved cells (p2p.hip's session-major layout), ring_frame [R][S] their frames
//   iq    [Q][S] u32        the InputQueues' inputs: byte k = player k's input of frame q (slot q % Q,
//                           Q = INPUT_QUEUE_LENGTH = 128, input_queue.rs:6); local bytes written by
//                           add_local_input, remote bytes by the poll
//   sst   [fields][S] i32   SyncLayer current/last_confirmed/last_saved frames, disconnect_frame,
//                           the newest delivered remote frame, local players' last queued frame,
//                           skipped calls, the session's error, the disconnected mask, and per
//                           player last_frame (local_connect_status), prediction frame / input,
//                           first_incorrect_frame, last_requested_frame (input_queue.rs:10-37)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "common.h"
#include "p2p_engine.h"

#pragma clang fp contract(off)

using namespace ggrs;

namespace {

constexpr int32_t kNull = GGRS_NULL_FRAME;
constexpr int kQ = 128;  // INPUT_QUEUE_LENGTH (input_queue.rs:6)
constexpr int kBlock = 64;

enum : int { kCur = 0, kLconf, kDframe, kLastSaved, kDelivered, kLocalLast, kSkips, kErr, kDisc, kPl0 };
constexpr int kPlFields = 5;  // per player: last_frame, prediction.frame, prediction.input, first_incorrect, last_requested
__host__ __device__ constexpr int sched_fields(int P) { return kPl0 + kPlFields * P; }
__host__ __device__ constexpr int cell_dwords_s(int p) { return (state_fields(p) + 1 + 3) & ~3; }

struct SchedParams {
  int64_t S;
  int32_t R, delay, cap, maxp, c0, n, predictor, sparse;
  uint32_t local_mask;
  uint32_t* cur;
  uint32_t* ring;
  int32_t* ring_frame;
  const uint8_t* inputs;
  const int32_t* row_tag;
  const int32_t* arrive;
  const uint8_t* events;
  uint32_t* iq;
  int32_t* sst;
  int32_t* rollbacks;
  int64_t* resim;
};

template <int P>
__device__ inline uint4* sched_cell(const SchedParams& p, int32_t slot, int64_t s) {
  return reinterpret_cast<uint4*>(p.ring + ((int64_t)s * p.R + slot) * cell_dwords_s(P));
}

template <int P>
__device__ inline void load_cell_s(BoxState<P>& st, const uint4* c) {
  constexpr int F = state_fields(P);
#pragma unroll
  for (int k = 0; k < cell_dwords_s(P) / 4; k++) {
    const uint4 v = c[k];
    const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (4 * k + i < F) st.w[4 * k + i] = x[i];
  }
}
// a cell = the state's F fields, then the fletcher16 handed to GameStateCell::save, zero padding
template <int P>
__device__ inline void store_cell_s(const BoxState<P>& st, uint32_t ck, uint4* c) {
  constexpr int F = state_fields(P);
#pragma unroll
  for (int k = 0; k < cell_dwords_s(P) / 4; k++) {
    uint32_t x[4];
#pragma unroll
    for (int i = 0; i < 4; i++) x[i] = 4 * k + i < F ? st.w[4 * k + i] : (4 * k + i == F ? ck : 0u);
    c[k] = make_uint4(x[0], x[1], x[2], x[3]);
  }
}

template <int P>
__global__ __launch_bounds__(kBlock) void p2p_sched_kernel(SchedParams p) {
  const int64_t S = p.S;
  const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (s >= S) return;  // (no block-level synchronisation in this kernel)
  const uint32_t lmask = p.local_mask;
  uint32_t lbytes = 0;
#pragma unroll
  for (int k = 0; k < P; k++) lbytes |= ((lmask >> k) & 1u) ? 0xffu << (8 * k) : 0u;
  const int32_t maxp = p.maxp, R = p.R;

  // ---- the session's state
  BoxState<P> st;
  load_state<P>(st, p.cur + s, S);
  auto fld = [&](int f) -> int32_t& { return p.sst[(int64_t)f * S + s]; };
  int32_t cur = fld(kCur), lconf = fld(kLconf), dframe = fld(kDframe), last_saved = fld(kLastSaved);
  int32_t delivered = fld(kDelivered), local_last = fld(kLocalLast), skips = fld(kSkips), err = fld(kErr);
  uint32_t disc = (uint32_t)fld(kDisc);
  int32_t lf[P], pf[P], pin[P], finc[P], lreq[P];
#pragma unroll
  for (int k = 0; k < P; k++) {
    lf[k] = fld(kPl0 + kPlFields * k + 0);
    pf[k] = fld(kPl0 + kPlFields * k + 1);
    pin[k] = fld(kPl0 + kPlFields * k + 2);
    finc[k] = fld(kPl0 + kPlFields * k + 3);
    lreq[k] = fld(kPl0 + kPlFields * k + 4);
  }
  int32_t rollbacks = 0;
  int64_t resim = 0;
  // every state the launch steps descends from cur or from a ring cell this engine wrote, all in the
  // lean step's rotation domain: one wave-wide test instead of one per player per step
  const bool lean_ok = __all(rot_in_domain<P>(st));

  uint32_t* const iq = p.iq + s;
  auto iq_at = [&](int32_t q) -> uint32_t& { return iq[(int64_t)(q & (kQ - 1)) * S]; };
  auto next_slot = [&](int32_t x) { return x + 1 == R ? 0 : x + 1; };
  int32_t slot_f = cur % R;  // ring slot of the current frame

  // SaveGameState(h) into `slot` (sync_layer.rs:208-215 + ex_game.rs:103-108)
  auto save = [&](int32_t h, int32_t slot) {
    store_cell_s<P>(st, fletcher16_state<P>(st), sched_cell<P>(p, slot, s));
    p.ring_frame[(int64_t)slot * S + s] = h;
    last_saved = h;
  };

  // synchronized_inputs(h) (sync_layer.rs:280-293) with InputQueue::input (input_queue.rs:104-167)
  auto sync_inputs = [&](int32_t h) -> uint32_t {
    const uint32_t w = iq_at(h);
    uint32_t in = 0;
#pragma unroll
    for (int k = 0; k < P; k++) {
      uint32_t v;
      if ((lmask >> k) & 1u) {
        v = (w >> (8 * k)) & 0xffu;  // local queues hold every frame <= current + delay
      } else if (((disc >> k) & 1u) && lf[k] < h) {
        v = 4u;  // InputStatus::Disconnected: ex_game spins the ship (ex_game.rs:280)
      } else {
        lreq[k] = h;
        if (pf[k] < 0 && h <= lf[k]) {
          v = (w >> (8 * k)) & 0xffu;  // confirmed
        } else {
          if (pf[k] < 0) {  // a new prediction from the last added input
            const bool prev = !(h == 0 || lf[k] == kNull);
            const uint32_t last = prev ? (iq_at(lf[k]) >> (8 * k)) & 0xffu : 0u;
            pin[k] = (int32_t)(prev ? (p.predictor == 0 ? last : 0u) : 0u);  // lib.rs:390-406
            pf[k] = (prev ? lf[k] : kNull) + 1;
          }
          v = (uint32_t)pin[k];
        }
      }
      in |= v << (8 * k);
    }
    return in;
  };

  const int32_t c_end = p.c0 + p.n;
  int32_t c = err ? c_end : p.c0;
  bool at_start = true, replaying = false, window_done = false, save_own = false;
  int32_t h = 0, load = 0, slot_h = 0, confirmed = kNull;
  // adjust_gamestate's LoadGameState + reset_prediction (p2p_session.rs:658-714)
  auto begin_replay = [&](int32_t from) -> bool {
    if (from == kNull || from >= cur || from < cur - maxp) return false;  // load_frame's asserts
    const int32_t sh = slot_f - (cur - from);
    slot_h = sh < 0 ? sh + R : sh;
    if (p.ring_frame[(int64_t)slot_h * S + s] != from) return false;  // cell.frame == frame_to_load
    load_cell_s<P>(st, sched_cell<P>(p, slot_h, s));
#pragma unroll
    for (int k = 0; k < P; k++) {
      pf[k] = kNull;
      finc[k] = kNull;
      lreq[k] = kNull;
    }
    load = from;
    h = from;
    replaying = true;
    rollbacks += 1;
    resim += cur - from;
    return true;
  };

  while (c < c_end) {
    if (at_start) {
      const int32_t ci = c % p.cap;
      // 1. poll_remote_clients: the burst of remote frames (delivered, arrive_upto[c]]
      const int32_t up = p.arrive[(int64_t)ci * S + s];
      if (up > c) { err = GGRS_E_INVALID; break; }  // the remote peer cannot have sent a later frame
      uint32_t cbytes = 0;  // bytes of the remote players still connected
#pragma unroll
      for (int k = 0; k < P; k++)
        if (!((lmask >> k) & 1u) && !((disc >> k) & 1u)) cbytes |= 0xffu << (8 * k);
      for (int32_t g = delivered + 1; g <= up; ++g) {
        // the device queue keeps 128 frames (INPUT_QUEUE_LENGTH); a frame this far ahead of the
        // session would overwrite one a rollback may still read (the reference's queue panics)
        if (g >= cur - maxp + kQ - 1) { err = GGRS_E_PRECONDITION; break; }
        const int32_t gi = g % p.cap;
        if (p.row_tag[gi] != g) { err = GGRS_E_PRECONDITION; break; }  // input row no longer queued
        const uint32_t row = load_inputs<P>(p.inputs, (int64_t)gi * S + s);
        uint32_t& q = iq_at(g);
        q = (q & ~cbytes) | (row & cbytes);
#pragma unroll
        for (int k = 0; k < P; k++) {  // Event::Input -> add_remote_input (p2p_session.rs:880-895)
          if (!((cbytes >> (8 * k)) & 1u)) continue;
          const int32_t v = (int32_t)((row >> (8 * k)) & 0xffu);
          if (pf[k] != kNull) {  // add_input_by_frame (input_queue.rs:190-230)
            if (finc[k] == kNull && pin[k] != v) finc[k] = g;
            if (pf[k] == lreq[k] && finc[k] == kNull) pf[k] = kNull;
            else pf[k] += 1;
          }
          lf[k] = g;
        }
      }
      if (err) break;
      delivered = max(delivered, up);
      // Event::Disconnected (p2p_session.rs:866-878 -> disconnect_player_at_frame :618-655)
      const uint32_t ev = p.events ? p.events[(int64_t)ci * S + s] : 0u;
#pragma unroll
      for (int k = 0; k < P; k++) {
        if (!((ev >> k) & 1u) || ((lmask >> k) & 1u) || ((disc >> k) & 1u)) continue;
        disc |= 1u << k;
        if (cur > lf[k]) dframe = lf[k] + 1;
      }
      // 2. the first frame's save (:305-308)
      if (cur == 0) save(0, slot_f);
      // confirmed_frame (:542-553): the newest frame every connected player has sent
      confirmed = INT32_MAX;
#pragma unroll
      for (int k = 0; k < P; k++) {
        if ((disc >> k) & 1u) continue;
        confirmed = min(confirmed, ((lmask >> k) & 1u) ? local_last : lf[k]);
      }
      if (confirmed == INT32_MAX) { err = GGRS_E_PRECONDITION; break; }  // assert!(confirmed < i32::MAX)
      // 3. check_simulation_consistency(disconnect_frame) (sync_layer.rs:343-353) + adjust_gamestate
      int32_t first_inc = dframe;
#pragma unroll
      for (int k = 0; k < P; k++)
        if (finc[k] != kNull && (first_inc == kNull || finc[k] < first_inc)) first_inc = finc[k];
      if (first_inc != kNull) {
        if (!begin_replay(p.sparse ? last_saved : first_inc)) { err = GGRS_E_PRECONDITION; break; }
        dframe = kNull;
      }
      window_done = false;
      save_own = false;
      at_start = false;
    }
    // sparse saving: check_last_saved_state (:819-843) once the rollback's replay is done
    if (p.sparse && !replaying && !window_done) {
      window_done = true;
      if (cur - last_saved >= maxp) {
        if (confirmed >= cur) save_own = true;
        else if (!begin_replay(last_saved)) { err = GGRS_E_PRECONDITION; break; }
      }
    }
    bool do_save, adv;
    int32_t fr, sslot;
    if (replaying) {
      fr = h;
      sslot = slot_h;
      do_save = p.sparse ? h == confirmed : h > load;  // (:692-702)
      adv = true;
    } else {
      fr = cur;
      sslot = slot_f;
      do_save = p.sparse ? save_own : true;  // SaveGameState(current) (:337)
      // set_last_confirmed_frame (sync_layer.rs:313-340), after this call's saves
      int32_t lc = confirmed;
      const int32_t ls = do_save ? cur : last_saved;
      if (p.sparse && ls < lc) lc = ls;
      if (cur < lc) lc = cur;
      lconf = lc;
      // add_local_input for every local player (:362-377, input_queue.rs:170-186): queue frame
      // current + delay, dropped unless it is the next one; the first fills the frames below the
      // delay with the default input
      if (lbytes) {
        const int32_t qf = cur + p.delay;
        if (local_last == kNull || qf == local_last + 1) {
          if (local_last == kNull)
            for (int32_t q = 0; q < p.delay; q++) iq_at(q) &= ~lbytes;
          const uint32_t row = load_inputs<P>(p.inputs, (int64_t)(c % p.cap) * S + s);
          uint32_t& w = iq_at(qf);
          w = (w & ~lbytes) | (row & lbytes);
          local_last = qf;
        }
      }
      // the prediction threshold (:393-423)
      const int32_t ahead = lconf == kNull ? cur : cur - lconf;
      adv = ahead < maxp;
    }
    uint32_t in = 0;
    if (adv) in = sync_inputs(fr);
    if (do_save) save(fr, sslot);
    if (adv) {
      if (lean_ok) advance_state_lean<P>(st, in);
      else advance_state<P>(st, in, 0u);
    }
    if (replaying) {
      ++h;
      slot_h = next_slot(slot_h);
      replaying = h != cur;
    } else {
      if (adv) {
        ++cur;
        slot_f = next_slot(slot_f);
      } else {
        ++skips;
      }
      ++c;
      at_start = true;
    }
  }
  store_state<P>(st, p.cur + s, S);
  fld(kCur) = cur;
  fld(kLconf) = lconf;
  fld(kDframe) = dframe;
  fld(kLastSaved) = last_saved;
  fld(kDelivered) = delivered;
  fld(kLocalLast) = local_last;
  fld(kSkips) = skips;
  fld(kErr) = err;
  fld(kDisc) = (int32_t)disc;
#pragma unroll
  for (int k = 0; k < P; k++) {
    fld(kPl0 + kPlFields * k + 0) = lf[k];
    fld(kPl0 + kPlFields * k + 1) = pf[k];
    fld(kPl0 + kPlFields * k + 2) = pin[k];
    fld(kPl0 + kPlFields * k + 3) = finc[k];
    fld(kPl0 + kPlFields * k + 4) = lreq[k];
  }
  p.rollbacks[s] += rollbacks;
  p.resim[s] += resim;
}

// every session at frame 0, nothing arrived, every player connected (SyncLayer::new,
// InputQueue::new, P2PSession::new: input_queue.rs:40-53, sync_layer.rs:183-198)
__global__ void sched_init_kernel(int32_t* sst, int64_t S, int32_t P) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)sched_fields(P) * S) return;
  const int f = (int)(i / S);
  int32_t v = kNull;
  if (f == kCur || f == kSkips || f == kErr || f == kDisc) v = 0;
  if (f >= kPl0 && (f - kPl0) % kPlFields == 2) v = 0;  // prediction.input
  sst[i] = v;
}

}  // namespace

namespace ggrs {

int p2p_sched_free(ggrs_p2p_engine* e) {
  void* bufs[] = {e->arrive, e->events, e->row_tag, e->iq, e->sst};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  e->arrive = nullptr;
  e->events = nullptr;
  e->row_tag = nullptr;
  e->iq = nullptr;
  e->sst = nullptr;
  return GGRS_OK;
}

int p2p_sched_enable(ggrs_p2p_engine* e) {
  const int64_t S = e->cfg.num_sessions;
  const int P = e->cfg.num_players;
  HIP_TRY(hipSetDevice(e->cfg.device));
  if (!e->sst) {
    HIP_TRY(hipMalloc(&e->arrive, sizeof(int32_t) * (size_t)e->cap * S));
    HIP_TRY(hipMalloc(&e->events, (size_t)e->cap * S));
    HIP_TRY(hipMalloc(&e->row_tag, sizeof(int32_t) * (size_t)e->cap));
    HIP_TRY(hipMalloc(&e->iq, sizeof(uint32_t) * (size_t)kQ * S));
    HIP_TRY(hipMalloc(&e->sst, sizeof(int32_t) * (size_t)sched_fields(P) * S));
  }
  if (!e->ring_frame) HIP_TRY(hipMalloc(&e->ring_frame, sizeof(int32_t) * e->R * S));
  HIP_TRY(hipMemsetAsync(e->ring_frame, 0xff, sizeof(int32_t) * e->R * S, e->stream));  // NULL_FRAME
  HIP_TRY(hipMemsetAsync(e->events, 0, (size_t)e->cap * S, e->stream));
  HIP_TRY(hipMemsetAsync(e->iq, 0, sizeof(uint32_t) * (size_t)kQ * S, e->stream));
  e->row_tag_host.assign((size_t)e->cap, kNull);
  for (int32_t g = 0; g < e->next_input_frame; g++)
    if (g > e->next_input_frame - 1 - e->cap) e->row_tag_host[(size_t)(g % e->cap)] = g;
  HIP_TRY(hipMemcpyAsync(e->row_tag, e->row_tag_host.data(), sizeof(int32_t) * e->cap, hipMemcpyHostToDevice,
                         e->stream));
  sched_init_kernel<<<grid_of((int64_t)sched_fields(P) * S, 256), 256, 0, e->stream>>>(e->sst, S, P);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->sched = 1;
  return GGRS_OK;
}

int p2p_sched_advance(ggrs_p2p_engine* e, int32_t n) {
  if ((int64_t)e->current_frame + n > e->next_arrival_call)
    return set_error(GGRS_E_INVALID, "Missing arrivals: arrival rows are queued up to call %d, calls need up to %d",
                     e->next_arrival_call - 1, e->current_frame + n - 1);
  if (n > e->cap) {  // a launch reads at most cap calls' arrival rows
    int rc = p2p_sched_advance(e, e->cap);
    if (rc) return rc;
    return p2p_sched_advance(e, n - e->cap);
  }
  SchedParams p;
  p.S = e->cfg.num_sessions;
  p.R = e->R;
  p.delay = e->cfg.input_delay;
  p.cap = e->cap;
  p.maxp = e->cfg.max_prediction;
  p.c0 = e->current_frame;
  p.n = n;
  p.predictor = e->cfg.predictor;
  p.sparse = e->sparse;
  p.local_mask = (uint32_t)e->cfg.local_mask;
  p.cur = e->cur;
  p.ring = e->ring;
  p.ring_frame = e->ring_frame;
  p.inputs = e->inputs;
  p.row_tag = e->row_tag;
  p.arrive = e->arrive;
  p.events = e->events;
  p.iq = e->iq;
  p.sst = e->sst;
  p.rollbacks = e->rollbacks;
  p.resim = e->resim;
  if (int rc = e->timer.before(e->stream)) return rc;
  dispatch_players(e->cfg.num_players, [&](auto PC) {
    constexpr int PP = decltype(PC)::value;
    p2p_sched_kernel<PP><<<(unsigned)grid_of(p.S, kBlock), kBlock, 0, e->stream>>>(p);
  });
  HIP_TRY(hipGetLastError());
  e->timer.count();
  e->current_frame += n;
  return GGRS_OK;
}

}  // namespace ggrs

extern "C" {

int ggrs_p2p_set_arrival_schedule(ggrs_p2p_engine_t* e, int32_t on) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (e->current_frame != 0)
    return set_error(GGRS_E_STATE, "the network model is part of the session's configuration (set before the first call)");
  if (!on) {
    e->sched = 0;
    return GGRS_OK;
  }
  if (e->cfg.max_prediction < 1)
    return set_error(GGRS_E_INVALID, "scheduled arrivals need rollback mode (max_prediction >= 1)");
  if (e->cfg.max_prediction + e->cfg.input_delay + 2 >= kQ)
    return set_error(GGRS_E_INVALID, "max_prediction + input_delay must be < %d (the device input queue)", kQ - 2);
  if (e->desync_interval > 0 || e->trace)
    return set_error(GGRS_E_STATE, "scheduled arrivals support neither desync detection nor the display-checksum trace");
  return p2p_sched_enable(e);
}

int ggrs_p2p_add_arrivals(ggrs_p2p_engine_t* e, int32_t first_call, int32_t n, const int32_t* arrive_upto,
                          const uint8_t* events) {
  if (!e || (!arrive_upto && n > 0)) return set_error(GGRS_E_INVALID, "null argument");
  if (!e->sched) return set_error(GGRS_E_STATE, "arrival schedules need ggrs_p2p_set_arrival_schedule(e, 1)");
  if (n < 0) return set_error(GGRS_E_INVALID, "n_calls must be >= 0");
  if (first_call != e->next_arrival_call)
    return set_error(GGRS_E_INVALID, "arrivals must be added in call order (expected call %d, got %d)",
                     e->next_arrival_call, first_call);
  if (n == 0) return GGRS_OK;
  if ((int64_t)first_call + n - 1 - e->current_frame >= e->cap)
    return set_error(GGRS_E_INVALID, "arrival queue full (capacity %d calls)", e->cap);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t S = e->cfg.num_sessions;
  // rows wrap at cap: copy in at most two pieces per table
  for (int32_t k = 0; k < n;) {
    const int32_t slot = (first_call + k) % e->cap;
    const int32_t m = std::min(n - k, e->cap - slot);
    HIP_TRY(hipMemcpyAsync(e->arrive + (int64_t)slot * S, arrive_upto + (int64_t)k * S, sizeof(int32_t) * m * S,
                           hipMemcpyHostToDevice, e->stream));
    if (events)
      HIP_TRY(hipMemcpyAsync(e->events + (int64_t)slot * S, events + (int64_t)k * S, (size_t)m * S,
                             hipMemcpyHostToDevice, e->stream));
    else
      HIP_TRY(hipMemsetAsync(e->events + (int64_t)slot * S, 0, (size_t)m * S, e->stream));
    k += m;
  }
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->next_arrival_call = first_call + n;
  return GGRS_OK;
}

int ggrs_p2p_read_sessions(ggrs_p2p_engine_t* e, int32_t* frames, int32_t* skipped, int32_t* errors) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (!e->sched) return set_error(GGRS_E_STATE, "per-session frames exist in scheduled mode only");
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t S = e->cfg.num_sessions;
  if (frames) HIP_TRY(hipMemcpyAsync(frames, e->sst + (int64_t)kCur * S, 4 * S, hipMemcpyDeviceToHost, e->stream));
  if (skipped) HIP_TRY(hipMemcpyAsync(skipped, e->sst + (int64_t)kSkips * S, 4 * S, hipMemcpyDeviceToHost, e->stream));
  if (errors) HIP_TRY(hipMemcpyAsync(errors, e->sst + (int64_t)kErr * S, 4 * S, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

}  // extern "C"
