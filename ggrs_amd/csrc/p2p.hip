// p2p.hip -- the P2P rollback decision on the device: one peer's P2PSession::advance_frame
// (src/sessions/p2p_session.rs:265-426) for S independent sessions, one thread per session,
// with the remote players' InputQueue prediction (src/input_queue.rs:104-230) kept per session in
// registers.  Network model (the oracle's, oracle/ggrs_oracle.c oracle_p2p_run): the remote
// players' input of frame g arrives at the start of call g + D (D = remote_latency); local
// players' inputs enter every call with the session's input delay.
//
// What a call does for every session (rollback mode, sparse saving off, every player connected):
//   1. poll: each remote queue gets frame g = f - D (add_input_by_frame, input_queue.rs:190-230):
//      a prediction that disagrees sets first_incorrect_frame = g;
//   2. f == 0: SaveGameState(0)  (:305-308);
//   3. first_incorrect = min over queues (check_simulation_consistency, sync_layer.rs:343-353);
//      if set: LoadGameState(first_incorrect), reset_prediction, then (Save unless first, Advance)
//      for frames first_incorrect .. f-1 with synchronized_inputs (adjust_gamestate :658-714);
//   4. SaveGameState(f) (:337);
//   5. AdvanceFrame with synchronized_inputs(f): local inputs confirmed (queue frame f holds user
//      input f - delay, the default input below the delay), remote inputs predicted.
// D < max_prediction is required, so the prediction threshold (:400-421) never stops a call and
// every confirmed frame the reference would discard is older than anything read again.
//
// Because the remote input of frame g arrives exactly at call g + D, a rollback always loads
// frame f - D; which sessions roll back is decided per session by its own predictions.
//
// HBM layout (session-fastest SoA, as the SyncTest engine):
//   cur      [F][S]     u32   state after the last call
//   ring     [S][R][C]  u32   R = max_prediction + 1, slot = frame % R (sync_layer.rs:161-166); one
//                            session's cells are contiguous, C = F rounded up to whole 16-byte pieces
//                            (a save is C/4 dwordx4 stores into 1-2 cache lines that the session's
//                            next saves complete, whatever frame the other lanes of the wave are at)
//            (cell dword F: the fletcher16 handed to GameStateCell::save, so a save is one record)
//   inputs   [C][S][Pp] u8    row g: local add_local_input of call g, remote inputs of frame g
//   queue    [4][P][S]  i32   prediction.frame, prediction.input, first_incorrect, last_requested
//   stats    rollbacks [S] i32, resim [S] i64
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "p2p_engine.h"

#pragma clang fp contract(off)

using namespace ggrs;

namespace {

constexpr int32_t kNull = -1;  // NULL_FRAME (src/lib.rs:44)

struct P2PParams {
  int64_t S;
  int32_t R, D, delay, cap, trace_cap, f0, n, predictor;
  uint32_t local_mask;
  uint32_t* cur;
  uint32_t* ring;
  const uint8_t* inputs;
  int32_t* queue;
  int32_t* rollbacks;
  int64_t* resim;
  uint16_t* trace;
  // desync detection (p2p_session.rs:939-975): interval (0 off) and the local checksum history,
  // [kHist][S] u16, slot (frame / interval) % kHist
  int32_t desync_interval;
  uint16_t* hist;
  // debug: the advance FROM dbg_frame of session dbg_sess flips x0's lowest bit (every replay)
  int64_t dbg_sess;
  int32_t dbg_frame;
  // sparse saving (builder.rs:160-169): saves only at min_confirmed, rollbacks from the last save
  int32_t sparse;
  int32_t* last_saved;  // [S] SyncLayer::last_saved_frame (sparse mode)
  int32_t* ring_frame;  // [R][S] frame each cell holds (sparse mode: saves vary per session)
};

constexpr int kHist = 32;  // MAX_CHECKSUM_HISTORY_SIZE (protocol.rs:27)

// The per-session state of every remote player's InputQueue that the P2P program reads.
template <int P>
struct RemoteQueues {
  int32_t pred_frame[P];  // prediction.frame (NULL: not predicting)
  uint32_t pred_in[P];    // prediction.input
  int32_t first_inc[P];   // first_incorrect_frame
  int32_t last_req[P];    // last_requested_frame
};

// dwords of one ring cell: the state's F fields and the checksum, padded to whole 16-byte pieces
__host__ __device__ constexpr int cell_dwords(int p) { return (state_fields(p) + 1 + 3) & ~3; }

template <int P>
__device__ inline uint4* ring_cell(const P2PParams& p, int32_t slot, int64_t sess) {
  return reinterpret_cast<uint4*>(p.ring + ((int64_t)sess * p.R + slot) * cell_dwords(P));
}
template <int P>
__device__ inline void load_cell(BoxState<P>& s, const uint4* c) {
  constexpr int F = state_fields(P);
#pragma unroll
  for (int k = 0; k < cell_dwords(P) / 4; k++) {
    const uint4 v = c[k];
    const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (4 * k + i < F) s.w[4 * k + i] = x[i];
  }
}
template <int P>
__device__ inline void store_cell(const BoxState<P>& s, uint32_t ck, uint4* c) {
  constexpr int F = state_fields(P);
#pragma unroll
  for (int k = 0; k < cell_dwords(P) / 4; k++) {
    uint32_t x[4];
#pragma unroll
    for (int i = 0; i < 4; i++) x[i] = 4 * k + i < F ? s.w[4 * k + i] : (4 * k + i == F ? ck : 0u);
    c[k] = make_uint4(x[0], x[1], x[2], x[3]);
  }
}
// the checksum stored with the cell of `slot`
template <int P>
__device__ inline uint16_t cell_checksum(const P2PParams& p, int32_t slot, int64_t sess) {
  return (uint16_t)(p.ring + ((int64_t)sess * p.R + slot) * cell_dwords(P))[state_fields(P)];
}

template <int P>
__device__ inline void save_cell(const P2PParams& p, const BoxState<P>& s, int32_t frame, int64_t sess) {
  store_cell<P>(s, fletcher16_state<P>(s), ring_cell<P>(p, frame % p.R, sess));
}

// Input rows as the calls read them: from global memory, or (staged kernel) from the block's LDS
// copy of rows [lo, lo + kP2PRows) -- one LDS byte read instead of a dependent global load.
constexpr int kP2PRows = 64;
constexpr int kP2PBlock = 256;

template <int P>
struct GlobalRows {
  const P2PParams& p;
  int64_t sess;
  __device__ inline uint32_t operator()(int32_t g) const {
    return load_inputs<P>(p.inputs, (int64_t)(g % p.cap) * p.S + sess);
  }
};
template <int P>
struct LdsRows {
  const uint8_t* lds;  // [kP2PRows][kP2PBlock][Pp]
  int32_t lo;
  int tid;
  __device__ inline uint32_t operator()(int32_t g) const {
    using T = typename InputWord<P>::T;
    return (uint32_t)reinterpret_cast<const T*>(lds)[(g - lo) * kP2PBlock + tid];
  }
};

// synchronized_inputs(h) (sync_layer.rs:280-293) with InputQueue::input (input_queue.rs:104-167).
// last_added: the remote queues' last_added_frame (f - D after this call's poll, or NULL).
template <int P, typename Rows>
__device__ inline uint32_t sync_inputs(const P2PParams& p, RemoteQueues<P>& q, int32_t h, int32_t last_added,
                                       const Rows& input_row, uint32_t local_mask) {
  uint32_t in = 0;
  // local queues hold every frame <= f + delay: queue frame h is user input h - delay, and the
  // frames below the delay replicate the default input (input_queue.rs:233-265)
  const uint32_t local_row = (local_mask && h >= p.delay) ? input_row(h - p.delay) : 0u;
  uint32_t confirmed_row = 0u, last_row = 0u;
  const bool confirmed = last_added != kNull && h <= last_added;
  if (confirmed) confirmed_row = input_row(h);
  else if (last_added != kNull && h != 0) last_row = input_row(last_added);
#pragma unroll
  for (int k = 0; k < P; k++) {
    uint32_t v;
    if ((local_mask >> k) & 1u) {
      v = (local_row >> (8 * k)) & 0xffu;
    } else {
      q.last_req[k] = h;
      if (q.pred_frame[k] < 0) {
        if (confirmed) {  // the queue holds frame h
          in |= ((confirmed_row >> (8 * k)) & 0xffu) << (8 * k);
          continue;
        }
        const bool prev = !(h == 0 || last_added == kNull);
        const uint32_t last = (last_row >> (8 * k)) & 0xffu;
        q.pred_in[k] = prev ? (p.predictor == 0 ? last : 0u) : 0u;  // lib.rs:390-406, unwrap_or_default
        q.pred_frame[k] = (prev ? last_added : kNull) + 1;
      }
      v = q.pred_in[k];
    }
    in |= v << (8 * k);
  }
  return in;
}

// kStaged: the block's input rows are copied to LDS per chunk of calls (one coalesced pass over
// rows [f - back, chunk end)), so the calls' input reads are LDS reads; every thread of the block
// runs the same calls, idle tail threads included (they never store).
template <int P, bool kStaged>
__global__ __launch_bounds__(kP2PBlock) void p2p_kernel(P2PParams p) {
  const uint32_t lmask = p.local_mask;
  constexpr int Pp = P <= 1 ? 1 : (P == 2 ? 2 : 4);
  __shared__ __attribute__((aligned(16))) uint8_t lds_rows[kStaged ? kP2PRows * kP2PBlock * Pp : 4];
  const int64_t sess0 = (int64_t)blockIdx.x * kP2PBlock;
  const int64_t S = p.S;
  const bool live = sess0 + threadIdx.x < S;
  if (!kStaged && !live) return;
  const int64_t sess = live ? sess0 + threadIdx.x : sess0;  // idle threads shadow the block's first
  const int nb = (int)((S - sess0) < kP2PBlock ? (S - sess0) : kP2PBlock);
  BoxState<P> st;
  load_state<P>(st, p.cur + sess, S);
  RemoteQueues<P> q;
#pragma unroll
  for (int k = 0; k < P; k++) {
    q.pred_frame[k] = p.queue[(0 * P + k) * S + sess];
    q.pred_in[k] = (uint32_t)p.queue[(1 * P + k) * S + sess];
    q.first_inc[k] = p.queue[(2 * P + k) * S + sess];
    q.last_req[k] = p.queue[(3 * P + k) * S + sess];
  }
  int32_t rollbacks = 0;
  int64_t resim = 0;
  const bool dbg = live && sess == p.dbg_sess;
  int32_t last_saved = p.sparse ? p.last_saved[sess] : kNull;
  auto save = [&](int32_t h) {
    if (live) {
      save_cell<P>(p, st, h, sess);
      if (p.sparse) p.ring_frame[(int64_t)(h % p.R) * S + sess] = h;  // GameStateCell.frame
    }
    last_saved = h;
  };
  // rows a call f reads: >= f - back (rollback start, local rows h - delay), <= f
  const int32_t back = (p.sparse ? p.R - 1 : p.D) + p.delay;
  int32_t row_lo = 0;
  auto stage = [&](int32_t lo, int32_t nrows) {
    __syncthreads();
    row_lo = lo;
    const int row_bytes = nb * Pp;
    if (nb == kP2PBlock && ((S * Pp) & 3) == 0) {  // whole dwords: rows are dword aligned
      const int dpr = row_bytes / 4;
      for (int q = threadIdx.x; q < nrows * dpr; q += kP2PBlock) {
        const int r = q / dpr, c = q - r * dpr;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(p.inputs + ((int64_t)((lo + r) % p.cap) * S + sess0) * Pp);
        reinterpret_cast<uint32_t*>(lds_rows + r * kP2PBlock * Pp)[c] = src[c];
      }
    } else {
      for (int q = threadIdx.x; q < nrows * row_bytes; q += kP2PBlock) {
        const int r = q / row_bytes, b = q - r * row_bytes;
        lds_rows[r * kP2PBlock * Pp + b] = p.inputs[((int64_t)((lo + r) % p.cap) * S + sess0) * Pp + b];
      }
    }
    __syncthreads();
  };
  const int tid = live ? (int)threadIdx.x : 0;
  // every state the launch steps descends from cur or from a ring cell; both only ever hold
  // State::new, zeros or advances of such states, all inside the lean step's rotation domain, so
  // one test of cur (and of the prefetched cell, below) replaces a wave vote per player per step
  bool lean_ok = __all(rot_in_domain<P>(st));
  auto advance = [&](uint32_t in) {
    const uint32_t from = st.w[0];
    if (lean_ok) advance_state_lean<P>(st, in);
    else advance_state<P>(st, in, 0u);
    if (dbg && (int32_t)from == p.dbg_frame) st.w[fld_x(P, 0)] ^= 1u;
  };
  // Without sparse saving a rollback at call f always loads frame f - D (the remote input of that
  // frame is the one arriving), and that cell is final once call f - 1 has ended (its last
  // re-save is by call f - 1's rollback at the latest).  So the cell is read at the end of call
  // f - 1, and its load latency overlaps the next poll instead of stalling the rollback.
  BoxState<P> pre;
  int32_t pre_frame = kNull;
  auto prefetch = [&](int32_t fr) {
    if (!p.sparse && fr >= 0) {
      load_cell<P>(pre, ring_cell<P>(p, fr % p.R, sess));
      pre_frame = fr;
    }
  };
  prefetch(p.f0 - p.D);
  lean_ok = lean_ok && __all(pre_frame == kNull || rot_in_domain<P>(pre));
  auto call = [&](int32_t f, const auto& input_row) {
    // 0. check_checksum_send_interval (p2p_session.rs:939-975), before any rollback of this call:
    //    last_confirmed_frame = f - 1 - D and last_saved_frame = f - 1 here, so frame_to_send =
    //    interval, 2 interval, ... goes out at call frame_to_send + D + 1; its cell is in the ring
    //    (D + 1 < R), its checksum enters the local history
    if (p.desync_interval > 0 && live) {
      const int32_t fts = f - 1 - p.D;
      if (fts >= p.desync_interval && fts % p.desync_interval == 0)
        p.hist[(int64_t)((fts / p.desync_interval) % kHist) * S + sess] = cell_checksum<P>(p, fts % p.R, sess);
    }
    // 1. poll_remote_clients: the remote input of frame g = f - D (add_input_by_frame)
    const int32_t g = f - p.D;
    const int32_t last_added = g >= 0 ? g : kNull;
    if (g >= 0) {
      const uint32_t row = input_row(g);
#pragma unroll
      for (int k = 0; k < P; k++) {
        if ((p.local_mask >> k) & 1u) continue;
        if (q.pred_frame[k] != kNull) {
          const uint32_t v = (row >> (8 * k)) & 0xffu;
          if (q.first_inc[k] == kNull && q.pred_in[k] != v) q.first_inc[k] = g;
          if (q.pred_frame[k] == q.last_req[k] && q.first_inc[k] == kNull) q.pred_frame[k] = kNull;
          else q.pred_frame[k] += 1;
        }
      }
    }
    // 2. the first frame's save
    if (f == 0) save(0);
    // confirmed_frame (:542-553): remote players have sent through f - D, local ones through
    // f - 1 + delay, so the minimum is f - D (NULL before the first remote input)
    const int32_t confirmed = f >= p.D ? f - p.D : kNull;
    // 3. check_simulation_consistency + adjust_gamestate (:658-714)
    auto adjust = [&](int32_t first_incorrect) {
      const int32_t load = p.sparse ? last_saved : first_incorrect;  // sparse: the last save
      if (load == pre_frame) st = pre;
      else load_cell<P>(st, ring_cell<P>(p, load % p.R, sess));
#pragma unroll
      for (int k = 0; k < P; k++) {  // reset_prediction (input_queue.rs:63-67)
        q.pred_frame[k] = kNull;
        q.first_inc[k] = kNull;
        q.last_req[k] = kNull;
      }
      for (int32_t h = load; h < f; ++h) {
        const uint32_t in = sync_inputs<P>(p, q, h, last_added, input_row, lmask);
        if (p.sparse ? h == confirmed : h > load) save(h);
        advance(in);
      }
      rollbacks += 1;
      resim += f - load;
    };
    int32_t first_inc = kNull;
#pragma unroll
    for (int k = 0; k < P; k++)
      if (q.first_inc[k] != kNull && (first_inc == kNull || q.first_inc[k] < first_inc)) first_inc = q.first_inc[k];
    if (first_inc != kNull) adjust(first_inc);
    // 4. save the current frame (sparse: check_last_saved_state, :819-843); 5. advance
    if (!p.sparse) {
      save(f);
    } else if (f - last_saved >= p.R - 1) {  // would leave the prediction window
      if (confirmed >= f) save(f);
      else adjust(last_saved);
    }
    const uint32_t in = sync_inputs<P>(p, q, f, last_added, input_row, lmask);
    advance(in);
    if (p.trace && live) p.trace[(int64_t)(f % p.trace_cap) * S + sess] = fletcher16_state<P>(st);
    prefetch(f + 1 - p.D);
  };
  const int32_t f_end = p.f0 + p.n;
  if constexpr (kStaged) {
    const int32_t calls_per_stage = kP2PRows - back;  // >= 1 (host)
    for (int32_t f = p.f0; f < f_end;) {
      const int32_t chunk_end = min(f_end, f + calls_per_stage);
      const int32_t lo = max(0, f - back);
      stage(lo, chunk_end - lo);
      const LdsRows<P> rows{lds_rows, row_lo, tid};
      for (; f < chunk_end; ++f) call(f, rows);
    }
  } else {
    const GlobalRows<P> rows{p, sess};
    for (int32_t f = p.f0; f < f_end; ++f) call(f, rows);
  }
  if (!live) return;
  store_state<P>(st, p.cur + sess, S);
#pragma unroll
  for (int k = 0; k < P; k++) {
    p.queue[(0 * P + k) * S + sess] = q.pred_frame[k];
    p.queue[(1 * P + k) * S + sess] = (int32_t)q.pred_in[k];
    p.queue[(2 * P + k) * S + sess] = q.first_inc[k];
    p.queue[(3 * P + k) * S + sess] = q.last_req[k];
  }
  p.rollbacks[sess] += rollbacks;
  p.resim[sess] += resim;
  if (p.sparse) p.last_saved[sess] = last_saved;
}

// Flattened form (the default without sparse saving): each thread runs its own session's calls
// as a sequence of steps -- one save + one AdvanceFrame per step, a rollback call taking
// f - first_incorrect replay steps before its own -- instead of the calls in lockstep.  In
// lockstep a wave pays a rollback whenever any of its 64 sessions mispredicted (almost every
// call), so every call cost ~D + 1 advances for every session; here a session that did not roll
// back goes on to its next call meanwhile, and a wave's step count is the largest per-session
// count (calls + replays) of a stage.  Same Loads, Saves, AdvanceFrames and InputQueue updates per
// session, in the same order, as p2p_kernel.  One wave per block; input rows staged per stage of
// calls as in the staged form (rows [stage start - back, stage end)), all lanes meeting at the
// stage end.
constexpr int kFlatBlock = 64;
// rows per stage: a wave's steps in a stage are its slowest session's, so fewer, longer stages
// cost less (128 rows: one stage per 64-call launch at back = 6)
constexpr int kFlatRows = 128;
// with the LDS ring: 12 KB of rows (96 at two players: a 64-call launch is one stage) beside a
// ring of at most 28 KB per block, four blocks per CU in 160 KB
template <int P>
constexpr int flat_rows_lds() {
  return 12 * 1024 / (kFlatBlock * (P <= 1 ? 1 : (P == 2 ? 2 : 4)));
}

template <int P>
struct LdsRowsFlat {
  const uint8_t* lds;  // [kFlatRows][kFlatBlock][Pp]
  int32_t lo;
  int tid;
  __device__ inline uint32_t operator()(int32_t g) const {
    using T = typename InputWord<P>::T;
    return (uint32_t)reinterpret_cast<const T*>(lds)[(g - lo) * kFlatBlock + tid];
  }
};

// sync_inputs for the flat kernel's LDS rows: the three rows a step may need (local h - delay,
// confirmed h, last added) are read unconditionally, with indices clamped into the stage (every
// index the reference reads lies in it: h >= f - D >= lo + delay), and the choices are selects --
// no exec-mask branches around LDS reads in a wave whose lanes sit at different frames.
template <int P>
__device__ inline uint32_t sync_inputs_flat(const P2PParams& p, RemoteQueues<P>& q, int32_t h, int32_t last_added,
                                            const LdsRowsFlat<P>& rows, uint32_t local_mask) {
  const uint32_t local_row = rows(max(h - p.delay, rows.lo));
  const uint32_t h_row = rows(h);
  const uint32_t last_row = rows(max(last_added, rows.lo));
  const bool confirmed = last_added != kNull && h <= last_added;
  const bool prev = !(h == 0 || last_added == kNull);
  uint32_t in = 0;
#pragma unroll
  for (int k = 0; k < P; k++) {
    uint32_t v;
    if ((local_mask >> k) & 1u) {
      v = h >= p.delay ? (local_row >> (8 * k)) & 0xffu : 0u;
    } else {
      q.last_req[k] = h;
      const bool predicting = q.pred_frame[k] >= 0;
      const bool take_confirmed = !predicting && confirmed;
      const bool start = !predicting && !confirmed;  // a new prediction from the last added input
      const uint32_t start_in = prev ? (p.predictor == 0 ? (last_row >> (8 * k)) & 0xffu : 0u) : 0u;
      q.pred_in[k] = start ? start_in : q.pred_in[k];
      q.pred_frame[k] = start ? (prev ? last_added : kNull) + 1 : q.pred_frame[k];
      v = take_confirmed ? (h_row >> (8 * k)) & 0xffu : q.pred_in[k];
    }
    in |= v << (8 * k);
  }
  return in;
}

// kLocal >= 0: the local-player mask as a compile-time constant (the two-player configurations),
// so the per-player local/remote tests of the poll and of synchronized_inputs fold away.
// kPlain: no desync history, display-checksum trace or debug flip in this launch (host-checked),
// so none of their tests sits in the step loop.
// kSparse: sparse saving (p2p_session.rs:666-702,819-843), as p2p_kernel does it: a rollback
// loads the last save and saves only min_confirmed while replaying; before the call's own step,
// check_last_saved_state either saves the current frame or replays again from the last save.
// kLds: the block's 64 session rings live in LDS for the launch (dynamic shared memory,
// [R][pieces][64 lanes] uint4: a save is three conflict-free ds_write_b128, a rollback's load three
// ds_read_b128); they are copied in from the HBM ring at the start and back at the end, so the HBM
// ring is exact between launches.  A ring cell is only ever read by its own session's thread, so
// the launch needs no other exchange.  Saves no longer go to HBM as partial lines (the PMC traffic
// of the HBM-ring form was 1.7x its algorithmic bytes, nearly all WRITE_SIZE), and the rollback
// cell needs no prefetch.  Used when R x cell fits 28 KB per block (four blocks per CU).
template <int P, int kLocal, bool kPlain, bool kSparse, bool kLds>
__global__ __launch_bounds__(kFlatBlock) void p2p_flat_kernel(P2PParams p) {
  const uint32_t lmask = kLocal >= 0 ? (uint32_t)kLocal : p.local_mask;
  constexpr int Pp = P <= 1 ? 1 : (P == 2 ? 2 : 4);
  constexpr int kRows = kLds ? flat_rows_lds<P>() : kFlatRows;
  constexpr int PC = cell_dwords(P) / 4;  // 16-byte pieces per cell
  __shared__ __attribute__((aligned(16))) uint8_t lds_rows[kRows * kFlatBlock * Pp];
  extern __shared__ uint4 lds_ring[];  // kLds: [R][PC][kFlatBlock]
  const int64_t sess0 = (int64_t)blockIdx.x * kFlatBlock;
  const int64_t S = p.S;
  const bool live = sess0 + threadIdx.x < S;
  const int64_t sess = live ? sess0 + threadIdx.x : sess0;  // idle threads shadow the block's first
  const int nb = (int)((S - sess0) < kFlatBlock ? (S - sess0) : kFlatBlock);
  BoxState<P> st;
  load_state<P>(st, p.cur + sess, S);
  RemoteQueues<P> q;
#pragma unroll
  for (int k = 0; k < P; k++) {
    q.pred_frame[k] = p.queue[(0 * P + k) * S + sess];
    q.pred_in[k] = (uint32_t)p.queue[(1 * P + k) * S + sess];
    q.first_inc[k] = p.queue[(2 * P + k) * S + sess];
    q.last_req[k] = p.queue[(3 * P + k) * S + sess];
  }
  int32_t rollbacks = 0;
  int64_t resim = 0;
  const bool dbg = !kPlain && live && sess == p.dbg_sess;
  const int tid = live ? (int)threadIdx.x : 0;
  const int32_t back = (kSparse ? p.R - 1 : p.D) + p.delay;
  // ring slots kept as counters (no integer division per step): slot_f = f % R of the session's
  // call, slot_h = h % R of its replayed frame, pre_slot of the prefetched cell, saved_slot of the
  // last save (sparse)
  uint4* const my_ring = reinterpret_cast<uint4*>(p.ring + (int64_t)sess * p.R * cell_dwords(P));
  auto cell = [&](int32_t slot) { return my_ring + slot * (cell_dwords(P) / 4); };
  auto next_slot = [&](int32_t x) { return x + 1 == p.R ? 0 : x + 1; };
  // the ring cell of `slot`: HBM (session-major) or this lane's LDS column (piece stride 64)
  const int lt = threadIdx.x;  // LDS column: idle threads keep their own, unused one
  auto cell_load = [&](BoxState<P>& dst, int32_t slot) {
    if constexpr (kLds) {
      constexpr int F = state_fields(P);
#pragma unroll
      for (int k = 0; k < PC; k++) {
        const uint4 v = lds_ring[(slot * PC + k) * kFlatBlock + lt];
        const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; i++)
          if (4 * k + i < F) dst.w[4 * k + i] = x[i];
      }
    } else {
      load_cell<P>(dst, cell(slot));
    }
  };
  auto cell_store = [&](const BoxState<P>& src, uint32_t ck, int32_t slot) {
    if constexpr (kLds) {
      constexpr int F = state_fields(P);
#pragma unroll
      for (int k = 0; k < PC; k++) {
        uint32_t x[4];
#pragma unroll
        for (int i = 0; i < 4; i++) x[i] = 4 * k + i < F ? src.w[4 * k + i] : (4 * k + i == F ? ck : 0u);
        lds_ring[(slot * PC + k) * kFlatBlock + lt] = make_uint4(x[0], x[1], x[2], x[3]);
      }
    } else {
      store_cell<P>(src, ck, cell(slot));
    }
  };
  auto cell_ck = [&](int32_t slot) -> uint16_t {
    if constexpr (kLds) {
      constexpr int F = state_fields(P);
      const uint4 v = lds_ring[(slot * PC + F / 4) * kFlatBlock + lt];
      const uint32_t x[4] = {v.x, v.y, v.z, v.w};
      return (uint16_t)x[F % 4];
    } else {
      return cell_checksum<P>(p, slot, sess);
    }
  };
  // kLds: the block's rings into LDS (HBM pieces are contiguous per block: coalesced reads)
  const int ring_pieces = p.R * PC;
  if constexpr (kLds) {
    const int n = nb * ring_pieces;
    const uint4* src = reinterpret_cast<const uint4*>(p.ring) + sess0 * ring_pieces;
#pragma unroll 4
    for (int i = lt; i < n; i += kFlatBlock) {
      const int sl = i / ring_pieces, rem = i - sl * ring_pieces;
      lds_ring[rem * kFlatBlock + sl] = src[i];
    }
    __syncthreads();
  }
  int32_t slot_f = p.f0 % p.R, slot_h = 0, pre_slot = 0;
  int32_t last_saved = kSparse ? p.last_saved[sess] : kNull;
  int32_t saved_slot = (kSparse && last_saved >= 0) ? last_saved % p.R : 0;
  auto save = [&](int32_t h, int32_t slot) {  // SaveGameState(h) into its cell
    if (kLds) cell_store(st, fletcher16_state<P>(st), slot);  // idle threads: their own column
    if (live) {
      if (!kLds) cell_store(st, fletcher16_state<P>(st), slot);
      if (kSparse) p.ring_frame[(int64_t)slot * S + sess] = h;  // GameStateCell.frame
    }
    if constexpr (kSparse) {
      last_saved = h;
      saved_slot = slot;
    }
  };
  // the rollback cell of the next call (frame f + 1 - D), read at the end of call f (p2p_kernel);
  // sparse saving loads the last save instead, read where the rollback happens
  BoxState<P> pre;
  int32_t pre_frame = kNull;
  // prefetch(fr, slot): fr = f + 1 - D with 1 <= D < R, so its slot is slot_f + 1 - D mod R
  auto prefetch = [&](int32_t fr, int32_t slot) {
    if (!kSparse && !kLds && fr >= 0) {  // (an LDS cell is read where the rollback happens)
      load_cell<P>(pre, cell(slot));
      pre_frame = fr;
      pre_slot = slot;
    }
  };
  {
    const int32_t s0 = slot_f - p.D;
    prefetch(p.f0 - p.D, s0 < 0 ? s0 + p.R : s0);
  }
  // every state this launch steps descends from cur or from a ring cell, all written by this
  // engine (or zero-initialised) and so inside the lean step's rotation domain; one wave-wide test
  // here instead of one per player per step (a foreign state takes the general step throughout)
  const bool lean_ok = __all(rot_in_domain<P>(st) && (pre_frame == kNull || rot_in_domain<P>(pre)));
  const int32_t f_end = p.f0 + p.n;
  const int32_t calls_per_stage = kRows - back;  // >= 1 (host)
  for (int32_t fs = p.f0; fs < f_end;) {
    const int32_t chunk_end = min(f_end, fs + calls_per_stage);
    const int32_t lo = max(0, fs - back);
    {  // stage rows [lo, chunk_end)
      __syncthreads();
      const int nrows = chunk_end - lo, row_bytes = nb * Pp;
      if (nb == kFlatBlock && ((S * Pp) & 15) == 0) {  // whole 16-byte pieces, every load in flight
        constexpr int kPieces = kFlatBlock * Pp / 16;
#pragma unroll 4
        for (int c = threadIdx.x; c < nrows * kPieces; c += kFlatBlock) {
          const int r = c / kPieces, k = c - r * kPieces;
          const uint4* src = reinterpret_cast<const uint4*>(p.inputs + ((int64_t)((lo + r) % p.cap) * S + sess0) * Pp);
          reinterpret_cast<uint4*>(lds_rows + r * kFlatBlock * Pp)[k] = src[k];
        }
      } else {
        for (int c = threadIdx.x; c < nrows * row_bytes; c += kFlatBlock) {
          const int r = c / row_bytes, b = c - r * row_bytes;
          lds_rows[r * kFlatBlock * Pp + b] = p.inputs[((int64_t)((lo + r) % p.cap) * S + sess0) * Pp + b];
        }
      }
      __syncthreads();
    }
    const LdsRowsFlat<P> rows{lds_rows, lo, tid};
    int32_t f = fs;              // this session's call
    bool at_start = true, replaying = false, window_done = false;
    int32_t h = 0, load = 0, last_added = kNull, confirmed = kNull;
    // adjust_gamestate's load (p2p_session.rs:658-714): the cell of `from` (sparse: the last save)
    auto begin_replay = [&](int32_t from) {
      load = from;
      if (kSparse) {
        slot_h = saved_slot;
        cell_load(st, slot_h);
      } else if (!kLds && load == pre_frame) {
        st = pre;
        slot_h = pre_slot;
      } else {
        // load >= f - max_prediction (the remote input of frame f - D arrives at call f, D <
        // max_prediction), so its slot is slot_f - (f - load) with at most one wrap
        const int32_t sh = slot_f - (f - load);
        slot_h = sh < 0 ? sh + p.R : sh;
        cell_load(st, slot_h);
      }
#pragma unroll
      for (int k = 0; k < P; k++) {  // reset_prediction (input_queue.rs:63-67)
        q.pred_frame[k] = kNull;
        q.first_inc[k] = kNull;
        q.last_req[k] = kNull;
      }
      h = load;
      replaying = true;  // load < f
      rollbacks += 1;
      resim += f - load;
    };
    // sparse: check_last_saved_state (:819-843) before the call's own step
    auto window_check = [&]() {
      window_done = true;
      if (f - last_saved >= p.R - 1) {
        if (confirmed >= f) save(f, slot_f);
        else begin_replay(last_saved);
      }
    };
    while (f < chunk_end) {
      if (at_start) {
        // 0. check_checksum_send_interval (as p2p_kernel)
        if (!kPlain && p.desync_interval > 0 && live) {
          const int32_t fts = f - 1 - p.D;
          if (fts >= p.desync_interval && fts % p.desync_interval == 0)
            p.hist[(int64_t)((fts / p.desync_interval) % kHist) * S + sess] = cell_ck(fts % p.R);
        }
        // 1. poll_remote_clients: the remote input of frame g = f - D (add_input_by_frame)
        const int32_t g = f - p.D;
        last_added = g >= 0 ? g : kNull;
        confirmed = g >= 0 ? g : kNull;  // confirmed_frame (:542-553)
        {  // the row read unconditionally (clamped into the stage), its effects by selects
          const uint32_t row = rows(max(g, lo));
#pragma unroll
          for (int k = 0; k < P; k++) {
            if ((lmask >> k) & 1u) continue;
            const bool act = g >= 0 && q.pred_frame[k] != kNull;
            const uint32_t v = (row >> (8 * k)) & 0xffu;
            q.first_inc[k] = (act && q.first_inc[k] == kNull && q.pred_in[k] != v) ? g : q.first_inc[k];
            const bool stop = q.pred_frame[k] == q.last_req[k] && q.first_inc[k] == kNull;
            q.pred_frame[k] = act ? (stop ? kNull : q.pred_frame[k] + 1) : q.pred_frame[k];
          }
        }
        // 2. the first frame's save
        if (f == 0) save(0, slot_f);
        // 3. check_simulation_consistency: a rollback loads first_incorrect (sparse: the last
        //    save) and replays from it
        int32_t first_inc = kNull;
#pragma unroll
        for (int k = 0; k < P; k++)
          if (q.first_inc[k] != kNull && (first_inc == kNull || q.first_inc[k] < first_inc)) first_inc = q.first_inc[k];
        window_done = false;
        if (first_inc != kNull) begin_replay(kSparse ? last_saved : first_inc);
        if (kSparse && !replaying) window_check();
        at_start = false;
      }
      // one step: a replayed frame h or the call's own frame f (non-sparse: SaveGameState(f)
      // first), then AdvanceFrame with synchronized_inputs
      const int32_t fr = replaying ? h : f;
      const uint32_t in = sync_inputs_flat<P>(p, q, fr, last_added, rows, lmask);
      if (kLds && !kSparse) {
        // every step saves: the one replay step the reference does not save (h == load, the
        // frame just loaded) rewrites the loaded cell with the same state and checksum, so the
        // save needs no branch in a wave whose lanes sit at different frames
        save(fr, replaying ? slot_h : slot_f);
      } else if (replaying ? (kSparse ? h == confirmed : h > load) : !kSparse) {
        save(fr, replaying ? slot_h : slot_f);
      }
      const uint32_t from = st.w[0];
      if (lean_ok) advance_state_lean<P>(st, in);
      else advance_state<P>(st, in, 0u);
      if (dbg && (int32_t)from == p.dbg_frame) st.w[fld_x(P, 0)] ^= 1u;
      if constexpr (kPlain && kLds && !kSparse) {  // the same bookkeeping as selects
        const bool rep = replaying;
        slot_h = rep ? next_slot(slot_h) : slot_h;
        h = rep ? h + 1 : h;
        replaying = rep && h != f;
        slot_f = rep ? slot_f : next_slot(slot_f);
        f = rep ? f : f + 1;
        at_start = !rep;
      } else if (replaying) {
        slot_h = next_slot(slot_h);
        if (++h == f) {
          replaying = false;
          if (kSparse && !window_done) window_check();  // may replay again from the last save
        }
      } else {
        if (!kPlain && p.trace && live) p.trace[(int64_t)(f % p.trace_cap) * S + sess] = fletcher16_state<P>(st);
        const int32_t ps = slot_f + 1 - p.D;
        prefetch(f + 1 - p.D, ps < 0 ? ps + p.R : ps);
        slot_f = next_slot(slot_f);
        ++f;
        at_start = true;
      }
    }
    fs = chunk_end;
  }
  if constexpr (kLds) {  // the rings back to HBM
    __syncthreads();
    const int n = nb * ring_pieces;
    uint4* dst = reinterpret_cast<uint4*>(p.ring) + sess0 * ring_pieces;
    for (int i = lt; i < n; i += kFlatBlock) {
      const int sl = i / ring_pieces, rem = i - sl * ring_pieces;
      dst[i] = lds_ring[rem * kFlatBlock + sl];
    }
  }
  if (!live) return;
  store_state<P>(st, p.cur + sess, S);
#pragma unroll
  for (int k = 0; k < P; k++) {
    p.queue[(0 * P + k) * S + sess] = q.pred_frame[k];
    p.queue[(1 * P + k) * S + sess] = (int32_t)q.pred_in[k];
    p.queue[(2 * P + k) * S + sess] = q.first_inc[k];
    p.queue[(3 * P + k) * S + sess] = q.last_req[k];
  }
  p.rollbacks[sess] += rollbacks;
  p.resim[sess] += resim;
  if (kSparse) p.last_saved[sess] = last_saved;
}

// ------------------------------------------------------------------------------------------
// Canonical flat form (plain launches, full saving, f0 >= D: the default for many sessions).  With
// the remote inputs of frame g arriving exactly at call g + D, the InputQueue state the flat
// kernel carries is a function of the inputs (the chains form's argument, below): before call c
// the prediction made for frame g = c - D is the input of frame g - 1 (repeat-last; 0 for
// PredictDefault), so call c rolls back iff some remote player's input of frame g differs from it
// (add_input_by_frame's first_incorrect, input_queue.rs:190-230 -- always frame g); a rollback
// loads cell g and replays frames g .. c - 1, frame g with the confirmed remote inputs and every
// later frame -- like the call's own -- with the prediction made from frame g (lib.rs:390-406);
// without one every frame keeps that prediction.  So each call is: one LDS row read, one compare,
// then the same Loads, Saves and AdvanceFrames as the reference in the same order, with none of the
// per-player queue bookkeeping (pred_frame / first_incorrect / last_requested updates and selects)
// in the step loop; the queues are written back in their canonical form at the end.  Rings in LDS
// as the kLds flat kernel (every step saves: the first replay step rewrites the loaded cell with its
// own bytes), input rows staged per stage of calls.
template <int P, int kLocal>
__global__ __launch_bounds__(kFlatBlock) void p2p_canon_kernel(P2PParams p) {
  const uint32_t lmask = kLocal >= 0 ? (uint32_t)kLocal : p.local_mask;
  constexpr int Pp = P <= 1 ? 1 : (P == 2 ? 2 : 4);
  constexpr int kRows = flat_rows_lds<P>();
  constexpr int PC = cell_dwords(P) / 4;
  constexpr int F = state_fields(P);
  __shared__ __attribute__((aligned(16))) uint8_t lds_rows[kRows * kFlatBlock * Pp];
  extern __shared__ uint4 lds_ring[];  // [R][PC][kFlatBlock]
  const int64_t sess0 = (int64_t)blockIdx.x * kFlatBlock;
  const int64_t S = p.S;
  const bool live = sess0 + threadIdx.x < S;
  const int64_t sess = live ? sess0 + threadIdx.x : sess0;
  const int nb = (int)((S - sess0) < kFlatBlock ? (S - sess0) : kFlatBlock);
  const int lt = threadIdx.x;
  const int tid = live ? lt : 0;
  // byte masks of the local and remote players' inputs in a packed row
  uint32_t lbytes = 0;
#pragma unroll
  for (int k = 0; k < P; k++) lbytes |= ((lmask >> k) & 1u) ? 0xffu << (8 * k) : 0u;
  const uint32_t rbytes = (P == 4 ? 0xffffffffu : ((1u << (8 * P)) - 1u)) & ~lbytes;
  BoxState<P> st;
  load_state<P>(st, p.cur + sess, S);
  // the prediction in effect before the launch: the remote inputs of frame f0 - 1 - D (canonical
  // queues; PredictDefault predicts 0)
  uint32_t prev_rem = 0;
#pragma unroll
  for (int k = 0; k < P; k++)
    if (!((lmask >> k) & 1u)) prev_rem |= ((uint32_t)p.queue[(1 * P + k) * S + sess] & 0xffu) << (8 * k);
  const int ring_pieces = p.R * PC;
  // Only the cells the launch may read before it Saves them come in: a rollback at call f loads
  // frame f - D, the desync history reads frame f - 1 - D, and every frame >= f0 is saved by its
  // own call first, so the cells of frames f0 - 1 - D .. f0 - 1 (from frame 0; D + 1 < R).  The
  // cells the launch may have written go back: its own frames f0 .. f0 + n - 1 and, because a
  // rollback at call f re-saves frames f - D + 1 .. f - 1 (adjust_gamestate saves every replayed
  // frame but the loaded one, p2p_session.rs:696-706), the frames f0 - D + 1 .. f0 - 1 a rollback
  // in the launch's first D - 1 calls rewrites -- the newest R of frames max(0, f0 - D + 1) ..
  // f0 + n - 1 (every one of them is in LDS: copied in, or saved by the launch).  The other cells
  // stay as they are in HBM.
  const uint4* const gring = reinterpret_cast<const uint4*>(p.ring) + sess0 * ring_pieces;
  {
    const int32_t first_in = max(0, p.f0 - 1 - p.D);
    const int in_pieces = (p.f0 - first_in) * PC;
    const int slot_in = first_in % p.R;
    const int n = nb * in_pieces;
#pragma unroll 4
    for (int i = lt; i < n; i += kFlatBlock) {
      const int sl = i / in_pieces, q = i - sl * in_pieces;
      const int d = q / PC, k = q - d * PC;
      const int slot = slot_in + d >= p.R ? slot_in + d - p.R : slot_in + d;
      const int rem = slot * PC + k;
      lds_ring[rem * kFlatBlock + sl] = gring[sl * ring_pieces + rem];
    }
  }
  __syncthreads();
  auto cell_load = [&](int32_t slot) {
#pragma unroll
    for (int k = 0; k < PC; k++) {
      const uint4 v = lds_ring[(slot * PC + k) * kFlatBlock + lt];
      const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 4; i++)
        if (4 * k + i < F) st.w[4 * k + i] = x[i];
    }
  };
  auto cell_store = [&](int32_t slot) {
    const uint32_t ck = fletcher16_state<P>(st);
#pragma unroll
    for (int k = 0; k < PC; k++) {
      uint32_t x[4];
#pragma unroll
      for (int i = 0; i < 4; i++) x[i] = 4 * k + i < F ? st.w[4 * k + i] : (4 * k + i == F ? ck : 0u);
      lds_ring[(slot * PC + k) * kFlatBlock + lt] = make_uint4(x[0], x[1], x[2], x[3]);
    }
  };
  auto next_slot = [&](int32_t x) { return x + 1 == p.R ? 0 : x + 1; };
  const bool lean_ok = __all(rot_in_domain<P>(st));
  int32_t rollbacks = 0;
  int32_t slot_f = p.f0 % p.R, slot_h = 0;
  const int32_t f_end = p.f0 + p.n;
  const int32_t back = p.D + p.delay;
  const int32_t calls_per_stage = kRows - back;  // >= 1 (host)
  for (int32_t fs = p.f0; fs < f_end;) {
    const int32_t chunk_end = min(f_end, fs + calls_per_stage);
    const int32_t lo = max(0, fs - back);
    {
      __syncthreads();
      const int nrows = chunk_end - lo, row_bytes = nb * Pp;
      if (nb == kFlatBlock && ((S * Pp) & 15) == 0) {
        constexpr int kPieces = kFlatBlock * Pp / 16;
#pragma unroll 4
        for (int c = lt; c < nrows * kPieces; c += kFlatBlock) {
          const int r = c / kPieces, k = c - r * kPieces;
          const uint4* src = reinterpret_cast<const uint4*>(p.inputs + ((int64_t)((lo + r) % p.cap) * S + sess0) * Pp);
          reinterpret_cast<uint4*>(lds_rows + r * kFlatBlock * Pp)[k] = src[k];
        }
      } else {
        for (int c = lt; c < nrows * row_bytes; c += kFlatBlock) {
          const int r = c / row_bytes, b = c - r * row_bytes;
          lds_rows[r * kFlatBlock * Pp + b] = p.inputs[((int64_t)((lo + r) % p.cap) * S + sess0) * Pp + b];
        }
      }
      __syncthreads();
    }
    const LdsRowsFlat<P> rows{lds_rows, lo, tid};
    int32_t f = fs, h = 0, g = 0;
    bool at_start = true, replaying = false;
    uint32_t rem_conf = 0, rem_pred = 0;
    // the next call's remote row, read one call ahead (its LDS latency behind this call's steps)
    uint32_t next_rem = rows(fs - p.D) & rbytes;
    while (f < chunk_end) {
      if (at_start) {
        // check_checksum_send_interval (p2p_session.rs:939-975), before any rollback of this call
        // (as p2p_kernel); a launch-uniform switch
        if (p.desync_interval > 0) {
          const int32_t fts = f - 1 - p.D;
          if (live && fts >= p.desync_interval && fts % p.desync_interval == 0) {
            const int32_t cs = fts % p.R;
            const uint4 v = lds_ring[(cs * PC + F / 4) * kFlatBlock + lt];
            const uint32_t x[4] = {v.x, v.y, v.z, v.w};
            p.hist[(int64_t)((fts / p.desync_interval) % kHist) * S + sess] = (uint16_t)x[F % 4];
          }
        }
        // poll of call f: the remote inputs of frame g = f - D against the prediction made for them
        g = f - p.D;
        rem_conf = next_rem;
        next_rem = rows(min(f + 1, chunk_end - 1) - p.D) & rbytes;
        const bool miss = rem_conf != (p.predictor == 0 ? prev_rem : 0u);
        prev_rem = rem_conf;
        rem_pred = p.predictor == 0 ? rem_conf : 0u;
        if (miss) {  // adjust_gamestate: LoadGameState(g), replay g .. f - 1
          const int32_t sh = slot_f - p.D;
          slot_h = sh < 0 ? sh + p.R : sh;
          cell_load(slot_h);
          h = g;
          replaying = true;
          rollbacks += 1;
        }
        at_start = false;
      }
      const int32_t fr = replaying ? h : f;
      const uint32_t rem = (replaying && h == g) ? rem_conf : rem_pred;
      const uint32_t local = fr >= p.delay ? rows(max(fr - p.delay, rows.lo)) & lbytes : 0u;
      cell_store(replaying ? slot_h : slot_f);  // SaveGameState(fr) (the first replay step: same bytes)
      if (lean_ok) advance_state_lean<P>(st, local | rem);
      else advance_state<P>(st, local | rem, 0u);
      const bool rep = replaying;
      slot_h = rep ? next_slot(slot_h) : slot_h;
      h = rep ? h + 1 : h;
      replaying = rep && h != f;
      slot_f = rep ? slot_f : next_slot(slot_f);
      f = rep ? f : f + 1;
      at_start = !rep;
    }
    fs = chunk_end;
  }
  __syncthreads();
  {
    // frames f_end - saved .. f_end - 1: the launch's own and those its early rollbacks re-saved
    const int32_t first_out = max(max(0, p.f0 - p.D + 1), f_end - p.R);
    const int saved = f_end - first_out;
    const int out_pieces = saved * PC;
    const int slot_out = (f_end - saved) % p.R;
    const int n = nb * out_pieces;
    uint4* const dst = reinterpret_cast<uint4*>(p.ring) + sess0 * ring_pieces;
    for (int i = lt; i < n; i += kFlatBlock) {
      const int sl = i / out_pieces, q = i - sl * out_pieces;
      const int d = q / PC, k = q - d * PC;
      const int slot = slot_out + d >= p.R ? slot_out + d - p.R : slot_out + d;
      const int rem = slot * PC + k;
      dst[sl * ring_pieces + rem] = lds_ring[rem * kFlatBlock + sl];
    }
  }
  if (!live) return;
  store_state<P>(st, p.cur + sess, S);
  const int32_t t_last = f_end - 1;
#pragma unroll
  for (int k = 0; k < P; k++) {
    if ((lmask >> k) & 1u) continue;
    p.queue[(0 * P + k) * S + sess] = t_last - p.D + 1;
    p.queue[(1 * P + k) * S + sess] = (int32_t)(p.predictor == 0 ? (prev_rem >> (8 * k)) & 0xffu : 0u);
    p.queue[(2 * P + k) * S + sess] = kNull;
    p.queue[(3 * P + k) * S + sess] = t_last;
  }
  p.rollbacks[sess] += rollbacks;
  p.resim[sess] += (int64_t)rollbacks * p.D;
}

// ------------------------------------------------------------------------------------------
// Canonical flat form with sparse saving (plain launches, f0 >= D): the canonical kernel's call
// (one row read and compare for the rollback decision, the inputs from the rows by the frame's
// position against g = f - D) with the flat kernel's sparse schedule (p2p_session.rs:658-714,
// 819-843): a rollback loads the LAST SAVE and replays from it -- frames <= g with their confirmed
// remote inputs, later frames with the prediction input[g] (repeat-last) or 0 (PredictDefault) --
// saving only min_confirmed (frame g); check_last_saved_state replays again from the last save
// when the call would leave it max_prediction frames behind (the current frame is never
// confirmed here: g < f).  The whole ring comes in and goes back (a load reaches up to R - 1
// frames back); cell frame tags go to HBM as the flat kernel writes them.
template <int P, int kLocal>
__global__ __launch_bounds__(kFlatBlock) void p2p_canon_sparse_kernel(P2PParams p) {
  const uint32_t lmask = kLocal >= 0 ? (uint32_t)kLocal : p.local_mask;
  constexpr int Pp = P <= 1 ? 1 : (P == 2 ? 2 : 4);
  constexpr int kRows = flat_rows_lds<P>();
  constexpr int PC = cell_dwords(P) / 4;
  constexpr int F = state_fields(P);
  __shared__ __attribute__((aligned(16))) uint8_t lds_rows[kRows * kFlatBlock * Pp];
  extern __shared__ uint4 lds_ring[];  // [R][PC][kFlatBlock]
  const int64_t sess0 = (int64_t)blockIdx.x * kFlatBlock;
  const int64_t S = p.S;
  const bool live = sess0 + threadIdx.x < S;
  const int64_t sess = live ? sess0 + threadIdx.x : sess0;
  const int nb = (int)((S - sess0) < kFlatBlock ? (S - sess0) : kFlatBlock);
  const int lt = threadIdx.x;
  const int tid = live ? lt : 0;
  uint32_t lbytes = 0;
#pragma unroll
  for (int k = 0; k < P; k++) lbytes |= ((lmask >> k) & 1u) ? 0xffu << (8 * k) : 0u;
  const uint32_t rbytes = (P == 4 ? 0xffffffffu : ((1u << (8 * P)) - 1u)) & ~lbytes;
  BoxState<P> st;
  load_state<P>(st, p.cur + sess, S);
  uint32_t prev_rem = 0;
#pragma unroll
  for (int k = 0; k < P; k++)
    if (!((lmask >> k) & 1u)) prev_rem |= ((uint32_t)p.queue[(1 * P + k) * S + sess] & 0xffu) << (8 * k);
  int32_t last_saved = p.last_saved[sess];
  int32_t saved_slot = last_saved >= 0 ? last_saved % p.R : 0;
  const int ring_pieces = p.R * PC;
  {
    const int n = nb * ring_pieces;
    const uint4* src = reinterpret_cast<const uint4*>(p.ring) + sess0 * ring_pieces;
#pragma unroll 4
    for (int i = lt; i < n; i += kFlatBlock) {
      const int sl = i / ring_pieces, rem = i - sl * ring_pieces;
      lds_ring[rem * kFlatBlock + sl] = src[i];
    }
  }
  __syncthreads();
  auto cell_load = [&](int32_t slot) {
#pragma unroll
    for (int k = 0; k < PC; k++) {
      const uint4 v = lds_ring[(slot * PC + k) * kFlatBlock + lt];
      const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 4; i++)
        if (4 * k + i < F) st.w[4 * k + i] = x[i];
    }
  };
  auto save = [&](int32_t h, int32_t slot) {  // SaveGameState(h): the cell and its frame tag
    const uint32_t ck = fletcher16_state<P>(st);
#pragma unroll
    for (int k = 0; k < PC; k++) {
      uint32_t x[4];
#pragma unroll
      for (int i = 0; i < 4; i++) x[i] = 4 * k + i < F ? st.w[4 * k + i] : (4 * k + i == F ? ck : 0u);
      lds_ring[(slot * PC + k) * kFlatBlock + lt] = make_uint4(x[0], x[1], x[2], x[3]);
    }
    if (live) p.ring_frame[(int64_t)slot * S + sess] = h;
    last_saved = h;
    saved_slot = slot;
  };
  auto next_slot = [&](int32_t x) { return x + 1 == p.R ? 0 : x + 1; };
  const bool lean_ok = __all(rot_in_domain<P>(st));
  int32_t rollbacks = 0;
  int64_t resim = 0;
  int32_t slot_f = p.f0 % p.R, slot_h = 0;
  const int32_t f_end = p.f0 + p.n;
  const int32_t back = p.R - 1 + p.delay;       // a replay reaches back to the last save
  const int32_t calls_per_stage = kRows - back;  // >= 1 (host)
  for (int32_t fs = p.f0; fs < f_end;) {
    const int32_t chunk_end = min(f_end, fs + calls_per_stage);
    const int32_t lo = max(0, fs - back);
    {
      __syncthreads();
      const int nrows = chunk_end - lo, row_bytes = nb * Pp;
      if (nb == kFlatBlock && ((S * Pp) & 15) == 0) {
        constexpr int kPieces = kFlatBlock * Pp / 16;
#pragma unroll 4
        for (int c = lt; c < nrows * kPieces; c += kFlatBlock) {
          const int r = c / kPieces, k = c - r * kPieces;
          const uint4* src = reinterpret_cast<const uint4*>(p.inputs + ((int64_t)((lo + r) % p.cap) * S + sess0) * Pp);
          reinterpret_cast<uint4*>(lds_rows + r * kFlatBlock * Pp)[k] = src[k];
        }
      } else {
        for (int c = lt; c < nrows * row_bytes; c += kFlatBlock) {
          const int r = c / row_bytes, b = c - r * row_bytes;
          lds_rows[r * kFlatBlock * Pp + b] = p.inputs[((int64_t)((lo + r) % p.cap) * S + sess0) * Pp + b];
        }
      }
      __syncthreads();
    }
    const LdsRowsFlat<P> rows{lds_rows, lo, tid};
    int32_t f = fs, h = 0, g = 0;
    bool at_start = true, replaying = false, window_done = false;
    uint32_t rem_pred = 0;
    // adjust_gamestate from the last save (sparse: frame_to_load = last_saved_frame)
    auto begin_replay = [&]() {
      slot_h = saved_slot;
      cell_load(slot_h);
      h = last_saved;
      replaying = true;
      rollbacks += 1;
      resim += f - last_saved;
    };
    // check_last_saved_state: the current frame f is unconfirmed (g < f), so a save that would
    // leave the window means a replay from it
    auto window_check = [&]() {
      window_done = true;
      if (f - last_saved >= p.R - 1) begin_replay();
    };
    while (f < chunk_end) {
      if (at_start) {
        if (p.desync_interval > 0) {  // check_checksum_send_interval (as the canonical kernel)
          const int32_t fts = f - 1 - p.D;
          if (live && fts >= p.desync_interval && fts % p.desync_interval == 0) {
            const int32_t cs = fts % p.R;
            const uint4 v = lds_ring[(cs * PC + F / 4) * kFlatBlock + lt];
            const uint32_t x[4] = {v.x, v.y, v.z, v.w};
            p.hist[(int64_t)((fts / p.desync_interval) % kHist) * S + sess] = (uint16_t)x[F % 4];
          }
        }
        g = f - p.D;
        const uint32_t rem_conf = rows(g) & rbytes;
        const bool miss = rem_conf != (p.predictor == 0 ? prev_rem : 0u);
        prev_rem = rem_conf;
        rem_pred = p.predictor == 0 ? rem_conf : 0u;
        window_done = false;
        if (miss) begin_replay();
        if (!replaying) window_check();
        at_start = false;
      }
      const int32_t fr = replaying ? h : f;
      // frames <= g: the confirmed remote inputs; later ones: the prediction made from frame g
      const uint32_t rem = fr <= g ? rows(max(fr, rows.lo)) & rbytes : rem_pred;
      const uint32_t local = fr >= p.delay ? rows(max(fr - p.delay, rows.lo)) & lbytes : 0u;
      if (replaying && h == g) save(h, slot_h);  // sparse: only min_confirmed, while replaying
      if (lean_ok) advance_state_lean<P>(st, local | rem);
      else advance_state<P>(st, local | rem, 0u);
      if (replaying) {
        slot_h = next_slot(slot_h);
        if (++h == f) {
          replaying = false;
          if (!window_done) window_check();  // may replay again from the last save
        }
      } else {
        slot_f = next_slot(slot_f);
        ++f;
        at_start = true;
      }
    }
    fs = chunk_end;
  }
  __syncthreads();
  {
    const int n = nb * ring_pieces;
    uint4* dst = reinterpret_cast<uint4*>(p.ring) + sess0 * ring_pieces;
    for (int i = lt; i < n; i += kFlatBlock) {
      const int sl = i / ring_pieces, rem = i - sl * ring_pieces;
      dst[i] = lds_ring[rem * kFlatBlock + sl];
    }
  }
  if (!live) return;
  store_state<P>(st, p.cur + sess, S);
  const int32_t t_last = f_end - 1;
#pragma unroll
  for (int k = 0; k < P; k++) {
    if ((lmask >> k) & 1u) continue;
    p.queue[(0 * P + k) * S + sess] = t_last - p.D + 1;
    p.queue[(1 * P + k) * S + sess] = (int32_t)(p.predictor == 0 ? (prev_rem >> (8 * k)) & 0xffu : 0u);
    p.queue[(2 * P + k) * S + sess] = kNull;
    p.queue[(3 * P + k) * S + sess] = t_last;
  }
  p.rollbacks[sess] += rollbacks;
  p.resim[sess] += resim;
  p.last_saved[sess] = last_saved;
}

// ------------------------------------------------------------------------------------------
// Chains form (few sessions: the flat kernel runs one thread per session, so 4096 sessions fill 64
// of the chip's 1024 SIMDs).  With the remote inputs of frame g arriving exactly at call g + D,
// the state a call works on is a function of the inputs alone: after call c every remote player's
// input of frame h is the real one for h <= g = c - D and the prediction made from frame g after
// it (repeat-last: input[g]; PredictDefault: 0; lib.rs:390-406) -- a misprediction rolls back to
// g and replays with exactly those inputs (adjust_gamestate, p2p_session.rs:658-714), and without
// one every confirmation matched the prediction, so the frames already simulated used them too.
// So call c = LoadGameState(g) of the confirmed state T_g (cell g holds it from call c - 1 on),
// then D + 1 advances: frame g with the real remote inputs, frames g + 1 .. c with the prediction
// input[g] -- whether or not the reference rolls back at c -- exactly the chain of a SyncTest call
// with check_distance D, except that the predicted remote inputs differ per chain.  The kernel runs
// it as the v4 SyncTest pipeline: per session K = D + 1 chain roles x Pp player lanes; at step t
// role j holds chain t - j at frame t - D and advances it with the local input of frame t - D and
// the remote input of frame t - D - j (role 0: the confirmed input of frame t - D; roles j >= 1:
// the prediction of chain t - j, repeat-last input[t - j - D]); then the chains move one role up
// and role 0 keeps its own: T_{t-D+1}, which chain t + 1 loads at step t + 1.
// Ring: after call c the cell of every frame h in (g, c] holds chain c's state at h (a cell
// re-saved by a rollback gets chain c's state; one not re-saved already held the same bytes, for
// the reason above), and the cells of frames <= g hold the confirmed states.  So frame t - D + 1
// is stored once, at step t, by the newest chain of the launch that holds it (role 0 inside the
// launch, role t - (f0 + n - 1) in its tail), with its Fletcher-16 -- the cell the reference ends
// the launch with.  Rollbacks (a remote input of frame t - D unlike the prediction made for it,
// counted by role 0) and resimulated frames (D per rollback) are the reference's; the queue's
// prediction state is written in its canonical form at the end.  Preconditions (host): plain
// launches (no desync detection, trace or debug flip, never sparse saving), f0 >= D (the first D
// calls run on the flat kernel), K * Pp <= 64.
constexpr uint32_t kChainOob = 0x40000000u;  // past every descriptor's range: a lane that never stores
constexpr int kChainLdsRows = 16 * 1024;      // bytes of staged input rows per block

//   kB (2 <= D <= 8): roles 0 .. D - 1 only, as the v5 SyncTest kernel does: role D -- each chain's
// last AdvanceFrame, the call's own frame, whose state no other role consumes -- leaves the
// lockstep; role D - 1's post-advance state is stashed in LDS every step and every D steps one
// batch sub-step advances the D stashed states (role lane j takes step j's).  D x Pp lanes per
// session instead of (D + 1) x Pp (config 2's P2P shape, D = 8 and two players: four sessions
// per wave instead of three), one extra step's work per D steps.
constexpr int kStashEntry = 32;  // bytes per (session, player) entry of a stash slot: 5 fields

//   kD = 8 at two players (config 2's P2P shape; the host picks it when remote_latency is 8): D
// is a compile-time constant and a session's 16 lanes are one DPP row, so the lean steps run as
// the v5 SyncTest kernel's do -- the rotation one row_shr:2 move per field (no LDS round trip),
// every input byte decoded once per launch into an InputRec in LDS, and each step's sin/cos
// computed one step ahead, inside the previous step, from the rotated rot.  Same operations on
// the same values as the general step: the same bits.
constexpr int kChainFastLds = 40 * 1024;  // the kD form's LDS budget per block (four blocks per CU)

template <int P, bool kB, int kD = 0>
__global__ __launch_bounds__(kWave) void p2p_chains_kernel(P2PParams p, int32_t spw) {
  constexpr int Pp = P <= 1 ? 1 : (P == 2 ? 2 : 4);
  constexpr int F = state_fields(P);
  constexpr int C = cell_dwords(P);
  constexpr int n_bytes = Fletcher<P>::n;
  constexpr bool kFast = kB && kD == 8 && Pp == 2;
  static_assert(kD == 0 || kFast, "the compile-time latency form is the D = 8, two-player one");
  // [rows][spw * Pp]: input rows lo .. f0 + n - 1; kB: then (D + 1) stash slots (the last the
  // dump every lane other than role D - 1 writes) of kWave entries; kFast: then the rows' InputRecs
  // and one more, the record of input 0 (PredictDefault's prediction)
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_rows[];
  const int D = kD ? kD : p.D, G = (kB ? D : D + 1) * Pp;
  const int wl = threadIdx.x;
  const int g = wl / G, r = wl - g * G;
  const int j = r / Pp, pl = r - j * Pp;  // static role, player lane
  const int64_t S = p.S;
  const int64_t s0 = xcd_block(blockIdx.x, gridDim.x) * spw;
  const int nsess = (int)((S - s0) < spw ? (S - s0) : spw);
  const bool valid = g < nsess;
  const bool owner = valid && pl < P;
  const int64_t s = valid ? s0 + g : s0;
  const int plc = pl < P ? pl : 0;
  const bool local = ((p.local_mask >> plc) & 1u) != 0;
  const int kq[5] = {fld_x(P, plc), fld_y(P, plc), fld_vx(P, plc), fld_vy(P, plc), fld_rot(P, plc)};
  const int row_bytes = spw * Pp;
  // rows lo .. f0 + n - 1: role D reads frame t - 2D, the local players user input t - D - delay
  const int32_t lo = p.f0 - 2 * D - p.delay;
  const int32_t nrows = p.f0 + p.n - lo;
  // (issued before the row staging: their memory latency behind its loads)
  // every role starts from T_{f0-D}, the cell chain f0 loads (roles > 0 hold chains of the previous
  // launch: stepped, never stored)
  uint32_t w[5];
  {
    const uint32_t* cell = p.ring + ((int64_t)s * p.R + (p.f0 - D) % p.R) * C;
#pragma unroll
    for (int q = 0; q < 5; q++) w[q] = cell[kq[q]];
  }
  // the remote players' prediction before the launch (the input of frame f0 - 1 - D, or 0)
  uint32_t prev_in = (uint32_t)p.queue[(1 * P + plc) * S + s];
  {
    // eight loads in flight per thread before their LDS stores (one memory latency per 512 bytes)
    constexpr int kBatch = 8;
    const int used = nsess * Pp, total = nrows * row_bytes;
    for (int i0 = 0; i0 < total; i0 += kBatch * kWave) {
      uint8_t v[kBatch];
#pragma unroll
      for (int u = 0; u < kBatch; u++) {
        const int i = i0 + u * kWave + wl;
        const int rr = i / row_bytes, b = i - rr * row_bytes;
        const int32_t row = lo + rr;
        v[u] = (i < total && row >= 0 && b < used) ? p.inputs[((int64_t)(row % p.cap) * S + s0) * Pp + b] : (uint8_t)0;
      }
#pragma unroll
      for (int u = 0; u < kBatch; u++) {
        const int i = i0 + u * kWave + wl;
        if (i < total) lds_rows[i] = v[u];
      }
    }
  }
  __syncthreads();
  const int n_entries = nrows * row_bytes;
  // kFast layout after the rows: the stash as D slots of spw x Pp entries, then D dump slots (the
  // lanes other than role D - 1 all write one dump entry of the step's dump slot, so every step's
  // stash store has the same static offset as its slot), then the decoded input records
  const uint32_t fslot = (uint32_t)(row_bytes * kStashEntry);
  uint8_t* const fstash = lds_rows + ((n_entries + 15) & ~15);
  uint4* const lds_rec = reinterpret_cast<uint4*>(fstash + 2 * D * fslot);
  if constexpr (kFast) {
    for (int i = wl; i <= n_entries; i += kWave) {
      const InputRec r = make_input_rec(i < n_entries ? lds_rows[i] : 0u);
      lds_rec[i] = make_uint4(r.delta, r.thr, r.sgn, r.keep);
    }
    __syncthreads();
  }
  const bool lean_ok = __all(w[4] <= kTwoPiBits);
  // the input a lane's chain reads at step t: row t - back
  const int32_t back = local ? D + p.delay : D + j;
  const bool zero_in = !local && j >= 1 && p.predictor != 0;  // PredictDefault's prediction
  const int in_col = valid ? g * Pp + (pl < P ? pl : 0) : 0;  // (lanes past the wave's sessions: column 0)
  // store offsets: a lane's fields of its session's cell (session-major ring, slot offset in soffset)
  const uint32_t cell_base = (uint32_t)((uint64_t)s * p.R * C * 4);
  uint32_t fo[5];
#pragma unroll
  for (int q = 0; q < 5; q++) fo[q] = owner ? cell_base + (uint32_t)kq[q] * 4 : kChainOob;
  const bool lead = valid && pl == 0;  // the session's frame field, checksum and padding
  const uint32_t fo_frame = lead ? cell_base : kChainOob;
  const uint32_t fo_ck = lead ? cell_base + F * 4 : kChainOob;
  const __amdgpu_buffer_rsrc_t rs_ring =
      __builtin_amdgcn_make_buffer_rsrc(p.ring, (short)0, (int)((uint64_t)S * p.R * C * 4), 0x00020000);
  uint32_t wt[5];
#pragma unroll
  for (int q = 0; q < 5; q++) wt[q] = owner ? 2u * weights_at(n_bytes, fld_offset(P, kq[q])) : 0u;
  const uint32_t one2 = owner ? 0x02020202u : 0u;
  const uint32_t wf1 = pl == 0 ? 0x02020202u : 0u, wf2 = pl == 0 ? 2u * weights_at(n_bytes, 0) : 0u;
  const uint32_t c1 = pl == 0 ? 2u * Fletcher<P>::kSum1Const : 0u;
  const uint32_t c2 = pl == 0 ? 2u * Fletcher<P>::kSum2Const : 0u;
  const int src_rot = (j == 0 ? wl : g * G + (j - 1) * Pp + pl) * 4;
  const bool counts = valid && j == 0 && pl < P && !local;  // role 0's remote lanes see each arrival
  // kB stash: slot of step t = (t - f0) mod D; lane entry g * Pp + pl
  uint8_t* const stash = lds_rows + (((nrows * row_bytes) + 15) & ~15);
  const uint32_t entry = (uint32_t)(g * Pp + pl) * kStashEntry;
  const uint32_t stash_w = (valid && j == D - 1) ? entry : (uint32_t)(D * kWave * kStashEntry) + (uint32_t)wl * kStashEntry;
  // batch: role lane j advances slot j's chain c = tb + j - (D - 1) at its own frame c, with the
  // local input of frame c and the remote prediction of chain c (the input of frame c - D)
  const int32_t back_b = local ? p.delay : D;
  const bool zero_b = !local && p.predictor != 0;
  const uint32_t pmask = (1u << Pp) - 1u;
  const int gbase = g * G;
  int32_t rollbacks = 0;
  const int32_t t_last = p.f0 + p.n - 1;  // the launch's last call
  const int32_t t_end = t_last + D + (kB ? 0 : 1);  // kB: role D's last advance is the batch's
  int32_t slot = __builtin_amdgcn_readfirstlane((p.f0 - D + 1) % p.R);  // slot of frame t - D + 1
  const uint32_t ck_pad = fo_ck + 4;  // (P = 4: the cell's padding dwords after the checksum)
  // One step t.  kCore: a call of the launch (t <= t_last): its poll, and role 0 -- the newest chain
  // -- stores frame t - D + 1; the tail steps' storing role is t - t_last.  kLean: the states are in
  // the lean step's rotation domain (every role starts from the loaded cell, which this engine wrote).
  auto step = [&](int32_t t, auto core_tag, auto lean_tag) {
    constexpr bool kCore = decltype(core_tag)::value;
    constexpr bool kLean = decltype(lean_tag)::value;
    const int32_t row = t - back;
    const uint32_t in = (row >= 0 && !zero_in) ? (uint32_t)lds_rows[(row - lo) * row_bytes + in_col] : 0u;
    if constexpr (kCore) {
      // poll of call t: the arriving input of frame t - D against the prediction made for it
      // (add_input_by_frame, input_queue.rs:190-230); any remote player's miss rolls the session back
      const bool miss = counts && in != (p.predictor == 0 ? prev_in : 0u);
      const uint64_t mb = __ballot(miss);
      if (j == 0 && pl == 0 && valid && ((uint32_t)(mb >> gbase) & pmask)) rollbacks += 1;
      prev_in = in;
    }
    // AdvanceFrame(t - D) of chain t - j
    {
      float x = __builtin_bit_cast(float, w[0]), y = __builtin_bit_cast(float, w[1]);
      float vx = __builtin_bit_cast(float, w[2]), vy = __builtin_bit_cast(float, w[3]);
      float rot = __builtin_bit_cast(float, w[4]);
      if constexpr (kLean) advance_player_lean(x, y, vx, vy, rot, in);
      else advance_player(x, y, vx, vy, rot, in);
      w[0] = __builtin_bit_cast(uint32_t, x);
      w[1] = __builtin_bit_cast(uint32_t, y);
      w[2] = __builtin_bit_cast(uint32_t, vx);
      w[3] = __builtin_bit_cast(uint32_t, vy);
      w[4] = __builtin_bit_cast(uint32_t, rot);
    }
    uint32_t nx[5];
#pragma unroll
    for (int q = 0; q < 5; q++) nx[q] = (uint32_t)__builtin_amdgcn_ds_bpermute(src_rot, (int)w[q]);
    if constexpr (kB) {  // role D - 1's post-advance state (its chain's own frame) for the batch
      uint8_t* st = stash + (uint32_t)((t - p.f0) % D) * (uint32_t)(kWave * kStashEntry) + stash_w;
      if (stash_w >= (uint32_t)(D * kWave * kStashEntry)) st = stash + stash_w;  // the dump slot
      *reinterpret_cast<uint4*>(st) = make_uint4(w[0], w[1], w[2], w[3]);
      *reinterpret_cast<uint32_t*>(st + 16) = w[4];
    }
    __builtin_amdgcn_sched_barrier(0);  // the rotation's LDS latency behind the checksum and stores
    const uint32_t frame1 = (uint32_t)(t - D + 1);
    const int js = kCore ? 0 : t - t_last;  // the newest chain of the launch holding frame1
    if (kCore || js < D) {
      uint32_t d1 = dot4_u8(frame1, wf1, c1), d2 = dot4_u8(frame1, wf2, c2);
#pragma unroll
      for (int q = 0; q < 5; q++) {
        d1 = dot4_u8(w[q], one2, d1);
        d2 = dot4_u8(w[q], wt[q], d2);
      }
      if constexpr (Pp >= 2) {
        d1 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d1, 0xB1, 0xF, 0xF, true);  // xor 1
        d2 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d2, 0xB1, 0xF, 0xF, true);
      }
      if constexpr (Pp >= 4) {
        d1 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d1, 0x4E, 0xF, 0xF, true);  // xor 2
        d2 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d2, 0x4E, 0xF, 0xF, true);
      }
      const uint32_t ck = fletcher_from_doubled(d1, d2);
      const bool me = kCore ? j == 0 : j == js;
      const uint32_t so = (uint32_t)slot * (uint32_t)(C * 4);
#pragma unroll
      for (int q = 0; q < 5; q++) __builtin_amdgcn_raw_buffer_store_b32(w[q], rs_ring, me ? fo[q] : kChainOob, so, 0);
      __builtin_amdgcn_raw_buffer_store_b32(frame1, rs_ring, me ? fo_frame : kChainOob, so, 0);
      __builtin_amdgcn_raw_buffer_store_b32(ck, rs_ring, me ? fo_ck : kChainOob, so, 0);
#pragma unroll
      for (int k = F + 1; k < C; k++)
        __builtin_amdgcn_raw_buffer_store_b32(0u, rs_ring, me && lead ? ck_pad + (k - F - 1) * 4 : kChainOob, so, 0);
    } else if (!kB && t == t_end - 1 && j == D) {
      // role D: chain f0 + n - 1 after its call's own AdvanceFrame -- the current state
      if (owner) {
#pragma unroll
        for (int q = 0; q < 5; q++) p.cur[(int64_t)kq[q] * S + s] = w[q];
      }
      if (lead) p.cur[s] = frame1;
    }
#pragma unroll
    for (int q = 0; q < 5; q++) w[q] = nx[q];
    slot = slot + 1 == p.R ? 0 : slot + 1;
  };
  // kB: the batch over the stashes of steps tb .. tb + count - 1 (role D's AdvanceFrames)
  auto batch = [&](int32_t tb, int count, auto lean_tag) {
    constexpr bool kLean = decltype(lean_tag)::value;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int32_t c = tb + j - (D - 1);
    const bool act = valid && j < count;
    const uint8_t* st = stash + (uint32_t)((tb - p.f0 + j) % D) * (uint32_t)(kWave * kStashEntry) + entry;
    const uint4 a = *reinterpret_cast<const uint4*>(st);
    uint32_t v[5] = {a.x, a.y, a.z, a.w, *reinterpret_cast<const uint32_t*>(st + 16)};
    const int32_t row = c - back_b;
    const uint32_t in = (row >= lo && !zero_b && j < count) ? (uint32_t)lds_rows[(row - lo) * row_bytes + in_col] : 0u;
    float x = __builtin_bit_cast(float, v[0]), y = __builtin_bit_cast(float, v[1]);
    float vx = __builtin_bit_cast(float, v[2]), vy = __builtin_bit_cast(float, v[3]);
    float rot = __builtin_bit_cast(float, v[4]);
    if constexpr (kLean) advance_player_lean(x, y, vx, vy, rot, in);
    else advance_player(x, y, vx, vy, rot, in);
    if (act && c == t_last) {  // the launch's last call: the current state
      v[0] = __builtin_bit_cast(uint32_t, x);
      v[1] = __builtin_bit_cast(uint32_t, y);
      v[2] = __builtin_bit_cast(uint32_t, vx);
      v[3] = __builtin_bit_cast(uint32_t, vy);
      v[4] = __builtin_bit_cast(uint32_t, rot);
      if (owner) {
#pragma unroll
        for (int q = 0; q < 5; q++) p.cur[(int64_t)kq[q] * S + s] = v[q];
      }
      if (lead) p.cur[s] = (uint32_t)(c + 1);
    }
  };
  auto run = [&](auto lean_tag) {
    int32_t t = p.f0;
    for (; t <= t_last; ++t) {
      step(t, std::true_type(), lean_tag);
      if (kB && (t - p.f0) % D == D - 1) batch(t - (D - 1), D, lean_tag);
    }
    for (; t < t_end; ++t) {
      step(t, std::false_type(), lean_tag);
      if (kB && ((t - p.f0) % D == D - 1 || t == t_end - 1)) {
        const int count = (t - p.f0) % D + 1;
        batch(t - (count - 1), count, lean_tag);
      }
    }
  };
  // kFast: the lean steps as the v5 SyncTest kernel runs them (see above the kernel)
  auto run_fast = [&] {
    // a lane's input record and raw byte of call f0 + rel sit at base + rel x stride (PredictDefault
    // roles: the record of input 0, stride 0)
    const uint32_t zero_idx = (uint32_t)n_entries;
    const int32_t row0 = p.f0 - back - lo;  // the lane's row of call f0
    const uint32_t rec_base = (zero_in ? zero_idx : (uint32_t)(row0 * row_bytes + in_col)) * 16u;
    const uint32_t rec_stride = zero_in ? 0u : (uint32_t)row_bytes * 16u;
    const uint32_t raw_base = (uint32_t)(row0 * row_bytes + in_col);
    const uint8_t* const rec_bytes = reinterpret_cast<const uint8_t*>(lds_rec);
    auto rec_at = [&](int32_t rel) { return *reinterpret_cast<const uint4*>(rec_bytes + rec_base + (uint32_t)rel * rec_stride); };
    auto raw_at = [&](int32_t rel) { return (uint32_t)lds_rows[raw_base + (uint32_t)rel * (uint32_t)row_bytes]; };
    const uint32_t stash_w8 = (valid && j == D - 1) ? entry : (uint32_t)D * fslot;
    float sc_s, sc_c;
    uint32_t sc_qs, sc_qc;
    glibc_sincosf_domain_raw(__builtin_bit_cast(float, w[4]), &sc_s, &sc_c, &sc_qs, &sc_qc);
    auto fstep = [&](int32_t t, auto core_tag, const uint4 rv, uint32_t in, uint32_t slot_off) {
      constexpr bool kCore = decltype(core_tag)::value;
      if constexpr (kCore) {
        // poll of call t, branch-free: a remote lane of role 0 whose arriving input differs from the
        // prediction; either player lane's miss rolls the session back (xor-1 lane = the other player)
        const uint32_t m = (counts && in != (p.predictor == 0 ? prev_in : 0u)) ? 1u : 0u;
        rollbacks += (int32_t)(m | (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0xB1, 0xF, 0xF, true));
        prev_in = in;
      }
      {
        float x = __builtin_bit_cast(float, w[0]), y = __builtin_bit_cast(float, w[1]);
        float vx = __builtin_bit_cast(float, w[2]), vy = __builtin_bit_cast(float, w[3]);
        float rot = __builtin_bit_cast(float, w[4]);
        // the next step's rot is this lane's new rot one role up (role 0 keeps its own)
        advance_player_rec_q(x, y, vx, vy, rot, InputRec{rv.x, rv.y, rv.z, rv.w}, sc_s, sc_c, sc_qs, sc_qc,
                             [&](float rn) {
                               const uint32_t rb = __builtin_bit_cast(uint32_t, rn);
                               const uint32_t nb = (uint32_t)__builtin_amdgcn_update_dpp((int)rb, (int)rb, 0x112, 0xF, 0xF, false);
                               glibc_sincosf_domain_raw(__builtin_bit_cast(float, nb), &sc_s, &sc_c, &sc_qs, &sc_qc);
                             });
        w[0] = __builtin_bit_cast(uint32_t, x);
        w[1] = __builtin_bit_cast(uint32_t, y);
        w[2] = __builtin_bit_cast(uint32_t, vx);
        w[3] = __builtin_bit_cast(uint32_t, vy);
        w[4] = __builtin_bit_cast(uint32_t, rot);
      }
      {  // role D - 1's post-advance state for the batch (every other lane: the dump slot)
        uint8_t* st = fstash + stash_w8 + slot_off;
        *reinterpret_cast<uint4*>(st) = make_uint4(w[0], w[1], w[2], w[3]);
        *reinterpret_cast<uint32_t*>(st + 16) = w[4];
      }
      const uint32_t frame1 = (uint32_t)(t - D + 1);
      const int js = kCore ? 0 : t - t_last;
      if (kCore || js < D) {
        uint32_t d1 = dot4_u8(frame1, wf1, c1), d2 = dot4_u8(frame1, wf2, c2);
#pragma unroll
        for (int q = 0; q < 5; q++) {
          d1 = dot4_u8(w[q], one2, d1);
          d2 = dot4_u8(w[q], wt[q], d2);
        }
        d1 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d1, 0xB1, 0xF, 0xF, true);  // xor 1
        d2 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d2, 0xB1, 0xF, 0xF, true);
        const uint32_t ck = fletcher_from_doubled(d1, d2);
        const bool me = kCore ? j == 0 : j == js;
        const uint32_t so = (uint32_t)slot * (uint32_t)(C * 4);
#pragma unroll
        for (int q = 0; q < 5; q++) __builtin_amdgcn_raw_buffer_store_b32(w[q], rs_ring, me ? fo[q] : kChainOob, so, 0);
        __builtin_amdgcn_raw_buffer_store_b32(frame1, rs_ring, me ? fo_frame : kChainOob, so, 0);
        __builtin_amdgcn_raw_buffer_store_b32(ck, rs_ring, me ? fo_ck : kChainOob, so, 0);
#pragma unroll
        for (int k = F + 1; k < C; k++)
          __builtin_amdgcn_raw_buffer_store_b32(0u, rs_ring, me && lead ? ck_pad + (k - F - 1) * 4 : kChainOob, so, 0);
      }
#pragma unroll
      for (int q = 0; q < 5; q++) w[q] = (uint32_t)__builtin_amdgcn_update_dpp((int)w[q], (int)w[q], 0x112, 0xF, 0xF, false);
      slot = slot + 1 == p.R ? 0 : slot + 1;
    };
    auto fbatch = [&](int32_t tb, int count) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int32_t c = tb + j - (D - 1);
      const bool act = valid && j < count;
      const uint8_t* st = fstash + (uint32_t)((tb - p.f0 + j) & (D - 1)) * fslot + entry;
      const uint4 a = *reinterpret_cast<const uint4*>(st);
      uint32_t v[5] = {a.x, a.y, a.z, a.w, *reinterpret_cast<const uint32_t*>(st + 16)};
      const int32_t row = c - back_b;
      const uint32_t ri = (row >= lo && !zero_b && j < count) ? (uint32_t)((row - lo) * row_bytes + in_col) : zero_idx;
      const uint4 rv = lds_rec[ri];
      float x = __builtin_bit_cast(float, v[0]), y = __builtin_bit_cast(float, v[1]);
      float vx = __builtin_bit_cast(float, v[2]), vy = __builtin_bit_cast(float, v[3]);
      float rot = __builtin_bit_cast(float, v[4]);
      float bs, bc;
      uint32_t bqs, bqc;
      glibc_sincosf_domain_raw(rot, &bs, &bc, &bqs, &bqc);
      advance_player_rec_q(x, y, vx, vy, rot, InputRec{rv.x, rv.y, rv.z, rv.w}, bs, bc, bqs, bqc);
      if (act && c == t_last) {  // the launch's last call: the current state
        v[0] = __builtin_bit_cast(uint32_t, x);
        v[1] = __builtin_bit_cast(uint32_t, y);
        v[2] = __builtin_bit_cast(uint32_t, vx);
        v[3] = __builtin_bit_cast(uint32_t, vy);
        v[4] = __builtin_bit_cast(uint32_t, rot);
        if (owner) {
#pragma unroll
          for (int q = 0; q < 5; q++) p.cur[(int64_t)kq[q] * S + s] = v[q];
        }
        if (lead) p.cur[s] = (uint32_t)(c + 1);
      }
    };
    int32_t t = p.f0;
    // whole blocks of D calls: their input records and bytes read up front, then the batch
    for (; t + D - 1 <= t_last; t += D) {
      const int32_t rel = t - p.f0;
      uint4 in[kD > 0 ? kD : 1];
      uint32_t raw[kD > 0 ? kD : 1];
#pragma unroll
      for (int u = 0; u < kD; u++) {
        in[u] = rec_at(rel + u);
        raw[u] = raw_at(rel + u);
      }
#pragma unroll
      for (int u = 0; u < kD; u++) fstep(t + u, std::true_type(), in[u], raw[u], (uint32_t)u * fslot);
      fbatch(t, D);
    }
    for (; t <= t_last; ++t) {
      const int32_t rel = t - p.f0;
      fstep(t, std::true_type(), rec_at(rel), raw_at(rel), (uint32_t)(rel & (D - 1)) * fslot);
      if ((rel & (D - 1)) == D - 1) fbatch(t - (D - 1), D);
    }
    for (; t < t_end; ++t) {
      const int32_t rel = t - p.f0;
      fstep(t, std::false_type(), rec_at(rel), 0u, (uint32_t)(rel & (D - 1)) * fslot);
      if ((rel & (D - 1)) == D - 1 || t == t_end - 1) {
        const int count = (rel & (D - 1)) + 1;
        fbatch(t - (count - 1), count);
      }
    }
  };
  if (lean_ok) {
    if constexpr (kFast) run_fast();
    else run(std::true_type());
  } else {
    run(std::false_type());
  }
  if (valid && j == 0 && pl == 0) {
    p.rollbacks[s] += rollbacks;
    p.resim[s] += (int64_t)rollbacks * D;
  }
  if (counts) {
    // the remote queue after call f0 + n - 1 (canonical): predicting from frame g + 1 with the
    // input of frame g = f0 + n - 1 - D, no incorrect frame, last request = the call's own frame
    const int32_t gl = t_last - D;
    const uint32_t last_in = (uint32_t)lds_rows[(gl - lo) * row_bytes + in_col];
    p.queue[(0 * P + plc) * S + s] = gl + 1;
    p.queue[(1 * P + plc) * S + s] = (int32_t)(p.predictor == 0 ? last_in : 0u);
    p.queue[(2 * P + plc) * S + s] = kNull;
    p.queue[(3 * P + plc) * S + s] = t_last;
  }
}

// Lockstep mode (max_prediction 0; builder.rs:134-147, p2p_session.rs:301-310,393-407): a call
// never saves, loads or resimulates; it advances only when the current frame's inputs are confirmed
// from every player.  Which calls advance, and which input rows their AdvanceFrame reads, depend
// only on the arrival schedule -- the same for every session of the engine -- so the host replays
// the control flow (poll, confirmed_frame, set_last_confirmed_frame, add_local_input with its
// delay and drops, can_advance) and hands the kernel one (local row, remote row) pair per call:
// remote row -1 = the call does not advance; local row -1 = the default input (queue frames below
// the input delay).  One thread per session applies them.
template <int P>
__global__ __launch_bounds__(256) void p2p_lockstep_kernel(P2PParams p, const int32_t* prog) {
  const int64_t sess = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (sess >= p.S) return;
  const int64_t S = p.S;
  BoxState<P> st;
  load_state<P>(st, p.cur + sess, S);
  uint32_t lbytes = 0;  // the local players' bytes of the packed input word
#pragma unroll
  for (int k = 0; k < P; k++)
    if ((p.local_mask >> k) & 1u) lbytes |= 0xffu << (8 * k);
  for (int32_t k = 0; k < p.n; k++) {
    const int32_t lrow = prog[2 * k], rrow = prog[2 * k + 1];
    if (rrow >= 0) {  // AdvanceFrame with synchronized_inputs (all confirmed)
      const uint32_t local = lrow >= 0 ? load_inputs<P>(p.inputs, (int64_t)(lrow % p.cap) * S + sess) & lbytes : 0u;
      const uint32_t remote = load_inputs<P>(p.inputs, (int64_t)(rrow % p.cap) * S + sess) & ~lbytes;
      advance_state<P>(st, local | remote, 0u);
    }
    // the display checksum of the last AdvanceFrame (ex_game.rs:121-126); 0 before the first
    if (p.trace) p.trace[(int64_t)((p.f0 + k) % p.trace_cap) * S + sess] = st.w[0] > 0 ? fletcher16_state<P>(st) : 0;
  }
  store_state<P>(st, p.cur + sess, S);
}

// compare_local_checksums_against_peers for one report frame, every session at once: bit s of
// mask = local[s] != remote[s] (p2p_session.rs:915-926), count = number of set bits.
__global__ __launch_bounds__(256) void compare_checksums_kernel(const uint16_t* local, const uint16_t* remote, int64_t S,
                                                                 uint64_t* mask, int32_t* count) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool differ = s < S && local[s] != remote[s];
  const uint64_t bits = __ballot(differ);
  if ((threadIdx.x & 63) == 0 && s < S) {
    mask[s >> 6] = bits;
    if (bits) atomicAdd(count, __popcll(bits));
  }
}

// every queue starts empty: prediction.frame, first_incorrect, last_requested = NULL, input 0
__global__ void init_queue_kernel(int32_t* queue, int64_t n_per_field, int32_t P) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 4 * n_per_field) return;
  const int64_t field = i / n_per_field;
  queue[i] = field == 1 ? 0 : kNull;
  (void)P;
}

}  // namespace


namespace {

template <typename K>
int p2p_launch_timed(ggrs_p2p_engine* e, K&& launch) {
  if (int rc = e->timer.before(e->stream)) return rc;
  launch();
  HIP_TRY(hipGetLastError());
  e->timer.count();
  return GGRS_OK;
}

// oldest input row a call at frame f still reads: user input (f - D) - delay of the local
// players' replay, and the remote input f - D; with sparse saving a replay starts at the last
// save, up to max_prediction frames back
int32_t oldest_row(const ggrs_p2p_engine* e, int32_t f) {
  // scheduled arrivals: the local rows of the calls still to run (a remote row is checked against
  // its tag on the device when it arrives)
  if (e->sched) return f;
  if (e->cfg.max_prediction == 0) {  // lockstep: the current frame's remote row, the next local rows
    int32_t oldest = std::min(f, e->ls_frame);
    const int32_t q = std::max(e->ls_frame, e->cfg.input_delay);
    if (e->cfg.local_mask && q <= e->ls_local_last)
      oldest = std::min(oldest, e->ls_row_of[(size_t)q % e->ls_row_of.size()]);
    return std::max(0, oldest);
  }
  const int32_t back = e->sparse ? e->cfg.max_prediction : e->cfg.remote_latency;
  return std::max(0, f - back - e->cfg.input_delay);
}

// Lockstep: replay calls f0 .. f0+n-1 of P2PSession::advance_frame's control flow (the same for
// every session) into prog[n][2]; updates the engine's lockstep state.
void lockstep_program(ggrs_p2p_engine* e, int32_t f0, int32_t n, std::vector<int32_t>& prog) {
  const int32_t D = e->cfg.remote_latency, delay = e->cfg.input_delay;
  const bool has_local = e->cfg.local_mask != 0;
  const size_t Q = e->ls_row_of.size();
  prog.assign(2 * (size_t)n, -1);
  for (int32_t k = 0; k < n; k++) {
    const int32_t f = f0 + k;
    // poll_remote_clients: the remote players' inputs up to frame f - D have arrived
    const int32_t remote_last = f - D >= 0 ? f - D : kNull;
    // confirmed_frame (:542-553) over every player, before this call's local input
    int32_t confirmed = remote_last;
    if (has_local) confirmed = std::min(confirmed, e->ls_local_last);
    // set_last_confirmed_frame (sync_layer.rs:313-340): never ahead of the current frame
    const int32_t last_confirmed = std::min(confirmed, e->ls_frame);
    // add_local_input (:362-377): queue frame current + delay, dropped unless it is the next one
    // (input_queue.rs:170-186; the first add fills the frames below the delay with the default)
    if (has_local) {
      const int32_t qf = e->ls_frame + delay;
      if (e->ls_local_last == kNull || qf == e->ls_local_last + 1) {
        e->ls_row_of[(size_t)qf % Q] = f;
        e->ls_local_last = qf;
      }
    }
    // :393-407: advance only with the current frame confirmed by everyone
    if (last_confirmed == e->ls_frame) {
      const int32_t c = e->ls_frame;
      prog[2 * k] = (has_local && c >= delay) ? e->ls_row_of[(size_t)c % Q] : -1;
      prog[2 * k + 1] = c;
      e->ls_frame += 1;
    }
  }
}

}  // namespace

extern "C" {

int ggrs_p2p_engine_destroy(ggrs_p2p_engine_t* e) {
  if (!e) return GGRS_OK;
  (void)hipSetDevice(e->cfg.device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  p2p_sched_free(e);
  void* bufs[] = {e->cur, e->ring, e->inputs, e->queue, e->rollbacks, e->resim, e->trace, e->staging,
                  e->hist, e->cmp_mask, e->cmp_count, e->last_saved, e->ring_frame, e->ls_prog};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  e->timer.destroy();
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
  return GGRS_OK;
}

int ggrs_p2p_engine_create(const ggrs_p2p_config_t* cfg, ggrs_p2p_engine_t** out) {
  if (!cfg || !out) return set_error(GGRS_E_INVALID, "null argument");
  *out = nullptr;
  ggrs_p2p_config_t c = *cfg;
  if (c.num_sessions < 1) return set_error(GGRS_E_INVALID, "num_sessions must be >= 1");
  if (c.num_players < 1 || c.num_players > 4) return set_error(GGRS_E_INVALID, "num_players must be in 1..4 (ex_game.rs:70)");
  if ((c.local_mask & ~((1 << c.num_players) - 1)) != 0)
    return set_error(GGRS_E_INVALID, "local_mask names a player the session does not have");
  if (c.local_mask == (1 << c.num_players) - 1)
    return set_error(GGRS_E_INVALID, "a P2P session needs at least one remote player");
  if (c.input_delay < 0) return set_error(GGRS_E_INVALID, "input_delay must be >= 0");
  if (c.max_prediction < 0) return set_error(GGRS_E_INVALID, "max_prediction must be >= 0 (0: lockstep mode)");
  if (c.remote_latency < 1 || (c.max_prediction > 0 && c.remote_latency >= c.max_prediction))
    return set_error(GGRS_E_INVALID, "remote_latency must be in 1..max_prediction-1 (else the prediction threshold stalls)");
  if (c.predictor != 0 && c.predictor != 1) return set_error(GGRS_E_INVALID, "predictor must be 0 (repeat last) or 1 (default)");
  if (c.input_capacity == 0) c.input_capacity = 256;
  if (c.input_capacity < c.remote_latency + c.input_delay + 2)
    return set_error(GGRS_E_INVALID, "input_capacity must be >= remote_latency + input_delay + 2");
  if (c.trace_capacity < 0) return set_error(GGRS_E_INVALID, "trace_capacity must be >= 0");
  ggrs_p2p_engine* e = new ggrs_p2p_engine();
  e->cfg = c;
  e->Pp = padded_players(c.num_players);
  e->F = state_fields(c.num_players);
  e->R = c.max_prediction + 1;
  e->cap = c.input_capacity;
  if (c.max_prediction == 0) e->ls_row_of.assign((size_t)std::max(64, c.input_delay + 8), kNull);
  auto fail = [&](int rc) {
    std::string msg = ggrs_last_error();
    ggrs_p2p_engine_destroy(e);
    set_error(rc, "%s", msg.c_str());
    return rc;
  };
#define CTRY(expr)                                                                      \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) return fail(set_error(GGRS_E_HIP, "%s: %s", #expr, hipGetErrorString(e_))); \
  } while (0)
  const int64_t S = c.num_sessions;
  const int P = c.num_players;
  CTRY(hipSetDevice(c.device));
  CTRY(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
  CTRY(hipDeviceGetAttribute(&e->num_cus, hipDeviceAttributeMultiprocessorCount, c.device));
  if (e->num_cus < 1) e->num_cus = 1;
  if (e->timer.create()) return fail(GGRS_E_HIP);
  CTRY(hipMalloc(&e->cur, sizeof(uint32_t) * e->F * S));
  CTRY(hipMalloc(&e->ring, sizeof(uint32_t) * (size_t)e->R * cell_dwords(P) * S));
  CTRY(hipMalloc(&e->inputs, (size_t)e->cap * S * e->Pp));
  CTRY(hipMalloc(&e->queue, sizeof(int32_t) * 4 * P * S));
  CTRY(hipMalloc(&e->rollbacks, sizeof(int32_t) * S));
  CTRY(hipMalloc(&e->resim, sizeof(int64_t) * S));
  if (c.trace_capacity > 0) CTRY(hipMalloc(&e->trace, sizeof(uint16_t) * (size_t)c.trace_capacity * S));
  CTRY(hipMemsetAsync(e->ring, 0, sizeof(uint32_t) * (size_t)e->R * cell_dwords(P) * S, e->stream));
  CTRY(hipMemsetAsync(e->inputs, 0, (size_t)e->cap * S * e->Pp, e->stream));
  CTRY(hipMemsetAsync(e->rollbacks, 0, sizeof(int32_t) * S, e->stream));
  CTRY(hipMemsetAsync(e->resim, 0, sizeof(int64_t) * S, e->stream));
  if (e->trace) CTRY(hipMemsetAsync(e->trace, 0, sizeof(uint16_t) * (size_t)c.trace_capacity * S, e->stream));
  init_queue_kernel<<<grid_of(4 * P * S, 256), 256, 0, e->stream>>>(e->queue, (int64_t)P * S, P);
  dispatch_players(P, [&](auto PC) {
    constexpr int PP = decltype(PC)::value;
    init_states_kernel<PP><<<grid_of(S, 256), 256, 0, e->stream>>>(e->cur, S);
  });
  CTRY(hipGetLastError());
  CTRY(hipStreamSynchronize(e->stream));
#undef CTRY
  *out = e;
  return GGRS_OK;
}

int ggrs_p2p_engine_config(const ggrs_p2p_engine_t* e, ggrs_p2p_config_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  *out = e->cfg;
  return GGRS_OK;
}

int ggrs_p2p_add_inputs(ggrs_p2p_engine_t* e, int32_t first_frame, int32_t n, const uint8_t* inputs) {
  if (!e || (!inputs && n > 0)) return set_error(GGRS_E_INVALID, "null argument");
  if (n < 0) return set_error(GGRS_E_INVALID, "n_frames must be >= 0");
  if (first_frame != e->next_input_frame)
    return set_error(GGRS_E_INVALID, "inputs must be added sequentially (expected frame %d, got %d)",
                     e->next_input_frame, first_frame);
  if (n == 0) return GGRS_OK;
  if ((int64_t)first_frame + n - 1 - oldest_row(e, e->current_frame) >= e->cap)
    return set_error(GGRS_E_INVALID, "input queue full (capacity %d)", e->cap);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t S = e->cfg.num_sessions;
  const int P = e->cfg.num_players;
  const size_t bytes = (size_t)n * S * P;
  if (bytes > e->staging_bytes) {
    if (e->staging) HIP_TRY(hipFree(e->staging));
    e->staging = nullptr;
    e->staging_bytes = 0;
    HIP_TRY(hipMalloc(&e->staging, bytes));
    e->staging_bytes = bytes;
  }
  HIP_TRY(hipMemcpyAsync(e->staging, inputs, bytes, hipMemcpyHostToDevice, e->stream));
  pack_inputs_kernel<<<grid_of((int64_t)n * S, 256), 256, 0, e->stream>>>(e->staging, e->inputs, S, P, e->Pp, n,
                                                                          first_frame % e->cap, e->cap);
  HIP_TRY(hipGetLastError());
  if (e->sched) {  // the frame each row slot now holds (a remote row is checked against it on arrival)
    for (int32_t k = 0; k < n; k++) e->row_tag_host[(size_t)((first_frame + k) % e->cap)] = first_frame + k;
    HIP_TRY(hipMemcpyAsync(e->row_tag, e->row_tag_host.data(), sizeof(int32_t) * e->cap, hipMemcpyHostToDevice,
                           e->stream));
  }
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->next_input_frame = first_frame + n;
  return GGRS_OK;
}

int ggrs_p2p_advance_frames(ggrs_p2p_engine_t* e, int32_t n) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (n < 0) return set_error(GGRS_E_INVALID, "n_frames must be >= 0");
  if (n == 0) return GGRS_OK;
  if ((int64_t)e->current_frame + n > e->next_input_frame)
    return set_error(GGRS_E_INVALID, "Missing local input: inputs are queued up to frame %d, calls need up to %d",
                     e->next_input_frame - 1, e->current_frame + n - 1);
  HIP_TRY(hipSetDevice(e->cfg.device));
  if (e->sched) return p2p_sched_advance(e, n);  // per-session arrival schedules (p2p_sched.hip)
  P2PParams p;
  p.S = e->cfg.num_sessions;
  p.R = e->R;
  p.D = e->cfg.remote_latency;
  p.delay = e->cfg.input_delay;
  p.cap = e->cap;
  p.trace_cap = e->cfg.trace_capacity;
  p.f0 = e->current_frame;
  p.n = n;
  p.predictor = e->cfg.predictor;
  p.local_mask = (uint32_t)e->cfg.local_mask;
  p.cur = e->cur;
  p.ring = e->ring;
  p.inputs = e->inputs;
  p.queue = e->queue;
  p.rollbacks = e->rollbacks;
  p.resim = e->resim;
  p.trace = e->trace;
  p.desync_interval = e->desync_interval;
  p.hist = e->hist;
  p.dbg_sess = e->dbg_sess;
  p.dbg_frame = e->dbg_frame;
  p.sparse = e->sparse;
  p.last_saved = e->last_saved;
  p.ring_frame = e->ring_frame;
  // rows the calls read must still be in the ring: rows >= oldest_row(f0) up to f0 + n - 1
  if ((int64_t)p.f0 + n - 1 - oldest_row(e, p.f0) >= e->cap)
    return set_error(GGRS_E_INVALID, "advance of %d frames reads more input rows than input_capacity (%d)", n, e->cap);
  if (e->cfg.max_prediction == 0) {  // lockstep mode
    std::vector<int32_t> prog;
    lockstep_program(e, p.f0, n, prog);
    if (n > e->ls_prog_cap) {
      if (e->ls_prog) HIP_TRY(hipFree(e->ls_prog));
      e->ls_prog = nullptr;
      e->ls_prog_cap = 0;
      HIP_TRY(hipMalloc(&e->ls_prog, sizeof(int32_t) * 2 * (size_t)n));
      e->ls_prog_cap = n;
    }
    HIP_TRY(hipMemcpyAsync(e->ls_prog, prog.data(), sizeof(int32_t) * 2 * (size_t)n, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));  // prog is host memory that goes out of scope
    int rc = p2p_launch_timed(e, [&] {
      dispatch_players(e->cfg.num_players, [&](auto PC) {
        constexpr int P = decltype(PC)::value;
        p2p_lockstep_kernel<P><<<grid_of(p.S, 256), 256, 0, e->stream>>>(p, e->ls_prog);
      });
    });
    if (rc) return rc;
    e->current_frame += n;
    return GGRS_OK;
  }
  // the chains form: forced (form 4), or by default when the flat kernel's one thread per session
  // would leave most SIMDs idle
  const int P = e->cfg.num_players;
  // the chains form's lanes per session: D roles + the batch for 2 <= D <= 8, else D + 1 roles
  const bool chain_batch = p.D >= 2 && p.D <= 8;
  const int G = (chain_batch ? p.D : p.D + 1) * padded_players(P);
  // plain history: the session's states are the canonical ones the remote inputs determine (the
  // canonical flat kernel also keeps the desync history; the chains form does not)
  const bool plain_hist = !e->sparse && !p.trace && !e->dbg_ever;
  const bool chains_ok = plain_hist && e->desync_interval == 0 && G <= kWave &&
                         (uint64_t)p.S * e->R * cell_dwords(P) * 4 < ((uint64_t)1 << 30);
  const bool chains = chains_ok && (e->form == 4 || (e->form == 0 && grid_of(p.S, kFlatBlock) <= e->num_cus));
  if (e->form == 4 && !chains_ok)
    return set_error(GGRS_E_STATE, "the chains form needs plain launches (no desync detection, trace, debug flip or "
                                   "sparse saving), (remote_latency + 1) x padded players <= 64 lanes and a ring < 1 GiB");
  // the canonical flat kernel needs the same plain history and the remote inputs flowing (f0 >= D)
  const bool canon_ok = plain_hist && (e->form == 0 || e->form == 6);
  // and its sparse-saving form the same launches with sparse saving on
  const bool canon_sparse_ok = e->sparse && !p.trace && !e->dbg_ever && (e->form == 0 || e->form == 6);
  if ((chains || canon_ok || canon_sparse_ok) && p.f0 < p.D) {  // the first D calls (no remote input yet): general flat
    const int32_t m = std::min(n, p.D - p.f0);
    const int32_t form = e->form;
    e->form = 5;
    int rc = ggrs_p2p_advance_frames(e, m);
    e->form = form;
    if (rc || m == n) return rc;
    return ggrs_p2p_advance_frames(e, n - m);
  }
  if (chains) {
    const int spw = kWave / G;
    const int row_bytes = spw * padded_players(P);
    // a launch's rows (f0 - 2D - delay .. f0 + n - 1) must fit the block's LDS: longer runs split
    const int32_t max_n = kChainLdsRows / row_bytes - 2 * p.D - p.delay;
    if (max_n < 1) return set_error(GGRS_E_INVALID, "remote_latency / input_delay too large for the chains form");
    if (n > max_n) {
      int rc = ggrs_p2p_advance_frames(e, max_n);
      if (rc) return rc;
      return ggrs_p2p_advance_frames(e, n - max_n);
    }
    // config 2's P2P shape (latency 8, two players): the compile-time form, whose decoded input
    // records cap a launch's rows by its LDS budget
    const size_t fast_fixed = (size_t)2 * 8 * row_bytes * kStashEntry + 16 + 16;  // stash, alignment, input-0 record
    const int32_t fast_n = (int32_t)((kChainFastLds - fast_fixed) / ((size_t)row_bytes * 17)) - 2 * p.D - p.delay;
    // (an input delay so long that no call fits the budget: the general form)
    const bool fast = chain_batch && p.D == 8 && P == 2 && fast_n >= 1;
    if (fast) {
      if (n > fast_n) {
        int rc = ggrs_p2p_advance_frames(e, fast_n);
        if (rc) return rc;
        return ggrs_p2p_advance_frames(e, n - fast_n);
      }
    }
    size_t lds = (size_t)(n + 2 * p.D + p.delay) * row_bytes;
    const size_t n_entries = lds;
    if (chain_batch) lds = ((lds + 15) & ~(size_t)15) + (size_t)(p.D + 1) * kWave * kStashEntry;
    if (fast)  // rows, the stash's 2D slots of row_bytes entries, the input records
      lds = ((n_entries + 15) & ~(size_t)15) + (size_t)2 * p.D * row_bytes * kStashEntry + (n_entries + 1) * 16;
    int rc = p2p_launch_timed(e, [&] {
      dispatch_players(P, [&](auto PC) {
        constexpr int PP = decltype(PC)::value;
        if constexpr (PP == 2) {
          if (fast) {
            p2p_chains_kernel<PP, true, 8><<<(unsigned)grid_of(p.S, spw), kWave, lds, e->stream>>>(p, spw);
            return;
          }
        }
        if (chain_batch) p2p_chains_kernel<PP, true><<<(unsigned)grid_of(p.S, spw), kWave, lds, e->stream>>>(p, spw);
        else p2p_chains_kernel<PP, false><<<(unsigned)grid_of(p.S, spw), kWave, lds, e->stream>>>(p, spw);
      });
    });
    if (rc) return rc;
    e->current_frame += n;
    return GGRS_OK;
  }
  int rc = p2p_launch_timed(e, [&] {
    // stage input rows in LDS unless a call reaches further back than a stage holds
    const int32_t back = (e->sparse ? e->R - 1 : p.D) + p.delay;
    const bool staged = back + 1 <= kP2PRows - 1 && e->form != 1;
    // the flat form by default: with the session-major ring its saves stay whole cache lines
    // whatever frame each lane is at (1.82e10 vs lockstep 1.26e10 session-frames/s at 65,536
    // sessions, 1.98e10 vs 1.89e10 at 131,072; with the frame-major ring of round 1 the flat
    // form's partial lines went out to HBM 3.5x over -- DESIGN.md section 5)
    const bool flat = staged && (e->form == 0 || e->form == 3 || e->form == 5 || e->form == 6);
    dispatch_players(e->cfg.num_players, [&](auto PC) {
      constexpr int P = decltype(PC)::value;
      if (flat) {
        const dim3 grid((unsigned)grid_of(p.S, kFlatBlock));
        // the LDS ring when a stage of rows holds a call's reach and the block's rings fit: 28 KB
        // (four blocks, one per SIMD, in a CU's 160 KB beside 12 KB of rows each), or more when the
        // grid puts fewer blocks on each CU (config 2's P2P shape: 4096 sessions = 64 blocks, R = 10:
        // 30 KB of rings)
        const size_t ring_lds = (size_t)e->R * (cell_dwords(P) / 4) * kFlatBlock * 16;
        const size_t rows_lds = (size_t)flat_rows_lds<P>() * kFlatBlock * (P <= 1 ? 1 : (P == 2 ? 2 : 4));
        const int64_t per_cu = (grid.x + e->num_cus - 1) / e->num_cus;
        const bool fits = ring_lds <= 28 * 1024 ||
                          (ring_lds + rows_lds <= 64 * 1024 && per_cu * (int64_t)(ring_lds + rows_lds) <= 160 * 1024);
        const bool lds = e->form != 3 && fits && back + 1 <= flat_rows_lds<P>() - 1;
        auto go = [&](auto plain_tag, auto lds_tag) {
          constexpr bool kPl = decltype(plain_tag)::value;
          constexpr bool kL = decltype(lds_tag)::value;
          const size_t shm = kL ? ring_lds : 0;
          if (e->sparse) {
            p2p_flat_kernel<P, -1, kPl, true, kL><<<grid, kFlatBlock, shm, e->stream>>>(p);
          } else if constexpr (P == 2) {
            if (p.local_mask == 1u) p2p_flat_kernel<P, 1, kPl, false, kL><<<grid, kFlatBlock, shm, e->stream>>>(p);
            else if (p.local_mask == 2u) p2p_flat_kernel<P, 2, kPl, false, kL><<<grid, kFlatBlock, shm, e->stream>>>(p);
            else p2p_flat_kernel<P, -1, kPl, false, kL><<<grid, kFlatBlock, shm, e->stream>>>(p);
          } else {
            p2p_flat_kernel<P, -1, kPl, false, kL><<<grid, kFlatBlock, shm, e->stream>>>(p);
          }
        };
        const bool plain = p.desync_interval == 0 && !p.trace && p.dbg_sess < 0;
        if (lds && canon_sparse_ok) {  // the canonical flat kernel with sparse saving (f0 >= D here)
          const size_t shm = ring_lds;
          if constexpr (P == 2) {
            if (p.local_mask == 1u) p2p_canon_sparse_kernel<P, 1><<<grid, kFlatBlock, shm, e->stream>>>(p);
            else if (p.local_mask == 2u) p2p_canon_sparse_kernel<P, 2><<<grid, kFlatBlock, shm, e->stream>>>(p);
            else p2p_canon_sparse_kernel<P, -1><<<grid, kFlatBlock, shm, e->stream>>>(p);
          } else {
            p2p_canon_sparse_kernel<P, -1><<<grid, kFlatBlock, shm, e->stream>>>(p);
          }
          return;
        }
        if (lds && canon_ok) {  // the canonical flat kernel (f0 >= D here)
          const size_t shm = ring_lds;
          if constexpr (P == 2) {
            if (p.local_mask == 1u) p2p_canon_kernel<P, 1><<<grid, kFlatBlock, shm, e->stream>>>(p);
            else if (p.local_mask == 2u) p2p_canon_kernel<P, 2><<<grid, kFlatBlock, shm, e->stream>>>(p);
            else p2p_canon_kernel<P, -1><<<grid, kFlatBlock, shm, e->stream>>>(p);
          } else {
            p2p_canon_kernel<P, -1><<<grid, kFlatBlock, shm, e->stream>>>(p);
          }
          return;
        }
        if (lds) {
          if (plain) go(std::true_type(), std::true_type());
          else go(std::false_type(), std::true_type());
        } else {
          if (plain) go(std::true_type(), std::false_type());
          else go(std::false_type(), std::false_type());
        }
      }
      else if (staged) p2p_kernel<P, true><<<grid_of(p.S, kP2PBlock), kP2PBlock, 0, e->stream>>>(p);
      else p2p_kernel<P, false><<<grid_of(p.S, kP2PBlock), kP2PBlock, 0, e->stream>>>(p);
    });
  });
  if (rc) return rc;
  e->current_frame += n;
  return GGRS_OK;
}

int ggrs_p2p_set_desync_detection(ggrs_p2p_engine_t* e, int32_t interval) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (interval < 0) return set_error(GGRS_E_INVALID, "interval must be >= 0 (0 = DesyncDetection::Off)");
  if (interval > 0 && e->sparse)
    return set_error(GGRS_E_STATE, "desync detection with sparse saving is not supported: the reference sends a "
                                   "report only for a frame it saved (p2p_session.rs:948-962, sync_layer.rs:323-326)");
  if (e->current_frame != 0)
    return set_error(GGRS_E_STATE, "desync detection is part of the session's configuration (set before the first frame)");
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t S = e->cfg.num_sessions;
  if (interval > 0 && !e->hist) {
    HIP_TRY(hipMalloc(&e->hist, sizeof(uint16_t) * kHist * S));
    HIP_TRY(hipMemsetAsync(e->hist, 0, sizeof(uint16_t) * kHist * S, e->stream));
    HIP_TRY(hipMalloc(&e->cmp_mask, sizeof(uint64_t) * ((S + 63) / 64)));
    HIP_TRY(hipMalloc(&e->cmp_count, sizeof(int32_t)));
  }
  e->desync_interval = interval;
  if (interval > 0 && e->sched) return p2p_sched_desync_alloc(e);
  return GGRS_OK;
}

int ggrs_p2p_set_sparse_saving(ggrs_p2p_engine_t* e, int32_t on) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (e->current_frame != 0)
    return set_error(GGRS_E_STATE, "sparse saving is part of the session's configuration (set before the first frame)");
  if (on && e->desync_interval > 0)
    return set_error(GGRS_E_STATE, "sparse saving with desync detection is not supported: the reference sends a "
                                   "report only for a frame it saved (p2p_session.rs:948-962, sync_layer.rs:323-326)");
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t S = e->cfg.num_sessions;
  if (on && !e->last_saved) {
    HIP_TRY(hipMalloc(&e->last_saved, sizeof(int32_t) * S));
    HIP_TRY(hipMemsetAsync(e->last_saved, 0xff, sizeof(int32_t) * S, e->stream));  // NULL_FRAME
    // (scheduled mode may have allocated the cell frames already: p2p_sched_enable)
    if (!e->ring_frame) HIP_TRY(hipMalloc(&e->ring_frame, sizeof(int32_t) * e->R * S));
    HIP_TRY(hipMemsetAsync(e->ring_frame, 0xff, sizeof(int32_t) * e->R * S, e->stream));
  }
  // ignored in lockstep mode, as the reference does (p2p_session.rs:187-197)
  e->sparse = (on && e->cfg.max_prediction > 0) ? 1 : 0;
  return GGRS_OK;
}

int ggrs_p2p_set_unstaged(ggrs_p2p_engine_t* e, int32_t form) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (form < 0 || form > 6)
    return set_error(GGRS_E_INVALID, "kernel form %d (0 default, 1 unstaged, 2 lockstep, 3 flat HBM rings, 4 chains, "
                                     "5 flat LDS rings with the queue bookkeeping, 6 canonical flat)", form);
  e->form = form;
  return GGRS_OK;
}

int ggrs_p2p_debug_desync(ggrs_p2p_engine_t* e, int32_t session, int32_t frame) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (session >= e->cfg.num_sessions) return set_error(GGRS_E_INVALID, "session out of range");
  e->dbg_sess = session;
  e->dbg_frame = session < 0 ? -1 : frame;
  if (session >= 0) e->dbg_ever = true;
  return GGRS_OK;
}

// The local history row of report frame `frame`: sent at call frame + D + 1, kept while it is one
// of the kHist newest reports (local_checksum_history retention, p2p_session.rs:965-970).
static int hist_row(ggrs_p2p_engine_t* e, int32_t frame, const uint16_t** row) {
  const int32_t I = e->desync_interval, D = e->cfg.remote_latency;
  if (I <= 0) return set_error(GGRS_E_STATE, "desync detection is off");
  if (e->cfg.max_prediction == 0)
    return set_error(GGRS_E_PRECONDITION, "frame %d not reported: lockstep mode saves no state, so no checksum "
                                          "report is ever sent (p2p_session.rs:948-962)", frame);
  if (frame < I || frame % I != 0) return set_error(GGRS_E_PRECONDITION, "frame %d is not a checksum report frame", frame);
  const int32_t newest = e->current_frame - 2 - D;  // frame_to_send of the last call run
  if (frame > newest) return set_error(GGRS_E_PRECONDITION, "frame %d not reported yet", frame);
  if (frame <= newest - kHist * I) return set_error(GGRS_E_PRECONDITION, "frame %d left the checksum history", frame);
  *row = e->hist + (int64_t)((frame / I) % kHist) * e->cfg.num_sessions;
  return GGRS_OK;
}

int ggrs_p2p_local_checksums(ggrs_p2p_engine_t* e, int32_t frame, uint16_t* out, int32_t out_on_device) {
  if (e && e->sched) return set_error(GGRS_E_STATE, "arrival schedules report per session: ggrs_p2p_read_reports");
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  const uint16_t* row = nullptr;
  int rc = hist_row(e, frame, &row);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(e->cfg.device));
  HIP_TRY(hipMemcpyAsync(out, row, 2 * (size_t)e->cfg.num_sessions,
                         out_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

int ggrs_p2p_compare_checksums(ggrs_p2p_engine_t* e, int32_t frame, const uint16_t* remote, int32_t remote_on_device,
                               uint64_t* mask, int32_t* n_differ) {
  if (e && e->sched) return set_error(GGRS_E_STATE, "arrival schedules report per session: ggrs_p2p_read_reports");
  if (!e || !remote || !mask || !n_differ) return set_error(GGRS_E_INVALID, "null argument");
  const uint16_t* row = nullptr;
  int rc = hist_row(e, frame, &row);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t S = e->cfg.num_sessions;
  const uint16_t* rdev = remote;
  if (!remote_on_device) {
    if ((size_t)2 * S > e->staging_bytes) {
      if (e->staging) HIP_TRY(hipFree(e->staging));
      e->staging = nullptr;
      e->staging_bytes = 0;
      HIP_TRY(hipMalloc(&e->staging, 2 * S));
      e->staging_bytes = 2 * S;
    }
    HIP_TRY(hipMemcpyAsync(e->staging, remote, 2 * S, hipMemcpyHostToDevice, e->stream));
    rdev = (const uint16_t*)e->staging;
  }
  HIP_TRY(hipMemsetAsync(e->cmp_count, 0, sizeof(int32_t), e->stream));
  compare_checksums_kernel<<<grid_of(S, 256), 256, 0, e->stream>>>(row, rdev, S, e->cmp_mask, e->cmp_count);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(mask, e->cmp_mask, 8 * (size_t)((S + 63) / 64), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipMemcpyAsync(n_differ, e->cmp_count, sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

int ggrs_p2p_current_frame(const ggrs_p2p_engine_t* e, int32_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  // P2PSession::current_frame (:555-558): every call advances in rollback mode; in lockstep mode
  // calls wait for confirmed inputs
  if (e->sched)
    return set_error(GGRS_E_STATE, "with arrival schedules every session has its own frame (ggrs_p2p_read_sessions)");
  *out = e->cfg.max_prediction == 0 ? e->ls_frame : e->current_frame;
  return GGRS_OK;
}

int ggrs_p2p_calls(const ggrs_p2p_engine_t* e, int32_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  *out = e->current_frame;
  return GGRS_OK;
}

int ggrs_p2p_synchronize(ggrs_p2p_engine_t* e) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

// field k of the record at base[k * stride] (cur: stride S from the session's lane; ring: the
// session's contiguous cell, stride 1)
static int read_record(ggrs_p2p_engine_t* e, const uint32_t* base, int64_t stride, uint8_t* out) {
  std::vector<uint32_t> w(e->F);
  for (int k = 0; k < e->F; k++)
    HIP_TRY(hipMemcpyAsync(&w[k], base + (int64_t)k * stride, 4, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  serialize_state_bytes(w.data(), e->cfg.num_players, out);
  return GGRS_OK;
}

int ggrs_p2p_read_state(ggrs_p2p_engine_t* e, int32_t session, uint8_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  if (session < 0 || session >= e->cfg.num_sessions) return set_error(GGRS_E_INVALID, "session out of range");
  HIP_TRY(hipSetDevice(e->cfg.device));
  return read_record(e, e->cur + session, e->cfg.num_sessions, out);
}

int ggrs_p2p_read_states(ggrs_p2p_engine_t* e, uint8_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t S = e->cfg.num_sessions;
  const size_t sb = 36 + 20 * (size_t)e->cfg.num_players;
  std::vector<uint32_t> soa((size_t)e->F * S);  // field k of every session, one copy
  HIP_TRY(hipMemcpyAsync(soa.data(), e->cur, soa.size() * 4, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  std::vector<uint32_t> w(e->F);
  for (int64_t s = 0; s < S; s++) {
    for (int k = 0; k < e->F; k++) w[k] = soa[(size_t)k * S + s];
    serialize_state_bytes(w.data(), e->cfg.num_players, out + (size_t)s * sb);
  }
  return GGRS_OK;
}

int ggrs_p2p_read_ring(ggrs_p2p_engine_t* e, int32_t session, int32_t* frames, uint16_t* checksums, uint8_t* states) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (session < 0 || session >= e->cfg.num_sessions) return set_error(GGRS_E_INVALID, "session out of range");
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t S = e->cfg.num_sessions;
  const int32_t R = e->R, f = e->current_frame;
  const size_t sb = 36 + 20 * (size_t)e->cfg.num_players;
  for (int32_t slot = 0; slot < R; slot++) {
    // after call f-1 the cells hold frames f-R .. f-1 (every call saves its current frame);
    // with sparse saving the per-session tags say
    int32_t fr = kNull;
    if (e->cfg.max_prediction == 0) {
      // lockstep mode never saves
    } else if (e->sparse || e->sched) {
      HIP_TRY(hipMemcpy(&fr, e->ring_frame + (int64_t)slot * S + session, 4, hipMemcpyDeviceToHost));
    } else {
      for (int32_t g = f - 1; g >= 0 && g >= f - R; g--)
        if (g % R == slot) { fr = g; break; }
    }
    if (frames) frames[slot] = fr;
    if (checksums) {
      checksums[slot] = 0;
      if (fr != kNull)
        HIP_TRY(hipMemcpy(&checksums[slot], e->ring + ((int64_t)session * R + slot) * cell_dwords(e->cfg.num_players) +
                                                 e->F, 2, hipMemcpyDeviceToHost));
    }
    if (states) {
      if (fr == kNull) {
        std::memset(states + slot * sb, 0, sb);
      } else {
        int rc = read_record(e, e->ring + ((int64_t)session * R + slot) * cell_dwords(e->cfg.num_players), 1,
                             states + slot * sb);
        if (rc) return rc;
      }
    }
  }
  return GGRS_OK;
}

int ggrs_p2p_read_stats(ggrs_p2p_engine_t* e, int32_t* rollbacks, int64_t* resim_frames) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t S = e->cfg.num_sessions;
  if (rollbacks) HIP_TRY(hipMemcpyAsync(rollbacks, e->rollbacks, 4 * S, hipMemcpyDeviceToHost, e->stream));
  if (resim_frames) HIP_TRY(hipMemcpyAsync(resim_frames, e->resim, 8 * S, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

int ggrs_p2p_read_queues(ggrs_p2p_engine_t* e, int32_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  if (e->sched) return set_error(GGRS_E_STATE, "the queue words of scheduled mode are per session (ggrs_p2p_read_sessions)");
  HIP_TRY(hipSetDevice(e->cfg.device));
  const size_t bytes = sizeof(int32_t) * 4 * e->cfg.num_players * (size_t)e->cfg.num_sessions;
  HIP_TRY(hipMemcpyAsync(out, e->queue, bytes, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

int ggrs_p2p_read_trace(ggrs_p2p_engine_t* e, int32_t first_frame, int32_t n, uint16_t* out) {
  if (!e || (!out && n > 0)) return set_error(GGRS_E_INVALID, "null argument");
  if (!e->trace) return set_error(GGRS_E_PRECONDITION, "engine created with trace_capacity 0");
  const int32_t T = e->cfg.trace_capacity;
  if (n < 0 || first_frame < 0 || first_frame + n > e->current_frame || first_frame + T < e->current_frame)
    return set_error(GGRS_E_INVALID, "trace frames out of the retained range");
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t S = e->cfg.num_sessions;
  for (int32_t i = 0; i < n; i++)
    HIP_TRY(hipMemcpyAsync(out + (int64_t)i * S, e->trace + (int64_t)((first_frame + i) % T) * S, 2 * S,
                           hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

int ggrs_p2p_timing_reset(ggrs_p2p_engine_t* e) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  return e->timer.reset(e->stream);
}

int ggrs_p2p_timing_stop(ggrs_p2p_engine_t* e) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  return e->timer.stop(e->stream);
}

int ggrs_p2p_timing_read(ggrs_p2p_engine_t* e, float* total_ms, int32_t* launches) {
  if (!e || !total_ms || !launches) return set_error(GGRS_E_INVALID, "null argument");
  HIP_TRY(hipSetDevice(e->cfg.device));
  return e->timer.read(e->stream, total_ms, launches);
}

}  // extern "C"
