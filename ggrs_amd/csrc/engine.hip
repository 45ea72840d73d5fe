// engine.hip -- the MI355X batched rollback-resimulation engine: HBM-resident SoA state ring,
// fused SyncTest / request-program kernels (one lane per (session, branch)), C ABI.
//
// Reference path (caspark/ggrs 0.10.2): SyncTestSession::advance_frame
// (src/sessions/sync_test_session.rs:85-150) driving SyncLayer (src/sync_layer.rs:144-375) and the
// user's request handler Game::handle_requests (examples/ex_game/ex_game.rs:79-127).  The C ABI is
// declared in include/ggrs_amd.h (each entry point cites the reference interface it replaces).
//
// HBM layout (lane-fastest structure of arrays, every access coalesced across a wavefront):
//   cur      [F][L]     u32  current game state; F = 1 + 5P fields in bincode order
//   ring     [R][F][L]  u32  saved-state ring, slot = frame % R (SavedStates::get_cell :161-166)
//   ring_ck  [R][L]     u16  checksum stored with each saved cell (GameStateCell.checksum)
//   first_ck [R][L]     u16  SyncTest checksum_history: first checksum seen for each frame
//   inputs   [C][L][Pp] u8   input queue, slot = queue frame % C (InputQueue, input_queue.rs:10-37)
//   trace    [T][L]     u16  optional per-frame display checksum (ex_game.rs:121-126)
// Frame bookkeeping (current frame, which frame each ring slot holds) is identical for all lanes
// of an engine -- lanes run the same request program -- so it lives on the host and reaches the
// kernels as scalars; only halted lanes (MismatchedChecksum) leave the common program.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "engine.h"

#pragma clang fp contract(off)

using namespace ggrs;

namespace ggrs {

thread_local std::string g_last_error;

int set_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

}  // namespace ggrs

namespace {

// ------------------------------------------------------------------------------ kernels
struct SyncTestParams {
  int64_t L;
  int32_t R, cd, f0, n, cap, trace_cap;
  int32_t corrupt_lane, corrupt_frame;
  uint32_t* cur;
  uint32_t* ring;
  uint16_t* ring_ck;
  uint16_t* first_ck;
  const uint8_t* inputs;
  int32_t* lane_status;
  int32_t* mis_frame;
  uint64_t* mis_mask;
  uint16_t* trace;
};

template <int P>
__device__ inline uint16_t save_cell(const SyncTestParams& p, const BoxState<P>& s, int slot,
                                     int64_t lane) {
  store_state<P>(s, p.ring + (int64_t)slot * state_fields(P) * p.L + lane, p.L);
  const uint16_t ck = fletcher16_state<P>(s);
  p.ring_ck[(int64_t)slot * p.L + lane] = ck;
  return ck;
}

// n SyncTest frames for every running lane, each: [checksums_consistent over f-cd..f]
// [Load f-cd, (Advance, Save)..., Advance]  Save f, Advance  -- sync_test_session.rs:85-150.
// Which cells and history entries exist is a pure function of (f, cd, R) for a session driven
// only by this program since frame 0 (see DESIGN.md "SyncTest bookkeeping"):
//   * at call f the ring holds every frame in [f-R, f-1], so each frame in [f-cd, f-1] is present
//     and frame f is not;
//   * frame fc enters checksum_history at call max(fc+1, cd+1) with the checksum of its first
//     save (call fc's "save current state"), kept in first_ck; it is compared against the cell at
//     every later call while fc >= f-cd, i.e. at call f >= cd+2 for fc in [f-cd, f-2].
template <int P>
__global__ __launch_bounds__(kWave) void synctest_kernel(SyncTestParams p) {
  const int64_t lane = (int64_t)blockIdx.x * kWave + threadIdx.x;
  if (lane >= p.L) return;
  if (p.lane_status[lane] != GGRS_LANE_RUNNING) return;
  const int64_t L = p.L;
  BoxState<P> s;
  load_state<P>(s, p.cur + lane, L);
  const int32_t cd = p.cd, R = p.R;
  for (int32_t f = p.f0; f < p.f0 + p.n; ++f) {
    if (cd > 0 && f > cd) {
      if (f >= cd + 2) {
        uint64_t mism = 0;
        for (int32_t fc = f - cd; fc <= f - 2; ++fc) {
          const int64_t o = (int64_t)(fc % R) * L + lane;
          if (p.ring_ck[o] != p.first_ck[o]) mism |= 1ull << (fc - (f - cd));
        }
        if (mism) {  // GgrsError::MismatchedChecksum: the session stops before the rollback
          p.lane_status[lane] = GGRS_LANE_MISMATCH;
          p.mis_frame[lane] = f;
          p.mis_mask[lane] = mism;
          break;
        }
      }
      int32_t g = f - cd;  // adjust_gamestate(f - cd): Load, then cd x (Save unless first, Advance)
      load_state<P>(s, p.ring + (int64_t)(g % R) * state_fields(P) * L + lane, L);
      if (lane == p.corrupt_lane && f == p.corrupt_frame) s.w[fld_x(P, 0)] ^= 1u;
      for (int32_t i = 0; i < cd; ++i, ++g) {
        if (i > 0) save_cell<P>(p, s, g % R, lane);
        advance_state<P>(s, load_inputs<P>(p.inputs, (int64_t)(g % p.cap) * L + lane), 0u);
      }
    }
    if (cd > 0) {  // save_current_state + its first sighting in checksum_history
      const uint16_t ck = save_cell<P>(p, s, f % R, lane);
      p.first_ck[(int64_t)(f % R) * L + lane] = ck;
    }
    advance_state<P>(s, load_inputs<P>(p.inputs, (int64_t)(f % p.cap) * L + lane), 0u);
    if (p.trace) p.trace[(int64_t)(f % p.trace_cap) * L + lane] = fletcher16_state<P>(s);
  }
  store_state<P>(s, p.cur + lane, L);
}

// ------------------------------------------------------------------------------------------
// Pipelined SyncTest program (the fast path for calls f > cd).
//
// Call c's replay (adjust_gamestate, sync_test_session.rs:192-217) loads the cell of frame c-cd,
// which call c-1 saved right after its FIRST replayed advance; everything else call c does hangs
// off that state as a chain of cd+1 advances (cd-1 re-saves, the save of frame c, the new frame's
// advance).  So with K = cd+1 lanes per session, chain c runs on lane c mod K over time steps
// t = c .. c+cd (step i = t-c), and the K chains of a session advance in lockstep:
//   * at step t every chain holds (its own replay of) frame t-cd, advances it with input t-cd
//     (one input load per session), and - unless it just loaded - saves it first;
//   * the chain starting at t (i = 0) takes the state chain t-1 is about to save (the cell of
//     frame t-cd, i.e. its LoadGameState) from that lane's registers; the first chain of a launch
//     loads it from the HBM ring, where the previous launch saved it;
//   * chain t-cd saves frame t-cd as "current" (its first-seen checksum, first_ck) in the same
//     step in which chains t-cd+1 .. t-1 re-save it, so their comparison against the first-seen
//     value (checksums_consistent at their next call) is a register broadcast.
// Every Load, Save (state + Fletcher-16 into the ring) and AdvanceFrame of the reference program
// is executed; only the schedule changes.  A chain whose re-saves mismatch records the launch in
// *fail_f0; the host then restores the checkpoint taken before the launch and replays it with the
// sequential kernel above, which reproduces the reference's Err state exactly (stop at the first
// failing call, ring and state as the reference leaves them).
struct PipeParams {
  int64_t L;
  int32_t R, cd, K, spw, f0, n, cap, trace_cap;
  int32_t corrupt_lane, corrupt_frame;
  uint32_t* cur;
  uint32_t* ring;
  uint16_t* ring_ck;
  uint16_t* first_ck;
  const uint8_t* inputs;
  const int32_t* lane_status;
  int32_t* fail_f0;
  uint16_t* trace;
  // the launch checkpoint, taken by the kernel itself: each block copies its own sessions' cur /
  // ring / ring_ck / first_ck entries into its own contiguous `block_bytes` piece of `shadow`
  // (whole cache lines, not a scatter into an arena-shaped copy) before it writes any of them
  uint8_t* shadow;
  int64_t block_bytes;
};

// Shadow layout of one block's checkpoint (sessions [s0, s0 + nsess)): first every 32-bit row
// entry q of cur (F rows) and ring (R*F rows), q = row * nsess + session, then every 16-bit entry
// of ring_ck (R rows) and first_ck (R rows).  checkpoint_sessions writes it, restore_kernel maps it
// back; both index through these two functions.
struct CheckpointMap {
  int64_t L;
  int R, F, spw;
  uint32_t* cur;
  uint32_t* ring;
  uint16_t* ring_ck;
  uint16_t* first_ck;
  __device__ uint32_t* at32(int64_t s0, int nsess, int q) const {
    const int row = q / nsess, ss = q - row * nsess;
    return row < F ? cur + (int64_t)row * L + s0 + ss : ring + (int64_t)(row - F) * L + s0 + ss;
  }
  __device__ uint16_t* at16(int64_t s0, int nsess, int q) const {
    const int row = q / nsess, ss = q - row * nsess;
    return row < R ? ring_ck + (int64_t)row * L + s0 + ss : first_ck + (int64_t)(row - R) * L + s0 + ss;
  }
};

__host__ __device__ inline int64_t checkpoint_block_bytes(int R, int F, int spw) {
  const int64_t b32 = (int64_t)(1 + R) * F * spw * 4, b16 = (int64_t)2 * R * spw * 2;
  return (b32 + b16 + 15) & ~(int64_t)15;
}

// Copy of sessions [s0, s0 + nsess) into this block's shadow piece, eight loads in flight per
// thread before their stores.
__device__ inline void checkpoint_sessions(const CheckpointMap& m, uint8_t* piece, int64_t s0, int nsess, int tid,
                                           int nthreads) {
  const int n32 = (1 + m.R) * m.F * nsess, n16 = 2 * m.R * nsess;
  uint32_t* d32 = (uint32_t*)piece;
  uint16_t* d16 = (uint16_t*)(piece + (int64_t)(1 + m.R) * m.F * m.spw * 4);
  for (int base = 0; base < n32; base += 8 * nthreads) {
    uint32_t v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int q = base + u * nthreads + tid;
      if (q < n32) v[u] = *m.at32(s0, nsess, q);
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int q = base + u * nthreads + tid;
      if (q < n32) d32[q] = v[u];
    }
  }
  for (int base = 0; base < n16; base += 8 * nthreads) {
    uint16_t v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int q = base + u * nthreads + tid;
      if (q < n16) v[u] = *m.at16(s0, nsess, q);
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int q = base + u * nthreads + tid;
      if (q < n16) d16[q] = v[u];
    }
  }
}

// Restore of a failed launch's checkpoint: block b writes its piece back into the arena.
__global__ __launch_bounds__(256) void restore_kernel(CheckpointMap m, const uint8_t* shadow, int64_t block_bytes) {
  const int64_t s0 = (int64_t)blockIdx.x * m.spw;
  const int nsess = (int)((m.L - s0) < m.spw ? (m.L - s0) : m.spw);
  const uint8_t* piece = shadow + (int64_t)blockIdx.x * block_bytes;
  const uint32_t* s32 = (const uint32_t*)piece;
  const uint16_t* s16 = (const uint16_t*)(piece + (int64_t)(1 + m.R) * m.F * m.spw * 4);
  const int n32 = (1 + m.R) * m.F * nsess, n16 = 2 * m.R * nsess;
  for (int q = threadIdx.x; q < n32; q += blockDim.x) *m.at32(s0, nsess, q) = s32[q];
  for (int q = threadIdx.x; q < n16; q += blockDim.x) *m.at16(s0, nsess, q) = s16[q];
}

// Every store of the v4 kernel is a buffer store whose offset is pushed out of the descriptor's
// range on lanes that must not store (no exec-mask branches); buffers must be < 1 GiB.
constexpr uint32_t kOob = 0x40000000u;  // >= every descriptor's num_records; two of them never wrap

__device__ inline __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// LDS staging of the inputs: every chain of a session reads the same input byte per step, and a
// global load inside the step loop would be waited on with vmcnt, which also counts the step's
// ring stores (they retire in order) -- so inputs for kStageFrames frames at a time are copied to
// LDS, and the loop body issues no global loads at all.
constexpr int kStageFrames = 256;
constexpr int kMaxRampFrames = 64;  // first-seen checksums of frames f0-cd .. f0-1 (cd <= 62)

// LDS staging of input-queue rows: frames gf .. gf + nf - 1 (queue slot (gf + ff) % cap; every
// staged frame is held by the queue at once, so nf <= cap and the slot wraps at most once) for the
// block's sessions [s0, s0 + nsess): row ff's first `used` = nsess * Pp bytes are the sessions'
// input records, bytes up to `row` are zero.  Every load of a thread is issued before its LDS
// stores, so a stage costs one memory latency (a load-wait-store loop paid one per byte).
// Full 8-byte rows whose source is 8-byte aligned move as one 64-bit load per row.
// s_waitcnt vmcnt(0) (gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15) at the end of a stage.  A
// thread's loads whose LDS store is skipped (row past the stage) stay counted at the stage's exit,
// so the compiler's wait pass put a vmcnt(0) into the step loop's first block, where the first
// write of those registers is -- there it waited, every 8 steps, for all the ring stores in flight
// (the v5 kernel's SQ_WAIT_ANY).  Draining here, once per stage, clears that state.
__device__ inline void drain_loads() { __builtin_amdgcn_s_waitcnt(0x0F70); }

template <int kRow>
__device__ inline void stage_input_rows(uint8_t* lds, const uint8_t* inputs, int64_t L, int Pp, int32_t cap,
                                        int32_t gf, int nf, int64_t s0, int used, int row_rt, int tid) {
  const int row = kRow > 0 ? kRow : row_rt;
  const int32_t q0 = gf % cap;
  auto slot = [&](int ff) {
    const int32_t q = q0 + ff;
    return q >= cap ? q - cap : q;
  };
  if (kRow == 8 && used == 8 && ((L * Pp) & 7) == 0) {
    for (int base = 0; base < nf; base += 4 * kWave) {
      uint64_t v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int ff = base + u * kWave + tid;
        if (ff < nf) v[u] = *reinterpret_cast<const uint64_t*>(inputs + ((int64_t)slot(ff) * L + s0) * Pp);
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int ff = base + u * kWave + tid;
        if (ff < nf) *reinterpret_cast<uint64_t*>(lds + ff * 8) = v[u];
      }
    }
    drain_loads();
    return;
  }
  const int total = nf * row;
  for (int base = 0; base < total; base += 8 * kWave) {
    uint8_t v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int q = base + u * kWave + tid;
      if (q < total) {
        const int ff = q / row, b = q - ff * row;
        v[u] = b < used ? inputs[((int64_t)slot(ff) * L + s0) * Pp + b] : 0;
      }
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int q = base + u * kWave + tid;
      if (q < total) lds[q] = v[u];
    }
  }
  drain_loads();
}

// ------------------------------------------------------------------------------------------
// Pipelined SyncTest, v4: static chain roles.  Same schedule and the same Loads, Saves and
// AdvanceFrames as v3, re-indexed so that no lane's role changes from step to step:
//   * lane role j (0..cd) always holds chain t - j at step t.  After every advance the chains move
//     one lane up (role j takes role j-1's post-advance state, one ds_bpermute per field) and
//     role 0 keeps its own: that state -- chain t-1 after its first replayed advance, the cell of
//     frame t-cd -- is exactly what chain t loads at step t (and what chain t-1 saves at step t);
//   * saves are issued by the producer: role j's post-advance state is the cell role j+1 saves at
//     step t+1, so roles 0..cd-1 store it (and its Fletcher-16) right after their advance, role
//     cd-1 also as the first-seen checksum, role cd's is the call's display checksum; the
//     rotation's LDS round trip overlaps the Fletcher sums and stores instead of stalling them;
//   * every per-lane predicate (save, first-seen, compare, trace) is static, so store offsets are
//     precomputed per lane (kOob where the lane never stores) plus a wave-uniform slot offset in
//     soffset, and the step has no exec-mask branches outside the ramp and tail;
//   * a mismatching re-save only sets a wave-uniform flag (the host replays a failed launch on the
//     sequential kernel anyway), folded into *fail_f0 once at the end;
//   * step arithmetic: advance_player_lean (one add per thrust axis, clamp test s > 49, med3),
//     Fletcher-16 mod 255 from doubled sums on 24-bit multiplies.
template <int P>
__global__ __launch_bounds__(kWave) void synctest_pipelined_v4_kernel(PipeParams p) {
  constexpr int Pp = P <= 1 ? 1 : (P == 2 ? 2 : 4);
  constexpr int F = state_fields(P);
  constexpr int n_bytes = Fletcher<P>::n;
  // [frame][session-in-block][Pp], one slack frame for the core loop's read-ahead past a chunk
  __shared__ uint8_t lds_in[(kStageFrames + 1) * kWave];
  __shared__ uint16_t lds_first[kMaxRampFrames * kWave];  // [ramp frame][session-in-block]
  __shared__ uint32_t lds_cell[kWave * 5];                // chain f0's LoadGameState, per lane
  // An earlier launch failed: the shadow must keep the checkpoint from before that launch (the host
  // restores it and replays from there), so this launch neither checkpoints nor runs.  A block of
  // the failing launch itself still takes its checkpoint -- another block may have flagged the
  // launch before this one was scheduled -- and only then stops.
  const int32_t failed_f0 = *p.fail_f0;
  if (failed_f0 >= 0 && failed_f0 != p.f0) return;
  const int wl = threadIdx.x;
  const int K = p.K, cd = p.cd, R = p.R;
  const int G = K * Pp;
  const int g = wl / G, r = wl - g * G;
  const int j = r / Pp, pl = r - j * Pp;  // static role, player
  const int64_t L = p.L;
  const int spw = p.spw;
  const int64_t blk = xcd_block(blockIdx.x, gridDim.x);
  const int64_t s0 = blk * spw;
  const int64_t s = s0 + g;
  const int nsess = (int)((L - s0) < spw ? (L - s0) : spw);
  const bool valid = g < spw && s < L && p.lane_status[s] == GGRS_LANE_RUNNING;
  const bool owner = valid && pl < P;
  const int64_t sl = valid ? s : 0;
  const int plc = pl < P ? pl : 0;
  const int base = g * G;
  const int src_first = ((base + (cd - 1) * Pp) & (kWave - 1)) * 4;
  const int src_rot = (j == 0 ? wl : base + (j - 1) * Pp + pl) * 4;  // ds_bpermute form
  const int kq[5] = {fld_x(P, plc), fld_y(P, plc), fld_vx(P, plc), fld_vy(P, plc), fld_rot(P, plc)};
  const uint32_t slot_bytes = (uint32_t)(F * L * 4), ck_slot_bytes = (uint32_t)(L * 2);
  // ring, ring_ck and first_ck are consecutive in the engine's arena: one descriptor from the
  // ring's base covers all three (fewer live SGPRs keeps the slot counters scalar)
  const uint32_t ck_base = (uint32_t)((const uint8_t*)p.ring_ck - (const uint8_t*)p.ring);
  const uint32_t first_base = (uint32_t)((const uint8_t*)p.first_ck - (const uint8_t*)p.ring);
  // the trace follows them in the same allocation (engine create), so the descriptor reaches it too
  const uint32_t trace_base = p.trace ? (uint32_t)((const uint8_t*)p.trace - (const uint8_t*)p.ring) : 0u;
  const __amdgpu_buffer_rsrc_t rs_ring = make_rsrc(
      p.ring, p.trace ? trace_base + ck_slot_bytes * (uint32_t)p.trace_cap : first_base + ck_slot_bytes * (uint32_t)R);
  // static store offsets: producers (roles 0..cd-1) save; role cd-1 also writes first_ck; role cd
  // writes the display checksum
  const bool producer = valid && j <= cd - 1;
  uint32_t fo[5];
#pragma unroll
  for (int q = 0; q < 5; q++) fo[q] = (producer && pl < P) ? (uint32_t)((kq[q] * L + s) * 4) : kOob;
  const uint32_t fo_frame = (producer && pl == 0) ? (uint32_t)(s * 4) : kOob;
  const uint32_t co = (producer && pl == 0) ? ck_base + (uint32_t)(s * 2) : kOob;
  const uint32_t co_first = (valid && pl == 0 && j == cd - 1) ? first_base + (uint32_t)(s * 2) : kOob;
  const uint32_t co_trace = (p.trace && valid && pl == 0 && j == cd) ? trace_base + (uint32_t)(s * 2) : kOob;
  // re-saves compared against the first-seen value: producers for roles 1..cd-1, player-0 lane
  const uint64_t cmp_lanes = __ballot(valid && pl == 0 && j <= cd - 2);
  // doubled Fletcher weights (fletcher_from_doubled); the frame field and the constant length
  // prefixes go to the player-0 lane
  uint32_t wt[5];
#pragma unroll
  for (int q = 0; q < 5; q++) wt[q] = owner ? 2u * weights_at(n_bytes, fld_offset(P, kq[q])) : 0u;
  const uint32_t one2 = owner ? 0x02020202u : 0u;
  const uint32_t wf1 = pl == 0 ? 0x02020202u : 0u, wf2 = pl == 0 ? 2u * weights_at(n_bytes, 0) : 0u;
  const uint32_t c1 = pl == 0 ? 2u * Fletcher<P>::kSum1Const : 0u;
  const uint32_t c2 = pl == 0 ? 2u * Fletcher<P>::kSum2Const : 0u;

  // the launch checkpoint of this block's sessions (all of them, halted ones included: a restore
  // copies the whole shadow back), before any of this launch's stores
  {
    const CheckpointMap m{L, R, F, spw, p.cur, p.ring, p.ring_ck, p.first_ck};
    checkpoint_sessions(m, p.shadow + blk * p.block_bytes, s0, nsess, wl, kWave);
  }
  if (failed_f0 >= 0) return;  // this launch is replayed from its checkpoint anyway
  const int32_t g0 = p.f0 - cd;
  for (int q = wl; q < cd * nsess; q += kWave) {
    const int gg = q / nsess, ss = q - gg * nsess;
    lds_first[gg * kWave + ss] = p.first_ck[(int64_t)((g0 + gg) % R) * L + s0 + ss];
  }
  {
    const uint32_t* cell = p.ring + (int64_t)(g0 % R) * F * L + sl;
#pragma unroll
    for (int q = 0; q < 5; q++) lds_cell[wl * 5 + q] = cell[kq[q] * L];
  }
  __syncthreads();
  // every role starts from the loaded cell (roles > 0 hold chains of the previous launch, which
  // this launch neither saves nor compares, but they must hold in-domain states)
  uint32_t w[5];
#pragma unroll
  for (int q = 0; q < 5; q++) w[q] = lds_cell[wl * 5 + q];

  uint64_t bad = 0;                 // wave-uniform: some re-save disagreed with its first-seen value
  uint32_t pend_ck = 0, pend_first = 0;
  uint64_t pend_lanes = 0;          // the previous step's comparison, finished one step later
  const int32_t t_end = p.f0 + p.n + cd;
  const int row = nsess * Pp;
  const int in_lane = g * Pp + pl;
  // ring slot of frame t-cd+1 and trace slot of chain t-cd, from the step index rel = t - f0
  // (scalar multiply-high modulo: a loop-carried counter would be widened to a VGPR)
  // (integer division runs on the VALU; readfirstlane brings the uniform results back to SGPRs,
  // otherwise every buffer store using them as soffset would be waterfalled)
  int32_t sr = __builtin_amdgcn_readfirstlane((g0 + 1) % R);
  int32_t st = __builtin_amdgcn_readfirstlane(p.trace_cap ? g0 % p.trace_cap : 0);
  const int32_t tcap = p.trace_cap > 0 ? p.trace_cap : 1;
  const bool corrupt_here = p.corrupt_frame >= p.f0 && p.corrupt_frame < p.f0 + p.n;
  const uint32_t corrupt_on = (corrupt_here && s == p.corrupt_lane && pl == 0 && j == 0) ? 1u : 0u;
  const int32_t ramp_end = min(p.f0 + cd, t_end);
  // the core loop steps through advance_player_lean without the per-step domain test: every role
  // starts from the loaded cell and every later state is an advance of an in-domain state, so one
  // test of the loaded rot suffices (a cell from outside the domain runs every step in the general
  // per-step dispatch instead)
  const bool lean_ok = __all(w[4] <= kTwoPiBits);
  const int32_t core_end = (corrupt_here || !lean_ok) ? ramp_end : max(ramp_end, p.f0 + p.n);

  auto stage = [&](int32_t t) {
    __syncthreads();
    const int32_t gf = t - cd;
    const int nf = (t_end - t) < kStageFrames ? (t_end - t) : kStageFrames;
    stage_input_rows<0>(lds_in, p.inputs, L, Pp, p.cap, gf, nf, s0, row, row, wl);
    __syncthreads();
  };

  uint32_t acc = 0;  // core steps: OR of (re-save ^ first-seen) per lane, masked by cmp_lanes at the end
  const uint32_t in_at = (uint32_t)in_lane;

  // One step t with its input byte.  kCore: every chain is active (t in [f0 + cd, f0 + n)), no
  // injected corruption, states in the lean domain.
  auto step = [&](auto core_tag, int32_t t, uint32_t in) {
    constexpr bool kCore = decltype(core_tag)::value;
    const int32_t rel = t - p.f0;
    const int32_t c = t - j;  // this lane's chain
    const bool active = kCore ? valid : (valid && c >= p.f0 && c < p.f0 + p.n);
    if (!kCore) {
      bad |= __ballot(pend_ck != pend_first) & pend_lanes;
      w[0] ^= (t == p.corrupt_frame) ? corrupt_on : 0u;  // role 0 = chain t's load
    }
    // AdvanceFrame(t - cd) on every lane
    {
      float x = __builtin_bit_cast(float, w[0]), y = __builtin_bit_cast(float, w[1]);
      float vx = __builtin_bit_cast(float, w[2]), vy = __builtin_bit_cast(float, w[3]);
      float rot = __builtin_bit_cast(float, w[4]);
      if constexpr (kCore) advance_player_lean(x, y, vx, vy, rot, in);
      else advance_player(x, y, vx, vy, rot, in);
      w[0] = __builtin_bit_cast(uint32_t, x);
      w[1] = __builtin_bit_cast(uint32_t, y);
      w[2] = __builtin_bit_cast(uint32_t, vx);
      w[3] = __builtin_bit_cast(uint32_t, vy);
      w[4] = __builtin_bit_cast(uint32_t, rot);
    }
    // the previous step's comparison, one advance after its first-seen value was requested
    if (kCore) acc |= pend_ck ^ pend_first;
    const uint32_t frame1 = (uint32_t)(t - cd + 1);
    // rotation for step t+1: role j takes role j-1's state, Pp lanes down (one ds_bpermute per
    // field); role 0 keeps its own
    uint32_t nx[5];
#pragma unroll
    for (int q = 0; q < 5; q++) nx[q] = (uint32_t)__builtin_amdgcn_ds_bpermute(src_rot, (int)w[q]);
    __builtin_amdgcn_sched_barrier(0);  // LDS latency behind the Fletcher sums and the saves
    // Fletcher-16 of the post-advance state (frame t-cd+1): the cell role j+1 saves at step t+1
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
    uint32_t first = (uint32_t)__builtin_amdgcn_ds_bpermute(src_first, (int)ck);
    // the first save of frame t-cd+1 happened in the previous launch while its chain is not ours
    if (!kCore && rel + 1 < cd) first = lds_first[(rel + 1) * kWave + g];
    // SaveGameState(t-cd+1) for role j+1, first-seen, display checksum
    const uint32_t sru = (uint32_t)sr, stu = (uint32_t)st;
    auto stores = [&]() {
      const uint32_t so = sru * slot_bytes, cso = sru * ck_slot_bytes;
#pragma unroll
      for (int q = 0; q < 5; q++) __builtin_amdgcn_raw_buffer_store_b32(w[q], rs_ring, fo[q], so, 0);
      __builtin_amdgcn_raw_buffer_store_b32(frame1, rs_ring, fo_frame, so, 0);
      __builtin_amdgcn_raw_buffer_store_b16((uint16_t)ck, rs_ring, co, cso, 0);
      __builtin_amdgcn_raw_buffer_store_b16((uint16_t)ck, rs_ring, co_first, cso, 0);
      __builtin_amdgcn_raw_buffer_store_b16((uint16_t)ck, rs_ring, co_trace, stu * ck_slot_bytes, 0);
    };
    if (kCore) {
      stores();
      pend_lanes = cmp_lanes;
    } else {
      if (active) stores();
      pend_lanes = cmp_lanes & __ballot(active);
      if (active && j == cd && c == p.f0 + p.n - 1) {  // the launch's last call: current state
        uint32_t* cur = p.cur + s;
        if (owner) {
#pragma unroll
          for (int q = 0; q < 5; q++) cur[kq[q] * L] = w[q];
        }
        if (pl == 0) cur[0] = frame1;
      }
    }
    pend_ck = ck;
    pend_first = first;
#pragma unroll
    for (int q = 0; q < 5; q++) w[q] = nx[q];
    // wave-uniform slot counters (their readfirstlane'd start keeps them in SGPRs: a start value
    // from the VALU's integer division would widen them and waterfall every store using them)
    sr = sr + 1 == R ? 0 : sr + 1;
    st = st + 1 == tcap ? 0 : st + 1;
  };

  auto input_at = [&](int32_t t) -> uint32_t {
    return lds_in[(((t - p.f0) & (kStageFrames - 1)) * row) + in_at];
  };
  int32_t t = p.f0;
  for (; t < ramp_end; ++t) {
    if (((t - p.f0) & (kStageFrames - 1)) == 0) stage(t);
    step(std::false_type(), t, input_at(t));
  }
  if (t < core_end) {
    // the ramp's last comparison is finished here; inside the core every step compares the same
    // static lane set (cmp_lanes), accumulated per lane and tested once after the loop
    bad |= __ballot(pend_ck != pend_first) & pend_lanes;
    pend_ck = pend_first = 0;
    pend_lanes = cmp_lanes;
  }
  while (t < core_end) {
    const int32_t rel = t - p.f0;
    if ((rel & (kStageFrames - 1)) == 0) stage(t);
    const int32_t chunk_end = min(core_end, t + (kStageFrames - (rel & (kStageFrames - 1))));
    // two steps per iteration; each step's input byte is read one step ahead through a pointer
    // that advances a row per step (the read past the chunk's last step lands in the slack row
    // and is discarded)
    uint32_t ip = (uint32_t)((t - p.f0) & (kStageFrames - 1)) * (uint32_t)row + in_at;
    uint32_t in = lds_in[ip];
    for (; t + 1 < chunk_end; t += 2) {
      const uint32_t in1 = lds_in[ip + row];
      step(std::true_type(), t, in);
      ip += 2 * row;
      in = lds_in[ip];
      step(std::true_type(), t + 1, in1);
    }
    if (t < chunk_end) {
      step(std::true_type(), t, in);
      ++t;
    }
  }
  bad |= __ballot(acc != 0) & cmp_lanes;
  for (; t < t_end; ++t) {
    if (((t - p.f0) & (kStageFrames - 1)) == 0) stage(t);
    step(std::false_type(), t, input_at(t));
  }
  bad |= __ballot(pend_ck != pend_first) & pend_lanes;
  if (bad && wl == __builtin_ctzll(bad)) atomicCAS(p.fail_f0, -1, p.f0);
}

// ------------------------------------------------------------------------------------------
// Pipelined SyncTest, v5 (check_distance 8): cd chain roles per session instead of cd + 1, the
// chains' last advance batched.  v4 gives each session K = cd + 1 roles x Pp player lanes; at cd 8
// and two players that is 18 lanes, three sessions per wave (54 of 64 lanes busy) and 1366 waves
// for 4096 sessions -- a third of the SIMDs then run two waves, and one SIMD's two waves take
// ~1.32x one wave's time.  Role cd (the chain's last AdvanceFrame: the new frame, whose checksum
// is the display checksum, ex_game.rs:121-126) is the only role whose result no other role
// consumes, so v5 drops it from the lockstep:
//   * roles 0..cd-1 run exactly as in v4 (same Loads, Saves, comparisons, static store offsets);
//   * role cd-1's post-advance state (the chain's "current" frame, which role cd would advance at
//     the next step) is stashed in LDS, one slot per step;
//   * every 8 steps one batch sub-step advances the 8 stashed states, one per role lane (role j
//     takes the stash of the batch's j-th step), with the input the next step would have read,
//     and stores their display checksums; the launch's last chain also writes the current state.
// 16 lanes per session at cd 8 / two players: four sessions per wave, 1024 waves for 4096
// sessions, one per SIMD; the batch adds about one step's work per 8 steps.
// v5 step kinds: std::false_type the general step (raw input, per-step domain test, stores only for
// the launch's chains), std::true_type the core step, EdgeStep the core step's arithmetic for the
// launch's first and last steps (some roles hold chains of other launches: their stores write the
// same bytes the launch's own chains store at the same step -- every role replays the same frame
// from the same state -- but their comparisons, first-seen sources and display checksums are the
// general step's)
struct EdgeStep : std::true_type {};
template <class T> struct IsEdge : std::false_type {};
template <> struct IsEdge<EdgeStep> : std::true_type {};

template <int P>
__global__ __launch_bounds__(kWave) void synctest_pipelined_v5_kernel(PipeParams p) {
  constexpr int Pp = P <= 1 ? 1 : (P == 2 ? 2 : 4);
  constexpr int F = state_fields(P);
  constexpr int n_bytes = Fletcher<P>::n;
  constexpr int CD = 8;             // check_distance this kernel is built for (the host checks)
  constexpr int G = CD * Pp;        // lanes per session
  constexpr int SPW = kWave / G;    // sessions per wave
  constexpr int ROW = SPW * Pp;     // staged input bytes per frame (= 8)
  constexpr int kB = 8;             // steps per batch (= role lanes that run it)
  constexpr int kEntry = 32;        // stash bytes per (session, player): 5 fields, 16-B aligned
  constexpr int kSlot = 8 * kEntry; // one step's stash (ROW entries)
  // inputs: the raw bytes of up to kRaw frames (the whole launch at n <= kRaw - CD, read in the
  // prologue beside every other global read: one memory latency per launch), and their decoded
  // InputRec for kStage5 frames at a time (+1 slack row for the batch's look-ahead), decoded from
  // LDS every kStage5 steps; the non-core steps read the raw bytes
  constexpr int kStage5 = 128;
  constexpr int kRaw = 528;
  __shared__ __attribute__((aligned(16))) uint8_t lds_raw[kRaw * ROW];
  __shared__ uint4 lds_rec[(kStage5 + 1) * ROW];
  __shared__ uint16_t lds_first[CD * SPW];
  __shared__ __attribute__((aligned(16))) uint8_t lds_stash[2 * kB * kSlot];  // slots, then the dump
  const int wl = threadIdx.x;
  const int R = p.R;
  const int g = wl / G, r = wl - g * G;
  const int j = r / Pp, pl = r - j * Pp;  // static role, player
  const int64_t L = p.L;
  const int64_t blk = xcd_block(blockIdx.x, gridDim.x);
  const int64_t s0 = blk * SPW;
  const int64_t s = s0 + g;
  const int nsess = (int)((L - s0) < SPW ? (L - s0) : SPW);
  const int32_t g0 = p.f0 - CD;
  const int32_t t_stage_end = p.f0 + p.n + CD;  // inputs are staged up to v4's last step
  const int raw_rows = kRaw < p.cap ? kRaw : p.cap;  // a chunk of queue rows is held at once
  // The prologue's global reads, issued together (one memory latency instead of one per phase):
  // the launch checkpoint's rows, the first-seen checksums of frames g0 .. g0 + cd - 1, the cell
  // of frame g0, and the raw input rows; then the early-outs, the checkpoint's stores and the LDS.
  // Fast form for full blocks of 8-byte-aligned input rows; otherwise the generic copies.
  constexpr int kCkRegs = 16;  // checkpoint words per thread in the fast form
  constexpr int kRawRegs = (kRaw + kWave - 1) / kWave;
  const int ck_words32 = (1 + R) * F * SPW, ck_words16 = R * SPW;  // 16-bit rows as word pairs
  const bool fast = nsess == SPW && ((L * Pp) & 7) == 0 && (L & 1) == 0 && ck_words32 + ck_words16 <= kCkRegs * kWave;
  const int32_t failed_f0 = *p.fail_f0;
  const int32_t lstat = p.lane_status[s < L ? s : L - 1];
  uint32_t ckv[kCkRegs];
  uint2 rawv[kRawRegs];
  uint16_t firstv = 0;
  const int nraw = (t_stage_end - p.f0) < raw_rows ? (t_stage_end - p.f0) : raw_rows;
  const int32_t slot_g0 = g0 % R;
  const int32_t q0 = g0 % p.cap;
  if (fast) {
#pragma unroll
    for (int i = 0; i < kCkRegs; i++) {
      const int q = wl + i * kWave;
      if (q < ck_words32) {
        const int row = q / SPW, ss = q % SPW;  // SPW is a power of two: shifts
        ckv[i] = row < F ? p.cur[(int64_t)row * L + s0 + ss] : p.ring[(int64_t)(row - F) * L + s0 + ss];
      } else if (q < ck_words32 + ck_words16) {
        const int e16 = 2 * (q - ck_words32), row = e16 / SPW, ss = e16 % SPW;
        const uint16_t* src = row < R ? p.ring_ck + (int64_t)row * L : p.first_ck + (int64_t)(row - R) * L;
        ckv[i] = *reinterpret_cast<const uint32_t*>(src + s0 + ss);
      }
    }
#pragma unroll
    for (int i = 0; i < kRawRegs; i++) {
      const int ff = wl + i * kWave;
      if (ff < nraw) {
        const int32_t slot = q0 + ff >= p.cap ? q0 + ff - p.cap : q0 + ff;
        rawv[i] = *reinterpret_cast<const uint2*>(p.inputs + ((int64_t)slot * L + s0) * Pp);
      }
    }
  }
  if (wl < CD * nsess) {
    const int gg = wl / nsess, ss = wl - gg * nsess;
    const int32_t sl = slot_g0 + gg >= R ? slot_g0 + gg - R : slot_g0 + gg;
    firstv = p.first_ck[(int64_t)sl * L + s0 + ss];
  }
  const bool valid = s < L && lstat == GGRS_LANE_RUNNING;
  const bool owner = valid && pl < P;
  const int64_t sl = valid ? s : 0;
  const int plc = pl < P ? pl : 0;
  const int base = g * G;
  const int src_first = (base + (CD - 1) * Pp) * 4;
  const int src_rot = (j == 0 ? wl : base + (j - 1) * Pp + pl) * 4;
  const int kq[5] = {fld_x(P, plc), fld_y(P, plc), fld_vx(P, plc), fld_vy(P, plc), fld_rot(P, plc)};
  const uint32_t slot_bytes = (uint32_t)(F * L * 4), ck_slot_bytes = (uint32_t)(L * 2);
  const uint32_t ck_base = (uint32_t)((const uint8_t*)p.ring_ck - (const uint8_t*)p.ring);
  const uint32_t first_base = (uint32_t)((const uint8_t*)p.first_ck - (const uint8_t*)p.ring);
  const uint32_t trace_base = p.trace ? (uint32_t)((const uint8_t*)p.trace - (const uint8_t*)p.ring) : 0u;
  const __amdgpu_buffer_rsrc_t rs_ring = make_rsrc(
      p.ring, p.trace ? trace_base + ck_slot_bytes * (uint32_t)p.trace_cap : first_base + ck_slot_bytes * (uint32_t)R);
  // every role is a producer (v4's roles 0..cd-1)
  uint32_t fo[5];
#pragma unroll
  for (int q = 0; q < 5; q++) fo[q] = owner ? (uint32_t)((kq[q] * L + s) * 4) : kOob;
  const uint32_t fo_frame = (valid && pl == 0) ? (uint32_t)(s * 4) : kOob;
  // checksum stores: the player-0 lane writes ring_ck; with two or more player lanes the player-1
  // lane of role cd-1 writes the same checksum (the DPP combine leaves it on both) into first_ck
  // in the same store instruction -- both at the ring slot's index
  constexpr bool kMergedCk = Pp >= 2;
  const uint32_t co = (valid && pl == 0)                                ? ck_base + (uint32_t)(s * 2)
                      : (kMergedCk && valid && pl == 1 && j == CD - 1) ? first_base + (uint32_t)(s * 2)
                                                                        : kOob;
  const uint32_t co_first = (!kMergedCk && valid && pl == 0 && j == CD - 1) ? first_base + (uint32_t)(s * 2) : kOob;
  const uint64_t cmp_lanes = __ballot(valid && pl == 0 && j <= CD - 2);
  uint32_t wt[5];
#pragma unroll
  for (int q = 0; q < 5; q++) wt[q] = owner ? 2u * weights_at(n_bytes, fld_offset(P, kq[q])) : 0u;
  const uint32_t one2 = owner ? 0x02020202u : 0u;
  const uint32_t wf1 = pl == 0 ? 0x02020202u : 0u, wf2 = pl == 0 ? 2u * weights_at(n_bytes, 0) : 0u;
  const uint32_t c1 = pl == 0 ? 2u * Fletcher<P>::kSum1Const : 0u;
  const uint32_t c2 = pl == 0 ? 2u * Fletcher<P>::kSum2Const : 0u;
  // stash addresses: role cd-1 lanes write their (session, player) entry of the step's slot, every
  // other lane the dump (no exec-mask branch around the write); role j < 8 reads slot j in a batch
  const uint32_t entry = (uint32_t)(g * Pp + pl) * kEntry;
  const uint32_t stash_w = (valid && j == CD - 1) ? entry : (uint32_t)(kB * kSlot);
  const uint32_t stash_r = (uint32_t)(j & (kB - 1)) * kSlot + entry;
  // the batch's display-checksum store: player-0 lanes of roles 0..7, slot added per batch
  const uint32_t co_trace = (p.trace && valid && pl == 0 && j < kB) ? trace_base + (uint32_t)(s * 2) : kOob;
  const int32_t tcap = p.trace_cap > 0 ? p.trace_cap : 1;
  const int32_t jm = j % tcap;

  // the cell of frame g0 (every role's Load): read straight into the lane's registers
  uint32_t w[5];
  {
    const uint32_t* cell = p.ring + (int64_t)slot_g0 * F * L + sl;
#pragma unroll
    for (int q = 0; q < 5; q++) w[q] = cell[kq[q] * L];
  }
  if (failed_f0 >= 0 && failed_f0 != p.f0) return;
  {
    uint8_t* piece = p.shadow + blk * p.block_bytes;
    if (fast) {
#pragma unroll
      for (int i = 0; i < kCkRegs; i++) {
        const int q = wl + i * kWave;
        if (q < ck_words32 + ck_words16) reinterpret_cast<uint32_t*>(piece)[q] = ckv[i];
      }
    } else {
      const CheckpointMap m{L, R, F, SPW, p.cur, p.ring, p.ring_ck, p.first_ck};
      checkpoint_sessions(m, piece, s0, nsess, wl, kWave);
    }
  }
  if (failed_f0 >= 0) return;
  if (wl < CD * nsess) {
    const int gg = wl / nsess, ss = wl - gg * nsess;
    lds_first[gg * SPW + ss] = firstv;
  }
  int32_t raw0 = p.f0;  // step whose frame (raw0 - cd) is lds_raw's row 0
  if (fast) {
#pragma unroll
    for (int i = 0; i < kRawRegs; i++) {
      const int ff = wl + i * kWave;
      if (ff < nraw) reinterpret_cast<uint2*>(lds_raw)[ff] = rawv[i];
    }
  } else {
    stage_input_rows<ROW>(lds_raw, p.inputs, L, Pp, p.cap, g0, nraw, s0, nsess * Pp, ROW, wl);
  }
  // the block is one wave: LDS written by one lane and read by another needs only the wave's own
  // in-order LDS queue and a compiler fence (a __syncthreads would also wait for the checkpoint's
  // stores; inside the step loop, for every ring store in flight)
  auto wave_lds_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  wave_lds_sync();

  uint64_t bad = 0;
  uint32_t pend_ck = 0, pend_first = 0;
  uint64_t pend_lanes = 0;
  const int32_t t_end = t_stage_end - 1;        // the last step role cd-1 works in
  const int in_lane = g * Pp + pl;
  int32_t sr = __builtin_amdgcn_readfirstlane((g0 + 1) % R);
  // trace slot of the current batch's first chain (f0 - (cd-1) + 8m), advanced 8 per batch
  int32_t sb = __builtin_amdgcn_readfirstlane(p.trace_cap ? (p.f0 - (CD - 1)) % p.trace_cap : 0);
  const int32_t sb_step = __builtin_amdgcn_readfirstlane(kB % tcap);
  const bool corrupt_here = p.corrupt_frame >= p.f0 && p.corrupt_frame < p.f0 + p.n;
  const uint32_t corrupt_on = (corrupt_here && s == p.corrupt_lane && pl == 0 && j == 0) ? 1u : 0u;
  const int32_t ramp_end = min(p.f0 + CD, t_end);
  const bool lean_ok = __all(w[4] <= kTwoPiBits);
  const int32_t core_end = (corrupt_here || !lean_ok) ? ramp_end : max(ramp_end, p.f0 + p.n);
  int32_t chunk0 = p.f0;  // step of lds_rec's row 0

  // decode the records of steps t .. t + kStage5 (from lds_raw; a launch longer than the raw chunk
  // re-reads its raw rows first, the only global read inside the step loop)
  auto stage = [&](int32_t t) {
    const int nf = (t_stage_end - t) < kStage5 + 1 ? (t_stage_end - t) : kStage5 + 1;
    if (t - raw0 + nf > raw_rows) {
      wave_lds_sync();
      const int nr = (t_stage_end - t) < raw_rows ? (t_stage_end - t) : raw_rows;
      stage_input_rows<ROW>(lds_raw, p.inputs, L, Pp, p.cap, t - CD, nr, s0, nsess * Pp, ROW, wl);
      raw0 = t;
    }
    wave_lds_sync();
    const uint8_t* src = lds_raw + (t - raw0) * ROW;
    for (int q = wl; q < nf * ROW; q += kWave) {
      const InputRec r = make_input_rec(src[q]);
      lds_rec[q] = make_uint4(r.delta, r.thr, r.sgn, r.keep);
    }
    chunk0 = t;
    wave_lds_sync();
  };

  uint32_t acc = 0;
  const uint32_t in_at = (uint32_t)in_lane;
  // core steps: sin/cos of the rot each lane holds at the step's start, computed one step ahead
  // (inside the previous step, from the rotated rot, before its speed clamp)
  float sc_s = 0.0f, sc_c = 0.0f;  // the raw polynomial values (glibc_sincosf_domain_raw)
  uint32_t sc_qs = 0u, sc_qc = 0u;   // and their quadrant signs

  auto rec_of = [](const uint4 v) { return InputRec{v.x, v.y, v.z, v.w}; };
  // core steps take the staged InputRec, non-core steps the raw input byte
  auto step = [&](auto core_tag, int32_t t, auto in, uint32_t slot_off) {
    constexpr bool kCore = decltype(core_tag)::value;
    constexpr bool kEdge = IsEdge<decltype(core_tag)>::value;
    const int32_t rel = t - p.f0;
    const int32_t c = t - j;
    const bool active = (kCore && !kEdge) ? valid : (valid && c >= p.f0 && c < p.f0 + p.n);
    if (!kCore || kEdge) bad |= __ballot(pend_ck != pend_first) & pend_lanes;
    if (!kCore) w[0] ^= (t == p.corrupt_frame) ? corrupt_on : 0u;
    {
      float x = __builtin_bit_cast(float, w[0]), y = __builtin_bit_cast(float, w[1]);
      float vx = __builtin_bit_cast(float, w[2]), vy = __builtin_bit_cast(float, w[3]);
      float rot = __builtin_bit_cast(float, w[4]);
      if constexpr (kCore) {
        // the next step's rot is this lane's new rot rotated one role up (role 0 keeps its own)
        advance_player_rec_q(x, y, vx, vy, rot, rec_of(in), sc_s, sc_c, sc_qs, sc_qc, [&](float rn) {
          const uint32_t rb = __builtin_bit_cast(uint32_t, rn);
          const uint32_t nb = Pp == 2 ? (uint32_t)__builtin_amdgcn_update_dpp((int)rb, (int)rb, 0x112, 0xF, 0xF, false)
                                      : (uint32_t)__builtin_amdgcn_ds_bpermute(src_rot, (int)rb);
          glibc_sincosf_domain_raw(__builtin_bit_cast(float, nb), &sc_s, &sc_c, &sc_qs, &sc_qc);
        });
      } else {
        advance_player(x, y, vx, vy, rot, (uint32_t)in);
      }
      w[0] = __builtin_bit_cast(uint32_t, x);
      w[1] = __builtin_bit_cast(uint32_t, y);
      w[2] = __builtin_bit_cast(uint32_t, vx);
      w[3] = __builtin_bit_cast(uint32_t, vy);
      w[4] = __builtin_bit_cast(uint32_t, rot);
    }
    if (kCore && !kEdge) acc |= pend_ck ^ pend_first;
    const uint32_t frame1 = (uint32_t)(t - CD + 1);
    // rotation: role j takes role j-1's state, role 0 keeps its own.  At two players a session is
    // one 16-lane DPP row (role j = lanes 2j, 2j+1): one row_shr:2 move per field, the row's first
    // two lanes keep their value (bound_ctrl off); otherwise one ds_bpermute per field.
    // (the DPP moves come after the state's last use below, in place)
    uint32_t nx[5];
    if constexpr (Pp != 2) {
#pragma unroll
      for (int q = 0; q < 5; q++) nx[q] = (uint32_t)__builtin_amdgcn_ds_bpermute(src_rot, (int)w[q]);
    }
    // role cd-1's post-advance state for the batch (every other lane writes the dump)
    {
      uint8_t* st = lds_stash + stash_w + slot_off;
      *reinterpret_cast<uint4*>(st) = make_uint4(w[0], w[1], w[2], w[3]);
      *reinterpret_cast<uint32_t*>(st + 16) = w[4];
    }
    if constexpr (Pp != 2) __builtin_amdgcn_sched_barrier(0);  // LDS latency behind the sums
    uint32_t d1 = dot4_u8(frame1, wf1, c1), d2 = dot4_u8(frame1, wf2, c2);
#pragma unroll
    for (int q = 0; q < 5; q++) {
      d1 = dot4_u8(w[q], one2, d1);
      d2 = dot4_u8(w[q], wt[q], d2);
    }
    if constexpr (Pp >= 2) {
      d1 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d1, 0xB1, 0xF, 0xF, true);
      d2 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d2, 0xB1, 0xF, 0xF, true);
    }
    if constexpr (Pp >= 4) {
      d1 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d1, 0x4E, 0xF, 0xF, true);
      d2 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d2, 0x4E, 0xF, 0xF, true);
    }
    const uint32_t ck = fletcher_from_doubled(d1, d2);
    // role cd-1's first-seen checksum to every lane of the session (two players: DPP
    // row_newbcast of the row's lane 14)
    uint32_t first = Pp == 2 ? (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ck, 0x150 + (CD - 1) * Pp, 0xF, 0xF, true)
                             : (uint32_t)__builtin_amdgcn_ds_bpermute(src_first, (int)ck);
    if ((!kCore || kEdge) && rel + 1 < CD) first = lds_first[(rel + 1) * SPW + g];
    const uint32_t sru = (uint32_t)sr;
    auto stores = [&]() {
      const uint32_t so = sru * slot_bytes, cso = sru * ck_slot_bytes;
#pragma unroll
      for (int q = 0; q < 5; q++) __builtin_amdgcn_raw_buffer_store_b32(w[q], rs_ring, fo[q], so, 0);
      __builtin_amdgcn_raw_buffer_store_b32(frame1, rs_ring, fo_frame, so, 0);
      __builtin_amdgcn_raw_buffer_store_b16((uint16_t)ck, rs_ring, co, cso, 0);
      if constexpr (!kMergedCk) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)ck, rs_ring, co_first, cso, 0);
    };
    if (kCore) {
      stores();
      pend_lanes = kEdge ? cmp_lanes & __ballot(active) : cmp_lanes;
    } else {
      if (active) stores();
      pend_lanes = cmp_lanes & __ballot(active);
    }
    pend_ck = ck;
    pend_first = first;
#pragma unroll
    for (int q = 0; q < 5; q++)
      w[q] = Pp == 2 ? (uint32_t)__builtin_amdgcn_update_dpp((int)w[q], (int)w[q], 0x112, 0xF, 0xF, false) : nx[q];
    sr = sr + 1 == R ? 0 : sr + 1;
  };

  // The batch over the stashes of steps tb .. tb + count - 1 (count <= 8; tb - f0 a multiple of
  // 8): role j < count advances step tb + j's stash -- chain cb = tb + j - (cd - 1), its frame cb,
  // with input cb, which step tb + j + 1 reads -- and stores the display checksum of frame cb + 1.
  auto batch = [&](auto core_tag, int32_t tb, int count) {
    constexpr bool kCore = decltype(core_tag)::value;
    constexpr bool kEdge = IsEdge<decltype(core_tag)>::value;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int32_t cb = tb + j - (CD - 1);
    const bool act = (kCore && !kEdge) ? (valid && j < kB) : (valid && j < count && cb >= p.f0 && cb < p.f0 + p.n);
    uint32_t v[5];
    {
      const uint8_t* st = lds_stash + stash_r;
      const uint4 a = *reinterpret_cast<const uint4*>(st);
      v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w;
      v[4] = *reinterpret_cast<const uint32_t*>(st + 16);
    }
    const uint32_t ri = (uint32_t)(tb + (j & (kB - 1)) + 1 - chunk0) * ROW + in_at;
    const uint32_t rr = (uint32_t)(tb + (j & (kB - 1)) + 1 - raw0) * ROW + in_at;
    {
      float x = __builtin_bit_cast(float, v[0]), y = __builtin_bit_cast(float, v[1]);
      float vx = __builtin_bit_cast(float, v[2]), vy = __builtin_bit_cast(float, v[3]);
      float rot = __builtin_bit_cast(float, v[4]);
      if constexpr (kCore) {
        float bs, bc;
        uint32_t bqs, bqc;
        glibc_sincosf_domain_raw(rot, &bs, &bc, &bqs, &bqc);
        advance_player_rec_q(x, y, vx, vy, rot, rec_of(lds_rec[ri]), bs, bc, bqs, bqc);
      } else {
        advance_player(x, y, vx, vy, rot, lds_raw[rr]);
      }
      v[0] = __builtin_bit_cast(uint32_t, x);
      v[1] = __builtin_bit_cast(uint32_t, y);
      v[2] = __builtin_bit_cast(uint32_t, vx);
      v[3] = __builtin_bit_cast(uint32_t, vy);
      v[4] = __builtin_bit_cast(uint32_t, rot);
    }
    const uint32_t framen = (uint32_t)(cb + 1);
    uint32_t d1 = dot4_u8(framen, wf1, c1), d2 = dot4_u8(framen, wf2, c2);
#pragma unroll
    for (int q = 0; q < 5; q++) {
      d1 = dot4_u8(v[q], one2, d1);
      d2 = dot4_u8(v[q], wt[q], d2);
    }
    if constexpr (Pp >= 2) {
      d1 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d1, 0xB1, 0xF, 0xF, true);
      d2 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d2, 0xB1, 0xF, 0xF, true);
    }
    if constexpr (Pp >= 4) {
      d1 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d1, 0x4E, 0xF, 0xF, true);
      d2 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d2, 0x4E, 0xF, 0xF, true);
    }
    const uint32_t ck = fletcher_from_doubled(d1, d2);
    int32_t ti = sb + jm;
    ti = ti >= tcap ? ti - tcap : ti;
    const uint32_t tro = act ? co_trace + (uint32_t)ti * ck_slot_bytes : kOob;
    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)ck, rs_ring, tro, 0, 0);
    if ((!kCore || kEdge) && act && cb == p.f0 + p.n - 1) {  // the launch's last call: the current state
      uint32_t* cur = p.cur + s;
      if (owner) {
#pragma unroll
        for (int q = 0; q < 5; q++) cur[kq[q] * L] = v[q];
      }
      if (pl == 0) cur[0] = framen;
    }
    sb = sb + sb_step;
    sb = sb >= tcap ? sb - tcap : sb;
  };

  auto input_at = [&](int32_t t) -> uint32_t { return lds_raw[(uint32_t)(t - raw0) * ROW + in_at]; };
  auto general = [&](int32_t t) {
    const int32_t rel = t - p.f0;
    if ((rel & (kStage5 - 1)) == 0) stage(t);
    step(std::false_type(), t, input_at(t), (uint32_t)(rel & (kB - 1)) * kSlot);
    if ((rel & (kB - 1)) == kB - 1) batch(std::false_type(), t - (kB - 1), kB);
  };
  int32_t t = p.f0;
  // lean launches of whole 8-step blocks run their first and last steps as edge steps (the core
  // step's code, already warm in the instruction cache, with the general step's bookkeeping);
  // others take the general step there
  const bool edge_ok = core_end == p.f0 + p.n && (p.n & (kB - 1)) == 0 && p.n >= 2 * kB;
  auto edge_block = [&](int32_t tb, int count) {
    if (((tb - p.f0) & (kStage5 - 1)) == 0 || tb + count + 1 > chunk0 + kStage5 + 1) stage(tb);
    const uint32_t ip = (uint32_t)(tb - chunk0) * ROW + in_at;
    uint4 in[kB];
#pragma unroll
    for (int u = 0; u < kB; u++) in[u] = lds_rec[ip + u * ROW];
#pragma unroll
    for (int u = 0; u < kB; u++)
      if (u < count) step(EdgeStep(), tb + u, in[u], (uint32_t)(u * kSlot));
    batch(EdgeStep(), tb, count);
  };
  if (edge_ok) {
    glibc_sincosf_domain_raw(__builtin_bit_cast(float, w[4]), &sc_s, &sc_c, &sc_qs, &sc_qc);
    edge_block(t, kB);
    t += kB;
  } else {
    for (; t < ramp_end; ++t) general(t);
    // core blocks of 8 steps + their batch, aligned to the batch grid
    for (; t < core_end && ((t - p.f0) & (kB - 1)) != 0; ++t) general(t);
  }
  if (t + kB <= core_end) {
    bad |= __ballot(pend_ck != pend_first) & pend_lanes;
    pend_ck = pend_first = 0;
    pend_lanes = cmp_lanes;
    glibc_sincosf_domain_raw(__builtin_bit_cast(float, w[4]), &sc_s, &sc_c, &sc_qs, &sc_qc);
    for (; t + kB <= core_end; t += kB) {
      if (((t - p.f0) & (kStage5 - 1)) == 0) stage(t);
      const uint32_t ip = (uint32_t)(t - chunk0) * ROW + in_at;
      uint4 in[kB];
#pragma unroll
      for (int u = 0; u < kB; u++) in[u] = lds_rec[ip + u * ROW];
#pragma unroll
      for (int u = 0; u < kB; u++) step(std::true_type(), t + u, in[u], (uint32_t)(u * kSlot));
      batch(std::true_type(), t, kB);
    }
    bad |= __ballot(acc != 0) & cmp_lanes;
  }
  if (edge_ok) {
    edge_block(t, t_end - t);  // the last cd - 1 steps and their batch
  } else {
    for (; t < t_end; ++t) general(t);
    const int rem = (t_end - p.f0) & (kB - 1);
    if (rem) batch(std::false_type(), t_end - rem, rem);
  }
  bad |= __ballot(pend_ck != pend_first) & pend_lanes;
  if (bad && wl == __builtin_ctzll(bad)) atomicCAS(p.fail_f0, -1, p.f0);
}

struct RequestParams {
  int64_t L;
  int32_t R, n_reqs, trace_cap;
  const int32_t* reqs;        // [n_reqs][2] kind, frame
  const uint8_t* inputs;      // [n_adv][L][Pp]
  const uint8_t* status;      // [n_adv][L][Pp] or null
  uint32_t* cur;
  uint32_t* ring;
  uint16_t* ring_ck;
  uint16_t* trace;
};

// Game::handle_requests (ex_game.rs:79-99) for one ordered request list on every lane.
template <int P>
__global__ __launch_bounds__(kWave) void requests_kernel(RequestParams p) {
  const int64_t lane = (int64_t)blockIdx.x * kWave + threadIdx.x;
  if (lane >= p.L) return;
  const int64_t L = p.L;
  BoxState<P> s;
  load_state<P>(s, p.cur + lane, L);
  int64_t adv = 0;
  for (int32_t r = 0; r < p.n_reqs; ++r) {
    const int32_t kind = p.reqs[2 * r], frame = p.reqs[2 * r + 1];
    const int32_t slot = frame % p.R;
    if (kind == GGRS_REQ_LOAD) {
      load_state<P>(s, p.ring + (int64_t)slot * state_fields(P) * L + lane, L);
    } else if (kind == GGRS_REQ_SAVE) {
      store_state<P>(s, p.ring + (int64_t)slot * state_fields(P) * L + lane, L);
      p.ring_ck[(int64_t)slot * L + lane] = fletcher16_state<P>(s);
    } else {
      const int64_t idx = adv * L + lane;
      uint32_t disc = 0;
      if (p.status) {
        const uint32_t st = load_inputs<P>(p.status, idx);
#pragma unroll
        for (int i = 0; i < P; i++)
          if (((st >> (8 * i)) & 0xffu) == GGRS_STATUS_DISCONNECTED) disc |= 1u << i;
      }
      advance_state<P>(s, load_inputs<P>(p.inputs, idx), disc);
      if (p.trace) p.trace[(int64_t)((int32_t)s.w[0] - 1) % p.trace_cap * L + lane] = fletcher16_state<P>(s);
      ++adv;
    }
  }
  store_state<P>(s, p.cur + lane, L);
}

}  // namespace

// ------------------------------------------------------------------------------ engine object
// (struct ggrs_engine and launch_timed live in engine.h, shared with requests.hip)
namespace {

int ensure_staging(ggrs_engine* e, size_t bytes) {
  if (bytes <= e->staging_bytes) return GGRS_OK;
  if (e->staging) HIP_TRY(hipFree(e->staging));
  e->staging = nullptr;
  e->staging_bytes = 0;
  HIP_TRY(hipMalloc(&e->staging, bytes));
  e->staging_bytes = bytes;
  return GGRS_OK;
}

// The pipelined SyncTest kernels' geometry: sessions per 64-lane block, or 0 when a session does
// not fit one wavefront or a buffer the kernel's descriptors address would exceed kOob (then the
// sequential kernel runs).  v4: K = cd + 1 chain roles x Pp player lanes per session; v5 (cd 8
// only): cd roles, the chains' last advance batched.
bool pipe_buffers_fit(const ggrs_engine* e) {
  const uint64_t L = (uint64_t)e->cfg.num_lanes;
  const uint64_t ring_span = (uint64_t)((const uint8_t*)e->first_ck - (const uint8_t*)e->ring) + 2 * L * e->R;
  const uint64_t trace_span =
      e->trace ? (uint64_t)((const uint8_t*)e->trace - (const uint8_t*)e->ring) + 2 * L * e->cfg.trace_capacity : 0;
  return (uint64_t)e->F * 4 * L * e->R < kOob && ring_span < kOob && trace_span < kOob;
}

int v4_sessions_per_block(const ggrs_engine* e) {
  const int K = e->cfg.check_distance + 1;
  if (e->cfg.check_distance < 2 || K * e->Pp > kWave || !pipe_buffers_fit(e)) return 0;
  return kWave / (K * e->Pp);
}

int v5_sessions_per_block(const ggrs_engine* e) {
  if (e->cfg.check_distance != 8 || !pipe_buffers_fit(e)) return 0;
  return kWave / (8 * e->Pp);
}

// Which pipelined kernel a launch takes (4, 5, or 0 = sequential only).  The default picks v5
// where it packs more sessions into a wave than v4 (cd 8: 4 vs 3 sessions at two players, 2 vs 1
// at four).
int pipe_kernel(const ggrs_engine* e) {
  const int s4 = v4_sessions_per_block(e), s5 = v5_sessions_per_block(e);
  switch (e->path) {
    case GGRS_PATH_SEQUENTIAL: return 0;
    case GGRS_PATH_PIPELINED_CHAINS: return s4 > 0 ? 4 : 0;
    case GGRS_PATH_PIPELINED_BATCHED: return s5 > 0 ? 5 : (s4 > 0 ? 4 : 0);
    default: return s5 > s4 ? 5 : (s4 > 0 ? 4 : 0);
  }
}

int pipe_sessions_per_block(const ggrs_engine* e) {
  const int k = pipe_kernel(e);
  return k == 5 ? v5_sessions_per_block(e) : (k == 4 ? v4_sessions_per_block(e) : 0);
}

}  // namespace

extern "C" {

int32_t ggrs_abi_version(void) { return GGRS_ABI_VERSION; }

const char* ggrs_last_error(void) { return g_last_error.c_str(); }

int ggrs_engine_destroy(ggrs_engine_t* e) {
  if (!e) return GGRS_OK;
  (void)hipSetDevice(e->cfg.device);
  (void)lane_server_stop(e);
  lane_server_release(e);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  void* bufs[] = {e->arena, e->shadow, e->fail_f0, e->inputs, e->lane_status,
                  e->mis_frame, e->mis_mask, e->staging};  // trace lives in the arena allocation
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (e->host_staging) (void)hipHostFree(e->host_staging);
  if (e->batch.base) (void)hipHostFree(e->batch.base);
  if (e->server.mem) (void)hipHostFree(e->server.mem);
  if (e->server.dev) (void)hipFree(e->server.dev);
  if (e->ev_begin) (void)hipEventDestroy(e->ev_begin);
  if (e->ev_end) (void)hipEventDestroy(e->ev_end);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
  return GGRS_OK;
}

int ggrs_engine_create(const ggrs_config_t* cfg, ggrs_engine_t** out) {
  if (!cfg || !out) return set_error(GGRS_E_INVALID, "null argument");
  *out = nullptr;
  const ggrs_config_t c = *cfg;
  if (c.num_lanes < 1) return set_error(GGRS_E_INVALID, "num_lanes must be >= 1");
  if (c.num_players < 1 || c.num_players > 4)
    return set_error(GGRS_E_INVALID, "num_players must be in 1..4 (ex_game.rs:70)");
  if (c.max_prediction < 1 || c.max_prediction > 63)
    return set_error(GGRS_E_INVALID, "max_prediction must be in 1..63");
  if (c.check_distance < 0 || c.check_distance >= c.max_prediction)
    return set_error(GGRS_E_INVALID, "Check distance too big. (check_distance must be < max_prediction)");
  if (c.input_delay < 0 || c.input_delay > 1024) return set_error(GGRS_E_INVALID, "bad input_delay");
  if (c.input_capacity < 0 || c.trace_capacity < 0) return set_error(GGRS_E_INVALID, "negative capacity");
  ggrs_engine* e = new ggrs_engine();
  e->cfg = c;
  e->Pp = padded_players(c.num_players);
  e->F = state_fields(c.num_players);
  e->R = c.max_prediction + 1;
  e->cap = c.input_capacity ? c.input_capacity : 128;
  if (e->cap < c.input_delay + c.check_distance + 2) {
    delete e;
    return set_error(GGRS_E_INVALID, "input_capacity must be >= input_delay + check_distance + 2");
  }
  e->ring_tag.assign(e->R, GGRS_NULL_FRAME);
  e->cfg.input_capacity = e->cap;
  auto fail = [&](int rc) {
    std::string msg = g_last_error;
    ggrs_engine_destroy(e);
    g_last_error = msg;
    return rc;
  };
#define CTRY(expr)                                                                      \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) return fail(set_error(GGRS_E_HIP, "%s: %s", #expr, hipGetErrorString(e_))); \
  } while (0)
  const int64_t L = c.num_lanes;
  CTRY(hipSetDevice(c.device));
  CTRY(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
  CTRY(hipEventCreate(&e->ev_begin));
  CTRY(hipEventCreate(&e->ev_end));
  {
    auto up16 = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t b_cur = up16(sizeof(uint32_t) * e->F * L);
    const size_t b_ring = up16(sizeof(uint32_t) * (size_t)e->R * e->F * L);
    const size_t b_ck = up16(sizeof(uint16_t) * (size_t)e->R * L);
    e->arena_bytes = b_cur + b_ring + 2 * b_ck;
    // the display-checksum trace follows the arena in the same allocation: the v4 kernel's stores
    // then all go through one buffer descriptor
    const size_t b_trace = c.trace_capacity > 0 ? up16(sizeof(uint16_t) * (size_t)c.trace_capacity * L) : 0;
    CTRY(hipMalloc(&e->arena, e->arena_bytes + b_trace));
    if (b_trace) e->trace = (uint16_t*)(e->arena + e->arena_bytes);
    CTRY(hipMemsetAsync(e->arena, 0, e->arena_bytes, e->stream));
    e->cur = (uint32_t*)e->arena;
    e->ring = (uint32_t*)(e->arena + b_cur);
    e->ring_ck = (uint16_t*)(e->arena + b_cur + b_ring);
    e->first_ck = (uint16_t*)(e->arena + b_cur + b_ring + b_ck);
    // every ring cell starts as GameState::default's NULL_FRAME (frame_info.rs:16-23): the frame
    // field is the cell's tag for per-lane request lists (requests.hip)
    for (int s = 0; s < e->R; s++)
      CTRY(hipMemsetD32Async((hipDeviceptr_t)(e->ring + (size_t)s * e->F * L), (int)GGRS_NULL_FRAME, (size_t)L,
                             e->stream));
    // the pipelined kernel's launch checkpoint: one contiguous piece per 64-lane block
    size_t shadow = 0;
    for (int spw : {v4_sessions_per_block(e), v5_sessions_per_block(e)})
      if (spw > 0)
        shadow = std::max(shadow, (size_t)grid_of(L, spw) * (size_t)checkpoint_block_bytes(e->R, e->F, spw));
    if (shadow > 0) {
      e->shadow_bytes = shadow;
      CTRY(hipMalloc(&e->shadow, e->shadow_bytes));
      CTRY(hipMemsetAsync(e->shadow, 0, e->shadow_bytes, e->stream));
    }
  }
  CTRY(hipMalloc(&e->fail_f0, sizeof(int32_t)));
  CTRY(hipMemsetAsync(e->fail_f0, 0xff, sizeof(int32_t), e->stream));
  CTRY(hipMalloc(&e->inputs, (size_t)e->cap * L * e->Pp));
  CTRY(hipMalloc(&e->lane_status, sizeof(int32_t) * L));
  CTRY(hipMalloc(&e->mis_frame, sizeof(int32_t) * L));
  CTRY(hipMalloc(&e->mis_mask, sizeof(uint64_t) * L));
  // default input (Input::default(), inp = 0) for every queue frame, covering frames < delay
  CTRY(hipMemsetAsync(e->inputs, 0, (size_t)e->cap * L * e->Pp, e->stream));
  CTRY(hipMemsetAsync(e->lane_status, 0, sizeof(int32_t) * L, e->stream));
  CTRY(hipMemsetAsync(e->mis_frame, 0xff, sizeof(int32_t) * L, e->stream));
  CTRY(hipMemsetAsync(e->mis_mask, 0, sizeof(uint64_t) * L, e->stream));
  if (e->trace) CTRY(hipMemsetAsync(e->trace, 0, sizeof(uint16_t) * (size_t)c.trace_capacity * L, e->stream));
  const int64_t grid = grid_of(L, 256);
  switch (c.num_players) {
    case 1: init_states_kernel<1><<<grid, 256, 0, e->stream>>>(e->cur, L); break;
    case 2: init_states_kernel<2><<<grid, 256, 0, e->stream>>>(e->cur, L); break;
    case 3: init_states_kernel<3><<<grid, 256, 0, e->stream>>>(e->cur, L); break;
    default: init_states_kernel<4><<<grid, 256, 0, e->stream>>>(e->cur, L); break;
  }
  CTRY(hipGetLastError());
  CTRY(hipStreamSynchronize(e->stream));
#undef CTRY
  *out = e;
  return GGRS_OK;
}

int ggrs_engine_config(const ggrs_engine_t* e, ggrs_config_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  *out = e->cfg;
  return GGRS_OK;
}

static int resolve(ggrs_engine_t* e);

static int add_inputs_common(ggrs_engine_t* e, int32_t first_frame, int32_t n, const void* src,
                             bool device) {
  if (!e || (!src && n > 0)) return set_error(GGRS_E_INVALID, "null argument");
  if (n < 0) return set_error(GGRS_E_INVALID, "n_frames must be >= 0");
  if (first_frame != e->next_user_frame)
    return set_error(GGRS_E_INVALID,
                     "inputs must be added sequentially (expected frame %d, got %d; input_queue.rs:171-177)",
                     e->next_user_frame, first_frame);
  if (n == 0) return GGRS_OK;
  { int rc_ = resolve(e); if (rc_) return rc_; }  // oldest needed input is then current - cd
  const int32_t delay = e->cfg.input_delay;
  // oldest queue frame a later call still reads: the rollback start current - cd
  const int64_t oldest_needed = (int64_t)e->current_frame - e->cfg.check_distance;
  const int64_t newest = (int64_t)first_frame + n - 1 + delay;
  if (newest - oldest_needed >= e->cap)
    return set_error(GGRS_E_INVALID,
                     "input queue full: frames up to %lld would overwrite frame %lld still needed (capacity %d)",
                     (long long)newest, (long long)oldest_needed, e->cap);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t L = e->cfg.num_lanes;
  const int P = e->cfg.num_players;
  const size_t bytes = (size_t)n * L * P;
  const uint8_t* dsrc = (const uint8_t*)src;
  if (!device) {
    int rc = ensure_staging(e, bytes);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(e->staging, src, bytes, hipMemcpyHostToDevice, e->stream));
    dsrc = e->staging;
  }
  const int64_t total = (int64_t)n * L;
  pack_inputs_kernel<<<grid_of(total, 256), 256, 0, e->stream>>>(dsrc, e->inputs, L, P, e->Pp, n,
                                                                 (first_frame + delay) % e->cap, e->cap);
  HIP_TRY(hipGetLastError());
  if (!device) HIP_TRY(hipStreamSynchronize(e->stream));  // staging is reused by the next call
  e->next_user_frame = first_frame + n;
  return GGRS_OK;
}

int ggrs_add_local_inputs(ggrs_engine_t* e, int32_t first_frame, int32_t n, const uint8_t* inputs) {
  return add_inputs_common(e, first_frame, n, inputs, false);
}

int ggrs_add_local_inputs_device(ggrs_engine_t* e, int32_t first_frame, int32_t n, const void* inputs) {
  return add_inputs_common(e, first_frame, n, inputs, true);
}

static int launch_sequential(ggrs_engine_t* e, int32_t f0, int32_t n) {
  SyncTestParams p;
  p.L = e->cfg.num_lanes;
  p.R = e->R;
  p.cd = e->cfg.check_distance;
  p.f0 = f0;
  p.n = n;
  p.cap = e->cap;
  p.trace_cap = e->cfg.trace_capacity;
  p.corrupt_lane = e->corrupt_lane;
  p.corrupt_frame = e->corrupt_frame;
  p.cur = e->cur;
  p.ring = e->ring;
  p.ring_ck = e->ring_ck;
  p.first_ck = e->first_ck;
  p.inputs = e->inputs;
  p.lane_status = e->lane_status;
  p.mis_frame = e->mis_frame;
  p.mis_mask = e->mis_mask;
  p.trace = e->trace;
  const int64_t grid = grid_of(p.L, kWave);
  return launch_timed(e, [&] {
    switch (e->cfg.num_players) {
      case 1: synctest_kernel<1><<<grid, kWave, 0, e->stream>>>(p); break;
      case 2: synctest_kernel<2><<<grid, kWave, 0, e->stream>>>(p); break;
      case 3: synctest_kernel<3><<<grid, kWave, 0, e->stream>>>(p); break;
      default: synctest_kernel<4><<<grid, kWave, 0, e->stream>>>(p); break;
    }
  });
}

static int launch_pipelined(ggrs_engine_t* e, int32_t f0, int32_t n) {
  PipeParams p;
  p.L = e->cfg.num_lanes;
  p.R = e->R;
  p.cd = e->cfg.check_distance;
  const int kernel = pipe_kernel(e);
  p.K = kernel == 5 ? p.cd : p.cd + 1;
  p.spw = pipe_sessions_per_block(e);
  p.f0 = f0;
  p.n = n;
  p.cap = e->cap;
  p.trace_cap = e->cfg.trace_capacity;
  p.corrupt_lane = e->corrupt_lane;
  p.corrupt_frame = e->corrupt_frame;
  p.cur = e->cur;
  p.ring = e->ring;
  p.ring_ck = e->ring_ck;
  p.first_ck = e->first_ck;
  p.inputs = e->inputs;
  p.lane_status = e->lane_status;
  p.fail_f0 = e->fail_f0;
  p.trace = e->trace;
  p.shadow = e->shadow;
  p.block_bytes = checkpoint_block_bytes(p.R, e->F, p.spw);
  e->unverified = true;
  const int64_t grid = grid_of(p.L, p.spw);
  return launch_timed(e, [&] {
    if (kernel == 5) {
      switch (e->cfg.num_players) {
        case 1: synctest_pipelined_v5_kernel<1><<<grid, kWave, 0, e->stream>>>(p); break;
        case 2: synctest_pipelined_v5_kernel<2><<<grid, kWave, 0, e->stream>>>(p); break;
        case 3: synctest_pipelined_v5_kernel<3><<<grid, kWave, 0, e->stream>>>(p); break;
        default: synctest_pipelined_v5_kernel<4><<<grid, kWave, 0, e->stream>>>(p); break;
      }
      return;
    }
    switch (e->cfg.num_players) {
      case 1: synctest_pipelined_v4_kernel<1><<<grid, kWave, 0, e->stream>>>(p); break;
      case 2: synctest_pipelined_v4_kernel<2><<<grid, kWave, 0, e->stream>>>(p); break;
      case 3: synctest_pipelined_v4_kernel<3><<<grid, kWave, 0, e->stream>>>(p); break;
      default: synctest_pipelined_v4_kernel<4><<<grid, kWave, 0, e->stream>>>(p); break;
    }
  });
}

// Settle pipelined launches: if one of them saw a checksum mismatch, roll every lane back to the
// checkpoint taken before it and replay the frames since with the sequential kernel, which halts
// lanes exactly where the reference returns MismatchedChecksum.
static int resolve(ggrs_engine_t* e) {
  if (int rc = lane_server_stop(e)) return rc;
  if (!e->unverified) return GGRS_OK;
  HIP_TRY(hipSetDevice(e->cfg.device));
  int32_t f = -1;
  HIP_TRY(hipMemcpyAsync(&f, e->fail_f0, sizeof f, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->unverified = false;
  if (f < 0) return GGRS_OK;
  const int spw = pipe_sessions_per_block(e);
  const CheckpointMap m{(int64_t)e->cfg.num_lanes, e->R, e->F, spw, e->cur, e->ring, e->ring_ck, e->first_ck};
  restore_kernel<<<grid_of(e->cfg.num_lanes, spw), 256, 0, e->stream>>>(m, e->shadow,
                                                                         checkpoint_block_bytes(e->R, e->F, spw));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemsetAsync(e->fail_f0, 0xff, sizeof(int32_t), e->stream));
  int rc = launch_sequential(e, f, e->current_frame - f);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

int ggrs_synctest_advance_frames(ggrs_engine_t* e, int32_t n) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (n < 0) return set_error(GGRS_E_INVALID, "n_frames must be >= 0");
  if (e->mode == kModeLockstepRequests || e->mode == kModeLaneRequests)
    return set_error(GGRS_E_STATE, "engine already driven by request lists");
  if (n == 0) return GGRS_OK;
  // every frame run needs its (delayed) input queued: SyncTestSession requires input for all
  // players before advance_frame ("Missing local input", sync_test_session.rs:110-114)
  const int64_t last_needed_user = (int64_t)e->current_frame + n - 1 - e->cfg.input_delay;
  if (last_needed_user >= e->next_user_frame)
    return set_error(GGRS_E_INVALID,
                     "Missing local input while calling advance_frame(): frame %lld not added",
                     (long long)last_needed_user);
  e->mode = kModeSyncTest;
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int32_t cd = e->cfg.check_distance;
  int32_t f0 = e->current_frame, left = n;
  // warm-up calls (f <= cd: no rollback yet), cd <= 1 and sessions that do not fit the pipelined
  // kernel take the sequential kernel
  if (pipe_kernel(e) == 0) {
    int rc = launch_sequential(e, f0, left);
    if (rc) return rc;
    left = 0;
  } else if (f0 <= cd) {
    const int32_t m = std::min(left, cd + 1 - f0);
    int rc = launch_sequential(e, f0, m);
    if (rc) return rc;
    f0 += m;
    left -= m;
  }
  if (left > 0) {
    int rc = launch_pipelined(e, f0, left);
    if (rc) return rc;
  }
  // lane-uniform bookkeeping: after call f the ring holds, in slot s, the newest frame <= f
  // congruent to s (every frame 0..f has been saved; cd == 0 saves nothing)
  e->current_frame += n;
  if (cd > 0)
    for (int s = 0; s < e->R; s++) {
      int32_t last = e->current_frame - 1;
      int32_t fr = last - (((last - s) % e->R) + e->R) % e->R;
      e->ring_tag[s] = fr >= 0 ? fr : GGRS_NULL_FRAME;
    }
  return GGRS_OK;
}

int ggrs_set_synctest_path(ggrs_engine_t* e, int32_t path) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (path != GGRS_PATH_PIPELINED && path != GGRS_PATH_SEQUENTIAL && path != GGRS_PATH_PIPELINED_CHAINS &&
      path != GGRS_PATH_PIPELINED_BATCHED)
    return set_error(GGRS_E_INVALID, "unknown path %d", path);
  int rc = resolve(e);
  if (rc) return rc;
  e->path = path;
  return GGRS_OK;
}

int ggrs_handle_requests(ggrs_engine_t* e, const ggrs_request_t* reqs, int32_t n_reqs,
                         const uint8_t* inputs, const uint8_t* status) {
  if (!e || (!reqs && n_reqs > 0)) return set_error(GGRS_E_INVALID, "null argument");
  if (e->mode == kModeSyncTest) return set_error(GGRS_E_STATE, "engine already driven by ggrs_synctest_advance_frames");
  if (e->mode == kModeLaneRequests) return set_error(GGRS_E_STATE, "engine already driven by per-lane request lists");
  if (n_reqs <= 0) return GGRS_OK;
  // validate the whole list against the lane-uniform cell bookkeeping before touching the device
  std::vector<int32_t> tags = e->ring_tag;
  int32_t frame = e->current_frame;
  int32_t n_adv = 0;
  for (int32_t r = 0; r < n_reqs; r++) {
    const int32_t k = reqs[r].kind, f = reqs[r].frame;
    if (k == GGRS_REQ_SAVE) {
      if (f == GGRS_NULL_FRAME) return set_error(GGRS_E_PRECONDITION, "request %d: save of NULL_FRAME (sync_layer.rs:20)", r);
      if (f != frame) return set_error(GGRS_E_PRECONDITION, "request %d: save frame %d != state frame %d (ex_game.rs:104)", r, f, frame);
      tags[f % e->R] = f;
    } else if (k == GGRS_REQ_LOAD) {
      if (f < 0 || tags[f % e->R] != f)
        return set_error(GGRS_E_PRECONDITION, "request %d: no saved state for frame %d (sync_layer.rs:248, ex_game.rs:112)", r, f);
      frame = f;
    } else if (k == GGRS_REQ_ADVANCE) {
      frame += 1;
      n_adv++;
    } else {
      return set_error(GGRS_E_INVALID, "request %d: unknown kind %d", r, k);
    }
  }
  if (n_adv > 0 && !inputs) return set_error(GGRS_E_INVALID, "inputs required for AdvanceFrame requests");
  if (e->trace && n_adv > e->cfg.trace_capacity) return set_error(GGRS_E_INVALID, "more advances than trace_capacity");
  e->mode = kModeLockstepRequests;
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t L = e->cfg.num_lanes;
  const int P = e->cfg.num_players, Pp = e->Pp;
  const size_t req_bytes = sizeof(int32_t) * 2 * n_reqs;
  const size_t in_bytes = (size_t)n_adv * L * Pp;
  const size_t raw_bytes = (size_t)n_adv * L * P;
  // one host-to-device copy from pinned memory: [request list | raw inputs | raw status]; the
  // raw [n][L][P] rows are the kernel's [n][L][Pp] layout already when P == Pp (1, 2, 4 players)
  const size_t req_pad = (req_bytes + 15) & ~(size_t)15, raw_pad = (raw_bytes + 15) & ~(size_t)15;
  const size_t up_bytes = req_pad + 2 * raw_pad;
  const size_t total = up_bytes + 2 * in_bytes + 64;
  int rc = ensure_staging(e, total);
  if (rc) return rc;
  if (up_bytes > e->host_staging_bytes) {
    if (e->host_staging) HIP_TRY(hipHostFree(e->host_staging));
    e->host_staging = nullptr;
    e->host_staging_bytes = 0;
    HIP_TRY(hipHostMalloc((void**)&e->host_staging, up_bytes, hipHostMallocDefault));
    e->host_staging_bytes = up_bytes;
  }
  uint8_t* h = e->host_staging;
  int32_t* flat = reinterpret_cast<int32_t*>(h);
  for (int32_t r = 0; r < n_reqs; r++) {
    flat[2 * r] = reqs[r].kind;
    flat[2 * r + 1] = reqs[r].frame;
  }
  if (n_adv > 0) std::memcpy(h + req_pad, inputs, raw_bytes);
  if (n_adv > 0 && status) std::memcpy(h + req_pad + raw_pad, status, raw_bytes);
  uint8_t* d_reqs = e->staging;
  uint8_t* d_raw = d_reqs + req_pad;
  uint8_t* d_in = d_raw + 2 * raw_pad;
  uint8_t* d_st = d_in + in_bytes;
  HIP_TRY(hipMemcpyAsync(d_reqs, h, req_pad + (n_adv > 0 ? (status ? 2 * raw_pad : raw_bytes) : 0),
                         hipMemcpyHostToDevice, e->stream));
  if (n_adv > 0) {
    if (P == Pp) {
      d_in = d_raw;
      d_st = d_raw + raw_pad;
    } else {
      pack_inputs_kernel<<<grid_of((int64_t)n_adv * L, 256), 256, 0, e->stream>>>(d_raw, d_in, L, P, Pp, n_adv, 0, n_adv);
      HIP_TRY(hipGetLastError());
      if (status) {
        pack_inputs_kernel<<<grid_of((int64_t)n_adv * L, 256), 256, 0, e->stream>>>(d_raw + raw_pad, d_st, L, P, Pp, n_adv, 0, n_adv);
        HIP_TRY(hipGetLastError());
      }
    }
  }
  RequestParams p;
  p.L = L;
  p.R = e->R;
  p.n_reqs = n_reqs;
  p.trace_cap = e->cfg.trace_capacity;
  p.reqs = (const int32_t*)d_reqs;
  p.inputs = d_in;
  p.status = status ? d_st : nullptr;
  p.cur = e->cur;
  p.ring = e->ring;
  p.ring_ck = e->ring_ck;
  p.trace = e->trace;
  const int64_t grid = grid_of(L, kWave);
  rc = launch_timed(e, [&] {
    switch (P) {
      case 1: requests_kernel<1><<<grid, kWave, 0, e->stream>>>(p); break;
      case 2: requests_kernel<2><<<grid, kWave, 0, e->stream>>>(p); break;
      case 3: requests_kernel<3><<<grid, kWave, 0, e->stream>>>(p); break;
      default: requests_kernel<4><<<grid, kWave, 0, e->stream>>>(p); break;
    }
  });
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(e->stream));  // staging reuse
  e->ring_tag = tags;
  e->current_frame = frame;
  return GGRS_OK;
}

int ggrs_synchronize(ggrs_engine_t* e) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  { int rc_ = resolve(e); if (rc_) return rc_; }
  HIP_TRY(hipSetDevice(e->cfg.device));
  // an idle lane server is done with its work: stop it (it restarts with the next batch) instead of
  // waiting out its idle watchdog
  if (int rc = lane_server_stop(e)) return rc;
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

int ggrs_current_frame(const ggrs_engine_t* e, int32_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  if (e->mode == kModeLaneRequests)
    return set_error(GGRS_E_STATE, "per-lane request lists: every lane has its own frame (ggrs_read_lane_frames)");
  *out = e->current_frame;
  return GGRS_OK;
}

int ggrs_read_mismatches(ggrs_engine_t* e, int32_t* st, int32_t* mf, uint64_t* mm) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  { int rc_ = resolve(e); if (rc_) return rc_; }
  HIP_TRY(hipSetDevice(e->cfg.device));
  const size_t L = e->cfg.num_lanes;
  if (st) HIP_TRY(hipMemcpyAsync(st, e->lane_status, 4 * L, hipMemcpyDeviceToHost, e->stream));
  if (mf) HIP_TRY(hipMemcpyAsync(mf, e->mis_frame, 4 * L, hipMemcpyDeviceToHost, e->stream));
  if (mm) HIP_TRY(hipMemcpyAsync(mm, e->mis_mask, 8 * L, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

int ggrs_read_save_checksums(ggrs_engine_t* e, int32_t frame, uint16_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  { int rc_ = resolve(e); if (rc_) return rc_; }
  if (e->mode == kModeLaneRequests)
    return set_error(GGRS_E_STATE, "per-lane request lists return their save checksums from each call");
  if (frame < 0 || e->ring_tag[frame % e->R] != frame)
    return set_error(GGRS_E_PRECONDITION, "no saved cell for frame %d", frame);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const size_t L = e->cfg.num_lanes;
  HIP_TRY(hipMemcpyAsync(out, e->ring_ck + (size_t)(frame % e->R) * L, 2 * L, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

int ggrs_read_save_checksums_frames(ggrs_engine_t* e, const int32_t* frames, int32_t n, uint16_t* out) {
  if (!e || (n > 0 && (!frames || !out)) || n < 0) return set_error(GGRS_E_INVALID, "null argument or negative count");
  { int rc_ = resolve(e); if (rc_) return rc_; }
  if (e->mode == kModeLaneRequests)
    return set_error(GGRS_E_STATE, "per-lane request lists return their save checksums from each call");
  for (int32_t k = 0; k < n; k++)
    if (frames[k] < 0 || e->ring_tag[frames[k] % e->R] != frames[k])
      return set_error(GGRS_E_PRECONDITION, "no saved cell for frame %d", frames[k]);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const size_t L = e->cfg.num_lanes;
  for (int32_t k = 0; k < n; k++)
    HIP_TRY(hipMemcpyAsync(out + (size_t)k * L, e->ring_ck + (size_t)(frames[k] % e->R) * L, 2 * L,
                           hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

static int gather_lane(ggrs_engine_t* e, const uint32_t* base, int32_t lane, uint32_t* w) {
  const size_t L = e->cfg.num_lanes;
  for (int k = 0; k < e->F; k++)
    HIP_TRY(hipMemcpyAsync(&w[k], base + (size_t)k * L + lane, 4, hipMemcpyDeviceToHost, e->stream));
  return GGRS_OK;
}

int ggrs_read_state(ggrs_engine_t* e, int32_t lane, uint8_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  { int rc_ = resolve(e); if (rc_) return rc_; }
  if (lane < 0 || lane >= e->cfg.num_lanes) return set_error(GGRS_E_INVALID, "lane out of range");
  HIP_TRY(hipSetDevice(e->cfg.device));
  uint32_t w[32];
  int rc = gather_lane(e, e->cur, lane, w);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(e->stream));
  serialize_state_bytes(w, e->cfg.num_players, out);
  return GGRS_OK;
}

int ggrs_read_states(ggrs_engine_t* e, uint8_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  { int rc_ = resolve(e); if (rc_) return rc_; }
  HIP_TRY(hipSetDevice(e->cfg.device));
  const size_t L = e->cfg.num_lanes;
  const int sb = bincode_bytes(e->cfg.num_players);
  std::vector<uint32_t> soa((size_t)e->F * L);  // word k of every lane, one copy
  HIP_TRY(hipMemcpyAsync(soa.data(), e->cur, soa.size() * 4, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  uint32_t w[32];
  for (size_t l = 0; l < L; l++) {
    for (int k = 0; k < e->F; k++) w[k] = soa[(size_t)k * L + l];
    serialize_state_bytes(w, e->cfg.num_players, out + l * sb);
  }
  return GGRS_OK;
}

int ggrs_read_ring(ggrs_engine_t* e, int32_t lane, int32_t* frames, uint16_t* cks, uint8_t* states) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  { int rc_ = resolve(e); if (rc_) return rc_; }
  if (lane < 0 || lane >= e->cfg.num_lanes) return set_error(GGRS_E_INVALID, "lane out of range");
  HIP_TRY(hipSetDevice(e->cfg.device));
  const size_t L = e->cfg.num_lanes;
  const int sb = bincode_bytes(e->cfg.num_players);
  std::vector<uint32_t> w((size_t)e->R * e->F);
  std::vector<uint16_t> c(e->R);
  for (int s = 0; s < e->R; s++) {
    int rc = gather_lane(e, e->ring + (size_t)s * e->F * L, lane, &w[(size_t)s * e->F]);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(&c[s], e->ring_ck + (size_t)s * L + lane, 2, hipMemcpyDeviceToHost, e->stream));
  }
  HIP_TRY(hipStreamSynchronize(e->stream));
  for (int s = 0; s < e->R; s++) {
    // per-lane request lists: a lane's cell tags are the frame fields of its own ring cells
    const int32_t tag = e->mode == kModeLaneRequests ? (int32_t)w[(size_t)s * e->F] : e->ring_tag[s];
    const bool has = tag != GGRS_NULL_FRAME;
    if (frames) frames[s] = tag;
    if (cks) cks[s] = has ? c[s] : 0;
    if (states) {
      if (has) serialize_state_bytes(&w[(size_t)s * e->F], e->cfg.num_players, states + (size_t)s * sb);
      else memset(states + (size_t)s * sb, 0, sb);
    }
  }
  return GGRS_OK;
}

int ggrs_read_trace(ggrs_engine_t* e, int32_t first_frame, int32_t n, uint16_t* out) {
  if (!e || (!out && n > 0)) return set_error(GGRS_E_INVALID, "null argument");
  { int rc_ = resolve(e); if (rc_) return rc_; }
  if (!e->trace) return set_error(GGRS_E_STATE, "engine created with trace_capacity = 0");
  const int32_t T = e->cfg.trace_capacity;
  if (n < 0 || first_frame < 0 || first_frame + n > e->current_frame || first_frame < e->current_frame - T)
    return set_error(GGRS_E_INVALID, "trace frames [%d, %d) not held (current %d, capacity %d)", first_frame,
                     first_frame + n, e->current_frame, T);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const size_t L = e->cfg.num_lanes;
  for (int32_t i = 0; i < n; i++)
    HIP_TRY(hipMemcpyAsync(out + (size_t)i * L, e->trace + (size_t)((first_frame + i) % T) * L, 2 * L,
                           hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

int ggrs_debug_corrupt_on_load(ggrs_engine_t* e, int32_t lane, int32_t frame) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  e->corrupt_lane = lane;
  e->corrupt_frame = frame;
  return GGRS_OK;
}

int ggrs_last_launch_ms(ggrs_engine_t* e, float* ms) {
  if (!e || !ms) return set_error(GGRS_E_INVALID, "null argument");
  if (e->last_span_launches <= 0) return set_error(GGRS_E_STATE, "no timed span with a fused launch yet");
  *ms = e->last_span_ms / (float)e->last_span_launches;
  return GGRS_OK;
}

int ggrs_timing_reset(ggrs_engine_t* e) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  if (int rc = lane_server_stop(e)) return rc;
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->collecting = true;
  e->span_open = false;
  e->span_stopped = false;
  e->span_launches = 0;
  return GGRS_OK;
}

int ggrs_timing_stop(ggrs_engine_t* e) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  if (int rc = lane_server_stop(e)) return rc;
  if (e->span_open && !e->span_stopped) {
    HIP_TRY(hipEventRecord(e->ev_end, e->stream));
    e->span_stopped = true;
  }
  e->collecting = false;
  return GGRS_OK;
}

int ggrs_timing_read(ggrs_engine_t* e, float* total_ms, int32_t* launches) {
  if (!e || !total_ms || !launches) return set_error(GGRS_E_INVALID, "null argument");
  HIP_TRY(hipSetDevice(e->cfg.device));
  if (int rc = lane_server_stop(e)) return rc;
  float ms = 0.0f;
  if (e->span_open) {
    if (!e->span_stopped) HIP_TRY(hipEventRecord(e->ev_end, e->stream));
    HIP_TRY(hipEventSynchronize(e->ev_end));
    HIP_TRY(hipEventElapsedTime(&ms, e->ev_begin, e->ev_end));
  } else {
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  *total_ms = ms;
  *launches = e->span_launches;
  e->last_span_ms = ms;
  e->last_span_launches = e->span_launches;
  e->collecting = false;
  e->span_open = false;
  e->span_stopped = false;
  e->span_launches = 0;
  return GGRS_OK;
}

}  // extern "C"
