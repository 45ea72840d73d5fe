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
// One thread per session.  Per stage of K calls: the input rows are staged in LDS, a control pass
// takes every decision of the stage's calls (poll, disconnect events, confirmed frame, rollback and
// its depth, check_last_saved_state, the threshold, the saves' frames, errors) without the game
// state, call by call, and writes one record per call; then the step loop replays and advances, each
// lane its own step sequence (an iteration is one AdvanceFrame -- a replayed frame or the call's own
// -- or a call that does not advance).  With one block per CU the control pass of stage i + 1 runs
// on a second wave beside stage i's step loop.
//
// Per-session device state (between launches, HBM):
//   cur   [F][S] u32        the game state after the last call (the handler's State)
//   ring  [S][R][C] u32     saved cells (p2p.hip's session-major layout), ring_frame [R][S] their frames
//   lq    [WL][S] u32       the local players' InputQueues: their input of frame q in slot q % WL
//                           (WL >= max_prediction + input_delay + 2); the remote players' inputs are
//                           read from the input rows themselves (row g = frame g), whose slots carry
//                           the frame they hold (row_tag), so a remote input no longer queued is an
//                           error rather than a stale byte
//   sst   [fields][S] i32   SyncLayer current/last_confirmed/last_saved frames, disconnect_frame,
//                           the newest delivered remote frame, local players' last queued frame,
//                           skipped calls, the session's error, the disconnected mask, and per
//                           player last_frame (local_connect_status); the remote InputQueues'
//                           prediction state is implied (the canonical form, in the kernel)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "common.h"
#include "p2p_engine.h"

#pragma clang fp contract(off)

using namespace ggrs;

namespace {

constexpr int32_t kNull = GGRS_NULL_FRAME;
constexpr int kQ = 128;  // INPUT_QUEUE_LENGTH (input_queue.rs:6)
constexpr int kBlock = 64;

enum : int { kCur = 0, kLconf, kDframe, kLastSaved, kDelivered, kLocalLast, kSkips, kErr, kDisc, kLastSent, kRmask, kLastCk, kPl0 };
constexpr int kPlFields = 1;  // per player: last_frame (local_connect_status; remote players)
// then the peers' disconnect reports: [reporter r][player k] the last frame r's endpoint reports
// (valid where bit 4r + k of kRmask is set)
__host__ __device__ constexpr int sched_rep0(int P) { return kPl0 + kPlFields * P; }
__host__ __device__ constexpr int sched_fields(int P) { return sched_rep0(P) + P * P; }
constexpr uint32_t kEvPeerReport = 0x10u;  // an events byte's flag: the call carries a peer report
__host__ __device__ constexpr int cell_dwords_s(int p) { return (state_fields(p) + 1 + 3) & ~3; }

struct SchedParams {
  int64_t S;
  int32_t R, delay, cap, maxp, c0, n, predictor, sparse;
  int32_t K, B, WL;  // calls per stage, rows kept behind a stage's first call, local-queue frames (2^k)
  int32_t TW;        // the time-aligned form's table frames (2^k)
  uint32_t local_mask;
  uint32_t* cur;
  uint32_t* ring;
  int32_t* ring_frame;
  const uint8_t* inputs;
  const int32_t* row_tag;
  const int32_t* arrive;
  const uint8_t* events;
  const int32_t* reports;  // [cap][S] peers' disconnect reports (GGRS_PEER_REPORT), NULL when none were added
  uint32_t* lq;  // [WL][S] the local players' queued inputs by frame (slot frame % WL)
  int32_t* sst;
  int32_t* rollbacks;
  int64_t* resim;
  // desync detection (interval > 0): per call c (row c % cap) and session the checksum report sent
  // (frame, NULL_FRAME for none; its checksum), last_confirmed_frame when the call compared, and the
  // local players' last queued frame after it; fck [HF][S] the checksum of every frame's final cell
  // (slot frame & (HF - 1)), from which a report's checksum is read after the launch
  int32_t interval, HF;
  int32_t* rep_frame;
  uint16_t* rep_ck;
  int32_t* rep_lconf;
  int32_t* rep_ll;
  uint16_t* fck;
  // the display trace (trace_cap > 0): per call c (row c % trace_cap) and session the checksum of the
  // state after the call's last AdvanceFrame -- a replayed frame or its own -- as the handler keeps
  // it (ex_game.rs:115-127), the previous call's when it advanced nothing
  uint16_t* trace;
  int32_t trace_cap;
};

// The block's LDS (dynamic): its 64 sessions' rings [R][PC][64] uint4 (+ frame tags [R][64] with
// sparse saving; without it every frame 0 .. last save has been saved, so a cell's frame is the
// newest one <= the last save in its slot), local queues [WL][64], and per stage of K calls the
// calls' records [K][64] (u32, sparse saving u64) and the input rows [B + K][64] of frames / calls
// [stage start - B, stage end) with their row tags.
struct SchedLds {
  uint32_t o_tags, o_lq, o_arr, o_rowtag, o_rows, total;  // byte offsets (32-bit: scalar registers are scarce)
  uint32_t rec_b, rowtag_b, rows_b;                       // bytes of one stage buffer of each
};
__host__ __device__ inline uint32_t align16(uint32_t x) { return (x + 15) & ~15u; }
__host__ __device__ inline int input_word_bytes(int P) { return P <= 1 ? 1 : (P == 2 ? 2 : 4); }
// nbuf: stage buffers (records, row tags, rows): 2 when the control pass of stage i + 1 runs on a
// second wave beside stage i's step loop
__host__ __device__ inline SchedLds sched_lds(int P, int R, int sparse, int WL, int K, int B, int nbuf = 1) {
  SchedLds l;
  const uint32_t ring = (uint32_t)R * (cell_dwords_s(P) / 4) * kBlock * 16;
  l.o_tags = ring;
  l.o_lq = align16(l.o_tags + (sparse ? (uint32_t)R * kBlock * 4 : 0u));
  l.o_arr = align16(l.o_lq + (uint32_t)WL * kBlock * input_word_bytes(P));
  l.rec_b = align16((uint32_t)K * kBlock * (sparse ? 8 : 4));  // the calls' records
  l.o_rowtag = l.o_arr + (uint32_t)nbuf * l.rec_b;
  l.rowtag_b = align16((uint32_t)(K + B) * 4);
  l.o_rows = l.o_rowtag + (uint32_t)nbuf * l.rowtag_b;
  l.rows_b = align16((uint32_t)(K + B) * kBlock * input_word_bytes(P));
  l.total = l.o_rows + (uint32_t)nbuf * l.rows_b;
  return l;
}
constexpr int kArrTooFar = 0xfe;  // a burst of >= 254 frames: past the device queue (GGRS_E_PRECONDITION)


// A call's record, written by the control pass and read by the step loop (bits):
//   0-6 d1: replay depth of the rollback (0: none) | 7 adv: the own frame advances | 8-9 stop |
//   10 save_own (sparse saving) | 16-23 code: remote frames delivered | 24-27 Event::Disconnected
// and with sparse saving a second word: 0-6 d2: depth of check_last_saved_state's replay |
//   8-14 s1, 16-22 s2: 1 + the replayed frame saved (h == confirmed) in replay 1 / 2, 0 none.
// stop: where the session stops at this call with its error (the reference panics there, or an input
// row it needs is no longer held): 1 before the call's work, 2 after the first frame's save, 3 after
// the first replay.
enum : uint32_t { kStopNone = 0, kStopBefore = 1, kStopAfterSave0 = 2, kStopAfterReplay1 = 3 };

// The dynamic LDS of both scheduled kernels (regions addressed by byte offset at each use:
// pointer variables into dynamic LDS captured by lambdas become generic pointers, which this hipcc
// miscompiles)
extern __shared__ __attribute__((aligned(16))) uint8_t sched_lds_base[];

// One session's control state (SyncLayer / InputQueue / connect status), advanced call by call by
// the control pass; the step loops keep their own copies of what the inputs of a frame depend on.
template <int P>
struct SchedCtl {
  int32_t cur, lconf, dframe, last_saved, delivered, local_last, skips, err;
  int32_t last_sent;  // last_sent_checksum_frame (desync detection, p2p_session.rs:939-975)
  uint32_t disc;
  uint32_t rmask;  // the peers' standing disconnect reports (bit 4 r + k: r's endpoint reports k)
  int32_t lf[P];  // the remote players' last frames (local_connect_status[k].last_frame): the newest
                  // delivered frame for a connected player, frozen at its disconnect
  int32_t slot_f;  // ring slot of the current frame
  int32_t rollbacks;
  int64_t resim;
};

// What a call of the control pass reads besides the session's state: the stage's staged rows
// (LDS byte offsets of this stage's row tags and rows, `ns` sessions per row), the input ring, the
// sparse cell tags.
struct SchedCtlEnv {
  int32_t lo, maxp, R, delay, cap;
  int32_t interval;  // desync detection interval (0: off)
  int64_t S, s;
  uint32_t lmask, lbytes, rbytes;
  uint32_t o_rowtag, o_rows, o_tags;
  int ns, col;  // sessions per LDS row and this session's column
  const uint8_t* inputs;
  const int32_t* row_tag;
  const int32_t* reports;  // the peers' reports ([cap][S]) and the session's table of them (sst)
  int32_t* rtab;
};

// The control pass's fast form of call c (see sched_control_call): every player connected, no
// disconnect pending, the stage's rows staged and held (the change mask cm), nothing the reference
// would panic at.  Returns whether the call takes it; only then are q and rec updated (by selects:
// no branch).
template <int P, int kPred, bool kFeat = true>
__device__ __forceinline__ bool sched_fast_call(SchedCtl<P>& q, const SchedCtlEnv& x, uint64_t cm, int32_t c,
                                                int32_t a_c, uint32_t e_c, uint32_t& rec, int32_t& rep,
                                                bool en = true) {
  const int32_t lo = x.lo, maxp = x.maxp;
  const uint32_t lbytes = x.lbytes, rbytes = x.rbytes;
  const int32_t a = a_c;
  const int32_t up = max(a, q.delivered);
  const int32_t last = min(up, q.cur - 1);
  // the burst's simulated frames (delivered, last]: bits lo_b .. hi_b of the change mask
  const int lo_b = (q.delivered - lo + 1) & 63, hi_b = (last - lo) & 63;
  const uint64_t win = (last - lo >= 63 ? ~0ull : (2ull << hi_b) - 1) & ~((1ull << lo_b) - 1);
  const uint64_t hit = last > q.delivered ? cm & win : 0ull;
  const int32_t mis = hit ? lo + (int32_t)__builtin_ctzll(hit) : kNull;
  // (bitwise: every test evaluated, no branch per test)
  // check_checksum_send_interval (p2p_session.rs:939-975), before the call's rollback: the report of
  // frame_to_send once it is confirmed and saved; its cell must still be in the ring (else the
  // reference panics: the general form stops the session)
  const int32_t fts = q.last_sent == kNull ? x.interval : q.last_sent + x.interval;
  const bool send = kFeat && x.interval > 0 && fts <= q.lconf && fts <= q.last_saved;
  const bool fast = en & (maxp > 0) & (a <= c) & (q.disc == 0u) & (!kFeat || q.rmask == 0u) & (e_c == 0u) & (q.dframe == kNull) &
                    (q.cur >= 1) & (q.cur >= lo) &
                    (q.delivered >= (kPred == 0 ? lo : lo - 1)) & (lbytes == 0u || q.local_last != kNull) &
                    (up - q.delivered < kArrTooFar) & (up < q.cur - maxp + kQ - 1) & (mis == kNull || mis >= q.cur - maxp) &
                    (!send || fts >= q.last_saved - maxp);
  const int32_t code = up - q.delivered;
  int32_t confirmed = INT32_MAX;  // confirmed_frame (:542-553), every player connected
  if (lbytes) confirmed = q.local_last;
  if (rbytes) confirmed = min(confirmed, up);
  // adjust_gamestate from the first misprediction (its replay's saves end below the current frame's,
  // which becomes the last save)
  const bool rb = mis != kNull;
  const uint32_t d = rb ? (uint32_t)(q.cur - mis) : 0u;
  const int32_t lc = min(confirmed, q.cur);  // set_last_confirmed_frame
  const int32_t ll = (lbytes && q.cur + x.delay == q.local_last + 1) ? q.cur + x.delay : q.local_last;  // add_local_input
  // the prediction threshold (:393-423): frames_ahead is current_frame while nothing is confirmed
  // (PredictDefault lets a session with nothing delivered take this form)
  const bool adv = (lc == kNull ? q.cur : q.cur - lc) < maxp;
  const int32_t nslot = q.slot_f + 1 == x.R ? 0 : q.slot_f + 1;
  if (fast) {
    rep = send ? fts : kNull;
    q.last_sent = send ? fts : q.last_sent;
    q.delivered = up;
#pragma unroll
    for (int k = 0; k < P; k++)
      if ((rbytes >> (8 * k)) & 1u) q.lf[k] = up;
    q.rollbacks += rb ? 1 : 0;
    q.resim += d;
    q.local_last = ll;
    q.lconf = lc;
    q.last_saved = q.cur;
    q.slot_f = adv ? nslot : q.slot_f;
    q.cur = adv ? q.cur + 1 : q.cur;
    q.skips += adv ? 0 : 1;
    rec = d | (adv ? 1u << 7 : 0u) | 1u << 10 | (uint32_t)code << 16;
  }
  return fast;
}

// P2PSession::advance_frame's decisions for call c (p2p_session.rs:265-426) without the game state:
// updates `q` and returns the call's record (word 0; word 1 with sparse saving, see below).
// a_c: the newest remote frame this call's poll delivered; e_c: its Event::Disconnected bits;
// mask_ok / cm: the fast form's precondition and change mask over the stage's rows.
// kFeat false: an engine without desync detection or peer reports (the host's choice: no report is
// sent, none received, q.rmask stays 0), their code compiled out
template <int P, bool kSparse, int kPred, bool kFeat = true>
__device__ __forceinline__ uint2 sched_control_call(SchedCtl<P>& q, const SchedCtlEnv& x, bool mask_ok, uint64_t cm,
                                                    int32_t c, int32_t a_c, uint32_t e_c, int32_t& rep) {
  using T = typename InputWord<P>::T;
  const int32_t lo = x.lo, maxp = x.maxp, R = x.R;
  const uint32_t lmask = x.lmask, lbytes = x.lbytes, rbytes = x.rbytes;
  auto next_slot = [&](int32_t v) { return v + 1 == R ? 0 : v + 1; };
  auto back_slot = [&](int32_t v, int32_t d) { const int32_t y = v - d; return y < 0 ? y + R : y; };
  // a row's frame tag: staged, or (older than the stage's window: a session far behind its calls)
  // from the input ring
  auto row_ok = [&](int32_t g) -> bool {
    return g >= lo ? reinterpret_cast<const int32_t*>(sched_lds_base + x.o_rowtag)[g - lo] == g
                   : x.row_tag[g % x.cap] == g;
  };
  auto row = [&](int32_t g) -> uint32_t {
    if (g >= lo) return (uint32_t)reinterpret_cast<const T*>(sched_lds_base + x.o_rows)[(g - lo) * x.ns + x.col];
    return load_inputs<P>(x.inputs, (int64_t)(g % x.cap) * x.S + x.s);
  };
  auto tag = [&](int32_t slot) -> int32_t& {
    return reinterpret_cast<int32_t*>(sched_lds_base + x.o_tags)[slot * x.ns + x.col];
  };
  // the remote InputQueues in canonical form (the kernel comment): the prediction from frame d
  auto base_of = [&](int32_t d, uint32_t cb) -> uint32_t { return (kPred == 0 && d != kNull) ? row(d) & cb : 0u; };
  // the rows [a, b] all held (a replay's confirmed inputs)
  auto rows_ok = [&](int32_t a, int32_t b) -> bool {
    bool ok = true;
    for (int32_t g = a; g <= b; ++g) ok &= row_ok(g);
    return ok;
  };
  // load_frame's asserts (sync_layer.rs:218-241) and, with sparse saving, cell.frame == frame_to_load
  auto replay_ok = [&](int32_t from) -> bool {
    if (from == kNull || from >= q.cur || from < q.cur - maxp) return false;
    return !kSparse || tag(back_slot(q.slot_f, q.cur - from)) == from;
  };

  uint32_t rec = 0, rec2 = 0, stop = kStopNone;
  // Fast form: a lane with every player connected, no disconnect pending, its rows staged, and
  // nothing in this call that the reference would panic at -- the common call, branch-free.
  bool fast = false;
  rep = kNull;
  if (mask_ok && !q.err) fast = sched_fast_call<P, kPred, kFeat>(q, x, cm, c, a_c, e_c, rec, rep);
  if (fast) {
  } else if (q.err) {
    stop = kStopBefore;
  } else {
    // 1. poll_remote_clients: the burst of remote frames (delivered, up] for the remote players
    //    still connected (handle_event Event::Input, p2p_session.rs:880-895)
    const int32_t code = a_c > c ? -1 : (a_c > q.delivered ? min(a_c - q.delivered, kArrTooFar) : 0);
    uint32_t cb = rbytes;  // bytes of the remote players still connected
#pragma unroll
    for (int k = 0; k < P; k++)
      if ((q.disc >> k) & 1u) cb &= ~(0xffu << (8 * k));
    const int32_t up = q.delivered + code;
    bool bad = false;
    if (code < 0) {  // a frame after its call: the remote peer cannot have sent it yet
      q.err = GGRS_E_INVALID;
    } else if (code == kArrTooFar || up >= q.cur - maxp + kQ - 1) {
      // the reference's InputQueue holds 128 inputs (input_queue.rs:6) and panics past them; the
      // device keeps the same bound on how far the remote inputs may run ahead of the session
      q.err = GGRS_E_PRECONDITION;
    } else {
      // add_input_by_frame's first_incorrect_frame: the first frame of the burst the session has
      // simulated whose inputs differ from the prediction (the canonical form)
      int32_t mis = kNull;
      if (cb) {
        if (kPred == 0 && q.delivered != kNull) bad |= !row_ok(q.delivered);
        const uint32_t pb = base_of(q.delivered, cb);
        const int32_t last = min(up, q.cur - 1);
        for (int32_t g = q.delivered + 1; g <= last; ++g) {
          bad |= !row_ok(g);
          if ((row(g) & cb) != pb) {
            mis = g;
            break;
          }
        }
      }
      if (bad) {
        q.err = GGRS_E_PRECONDITION;  // a remote input no longer in the input rows
        goto call_done;
      }
      q.delivered = up;
#pragma unroll
      for (int k = 0; k < P; k++)
        if ((cb >> (8 * k)) & 1u) q.lf[k] = up;
      // Event::Disconnected (p2p_session.rs:866-878 -> disconnect_player_at_frame :618-655)
      const uint32_t ev = e_c & ((1u << P) - 1u);
#pragma unroll
      for (int k = 0; k < P; k++) {
        if (!((ev >> k) & 1u) || ((lmask >> k) & 1u) || ((q.disc >> k) & 1u)) continue;
        q.disc |= 1u << k;
        cb &= ~(0xffu << (8 * k));
        if (q.cur > q.lf[k]) q.dframe = q.lf[k] + 1;
      }
      // update_player_disconnects (p2p_session.rs:748-783) over the peers' reports (the call's new
      // one joins the session's table): for each player k, the endpoints still running that report k
      // disconnected bound queue_min_confirmed (the others are taken to have seen every reported
      // frame), with the local last frame while k is connected here; then disconnect_player_at_frame
      // (:618-655) while k is connected here or its local last frame is newer -- on every call that
      // holds, as the reference (local_connect_status[k].last_frame stays)
      uint32_t rdisc = 0;
      if (kFeat && (e_c & kEvPeerReport)) {
        const int32_t v = x.reports[(int64_t)(c % x.cap) * x.S + x.s];
        const int k = v & 3, r = (v >> 2) & 3;
        int32_t& t = x.rtab[(int64_t)(r * P + k) * x.S + x.s];
        // (the endpoint keeps the newest last_frame of every message, protocol.rs:576-584)
        t = ((q.rmask >> (4 * r + k)) & 1u) ? max(t, (v >> 5) - 1) : (v >> 5) - 1;
        q.rmask |= 1u << (4 * r + k);
      }
      if (kFeat && q.rmask) {
        for (int k = 0; k < P; k++) {
          bool reported = false;
          int32_t qmin = INT32_MAX;
          for (int r = 0; r < P; r++) {
            if (!((q.rmask >> (4 * r + k)) & 1u) || ((q.disc >> r) & 1u)) continue;  // (!endpoint.is_running())
            reported = true;
            qmin = min(qmin, x.rtab[(int64_t)(r * P + k) * x.S + x.s]);
          }
          if (!reported) continue;
          const bool here = !((q.disc >> k) & 1u);
          if (here) qmin = min(qmin, q.lf[k]);
          if (here || q.lf[k] > qmin) {
            rdisc |= here ? 1u << k : 0u;
            q.disc |= 1u << k;
            cb &= ~(0xffu << (8 * k));
            if (q.cur > qmin) q.dframe = qmin + 1;
          }
        }
      }
      if (kPred == 0 && q.delivered != kNull) bad |= !row_ok(q.delivered);  // the prediction's row
      rec = (uint32_t)code << 16 | (ev | rdisc) << 24;
      // check_checksum_send_interval (p2p_session.rs:939-975): after the poll, before the rollback
      const int32_t fts = q.last_sent == kNull ? x.interval : q.last_sent + x.interval;
      if (kFeat && !bad && x.interval > 0 && fts <= q.lconf && fts <= q.last_saved) {
        if (fts < q.last_saved - maxp) {
          q.err = GGRS_E_PRECONDITION;  // "cell not found!" (:951-954): the reference panics
          goto call_done;
        }
        q.last_sent = fts;
        rep = fts;
      }
      if (bad) {
        q.err = GGRS_E_PRECONDITION;  // a remote input no longer in the input rows
      } else {
        // 2. the first frame's save (:305-308; lockstep mode, max_prediction 0, never saves)
        const bool lockstep = maxp == 0;
        if (q.cur == 0 && !lockstep) {
          q.last_saved = 0;
          if (kSparse) tag(q.slot_f) = 0;
        }
        // confirmed_frame (:542-553): the newest frame every connected player has sent
        int32_t confirmed = INT32_MAX;
#pragma unroll
        for (int k = 0; k < P; k++) {
          if ((q.disc >> k) & 1u) continue;
          confirmed = min(confirmed, ((lmask >> k) & 1u) ? q.local_last : q.lf[k]);
        }
        stop = kStopAfterSave0;
        if (confirmed == INT32_MAX) {  // assert!(confirmed < i32::MAX)
          q.err = GGRS_E_PRECONDITION;
        } else {
          // 3. check_simulation_consistency(disconnect_frame) (sync_layer.rs:343-353) +
          //    adjust_gamestate (p2p_session.rs:658-714)
          //    (not in lockstep mode: no rollback)
          int32_t first_inc = lockstep ? kNull : q.dframe;
          if (!lockstep && mis != kNull && (first_inc == kNull || mis < first_inc)) first_inc = mis;
          if (first_inc != kNull) {
            const int32_t from = kSparse ? q.last_saved : first_inc;
            // the replay reads every read player's InputQueue from `from`, which the last
            // set_last_confirmed_frame trimmed to last_confirmed - 1 (input_queue.rs:83-101): older is
            // the reference's "requested frame no longer exists" panic (:104-110) -- a peer's report
            // of an old frame; a misprediction or a local disconnect is never behind it
            // (sparse saving: adjust_gamestate's assert!(frame_to_load <= first_incorrect), :675 --
            // again a report's rollback behind the last save)
            if (!replay_ok(from) || (kSparse && from > first_inc) || (q.lconf > 0 && from < q.lconf - 1) ||
                !rows_ok(from, min(q.cur - 1, q.delivered))) {
              q.err = GGRS_E_PRECONDITION;
            } else {
              const int32_t d = q.cur - from;
              rec |= (uint32_t)d;
              q.rollbacks += 1;
              q.resim += d;
              q.dframe = kNull;
              // the replay's saves (:692-702)
              if (kSparse) {
                if (confirmed >= from && confirmed < q.cur) {
                  rec2 |= (uint32_t)(confirmed - from + 1) << 8;
                  q.last_saved = confirmed;
                  tag(back_slot(q.slot_f, q.cur - confirmed)) = confirmed;
                }
              } else if (d >= 2) {
                q.last_saved = q.cur - 1;
              }
            }
          }
          bool save_own = !kSparse && !lockstep;
          // sparse saving: check_last_saved_state (:819-843) once the rollback's replay is done
          if (!q.err && kSparse && q.cur - q.last_saved >= maxp) {
            if (confirmed >= q.cur) {
              save_own = true;
            } else if (!replay_ok(q.last_saved)) {
              q.err = GGRS_E_PRECONDITION;
              stop = kStopAfterReplay1;
            } else if (!rows_ok(q.last_saved, min(q.cur - 1, q.delivered))) {
              q.err = GGRS_E_PRECONDITION;
            } else {
              const int32_t d2 = q.cur - q.last_saved;
              rec2 |= (uint32_t)d2;
              q.rollbacks += 1;
              q.resim += d2;
              if (confirmed >= q.last_saved && confirmed < q.cur) {
                rec2 |= (uint32_t)(confirmed - q.last_saved + 1) << 16;
                tag(back_slot(q.slot_f, q.cur - confirmed)) = confirmed;
                q.last_saved = confirmed;
              }
            }
          }
          if (!q.err) {
            // set_last_confirmed_frame (sync_layer.rs:313-340), after this call's saves
            int32_t lc = confirmed;
            const int32_t ls = save_own ? q.cur : q.last_saved;
            if (kSparse && ls < lc) lc = ls;
            if (q.cur < lc) lc = q.cur;
            // add_local_input for every local player (:362-377, input_queue.rs:170-186): queue
            // frame current + delay, dropped unless it is the next one
            int32_t ll = q.local_last;
            if (lbytes) {
              const int32_t qf = q.cur + x.delay;
              if (q.local_last == kNull || qf == q.local_last + 1) ll = qf;
            }
            // the prediction threshold (:393-423); lockstep mode: advance only at last_confirmed ==
            // current (:393-397)
            const int32_t ahead = lc == kNull ? q.cur : q.cur - lc;
            const bool adv = lockstep ? lc == q.cur : ahead < maxp;
            if ((lbytes && !row_ok(c)) || (adv && q.cur <= q.delivered && !row_ok(q.cur))) {
              q.err = GGRS_E_PRECONDITION;
            } else {
              q.lconf = lc;
              q.local_last = ll;
              if (save_own) {
                q.last_saved = q.cur;
                if (kSparse) tag(q.slot_f) = q.cur;
              }
              rec |= (adv ? 1u << 7 : 0u) | (save_own ? 1u << 10 : 0u);
              if (adv) {
                ++q.cur;
                q.slot_f = next_slot(q.slot_f);
              } else {
                ++q.skips;
              }
              stop = kStopNone;
            }
          }
        }
      }
    }
  call_done:
    if (q.err && stop == kStopNone) stop = kStopBefore;
  }
  rec |= stop << 8;
  return make_uint2(rec, rec2);
}

// Desync detection: a call's report row (the frame sent or NULL_FRAME, last_confirmed_frame at the
// comparison, the local players' last queued frame after the call)
__device__ inline void sched_store_report(const SchedParams& p, int32_t c, int64_t s, int32_t rep, int32_t lconf,
                                          int32_t ll) {
  const int64_t i = (int64_t)(c % p.cap) * p.S + s;
  p.rep_frame[i] = rep;
  p.rep_lconf[i] = lconf;
  p.rep_ll[i] = ll;
}
// ... and after the launch (every cell final): each report's checksum, the final cell checksum of its
// frame -- a confirmed frame's cell is never saved again (a rollback starts after every confirmed
// frame), so this is the checksum the reference read from the cell when it sent the report
__device__ inline void sched_report_checksums(const SchedParams& p, int64_t s) {
  for (int32_t c = p.c0; c < p.c0 + p.n; c++) {
    const int64_t i = (int64_t)(c % p.cap) * p.S + s;
    const int32_t f = p.rep_frame[i];
    p.rep_ck[i] = f == kNull ? (uint16_t)0 : p.fck[(int64_t)(f & (p.HF - 1)) * p.S + s];
  }
}

// A launch's end: the control state back to HBM (sst), the counts, and -- without sparse saving,
// where every frame 0 .. last save has been saved -- each cell's frame, the newest one <= the last
// save in its slot.
template <int P>
__device__ inline void sched_store_ctl(const SchedParams& p, const SchedCtl<P>& q, int64_t s, bool cell_frames) {
  const int64_t S = p.S;
  if (cell_frames) {
    for (int r = 0; r < p.R; r++) {
      int32_t fr = kNull;
      if (q.last_saved != kNull) {
        const int32_t d = (q.last_saved - r) % p.R;
        fr = q.last_saved - (d < 0 ? d + p.R : d);
        if (fr < 0) fr = kNull;
      }
      p.ring_frame[(int64_t)r * S + s] = fr;
    }
  }
  auto fld = [&](int f) -> int32_t& { return p.sst[(int64_t)f * S + s]; };
  fld(kCur) = q.cur;
  fld(kLconf) = q.lconf;
  fld(kDframe) = q.dframe;
  fld(kLastSaved) = q.last_saved;
  fld(kDelivered) = q.delivered;
  fld(kLocalLast) = q.local_last;
  fld(kSkips) = q.skips;
  fld(kErr) = q.err;
  fld(kDisc) = (int32_t)q.disc;
  fld(kLastSent) = q.last_sent;
  fld(kRmask) = (int32_t)q.rmask;
#pragma unroll
  for (int k = 0; k < P; k++) fld(kPl0 + kPlFields * k + 0) = q.lf[k];
  p.rollbacks[s] += q.rollbacks;
  p.resim[s] += q.resim;
}

// kSparse: sparse saving; kPred: the predictor (0 repeat-last, 1 PredictDefault) -- compile-time, so
// their tests leave the step loop and its scalar registers
// kLocal: the local-player mask when it is a compile-time one (two players, one of them local: the
// usual peer), else -1.  kSplit: two waves per block of 64 sessions -- wave 1 stages the input rows
// of stage i + 1 and runs its control pass while wave 0 runs stage i's step loop (double-buffered
// records and rows; one barrier per stage); chosen when a CU holds one block (few sessions), where
// the two waves sit on two SIMDs of an otherwise idle CU.  kFeat: desync detection, peer reports or
// the display trace may be on (false: the engine has none of them, and their code is compiled out of
// the control pass and the step loop).
template <int P, bool kSparse, int kPred, int kLocal, bool kSplit, bool kFeat>
__global__ __launch_bounds__(kSplit ? 2 * kBlock : kBlock) void p2p_sched_kernel(SchedParams p) {
  using T = typename InputWord<P>::T;
  using Rec = typename std::conditional<kSparse, uint2, uint32_t>::type;
  constexpr int F = state_fields(P);
  constexpr int PC = cell_dwords_s(P) / 4;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const SchedLds L = sched_lds(P, p.R, kSparse, p.WL, p.K, p.B, kSplit ? 2 : 1);
  int buf = 0;  // this wave's stage buffer
  // LDS regions addressed from the extern array itself at each use (pointer variables into dynamic
  // LDS captured by the lambdas below become generic pointers, which this hipcc miscompiles)
#define lring (reinterpret_cast<uint4*>(lds))
#define ltag (reinterpret_cast<int32_t*>(lds + L.o_tags))
#define llq (reinterpret_cast<T*>(lds + L.o_lq))
#define lrec (reinterpret_cast<Rec*>(lds + L.o_arr + buf * L.rec_b))
#define lrowtag (reinterpret_cast<int32_t*>(lds + L.o_rowtag + buf * L.rowtag_b))
#define lrows (reinterpret_cast<T*>(lds + L.o_rows + buf * L.rows_b))

  p.cur = in_vgpr_ptr(p.cur);
  p.ring = in_vgpr_ptr(p.ring);
  p.ring_frame = in_vgpr_ptr(p.ring_frame);
  p.lq = in_vgpr_ptr(p.lq);
  p.sst = in_vgpr_ptr(p.sst);
  p.rollbacks = in_vgpr_ptr(p.rollbacks);
  p.resim = in_vgpr_ptr(p.resim);
  p.row_tag = in_vgpr_ptr(p.row_tag);
  p.events = in_vgpr_ptr(p.events);
  p.inputs = in_vgpr_ptr(p.inputs);
  p.arrive = in_vgpr_ptr(p.arrive);
  p.cap = in_vgpr_i32(p.cap);
  p.delay = in_vgpr_i32(p.delay);
  const int64_t S = p.S;
  const int64_t sess0 = (int64_t)blockIdx.x * kBlock;
  const int lt = threadIdx.x & (kBlock - 1);
  const bool ctl_w = !kSplit || threadIdx.x >= kBlock;  // this wave stages and decides
  const bool stp_w = !kSplit || threadIdx.x < kBlock;   // this wave steps the game states
  const bool live = sess0 + lt < S;
  const int64_t s = live ? sess0 + lt : sess0;  // idle lanes shadow the block's first session, never store
  const int nb = (int)min((int64_t)kBlock, S - sess0);
  const uint32_t lmask = kLocal >= 0 ? (uint32_t)kLocal : p.local_mask;
  uint32_t lbytes = 0;
#pragma unroll
  for (int k = 0; k < P; k++) lbytes |= ((lmask >> k) & 1u) ? 0xffu << (8 * k) : 0u;
  const uint32_t rbytes = (P == 4 ? 0xffffffffu : ((1u << (8 * P)) - 1u)) & ~lbytes;  // remote players' bytes
  const int32_t maxp = p.maxp, R = p.R, WL = p.WL;
  const int ring_pieces = R * PC;

  // ---- copy in: rings (the block's sessions are contiguous in HBM), tags, local queues
  {
    const uint4* src = reinterpret_cast<const uint4*>(p.ring) + sess0 * ring_pieces;
    const int n = nb * ring_pieces;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const int sl = i / ring_pieces, rem = i - sl * ring_pieces;
      lring[rem * kBlock + sl] = src[i];
    }
  }
  if (kSparse) {
#pragma unroll 8
    for (int q = 0; q < R; q++) ltag[q * kBlock + lt] = live ? p.ring_frame[(int64_t)q * S + s] : kNull;
  }
#pragma unroll 8
  for (int q = 0; q < WL; q++) llq[q * kBlock + lt] = live ? (T)p.lq[(int64_t)q * S + s] : (T)0;

  BoxState<P> st;
  load_state<P>(st, p.cur + s, S);
  auto fld = [&](int f) -> int32_t& { return p.sst[(int64_t)f * S + s]; };
  // The control state, advanced call by call by the control pass (sched_control_call); the step loop
  // keeps its own copies of what the inputs of a frame depend on.
  SchedCtl<P> q;
  q.cur = fld(kCur);
  q.lconf = fld(kLconf);
  q.dframe = fld(kDframe);
  q.last_saved = fld(kLastSaved);
  q.delivered = fld(kDelivered);
  q.local_last = fld(kLocalLast);
  q.skips = fld(kSkips);
  q.err = fld(kErr);
  q.disc = (uint32_t)fld(kDisc);
  q.last_sent = fld(kLastSent);
  q.rmask = (uint32_t)fld(kRmask);
#pragma unroll
  for (int k = 0; k < P; k++) q.lf[k] = fld(kPl0 + kPlFields * k + 0);
  if (!live) q.err = 1;  // idle lanes run no call
  q.slot_f = q.cur % R;
  q.rollbacks = 0;
  q.resim = 0;
  int32_t s_cur = q.cur, s_delivered = q.delivered, s_local_last = q.local_last, s_lf[P];
  uint32_t s_disc = q.disc;
  bool s_done = q.err != 0;
#pragma unroll
  for (int k = 0; k < P; k++) s_lf[k] = q.lf[k];
  // every state the launch steps descends from cur or from a ring cell this engine wrote, all in the
  // lean step's rotation domain: one wave-wide test instead of one per player per step
  const bool lean_ok = __all(rot_in_domain<P>(st));
  // the glibc sinf/cosf constants in vector registers: beside this kernel's many uniform values
  // they would otherwise take 20 scalar registers and spill (glibc_sincosf.h, SincosConsts)
  const SincosConsts K = sincos_consts_vgpr();
  __syncthreads();

  auto next_slot = [&](int32_t x) { return x + 1 == R ? 0 : x + 1; };
  auto back_slot = [&](int32_t x, int32_t d) { const int32_t y = x - d; return y < 0 ? y + R : y; };
  int32_t s_slot_f = q.slot_f;  // step loop: ring slot of the current frame
  uint32_t s_last_ck = (uint32_t)fld(kLastCk);  // the display checksum (p.trace_cap > 0)
  auto cell_load = [&](int32_t slot) {
#pragma unroll
    for (int k = 0; k < PC; k++) {
      const uint4 v = lring[(slot * PC + k) * kBlock + lt];
      const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 4; i++)
        if (4 * k + i < F) st.w[4 * k + i] = x[i];
    }
  };
  // SaveGameState into `slot` (sync_layer.rs:208-215 + ex_game.rs:103-108); the frame tags and
  // last_saved are the control pass's
  auto save = [&](int32_t slot) {
    const uint32_t ck = fletcher16_state<P>(st);
    if (!kSparse && kFeat && p.interval > 0) p.fck[(int64_t)((int32_t)st.w[0] & (p.HF - 1)) * S + s] = (uint16_t)ck;
#pragma unroll
    for (int k = 0; k < PC; k++) {
      uint32_t x[4];
#pragma unroll
      for (int i = 0; i < 4; i++) x[i] = 4 * k + i < F ? st.w[4 * k + i] : (4 * k + i == F ? ck : 0u);
      lring[(slot * PC + k) * kBlock + lt] = make_uint4(x[0], x[1], x[2], x[3]);
    }
  };

  const int32_t c_end = p.c0 + p.n;
  int32_t lo = 0;  // the stage's rows: frames / calls [lo, ce)
  // input row g (frame g's remote inputs, call g's local ones); the control pass has checked that
  // every row the step loop reads is held
  auto row = [&](int32_t g) -> uint32_t {
    if (g >= lo) return (uint32_t)lrows[(g - lo) * kBlock + lt];
    return load_inputs<P>(p.inputs, (int64_t)(g % p.cap) * S + s);
  };
  const int nst = (p.n + p.K - 1) / p.K;
  for (int it = 0; it < nst + (kSplit ? 1 : 0); ++it) {
   if (ctl_w && it < nst) {
    const int32_t cs = p.c0 + it * p.K;
    const int32_t ce = min(c_end, cs + p.K);
    buf = kSplit ? (it & 1) : 0;
    lo = max(0, cs - p.B);
    const int nrows = ce - lo;
    if (!kSplit) __syncthreads();  // every lane is done with the previous stage
    // Staging: every load of a batch is issued before the first is used (one wave per SIMD: a
    // load-use chain per row or call would cost a full memory latency each).
    const int32_t lo_i = lo % p.cap;  // ring slot of row lo
    constexpr int kUnitT = 16 / sizeof(T);  // input words per 16-byte unit
    if (nb == kBlock && ((S * (int64_t)sizeof(T)) & 15) == 0) {  // rows [lo, ce) as 16-byte units
      constexpr int kUpr = kBlock / kUnitT;  // units per row
      const int units = nrows * kUpr;
#pragma unroll 8
      for (int u = lt; u < units; u += kBlock) {  // (unrolled: the global loads issue back to back)
        const int r = u / kUpr, k = u - r * kUpr;
        const int32_t ri = (lo_i + r) % p.cap;  // (a stage may span more rows than the ring holds)
        reinterpret_cast<uint4*>(lrows)[u] =
            reinterpret_cast<const uint4*>(p.inputs + ((int64_t)ri * S + sess0) * sizeof(T))[k];
      }
    } else {  // a partial last block: word by word
      const T* src = reinterpret_cast<const T*>(p.inputs) + sess0 + lt;
#pragma unroll 8
      for (int r = 0; r < nrows; r++) {
        const int32_t ri = (lo_i + r) % p.cap;  // (a stage may span more rows than the ring holds)
        if (lt < nb) lrows[r * kBlock + lt] = src[(int64_t)ri * S];
      }
    }
    bool tags_ok = true;
    for (int r = lt; r < nrows; r += kBlock) {
      const int32_t ri = (lo_i + r) % p.cap;
      const int32_t tag = p.row_tag[ri];
      lrowtag[r] = tag;
      tags_ok &= tag == lo + r;
    }
    if (kSplit) {  // this wave's rows in LDS before its lanes read each other's (no block barrier: one wave)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    } else {
      __syncthreads();
    }
    // The control pass's fast form (below): every staged row held, and at most 64 of them, so that a
    // lane's "where do the remote inputs change" is one 64-bit mask over the stage's rows (repeat-last:
    // row g differs from row g - 1; PredictDefault: row g is not 0).
    const bool mask_ok = !kSparse && nrows <= 64 && __all(tags_ok);
    uint64_t cm = 0;
    if (mask_ok) {
      uint32_t prev = 0;
      for (int r = 0; r < nrows; r++) {
        const uint32_t v = (uint32_t)lrows[r * kBlock + lt] & rbytes;
        if (kPred == 0 ? (r > 0 && v != prev) : v != 0u) cm |= 1ull << r;
        prev = v;
      }
    }

    // ---- control pass: P2PSession::advance_frame's decisions for calls [cs, ce), call by call
    // (every lane at the same call), without the game state; one record per call
    {
      SchedCtlEnv env;
      env.lo = lo;
      env.maxp = maxp;
      env.R = R;
      env.delay = p.delay;
      env.cap = p.cap;
      env.S = S;
      env.s = s;
      env.lmask = lmask;
      env.lbytes = lbytes;
      env.rbytes = rbytes;
      env.o_rowtag = L.o_rowtag + buf * L.rowtag_b;
      env.o_rows = L.o_rows + buf * L.rows_b;
      env.o_tags = L.o_tags;
      env.ns = kBlock;
      env.col = lt;
      env.inputs = p.inputs;
      env.row_tag = p.row_tag;
      env.interval = p.interval;
      env.reports = p.reports;
      env.rtab = p.sst + (int64_t)sched_rep0(P) * S;
      const int32_t ci0 = cs % p.cap;
      for (int32_t cb8 = cs; cb8 < ce; cb8 += 8) {
        int32_t up8[8];
        uint32_t ev8[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {  // this session's arrivals and Event::Disconnected bits, eight calls at a time
          const int32_t ci = (ci0 + (cb8 - cs) + j) % p.cap;
          const bool in = !q.err && cb8 + j < ce;
          up8[j] = in ? p.arrive[(int64_t)ci * S + s] : kNull;
          ev8[j] = (in && p.events) ? p.events[(int64_t)ci * S + s] : 0u;
          if (kFeat && in && p.reports && p.reports[(int64_t)ci * S + s] != 0) ev8[j] |= kEvPeerReport;
        }
        if constexpr (!kSparse) {
          // The batch's calls through the fast form first, back to back, by selects (as the chains
          // form's control wave); a batch where some session needs the general form runs call by
          // call below from the state before it.  A stopped session (q.err) runs no call: its
          // records say so.
          const int nj = min(8, ce - cb8);
          const bool idle = q.err != 0;
          const bool en = !idle & mask_ok;
          const SchedCtl<P> q0 = q;
          bool ok = true;
          uint32_t recs[8];
          int32_t reps[8], lcs[8], lls1[8];
#pragma unroll
          for (int j = 0; j < 8; j++) {
            recs[j] = 0u;
            reps[j] = kNull;
            lcs[j] = q.lconf;
            if (j < nj) ok &= sched_fast_call<P, kPred, kFeat>(q, env, cm, cb8 + j, up8[j], ev8[j], recs[j], reps[j], en);
            lls1[j] = q.local_last;
          }
          if (__builtin_expect(__all(ok | idle), 1)) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
              if (j < nj) {
                lrec[(cb8 + j - cs) * kBlock + lt] = (Rec)(idle ? kStopBefore << 8 : recs[j]);
                if (kFeat && p.interval > 0 && live) sched_store_report(p, cb8 + j, s, reps[j], lcs[j], lls1[j]);
              }
            }
            continue;
          }
          q = q0;
        }
        for (int j = 0; j < 8; j++) {
          const int32_t c = cb8 + j;
          if (c >= ce) break;
          // this call's arrival and events: the front of the batch, which shifts down a call per
          // iteration (indexing it by j would put it in scratch memory)
          const int32_t a_c = up8[0];
          const uint32_t e_c = ev8[0];
#pragma unroll
          for (int k = 0; k < 7; k++) {
            up8[k] = up8[k + 1];
            ev8[k] = ev8[k + 1];
          }
          const int32_t lconf0 = q.lconf;
          int32_t rep;
          const uint2 rr = sched_control_call<P, kSparse, kPred, kFeat>(q, env, mask_ok, cm, c, a_c, e_c, rep);
          if (kFeat && p.interval > 0 && live) sched_store_report(p, c, s, rep, lconf0, q.local_last);
          Rec r;
          if constexpr (kSparse) r = rr;
          else r = rr.x;
          lrec[(c - cs) * kBlock + lt] = r;
        }
      }
    }

   }
   if (stp_w && it >= (kSplit ? 1 : 0)) {
    const int si = kSplit ? it - 1 : it;
    const int32_t cs = p.c0 + si * p.K;
    const int32_t ce = min(c_end, cs + p.K);
    buf = kSplit ? (si & 1) : 0;
    lo = max(0, cs - p.B);
    // ---- step loop: the game states.  One thread per session, each its own step sequence: an
    // iteration is one AdvanceFrame of the lane's current work -- a replayed frame, or its call's own
    // frame -- or a call that does not advance.
    uint32_t conn = rbytes;  // the connected remote players' bytes
#pragma unroll
    for (int k = 0; k < P; k++)
      if ((s_disc >> k) & 1u) conn &= ~(0xffu << (8 * k));
    // synchronized_inputs(h) (sync_layer.rs:280-293): local players from their queues, connected
    // remote players confirmed or predicted -- the input of frame min(h, delivered) in the canonical
    // form (repeat-last; PredictDefault: 0 past delivered) --, disconnected ones
    // InputStatus::Disconnected past their last frame (ex_game spins the ship: input 4, ex_game.rs:280)
    auto sync_inputs = [&](int32_t h) -> uint32_t {
      uint32_t in = lbytes ? (uint32_t)llq[(h & (WL - 1)) * kBlock + lt] & lbytes : 0u;
      const bool conf = h <= s_delivered;  // (a disconnected player's last frame is <= delivered too)
      const uint32_t hrow = s_delivered == kNull ? 0u : row(conf ? h : s_delivered);
      in |= (kPred == 1 && !conf) ? 0u : hrow & conn;
      if (s_disc) {
#pragma unroll
        for (int k = 0; k < P; k++)
          if ((s_disc >> k) & 1u) in |= (h <= s_lf[k] ? (hrow >> (8 * k)) & 0xffu : 4u) << (8 * k);
      }
      return in;
    };
    int32_t c = s_done ? ce : cs;
    bool at_start = true, replaying = false, second = false;
    int32_t h = 0, load = 0, slot_h = 0, save_at = 0;  // save_at: sparse, the replayed frame saved
    uint32_t rec = 0, rec2 = 0;
    // the next call's record, read one call ahead (its LDS latency behind this call's steps)
    Rec nrec = lrec[(min(c, ce - 1) - cs) * kBlock + lt];
    while (c < ce) {
      if (at_start) {
        const Rec r = nrec;
        nrec = lrec[(min(c + 1, ce - 1) - cs) * kBlock + lt];
        if constexpr (kSparse) {
          rec = r.x;
          rec2 = r.y;
        } else {
          rec = r;
        }
        s_delivered += (int32_t)((rec >> 16) & 0xffu);
        // the rare call starts in one branch: a stop, a disconnect (the player's last frame is the
        // newest delivered one, ex_game spins it from the next), or the first call
        if ((rec & 0x0f000300u) != 0u || s_cur == 0) {
          const uint32_t stop = (rec >> 8) & 3u;
          if (stop == kStopBefore) break;
          const uint32_t ev = (rec >> 24) & ~lmask & ~s_disc;
#pragma unroll
          for (int k = 0; k < P; k++)
            if ((ev >> k) & 1u) {
              s_lf[k] = s_delivered;
              conn &= ~(0xffu << (8 * k));
            }
          s_disc |= ev;
          if (s_cur == 0) save(s_slot_f);  // the first frame's save
          if (stop == kStopAfterSave0) break;
        }
        const int32_t d = (int32_t)(rec & 0x7fu);
        second = false;
        if (d) {  // adjust_gamestate's LoadGameState (reset_prediction: nothing to reset in the canonical form)
          load = s_cur - d;
          h = load;
          slot_h = back_slot(s_slot_f, d);
          cell_load(slot_h);
          save_at = kSparse ? (int32_t)((rec2 >> 8) & 0x7fu) : 0;
          replaying = true;
        }
        at_start = false;
      }
      if (kSparse && !replaying && !second) {  // the first replay is done (or there was none)
        if ((rec >> 8 & 3u) == kStopAfterReplay1) break;
        second = true;
        {
          const int32_t d2 = (int32_t)(rec2 & 0x7fu);
          if (d2) {  // check_last_saved_state's rollback to the last save
            load = s_cur - d2;
            h = load;
            slot_h = back_slot(s_slot_f, d2);
            cell_load(slot_h);
            save_at = (int32_t)((rec2 >> 16) & 0x7fu);
            replaying = true;
          }
        }
      }
      // SaveGameState of the replayed frames after the loaded one (:692-702) and of the current
      // frame (:337); without sparse saving every step saves -- the first replay step rewrites the
      // loaded cell with its own bytes -- so the save needs no branch
      const int32_t fr = replaying ? h : s_cur;
      const int32_t sslot = replaying ? slot_h : s_slot_f;
      const bool do_save = !kSparse || (replaying ? h - load + 1 == save_at : ((rec >> 10) & 1u) != 0u);
      const bool adv = replaying || ((rec >> 7) & 1u);
      if (!replaying) {
        // add_local_input (:362-377): queue frame current + delay, dropped unless it is the next
        // one; the first fills the frames below the delay with the default input
        if (lbytes) {
          const int32_t qf = s_cur + p.delay;
          if (s_local_last == kNull || qf == s_local_last + 1) {
            if (s_local_last == kNull)
              for (int32_t q = 0; q < p.delay; q++) llq[(q & (WL - 1)) * kBlock + lt] = (T)0;
            llq[(qf & (WL - 1)) * kBlock + lt] = (T)(row(c) & lbytes);
            s_local_last = qf;
          }
        }
      }
      const uint32_t in = sync_inputs(fr);
      if (kSparse) {
        if (do_save) save(sslot);
      } else {
        save(sslot);
      }
      if (adv) {
        if (lean_ok) {  // State::advance: the players' lean steps side by side, constants in VGPRs
          advance_state_lean_k<P>(st, in, K);
        } else {
          advance_state<P>(st, in, 0u);
        }
      }
      if (kFeat && p.trace_cap > 0) {  // (uniform: only engines with a display trace)
        if (adv) s_last_ck = fletcher16_state<P>(st);
        if (!replaying) p.trace[(int64_t)(c % p.trace_cap) * S + s] = (uint16_t)s_last_ck;
      }
      const bool rep = replaying;
      h = rep ? h + 1 : h;
      slot_h = rep ? next_slot(slot_h) : slot_h;
      replaying = rep && h != s_cur;
      const bool own_adv = !rep && adv;
      s_cur = own_adv ? s_cur + 1 : s_cur;
      s_slot_f = own_adv ? next_slot(s_slot_f) : s_slot_f;
      c = rep ? c : c + 1;
      at_start = !rep;
    }
    if (c < ce) s_done = true;  // stopped at an error
   }
   if (kSplit) __syncthreads();  // stage it + 1's records ready, stage it's buffers free
  }
  __syncthreads();
  {  // rings back to HBM
    uint4* dst = reinterpret_cast<uint4*>(p.ring) + sess0 * ring_pieces;
    const int n = nb * ring_pieces;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const int sl = i / ring_pieces, rem = i - sl * ring_pieces;
      dst[i] = lring[rem * kBlock + sl];
    }
  }
  if (!live) return;
  if (stp_w) {  // the step loop's: the local queues, the game state, the display checksum
    for (int w = 0; w < WL; w++) p.lq[(int64_t)w * S + s] = (uint32_t)llq[w * kBlock + lt];
    store_state<P>(st, p.cur + s, S);
    if (kFeat && p.trace_cap > 0) p.sst[(int64_t)kLastCk * S + s] = (int32_t)s_last_ck;
  }
  if (!ctl_w) return;
  if (kSparse) {
    for (int r = 0; r < R; r++) p.ring_frame[(int64_t)r * S + s] = ltag[r * kBlock + lt];
    sched_store_ctl<P>(p, q, s, false);
  } else {
    sched_store_ctl<P>(p, q, s, true);
    if (kFeat && p.interval > 0) sched_report_checksums(p, s);  // (every save of the launch done: the barrier above)
  }
#undef lring
#undef ltag
#undef llq
#undef lrec
#undef lrowtag
#undef lrows
}

// ---------------------------------------------------------------------------------------------
// The time-aligned form (few sessions): a session's calls spread over 16 lanes.
//
// After call c every state a session holds -- its current state and every saved cell -- is S_c(h),
// the state at frame h under the inputs the session knows after call c (the remote players' inputs
// up to the newest delivered frame, the prediction after; the canonical form above).  A call that
// rolls back to frame m replays the frames m .. cur - 1 from S_{c-1}(m); every other call saves and
// advances its own frame.  Those replays are the reference's work (adjust_gamestate,
// p2p_session.rs:658-714), and they are independent of each other except through the states they
// start from: so each replay runs as a CHAIN on a lane of its own, and every chain advances frame h
// at time step h.  At time step h:
//   * slot 0 (the lineage) holds the session's state at frame h as the calls whose current frame is
//     h see it, saves the cell of h and advances it with the advancing call's inputs;
//   * a chain (slots 1..15) holds S_c(h) of its call c: it saves the cell of h and advances;
//   * a chain starts at its frame m by copying S_{c-1}(m) from the slot that holds it before the
//     step's exchange -- the newest chain covering m (started before m, ending at or after it),
//     else the lineage, else (m before the launch's first frame) the ring cell -- and at its call's
//     current frame hands its state to the lineage (the newest chain ending there);
//   * of the lanes saving frame h's cell only the newest call's write lands (all compute it).
// "Newest" is the chain's key -- its rank among the session's rollbacks, i.e. call order -- taken
// as a max-reduction over the session's 16 lanes (DPP within a row).  The control pass (a fifth
// wave) takes every call's decisions as in p2p_sched_kernel and only stores, per frame: whether a
// call has it as its current frame, whether that call advances and with which delivered frame /
// disconnect mask, the local players' queued input, and the chains starting there (slot, depth,
// key, inputs).  The step waves run one stage behind it and process frame h once no later call can
// start a chain at or before h (h < current frame - max_prediction).  A launch thus takes about as
// many time steps as frames it advances, instead of frames + replays in sequence; the replays cost
// idle lanes, not time.  Bit-exact with p2p_sched_kernel (the same control pass, the same cells,
// counts and states; tests/test_gpu_p2p_sched.py runs both forms).
//
// Requirements (the host picks p2p_sched_kernel otherwise): no sparse saving, max_prediction <= 12
// and at most two remote players.  Then chain slots can be dealt round-robin: the chains active at
// frame h start in [h - max_prediction, h] at strictly increasing frames except a disconnect's
// rollback to the player's last frame + 1 (at most one per remote player), so at most
// max_prediction + 3 <= 15 are in flight and the chain 15 ranks later starts after this one ended;
// and at most two start at one frame.
constexpr int kCS = 16;          // sessions per block
constexpr int kSL = 16;          // lanes per session: slot 0 the lineage, slots 1..15 chains
constexpr int kChainThreads = kCS * kSL + 64;  // four step waves + the control wave
constexpr int kMaxChainDepth = 12;              // max_prediction of the time-aligned form
constexpr int kChainMaxK = 32;                  // calls per stage (the control wave's prefetch registers)

// per (frame % TW, session): two uint4
//   e0.x  the delivered frame of the call at this current frame that advances (the last one there)
//   e0.y  bit 0 a call has this current frame | 1 it advances | 2-5 its disconnect mask
//   e0.zw chain 0 starting here: delivered frame, flags (bit 0 valid | 4-7 slot | 8-11 depth |
//         12-15 disconnect mask | 16-31 key)
//   e1.xy chain 1 (a second chain starting at the same frame), e1.z the local players' input
struct ChainLds {
  uint32_t o_tab, o_rowtag, o_rows, o_arr, o_ev, o_range, o_lf, total;
  uint32_t rowtag_b, rows_b, arr_b, ev_b;
};
__host__ __device__ inline ChainLds chain_lds(int P, int R, int TW, int K, int B) {
  ChainLds l;
  l.o_tab = (uint32_t)R * (cell_dwords_s(P) / 4) * kCS * 16;
  l.rowtag_b = align16((uint32_t)(K + B) * 4);
  l.rows_b = align16((uint32_t)(K + B) * kCS * input_word_bytes(P));
  l.arr_b = align16((uint32_t)K * kCS * 4);
  l.ev_b = align16((uint32_t)K * kCS);
  l.o_rowtag = l.o_tab + (uint32_t)TW * kCS * 32;
  l.o_rows = l.o_rowtag + 3 * l.rowtag_b;  // three stage buffers: the control's, the steps', the prefetch's
  l.o_arr = l.o_rows + 3 * l.rows_b;
  l.o_ev = l.o_arr + 2 * l.arr_b;
  l.o_range = l.o_ev + 2 * l.ev_b;
  l.o_lf = l.o_range + 2 * kCS * 8;
  l.total = l.o_lf + kCS * 4 * 4;
  return l;
}

// max over the 16 lanes of a DPP row, in every lane of it
// (mov_dpp with every row and bank enabled and bound_ctrl: the DPP combiner folds each move into
// its max as one v_max_i32_dpp; every lane of these patterns reads a lane of its own row)
__device__ inline int32_t rowmax16(int32_t v) {
  v = max(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, true));   // quad_perm [1,0,3,2]
  v = max(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, true));   // quad_perm [2,3,0,1]
  v = max(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xf, 0xf, true));  // row_half_mirror
  v = max(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xf, 0xf, true));  // row_mirror
  return v;
}

// the same for two 16-bit signed values at once (v_pk_max_i16 per DPP step)
typedef short ggrs_s2v __attribute__((ext_vector_type(2)));
__device__ inline uint32_t rowmax16_pk(uint32_t v) {
  ggrs_s2v x = __builtin_bit_cast(ggrs_s2v, v);
#define GGRS_PK_STEP(ctrl) \
  x = __builtin_elementwise_max(x, __builtin_bit_cast(ggrs_s2v, __builtin_amdgcn_mov_dpp((int)__builtin_bit_cast(uint32_t, x), ctrl, 0xf, 0xf, true)))
  GGRS_PK_STEP(0xB1);
  GGRS_PK_STEP(0x4E);
  GGRS_PK_STEP(0x141);
  GGRS_PK_STEP(0x140);
#undef GGRS_PK_STEP
  return __builtin_bit_cast(uint32_t, x);
}
constexpr int kChainMaxCalls = 2000;  // calls per launch: chain keys (ranks) << 4 | slot fit 15 bits

// A stage's global reads for the control wave (input rows and their tags, arrivals, events), held
// in registers from their issue to their store into LDS -- one stage ahead, behind the control pass
template <int P>
struct ChainStage {
  static constexpr int kUnitT = 16 / (int)sizeof(typename InputWord<P>::T);
  static constexpr int kUpr = kCS / kUnitT;  // 16-byte units of one row of the block's sessions
  uint4 rows[kUpr];
  int32_t tag;
  uint4 arr[(kChainMaxK * 4 + 63) / 64];
  uint4 ev;
};

// kFeat: desync detection on (false: its code compiled out; this form never takes peer reports or a
// trace)
template <int P, int kPred, int kLocal, bool kFeat>
__global__ __launch_bounds__(kChainThreads) void p2p_sched_chains_kernel(SchedParams p) {
  using T = typename InputWord<P>::T;
  constexpr int F = state_fields(P);
  constexpr int PC = cell_dwords_s(P) / 4;
  const int TW = p.TW;  // table frames (a power of two)
  const ChainLds L = chain_lds(P, p.R, TW, p.K, p.B);
#define lring (reinterpret_cast<uint4*>(sched_lds_base))
#define ltab (reinterpret_cast<uint4*>(sched_lds_base + L.o_tab))
#define lrange (reinterpret_cast<int2*>(sched_lds_base + L.o_range))
#define llf (reinterpret_cast<int32_t*>(sched_lds_base + L.o_lf))

  const int64_t S = p.S;
  const int64_t sess0 = (int64_t)blockIdx.x * kCS;
  const int nb = (int)min((int64_t)kCS, S - sess0);
  const bool ctl_w = threadIdx.x >= kCS * kSL;
  const uint32_t lmask = kLocal >= 0 ? (uint32_t)kLocal : p.local_mask;
  uint32_t lbytes = 0;
#pragma unroll
  for (int k = 0; k < P; k++) lbytes |= ((lmask >> k) & 1u) ? 0xffu << (8 * k) : 0u;
  const uint32_t rbytes = (P == 4 ? 0xffffffffu : ((1u << (8 * P)) - 1u)) & ~lbytes;
  const int32_t maxp = p.maxp, R = p.R;
  const int ring_pieces = R * PC;
  const int32_t c_end = p.c0 + p.n;
  const int nst = (p.n + p.K - 1) / p.K;
  auto tab0 = [&](int32_t f, int col) -> uint4& { return ltab[((f & (TW - 1)) * kCS + col) * 2]; };
  auto tab1 = [&](int32_t f, int col) -> uint4& { return ltab[((f & (TW - 1)) * kCS + col) * 2 + 1]; };
  auto stage_lo = [&](int st) { return max(0, p.c0 + st * p.K - p.B); };
  auto stage_rows = [&](int st) -> T* { return reinterpret_cast<T*>(sched_lds_base + L.o_rows + (st % 3) * L.rows_b); };

  // ---- copy in: the block's rings
  {
    const uint4* src = reinterpret_cast<const uint4*>(p.ring) + sess0 * ring_pieces;
    const int n = nb * ring_pieces;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const int sl = i / ring_pieces, rem = i - sl * ring_pieces;
      lring[rem * kCS + sl] = src[i];
    }
  }

  if (ctl_w) {
    // ================= the control wave: lanes 0..15 are the block's sessions =================
    const int lt = threadIdx.x - kCS * kSL;
    const int col = lt < kCS ? lt : 0;
    const bool live = lt < nb;
    const int64_t s = live ? sess0 + lt : sess0;
    auto fld = [&](int f) -> int32_t { return p.sst[(int64_t)f * S + s]; };
    SchedCtl<P> q;
    q.cur = fld(kCur);
    q.lconf = fld(kLconf);
    q.dframe = fld(kDframe);
    q.last_saved = fld(kLastSaved);
    q.delivered = fld(kDelivered);
    q.local_last = fld(kLocalLast);
    q.skips = fld(kSkips);
    q.err = fld(kErr);
    q.disc = (uint32_t)fld(kDisc);
    q.last_sent = fld(kLastSent);
    q.rmask = (uint32_t)fld(kRmask);
#pragma unroll
    for (int k = 0; k < P; k++) q.lf[k] = fld(kPl0 + kPlFields * k + 0);
    if (!live) q.err = 1;  // idle lanes run no call
    q.slot_f = q.cur % R;
    q.rollbacks = 0;
    q.resim = 0;
    const int32_t cur0 = q.cur;
    int32_t own_hi = cur0 - 1, minpre = INT32_MAX, tn = 0, nchain = 0, last_m = kNull, dups = 0;
    bool started = false;
    if (lt < kCS) {
      // the frames before the launch's first one: no call of this launch, no chain yet
      for (int32_t f = max(0, cur0 - maxp); f < cur0; f++) {
        tab0(f, col) = make_uint4(0u, 0u, 0u, 0u);
        *reinterpret_cast<uint2*>(&tab1(f, col)) = make_uint2(0u, 0u);
      }
      // the local players' queued inputs still read: frames cur - max_prediction - 1 .. local_last
      if (q.local_last != kNull)
        for (int32_t f = max(0, cur0 - maxp - 1); f <= q.local_last; f++)
          tab1(f, col).z = p.lq[(int64_t)(f & (p.WL - 1)) * S + s];
#pragma unroll
      for (int k = 0; k < P; k++) llf[col * 4 + k] = q.lf[k];
    }
    // Staging of stage st: its input rows [lo, ce) and their tags, its calls' arrivals and events.
    // issue() starts the global reads into registers; store() writes them to the stage's buffers.
    const bool full = nb == kCS && ((S * (int64_t)sizeof(T)) & 15) == 0;
    ChainStage<P> pf;
    auto issue = [&](int st) {
      const int32_t cs = p.c0 + st * p.K, ce = min(c_end, cs + p.K), lo = stage_lo(st);
      const int nrows = ce - lo, ncalls = ce - cs;
      const int32_t lo_i = lo % p.cap, ci0 = cs % p.cap;
#pragma unroll
      for (int k = 0; k < ChainStage<P>::kUpr; k++) {
        const int u = lt + 64 * k, r = u / ChainStage<P>::kUpr, kk = u - r * ChainStage<P>::kUpr;
        const int32_t ri = (lo_i + r) % p.cap;  // (a stage may span more rows than the ring holds)
        pf.rows[k] = (full && r < nrows)
                         ? reinterpret_cast<const uint4*>(p.inputs + ((int64_t)ri * S + sess0) * sizeof(T))[kk]
                         : make_uint4(0u, 0u, 0u, 0u);
      }
      {
        const int32_t ri = (lo_i + lt) % p.cap;
        pf.tag = lt < nrows ? p.row_tag[ri] : kNull;
      }
#pragma unroll
      for (int k = 0; k < (kChainMaxK * 4 + 63) / 64; k++) {
        const int u = lt + 64 * k, r = u / 4, kk = u - r * 4;
        const int32_t ci = (ci0 + min(r, ncalls - 1)) % p.cap;
        pf.arr[k] = (full && r < ncalls) ? reinterpret_cast<const uint4*>(p.arrive + (int64_t)ci * S + sess0)[kk]
                                         : make_uint4(0u, 0u, 0u, 0u);
      }
      {
        const int32_t ci = (ci0 + min(lt, ncalls - 1)) % p.cap;
        pf.ev = (full && lt < ncalls) ? *reinterpret_cast<const uint4*>(p.events + (int64_t)ci * S + sess0)
                                      : make_uint4(0u, 0u, 0u, 0u);
      }
    };
    auto store = [&](int st) -> bool {
      const int32_t cs = p.c0 + st * p.K, ce = min(c_end, cs + p.K), lo = stage_lo(st);
      const int nrows = ce - lo, ncalls = ce - cs;
      T* lrows = stage_rows(st);
      int32_t* lrowtag = reinterpret_cast<int32_t*>(sched_lds_base + L.o_rowtag + (st % 3) * L.rowtag_b);
      int32_t* larr = reinterpret_cast<int32_t*>(sched_lds_base + L.o_arr + (st & 1) * L.arr_b);
      uint8_t* lev = sched_lds_base + L.o_ev + (st & 1) * L.ev_b;
      if (full) {
#pragma unroll
        for (int k = 0; k < ChainStage<P>::kUpr; k++) {
          const int u = lt + 64 * k;
          if (u / ChainStage<P>::kUpr < nrows) reinterpret_cast<uint4*>(lrows)[u] = pf.rows[k];
        }
#pragma unroll
        for (int k = 0; k < (kChainMaxK * 4 + 63) / 64; k++) {
          const int u = lt + 64 * k;
          if (u / 4 < ncalls) reinterpret_cast<uint4*>(larr)[u] = pf.arr[k];
        }
        if (lt < ncalls) reinterpret_cast<uint4*>(lev)[lt] = pf.ev;
      } else {  // a partial last block: word by word, read here
        const int32_t lo_i = lo % p.cap, ci0 = cs % p.cap;
        for (int r = 0; r < nrows; r++) {
          const int32_t ri = (lo_i + r) % p.cap;
          if (lt < nb) lrows[r * kCS + col] = reinterpret_cast<const T*>(p.inputs)[(int64_t)ri * S + sess0 + col];
        }
        for (int r = 0; r < ncalls; r++) {
          int32_t ci = ci0 + r;
          ci = ci >= p.cap ? ci - p.cap : ci;
          if (lt < nb) {
            larr[r * kCS + col] = p.arrive[(int64_t)ci * S + sess0 + col];
            lev[r * kCS + col] = p.events[(int64_t)ci * S + sess0 + col];
          }
        }
      }
      if (lt < nrows) lrowtag[lt] = pf.tag;
      return lt >= nrows || pf.tag == lo + lt;
    };
    // One call's table entries (its record, the frame it was at, the local players' last queued
    // frame before / after it, its delivered frame and disconnect mask, its input row).
    auto emit = [&](int32_t tau, int32_t ll0, int32_t ll1, uint32_t rec, int32_t dlv, uint32_t disc, uint32_t rw_c) {
      const uint32_t stop = (rec >> 8) & 3u;
      // add_local_input: the local players' input of the queued frame (and, the first time, the
      // default input below the delay)
      if (lbytes && ll1 != ll0) {
        if (ll0 == kNull)
          for (int32_t f = 0; f < p.delay; f++) tab1(f, col).z = 0u;
        tab1(ll1, col).z = rw_c & lbytes;
      }
      if (stop == kStopBefore || (stop == kStopAfterSave0 && tau != 0)) return;
      const int32_t d = stop == kStopNone ? (int32_t)(rec & 0x7fu) : 0;
      if (d) {
        // the replay of frames m .. tau - 1 as a chain, on the next slot in round-robin order
        const int32_t m = tau - d;
        dups = m == last_m ? dups + 1 : 0;
        if (dups > 1) {
          q.err = GGRS_E_STATE;  // a third chain at one frame (cannot happen within the requirements)
          return;
        }
        const uint32_t cf = 1u | (uint32_t)(1 + nchain % (kSL - 1)) << 4 | (uint32_t)d << 8 | disc << 12 |
                            (uint32_t)nchain << 16;
        uint2* ce2 = dups ? reinterpret_cast<uint2*>(&tab1(m, col)) : reinterpret_cast<uint2*>(&tab0(m, col)) + 1;
        *ce2 = make_uint2((uint32_t)dlv, cf);
        ++nchain;
        last_m = m;
        if (m < cur0) minpre = min(minpre, m);
      }
      // the lineage's work at frame tau (the first call there opens the frame: no chain starts there
      // yet; a later call at the same frame overwrites the advance and inputs)
      const uint32_t y = 1u | (stop == kStopNone ? ((rec & 0x80u) ? 2u : 0u) | disc << 2 : 0u);
      const uint32_t xx = stop == kStopNone ? (uint32_t)dlv : 0u;
      if (tau > own_hi) {
        own_hi = tau;
        tab0(tau, col) = make_uint4(xx, y, 0u, 0u);
        *reinterpret_cast<uint2*>(&tab1(tau, col)) = make_uint2(0u, 0u);
      } else {
        *reinterpret_cast<uint2*>(&tab0(tau, col)) = make_uint2(xx, y);
      }
    };
    // emit() for a call the fast form took: no stop, no disconnect, the local queue not empty (the
    // form's preconditions) -- fewer branches in the batch's unrolled entries
    auto emit_fast = [&](int32_t tau, int32_t ll0, int32_t ll1, uint32_t rec, int32_t dlv, uint32_t rw_c) {
      if (lbytes && ll1 != ll0) tab1(ll1, col).z = rw_c & lbytes;
      const int32_t d = (int32_t)(rec & 0x7fu);
      if (d) {
        const int32_t m = tau - d;
        dups = m == last_m ? dups + 1 : 0;
        if (dups > 1) {
          q.err = GGRS_E_STATE;
          return;
        }
        const uint32_t cf = 1u | (uint32_t)(1 + nchain % (kSL - 1)) << 4 | (uint32_t)d << 8 | (uint32_t)nchain << 16;
        uint2* ce2 = dups ? reinterpret_cast<uint2*>(&tab1(m, col)) : reinterpret_cast<uint2*>(&tab0(m, col)) + 1;
        *ce2 = make_uint2((uint32_t)dlv, cf);
        ++nchain;
        last_m = m;
        if (m < cur0) minpre = min(minpre, m);
      }
      const uint32_t y = 1u | ((rec & 0x80u) ? 2u : 0u);
      if (tau > own_hi) {
        own_hi = tau;
        tab0(tau, col) = make_uint4((uint32_t)dlv, y, 0u, 0u);
        *reinterpret_cast<uint2*>(&tab1(tau, col)) = make_uint2(0u, 0u);
      } else {
        *reinterpret_cast<uint2*>(&tab0(tau, col)) = make_uint2((uint32_t)dlv, y);
      }
    };
    issue(0);
    bool tags_ok = store(0);
    __syncthreads();  // (1) tables and rings in
    // the previous stage's change mask over its rows (its rows from lo_prev, n_prev of them)
    uint64_t cm_prev = 0;
    int32_t lo_prev = 0;
    int n_prev = 0;
    bool ok_prev = false;

    for (int it = 0; it <= nst; ++it) {
      if (it < nst) {
        const int32_t cs = p.c0 + it * p.K;
        const int32_t ce = min(c_end, cs + p.K);
        const int32_t lo = stage_lo(it);
        const int nrows = ce - lo;
        const uint32_t o_rowtag = L.o_rowtag + (it % 3) * L.rowtag_b, o_rows = L.o_rows + (it % 3) * L.rows_b;
        const T* lrows = stage_rows(it);
        const int32_t* larr = reinterpret_cast<const int32_t*>(sched_lds_base + L.o_arr + (it & 1) * L.arr_b);
        const uint8_t* lev = sched_lds_base + L.o_ev + (it & 1) * L.ev_b;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // this stage's staging visible to the wave
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (it + 1 < nst) issue(it + 1);  // the next stage's reads fly behind this stage's calls
        const bool mask_ok = nrows <= 64 && __all(tags_ok);
        uint64_t cm = 0;
        if (mask_ok) {
          // the rows this stage shares with the previous one keep their bits (the same frames' rows):
          // only the new rows are read
          const int32_t sh = lo - lo_prev;
          int r0 = 0;
          if (ok_prev && sh > 0 && sh < n_prev) {
            cm = cm_prev >> sh;
            if (kPred == 0) cm &= ~1ull;  // (row 0 has no row before it in the stage)
            r0 = n_prev - sh;
          }
          uint32_t prev = (kPred == 0 && r0 > 0) ? (uint32_t)lrows[(r0 - 1) * kCS + col] & rbytes : 0u;
#pragma unroll 8
          for (int r = r0; r < nrows; r++) {
            const uint32_t v = (uint32_t)lrows[r * kCS + col] & rbytes;
            if (kPred == 0 ? (r > 0 && v != prev) : v != 0u) cm |= 1ull << r;
            prev = v;
          }
        }
        cm_prev = cm;
        lo_prev = lo;
        n_prev = nrows;
        ok_prev = mask_ok;
        SchedCtlEnv env;
        env.lo = lo;
        env.maxp = maxp;
        env.R = R;
        env.delay = p.delay;
        env.cap = p.cap;
        env.S = S;
        env.s = s;
        env.lmask = lmask;
        env.lbytes = lbytes;
        env.rbytes = rbytes;
        env.o_rowtag = o_rowtag;
        env.o_rows = o_rows;
        env.o_tags = 0;
        env.ns = kCS;
        env.col = col;
        env.inputs = p.inputs;
        env.row_tag = p.row_tag;
        env.interval = kFeat ? p.interval : 0;
        env.reports = nullptr;  // (this form runs only without peer reports: the host's choice)
        env.rtab = p.sst + (int64_t)sched_rep0(P) * S;
        for (int32_t cb8 = cs; cb8 < ce; cb8 += 8) {
          // eight calls' arrivals, events and input rows (the local players' input each call queues),
          // all read before the first is used
          int32_t up8[8];
          uint32_t ev8[8], rw8[8];
#pragma unroll
          for (int j = 0; j < 8; j++) {
            const int r = min(cb8 + j, ce - 1) - cs;
            up8[j] = larr[r * kCS + col];
            ev8[j] = lev[r * kCS + col];
            rw8[j] = (uint32_t)lrows[(r + cs - lo) * kCS + col];
          }
          // The batch's calls through the fast form first, back to back (they depend on each other
          // only through a few scalars of q); their table entries after.  A batch where some session
          // needs the general form runs call by call from the state before it.
          const int nj = min(8, ce - cb8);
          const bool idle = !live | (q.err != 0);  // runs no call (a stopped session: kStopBefore, no entry)
          const bool en = !idle & mask_ok;
          const SchedCtl<P> q0 = q;
          bool ok = true;
          uint32_t recs[8];
          int32_t taus[8], dlvs[8], lls0[8], lls1[8], reps[8], lcs[8];
#pragma unroll
          for (int j = 0; j < 8; j++) {
            recs[j] = 0u;
            reps[j] = kNull;
            taus[j] = q.cur;
            lls0[j] = q.local_last;
            lcs[j] = q.lconf;
            if (j < nj) ok &= sched_fast_call<P, kPred, kFeat>(q, env, cm, cb8 + j, up8[j], ev8[j], recs[j], reps[j], en);
            dlvs[j] = q.delivered;
            lls1[j] = q.local_last;
          }
          if (__builtin_expect(__all(ok | idle), 1)) {
            if (en) {
#pragma unroll
              for (int j = 0; j < 8; j++) {
                if (j < nj) emit_fast(taus[j], lls0[j], lls1[j], recs[j], dlvs[j], rw8[j]);
                if (kFeat && j < nj && p.interval > 0) sched_store_report(p, cb8 + j, s, reps[j], lcs[j], lls1[j]);
              }
            }
            if (kFeat && p.interval > 0 && live && !en) {  // (a stopped session: no report)
              for (int j = 0; j < nj; j++) sched_store_report(p, cb8 + j, s, kNull, q.lconf, q.local_last);
            }
            continue;
          }
          q = q0;
          for (int j = 0; j < 8; j++) {
            const int32_t c = cb8 + j;
            if (c >= ce) break;
            // the front of the batch, which shifts down a call per iteration (indexing it by j would
            // put it in scratch memory)
            const int32_t a_c = q.err ? kNull : up8[0];
            const uint32_t e_c = q.err ? 0u : ev8[0], rw_c = rw8[0];
#pragma unroll
            for (int k = 0; k < 7; k++) {
              up8[k] = up8[k + 1];
              ev8[k] = ev8[k + 1];
              rw8[k] = rw8[k + 1];
            }
            const int32_t tau = q.cur, ll0 = q.local_last, lconf0 = q.lconf;
            const uint32_t disc0 = q.disc;
            int32_t rep;
            const uint32_t rec = sched_control_call<P, false, kPred, kFeat>(q, env, mask_ok, cm, c, a_c, e_c, rep).x;
            if (!live) continue;
            if (kFeat && p.interval > 0) sched_store_report(p, c, s, rep, lconf0, q.local_last);
            if (q.disc != disc0) {  // the disconnected players' last frames, frozen now
#pragma unroll
              for (int k = 0; k < P; k++)
                if (((q.disc ^ disc0) >> k) & 1u) llf[col * 4 + k] = q.lf[k];
            }
            emit(tau, ll0, q.local_last, rec, q.delivered, q.disc, rw_c);
          }
        }
        if (it + 1 < nst) tags_ok = store(it + 1);
        // the frames the step waves may process: every chain that can still start has m >= cur - max_prediction
        if (lt < kCS) {
          const bool last = it == nst - 1 || q.err;
          const int32_t Tn = last ? own_hi + 1 : q.cur - maxp;
          if (!started && (last || Tn >= cur0)) {
            started = true;
            tn = min(cur0, minpre);
          }
          int2 rg = make_int2(0, 0);
          if (started) {
            rg = make_int2(tn, max(tn, Tn));
            tn = rg.y;
          }
          lrange[(it & 1) * kCS + col] = rg;
        }
      }
      __syncthreads();  // (2) stage it's tables ready; stage it - 1's steps done
    }
    __syncthreads();  // (3) every step done
    // rings back (every thread), then this session's control state and local queue
    {
      uint4* dst = reinterpret_cast<uint4*>(p.ring) + sess0 * ring_pieces;
      const int n = nb * ring_pieces;
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int sl = i / ring_pieces, rem = i - sl * ring_pieces;
        dst[i] = lring[rem * kCS + sl];
      }
    }
    if (!live || lt >= kCS) return;
    if (q.local_last != kNull)
      for (int32_t f = max(0, q.cur - maxp - 1); f <= q.local_last; f++)
        p.lq[(int64_t)(f & (p.WL - 1)) * S + s] = tab1(f, col).z;
    sched_store_ctl<P>(p, q, s, true);
    if (kFeat && p.interval > 0) sched_report_checksums(p, s);  // (every step done: barrier (3))
    return;
  }

  // ================= the step waves: lane = session (4 per wave) x slot =================
  const int lane = threadIdx.x;
  const int j = lane & (kSL - 1), sib = lane / kSL;
  const bool live = sib < nb;
  const int64_t s = live ? sess0 + sib : sess0;
  const int sbase = lane & ~(kSL - 1) & 63;  // the session's first lane in the wave
  const int32_t cur0 = p.sst[(int64_t)kCur * S + s];  // the launch's first frame (the lineage's)
  BoxState<P> st;
  if (j == 0) {
    load_state<P>(st, p.cur + s, S);
  } else {
#pragma unroll
    for (int k = 0; k < F; k++) st.w[k] = 0u;
  }
  const bool lean_ok = __all(j != 0 || rot_in_domain<P>(st));
  const SincosConsts K = sincos_consts_vgpr();
  // this slot's chain: active, its first frame, its call's current frame, key (rank), inputs
  bool act = false;
  int32_t cm = 0, cend = 0, ckey = 0, cdlv = kNull;
  uint32_t cdisc = 0;
  __syncthreads();  // (1)
  for (int it = 0; it <= nst; ++it) {
    if (it >= 1) {
      const int32_t lo = stage_lo(it - 1);
      const uint32_t o_rows = L.o_rows + ((it - 1) % 3) * L.rows_b;  // (an offset: see sched_lds_base)
      const int2 rg = lrange[((it - 1) & 1) * kCS + sib];
      int32_t tau = live ? rg.x : 0;
      const int32_t te = live ? rg.y : 0;
      int32_t slot_tau = tau % R;
      auto row = [&](int32_t g) -> uint32_t {
        if (g >= lo) return (uint32_t)reinterpret_cast<const T*>(sched_lds_base + o_rows)[(g - lo) * kCS + sib];
        return load_inputs<P>(p.inputs, (int64_t)(g % p.cap) * S + s);
      };
      // (the loop compiled once per advance form: the general one never runs on states this engine made)
      auto steps = [&](auto lean_c) {
      constexpr bool kLean = decltype(lean_c)::value;
      uint4 e0 = tab0(tau, sib), e1 = tab1(tau, sib);
      while (__any(tau < te)) {
        // (every decision by selects, gated by `on`: the wave iterates while any of its sessions has
        // a frame left)
        const bool on = tau < te;
        const int32_t tau1 = on ? tau + 1 : tau;
        const uint4 n0 = tab0(tau1, sib), n1 = tab1(tau1, sib);  // the next step's entries, read ahead
        // who holds S(tau) before the exchange (the newest chain started before tau and ending at or
        // after it), which chain ends here (the newest), and which replaying chain writes the cell of
        // tau last (the newest, a chain starting here included), by key over the session's 16 lanes
        const int32_t me = ckey << 4 | j;
        const bool hold_c = on & act & (cm < tau) & (tau <= cend);
        const bool hand_c = on & act & (cend == tau);
        // a chain starting on this slot at this frame
        const bool s0 = on & ((e0.w & 1u) != 0u) & (((e0.w >> 4) & 15u) == (uint32_t)j);
        const bool s1 = on & ((e1.y & 1u) != 0u) & (((e1.y >> 4) & 15u) == (uint32_t)j);
        const bool sn = s0 | s1;
        const int32_t hdmax = __builtin_amdgcn_ballot_w64(hand_c) ? rowmax16(hand_c ? me : -1) : -1;
        const uint32_t cf = s0 ? e0.w : e1.y;
        act = act | sn;
        cm = sn ? tau : cm;
        cend = sn ? tau + (int32_t)((cf >> 8) & 15u) : cend;
        ckey = sn ? (int32_t)(cf >> 16) : ckey;
        cdlv = sn ? (int32_t)(s0 ? e0.z : e1.x) : cdlv;
        cdisc = sn ? (cf >> 12) & 15u : cdisc;
        const bool rep = on & (j != 0) & act & (tau < cend);
        const int32_t me1 = ckey << 4 | j;
        const uint32_t red = rowmax16_pk((uint32_t)(hold_c ? me : 0xffff) | (uint32_t)(rep ? me1 : 0xffff) << 16);
        const int32_t hmax = (int32_t)(int16_t)(red & 0xffffu), lwmax = (int32_t)(int16_t)(red >> 16);
        const bool ring_ld = sn & (hmax < 0) & (tau < cur0);
        // the lineage: a call has this current frame; it takes the newest chain ending here
        const bool own = (j == 0) & on & ((e0.y & 1u) != 0u);
        const int src = sn ? (hmax >= 0 ? (sbase | (hmax & 15)) : sbase)
                           : ((own & (hdmax >= 0)) ? (sbase | (hdmax & 15)) : (lane & 63));
        const bool adv = rep | (own & ((e0.y & 2u) != 0u));
        // the cell of frame tau: the newest replaying chain writes it last, else the lineage
        const bool wr = (rep & (me1 == lwmax)) | (own & (lwmax < 0));
        // synchronized_inputs(tau) (sync_layer.rs:280-293) as the lane's call sees it -- before the
        // exchange, whose latency its row read shares (computed on every lane, used where it advances)
        const int32_t dlv = own ? (int32_t)e0.x : cdlv;
        const uint32_t disc = own ? (e0.y >> 2) & 15u : cdisc;
        const bool conf = tau <= dlv;
        const int32_t g = (adv & (dlv != kNull)) ? (conf ? tau : dlv) : lo;
        uint32_t hrow = (uint32_t)reinterpret_cast<const T*>(sched_lds_base + o_rows)[(max(g, lo) - lo) * kCS + sib];
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(g < lo) != 0, 0)) {
          if (g < lo) hrow = row(g);  // far behind its calls: the input ring
        }
        hrow = dlv == kNull ? 0u : hrow;
        uint32_t conn = rbytes;
#pragma unroll
        for (int k = 0; k < P; k++) conn &= ((disc >> k) & 1u) ? ~(0xffu << (8 * k)) : 0xffffffffu;
        uint32_t in = (lbytes ? e1.z & lbytes : 0u) | ((kPred == 1 && !conf) ? 0u : hrow & conn);
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(adv & (disc != 0u)) != 0, 0)) {
          // InputStatus::Disconnected past the player's last frame (ex_game spins it: input 4)
#pragma unroll
          for (int k = 0; k < P; k++)
            if ((disc >> k) & 1u) in |= (tau <= llf[sib * 4 + k] ? (hrow >> (8 * k)) & 0xffu : 4u) << (8 * k);
        }
        // the exchange: every lane reads its source's state from before it
        if (__builtin_amdgcn_ballot_w64(src != (lane & 63))) {
#pragma unroll
          for (int k = 0; k < F; k++) st.w[k] = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)st.w[k]);
        }
        if (__builtin_amdgcn_ballot_w64(ring_ld)) {
          if (ring_ld) {
#pragma unroll
            for (int k = 0; k < PC; k++) {
              const uint4 v = lring[(slot_tau * PC + k) * kCS + sib];
              const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
              for (int i = 0; i < 4; i++)
                if (4 * k + i < F) st.w[4 * k + i] = x[i];
            }
          }
        }
        // SaveGameState of frame tau (sync_layer.rs:208-215, ex_game.rs:103-108)
        {
          const uint32_t ck = fletcher16_state<P>(st);
          if (kFeat && wr && p.interval > 0) p.fck[(int64_t)(tau & (p.HF - 1)) * S + s] = (uint16_t)ck;
          if (wr) {
#pragma unroll
            for (int k = 0; k < PC; k++) {
              uint32_t x[4];
#pragma unroll
              for (int i = 0; i < 4; i++) x[i] = 4 * k + i < F ? st.w[4 * k + i] : (4 * k + i == F ? ck : 0u);
              lring[(slot_tau * PC + k) * kCS + sib] = make_uint4(x[0], x[1], x[2], x[3]);
            }
          }
        }
        if (adv) {
          if (kLean) advance_state_lean_k<P>(st, in, K);
          else advance_state<P>(st, in, 0u);
        }
        e0 = n0;
        e1 = n1;
        act = act & !(on & (tau >= cend));  // handed off this step (the lineage read it above)
        tau = tau1;
        slot_tau = on ? (slot_tau + 1 == R ? 0 : slot_tau + 1) : slot_tau;
      }
      };
      if (lean_ok) steps(std::true_type());
      else steps(std::false_type());
    }
    __syncthreads();  // (2)
  }
  __syncthreads();  // (3)
  {
    uint4* dst = reinterpret_cast<uint4*>(p.ring) + sess0 * ring_pieces;
    const int n = nb * ring_pieces;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const int sl = i / ring_pieces, rem = i - sl * ring_pieces;
      dst[i] = lring[rem * kCS + sl];
    }
  }
  if (live && j == 0) store_state<P>(st, p.cur + s, S);
#undef lring
#undef ltab
#undef lrange
#undef llf
}

// every session at frame 0, nothing arrived, every player connected (SyncLayer::new,
// InputQueue::new, P2PSession::new: input_queue.rs:40-53, sync_layer.rs:183-198)
__global__ void sched_init_kernel(int32_t* sst, int64_t S, int32_t P) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)sched_fields(P) * S) return;
  const int f = (int)(i / S);
  int32_t v = kNull;
  if (f == kCur || f == kSkips || f == kErr || f == kDisc || f == kRmask || f == kLastCk) v = 0;  // (kLastSent: NULL_FRAME)
  sst[i] = v;
}

}  // namespace

namespace ggrs {

int p2p_sched_free(ggrs_p2p_engine* e) {
  void* bufs[] = {e->arrive, e->events, e->row_tag, e->iq, e->sst, e->rep_frame, e->rep_ck, e->rep_lconf, e->rep_ll, e->fck,
                  e->peer_reports};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  e->arrive = nullptr;
  e->events = nullptr;
  e->row_tag = nullptr;
  e->iq = nullptr;
  e->sst = nullptr;
  e->rep_frame = nullptr;
  e->rep_ck = nullptr;
  e->rep_lconf = nullptr;
  e->rep_ll = nullptr;
  e->fck = nullptr;
  e->peer_reports = nullptr;
  return GGRS_OK;
}

// desync detection under arrival schedules: the per-call report rows and the frames' final cell
// checksums (a launch of n <= cap calls reports frames >= its first frame - max_prediction - 1, so
// cap + max_prediction + 2 frames of them suffice)
int p2p_sched_desync_alloc(ggrs_p2p_engine* e) {
  if (e->rep_frame) return GGRS_OK;
  const int64_t S = e->cfg.num_sessions;
  HIP_TRY(hipSetDevice(e->cfg.device));
  int hf = 2;
  while (hf < e->cap + e->cfg.max_prediction + 2) hf *= 2;
  e->sched_hf = hf;
  HIP_TRY(hipMalloc(&e->rep_frame, sizeof(int32_t) * (size_t)e->cap * S));
  HIP_TRY(hipMalloc(&e->rep_ck, sizeof(uint16_t) * (size_t)e->cap * S));
  HIP_TRY(hipMalloc(&e->rep_lconf, sizeof(int32_t) * (size_t)e->cap * S));
  HIP_TRY(hipMalloc(&e->rep_ll, sizeof(int32_t) * (size_t)e->cap * S));
  HIP_TRY(hipMalloc(&e->fck, sizeof(uint16_t) * (size_t)hf * S));
  HIP_TRY(hipMemsetAsync(e->rep_frame, 0xff, sizeof(int32_t) * (size_t)e->cap * S, e->stream));
  HIP_TRY(hipMemsetAsync(e->rep_ck, 0, sizeof(uint16_t) * (size_t)e->cap * S, e->stream));
  HIP_TRY(hipMemsetAsync(e->fck, 0, sizeof(uint16_t) * (size_t)hf * S, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
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
  // stage geometry: B rows behind a stage's first call (a rollback's confirmed inputs reach back
  // max_prediction frames, a burst after a stall a few more), K calls per stage as many as keep the
  // block's LDS within its share of the CU -- at least 8
  const int P = e->cfg.num_players;
  int WL = 2;
  while (WL < e->cfg.max_prediction + e->cfg.input_delay + 2) WL *= 2;
  const int B = 2 * e->cfg.max_prediction + 4;
  // the LDS a block may take without costing residency: 160 KB per CU shared by the blocks each CU
  // must hold at once (65,536 sessions: four, one per SIMD -> 40 KB; 4,096 sessions: one -> all of it)
  const int64_t blocks = grid_of(e->cfg.num_sessions, kBlock);
  const int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(4, (blocks + e->num_cus - 1) / e->num_cus));
  const uint32_t budget = (uint32_t)(160 * 1024 / per_cu) - 1024;
  // and at most 64 - B, so that a stage's rows fit the control pass's 64-bit change masks (its fast form)
  // Two waves per block (the control pass of the next stage beside the step loop) when each CU holds
  // one block: its second wave runs on a SIMD that would idle (GGRS_SCHED_SPLIT=0 turns it off)
  const char* split_env = getenv("GGRS_SCHED_SPLIT");
  const bool split = !e->sparse && per_cu == 1 && blocks <= e->num_cus && !(split_env && split_env[0] == '0');
  const int nbuf = split ? 2 : 1;
  // (the two-wave form overlaps all but the first stage's control pass, but shorter stages cost the
  // step wave more than they hide: 4,096 sessions 180 / 170 / 158 / 156 / 156 us at 8 / 12 / 16 / 24
  // / 42 calls per stage, profiles/r05ak_k*)
  int K = std::max(8, std::min(64, 64 - B));
  while (K > 8 && sched_lds(P, e->R, e->sparse, WL, K, B, nbuf).total > budget) K -= 4;
  const size_t shm = sched_lds(P, e->R, e->sparse, WL, K, B, nbuf).total;
  if (shm > 160 * 1024) return set_error(GGRS_E_INVALID, "max_prediction too large for the scheduled kernel's LDS");
  SchedParams p;
  p.K = K;
  p.B = B;
  p.WL = WL;
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
  p.reports = e->peer_reports;
  p.lq = e->iq;
  p.sst = e->sst;
  p.rollbacks = e->rollbacks;
  p.resim = e->resim;
  p.TW = 0;
  p.interval = e->desync_interval;
  p.HF = e->sched_hf;
  p.rep_frame = e->rep_frame;
  p.rep_ck = e->rep_ck;
  p.rep_lconf = e->rep_lconf;
  p.rep_ll = e->rep_ll;
  p.fck = e->fck;
  p.trace = e->trace;
  p.trace_cap = e->trace ? e->cfg.trace_capacity : 0;
  // desync detection, peer reports or the display trace: the flat kernel with their code (a session's
  // standing reports, q.rmask, can only come from an engine given reports)
  const bool feat = p.interval > 0 || p.reports != nullptr || p.trace_cap > 0;
  if (int rc = e->timer.before(e->stream)) return rc;
  hipError_t attr = hipSuccess;
  // The time-aligned form (a session's replays on 16 lanes) for few sessions: when its blocks of 16
  // sessions fill at most two per CU.  GGRS_SCHED_CHAINS=0 keeps the one-thread-per-session form.
  int remote = 0;
  for (int k = 0; k < P; k++) remote += !((e->cfg.local_mask >> k) & 1);
  const char* chains_env = getenv("GGRS_SCHED_CHAINS");
  const int64_t cblocks = grid_of(e->cfg.num_sessions, kCS);
  // (lockstep mode, peer reports and the display trace take the one-thread-per-session form)
  const bool chains = !e->sparse && e->cfg.max_prediction >= 1 && e->cfg.max_prediction <= kMaxChainDepth && remote <= 2 &&
                      !e->peer_reports && !e->trace && !(chains_env && chains_env[0] == '0') &&
                      (cblocks <= 2 * (int64_t)e->num_cus || (chains_env && chains_env[0] == '1'));
  if (chains && n > kChainMaxCalls) {
    int rc = p2p_sched_advance(e, kChainMaxCalls);
    if (rc) return rc;
    return p2p_sched_advance(e, n - kChainMaxCalls);
  }
  if (chains) {
    // K calls per stage: the step waves trail the control wave by a stage, so shorter stages overlap
    // more of the two; the tables hold the frames of two stages + max_prediction + the delay
    const char* k_env = getenv("GGRS_SCHED_K");
    int Kc = k_env ? atoi(k_env) : 16;
    Kc = std::max(4, std::min(std::min(Kc, 64 - B), kChainMaxK));
    int TW = 16;
    while (TW < 2 * Kc + e->cfg.max_prediction + e->cfg.input_delay + 8) TW *= 2;
    const ChainLds cl = chain_lds(P, e->R, TW, Kc, B);
    if (cl.total > 160 * 1024) return set_error(GGRS_E_INVALID, "input_delay too large for the scheduled kernel's LDS");
    p.K = Kc;
    p.TW = TW;
    dispatch_players(P, [&](auto PC) {
      constexpr int PP = decltype(PC)::value;
      auto go = [&](auto kern) {
        if (cl.total > 64 * 1024)
          attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)cl.total);
        if (attr == hipSuccess) kern<<<(unsigned)cblocks, kChainThreads, cl.total, e->stream>>>(p);
      };
      auto go_f = [&](auto k0, auto k1) { feat ? go(k1) : go(k0); };  // (feat: desync detection here)
      if constexpr (PP == 2) {
        if (p.predictor == 0 && p.local_mask == 1u)
          return go_f(&p2p_sched_chains_kernel<PP, 0, 1, false>, &p2p_sched_chains_kernel<PP, 0, 1, true>);
        if (p.predictor == 0 && p.local_mask == 2u)
          return go_f(&p2p_sched_chains_kernel<PP, 0, 2, false>, &p2p_sched_chains_kernel<PP, 0, 2, true>);
      }
      if (p.predictor == 0) go_f(&p2p_sched_chains_kernel<PP, 0, -1, false>, &p2p_sched_chains_kernel<PP, 0, -1, true>);
      else go_f(&p2p_sched_chains_kernel<PP, 1, -1, false>, &p2p_sched_chains_kernel<PP, 1, -1, true>);
    });
    HIP_TRY(attr);
    HIP_TRY(hipGetLastError());
    e->timer.count();
    e->current_frame += n;
    return GGRS_OK;
  }
  dispatch_players(P, [&](auto PC) {
    constexpr int PP = decltype(PC)::value;
    auto go = [&](auto kern) {
      if (shm > 64 * 1024)
        attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)shm);
      if (attr == hipSuccess)
        kern<<<(unsigned)grid_of(p.S, kBlock), split ? 2 * kBlock : kBlock, shm, e->stream>>>(p);
    };
    // (split, features) -> the kernel; sparse saving keeps the features compiled in
    auto go4 = [&](auto k00, auto k01, auto k10, auto k11) {
      if (split) feat ? go(k11) : go(k10);
      else feat ? go(k01) : go(k00);
    };
    if (p.sparse) {
      if (p.predictor == 0) go(&p2p_sched_kernel<PP, true, 0, -1, false, true>);
      else go(&p2p_sched_kernel<PP, true, 1, -1, false, true>);
    } else {
      bool done = false;
      if constexpr (PP == 2) {  // one local player of two, repeat-last: the usual peer, masks compile-time
        if (p.predictor == 0 && (p.local_mask == 1u || p.local_mask == 2u)) {
          if (p.local_mask == 1u)
            go4(&p2p_sched_kernel<PP, false, 0, 1, false, false>, &p2p_sched_kernel<PP, false, 0, 1, false, true>,
                &p2p_sched_kernel<PP, false, 0, 1, true, false>, &p2p_sched_kernel<PP, false, 0, 1, true, true>);
          else
            go4(&p2p_sched_kernel<PP, false, 0, 2, false, false>, &p2p_sched_kernel<PP, false, 0, 2, false, true>,
                &p2p_sched_kernel<PP, false, 0, 2, true, false>, &p2p_sched_kernel<PP, false, 0, 2, true, true>);
          done = true;
        }
      }
      if (!done) {
        if (p.predictor == 0)
          go4(&p2p_sched_kernel<PP, false, 0, -1, false, false>, &p2p_sched_kernel<PP, false, 0, -1, false, true>,
              &p2p_sched_kernel<PP, false, 0, -1, true, false>, &p2p_sched_kernel<PP, false, 0, -1, true, true>);
        else
          go4(&p2p_sched_kernel<PP, false, 1, -1, false, false>, &p2p_sched_kernel<PP, false, 1, -1, false, true>,
              &p2p_sched_kernel<PP, false, 1, -1, true, false>, &p2p_sched_kernel<PP, false, 1, -1, true, true>);
      }
    }
  });
  HIP_TRY(attr);
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
  if (e->cfg.max_prediction + e->cfg.input_delay + 2 >= kQ)
    return set_error(GGRS_E_INVALID, "max_prediction + input_delay must be < %d (the device input queue)", kQ - 2);
  if (int rc = p2p_sched_enable(e)) return rc;
  return e->desync_interval > 0 ? p2p_sched_desync_alloc(e) : GGRS_OK;
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
    if (e->peer_reports)  // (a slot's report from cap calls ago is not this call's)
      HIP_TRY(hipMemsetAsync(e->peer_reports + (int64_t)slot * S, 0, sizeof(int32_t) * m * S, e->stream));
    k += m;
  }
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->next_arrival_call = first_call + n;
  return GGRS_OK;
}

int ggrs_p2p_add_peer_reports(ggrs_p2p_engine_t* e, int32_t first_call, int32_t n, const int32_t* reports) {
  if (!e || (!reports && n > 0)) return set_error(GGRS_E_INVALID, "null argument");
  if (!e->sched) return set_error(GGRS_E_STATE, "peer reports need ggrs_p2p_set_arrival_schedule(e, 1)");
  if (n < 0 || first_call < e->current_frame || first_call + n > e->next_arrival_call)
    return set_error(GGRS_E_INVALID, "peer reports are for calls not yet run whose arrivals were added (calls %d .. %d)",
                     e->current_frame, e->next_arrival_call - 1);
  if (e->cfg.predictor != 0)
    return set_error(GGRS_E_INVALID, "peer reports need the repeat-last predictor (a disconnected player's trimmed "
                                     "queue answers with its prediction, input_queue.rs:104-167)");
  const int P = e->cfg.num_players;
  const int64_t S = e->cfg.num_sessions;
  const uint32_t lm = (uint32_t)e->cfg.local_mask;
  for (int32_t c = 0; c < n; c++)
    for (int64_t s = 0; s < S; s++) {
      const int32_t v = reports[(int64_t)c * S + s];
      if (v == 0) continue;
      const int k = v & 3, r = (v >> 2) & 3;
      const int32_t f = (v >> 5) - 1;
      if (!(v & 16) || k >= P || r >= P || k == r || ((lm >> k) & 1u) || ((lm >> r) & 1u) || f < kNull ||
          f > first_call + c)
        return set_error(GGRS_E_INVALID, "bad peer report %d (call %d, session %lld): GGRS_PEER_REPORT(player, "
                         "reporter, frame) of two remote players, frame <= the call", v, first_call + c, (long long)s);
    }
  if (n == 0) return GGRS_OK;
  HIP_TRY(hipSetDevice(e->cfg.device));
  if (!e->peer_reports) {
    HIP_TRY(hipMalloc(&e->peer_reports, sizeof(int32_t) * (size_t)e->cap * S));
    HIP_TRY(hipMemsetAsync(e->peer_reports, 0, sizeof(int32_t) * (size_t)e->cap * S, e->stream));
  }
  for (int32_t k = 0; k < n;) {  // rows wrap at cap: at most two pieces
    const int32_t slot = (first_call + k) % e->cap;
    const int32_t m = std::min(n - k, e->cap - slot);
    HIP_TRY(hipMemcpyAsync(e->peer_reports + (int64_t)slot * S, reports + (int64_t)k * S, sizeof(int32_t) * m * S,
                           hipMemcpyHostToDevice, e->stream));
    k += m;
  }
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

int ggrs_p2p_read_reports(ggrs_p2p_engine_t* e, int32_t first_call, int32_t n, int32_t* frames, uint16_t* checksums,
                          int32_t* last_confirmed, int32_t* local_last) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (!e->sched || e->desync_interval <= 0 || !e->rep_frame)
    return set_error(GGRS_E_STATE, "per-session reports exist with arrival schedules and desync detection only");
  if (n < 0 || first_call < 0 || first_call + n > e->current_frame || first_call < e->current_frame - e->cap)
    return set_error(GGRS_E_INVALID, "calls %d .. %d are not among the last %d calls run (%d run)", first_call,
                     first_call + n - 1, e->cap, e->current_frame);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t S = e->cfg.num_sessions;
  for (int32_t k = 0; k < n;) {  // rows wrap at cap: at most two pieces
    const int32_t slot = (first_call + k) % e->cap;
    const int32_t m = std::min(n - k, e->cap - slot);
    const size_t off = (size_t)slot * S, dst = (size_t)k * S, cnt = (size_t)m * S;
    if (frames) HIP_TRY(hipMemcpyAsync(frames + dst, e->rep_frame + off, 4 * cnt, hipMemcpyDeviceToHost, e->stream));
    if (checksums)
      HIP_TRY(hipMemcpyAsync(checksums + dst, e->rep_ck + off, 2 * cnt, hipMemcpyDeviceToHost, e->stream));
    if (last_confirmed)
      HIP_TRY(hipMemcpyAsync(last_confirmed + dst, e->rep_lconf + off, 4 * cnt, hipMemcpyDeviceToHost, e->stream));
    if (local_last) HIP_TRY(hipMemcpyAsync(local_last + dst, e->rep_ll + off, 4 * cnt, hipMemcpyDeviceToHost, e->stream));
    k += m;
  }
  HIP_TRY(hipStreamSynchronize(e->stream));
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
