// branch.hip -- speculative branch rollback: the P2P rollback replay (P2PSession::adjust_gamestate,
// src/sessions/p2p_session.rs:658-714, + the save of the current frame, :337) for every
// (session, branch) lane, with InputQueue prediction (src/input_queue.rs:104-167,
// src/lib.rs:390-395) replaced by a branch generator:
//   * B == 1: PredictRepeatLast -- every remote player plays its last confirmed input;
//   * B == A^E: branch b assumes the first remote player plays digit_k = (b / A^k) % A on the
//     k-th speculated frame (k < E; held at digit_{E-1} afterwards); other remote players repeat.
// A round is speculate (each lane: Load the session trunk, W x (Advance, Save) into its own ring)
// then confirm (the remote inputs of the trunk frame arrive: the trunk is replayed one frame with
// them -- the rollback to first_incorrect GGRS performs -- and each lane learns whether its branch
// survived, i.e. assumed exactly those inputs).  The next speculate checks that every surviving
// lane's saved state for the new trunk frame has the trunk's checksum (desync detection).
//
// HBM layout (lane = session * B + branch, lane-fastest SoA):
//   trunk    [F][S]     u32  confirmed state of each session at trunk_frame
//   ring     [R][F][L]  u32  R = W + 1 saved states per lane, slot = frame % R
//   ring_ck  [R][L]     u16
//   inputs   [C][S][Pp] u8   true inputs of every player (remote ones are read only once confirmed)
//   report   [S] u16 trunk checksum | pad | [ceil(L/64)] u64 survival bits  -- the all-gather payload
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "common.h"

#pragma clang fp contract(off)

using namespace ggrs;

namespace {

struct SpecParams {
  int64_t S, L;
  int32_t B, W, R, A, E, cap, P;
  int32_t f_c;          // trunk frame
  uint32_t remote_mask; // bit p: player p is remote
  int32_t first_remote; // index of the enumerated remote player (-1: none)
  int32_t check_prev;   // 1: verify survivors of the previous confirm
  const uint32_t* trunk;
  uint32_t* ring;
  uint16_t* ring_ck;
  const uint8_t* inputs;
  const uint64_t* prev_survive;  // survival bits of the previous confirm
  const uint16_t* trunk_ck;      // checksum of the current trunk (previous confirm's report)
  int32_t* desync;               // per session: first frame whose survivor disagreed, or -1
};

// The remote-input byte of branch b on speculated frame k for the enumerated player.
// (A is a kernel parameter: a power-of-two alphabet, 16 in configs 3/4, takes a shift and a mask
// instead of kk + 1 integer divisions by a runtime divisor)
__device__ inline uint32_t branch_digit(int32_t b, int32_t k, int32_t A, int32_t E) {
  int32_t kk = k < E ? k : E - 1;
  if ((A & (A - 1)) == 0) return ((uint32_t)b >> (kk * __builtin_ctz((uint32_t)A))) & (uint32_t)(A - 1);
  int32_t v = b;
  for (int32_t q = 0; q < kk; q++) v /= A;
  return (uint32_t)(v % A);
}

// Inputs lane (s, b) plays on frame f_c + k: local players from the queue, remote players
// predicted.  GGRS predicts from the last input added to the player's queue (input_queue.rs:
// 128-161), i.e. the confirmed input of frame f_c - 1, or the default input before frame 0.
template <int P>
__device__ inline uint32_t branch_inputs_from(const SpecParams& p, uint32_t truth, uint32_t last, int32_t b,
                                              int32_t k) {
  uint32_t in = 0;
#pragma unroll
  for (int q = 0; q < P; q++) {
    uint32_t v;
    if (!((p.remote_mask >> q) & 1u)) v = (truth >> (8 * q)) & 0xffu;          // local: confirmed
    else if (q == p.first_remote && p.B > 1) v = branch_digit(b, k, p.A, p.E);  // enumerated
    else v = (last >> (8 * q)) & 0xffu;                                         // repeat last
    in |= v << (8 * q);
  }
  return in;
}
template <int P>
__device__ inline uint32_t branch_inputs(const SpecParams& p, int64_t s, int32_t b, int32_t k) {
  const uint32_t truth = load_inputs<P>(p.inputs, (int64_t)((p.f_c + k) % p.cap) * p.S + s);
  const uint32_t last = p.f_c > 0 ? load_inputs<P>(p.inputs, (int64_t)((p.f_c - 1) % p.cap) * p.S + s) : 0u;
  return branch_inputs_from<P>(p, truth, last, b, k);
}

// The branch whose cell holds branch b's depth-k state (B = A^E): branches sharing their first
// k + 1 digits share it, and prefix_pipe_kernel saves it once, by the prefix's representative.
// The representatives of depth k < E - 1 are the A^(k+1) consecutive branches starting at
// base_k = A^(k+2) + ... + A^(E-1) (depth E - 2 at branch 0, each shallower depth right after the
// deeper one's range): base_k is a multiple of A^(k+1), so branch base_k + (b mod A^(k+1)) has
// b's prefix, and every depth's representatives fill whole waves of their own -- no wave
// represents two depths below E - 1, so no wave saves more than two cells per super-step (with
// every shallow depth at branch 0, branch 0's wave saved W of them and set the launch's pace).
// Depth >= E - 1 (and no enumeration): b itself.
__host__ __device__ inline int64_t rep_branch(int64_t b, int k, int64_t A, int E) {
  if (E <= 0 || k >= E - 1) return b;
  int64_t q = 1, base = 0;
  for (int j = 0; j < E - 1; j++) {
    q *= A;                        // A^(j+1)
    if (j > k) base += q;          // depths deeper than k, below E - 1
  }
  int64_t qk = 1;
  for (int j = 0; j <= k; j++) qk *= A;  // A^(k+1)
  return base + b % qk;
}

// The lane whose ring holds branch b's depth-0 cell (the state after the first speculated frame).
__device__ inline int64_t rep0_lane(const SpecParams& p, int64_t s, int32_t b) {
  return s * p.B + rep_branch(b, 0, p.A, p.E);
}

template <int P>
__global__ __launch_bounds__(256) void speculate_kernel(SpecParams p) {
  const int64_t lane = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= p.L) return;
  const int64_t s = lane / p.B;
  const int32_t b = (int32_t)(lane - s * p.B);
  constexpr int F = state_fields(P);
  if (p.check_prev && ((p.prev_survive[lane >> 6] >> (lane & 63)) & 1ull)) {
    // a surviving branch already saved the new trunk frame: it must match the replayed trunk (the
    // cell of its depth-0 representative, which prefix-shared rounds save for every such branch)
    const uint16_t mine = p.ring_ck[(int64_t)(p.f_c % p.R) * p.L + rep0_lane(p, s, b)];
    if (mine != p.trunk_ck[s]) atomicCAS(&p.desync[s], -1, p.f_c);
  }
  BoxState<P> st;
  load_state<P>(st, p.trunk + s, p.S);  // LoadGameState(f_c)
  for (int32_t k = 0; k < p.W; ++k) {
    advance_state<P>(st, branch_inputs<P>(p, s, b, k), 0u);  // AdvanceFrame(f_c + k)
    const int32_t slot = (p.f_c + k + 1) % p.R;                 // SaveGameState(f_c + k + 1)
    store_state<P>(st, p.ring + (int64_t)slot * F * p.L + lane, p.L);
    p.ring_ck[(int64_t)slot * p.L + lane] = fletcher16_state<P>(st);
  }
}

struct ConfirmParams {
  int64_t S, L;
  int32_t B, A, E, cap, P;
  int32_t f_c;
  uint32_t remote_mask;
  int32_t first_remote;
  uint32_t* trunk;
  const uint8_t* inputs;
  uint16_t* report_ck;   // [S]
  uint64_t* report_bits; // [ceil(L/64)]
};

// The remote inputs of frame f_c have arrived.  Branch survival: the lane assumed exactly the
// confirmed inputs for f_c (what add_input_by_frame checks, input_queue.rs:199-218).  Branch
// lane 0 of each session replays frame f_c with them into the new trunk and reports its checksum.
template <int P>
__global__ __launch_bounds__(256) void confirm_kernel(ConfirmParams p) {
  const int64_t lane = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in_range = lane < p.L;
  const int64_t s = in_range ? lane / p.B : 0;
  const int32_t b = in_range ? (int32_t)(lane - s * p.B) : 0;
  bool survive = false;
  if (in_range) {
    const uint32_t truth = load_inputs<P>(p.inputs, (int64_t)(p.f_c % p.cap) * p.S + s);
    const uint32_t last = p.f_c > 0 ? load_inputs<P>(p.inputs, (int64_t)((p.f_c - 1) % p.cap) * p.S + s) : 0u;
    survive = true;
#pragma unroll
    for (int q = 0; q < P; q++) {
      if (!((p.remote_mask >> q) & 1u)) continue;
      const uint32_t assumed = (q == p.first_remote && p.B > 1) ? branch_digit(b, 0, p.A, p.E)
                                                                : (last >> (8 * q)) & 0xffu;
      survive = survive && assumed == ((truth >> (8 * q)) & 0xffu);
    }
    if (b == 0) {
      BoxState<P> st;
      load_state<P>(st, p.trunk + s, p.S);
      advance_state<P>(st, truth, 0u);
      store_state<P>(st, p.trunk + s, p.S);
      p.report_ck[s] = fletcher16_state<P>(st);
    }
  }
  const uint64_t bits = __ballot(survive);
  if (in_range && (threadIdx.x & 63) == 0) p.report_bits[lane >> 6] = bits;
}

// n rounds of speculate + confirm in one launch (ggrs_branch_rounds on one GPU, where no exchange
// sits between rounds).  The only data a round passes across blocks is each session's trunk; every
// block keeps the trunks of its own sessions in LDS and replays them itself (the confirm step,
// done once per block instead of once per session: a few advances per block per round), and the
// block holding a session's branch-0 lane writes that trunk and its checksum out, as
// confirm_kernel does.  Survival bits pass from a round to the next in registers.  Rings, reports,
// trunks and desync records end exactly as after n speculate_kernel + confirm_kernel launches.
struct RoundsParams {
  SpecParams sp;  // sp.f_c: trunk frame of the first round
  int32_t n;
  uint32_t* trunk;
  uint16_t* report_ck;
  uint64_t* report_bits;
  uint16_t* copy_ck;    // optional second destination of the reports (the caller's exchange
  uint64_t* copy_bits;  // buffer, same layout): saves a device-to-device copy per round
  int64_t copy_stride;  // bytes between rounds' reports there (0: only the last round's)
};
constexpr int kRoundsBlock = 256;

template <int P>
__global__ __launch_bounds__(kRoundsBlock) void rounds_kernel(RoundsParams rp) {
  constexpr int F = state_fields(P);
  __shared__ uint32_t lds_trunk[kRoundsBlock][F];  // the block's sessions (<= 256)
  __shared__ uint16_t lds_ck[kRoundsBlock];
  const SpecParams& p = rp.sp;
  const int64_t lane0 = (int64_t)blockIdx.x * kRoundsBlock;
  const int64_t lane = lane0 + threadIdx.x;
  const bool in_range = lane < p.L;
  const int64_t s_first = lane0 / p.B;
  const int64_t s_last = (min(p.L, lane0 + kRoundsBlock) - 1) / p.B;
  const int ns = (int)(s_last - s_first + 1);
  const int64_t s = in_range ? lane / p.B : s_first;
  const int32_t b = (int32_t)(lane - s * p.B);
  const int ls = (int)(s - s_first);
  for (int q = threadIdx.x; q < ns * F; q += kRoundsBlock) {
    const int sl = q / F, k = q - sl * F;
    lds_trunk[sl][k] = p.trunk[(int64_t)k * p.S + s_first + sl];
  }
  bool survived = p.check_prev && in_range && ((p.prev_survive[lane >> 6] >> (lane & 63)) & 1ull);
  // every state the launch steps descends from the block's trunks, which this engine produced:
  // one block-wide test of their rotation domain instead of a wave vote per player per step
  bool trunk_ok = true;
  if ((int)threadIdx.x < ns) {
    BoxState<P> t0;
#pragma unroll
    for (int k = 0; k < F; k++) t0.w[k] = p.trunk[(int64_t)k * p.S + s_first + threadIdx.x];
    trunk_ok = rot_in_domain<P>(t0);
    // the trunk's checksum (the first round's survivor check) from the trunk itself: the report
    // buffer may already hold another block's first-round checksum
    lds_ck[threadIdx.x] = fletcher16_state<P>(t0);
  }
  const bool lean_ok = __syncthreads_and(trunk_ok);
  // input-queue rows and ring slots as wave-uniform counters (no runtime-divisor modulo per step):
  // row_c = f_c % cap, slot_c = f_c % R of the round's trunk frame
  auto wrap_inc = [](int32_t x, int32_t m) { return x + 1 == m ? 0 : x + 1; };
  int32_t row_c = p.f_c % p.cap, slot_c = p.f_c % p.R;
  // the last confirmed input row (f_c - 1) and the round's truth row (f_c); each round loads the
  // next round's truth row while it speculates
  uint32_t last = p.f_c > 0 ? load_inputs<P>(p.inputs, (int64_t)(row_c == 0 ? p.cap - 1 : row_c - 1) * p.S + s) : 0u;
  uint32_t truth = load_inputs<P>(p.inputs, (int64_t)row_c * p.S + s);
  const bool trunk_thread = (int)threadIdx.x < ns;
  const int64_t s2 = s_first + (trunk_thread ? threadIdx.x : 0);
  const int64_t rep0 = in_range ? rep0_lane(p, s, b) : 0;
  for (int32_t r = 0; r < rp.n; ++r) {
    SpecParams q = p;
    q.f_c = p.f_c + r;
    const int32_t row_n = wrap_inc(row_c, p.cap);
    const uint32_t truth_next = r + 1 < rp.n ? load_inputs<P>(p.inputs, (int64_t)row_n * p.S + s) : 0u;
    // speculate_kernel's check of the last survivors: the cell of f_c is not re-saved by this
    // round (its saves go to the W slots after it), so its load is issued here and compared after
    // the replays, while its latency is hidden behind them
    const bool check = (r > 0 || p.check_prev) && survived;
    // (the first round's cell was saved by an earlier launch, possibly only by the representative
    // of a prefix-shared launch; later rounds' by this lane itself -- another block's lanes may be
    // at another round of this launch)
    const uint16_t mine = check ? p.ring_ck[(int64_t)slot_c * p.L + (r == 0 ? rep0 : lane)] : (uint16_t)0;
    // the confirm step's trunk replay (the next round's trunk: AdvanceFrame(f_c) with the true
    // inputs) depends only on this round's trunk, so the block's trunk threads run it beside the
    // speculation instead of after it; it reaches LDS after every lane has loaded the old trunk
    BoxState<P> tr;
    uint16_t tr_ck = 0;
    if (trunk_thread) {
#pragma unroll
      for (int k = 0; k < F; k++) tr.w[k] = lds_trunk[threadIdx.x][k];
      const uint32_t tin = load_inputs<P>(p.inputs, (int64_t)row_c * p.S + s2);
      if (lean_ok) advance_state_lean<P>(tr, tin);
      else advance_state<P>(tr, tin, 0u);
      tr_ck = fletcher16_state<P>(tr);
    }
    BoxState<P> st;
#pragma unroll
    for (int k = 0; k < F; k++) st.w[k] = lds_trunk[ls][k];  // LoadGameState(f_c)
    if (in_range) {
      uint32_t tk = truth;
      int32_t row_k = row_c, slot = slot_c;
      for (int32_t k = 0; k < p.W; ++k) {
        row_k = wrap_inc(row_k, p.cap);  // row of frame f_c + k + 1
        slot = wrap_inc(slot, p.R);      // slot of frame f_c + k + 1
        const uint32_t next = k + 1 < p.W ? load_inputs<P>(p.inputs, (int64_t)row_k * p.S + s) : 0u;
        const uint32_t in = branch_inputs_from<P>(q, tk, last, b, k);  // AdvanceFrame(f_c + k)
        if (lean_ok) advance_state_lean<P>(st, in);
        else advance_state<P>(st, in, 0u);
        // SaveGameState(f_c + k + 1) into `slot`
        store_state<P>(st, p.ring + (int64_t)slot * F * p.L + lane, p.L);
        p.ring_ck[(int64_t)slot * p.L + lane] = fletcher16_state<P>(st);
        tk = next;
      }
    }
    if (check && mine != lds_ck[ls]) atomicCAS(&p.desync[s], -1, q.f_c);
    // confirm: survival of every lane
    bool survive = false;
    if (in_range) {
      survive = true;
#pragma unroll
      for (int qq = 0; qq < P; qq++) {
        if (!((p.remote_mask >> qq) & 1u)) continue;
        const uint32_t assumed = (qq == p.first_remote && p.B > 1) ? branch_digit(b, 0, p.A, p.E)
                                                                   : (last >> (8 * qq)) & 0xffu;
        survive = survive && assumed == ((truth >> (8 * qq)) & 0xffu);
      }
    }
    const uint64_t bits = __ballot(survive);
    if (in_range && (threadIdx.x & 63) == 0) {
      rp.report_bits[lane >> 6] = bits;
      if (rp.copy_bits && (rp.copy_stride || r + 1 == rp.n))
        reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(rp.copy_bits) + r * rp.copy_stride)[lane >> 6] = bits;
    }
    survived = survive;
    __syncthreads();  // every lane has read the trunk and its checksum
    if (trunk_thread) {
#pragma unroll
      for (int k = 0; k < F; k++) lds_trunk[threadIdx.x][k] = tr.w[k];
      lds_ck[threadIdx.x] = tr_ck;
      if (s2 * p.B >= lane0) {  // this block holds the session's branch-0 lane
        store_state<P>(tr, rp.trunk + s2, p.S);
        rp.report_ck[s2] = tr_ck;
        if (rp.copy_ck && (rp.copy_stride || r + 1 == rp.n))
          reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(rp.copy_ck) + r * rp.copy_stride)[s2] = tr_ck;
      }
    }
    __syncthreads();
    last = truth;
    truth = truth_next;
    row_c = wrap_inc(row_c, p.cap);
    slot_c = wrap_inc(slot_c, p.R);
  }
}

// Prefix-shared rounds, pipelined (ggrs_branch_rounds when the enumerated player is the only
// remote one: config 3).  Two facts about a round make most of its work common to many lanes:
//   * players are independent in State::advance (ex_game.rs:276-331 updates player i from its own
//     fields and input only) and every player except the enumerated one plays the session's
//     confirmed inputs, so the local players' part of every depth-k cell is the trunk's local
//     players one frame later -- the same in every branch of the session;
//   * branch b's enumerated player plays digits d_0 .. d_k up to frame f_c + k, so branches sharing
//     their first k + 1 digits hold the same state after k + 1 frames: A^min(k+1, E) distinct cells
//     per session at depth k (config 3: 16, 256, 4096, 65,536 of the 4 x 65,536 logical saves),
//     saved by the prefix's representative (rep_branch) of the same session
//     (ggrs_branch_read_lane resolves a lane's cell to it).
// A round is W dependent steps (speculated frames); consecutive rounds are independent given their
// trunks, and round r's trunk is the confirmed replay of round r - 1's -- inputs only.  So the
// kernel runs the rounds as a pipeline: super-step u advances, on every lane, stage k of round
// u - k for every k < W (W independent enumerated-player steps, the only state chains: stage k
// takes stage k - 1's state of the previous super-step, stage 0 the trunk) and the trunk itself
// one frame (all players, confirmed inputs: the local players of every cell saved in super-step
// u, the next round's stage-0 state, the round's report).  Every stage of super-step u saves the
// same frame f_c + u + 1 (round u - k's depth k), in sequential order (the deepest stage -- the
// oldest round -- first, as the rounds would), so rings, ring checksums, trunks, reports, survivor
// sets and desync records end exactly as after n rounds of speculate_kernel + confirm_kernel.
// One wave per SIMD runs W + P independent player steps per super-step instead of W dependent
// ones per round, and no lane waits for another wave: no LDS window, no barrier in the loop (the
// trunk is replayed on every lane of the session -- the SIMD runs the whole wave's instruction
// stream once whatever its lanes hold).  The launch's input rows are staged in LDS in the prologue
// (a global load inside the loop would wait for the wave's saves: loads and stores retire in
// order on the vmcnt counter).  WT > 0 fixes W at compile time (config 3: W = 4); WT = 0 serves
// W <= kPipeMaxW with uniform per-stage guards.
constexpr int kPipeMaxW = 8;
constexpr uint32_t kPipeOob = 0x40000000u;  // past every descriptor's range: a lane that never stores

__device__ inline __amdgpu_buffer_rsrc_t prefix_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

template <int P, int EP, int WT, bool kPair>
__global__ __launch_bounds__(kRoundsBlock) void prefix_pipe_kernel(RoundsParams rp);

// A session's desync record keeps the earliest frame with a disagreeing survivor.  The prefix kernel
// spreads one session over many blocks, which reach a super-step at different times, so the record
// is a minimum (NULL_FRAME = -1 is the largest unsigned value), not a first-come CAS.
__device__ inline void desync_min(int32_t* dst, int32_t frame) {
  atomicMin(reinterpret_cast<unsigned int*>(dst), (unsigned int)frame);
}

// f(integral_constant<int, 0>) .. f(integral_constant<int, N - 1>)
template <int N, int I = 0, typename Fn>
__device__ inline void static_for(Fn&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>());
    static_for<N, I + 1>(f);
  }
}

// kPair (two players, an even branch count: lanes 2i and 2i + 1 belong to the same session): the
// trunk's two players are split over the lane pair -- the even lane steps player 0, the odd lane
// player 1, and each takes the other's new fields with one DPP swap per field -- instead of every
// lane stepping both (the trunk is the same on every lane of a session).
template <int P, int EP, int WT, bool kPair>
__global__ __launch_bounds__(kRoundsBlock) void prefix_pipe_kernel(RoundsParams rp) {
  static_assert(EP >= 0 && EP < P, "enumerated player");
  static_assert(!kPair || P == 2, "the lane-pair trunk split is for two players");
  constexpr int F = state_fields(P);
  constexpr int n_bytes = Fletcher<P>::n;
  constexpr int e = EP;
  constexpr int KW = WT > 0 ? WT : kPipeMaxW;
  extern __shared__ uint32_t lds_rows[];  // [n + W - 1][ns]: confirmed inputs of f_c .. f_c + n + W - 2
  const SpecParams& p = rp.sp;
  const int W = WT > 0 ? WT : p.W;
  const int n = rp.n;
  const int64_t lane0 = (int64_t)blockIdx.x * kRoundsBlock;
  const int64_t lane = lane0 + threadIdx.x;
  const bool in_range = lane < p.L;
  const int64_t s_first = lane0 / p.B;
  const int64_t s_last = (min(p.L, lane0 + kRoundsBlock) - 1) / p.B;
  const int ns = (int)(s_last - s_first + 1);
  const int64_t s = in_range ? lane / p.B : s_first;
  const int32_t b = in_range ? (int32_t)(lane - s * p.B) : 0;
  const int ls = (int)(s - s_first);
  // the prologue's global reads issued together (one memory latency): the lane's trunk, the
  // survivor bit and cell checksum of the first round's check, the launch's input rows
  BoxState<P> T;  // the trunk of the lane's session at frame f_c + u (every lane holds its own copy)
  load_state<P>(T, p.trunk + s, p.S);
  // (the first round's cell was saved by an earlier launch: its representative's; read whether or
  // not the lane survived, so that no load waits for another)
  const uint64_t prev_bits = p.check_prev && in_range ? p.prev_survive[lane >> 6] : 0ull;
  const uint16_t cell0 = p.check_prev ? p.ring_ck[(int64_t)(p.f_c % p.R) * p.L + rep0_lane(p, s, b)] : (uint16_t)0;
  {
    const int n_rows = n + W - 1;
    const int32_t row0 = p.f_c % p.cap;
    for (int i = threadIdx.x; i < n_rows * ns; i += kRoundsBlock) {
      const int k = i / ns, xs = i - k * ns;
      const int32_t row = row0 + k >= p.cap ? row0 + k - p.cap : row0 + k;
      lds_rows[i] = load_inputs<P>(p.inputs, (int64_t)row * p.S + s_first + xs);
    }
  }
  __syncthreads();
  bool survived = p.check_prev && in_range && ((prev_bits >> (lane & 63)) & 1ull);
  const bool check0 = p.check_prev && survived;
  const uint16_t mine0 = check0 ? cell0 : (uint16_t)0;
  // every state a wave steps descends from its lanes' trunks (produced by this engine): one test of
  // their rotation domain per wave, then the lean step throughout
  const bool lean_ok = __all(rot_in_domain<P>(T));
  constexpr int kq[5] = {fld_x(P, e), fld_y(P, e), fld_vx(P, e), fld_vy(P, e), fld_rot(P, e)};
  uint32_t wt[5];
#pragma unroll
  for (int q = 0; q < 5; q++) wt[q] = 2u * weights_at(n_bytes, fld_offset(P, kq[q]));
  // per-stage constants: the digit stage k plays, and whether this lane represents its depth-k prefix
  // (per-lane conditions live as VGPR offsets and one scalar bit set, not as 64-bit lane masks:
  // the loop's scalar registers would otherwise spill to VGPR lanes)
  uint32_t din[KW], off[KW], off_ck[KW];
  InputRec srec[KW];  // stage k's input decoded once: its digit is the lane's for the launch
  uint32_t wave_reps = 0;  // bit k: some lane of this wave represents its depth-k prefix
  {
#pragma unroll
    for (int k = 0; k < KW; k++) {
      din[k] = branch_digit(b, k, p.A, p.E);
      srec[k] = make_input_rec(din[k]);
      const bool rep = in_range && rep_branch(b, k, p.A, p.E) == b;
      off[k] = rep ? (uint32_t)(lane * 4) : kPipeOob;
      off_ck[k] = rep ? (uint32_t)(lane * 2) : kPipeOob;
      wave_reps |= (__builtin_amdgcn_ballot_w64(rep) != 0 ? 1u : 0u) << k;
    }
  }
  wave_reps = __builtin_amdgcn_readfirstlane(wave_reps);
  const uint32_t slot_bytes = (uint32_t)(F * p.L * 4);
  const __amdgpu_buffer_rsrc_t rs_ring = prefix_rsrc(p.ring, slot_bytes * (uint32_t)p.R);
  const __amdgpu_buffer_rsrc_t rs_ck = prefix_rsrc(p.ring_ck, (uint32_t)(2 * p.L * p.R));
  const uint32_t fstride = (uint32_t)(p.L * 4);
  const bool branch0 = in_range && b == 0;  // writes the session's trunk and report
  const bool podd = (threadIdx.x & 1) != 0;  // kPair: this lane steps the trunk's player 1
  // per-lane destinations (VGPR pointers: the loop's scalar registers are taken by its counters,
  // descriptors and masks, and uniform pointers kept there spilled to VGPR lanes)
  uint64_t* const bits_dst = rp.report_bits + (lane >> 6);
  uint8_t* const bits_copy = rp.copy_bits ? reinterpret_cast<uint8_t*>(rp.copy_bits + (lane >> 6)) : nullptr;
  uint32_t* const trunk_dst = rp.trunk + s;
  uint16_t* const ck_dst = rp.report_ck + s;
  uint8_t* const ck_copy = rp.copy_ck ? reinterpret_cast<uint8_t*>(rp.copy_ck + s) : nullptr;
  int32_t* const desync_dst = p.desync + s;
  const int64_t copy_stride = rp.copy_stride;

  // the doubled Fletcher sums of a cell's common part (frame + local players + length prefixes)
  auto common_sums = [&](const BoxState<P>& t, uint32_t& d1, uint32_t& d2) {
    d1 = 2u * Fletcher<P>::kSum1Const;
    d2 = 2u * Fletcher<P>::kSum2Const;
#pragma unroll
    for (int k = 0; k < F; k++) {
      bool mine = false;
#pragma unroll
      for (int q = 0; q < 5; q++) mine = mine || k == kq[q];
      if (mine) continue;
      d1 = dot4_u8(t.w[k], 0x02020202u, d1);
      d2 = dot4_u8(t.w[k], 2u * weights_at(n_bytes, fld_offset(P, k)), d2);
    }
  };
  auto enum_ck = [&](uint32_t d1, uint32_t d2, const uint32_t (&v)[5]) {
#pragma unroll
    for (int q = 0; q < 5; q++) {
      d1 = dot4_u8(v[q], 0x02020202u, d1);
      d2 = dot4_u8(v[q], wt[q], d2);
    }
    return fletcher_from_doubled<true>(d1, d2);  // (the 24-bit multiply-add form: 8 % faster here)
  };

  auto run = [&](auto lean_tag) {
    constexpr bool kLean = decltype(lean_tag)::value;
    auto adv = [&](uint32_t (&v)[5], uint32_t in) {
      float x = __builtin_bit_cast(float, v[0]), y = __builtin_bit_cast(float, v[1]);
      float vx = __builtin_bit_cast(float, v[2]), vy = __builtin_bit_cast(float, v[3]);
      float rot = __builtin_bit_cast(float, v[4]);
      if constexpr (kLean) advance_player_lean(x, y, vx, vy, rot, in);
      else advance_player_general(x, y, vx, vy, rot, in);
      v[0] = __builtin_bit_cast(uint32_t, x);
      v[1] = __builtin_bit_cast(uint32_t, y);
      v[2] = __builtin_bit_cast(uint32_t, vx);
      v[3] = __builtin_bit_cast(uint32_t, vy);
      v[4] = __builtin_bit_cast(uint32_t, rot);
    };
    uint32_t est[KW][5];  // stage k: the enumerated player of round u - k after its step k
#pragma unroll
    for (int k = 0; k < KW; k++)
#pragma unroll
      for (int q = 0; q < 5; q++) est[k][q] = 0u;
    int32_t slot = p.f_c % p.R;
    // the confirmed row of super-step u, read one super-step ahead (its LDS latency behind the
    // previous super-step's steps rather than in front of this one's trunk replay)
    const int32_t last_row = n + W - 2;
    uint32_t row_next = lds_rows[ls];
    const SincosConsts sck = sincos_consts_vgpr();
    // one super-step; kGuard: some stage belongs to no round of this launch (ramp / drain).  Only
    // stages [K0, K1) are stepped (the ramp and drain of a compile-time W step just the stages that
    // hold a round: a stage without one feeds only stages without one), and the trunk's enumerated
    // player only when kTE (in the drain no round reads the trunk's own enumerated player: stage 0
    // is idle and every save replaces those fields with its stage's)
    auto super_step = [&](int32_t u, auto guard_tag, auto k0_c, auto k1_c, auto te_c) {
      constexpr bool kGuard = decltype(guard_tag)::value;
      constexpr int K0 = decltype(k0_c)::value, K1 = decltype(k1_c)::value;
      constexpr bool kTE = decltype(te_c)::value;
      auto active = [&](int k) { return k >= K0 && k < K1 && (!kGuard || (k < W && u - k >= 0 && u - k < n)); };
      const int32_t f_c = p.f_c + u;  // round u's trunk frame; every save is frame f_c + 1
      const uint32_t row = row_next;
      row_next = lds_rows[min(u + 1, last_row) * ns + ls];
      slot = slot + 1 == p.R ? 0 : slot + 1;
      if (active(0)) {
        // speculate_kernel's check of round u - 1's survivors: the Fletcher-16 of their depth-0
        // cell against the replayed trunk's (GGRS compares checksums, p2p_session.rs:904-937).  The
        // cell's local players ARE the trunk's, so equal enumerated-player bits mean equal
        // checksums; only a lane whose bits differ (wave-uniform branch, never taken in a
        // deterministic run) compares the two checksums, so a collision is no desync here either
        // 
        bool same = true;
#pragma unroll
        for (int q = 0; q < 5; q++) same = same && est[0][q] == T.w[kq[q]];
        const bool differs = u > 0 && survived && !same;
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(differs) != 0, 0)) {
          if (differs) {
            uint32_t d1, d2, v[5];
            common_sums(T, d1, d2);
#pragma unroll
            for (int q = 0; q < 5; q++) v[q] = T.w[kq[q]];
            if (enum_ck(d1, d2, est[0]) != enum_ck(d1, d2, v)) desync_min(desync_dst, f_c);
          }
        }
        if (u == 0 && check0) {
          uint32_t d1, d2, v[5];
          common_sums(T, d1, d2);
#pragma unroll
          for (int q = 0; q < 5; q++) v[q] = T.w[kq[q]];
          if (mine0 != (uint16_t)enum_ck(d1, d2, v)) desync_min(desync_dst, f_c);
        }
      }
      // the stages' steps (round u - k's AdvanceFrame(f_c) with digit k: stage k takes stage k - 1's
      // state of the previous super-step, stage 0 the trunk's enumerated player) and the trunk's
      // confirmed replay of frame f_c (every player), as independent player steps
      // xs: stages K0 .. K1 - 1, then the trunk's players (all, or all but the enumerated one)
      constexpr bool kSplit = kPair && kTE;  // the trunk's two players over the lane pair
      constexpr int NK = K1 - K0, NT = kSplit ? 1 : (kTE ? P : P - 1), NS = NK + NT;
      uint32_t xs[NS][5], xin[NS];
      InputRec xrec[NS];
#pragma unroll
      for (int k = K0; k < K1; k++) {
#pragma unroll
        for (int q = 0; q < 5; q++) xs[k - K0][q] = k == 0 ? T.w[kq[q]] : est[k - 1][q];
        xin[k - K0] = din[k];
        xrec[k - K0] = srec[k];
      }
      auto trunk_index = [](int q) { return NK + (kTE || q < e ? q : q - 1); };
      constexpr int fk0[5] = {fld_x(P, 0), fld_y(P, 0), fld_vx(P, 0), fld_vy(P, 0), fld_rot(P, 0)};
      constexpr int fk1[5] = {fld_x(P, 1 % P), fld_y(P, 1 % P), fld_vx(P, 1 % P), fld_vy(P, 1 % P), fld_rot(P, 1 % P)};
      if constexpr (kSplit) {
#pragma unroll
        for (int u5 = 0; u5 < 5; u5++) xs[NK][u5] = podd ? T.w[fk1[u5]] : T.w[fk0[u5]];
        xin[NK] = (podd ? row >> 8 : row) & 0xffu;
        xrec[NK] = make_input_rec(xin[NK]);
      } else {
#pragma unroll
        for (int q = 0; q < P; q++) {
          if (!kTE && q == e) continue;
          const int fk[5] = {fld_x(P, q), fld_y(P, q), fld_vx(P, q), fld_vy(P, q), fld_rot(P, q)};
          const int i = trunk_index(q);
#pragma unroll
          for (int u5 = 0; u5 < 5; u5++) xs[i][u5] = T.w[fk[u5]];
          xin[i] = (row >> (8 * q)) & 0xffu;
          xrec[i] = make_input_rec(xin[i]);
        }
      }
      if constexpr (kLean) {
        advance_players_rec<NS>(xs, xrec, sck);
      } else {
#pragma unroll
        for (int i = 0; i < NS; i++) adv(xs[i], xin[i]);
      }
#pragma unroll
      for (int k = K0; k < K1; k++)
#pragma unroll
        for (int q = 0; q < 5; q++) est[k][q] = xs[k - K0][q];
      BoxState<P> Tn = T;  // (!kTE: the enumerated player's fields stay stale, never read)
      Tn.w[0] = (uint32_t)(f_c + 1);
      if constexpr (kSplit) {
#pragma unroll
        for (int u5 = 0; u5 < 5; u5++) {
          const uint32_t mine = xs[NK][u5];
          const uint32_t other = (uint32_t)__builtin_amdgcn_mov_dpp((int)mine, 0xB1, 0xF, 0xF, false);  // xor 1
          Tn.w[fk0[u5]] = podd ? other : mine;
          Tn.w[fk1[u5]] = podd ? mine : other;
        }
      } else {
#pragma unroll
        for (int q = 0; q < P; q++) {
          if (!kTE && q == e) continue;
          const int fk[5] = {fld_x(P, q), fld_y(P, q), fld_vx(P, q), fld_vy(P, q), fld_rot(P, q)};
#pragma unroll
          for (int u5 = 0; u5 < 5; u5++) Tn.w[fk[u5]] = xs[trunk_index(q)][u5];
        }
      }
      uint32_t c1, c2;
      common_sums(Tn, c1, c2);
      // SaveGameState(f_c + 1) of every stage, the oldest round first; a depth-k cell only by the
      // representatives of its prefix (wave-uniform skip when a wave holds none)
      const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)slot * slot_bytes);
      const uint32_t so_ck = __builtin_amdgcn_readfirstlane((uint32_t)slot * (uint32_t)(2 * p.L));
#pragma unroll
      for (int k = KW - 1; k >= 0; k--) {
        if (!active(k) || k >= W) continue;
        if (!((wave_reps >> k) & 1u)) continue;
        const uint32_t ck = enum_ck(c1, c2, est[k]);
        const uint32_t o = off[k], o_ck = off_ck[k];
        // write-through (sc1): the saves reach memory while the launch runs instead of in the
        // end-of-kernel L2 write-back of every line the launch dirtied (config 3: 26.8 -> 25.2 us
        // per 16-round launch, profiles/r04h)
#pragma unroll
        for (int f = 0; f < F; f++) {
          uint32_t v = Tn.w[f];
#pragma unroll
          for (int q = 0; q < 5; q++)
            if (f == kq[q]) v = est[k][q];
          __builtin_amdgcn_raw_buffer_store_b32(v, rs_ring, o + (uint32_t)f * fstride, so, kStoreWriteThrough);
        }
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)ck, rs_ck, o_ck, so_ck, kStoreWriteThrough);
      }
      if (active(0)) {
        // confirm of round u: a lane survives iff it assumed the confirmed input of f_c
        // (input_queue.rs:199-218); branch 0 writes the new trunk and its checksum
        const bool survive = in_range && din[0] == ((row >> (8 * e)) & 0xffu);
        const uint64_t bits = __ballot(survive);
        if (in_range && (threadIdx.x & 63) == 0) {
          *bits_dst = bits;
          if (bits_copy && (copy_stride || u + 1 == n))
            *reinterpret_cast<uint64_t*>(bits_copy + u * copy_stride) = bits;
        }
        if (branch0) {
          uint32_t v[5];
#pragma unroll
          for (int q = 0; q < 5; q++) v[q] = Tn.w[kq[q]];
          const uint16_t tck = (uint16_t)enum_ck(c1, c2, v);
          store_state<P>(Tn, trunk_dst, p.S);
          *ck_dst = tck;
          if (ck_copy && (copy_stride || u + 1 == n)) *reinterpret_cast<uint16_t*>(ck_copy + u * copy_stride) = tck;
        }
        survived = survive;
      }
      T = Tn;
    };
    using Z = std::integral_constant<int, 0>;
    using KWc = std::integral_constant<int, KW>;
    if (WT > 0 && n >= W - 1) {
      // compile-time W, a full ramp: super-step u < W - 1 steps stages [0, u + 1), drain super-step
      // n + j stages [j + 1, W) without the trunk's enumerated player
      static_for<(WT > 0 ? WT - 1 : 0)>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        super_step(j, std::true_type(), Z(), std::integral_constant<int, j + 1>(), std::true_type());
      });
      for (int32_t u = W - 1; u < n; ++u) super_step(u, std::false_type(), Z(), KWc(), std::true_type());
      static_for<(WT > 0 ? WT - 1 : 0)>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        super_step(n + j, std::true_type(), std::integral_constant<int, j + 1>(), KWc(), std::false_type());
      });
    } else {
      const int32_t steady0 = W - 1 < n ? W - 1 : n;  // first super-step with every stage active
      int32_t u = 0;
      for (; u < steady0; ++u) super_step(u, std::true_type(), Z(), KWc(), std::true_type());
      for (; u < n; ++u) super_step(u, std::false_type(), Z(), KWc(), std::true_type());
      for (; u < n + W - 1; ++u) super_step(u, std::true_type(), Z(), KWc(), std::true_type());
    }
  };
  if (lean_ok) run(std::true_type());
  else run(std::false_type());
}

// compare_local_checksums_against_peers (p2p_session.rs:904-937) over an all-gathered report
// block: sessions whose trunk checksum differs between this rank's row and its peer's each count
// one DesyncDetected (src/lib.rs:158-167); the first round with any is recorded.
// gathered = [world][rows][report_bytes]; blockIdx.y = the row (round) compared.  Rows are
// visited in any order, so the first round with a desync is an atomicMin over the rows' frames
// (first starts at -1 = none: the min runs on frame + 1 and is stored back minus one).
__global__ __launch_bounds__(256) void compare_peer_kernel(const uint8_t* gathered, int64_t report_bytes, int32_t rows,
                                                           int32_t rank, int32_t peer, int64_t S, int32_t frame0,
                                                           unsigned long long* count, unsigned long long* first) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int32_t row = blockIdx.y;
  bool bad = false;
  if (s < S) {
    const uint16_t* mine = (const uint16_t*)(gathered + ((int64_t)rank * rows + row) * report_bytes);
    const uint16_t* theirs = (const uint16_t*)(gathered + ((int64_t)peer * rows + row) * report_bytes);
    bad = mine[s] != theirs[s];
  }
  const uint64_t m = __ballot(bad);
  if ((threadIdx.x & 63) == 0 && m) {
    atomicAdd(count, (unsigned long long)__popcll(m));
    // first: -1 (all ones) or the earliest frame so far; as unsigned, frame + 1 orders -1 last
    const unsigned long long f = (unsigned long long)(int64_t)(frame0 + row);
    unsigned long long cur = *(volatile unsigned long long*)first;
    while (cur + 1ull == 0ull || f < cur) {
      const unsigned long long prev = atomicCAS(first, cur, f);
      if (prev == cur) break;
      cur = prev;
    }
  }
}

}  // namespace

struct ggrs_branch_engine {
  ggrs_branch_config_t cfg{};
  int Pp = 1, F = 1, R = 2, cap = 128, E = 0, first_remote = -1;
  int64_t L = 0;
  hipStream_t stream = nullptr;      // where every launch and copy goes (own_stream or the caller's)
  hipStream_t own_stream = nullptr;
  uint32_t* trunk = nullptr;
  uint32_t* trunk_alt = nullptr;     // the fused rounds' output trunk (swapped in after the launch)
  uint32_t* ring = nullptr;
  uint16_t* ring_ck = nullptr;
  uint8_t* inputs = nullptr;
  uint8_t* report = nullptr;  // report_bytes: [S] u16 | pad to 8 | [words] u64
  size_t report_bytes = 0;
  uint64_t* prev_bits = nullptr;
  int32_t round_form = 0;            // ggrs_branch_set_round_launches: 0 fused (prefix-shared when
                                     // eligible), 1 = 2 n launches, 2 fused without prefix sharing
  int32_t last_spec_fc = -1;         // trunk frame of the last speculation (read_lane's depth)
  int32_t* desync = nullptr;
  uint8_t* staging = nullptr;
  size_t staging_bytes = 0;
  int32_t trunk_frame = 0;
  int32_t next_input_frame = 0;
  bool have_prev = false;
  SpanTimer timer;
};

namespace {

size_t report_ck_bytes(int64_t S) { return ((size_t)S * 2 + 7) & ~(size_t)7; }
constexpr size_t kPrefixLdsBytes = 32 * 1024;

// prefix_pipe_kernel<P, EP> for the runtime enumerated player ep (0 <= ep < P)
template <int P, typename Fn>
void dispatch_enumerated(int ep, Fn&& fn) {
  switch (ep) {
    case 0: fn(std::integral_constant<int, 0>()); break;
    case 1: if constexpr (P > 1) fn(std::integral_constant<int, 1>()); break;
    case 2: if constexpr (P > 2) fn(std::integral_constant<int, 2>()); break;
    default: if constexpr (P > 3) fn(std::integral_constant<int, 3>()); break;
  }
}
int64_t report_words(int64_t L) { return (L + 63) / 64; }

template <typename K>
int branch_launch_timed(ggrs_branch_engine* e, K&& launch, int32_t counts_as = 1) {
  if (int rc = e->timer.before(e->stream)) return rc;
  launch();
  HIP_TRY(hipGetLastError());
  e->timer.count(counts_as);
  return GGRS_OK;
}

}  // namespace

extern "C" {

int ggrs_branch_engine_destroy(ggrs_branch_engine_t* e) {
  if (!e) return GGRS_OK;
  (void)hipSetDevice(e->cfg.device);
  if (e->own_stream) (void)hipStreamSynchronize(e->stream);  // the current stream, the null stream too
  void* bufs[] = {e->trunk, e->trunk_alt, e->ring, e->ring_ck, e->inputs, e->report, e->prev_bits, e->desync, e->staging};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  e->timer.destroy();
  if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
  delete e;
  return GGRS_OK;
}

int ggrs_branch_engine_create(const ggrs_branch_config_t* cfg, ggrs_branch_engine_t** out) {
  if (!cfg || !out) return set_error(GGRS_E_INVALID, "null argument");
  *out = nullptr;
  const ggrs_branch_config_t c = *cfg;
  if (c.num_sessions < 1) return set_error(GGRS_E_INVALID, "num_sessions must be >= 1");
  if (c.num_players < 1 || c.num_players > 4) return set_error(GGRS_E_INVALID, "num_players must be in 1..4 (ex_game.rs:70)");
  if ((c.remote_mask & ~((1 << c.num_players) - 1)) != 0 || c.remote_mask == 0)
    return set_error(GGRS_E_INVALID, "remote_mask must name at least one of the session's players");
  if (c.window < 1 || c.window > 62) return set_error(GGRS_E_INVALID, "window must be in 1..62");
  if (c.branches < 1) return set_error(GGRS_E_INVALID, "branches must be >= 1");
  if (c.alphabet < 2 || c.alphabet > 256) return set_error(GGRS_E_INVALID, "alphabet must be in 2..256");
  int E = 0;
  if (c.branches > 1) {
    int64_t v = 1;
    while (v < c.branches) { v *= c.alphabet; E++; }
    if (v != c.branches) return set_error(GGRS_E_INVALID, "branches must be 1 or a power of the alphabet");
    if (E > c.window) return set_error(GGRS_E_INVALID, "branches enumerate more frames than the window");
  }
  const int64_t L = (int64_t)c.num_sessions * c.branches;
  if (L > ((int64_t)1 << 31)) return set_error(GGRS_E_INVALID, "too many lanes");
  ggrs_branch_engine* e = new ggrs_branch_engine();
  e->cfg = c;
  e->L = L;
  e->E = E;
  e->Pp = padded_players(c.num_players);
  e->F = state_fields(c.num_players);
  e->R = c.window + 1;
  e->cap = c.input_capacity ? c.input_capacity : 128;
  e->cfg.input_capacity = e->cap;
  for (int q = 0; q < c.num_players; q++)
    if ((c.remote_mask >> q) & 1) { e->first_remote = q; break; }
  if (e->cap < c.window + 2) {
    delete e;
    return set_error(GGRS_E_INVALID, "input_capacity must be >= window + 2");
  }
  auto fail = [&](int rc) {
    std::string msg = ggrs_last_error();
    ggrs_branch_engine_destroy(e);
    set_error(rc, "%s", msg.c_str());
    return rc;
  };
#define CTRY(expr)                                                                      \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) return fail(set_error(GGRS_E_HIP, "%s: %s", #expr, hipGetErrorString(e_))); \
  } while (0)
  const int64_t S = c.num_sessions;
  CTRY(hipSetDevice(c.device));
  CTRY(hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking));
  e->stream = e->own_stream;
  if (e->timer.create()) return fail(GGRS_E_HIP);
  CTRY(hipMalloc(&e->trunk, sizeof(uint32_t) * e->F * S));
  CTRY(hipMalloc(&e->trunk_alt, sizeof(uint32_t) * e->F * S));
  CTRY(hipMalloc(&e->ring, sizeof(uint32_t) * (size_t)e->R * e->F * L));
  CTRY(hipMalloc(&e->ring_ck, sizeof(uint16_t) * (size_t)e->R * L));
  CTRY(hipMalloc(&e->inputs, (size_t)e->cap * S * e->Pp));
  e->report_bytes = report_ck_bytes(S) + 8 * report_words(L);
  CTRY(hipMalloc(&e->report, e->report_bytes));
  CTRY(hipMalloc(&e->prev_bits, 8 * report_words(L)));
  CTRY(hipMalloc(&e->desync, sizeof(int32_t) * S));
  CTRY(hipMemsetAsync(e->ring, 0, sizeof(uint32_t) * (size_t)e->R * e->F * L, e->stream));
  CTRY(hipMemsetAsync(e->ring_ck, 0, sizeof(uint16_t) * (size_t)e->R * L, e->stream));
  CTRY(hipMemsetAsync(e->inputs, 0, (size_t)e->cap * S * e->Pp, e->stream));
  CTRY(hipMemsetAsync(e->report, 0, e->report_bytes, e->stream));
  CTRY(hipMemsetAsync(e->prev_bits, 0, 8 * report_words(L), e->stream));
  CTRY(hipMemsetAsync(e->desync, 0xff, sizeof(int32_t) * S, e->stream));
  dispatch_players(c.num_players, [&](auto PC) {
    constexpr int P = decltype(PC)::value;
    init_states_kernel<P><<<grid_of(S, 256), 256, 0, e->stream>>>(e->trunk, S);
  });
  CTRY(hipGetLastError());
  CTRY(hipStreamSynchronize(e->stream));
#undef CTRY
  *out = e;
  return GGRS_OK;
}

int ggrs_branch_engine_config(const ggrs_branch_engine_t* e, ggrs_branch_config_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  *out = e->cfg;
  return GGRS_OK;
}

int ggrs_branch_add_inputs(ggrs_branch_engine_t* e, int32_t first_frame, int32_t n, const uint8_t* inputs) {
  if (!e || (!inputs && n > 0)) return set_error(GGRS_E_INVALID, "null argument");
  if (n < 0) return set_error(GGRS_E_INVALID, "n_frames must be >= 0");
  if (first_frame != e->next_input_frame)
    return set_error(GGRS_E_INVALID, "inputs must be added sequentially (expected frame %d, got %d)",
                     e->next_input_frame, first_frame);
  if (n == 0) return GGRS_OK;
  // the oldest frame still read is trunk_frame - 1 (the repeat-last prediction source)
  if ((int64_t)first_frame + n - 1 - ((int64_t)e->trunk_frame - 1) >= e->cap)
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
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->next_input_frame = first_frame + n;
  return GGRS_OK;
}

int ggrs_branch_speculate(ggrs_branch_engine_t* e) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  const int32_t W = e->cfg.window;
  if ((int64_t)e->trunk_frame + W - 1 >= e->next_input_frame)
    return set_error(GGRS_E_INVALID, "local inputs for frames up to %d are not queued", e->trunk_frame + W - 1);
  HIP_TRY(hipSetDevice(e->cfg.device));
  SpecParams p;
  p.S = e->cfg.num_sessions;
  p.L = e->L;
  p.B = e->cfg.branches;
  p.W = W;
  p.R = e->R;
  p.A = e->cfg.alphabet;
  p.E = e->E;
  p.cap = e->cap;
  p.P = e->cfg.num_players;
  p.f_c = e->trunk_frame;
  p.remote_mask = (uint32_t)e->cfg.remote_mask;
  p.first_remote = e->first_remote;
  p.check_prev = e->have_prev ? 1 : 0;
  p.trunk = e->trunk;
  p.ring = e->ring;
  p.ring_ck = e->ring_ck;
  p.inputs = e->inputs;
  // the previous confirm's survival bits, read in place from the report (stream order: no
  // confirm runs between that confirm and this speculate)
  p.prev_survive = (const uint64_t*)(e->report + report_ck_bytes(p.S));
  p.trunk_ck = (const uint16_t*)e->report;
  p.desync = e->desync;
  int rc = branch_launch_timed(e, [&] {
    dispatch_players(p.P, [&](auto PC) {
      constexpr int P = decltype(PC)::value;
      speculate_kernel<P><<<grid_of(p.L, 256), 256, 0, e->stream>>>(p);
    });
  });
  if (rc == GGRS_OK) e->last_spec_fc = p.f_c;
  return rc;
}

int ggrs_branch_confirm(ggrs_branch_engine_t* e, void* report_device) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (e->trunk_frame >= e->next_input_frame)
    return set_error(GGRS_E_INVALID, "inputs of frame %d are not queued", e->trunk_frame);
  HIP_TRY(hipSetDevice(e->cfg.device));
  ConfirmParams p;
  p.S = e->cfg.num_sessions;
  p.L = e->L;
  p.B = e->cfg.branches;
  p.A = e->cfg.alphabet;
  p.E = e->E;
  p.cap = e->cap;
  p.P = e->cfg.num_players;
  p.f_c = e->trunk_frame;
  p.remote_mask = (uint32_t)e->cfg.remote_mask;
  p.first_remote = e->first_remote;
  p.trunk = e->trunk;
  p.inputs = e->inputs;
  p.report_ck = (uint16_t*)e->report;
  p.report_bits = (uint64_t*)(e->report + report_ck_bytes(p.S));
  int rc = branch_launch_timed(e, [&] {
    dispatch_players(p.P, [&](auto PC) {
      constexpr int P = decltype(PC)::value;
      confirm_kernel<P><<<grid_of(p.L, 256), 256, 0, e->stream>>>(p);
    });
  });
  if (rc) return rc;
  if (report_device)
    HIP_TRY(hipMemcpyAsync(report_device, e->report, e->report_bytes, hipMemcpyDeviceToDevice, e->stream));
  e->trunk_frame += 1;
  e->have_prev = true;
  return GGRS_OK;
}

int ggrs_branch_report_bytes(const ggrs_branch_engine_t* e, int64_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  *out = (int64_t)e->report_bytes;
  return GGRS_OK;
}

int ggrs_branch_synchronize(ggrs_branch_engine_t* e) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

int ggrs_branch_trunk_frame(const ggrs_branch_engine_t* e, int32_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  *out = e->trunk_frame;
  return GGRS_OK;
}

int ggrs_branch_read_report(ggrs_branch_engine_t* e, uint16_t* checksums, uint64_t* survive_bits) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t S = e->cfg.num_sessions;
  if (checksums) HIP_TRY(hipMemcpyAsync(checksums, e->report, 2 * S, hipMemcpyDeviceToHost, e->stream));
  if (survive_bits)
    HIP_TRY(hipMemcpyAsync(survive_bits, e->report + report_ck_bytes(S), 8 * report_words(e->L),
                           hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

int ggrs_branch_read_desync(ggrs_branch_engine_t* e, int32_t* first_frame) {
  if (!e || !first_frame) return set_error(GGRS_E_INVALID, "null argument");
  HIP_TRY(hipSetDevice(e->cfg.device));
  HIP_TRY(hipMemcpyAsync(first_frame, e->desync, 4 * e->cfg.num_sessions, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return GGRS_OK;
}

int ggrs_branch_read_trunk(ggrs_branch_engine_t* e, int32_t session, uint8_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  if (session < 0 || session >= e->cfg.num_sessions) return set_error(GGRS_E_INVALID, "session out of range");
  HIP_TRY(hipSetDevice(e->cfg.device));
  std::vector<uint32_t> w(e->F);
  for (int k = 0; k < e->F; k++)
    HIP_TRY(hipMemcpyAsync(&w[k], e->trunk + (size_t)k * e->cfg.num_sessions + session, 4, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  serialize_state_bytes(w.data(), e->cfg.num_players, out);
  return GGRS_OK;
}

int ggrs_branch_read_lane(ggrs_branch_engine_t* e, int64_t lane, int32_t frame, uint16_t* checksum, uint8_t* out) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (lane < 0 || lane >= e->L) return set_error(GGRS_E_INVALID, "lane out of range");
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int slot = ((frame % e->R) + e->R) % e->R;
  // the cell of `frame` was saved at depth k = frame - f_c - 1 of the last speculation from trunk
  // frame f_c (the frame f_c itself at depth 0 of the one before); branches sharing their first
  // k + 1 digits share it, held by the prefix's representative (rep_branch, prefix_pipe_kernel)
  int64_t cell_lane = lane;
  if (e->E > 0 && e->last_spec_fc >= 0 && frame >= e->last_spec_fc && frame <= e->last_spec_fc + e->cfg.window) {
    const int k = frame > e->last_spec_fc ? frame - e->last_spec_fc - 1 : 0;
    const int64_t B = e->cfg.branches, sess = lane / B;
    cell_lane = sess * B + rep_branch(lane - sess * B, k, e->cfg.alphabet, e->E);
  }
  std::vector<uint32_t> w(e->F);
  for (int k = 0; k < e->F; k++)
    HIP_TRY(hipMemcpyAsync(&w[k], e->ring + ((size_t)slot * e->F + k) * e->L + cell_lane, 4, hipMemcpyDeviceToHost,
                           e->stream));
  uint16_t ck = 0;
  HIP_TRY(hipMemcpyAsync(&ck, e->ring_ck + (size_t)slot * e->L + cell_lane, 2, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (checksum) *checksum = ck;
  if (out) serialize_state_bytes(w.data(), e->cfg.num_players, out);
  return GGRS_OK;
}

int ggrs_branch_read_cells(ggrs_branch_engine_t* e, int32_t frame, uint16_t* checksums, uint8_t* states) {
  if (!e || !checksums) return set_error(GGRS_E_INVALID, "null argument");
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int slot = ((frame % e->R) + e->R) % e->R;
  const int64_t L = e->L, B = e->cfg.branches;
  std::vector<uint16_t> ck((size_t)L);
  std::vector<uint32_t> soa(states ? (size_t)e->F * L : 0);
  HIP_TRY(hipMemcpyAsync(ck.data(), e->ring_ck + (size_t)slot * L, (size_t)L * 2, hipMemcpyDeviceToHost, e->stream));
  if (states)
    HIP_TRY(hipMemcpyAsync(soa.data(), e->ring + (size_t)slot * e->F * L, soa.size() * 4, hipMemcpyDeviceToHost,
                           e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  // resolved as ggrs_branch_read_lane: a prefix-shared cell is held by the prefix's representative
  const bool shared = e->E > 0 && e->last_spec_fc >= 0 && frame >= e->last_spec_fc &&
                      frame <= e->last_spec_fc + e->cfg.window;
  const int k = shared && frame > e->last_spec_fc ? frame - e->last_spec_fc - 1 : 0;
  const int sb = 36 + 20 * e->cfg.num_players;
  uint32_t w[64];
  for (int64_t lane = 0; lane < L; lane++) {
    int64_t cell = lane;
    if (shared) {
      const int64_t sess = lane / B;
      cell = sess * B + rep_branch(lane - sess * B, k, e->cfg.alphabet, e->E);
    }
    checksums[lane] = ck[(size_t)cell];
    if (states) {
      for (int j = 0; j < e->F; j++) w[j] = soa[(size_t)j * L + cell];
      serialize_state_bytes(w, e->cfg.num_players, states + (size_t)lane * sb);
    }
  }
  return GGRS_OK;
}

int ggrs_branch_timing_reset(ggrs_branch_engine_t* e) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  return e->timer.reset(e->stream);
}

int ggrs_branch_timing_stop(ggrs_branch_engine_t* e) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  return e->timer.stop(e->stream);
}

int ggrs_branch_timing_read(ggrs_branch_engine_t* e, float* total_ms, int32_t* launches) {
  if (!e || !total_ms || !launches) return set_error(GGRS_E_INVALID, "null argument");
  HIP_TRY(hipSetDevice(e->cfg.device));
  return e->timer.read(e->stream, total_ms, launches);
}

namespace {

// n rounds in one rounds_kernel launch; the last round's report also to `copy` (may be null)
int launch_rounds(ggrs_branch_engine* e, int32_t n_rounds, void* copy, bool every_round = false) {
  RoundsParams rp;
  SpecParams& p = rp.sp;
  p.S = e->cfg.num_sessions;
  p.L = e->L;
  p.B = e->cfg.branches;
  p.W = e->cfg.window;
  p.R = e->R;
  p.A = e->cfg.alphabet;
  p.E = e->E;
  p.cap = e->cap;
  p.P = e->cfg.num_players;
  p.f_c = e->trunk_frame;
  p.remote_mask = (uint32_t)e->cfg.remote_mask;
  p.first_remote = e->first_remote;
  p.check_prev = e->have_prev ? 1 : 0;
  p.trunk = e->trunk;
  p.ring = e->ring;
  p.ring_ck = e->ring_ck;
  p.inputs = e->inputs;
  p.prev_survive = (const uint64_t*)(e->report + report_ck_bytes(p.S));
  p.trunk_ck = (const uint16_t*)e->report;
  p.desync = e->desync;
  rp.n = n_rounds;
  // the fused kernels read the trunks from p.trunk and write them to rp.trunk, another buffer: a
  // block still reading its sessions' trunks must not see another block's later rounds
  rp.trunk = e->trunk_alt;
  rp.report_ck = (uint16_t*)e->report;
  rp.report_bits = (uint64_t*)(e->report + report_ck_bytes(p.S));
  rp.copy_ck = copy ? (uint16_t*)copy : nullptr;
  rp.copy_bits = copy ? (uint64_t*)((uint8_t*)copy + report_ck_bytes(p.S)) : nullptr;
  rp.copy_stride = every_round ? (int64_t)e->report_bytes : 0;
  // prefix sharing (prefix_pipe_kernel) when the enumerated player is the only remote one, the
  // window fits its stage registers and the launch's input rows ([n + W - 1][ns] words) fit LDS
  const int ns_max = (int)std::min<int64_t>(kRoundsBlock / p.B + 2, p.S);
  const int64_t rows_fit = (int64_t)kPrefixLdsBytes / 4 / ns_max - (p.W - 1);
  const int32_t n_chunk = (int32_t)std::max<int64_t>(0, std::min<int64_t>(n_rounds, rows_fit));
  const size_t lds_words = (size_t)ns_max * (n_chunk + p.W - 1);
  const bool prefix = e->round_form == 0 && p.B > 1 && __builtin_popcount(p.remote_mask) == 1 && n_chunk >= 1 &&
                      p.W <= kPipeMaxW && (int64_t)p.R * e->F * p.L * 4 < ((int64_t)1 << 30);
  if (prefix && n_chunk < n_rounds) {  // launches of n_chunk rounds (their input rows fit LDS)
    for (int32_t r0 = 0; r0 < n_rounds; r0 += n_chunk) {
      const int32_t m = std::min(n_chunk, n_rounds - r0);
      void* c = !copy ? nullptr
                      : (every_round ? (void*)((uint8_t*)copy + (size_t)r0 * e->report_bytes)
                                     : (r0 + m == n_rounds ? copy : nullptr));
      if (int rc = launch_rounds(e, m, c, every_round)) return rc;
    }
    return GGRS_OK;
  }
  // counted as the 2 n speculate + confirm launches it replaces
  int rc = branch_launch_timed(e, [&] {
    const dim3 grid((unsigned)grid_of(p.L, kRoundsBlock));
    if (prefix) {
      const size_t lds = lds_words * 4;
      dispatch_players(p.P, [&](auto PC) {
        constexpr int P = decltype(PC)::value;
        dispatch_enumerated<P>(p.first_remote, [&](auto EC) {
          constexpr int EP = decltype(EC)::value;
          // lane pairs share a session when the branch count is even (two players only)
          const bool pair = P == 2 && (p.B & 1) == 0;
          if (pair) {
            if (p.W == 4) prefix_pipe_kernel<P, EP, 4, P == 2><<<grid, kRoundsBlock, lds, e->stream>>>(rp);
            else prefix_pipe_kernel<P, EP, 0, P == 2><<<grid, kRoundsBlock, lds, e->stream>>>(rp);
          } else {
            if (p.W == 4) prefix_pipe_kernel<P, EP, 4, false><<<grid, kRoundsBlock, lds, e->stream>>>(rp);
            else prefix_pipe_kernel<P, EP, 0, false><<<grid, kRoundsBlock, lds, e->stream>>>(rp);
          }
        });
      });
      return;
    }
    dispatch_players(p.P, [&](auto PC) {
      constexpr int P = decltype(PC)::value;
      rounds_kernel<P><<<grid, kRoundsBlock, 0, e->stream>>>(rp);
    });
  }, 2 * n_rounds);
  if (rc) return rc;
  std::swap(e->trunk, e->trunk_alt);
  e->last_spec_fc = e->trunk_frame + n_rounds - 1;
  e->trunk_frame += n_rounds;
  e->have_prev = true;
  return GGRS_OK;
}

int check_rounds_queued(const ggrs_branch_engine* e, int32_t n_rounds) {
  if ((int64_t)e->trunk_frame + n_rounds - 1 + e->cfg.window - 1 >= e->next_input_frame)
    return set_error(GGRS_E_INVALID, "inputs for %d rounds are not queued", n_rounds);
  return GGRS_OK;
}

}  // namespace

int ggrs_branch_rounds(ggrs_branch_engine_t* e, int32_t n_rounds) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (n_rounds < 0) return set_error(GGRS_E_INVALID, "n_rounds must be >= 0");
  if (int rc = check_rounds_queued(e, n_rounds)) return rc;
  if (n_rounds == 0) return GGRS_OK;
  HIP_TRY(hipSetDevice(e->cfg.device));
  if (e->round_form != 1) return launch_rounds(e, n_rounds, nullptr);
  int rc = GGRS_OK;
  for (int32_t r = 0; r < n_rounds && rc == GGRS_OK; r++) {
    rc = ggrs_branch_speculate(e);
    if (rc == GGRS_OK) rc = ggrs_branch_confirm(e, nullptr);
  }
  return rc;
}

int ggrs_branch_round(ggrs_branch_engine_t* e, void* report_device) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (int rc = check_rounds_queued(e, 1)) return rc;
  HIP_TRY(hipSetDevice(e->cfg.device));
  return launch_rounds(e, 1, report_device);
}

int ggrs_branch_rounds_reports(ggrs_branch_engine_t* e, int32_t n_rounds, void* reports_device) {
  if (!e || !reports_device) return set_error(GGRS_E_INVALID, "null argument");
  if (n_rounds < 0) return set_error(GGRS_E_INVALID, "negative round count");
  if (n_rounds == 0) return GGRS_OK;
  if (int rc = check_rounds_queued(e, n_rounds)) return rc;
  HIP_TRY(hipSetDevice(e->cfg.device));
  return launch_rounds(e, n_rounds, reports_device, true);
}

int ggrs_branch_compare_peer(ggrs_branch_engine_t* e, const void* gathered, int32_t world, int32_t rank,
                             int32_t peer, int32_t frame, int64_t* count_device, int64_t* first_frame_device) {
  if (!e || !gathered || !count_device || !first_frame_device) return set_error(GGRS_E_INVALID, "null argument");
  if (world < 2 || rank < 0 || rank >= world || peer < 0 || peer >= world || peer == rank)
    return set_error(GGRS_E_INVALID, "rank %d / peer %d out of range for world %d", rank, peer, world);
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t S = e->cfg.num_sessions;
  compare_peer_kernel<<<grid_of(S, 256), 256, 0, e->stream>>>((const uint8_t*)gathered, (int64_t)e->report_bytes, 1,
                                                             rank, peer, S, frame,
                                                             (unsigned long long*)count_device,
                                                             (unsigned long long*)first_frame_device);
  HIP_TRY(hipGetLastError());
  return GGRS_OK;
}

int ggrs_branch_compare_peer_rows(ggrs_branch_engine_t* e, const void* gathered, int32_t world, int32_t rows_per_rank,
                                  int32_t n_rows, int32_t rank, int32_t peer, int32_t first_frame,
                                  int64_t* count_device, int64_t* first_frame_device) {
  if (!e || !gathered || !count_device || !first_frame_device) return set_error(GGRS_E_INVALID, "null argument");
  if (world < 2 || rank < 0 || rank >= world || peer < 0 || peer >= world || peer == rank)
    return set_error(GGRS_E_INVALID, "rank %d / peer %d out of range for world %d", rank, peer, world);
  if (rows_per_rank < 1 || n_rows < 0 || n_rows > rows_per_rank || n_rows > 65535)
    return set_error(GGRS_E_INVALID, "%d rows of %d per rank", n_rows, rows_per_rank);
  if (n_rows == 0) return GGRS_OK;
  HIP_TRY(hipSetDevice(e->cfg.device));
  const int64_t S = e->cfg.num_sessions;
  const dim3 grid((unsigned)grid_of(S, 256), (unsigned)n_rows);
  compare_peer_kernel<<<grid, 256, 0, e->stream>>>((const uint8_t*)gathered, (int64_t)e->report_bytes, rows_per_rank,
                                                  rank, peer, S, first_frame, (unsigned long long*)count_device,
                                                  (unsigned long long*)first_frame_device);
  HIP_TRY(hipGetLastError());
  return GGRS_OK;
}

namespace {
// Every launch and copy from now on goes to `s`; work already queued on the old stream comes first
// (the new stream waits for it on the device).
int switch_stream(ggrs_branch_engine_t* e, hipStream_t s) {
  HIP_TRY(hipSetDevice(e->cfg.device));
  if (s == e->stream) return GGRS_OK;
  if (e->timer.collecting) return set_error(GGRS_E_STATE, "cannot switch streams while timing a span");
  hipEvent_t ev;
  HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(ev, e->stream));
  HIP_TRY(hipStreamWaitEvent(s, ev, 0));
  HIP_TRY(hipEventDestroy(ev));
  e->stream = s;
  return GGRS_OK;
}
}  // namespace

// NULL is HIP's null stream (what torch.cuda.current_stream() reports as handle 0), not the engine's
// own stream: the own stream is non-blocking, so mapping NULL to it left a caller on the null stream
// unordered with the engine's launches (ABI 2; ggrs_branch_use_own_stream selects it explicitly).
int ggrs_branch_set_stream(ggrs_branch_engine_t* e, void* stream) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  return switch_stream(e, (hipStream_t)stream);
}

int ggrs_branch_use_own_stream(ggrs_branch_engine_t* e) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  return switch_stream(e, e->own_stream);
}

int ggrs_branch_set_round_launches(ggrs_branch_engine_t* e, int32_t on) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  if (on < 0 || on > 2) return set_error(GGRS_E_INVALID, "round form %d: 0 fused, 1 per-round launches, 2 fused "
                                                         "without prefix sharing", on);
  e->round_form = on;
  return GGRS_OK;
}

}  // extern "C"
