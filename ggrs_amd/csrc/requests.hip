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
// The kernel: 256-thread lane blocks, a session's players on Pp adjacent lanes.  The batch lives in
// pinned host memory mapped into the device; each block copies its piece of every row into LDS up
// front (8-byte words spread over the block's threads, all in flight: one PCIe round trip instead
// of one per request), each session's list is validated against its cell tags (also in LDS), then
// executed with the state in registers; checksums collect in LDS and go back to host memory with
// the lane results as wide system-scope stores.
#include <atomic>
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <immintrin.h>

#include <algorithm>
#include <chrono>
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
  int32_t wide;                // L % 8 == 0: a block's piece of every host row is whole 8-byte words
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

// A session's players sit on Pp adjacent lanes (Pp = P rounded up to a power of two), each lane
// stepping one player (State::advance's per-player loop body is independent across players,
// ex_game.rs:275-332): a lane's dependent chain per AdvanceFrame is one player's step, not P of
// them.  Every lane of a session walks the same list; lane `pl` holds the frame and player pl's
// x, y, vx, vy, rot (padding lanes hold zeros and store nothing).
// Blocks of four wavefronts: the lane server's per-batch hand-offs (the relay poll, the done
// counter) scale with the block count, so fewer, larger blocks (tools/server_probe.hip).
constexpr int kLaneBlock = 256;

template <int P>
struct LaneGeom {
  static constexpr int Pp = P <= 1 ? 1 : (P == 2 ? 2 : 4);
  static constexpr int kSessions = kLaneBlock / Pp;  // sessions per block
};

struct Slice {
  uint32_t frame;
  uint32_t w[5];  // x, y, vx, vy, rot of this lane's player
};

template <int P>
__device__ inline int slice_field(int pl, int q) {
  const int c = pl < P ? pl : 0;
  return q == 0 ? fld_x(P, c) : q == 1 ? fld_y(P, c) : q == 2 ? fld_vx(P, c) : q == 3 ? fld_vy(P, c) : fld_rot(P, c);
}

template <int P>
__device__ inline void load_slice(Slice& s, const uint32_t* base, int64_t L, int pl) {
  s.frame = base[0];
#pragma unroll
  for (int q = 0; q < 5; q++) s.w[q] = pl < P ? base[(int64_t)slice_field<P>(pl, q) * L] : 0u;
}
template <int P>
__device__ inline void store_slice(const Slice& s, uint32_t* base, int64_t L, int pl) {
  if (pl == 0) base[0] = s.frame;
  if (pl < P) {
#pragma unroll
    for (int q = 0; q < 5; q++) base[(int64_t)slice_field<P>(pl, q) * L] = s.w[q];
  }
}

// fletcher16 of the session's bincode bytes (ex_game.rs:45-55,105-106) from the Pp lanes' slices:
// doubled per-lane partial sums (two v_dot4 per field, the frame and constant length prefixes on
// lane 0), summed across the group by DPP, reduced by fletcher_from_doubled (box_game.h).
template <int P>
__device__ inline uint32_t slice_fletcher(const Slice& s, int pl) {
  constexpr int Pp = LaneGeom<P>::Pp;
  constexpr int n = Fletcher<P>::n;
  uint32_t d1 = 0, d2 = 0;
  if (pl == 0) {
    d1 = dot4_u8(s.frame, 0x02020202u, 2u * Fletcher<P>::kSum1Const);
    d2 = dot4_u8(s.frame, 2u * weights_at(n, 0), 2u * Fletcher<P>::kSum2Const);
  }
  if (pl < P) {
#pragma unroll
    for (int q = 0; q < 5; q++) {
      d1 = dot4_u8(s.w[q], 0x02020202u, d1);
      d2 = dot4_u8(s.w[q], 2u * weights_at(n, fld_offset(P, slice_field<P>(pl, q))), d2);
    }
  }
  if constexpr (Pp >= 2) {
    d1 += (uint32_t)__builtin_amdgcn_mov_dpp((int)d1, 0xB1, 0xF, 0xF, false);  // xor 1
    d2 += (uint32_t)__builtin_amdgcn_mov_dpp((int)d2, 0xB1, 0xF, 0xF, false);
  }
  if constexpr (Pp >= 4) {
    d1 += (uint32_t)__builtin_amdgcn_mov_dpp((int)d1, 0x4E, 0xF, 0xF, false);  // xor 2
    d2 += (uint32_t)__builtin_amdgcn_mov_dpp((int)d2, 0x4E, 0xF, 0xF, false);
  }
  return fletcher_from_doubled(d1, d2);
}

// State::advance for this lane's player through the lean step, with the sin/cos of its rot
// supplied (sn, cs) and the NEXT step's computed by the step's hook as soon as the new rot exists
// (rot does not depend on the velocity chain, so the two run side by side, as in the v5 SyncTest
// kernel).  Only for states in the lean step's rotation domain (the caller's wave-wide test).
__device__ inline void slice_advance_lean(Slice& s, uint32_t in, bool owner, float& sn, float& cs) {
  s.frame = (uint32_t)((int32_t)s.frame + 1);
  float x = __builtin_bit_cast(float, s.w[0]), y = __builtin_bit_cast(float, s.w[1]);
  float vx = __builtin_bit_cast(float, s.w[2]), vy = __builtin_bit_cast(float, s.w[3]);
  float rot = __builtin_bit_cast(float, s.w[4]);
  const float s0 = sn, c0 = cs;
  advance_player_lean_sc(x, y, vx, vy, rot, in, s0, c0, [&](float r) { glibc_sincosf_domain(r, &sn, &cs); });
  if (owner) {
    s.w[0] = __builtin_bit_cast(uint32_t, x);
    s.w[1] = __builtin_bit_cast(uint32_t, y);
    s.w[2] = __builtin_bit_cast(uint32_t, vx);
    s.w[3] = __builtin_bit_cast(uint32_t, vy);
    s.w[4] = __builtin_bit_cast(uint32_t, rot);
  }
}

// State::advance for this lane's player (input byte `in`, already 4 for a Disconnected player)
__device__ inline void slice_advance(Slice& s, uint32_t in, bool owner) {
  s.frame = (uint32_t)((int32_t)s.frame + 1);
  float x = __builtin_bit_cast(float, s.w[0]), y = __builtin_bit_cast(float, s.w[1]);
  float vx = __builtin_bit_cast(float, s.w[2]), vy = __builtin_bit_cast(float, s.w[3]);
  float rot = __builtin_bit_cast(float, s.w[4]);
  advance_player(x, y, vx, vy, rot, in);
  if (owner) {
    s.w[0] = __builtin_bit_cast(uint32_t, x);
    s.w[1] = __builtin_bit_cast(uint32_t, y);
    s.w[2] = __builtin_bit_cast(uint32_t, vx);
    s.w[3] = __builtin_bit_cast(uint32_t, vy);
    s.w[4] = __builtin_bit_cast(uint32_t, rot);
  }
}

// LDS of a lane block (byte offsets, KS = the block's sessions, every row a multiple of 8 bytes):
//   tokens [W][KS] u32 | load frames [LD][KS] i32 | cell tags [R][KS] i32 | inputs [A][kInPitch] u8
//   | status [A][kInPitch] u8 (when used) | checksums out [S][KS] u16 | results [KS] i32
// Input and status rows keep the host's byte layout (session-major, P bytes per session), so a
// block stages its piece of every host row with wide copies.
struct LaneLds {
  int KS, in_pitch;
  size_t tok, ld, tag, in, st, ck, res, bytes;
  __host__ __device__ LaneLds(int P, int W, int LD, int R, int A, int S, int use_status) {
    const int Pp = P <= 1 ? 1 : (P == 2 ? 2 : 4);
    KS = kLaneBlock / Pp;
    in_pitch = (KS * P + 15) & ~15;
    tok = 0;
    ld = tok + (size_t)4 * KS * W;
    tag = ld + (size_t)4 * KS * LD;
    in = tag + (size_t)4 * KS * R;
    st = in + (size_t)in_pitch * A;
    ck = st + (use_status ? (size_t)in_pitch * A : 0);
    res = ck + (((size_t)2 * KS * S + 7) & ~(size_t)7);
    bytes = res + (size_t)4 * KS;
  }
};

// host memory is read and written with system-scope accesses: plain loads of pinned host memory may
// be served from the device's L2 (the persistent server re-reads the same rows every batch), and
// system-scope stores go straight out (sc0 sc1)
template <typename T>
__device__ inline T ld_sys(const T* ptr) {
  return __hip_atomic_load(ptr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ inline void st_sys(T* ptr, T v) {
  __hip_atomic_store(ptr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Stage the block's rows into LDS.  Wide form (p.wide: L % 8 == 0, so every host row piece of a
// block is whole 8-byte words): the block copies its pieces of the token, load-frame, input and
// status rows as 8-byte system-scope loads spread over all its threads, kStage of them in flight
// per thread (at 4096 lanes and a SyncTest list that is two loads per thread, one PCIe round trip);
// otherwise every lane loads its own dword / bytes row by row.  The cell tags (the frame field of
// each ring cell, device memory) are loaded per session.  Ends with a barrier.
template <int P>
__device__ inline void stage_rows(const LaneBatchParams& p, const LaneLds& g, uint8_t* lds, int64_t sess0, int nb,
                                  int64_t ln, int col, int pl) {
  const int t = threadIdx.x;
  const int64_t L = p.L;
  constexpr int F = state_fields(P);
  const int nrow = p.W + p.LD, nbr = p.A * (p.use_status ? 2 : 1);  // u32 rows, byte rows
  if (p.wide) {
    const int tp = nb / 2, ip = nb * P / 8;  // 8-byte words per u32 row / per byte row
    const int n_u32 = nrow * tp, total = n_u32 + nbr * ip;
    auto where = [&](int c, const uint64_t*& src, uint64_t*& dst) {
      if (c < n_u32) {
        const int r = c / tp, k = c - r * tp;
        const uint32_t* row = r < p.W ? p.tokens + (int64_t)r * L : (const uint32_t*)p.load_frames + (int64_t)(r - p.W) * L;
        src = reinterpret_cast<const uint64_t*>(row + sess0) + k;
        dst = reinterpret_cast<uint64_t*>(lds + g.tok + (size_t)4 * g.KS * r) + k;
      } else {
        c -= n_u32;
        const int r = c / ip, k = c - r * ip;
        const uint8_t* row = r < p.A ? p.inputs + ((int64_t)r * L + sess0) * P : p.status + ((int64_t)(r - p.A) * L + sess0) * P;
        src = reinterpret_cast<const uint64_t*>(row) + k;
        dst = reinterpret_cast<uint64_t*>(lds + g.in + (size_t)g.in_pitch * r) + k;
      }
    };
    constexpr int kStage = 8;
    for (int base = 0; base < total; base += kStage * kLaneBlock) {
      uint64_t v[kStage];
#pragma unroll
      for (int u = 0; u < kStage; u++) {
        const int c = base + u * kLaneBlock + t;
        if (c < total) {
          const uint64_t* s;
          uint64_t* d;
          where(c, s, d);
          v[u] = ld_sys(s);
        }
      }
#pragma unroll
      for (int u = 0; u < kStage; u++) {
        const int c = base + u * kLaneBlock + t;
        if (c < total) {
          const uint64_t* s;
          uint64_t* d;
          where(c, s, d);
          *d = v[u];
        }
      }
    }
  } else {
    // one row per load, kStageChunk rows in flight: u32 rows (tokens, load frames) from lane 0 of
    // the session, input / status bytes from each owner lane
    constexpr int kStageChunk = 32;
    uint32_t* tok = reinterpret_cast<uint32_t*>(lds + g.tok);
    uint8_t* in = lds + g.in;
    for (int base = 0; base < nrow + nbr; base += kStageChunk) {
      uint32_t v[kStageChunk];
#pragma unroll
      for (int u = 0; u < kStageChunk; u++) {
        const int i = base + u;
        v[u] = 0;
        if (i < nrow) {
          v[u] = i < p.W ? ld_sys(p.tokens + (int64_t)i * L + ln) : (uint32_t)ld_sys(p.load_frames + (int64_t)(i - p.W) * L + ln);
        } else if (i < nrow + nbr && pl < P) {
          const int r = i - nrow;
          const uint8_t* row = r < p.A ? p.inputs + (int64_t)r * L * P : p.status + (int64_t)(r - p.A) * L * P;
          v[u] = ld_sys(row + ln * P + pl);
        }
      }
#pragma unroll
      for (int u = 0; u < kStageChunk; u++) {
        const int i = base + u;
        if (i < nrow) {
          if (pl == 0) tok[i * g.KS + col] = v[u];
        } else if (i < nrow + nbr && pl < P) {
          in[(size_t)g.in_pitch * (i - nrow) + col * P + pl] = (uint8_t)v[u];
        }
      }
    }
  }
  {  // (the Pp lanes of a session store the same values)
    int32_t* tag = reinterpret_cast<int32_t*>(lds + g.tag);
    for (int r0 = 0; r0 < p.R; r0 += 16) {
      int32_t v[16];
#pragma unroll
      for (int u = 0; u < 16; u++)
        if (r0 + u < p.R) v[u] = (int32_t)p.ring[(int64_t)(r0 + u) * F * L + ln];
#pragma unroll
      for (int u = 0; u < 16; u++)
        if (r0 + u < p.R) tag[(r0 + u) * g.KS + col] = v[u];
    }
  }
  __syncthreads();
}

// Write the block's checksum rows (up to the most saves any of its sessions made) and lane
// results back to host memory: 8-byte system-scope stores spread over the block (wide form), or
// one element per store.  Returns after the stores have left (vmcnt(0)).
__device__ inline void write_back(const LaneBatchParams& p, const LaneLds& g, const uint8_t* lds, int64_t sess0, int nb,
                                  int rows) {
  const int t = threadIdx.x;
  const int64_t L = p.L;
  const uint16_t* ck = reinterpret_cast<const uint16_t*>(lds + g.ck);
  const int32_t* res = reinterpret_cast<const int32_t*>(lds + g.res);
  if (p.wide) {
    const int cp = nb / 4, rp = nb / 2;  // 8-byte words per checksum row / of the results
    const int n_ck = rows * cp;
    for (int c = t; c < n_ck + rp; c += kLaneBlock) {
      if (c < n_ck) {
        const int r = c / cp, k = c - r * cp;
        st_sys(reinterpret_cast<uint64_t*>(p.cks + (int64_t)r * L + sess0) + k,
               reinterpret_cast<const uint64_t*>(ck + (size_t)r * g.KS)[k]);
      } else {
        const int k = c - n_ck;
        st_sys(reinterpret_cast<uint64_t*>(p.result + sess0) + k, reinterpret_cast<const uint64_t*>(res)[k]);
      }
    }
  } else {
    for (int c = t; c < (rows + 1) * nb; c += kLaneBlock) {
      const int r = c / nb, j = c - r * nb;
      if (r < rows) st_sys(p.cks + (int64_t)r * L + sess0 + j, ck[(size_t)r * g.KS + j]);
      else st_sys(p.result + sess0 + j, res[j]);
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this thread's stores have left
}

// One block of sessions fulfils its lists: stage, validate, execute, write back.  `st` is this
// lane's slice (in registers); a session only writes its own ring cells and outputs.  Returns the
// number of the block's sessions that failed validation (on thread 0; every thread takes part).
template <int P>
__device__ inline int run_lanes(const LaneBatchParams& p, Slice& st, uint8_t* lds) {
  constexpr int Pp = LaneGeom<P>::Pp;
  constexpr int KS = LaneGeom<P>::kSessions;
  const int wl = threadIdx.x;
  const int col = wl / Pp, pl = wl % Pp;  // session column in the block, player
  const bool owner = pl < P;
  const int64_t L = p.L;
  const int64_t sess0 = (int64_t)blockIdx.x * KS;
  const int nb = (int)min((int64_t)KS, L - sess0);
  const int64_t lane = sess0 + col;
  const bool valid = col < nb;
  const int64_t ln = valid ? lane : sess0;
  const int R = p.R;
  constexpr int F = state_fields(P);
  const LaneLds g(P, p.W, p.LD, R, p.A, p.S, p.use_status);
  const uint32_t* l_tok = reinterpret_cast<const uint32_t*>(lds + g.tok);
  const int32_t* l_load = reinterpret_cast<const int32_t*>(lds + g.ld);
  int32_t* l_tag = reinterpret_cast<int32_t*>(lds + g.tag);
  const uint8_t* l_in = lds + g.in;
  const uint8_t* l_st = lds + g.st;
  uint16_t* l_ck = reinterpret_cast<uint16_t*>(lds + g.ck);
  int32_t* l_res = reinterpret_cast<int32_t*>(lds + g.res);
  __shared__ int s_rows, s_fails;
  // the checksum rows start zeroed (a session's rows past its own saves read 0)
  for (int i = wl; i < p.S * KS / 2; i += kLaneBlock) reinterpret_cast<uint32_t*>(l_ck)[i] = 0u;
  if (wl == 0) s_rows = s_fails = 0;
  stage_rows<P>(p, g, lds, sess0, nb, ln, col, pl);

  int32_t result = 0;
  int ns_done = 0;
  if (valid) {
    const int n_tok = p.W * GGRS_TOKENS_PER_WORD;
    // the first two token words in registers (every list GGRS emits at max_prediction <= 15 fits
    // them), longer lists read the rest from LDS
    const uint32_t tw0 = p.W > 0 ? l_tok[col] : 0xffffffffu, tw1 = p.W > 1 ? l_tok[KS + col] : 0xffffffffu;
    auto token = [&](int k) -> uint32_t {
      const uint32_t w = k < 16 ? tw0 : (k < 32 ? tw1 : l_tok[(k >> 4) * KS + col]);
      return (w >> (2 * (k & 15))) & 3u;
    };
    // (1) validation, nothing written.  Fast path for the lists GGRS emits (at most 32 requests,
    // at most one Load, placed before any Save): per-kind counts from the 2-bit fields by popcount,
    // and the Load's frame against the cell tag staged from the ring.  Anything else walks the list.
    int32_t frame = (int32_t)st.frame;
    int32_t err = -1;
    bool walk = true;
    if (p.W <= 2) {
      const uint64_t w = (uint64_t)tw0 | ((uint64_t)tw1 << 32);
      const uint64_t lo = w & 0x5555555555555555ull, hi = (w >> 1) & 0x5555555555555555ull;
      const uint64_t end = lo & hi;
      const uint64_t live = end ? ((end & (0 - end)) - 1) : ~0ull;  // fields before the first END
      const uint64_t m_save = ~lo & ~hi & 0x5555555555555555ull & live, m_adv = lo & ~hi & live,
                     m_load = hi & ~lo & live;
      const int ns = __builtin_popcountll(m_save), na = __builtin_popcountll(m_adv),
                nl = __builtin_popcountll(m_load);
      if (ns <= p.S && na <= p.A && nl <= p.LD && nl <= 1 && (nl == 0 || !m_save || (m_load & (0 - m_load)) < (m_save & (0 - m_save)))) {
        walk = false;
        if (nl == 1) {
          const int32_t f = l_load[col];
          if (f < 0 || l_tag[(f % R) * KS + col] != f) err = (int32_t)(__builtin_ctzll(m_load) >> 1);
        }
      }
    }
    if (walk) {
      // the walk records the saves it would make in the tag row (each lane of the session its own
      // identical store: it only reads what it wrote itself)
      int na = 0, ns = 0, nl = 0;
      int32_t slot = frame % R;
      for (int k = 0; k < n_tok; k++) {
        const uint32_t t = token(k);
        if (t == GGRS_TOK_END) break;
        if (t == GGRS_TOK_SAVE) {
          if (ns == p.S) { err = k; break; }
          l_tag[slot * KS + col] = frame;
          ++ns;
        } else if (t == GGRS_TOK_LOAD) {
          if (nl == p.LD) { err = k; break; }
          const int32_t f = l_load[nl * KS + col];
          if (f < 0 || l_tag[(f % R) * KS + col] != f) { err = k; break; }  // sync_layer.rs:248
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
    if (err >= 0) {  // the session does not run (a reference session would have panicked here)
      result = -(1 + err);
    } else {
      // (2) execution: Game::handle_requests, requests strictly in order (ex_game.rs:79-99)
      int na = 0, ns = 0, nl = 0;
      int32_t slot = (int32_t)st.frame % R;
      // this lane's field offsets inside a ring slot (frame on lane 0, player pl's five fields)
      int64_t fo[5];
#pragma unroll
      for (int q = 0; q < 5; q++) fo[q] = (int64_t)slice_field<P>(pl, q) * L + lane;
      const int64_t slot_stride = (int64_t)F * L;
      auto save_cell = [&](uint32_t* cell) {
        if (pl == 0) cell[lane] = st.frame;
        if (owner) {
#pragma unroll
          for (int q = 0; q < 5; q++) cell[fo[q]] = st.w[q];
        }
      };
      auto load_cell = [&](const uint32_t* cell) {
        st.frame = cell[lane];
#pragma unroll
        for (int q = 0; q < 5; q++) st.w[q] = owner ? cell[fo[q]] : 0u;
      };
      // every state a list steps is this lane's current one or a ring cell this engine saved, so one
      // wave-wide rotation-domain test here selects the lean step for the whole list; the lean
      // step carries sin/cos of the state's rot one step ahead (recomputed after a Load)
      const bool lean = __all(st.w[4] <= kTwoPiBits);
      float sn = 0.0f, cs = 1.0f;
      if (lean) glibc_sincosf_domain(__builtin_bit_cast(float, st.w[4]), &sn, &cs);
      for (int k = 0; k < n_tok; k++) {
        const uint32_t t = token(k);
        if (t == GGRS_TOK_END) break;
        if (t == GGRS_TOK_SAVE) {  // save_game_state (:103-108): state + fletcher16 into the cell
          save_cell(p.ring + slot * slot_stride);
          const uint32_t ck = slice_fletcher<P>(st, pl);
          if (pl == 0) {
            p.ring_ck[(int64_t)slot * L + lane] = (uint16_t)ck;
            l_ck[ns * KS + col] = (uint16_t)ck;
          }
          ++ns;
        } else if (t == GGRS_TOK_LOAD) {  // load_game_state (:111-113)
          const int32_t f = l_load[nl * KS + col];
          slot = f % R;
          load_cell(p.ring + slot * slot_stride);
          if (lean) glibc_sincosf_domain(__builtin_bit_cast(float, st.w[4]), &sn, &cs);
          ++nl;
        } else {  // advance_frame (:115-127); Disconnected players spin (input 4, :277-281)
          const size_t at = (size_t)g.in_pitch * na + col * P + pl;
          uint32_t in = owner ? l_in[at] : 0u;
          if (p.use_status && owner && l_st[at] == GGRS_STATUS_DISCONNECTED) in = 4u;
          if (lean) slice_advance_lean(st, in, owner, sn, cs);
          else slice_advance(st, in, owner);
          if (p.trace) {
            const uint32_t ck = slice_fletcher<P>(st, pl);
            if (pl == 0) p.trace[(int64_t)(((int32_t)st.frame - 1) % p.trace_cap) * L + lane] = (uint16_t)ck;
          }
          slot = slot + 1 == R ? 0 : slot + 1;
          ++na;
        }
      }
      result = (int32_t)st.frame;
      ns_done = ns;
    }
    if (pl == 0) {
      l_res[col] = result;
      if (ns_done) atomicMax(&s_rows, ns_done);
      if (result < 0) atomicAdd(&s_fails, 1);
    }
  }
  __syncthreads();
  write_back(p, g, lds, sess0, nb, s_rows);
  return s_fails;
}

// One launch per batch.
template <int P>
__global__ __launch_bounds__(kLaneBlock) void lane_requests_kernel(LaneBatchParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr int Pp = LaneGeom<P>::Pp;
  const int pl = threadIdx.x % Pp;
  const int64_t lane = (int64_t)blockIdx.x * LaneGeom<P>::kSessions + threadIdx.x / Pp;
  const bool valid = lane < p.L;
  Slice st;
  load_slice<P>(st, p.cur + (valid ? lane : 0), p.L, pl);
  run_lanes<P>(p, st, lds);
  if (valid) store_slice<P>(st, p.cur + lane, p.L, pl);
}

// The lane server: one persistent launch serving batch after batch, so a call costs a few PCIe
// round trips instead of a kernel launch plus a stream synchronisation (~26 us between calls
// measured, profiles/r02/req_diag.log).  Protocol (tools/server_probe.hip measures its pieces):
//   * the host publishes a batch by one 64-bit store of the control word (epoch + the batch's shape,
//     so the device reads both in one atomic load) into pinned fine-grained host memory;
//   * only block 0 polls host memory (64+ blocks polling it over PCIe slowed every round trip 4-10x,
//     tools/server_probe.hip) and relays the word through device memory, where the other blocks
//     poll it with agent-scope loads;
//   * each block writes its checksums and results with system-scope stores (no device-cache
//     write-back needed), waits for them, and stores the epoch and its count of failed sessions
//     into its own 64-bit done slot in host memory; the host waits for every slot (no device
//     atomic or last-block hand-off on the way back) and scans lane results only when a block
//     counted a failure.
// A lane's state stays in registers between batches and goes back to `cur` when the server exits:
// on the quit bit, or when no batch arrived for `idle_ticks` of the constant wall clock (a watchdog
// every block reaches, so an abandoned server drains by itself).
namespace ctlw {  // the 64-bit control word
constexpr uint64_t kQuit = 1ull << 45;
__host__ __device__ constexpr uint64_t pack(int32_t epoch, int32_t W, int32_t LD, int32_t A, int32_t S, int st) {
  return (uint64_t)(uint32_t)epoch | ((uint64_t)W << 32) | ((uint64_t)LD << 40) | ((uint64_t)(st != 0) << 44) |
         ((uint64_t)A << 46) | ((uint64_t)S << 54);
}
__host__ __device__ constexpr int32_t epoch(uint64_t c) { return (int32_t)(uint32_t)c; }
__host__ __device__ constexpr bool quit(uint64_t c) { return (c & kQuit) != 0; }
}  // namespace ctlw

struct ServerDev {  // device memory
  uint64_t relay;   // block 0's copy of the control word for the other blocks
};

template <int P>
__global__ __launch_bounds__(kLaneBlock) void lane_server_kernel(LaneBatchParams p, const uint64_t* ctl, uint64_t* slots,
                                                            ServerDev* dev, int32_t start_epoch, int64_t idle_ticks) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ uint64_t s_ctl;
  const int wl = threadIdx.x;
  constexpr int Pp = LaneGeom<P>::Pp;
  const int pl = wl % Pp;
  const int64_t lane = (int64_t)blockIdx.x * LaneGeom<P>::kSessions + wl / Pp;
  const bool valid = lane < p.L;
  Slice st;
  load_slice<P>(st, p.cur + (valid ? lane : 0), p.L, pl);
  int32_t last = start_epoch;
  for (;;) {
    if (wl == 0) {
      const int64_t t0 = wall_clock64();
      uint64_t c;
      for (;;) {
        if (blockIdx.x == 0) {
          c = __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          const bool idle = wall_clock64() - t0 > idle_ticks;
          if (idle) c |= ctlw::kQuit;
          if (ctlw::quit(c) || ctlw::epoch(c) != last) {
            __hip_atomic_store(&dev->relay, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        } else {
          c = __hip_atomic_load(&dev->relay, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (ctlw::quit(c) || ctlw::epoch(c) != last) break;
          if (wall_clock64() - t0 > 2 * idle_ticks) {  // block 0 gone: leave as well
            c |= ctlw::kQuit;
            break;
          }
        }
        __builtin_amdgcn_s_sleep(2);
      }
      s_ctl = c;
    }
    __syncthreads();
    const uint64_t c = s_ctl;
    __syncthreads();
    if (ctlw::quit(c)) break;
    LaneBatchParams q = p;
    q.W = (int32_t)((c >> 32) & 0xff);
    q.LD = (int32_t)((c >> 40) & 0xf);
    q.use_status = (int32_t)((c >> 44) & 1);
    q.A = (int32_t)((c >> 46) & 0xff);
    q.S = (int32_t)((c >> 54) & 0x1ff);
    const int fails = run_lanes<P>(q, st, lds);  // returns after this thread's host stores left
    __syncthreads();
    const int32_t e = ctlw::epoch(c);
    if (wl == 0)  // this block's part of the batch is in host memory
      __hip_atomic_store(&slots[blockIdx.x], (uint64_t)(uint32_t)e | ((uint64_t)(uint32_t)fails << 32), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    last = e;
  }
  if (valid) store_slice<P>(st, p.cur + lane, p.L, pl);
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
  // pinned, fine-grained (coherent) and mapped into the device's address space: the kernel reads
  // the rows and writes the results in place, and the persistent server sees every new batch
  if (int rc = lane_server_stop(e)) return rc;
  HIP_TRY(hipHostMalloc((void**)&n.base, n.bytes, hipHostMallocMapped | hipHostMallocCoherent));
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

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

LaneBatchParams batch_params(ggrs_engine* e, int32_t W, int32_t LD, int32_t A, int32_t S, int use_status) {
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
  p.wide = p.L % 8 == 0;
  p.tokens = device_view(v.tokens);
  p.load_frames = device_view(v.load_frames);
  p.inputs = device_view(v.inputs);
  p.status = device_view(v.status);
  p.cks = device_view(v.checksums);
  p.result = device_view(v.lane_result);
  p.cur = e->cur;
  p.ring = e->ring;
  p.ring_ck = e->ring_ck;
  p.trace = e->trace;
  return p;
}

constexpr double kServerIdleHost = 0.25;  // the host restarts a server idle this long (s) ...
constexpr double kServerIdleKernel = 1.0; // ... well before the kernel's own watchdog ends it

// Lane servers running per device.  Each persistent server holds a hardware queue; HIP spreads a
// process's streams over GPU_MAX_HW_QUEUES of them (default 4), so a server beyond that shares an
// in-order queue with another and waits for it to go idle.  Engines beyond the limit
// serve their batches with one launch each.
constexpr int kMaxDevices = 64;
std::atomic<int> g_servers[kMaxDevices];

int server_limit() {
  static const int lim = [] {
    const char* v = std::getenv("GPU_MAX_HW_QUEUES");
    const int n = v ? std::atoi(v) : 0;
    return n > 0 ? n : 4;
  }();
  return lim;
}

// take one of the device's server slots (false: all taken)
bool server_slot_take(ggrs_engine* e) {
  const int d = e->cfg.device;
  if (d < 0 || d >= kMaxDevices) return false;
  int n = g_servers[d].load();
  while (n < server_limit())
    if (g_servers[d].compare_exchange_weak(n, n + 1)) {
      e->server.counted = true;
      return true;
    }
  return false;
}

void server_slot_release(ggrs_engine* e) {
  if (!e->server.counted) return;
  e->server.counted = false;
  g_servers[e->cfg.device].fetch_sub(1);
}

int server_start(ggrs_engine* e) {
  LaneServerHost& s = e->server;
  const int64_t L = e->cfg.num_lanes;
  s.blocks = (int32_t)grid_of(L, kLaneBlock / padded_players(e->cfg.num_players));
  if (!s.mem) {  // control word, then one 64-bit done slot per block
    HIP_TRY(hipHostMalloc((void**)&s.mem, 64 + 8 * (size_t)s.blocks, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(s.mem, 0, 64 + 8 * (size_t)s.blocks);
    HIP_TRY(hipMalloc(&s.dev, sizeof(ServerDev)));
    int rate_khz = 0;
    HIP_TRY(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, e->cfg.device));
    s.idle_ticks = (int64_t)(kServerIdleKernel * 1e3 * (rate_khz > 0 ? rate_khz : 100000));
  }
  uint64_t* ctl = (uint64_t*)s.mem;
  __atomic_store_n(ctl, ctlw::pack(s.epoch, 0, 0, 0, 0, 0), __ATOMIC_RELEASE);
  ServerDev init{ctlw::pack(s.epoch, 0, 0, 0, 0, 0)};
  HIP_TRY(hipMemcpyAsync(s.dev, &init, sizeof init, hipMemcpyHostToDevice, e->stream));
  const LaneBatchHost& b = e->batch;
  LaneBatchParams p = batch_params(e, b.words, b.loads, b.adv, b.saves, 1);
  if (!p.tokens || !p.load_frames || !p.inputs || !p.status || !p.cks || !p.result)
    return set_error(GGRS_E_HIP, "hipHostGetDevicePointer failed for the lane batch");
  const uint64_t* dctl = device_view((const uint64_t*)ctl);
  uint64_t* ddone = device_view((uint64_t*)(s.mem + 64));
  if (!dctl || !ddone) return set_error(GGRS_E_HIP, "hipHostGetDevicePointer failed for the lane server");
  const size_t lds = LaneLds(e->cfg.num_players, b.words, b.loads, e->R, b.adv, b.saves, 1).bytes;
  // every block must be resident at once (block 0 relays the batches to the others)
  int per_cu = 0, cus = 0;
  int rc = GGRS_OK;
  dispatch_players(e->cfg.num_players, [&](auto PC) {
    constexpr int P = decltype(PC)::value;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lane_server_kernel<P>, kLaneBlock, lds) != hipSuccess) rc = 1;
  });
  HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, e->cfg.device));
  if (rc || (int64_t)per_cu * cus < s.blocks) {
    s.enabled = false;  // too many lanes to keep resident: one launch per batch instead
    return GGRS_OK;
  }
  if (!server_slot_take(e)) return GGRS_E_STATE;  // every server slot taken: this batch as a launch
  dispatch_players(e->cfg.num_players, [&](auto PC) {
    constexpr int P = decltype(PC)::value;
    lane_server_kernel<P><<<s.blocks, kLaneBlock, lds, e->stream>>>(p, dctl, ddone, (ServerDev*)s.dev, s.epoch,
                                                                s.idle_ticks);
  });
  if (hipError_t err = hipGetLastError(); err != hipSuccess) {
    server_slot_release(e);
    return set_error(GGRS_E_HIP, "lane server launch: %s", hipGetErrorString(err));
  }
  s.running = true;
  s.last_done = now_s();
  return GGRS_OK;
}

// Publish one batch to the running server (returns at once; server_collect waits for it).
int server_publish(ggrs_engine* e, int32_t W, int32_t LD, int32_t A, int32_t S, int use_status) {
  LaneServerHost& s = e->server;
  if (s.running && now_s() - s.last_done > kServerIdleHost) {
    if (int rc = lane_server_stop(e)) return rc;
  }
  if (!s.running) {
    if (int rc = server_start(e)) return rc;  // GGRS_E_STATE: no server slot free right now
    if (!s.enabled) return GGRS_E_STATE;  // caller falls back to a launch per batch
  }
  uint64_t* ctl = (uint64_t*)s.mem;
  const int32_t ep = ++s.epoch;
  __atomic_store_n(ctl, ctlw::pack(ep, W, LD, A, S, use_status), __ATOMIC_RELEASE);  // after the batch rows
  s.pending = 1;
  s.pending_epoch = ep;
  s.pending_t0 = now_s();
  return GGRS_OK;
}

// Spin until every block of the published batch reports it done; *fails = the batch's sessions
// that failed validation.  A batch not done within 10 s marks the engine failed: the quit bit is
// set, but the old server may still be inside that batch (and would see a new control word), so no
// later batch is published on this engine.
int server_collect(ggrs_engine* e, int32_t* fails) {
  LaneServerHost& s = e->server;
  const uint64_t* slots = (const uint64_t*)(s.mem + 64);
  const int32_t ep = s.pending_epoch;
  int spins = 0;
  int32_t b = 0;
  uint32_t failed = 0;
  for (;;) {  // every block's slot holds this epoch (blocks finish in any order)
    while (b < s.blocks) {
      const uint64_t d = __atomic_load_n(&slots[b], __ATOMIC_ACQUIRE);
      if ((int32_t)(uint32_t)d != ep) break;
      failed += (uint32_t)(d >> 32);
      ++b;
    }
    if (b == s.blocks) break;
    _mm_pause();
    if (++spins == 4096) {
      spins = 0;
      if (now_s() - s.pending_t0 > 10.0) {
        uint64_t* ctl = (uint64_t*)s.mem;
        __atomic_store_n(ctl, __atomic_load_n(ctl, __ATOMIC_ACQUIRE) | ctlw::kQuit, __ATOMIC_RELEASE);
        s.running = false;
        s.pending = 0;
        s.failed = true;
        return set_error(GGRS_E_HIP, "lane server did not finish batch %d within 10 s; the engine takes no "
                                     "further batches", ep);
      }
    }
  }
  s.pending = 0;
  s.last_done = now_s();
  *fails = (int32_t)failed;
  return GGRS_OK;
}

// Submits the engine's mapped batch with the given counts: to the lane server, or as one launch.
int submit_batch(ggrs_engine* e, int32_t W, int32_t LD, int32_t A, int32_t S, int use_status) {
  e->mode = kModeLaneRequests;
  if (e->server.failed) return set_error(GGRS_E_STATE, "an earlier lane batch timed out on this engine");
  e->server.orphan = false;  // a new batch: an earlier collected result is no longer waited for
  if (e->server.enabled) {
    const int rc = server_publish(e, W, LD, A, S, use_status);
    // GGRS_E_STATE: the grid cannot stay resident, or every server slot of the device is taken:
    // launch instead
    if (rc != GGRS_E_STATE) return rc;
  }
  LaneBatchParams p = batch_params(e, W, LD, A, S, use_status);
  if (!p.tokens || !p.load_frames || !p.inputs || !p.status || !p.cks || !p.result)
    return set_error(GGRS_E_HIP, "hipHostGetDevicePointer failed for the lane batch");
  const size_t lds = LaneLds(e->cfg.num_players, W, LD, e->R, A, S, use_status).bytes;
  const int64_t grid = grid_of(p.L, kLaneBlock / padded_players(e->cfg.num_players));
  int rc = launch_timed(e, [&] {
    dispatch_players(e->cfg.num_players, [&](auto PC) {
      constexpr int P = decltype(PC)::value;
      lane_requests_kernel<P><<<grid, kLaneBlock, lds, e->stream>>>(p);
    });
  });
  if (rc) return rc;
  e->server.pending = 2;
  return GGRS_OK;
}

// Waits for the submitted batch; *fails = the sessions that failed validation, or -1 when only
// the lane results tell (one launch per batch).
int wait_batch(ggrs_engine* e, int32_t* fails) {
  *fails = -1;
  const int pending = e->server.pending;
  if (pending == 1) return server_collect(e, fails);
  if (pending == 2) {
    e->server.pending = 0;
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  return GGRS_OK;
}

int run_batch(ggrs_engine* e, int32_t W, int32_t LD, int32_t A, int32_t S, int use_status, int32_t* fails) {
  *fails = -1;
  if (int rc = submit_batch(e, W, LD, A, S, use_status)) return rc;
  return wait_batch(e, fails);
}

int check_mode(const ggrs_engine* e) {
  if (e->mode == kModeSyncTest || e->mode == kModeLockstepRequests)
    return set_error(GGRS_E_STATE, "engine already driven by a lane-uniform program");
  return GGRS_OK;
}

// the device's LDS per workgroup (read once per engine; a non-positive report is taken as the
// 64 KiB every CDNA workgroup gets)
int lds_limit(ggrs_engine* e, int* out) {
  int& max_lds = e->max_lds_per_block;
  if (max_lds == 0) {
    int v = 0;
    HIP_TRY(hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, e->cfg.device));
    max_lds = v > 0 ? v : 65536;
  }
  *out = max_lds;
  return GGRS_OK;
}

size_t lane_lds_need(const ggrs_engine* e, int32_t W, int32_t LD, int32_t A, int32_t S) {
  return LaneLds(e->cfg.num_players, W, LD, e->R, A, S, 1).bytes + 64;  // + the static words
}

// the lane block's LDS for a batch shape must fit one workgroup's allotment on the device
int check_lds(ggrs_engine* e, int32_t W, int32_t LD, int32_t A, int32_t S) {
  int max_lds = 0;
  if (int rc = lds_limit(e, &max_lds)) return rc;
  const size_t need = lane_lds_need(e, W, LD, A, S);
  if (need > (size_t)max_lds)
    return set_error(GGRS_E_INVALID, "lane batch shape (%d words, %d loads, %d advances, %d saves) needs %zu bytes "
                                     "of LDS per lane block, more than the device's %d", W, LD, A, S, need, max_lds);
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

namespace ggrs {

int lane_server_stop(ggrs_engine* e) {
  LaneServerHost& s = e->server;
  if (s.pending) {  // a submitted batch first runs to completion (a quit word would skip it)
    int32_t fails;
    if (int rc = wait_batch(e, &fails)) return rc;
    s.orphan = true;  // the caller's ggrs_lane_batch_wait gets this batch's result
    s.orphan_fails = fails;
  }
  if (!s.running) {
    if (!s.failed) server_slot_release(e);  // a timed-out server may still hold its queue
    return GGRS_OK;
  }
  uint64_t* ctl = (uint64_t*)s.mem;
  __atomic_store_n(ctl, __atomic_load_n(ctl, __ATOMIC_ACQUIRE) | ctlw::kQuit, __ATOMIC_RELEASE);
  s.running = false;
  HIP_TRY(hipStreamSynchronize(e->stream));  // every block leaves its loop and stores its lanes' state
  server_slot_release(e);
  return GGRS_OK;
}

void lane_server_release(ggrs_engine* e) { server_slot_release(e); }

}  // namespace ggrs

extern "C" {

int ggrs_lane_batch_map(ggrs_engine_t* e, int32_t W, int32_t LD, int32_t A, int32_t S, ggrs_lane_batch_t* out) {
  if (!e || !out) return set_error(GGRS_E_INVALID, "null argument");
  int rc = check_shape(W, LD, A, S);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(e->cfg.device));
  if ((rc = check_lds(e, std::max(W, e->batch.words), std::max(LD, e->batch.loads), std::max(A, e->batch.adv),
                      std::max(S, e->batch.saves))))
    return rc;
  rc = map_batch(e, W, LD, A, S);
  if (rc) return rc;
  fill_batch_view(e, out);
  return GGRS_OK;
}

int ggrs_lane_batch_lds(ggrs_engine_t* e, int32_t W, int32_t LD, int32_t A, int32_t S, int64_t* need_bytes,
                        int64_t* limit_bytes) {
  if (!e || !need_bytes || !limit_bytes) return set_error(GGRS_E_INVALID, "null argument");
  if (int rc = check_shape(W, LD, A, S)) return rc;
  HIP_TRY(hipSetDevice(e->cfg.device));
  int lim = 0;
  if (int rc = lds_limit(e, &lim)) return rc;
  *need_bytes = (int64_t)lane_lds_need(e, W, LD, A, S);
  *limit_bytes = lim;
  return GGRS_OK;
}

int ggrs_lane_batch_submit(ggrs_engine_t* e, const ggrs_lane_batch_t* b, int32_t flags) {
  if (!e || !b) return set_error(GGRS_E_INVALID, "null argument");
  int rc = check_mode(e);
  if (rc) return rc;
  if (e->server.pending) return set_error(GGRS_E_STATE, "a submitted lane batch has not been waited for");
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
  e->lane_frame.clear();  // the lanes' frames move on the device only
  return submit_batch(e, b->token_words, b->load_slots, b->adv_rows, b->save_rows, (flags & GGRS_BATCH_STATUS) != 0);
}

int ggrs_lane_batch_wait(ggrs_engine_t* e, int32_t* n_failed) {
  if (!e) return set_error(GGRS_E_INVALID, "null argument");
  if (n_failed) *n_failed = 0;
  int32_t fails = -1;
  if (!e->server.pending) {
    // the batch was already collected by another call on the engine (which waits for it first)
    if (!e->server.orphan) return set_error(GGRS_E_STATE, "no lane batch submitted");
    e->server.orphan = false;
    fails = e->server.orphan_fails;
  } else {
    HIP_TRY(hipSetDevice(e->cfg.device));
    if (int rc = wait_batch(e, &fails)) return rc;
  }
  if (fails == 0) return GGRS_OK;  // the server counted no failed lane: no scan of the results
  ggrs_lane_batch_t v;
  fill_batch_view(e, &v);
  return report_failures(e, v.lane_result, n_failed);
}

int ggrs_lane_batch_run(ggrs_engine_t* e, const ggrs_lane_batch_t* b, int32_t flags, int32_t* n_failed) {
  if (!e || !b) return set_error(GGRS_E_INVALID, "null argument");
  if (n_failed) *n_failed = 0;
  int rc = check_mode(e);
  if (rc) return rc;
  if (e->server.pending) return set_error(GGRS_E_STATE, "a submitted lane batch has not been waited for");
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
  int32_t fails = -1;
  rc = run_batch(e, b->token_words, b->load_slots, b->adv_rows, b->save_rows, (flags & GGRS_BATCH_STATUS) != 0, &fails);
  if (rc) return rc;
  if (fails == 0) return GGRS_OK;  // the server counted no failed lane: no scan of the results
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
  if ((rc = check_lds(e, std::max(W, e->batch.words), std::max(max_ld, e->batch.loads),
                      std::max(max_adv, e->batch.adv), std::max(max_sv, e->batch.saves))))
    return rc;
  rc = map_batch(e, W, max_ld, max_adv, max_sv);
  if (rc) return rc;
  // every lane's frame at the start of its list: the Save frames are checked on the host
  if ((int64_t)e->lane_frame.size() != L) {
    if (int rc2 = lane_server_stop(e)) return rc2;
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
  int32_t fails = -1;
  rc = run_batch(e, W, max_ld, max_adv, max_sv, status != nullptr, &fails);
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

int ggrs_lane_server(ggrs_engine_t* e, int32_t on) {
  if (!e) return set_error(GGRS_E_INVALID, "null engine");
  HIP_TRY(hipSetDevice(e->cfg.device));
  if (!on) {
    if (int rc = lane_server_stop(e)) return rc;
  }
  e->server.enabled = on != 0;
  return GGRS_OK;
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
