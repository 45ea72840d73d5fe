// p2p_engine.h -- the P2P engine object shared by p2p.hip (fixed-latency network: every kernel form,
// desync detection, lockstep) and p2p_sched.hip (scheduled arrivals: per-session remote-arrival
// tables, the prediction threshold and disconnects).  Host-side only; no kernels here.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "common.h"

struct ggrs_p2p_engine {
  ggrs_p2p_config_t cfg{};
  int Pp = 1, F = 1, R = 2, cap = 256;
  int num_cus = 256;                 // the device's CUs (LDS-ring occupancy rule)
  hipStream_t stream = nullptr;
  uint32_t* cur = nullptr;
  uint32_t* ring = nullptr;
  uint8_t* inputs = nullptr;
  int32_t* queue = nullptr;
  int32_t* rollbacks = nullptr;
  int64_t* resim = nullptr;
  uint16_t* trace = nullptr;
  uint8_t* staging = nullptr;
  size_t staging_bytes = 0;
  int32_t current_frame = 0;         // advance_frame calls made (the session frame in rollback mode
                                     // with a fixed latency; per session in scheduled mode)
  int32_t next_input_frame = 0;
  int32_t desync_interval = 0;
  uint16_t* hist = nullptr;     // [kHist][S] local checksum history
  uint64_t* cmp_mask = nullptr; // [ceil(S/64)] compare result
  int32_t* cmp_count = nullptr;
  int64_t dbg_sess = -1;
  int32_t dbg_frame = -1;
  int32_t sparse = 0;
  int32_t form = 0;  // ggrs_p2p_set_unstaged: 0 default (canonical flat, or chains for few sessions),
                     // 1 global input reads, 2 lockstep staged, 3 flat with HBM rings, 4 chains,
                     // 5 flat with LDS rings and the queue bookkeeping, 6 canonical flat
  bool dbg_ever = false;  // a debug flip was armed: the states may no longer be the canonical ones
  int32_t* last_saved = nullptr;  // [S], sparse saving only
  int32_t* ring_frame = nullptr;  // [R][S]: the frame each cell holds (sparse saving, scheduled mode)
  // lockstep mode (max_prediction 0): the session-uniform control flow, replayed on the host
  int32_t ls_frame = 0;                     // SyncLayer::current_frame
  int32_t ls_local_last = GGRS_NULL_FRAME;  // local players' last queue frame (local_connect_status)
  std::vector<int32_t> ls_row_of;           // queue frame q -> the call (input row) that added it, q % size
  int32_t* ls_prog = nullptr;               // device copy of a launch's (local row, remote row) pairs
  int32_t ls_prog_cap = 0;
  // scheduled arrivals (ggrs_p2p_set_arrival_schedule; p2p_sched.hip)
  int32_t sched = 0;
  int32_t next_arrival_call = 0;
  int32_t* arrive = nullptr;      // [cap][S] newest remote frame delivered by call c, row c % cap
  uint8_t* events = nullptr;      // [cap][S] Event::Disconnected bits of call c
  int32_t* peer_reports = nullptr;  // [cap][S] the peers' disconnect reports of call c (ggrs_p2p_add_peer_reports)
  int32_t* row_tag = nullptr;     // [cap] the frame whose input row each row slot holds
  std::vector<int32_t> row_tag_host;
  uint32_t* iq = nullptr;         // [kSchedQueue][S] every player's queued input of frame q, q % kSchedQueue
  int32_t* sst = nullptr;         // [sched_fields(P)][S] SyncLayer / InputQueue / connect-status words
  // scheduled desync detection: per call (row c % cap) the report sent, its checksum, the
  // last_confirmed_frame compared against, the last queued local frame; every frame's final cell
  // checksum [sched_hf][S]
  int32_t* rep_frame = nullptr;
  uint16_t* rep_ck = nullptr;
  int32_t* rep_lconf = nullptr;
  int32_t* rep_ll = nullptr;
  uint16_t* fck = nullptr;
  int32_t sched_hf = 0;
  ggrs::SpanTimer timer;
};

namespace ggrs {
// p2p_sched.hip: enable scheduled mode (allocate and initialise its buffers), run n calls, upload arrival rows
int p2p_sched_enable(ggrs_p2p_engine* e);
int p2p_sched_advance(ggrs_p2p_engine* e, int32_t n);
int p2p_sched_free(ggrs_p2p_engine* e);
int p2p_sched_desync_alloc(ggrs_p2p_engine* e);  // desync detection's buffers (scheduled mode)
}  // namespace ggrs
