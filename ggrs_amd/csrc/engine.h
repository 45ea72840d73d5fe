// engine.h -- the SyncTest / request engine object shared by engine.hip (SyncTest program, lockstep
// request lists) and requests.hip (per-lane request lists).  Internal: not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "common.h"

// Engine modes: which program drives the lanes (they cannot be mixed on one engine: the SyncTest
// and lockstep request programs keep lane-uniform frame bookkeeping on the host, per-lane request
// lists keep each lane's frames on the device).
enum EngineMode { kModeFresh = 0, kModeSyncTest = 1, kModeLockstepRequests = 2, kModeLaneRequests = 3 };

// engine-owned host memory of a per-lane request batch (ggrs_lane_batch_t points into it)
struct LaneBatchHost {
  uint8_t* base = nullptr;  // one pinned, device-mapped allocation
  size_t bytes = 0;
  int32_t words = 0, loads = 0, adv = 0, saves = 0;  // the shape it was laid out for
  size_t off_tokens = 0, off_loads = 0, off_inputs = 0, off_status = 0, off_save_frames = 0,
         off_cks = 0, off_result = 0;
};

// the persistent lane server of requests.hip (ggrs_lane_server)
struct LaneServerHost {
  uint8_t* mem = nullptr;  // pinned, fine-grained, mapped: 64-bit control word | per-block done slots
  void* dev = nullptr;     // device memory: the relay word
  bool enabled = true, running = false;
  int32_t epoch = 0;
  int32_t blocks = 0;
  double last_done = 0.0;  // steady-clock seconds of the last finished batch
  int64_t idle_ticks = 0;  // the kernel's idle watchdog, in wall-clock ticks
  int pending = 0;         // a submitted batch not yet waited for: 1 on the server, 2 as a launch
  int32_t pending_epoch = 0;
  double pending_t0 = 0.0;
  bool failed = false;     // a batch timed out: the server may still hold it; no further batches
  bool counted = false;    // this engine's server holds one of the device's server slots
  bool orphan = false;     // a submitted batch was collected by another call (lane_server_stop):
  int32_t orphan_fails = 0;  // its failure count, returned by the next ggrs_lane_batch_wait
};

struct ggrs_engine {
  ggrs_config_t cfg{};
  int Pp = 1, F = 1, R = 1, cap = 128;
  int mode = kModeFresh;
  hipStream_t stream = nullptr;
  uint32_t* cur = nullptr;
  uint32_t* ring = nullptr;
  uint16_t* ring_ck = nullptr;
  uint16_t* first_ck = nullptr;
  uint8_t* inputs = nullptr;
  int32_t* lane_status = nullptr;
  int32_t* mis_frame = nullptr;
  uint64_t* mis_mask = nullptr;
  uint16_t* trace = nullptr;
  uint8_t* staging = nullptr;  // device scratch for request inputs / status / request list
  size_t staging_bytes = 0;
  uint8_t* host_staging = nullptr;  // pinned host copy of a request call's list + inputs (one DMA)
  size_t host_staging_bytes = 0;
  // cur | ring | ring_ck | first_ck live in one arena so a launch checkpoint is one copy
  uint8_t* arena = nullptr;
  uint8_t* shadow = nullptr;
  size_t arena_bytes = 0;
  size_t shadow_bytes = 0;
  bool shadow_blocked = false;  // the unverified launches' checkpoint is in the v4 block layout
  int32_t* fail_f0 = nullptr;   // f0 of the first pipelined launch whose checks failed, or -1
  bool unverified = false;      // pipelined launches enqueued since the last resolve()
  int path = GGRS_PATH_PIPELINED;
  // host-side (lane-uniform) bookkeeping
  int32_t current_frame = 0;
  int32_t next_user_frame = 0;  // next user frame add_local_inputs expects
  std::vector<int32_t> ring_tag;
  int32_t corrupt_lane = -1, corrupt_frame = -1;
  // timing: between ggrs_timing_reset and ggrs_timing_read one event pair brackets every fused
  // launch of the span (no per-launch events in the timed path)
  hipEvent_t ev_begin = nullptr, ev_end = nullptr;
  bool collecting = false, span_open = false, span_stopped = false;
  int32_t span_launches = 0;
  float last_span_ms = -1.0f;
  int32_t last_span_launches = 0;
  // per-lane request lists
  LaneBatchHost batch;
  LaneServerHost server;
  int max_lds_per_block = 0;        // the device's LDS per workgroup (read once, lane batches)
  std::vector<int32_t> lane_frame;  // each lane's frame, as ggrs_handle_requests_lanes last left it
                                    // (empty: unknown, read from the device when needed)
};

namespace ggrs {

// Ends the persistent lane server (requests.hip) if it runs: every other use of the engine's stream
// or device buffers must come after it.
int lane_server_stop(ggrs_engine* e);
// give back the engine's lane-server slot on the device (engine destruction)
void lane_server_release(ggrs_engine* e);

// Counts one fused launch of a timed span; the span's first launch records its begin event.
template <typename K>
inline int launch_timed(ggrs_engine* e, K&& launch) {
  if (e->collecting && !e->span_open) {
    HIP_TRY(hipEventRecord(e->ev_begin, e->stream));
    e->span_open = true;
  }
  launch();
  HIP_TRY(hipGetLastError());
  if (e->collecting) e->span_launches++;
  return GGRS_OK;
}

}  // namespace ggrs
