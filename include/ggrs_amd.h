/*
 * ggrs_amd.h -- C ABI of the MI355X batched rollback-resimulation engine.
 *
 * One engine owns L lanes.  A lane is one (session, branch): its own ex_game State, its own
 * saved-state ring and its own input stream.  Every call acts on all lanes at once: either one
 * request program for every lane (the fused SyncTest program, or a lockstep request list -- the
 * kinds and frames GGRS sessions in lockstep emit are identical, only inputs differ) or one list per
 * lane (ggrs_handle_requests_lanes / ggrs_lane_batch_run: P2P sessions that roll back to their own
 * frames).
 *
 * Replaces (caspark/ggrs 0.10.2, file:line):
 *   ggrs_engine_create         SessionBuilder::start_synctest_session (src/sessions/builder.rs:346-358)
 *                              + SyncLayer::new / SavedStates::new (src/sync_layer.rs:149-159,183-198)
 *                              + Game::new / State::new (examples/ex_game/ex_game.rs:67-76,246-269)
 *   ggrs_add_local_inputs      SyncTestSession::add_local_input (src/sessions/sync_test_session.rs:61-74)
 *                              feeding InputQueue::add_input (src/input_queue.rs:170-186) with the
 *                              session's input delay (src/input_queue.rs:233-265)
 *   ggrs_synctest_advance_frames
 *                              n x { SyncTestSession::advance_frame (sync_test_session.rs:85-150)
 *                              incl. checksums_consistent (:173-190) and adjust_gamestate (:192-217),
 *                              then Game::handle_requests (ex_game.rs:79-99) }
 *   ggrs_handle_requests       Game::handle_requests (ex_game.rs:79-99) for an ordered
 *                              Vec<GgrsRequest> (src/lib.rs:171-195): SaveGameState -> save_game_state
 *                              (ex_game.rs:103-108), LoadGameState -> load_game_state (:111-113),
 *                              AdvanceFrame -> advance_frame (:115-127)
 *   ggrs_read_save_checksums   the `Some(checksum)` a handler passes to GameStateCell::save
 *                              (sync_layer.rs:18-24), so a GGRS session can keep `data = None`
 *                              cells while the states live in HBM
 *   ggrs_read_mismatches       GgrsError::MismatchedChecksum { current_frame, mismatched_frames }
 *                              (src/error.rs:44-50), per lane
 *   ggrs_handle_requests_lanes Game::handle_requests for every lane's own Vec<GgrsRequest>, as
 *   ggrs_lane_batch_run        P2PSession::advance_frame emits them (p2p_session.rs:265-426)
 *
 * Errors: every function returns GGRS_OK (0) or a negative GGRS_E_* code; ggrs_last_error() gives
 * the message.  The reference panics (assert!) on precondition violations (sync_layer.rs:20,
 * 231-248; ex_game.rs:104); this ABI never unwinds and reports them as GGRS_E_PRECONDITION
 * without touching device state.  A checksum mismatch is data, not an error code.
 *
 * Threading: an engine is used by one host thread at a time; work is enqueued on the engine's
 * own HIP stream and the read functions synchronise with it.  No torch types cross this ABI.
 */
#ifndef GGRS_AMD_H
#define GGRS_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: GGRS_PATH_* renumbered (2, 3 = the pipelined forms), lane batches submitted and waited for
 * separately, host-side lane encoding, branch round forms
 * 3: ggrs_branch_set_stream(e, NULL) binds HIP's null stream (it used to select the engine's own
 * stream); ggrs_branch_use_own_stream returns to the engine's own
 * 4: P2P arrival schedules (ggrs_p2p_set_arrival_schedule, ggrs_p2p_add_arrivals,
 * ggrs_p2p_read_sessions)
 * 5: desync detection under arrival schedules (ggrs_p2p_read_reports)
 * 6: bulk reads for every-lane checks (ggrs_read_states, ggrs_p2p_read_states, ggrs_branch_read_cells);
 * lockstep mode under arrival schedules, peers' disconnect reports (ggrs_p2p_add_peer_reports) */
#define GGRS_ABI_VERSION 6

#define GGRS_OK 0
#define GGRS_E_INVALID (-1)      /* GgrsError::InvalidRequest: bad argument or configuration */
#define GGRS_E_PRECONDITION (-2) /* a reference assert! would have panicked */
#define GGRS_E_HIP (-3)          /* HIP runtime error (message from hipGetErrorString) */
#define GGRS_E_STATE (-4)        /* call not valid in the engine's current mode */

#define GGRS_NULL_FRAME (-1) /* src/lib.rs:47 */

/* GgrsRequest kinds (src/lib.rs:171-195) */
#define GGRS_REQ_SAVE 0
#define GGRS_REQ_LOAD 1
#define GGRS_REQ_ADVANCE 2

/* InputStatus (src/lib.rs:106-113) as carried per player in the status bytes of an advance */
#define GGRS_STATUS_CONFIRMED 0
#define GGRS_STATUS_PREDICTED 1
#define GGRS_STATUS_DISCONNECTED 2

/* SyncTest execution paths (ggrs_set_synctest_path) */
#define GGRS_PATH_PIPELINED 0  /* default: concurrent rollback chains per session, one lane per
                                  (chain, player); picks CHAINS or BATCHED by wave packing */
#define GGRS_PATH_SEQUENTIAL 1 /* one lane per session, calls in order */
#define GGRS_PATH_PIPELINED_CHAINS 2  /* cd+1 chain lanes per player, when (cd+1) * padded players <= 64 */
#define GGRS_PATH_PIPELINED_BATCHED 3 /* check_distance 8: cd chain lanes per player, the chains'
                                         last advance batched every 8 frames (CHAINS otherwise) */

/* per-lane status */
#define GGRS_LANE_RUNNING 0
#define GGRS_LANE_MISMATCH 1 /* halted: SyncTestSession::advance_frame returned MismatchedChecksum */

typedef struct ggrs_config {
  int32_t num_lanes;      /* L >= 1: independent (session, branch) lanes */
  int32_t num_players;    /* 1..4 (ex_game.rs:70) */
  int32_t max_prediction; /* ring holds max_prediction + 1 saved states (sync_layer.rs:149-159) */
  int32_t check_distance; /* SyncTest check distance; must be < max_prediction (builder.rs:347) */
  int32_t input_delay;    /* local input delay in frames (builder.rs:154-158) */
  int32_t input_capacity; /* frames of queued input per lane; 0 = 128 (INPUT_QUEUE_LENGTH) */
  int32_t device;         /* HIP device ordinal */
  int32_t trace_capacity; /* frames of per-frame checksum trace kept on device; 0 = none */
} ggrs_config_t;

typedef struct ggrs_engine ggrs_engine_t;

typedef struct ggrs_request {
  int32_t kind;  /* GGRS_REQ_* */
  int32_t frame; /* Save/Load: the request's frame; Advance: ignored */
} ggrs_request_t;

int32_t ggrs_abi_version(void);
const char* ggrs_last_error(void);

int ggrs_engine_create(const ggrs_config_t* cfg, ggrs_engine_t** out);
int ggrs_engine_destroy(ggrs_engine_t* eng);
int ggrs_engine_config(const ggrs_engine_t* eng, ggrs_config_t* out);

/* Queue user inputs for frames [first_frame, first_frame + n_frames) of every lane.
 * inputs: [n_frames][num_lanes][num_players] bytes (Input.inp).  Frames must be added in order
 * starting at 0 (input_queue.rs:171-177); they enter the queue at frame + input_delay, frames
 * below the delay hold the default input (input_queue.rs:251-257).  `_device` takes a device
 * pointer (same layout) readable on the engine's stream. */
int ggrs_add_local_inputs(ggrs_engine_t* eng, int32_t first_frame, int32_t n_frames,
                          const uint8_t* inputs);
int ggrs_add_local_inputs_device(ggrs_engine_t* eng, int32_t first_frame, int32_t n_frames,
                                 const void* inputs_device);

/* Run n_frames SyncTest frames on every running lane (fused: one kernel launch; warm-up frames
 * f <= check_distance take one extra launch). */
int ggrs_synctest_advance_frames(ggrs_engine_t* eng, int32_t n_frames);
/* Choose the SyncTest kernel: GGRS_PATH_PIPELINED (default; a mismatch found there is re-run on
 * the sequential kernel from a checkpoint, so results are identical; sessions whose chains do not
 * fit one wavefront run sequentially), one of its two forms explicitly (_CHAINS, _BATCHED), or
 * GGRS_PATH_SEQUENTIAL. */
int ggrs_set_synctest_path(ggrs_engine_t* eng, int32_t path);

/* Execute an ordered request list on every lane (fused: one kernel launch).
 * inputs: [n_advance][num_lanes][num_players] Input.inp bytes, status: same shape InputStatus
 * bytes (NULL = all confirmed), one slice per AdvanceFrame in order.  Save checksums are kept on
 * device; read them with ggrs_read_save_checksums. */
int ggrs_handle_requests(ggrs_engine_t* eng, const ggrs_request_t* reqs, int32_t n_reqs,
                         const uint8_t* inputs, const uint8_t* status);

/* ---- Per-lane request lists: every lane is its own GGRS session.  A P2PSession rolls back to its
 * own first_incorrect frame and replays its own count of frames (p2p_session.rs:322-337,658-714),
 * so lanes' lists differ in kind, length and frames.  Two forms of one program:
 *   ggrs_handle_requests_lanes  the requests themselves, CSR over lanes: lane l's ordered
 *                               Vec<GgrsRequest> (src/lib.rs:171-195) is reqs[offsets[l] ..
 *                               offsets[l+1]); one checksum out per SaveGameState, in request order.
 *   ggrs_lane_batch_run         the same lists pre-encoded per lane (2-bit request kinds + the Load
 *                               frames: SURVEY.md 8b's rollback(load_frame, n, save_mask)) in
 *                               engine-owned pinned host memory the kernel reads directly, results
 *                               written straight back there: one launch, no copies.
 * Each lane's list is validated on the device before the lane's state is touched: a Load of a frame
 * its cell does not hold (SyncLayer::load_frame's assert, sync_layer.rs:248; ex_game.rs:112's
 * expect) or more requests of a kind than the batch holds fails the lane, which is left as it was
 * (the reference panics); every other lane runs.  ggrs_handle_requests_lanes also checks every
 * Save's frame against the lane's state frame (ex_game.rs:104).  Once an engine runs per-lane lists,
 * each lane keeps its own frame (ggrs_read_lane_frames, ggrs_read_ring); the lane-uniform calls
 * (ggrs_synctest_advance_frames, ggrs_handle_requests, ggrs_current_frame,
 * ggrs_read_save_checksums) return GGRS_E_STATE. */
#define GGRS_TOK_SAVE 0
#define GGRS_TOK_ADVANCE 1
#define GGRS_TOK_LOAD 2
#define GGRS_TOK_END 3
#define GGRS_TOKENS_PER_WORD 16

#define GGRS_BATCH_STATUS 1 /* ggrs_lane_batch_run reads the status rows (else every input Confirmed) */

/* shape limits of a lane batch */
#define GGRS_BATCH_MAX_WORDS 32 /* 512 requests per lane */
#define GGRS_BATCH_MAX_LOADS 8
#define GGRS_BATCH_MAX_ADV 128
#define GGRS_BATCH_MAX_SAVES 256

typedef struct ggrs_lane_batch {
  int32_t token_words;  /* W: words of request kinds per lane (16 per word) */
  int32_t load_slots;   /* LD: Load frames per lane (GGRS 0.10.2 emits at most 2 per list) */
  int32_t adv_rows;     /* A: AdvanceFrame rows per lane */
  int32_t save_rows;    /* S: SaveGameState checksums per lane */
  uint32_t* tokens;     /* [W][L]: lane l's request kinds in order, GGRS_TOK_* in 2 bits each,
                           least significant first, GGRS_TOK_END after the last (or W*16 long) */
  int32_t* load_frames; /* [LD][L]: frame of the lane's k-th LoadGameState */
  uint8_t* inputs;      /* [A][L][num_players]: Input.inp of the lane's a-th AdvanceFrame */
  uint8_t* status;      /* [A][L][num_players]: its InputStatus (GGRS_STATUS_*) */
  uint16_t* checksums;  /* out [S][L]: fletcher16 of the lane's k-th SaveGameState (the checksum a
                           handler passes to GameStateCell::save, sync_layer.rs:18-24) */
  int32_t* lane_result; /* out [L]: >= 0 the lane's frame after its list; < 0 -(1 + k) where k is
                           the index of the lane's first request that failed validation */
} ggrs_lane_batch_t;

/* Lay out (allocating or growing engine-owned pinned host memory) a batch of at least this shape
 * and return pointers into it; the pointers stay valid until the next _map with a larger shape or
 * ggrs_engine_destroy.  The caller fills tokens / load_frames / inputs (/ status) per call. */
int ggrs_lane_batch_map(ggrs_engine_t* eng, int32_t token_words, int32_t load_slots, int32_t adv_rows,
                        int32_t save_rows, ggrs_lane_batch_t* out);
/* Run every lane's list of a mapped batch (the counts in *batch may be lowered per call: rows past
 * them are not read).  flags: GGRS_BATCH_STATUS.  Returns when checksums and lane_result are in
 * host memory; GGRS_E_PRECONDITION when *n_failed lanes failed validation (the rest ran). */
int ggrs_lane_batch_run(ggrs_engine_t* eng, const ggrs_lane_batch_t* batch, int32_t flags, int32_t* n_failed);
/* LDS one lane block needs for a batch shape, and the device's limit per workgroup (bytes): shapes
 * with need > limit are GGRS_E_INVALID at ggrs_lane_batch_map. */
int ggrs_lane_batch_lds(ggrs_engine_t* eng, int32_t token_words, int32_t load_slots, int32_t adv_rows,
                        int32_t save_rows, int64_t* need_bytes, int64_t* limit_bytes);
/* ggrs_lane_batch_run in two halves.  _submit publishes the batch (to the lane server, or enqueues
 * one launch) and returns at once; _wait returns when its checksums and lane_result are in host
 * memory, with ggrs_lane_batch_run's result.  Between them the caller must not touch this batch's
 * memory, but may work on another engine's: a handler serving its sessions as two lane groups (two
 * engines) encodes and hands back one group while the other's batch is on the device.  Any other
 * call on the engine first waits for a submitted batch; its result is kept, and the next _wait
 * returns it (failed lanes included) instead of GGRS_E_STATE. */
int ggrs_lane_batch_submit(ggrs_engine_t* eng, const ggrs_lane_batch_t* batch, int32_t flags);
int ggrs_lane_batch_wait(ggrs_engine_t* eng, int32_t* n_failed);
/* Host-side encoding of one session's ordered request list (src/lib.rs:171-195) into column `lane`
 * of a lane batch -- the per-session work of a request handler, shared by every caller (the Rust
 * crate, the bench's C driver).  reqs[n_reqs]; inputs / status: [n_advance][num_players], one row
 * per AdvanceFrame in order (status NULL = Confirmed).  Writes every token word of the batch (END
 * after the list), the lane's Load frames and input / status rows.  lane_frame = the lane's frame
 * before the list (its previous lane_result; 0 for a fresh engine; GGRS_NULL_FRAME skips the check):
 * the batch carries no Save frames, so each SaveGameState's frame is checked here against the frame
 * the list has reached (Game::handle_requests' assert, ex_game.rs:104); on a mismatch the lane is
 * encoded with an empty list (it will not run), *bad_request = the request's index and the call
 * returns GGRS_E_PRECONDITION.  GGRS_E_INVALID: the list does not fit the batch's shape.  No device
 * access: usable without a GPU. */
int ggrs_lane_encode(const ggrs_lane_batch_t* batch, int64_t num_lanes, int32_t num_players, int64_t lane,
                     const ggrs_request_t* reqs, int32_t n_reqs, const uint8_t* inputs, const uint8_t* status,
                     int32_t lane_frame, int32_t* bad_request);
/* The batch shape one list needs: shape = {token words (ceil(n_reqs / 16): a list of exactly 16 W
 * requests needs no END token), Loads, AdvanceFrames, SaveGameStates}. */
int ggrs_lane_shape(const ggrs_request_t* reqs, int32_t n_reqs, int32_t* shape);
/* The generic form.  reqs: every lane's requests back to back, offsets: [num_lanes + 1]
 * (offsets[0] = 0).  inputs / status: [n_advance][num_players], one row per AdvanceFrame in the
 * same (lane, request) order; status NULL = all Confirmed.  save_checksums (may be NULL): one per
 * SaveGameState in the same order.  lane_result (may be NULL): [num_lanes] as in the batch.
 * GGRS_E_PRECONDITION when some lane's list failed validation (those lanes did not run). */
int ggrs_handle_requests_lanes(ggrs_engine_t* eng, const ggrs_request_t* reqs, const int32_t* offsets,
                               const uint8_t* inputs, const uint8_t* status, uint16_t* save_checksums,
                               int32_t* lane_result);
/* The lane server (default on): the first per-lane batch launches one persistent kernel that
 * serves every later batch -- the host publishes a batch by bumping an epoch in pinned host memory
 * and spins on per-block done flags, so a call costs one PCIe round trip instead of a launch plus a
 * stream synchronisation.  It ends (lanes' states back in device memory) before any other call
 * touches the engine's stream, when the host has been idle for 0.25 s, or by its own watchdog
 * after 1 s without a batch.  on = 0: one launch per batch.  At most GPU_MAX_HW_QUEUES (default 4)
 * servers run on one device at a time (each holds a hardware queue; a second server on the same
 * in-order queue would wait for the first to go idle): an engine that finds them all taken serves
 * its batches with one launch each until a server stops. */
int ggrs_lane_server(ggrs_engine_t* eng, int32_t on);
/* Every lane's current frame (its state's frame field): [num_lanes]. */
int ggrs_read_lane_frames(ggrs_engine_t* eng, int32_t* frames);

/* Block until all work queued on the engine's stream has finished. */
int ggrs_synchronize(ggrs_engine_t* eng);
/* Frame the engine's session is at (SyncTestSession::current_frame, sync_test_session.rs:153). */
int ggrs_current_frame(const ggrs_engine_t* eng, int32_t* out);
/* Per-lane status / mismatch: each array has num_lanes entries (any may be NULL).  mask bit k
 * set <=> frame (mismatch_frame - check_distance + k) mismatched. */
int ggrs_read_mismatches(ggrs_engine_t* eng, int32_t* lane_status, int32_t* mismatch_frame,
                         uint64_t* mismatch_mask);
/* Checksum stored with the saved cell of `frame` for every lane (num_lanes u16). */
int ggrs_read_save_checksums(ggrs_engine_t* eng, int32_t frame, uint16_t* out);
/* The same for n frames in one device-to-host transfer wait: out [n][num_lanes] (a request list's
 * saves, read once after ggrs_handle_requests instead of one synchronisation per save). */
int ggrs_read_save_checksums_frames(ggrs_engine_t* eng, const int32_t* frames, int32_t n, uint16_t* out);
/* Current game state of one lane as bincode bytes (36 + 20 * num_players). */
int ggrs_read_state(ggrs_engine_t* eng, int32_t lane, uint8_t* out);
/* ggrs_read_state for every lane, one transfer: out[num_lanes][36 + 20 * num_players]. */
int ggrs_read_states(ggrs_engine_t* eng, uint8_t* out);
/* Saved-state ring of one lane: frames[R], checksums[R], states[R][36 + 20 * num_players]. */
int ggrs_read_ring(ggrs_engine_t* eng, int32_t lane, int32_t* frames, uint16_t* checksums,
                   uint8_t* states);
/* Per-frame display checksum trace (fletcher16 of the state after each frame's final
 * AdvanceFrame, ex_game.rs:121-126) for frames [first_frame, first_frame + n_frames):
 * out[n_frames][num_lanes].  Requires trace_capacity > 0 and frames still held. */
int ggrs_read_trace(ggrs_engine_t* eng, int32_t first_frame, int32_t n_frames, uint16_t* out);

/* Fault injection (tests): after the LoadGameState of SyncTest call `frame`, flip the lowest
 * bit of player 0's x on `lane` -- a non-deterministic simulation the SyncTest must catch. */
int ggrs_debug_corrupt_on_load(ggrs_engine_t* eng, int32_t lane, int32_t frame);

/* Average device time per fused launch of the last timed span (ggrs_timing_reset .. _read), ms. */
int ggrs_last_launch_ms(ggrs_engine_t* eng, float* ms);
/* Time the fused launches from now on: one HIP event pair on the engine's stream brackets the
 * whole span (no per-launch events); _read synchronises, returns the span's milliseconds (launch
 * gaps included) and the number of fused launches in it, and stops collecting. */
int ggrs_timing_reset(ggrs_engine_t* eng);
/* Close the span without waiting: records its end event right behind the last launch (a caller
 * that then synchronises the stream itself reads the same span without an extra host round trip
 * inside its own wall clock).  _read after _stop reports that span.  Exception: a running lane
 * server is stopped first (the event would otherwise queue behind the persistent kernel), which
 * waits for a submitted batch and for the server to leave its loop. */
int ggrs_timing_stop(ggrs_engine_t* eng);
int ggrs_timing_read(ggrs_engine_t* eng, float* total_ms, int32_t* launches);

/* ---------------------------------------------------------------------------------------------
 * Speculative branch rollback (P2P).  Lane = (session, branch), lane = session * branches + branch.
 * A round = ggrs_branch_speculate (every lane: LoadGameState(trunk frame) of its session, then
 * window x (AdvanceFrame, SaveGameState) -- P2PSession::adjust_gamestate, p2p_session.rs:658-714,
 * plus the save of the current frame, :337 -- with the remote players' inputs from the branch
 * generator that replaces InputQueue prediction, input_queue.rs:104-167) followed by
 * ggrs_branch_confirm (the remote inputs of the trunk frame arrive: the trunk replays that frame
 * with them, every lane learns whether its branch survived -- assumed exactly those inputs,
 * input_queue.rs:199-218 -- and the per-session checksum + survival bits form the report that
 * multi-GPU runs all-gather, the ChecksumReport exchange of p2p_session.rs:939-975).
 */
typedef struct ggrs_branch_config {
  int32_t num_sessions;   /* S >= 1 */
  int32_t num_players;    /* 1..4 */
  int32_t remote_mask;    /* bit p: player p is remote (inputs confirmed late); others local */
  int32_t window;         /* W: frames speculated per round (1..62); ring = W + 1 saved states */
  int32_t branches;       /* B per session: 1 = PredictRepeatLast (lib.rs:390-395); A^E =
                             enumerate the first remote player over E frames, then hold */
  int32_t alphabet;       /* A: remote input values enumerated (16 for ex_game's 4 buttons) */
  int32_t input_capacity; /* frames of queued inputs per session; 0 = 128 */
  int32_t device;
} ggrs_branch_config_t;

typedef struct ggrs_branch_engine ggrs_branch_engine_t;

int ggrs_branch_engine_create(const ggrs_branch_config_t* cfg, ggrs_branch_engine_t** out);
int ggrs_branch_engine_destroy(ggrs_branch_engine_t* eng);
int ggrs_branch_engine_config(const ggrs_branch_engine_t* eng, ggrs_branch_config_t* out);
/* True inputs of every player for frames [first_frame, first_frame + n_frames):
 * [n_frames][num_sessions][num_players].  Remote players' values are only read once the frame
 * is confirmed (and as the repeat-last prediction source for later frames). */
int ggrs_branch_add_inputs(ggrs_branch_engine_t* eng, int32_t first_frame, int32_t n_frames,
                           const uint8_t* inputs);
int ggrs_branch_speculate(ggrs_branch_engine_t* eng);
/* Confirm the trunk frame; if report_device != NULL the round's report is also copied there
 * (device pointer, ggrs_branch_report_bytes bytes: [S] u16 checksums, padded to 8 bytes, then
 * ceil(L/64) u64 survival words) on the engine's stream. */
int ggrs_branch_confirm(ggrs_branch_engine_t* eng, void* report_device);
int ggrs_branch_report_bytes(const ggrs_branch_engine_t* eng, int64_t* out);
int ggrs_branch_synchronize(ggrs_branch_engine_t* eng);
int ggrs_branch_trunk_frame(const ggrs_branch_engine_t* eng, int32_t* out);
int ggrs_branch_read_report(ggrs_branch_engine_t* eng, uint16_t* checksums, uint64_t* survive_bits);
/* per session: first trunk frame at which a surviving branch's saved state disagreed with the
 * replayed trunk (a desync), or -1 */
int ggrs_branch_read_desync(ggrs_branch_engine_t* eng, int32_t* first_frame);
int ggrs_branch_read_trunk(ggrs_branch_engine_t* eng, int32_t session, uint8_t* out);
/* the saved state (bincode) and checksum of `frame` in one lane's ring (after prefix-shared rounds:
 * the cell of the lane's prefix representative, which holds the same state) */
int ggrs_branch_read_lane(ggrs_branch_engine_t* eng, int64_t lane, int32_t frame, uint16_t* checksum,
                          uint8_t* out);
/* ggrs_branch_read_lane for every lane at once (checking every lane against a CPU replay):
 * checksums [num_sessions * branches], states [num_sessions * branches][36 + 20 P] or NULL */
int ggrs_branch_read_cells(ggrs_branch_engine_t* eng, int32_t frame, uint16_t* checksums, uint8_t* states);
int ggrs_branch_timing_reset(ggrs_branch_engine_t* eng);
int ggrs_branch_timing_stop(ggrs_branch_engine_t* eng); /* as ggrs_timing_stop */
int ggrs_branch_timing_read(ggrs_branch_engine_t* eng, float* total_ms, int32_t* launches);
/* n_rounds x (ggrs_branch_speculate, ggrs_branch_confirm without a report copy) issued back to
 * back from native code; while timing is collected one event pair brackets the whole batch */
int ggrs_branch_rounds(ggrs_branch_engine_t* eng, int32_t n_rounds);
/* rounds() as one launch (on = 0, default: every block replays the trunks of its own sessions, so
 * no launch boundary is needed between rounds; when the enumerated player is the only remote one the
 * launch is prefix-shared -- each lane advances only that player, the local players' frames are
 * computed once per block and session, and a cell at depth k is saved once per distinct k+1-digit
 * prefix, by branch b mod A^min(k+1, E); ggrs_branch_read_lane resolves a lane's cell to it), as
 * 2 n launches of speculate / confirm (on = 1), or as one launch without prefix sharing (on = 2) */
int ggrs_branch_set_round_launches(ggrs_branch_engine_t* eng, int32_t on);
/* Enqueue every launch and copy from now on on `stream` (a hipStream_t; NULL = HIP's null stream,
 * as torch.cuda.current_stream() reports its default stream -- ABI 3; before it NULL meant the
 * engine's own non-blocking stream, which does not order with the null stream),
 * e.g. the stream a collective library orders its all-gather after: speculate, confirm (with its
 * report copy) and the report exchange then follow each other on the device with no host
 * synchronisation (multi-GPU configs 3/4, ggrs_amd/exchange.py ReportExchange).  Work queued
 * before the switch is ordered before work queued after it. */
int ggrs_branch_set_stream(ggrs_branch_engine_t* eng, void* stream);
/* Back to the engine's own (non-blocking) stream, the one it was created with; work queued before
 * the switch is ordered before work queued after it. */
int ggrs_branch_use_own_stream(ggrs_branch_engine_t* eng);
/* One round (speculate + confirm) as one launch; the round's report is also written to
 * report_device (device pointer, same layout as ggrs_branch_confirm's copy; NULL = none) by the
 * kernel itself -- the per-round call of the multi-GPU exchange loop. */
int ggrs_branch_round(ggrs_branch_engine_t* eng, void* report_device);
/* n rounds as one launch (ggrs_branch_rounds) with every round's report also written by the
 * kernel into row r of reports_device ([n][report_bytes], device) -- a batch of the multi-GPU
 * exchange loop, all-gathered once. */
int ggrs_branch_rounds_reports(ggrs_branch_engine_t* eng, int32_t n_rounds, void* reports_device);
/* Desync detection between peer replicas (compare_local_checksums_against_peers,
 * p2p_session.rs:904-937): `gathered` = world all-gathered reports ([world][report_bytes], device);
 * sessions whose checksum differs between rows `rank` and `peer` are added to *count_device
 * (device int64), and *first_frame_device (device int64, initialise to -1) takes `frame` if it is
 * still -1 and any differ.  Enqueued on the engine's stream, no host synchronisation. */
int ggrs_branch_compare_peer(ggrs_branch_engine_t* eng, const void* gathered, int32_t world, int32_t rank,
                             int32_t peer, int32_t frame, int64_t* count_device, int64_t* first_frame_device);
/* The same over a batch of rounds gathered at once: `gathered` = [world][rows_per_rank][report_bytes]
 * (each rank's reports of rows_per_rank consecutive rounds, one all-gather per batch), rows 0 ..
 * n_rows-1 compared, row k standing for frame first_frame + k; one launch. */
int ggrs_branch_compare_peer_rows(ggrs_branch_engine_t* eng, const void* gathered, int32_t world,
                                  int32_t rows_per_rank, int32_t n_rows, int32_t rank, int32_t peer,
                                  int32_t first_frame, int64_t* count_device, int64_t* first_frame_device);

/* ---------------------------------------------------------------------------------------------
 * Config-5 large-state stress game (defined by this build; ggrs_amd/csrc/particles.h):
 * a session is one frame counter + num_entities x 100-byte entities (an ex_game ship + 80 bytes
 * of integer payload), ~1 MB at 10k entities, so every Load/Save of the SyncTest program
 * (sync_test_session.rs:85-150) is an HBM stream.  One engine = num_sessions sessions.
 */
typedef struct ggrs_particle_config {
  int32_t num_sessions;
  int32_t num_entities;     /* multiple of 4, <= 160000 */
  int32_t num_players;      /* input bytes per frame; entity e plays player e % num_players */
  int32_t max_prediction;   /* ring = max_prediction + 1 states per session */
  int32_t check_distance;   /* 0..62, < max_prediction */
  int32_t input_capacity;   /* frames of queued input; 0 = 128 */
  int32_t device;
  int32_t first_session_id; /* global id of session 0 (seeds the initial payload) */
} ggrs_particle_config_t;

typedef struct ggrs_particle_engine ggrs_particle_engine_t;

int ggrs_particle_engine_create(const ggrs_particle_config_t* cfg, ggrs_particle_engine_t** out);
int ggrs_particle_engine_destroy(ggrs_particle_engine_t* eng);
/* inputs [n_frames][num_sessions][num_players], frames added in order from 0 (no input delay) */
int ggrs_particle_add_local_inputs(ggrs_particle_engine_t* eng, int32_t first_frame, int32_t n_frames,
                                   const uint8_t* inputs);
int ggrs_particle_synctest_advance_frames(ggrs_particle_engine_t* eng, int32_t n_frames);
int ggrs_particle_synchronize(ggrs_particle_engine_t* eng);
int ggrs_particle_current_frame(const ggrs_particle_engine_t* eng, int32_t* out);
int ggrs_particle_read_mismatches(ggrs_particle_engine_t* eng, int32_t* status, int32_t* mismatch_frame,
                                  uint64_t* mismatch_mask);
/* current state of one session in the declared layout (4 + 100 * num_entities bytes) */
int ggrs_particle_read_state(ggrs_particle_engine_t* eng, int32_t session, uint8_t* out);
/* the saved cell of `frame` (checksum and/or declared-layout bytes) */
int ggrs_particle_read_saved(ggrs_particle_engine_t* eng, int32_t session, int32_t frame, uint16_t* checksum,
                             uint8_t* out);
int ggrs_particle_debug_corrupt_on_load(ggrs_particle_engine_t* eng, int32_t session, int32_t frame);
int ggrs_particle_timing_reset(ggrs_particle_engine_t* eng);
int ggrs_particle_timing_stop(ggrs_particle_engine_t* eng); /* as ggrs_timing_stop */
int ggrs_particle_timing_read(ggrs_particle_engine_t* eng, float* total_ms, int32_t* launches);

/* ---------------------------------------------------------------------------------------------
 * P2P rollback decision: num_sessions independent P2PSessions of one peer,
 * each call = P2PSession::advance_frame (src/sessions/p2p_session.rs:265-426) + the ex_game
 * handler, with every remote player's InputQueue prediction (src/input_queue.rs:104-230) on the
 * device.  Rollback mode, sparse saving off, every player connected.  Network model: the remote
 * players' input of frame g arrives at the start of call g + remote_latency (poll_remote_clients
 * :430-446 -> handle_event Event::Input :880-895 -> SyncLayer::add_remote_input,
 * src/sync_layer.rs:271-277); the remote peer runs with input delay 0.
 */
typedef struct ggrs_p2p_config {
  int32_t num_sessions;
  int32_t num_players;     /* 1..4 (ex_game.rs:70) */
  int32_t local_mask;      /* bit p: player p is local to this peer; at least one player is remote */
  int32_t input_delay;     /* local players' frame delay (SessionBuilder::with_input_delay, builder.rs:150) */
  int32_t max_prediction;  /* builder.rs with_max_prediction_window; ring = max_prediction + 1; 0 =
                              lockstep mode (builder.rs:134-147): a call advances only once the
                              current frame's inputs are confirmed from every player, and never
                              saves, loads or resimulates (p2p_session.rs:301-310,393-407) */
  int32_t remote_latency;  /* 1 .. max_prediction-1 frames (any >= 1 in lockstep mode) */
  int32_t predictor;       /* 0 PredictRepeatLast, 1 PredictDefault (src/lib.rs:390-406) */
  int32_t input_capacity;  /* frames of queued input rows; 0 = 256 */
  int32_t trace_capacity;  /* calls of display checksums kept (0: none) */
  int32_t device;
} ggrs_p2p_config_t;

typedef struct ggrs_p2p_engine ggrs_p2p_engine_t;

int ggrs_p2p_engine_create(const ggrs_p2p_config_t* cfg, ggrs_p2p_engine_t** out);
int ggrs_p2p_engine_destroy(ggrs_p2p_engine_t* eng);
int ggrs_p2p_engine_config(const ggrs_p2p_engine_t* eng, ggrs_p2p_config_t* out);
/* inputs [n_frames][num_sessions][num_players]: row g holds the local players' add_local_input
 * (p2p_session.rs:219-246) of call g and the remote players' input of frame g (what the remote
 * peer sends, src/network/protocol.rs:564-642); rows are added in order from 0 */
int ggrs_p2p_add_inputs(ggrs_p2p_engine_t* eng, int32_t first_frame, int32_t n_frames, const uint8_t* inputs);
/* n_frames calls of advance_frame for every session; InvalidRequest when a call's row is missing */
int ggrs_p2p_advance_frames(ggrs_p2p_engine_t* eng, int32_t n_frames);
/* P2PSession::current_frame (p2p_session.rs:555-558); ggrs_p2p_calls: advance_frame calls made (the
 * same in rollback mode, where every call advances) */
int ggrs_p2p_current_frame(const ggrs_p2p_engine_t* eng, int32_t* out);
int ggrs_p2p_calls(const ggrs_p2p_engine_t* eng, int32_t* out);
int ggrs_p2p_synchronize(ggrs_p2p_engine_t* eng);
int ggrs_p2p_read_state(ggrs_p2p_engine_t* eng, int32_t session, uint8_t* out);
/* ggrs_p2p_read_state for every session, one transfer: out[num_sessions][36 + 20 * num_players] */
int ggrs_p2p_read_states(ggrs_p2p_engine_t* eng, uint8_t* out);
/* the session's saved-state ring (SavedStates, sync_layer.rs:144-166): per slot frame, checksum,
 * bincode state (36 + 20 P bytes) */
int ggrs_p2p_read_ring(ggrs_p2p_engine_t* eng, int32_t session, int32_t* frames, uint16_t* checksums,
                       uint8_t* states);
/* per session: number of rollbacks (adjust_gamestate calls) and resimulated frames so far */
int ggrs_p2p_read_stats(ggrs_p2p_engine_t* eng, int32_t* rollbacks, int64_t* resim_frames);
/* every session's InputQueue prediction state, [4][num_players][num_sessions] i32: prediction.frame,
 * prediction.input, first_incorrect_frame, last_requested_frame (input_queue.rs:10-37) */
int ggrs_p2p_read_queues(ggrs_p2p_engine_t* eng, int32_t* out);
/* [n][num_sessions] fletcher16 of each session's state after the final AdvanceFrame of calls
 * first_frame .. first_frame+n-1 (ex_game.rs:121-126) */
int ggrs_p2p_read_trace(ggrs_p2p_engine_t* eng, int32_t first_frame, int32_t n, uint16_t* out);
int ggrs_p2p_timing_reset(ggrs_p2p_engine_t* eng);
int ggrs_p2p_timing_stop(ggrs_p2p_engine_t* eng); /* as ggrs_timing_stop */
int ggrs_p2p_timing_read(ggrs_p2p_engine_t* eng, float* total_ms, int32_t* launches);

/* ---- P2P desync detection (SessionBuilder::with_desync_detection_mode, builder.rs:197-203;
 * DesyncDetection::On { interval }, src/lib.rs:71-80).  Replaces P2PSession's
 * check_checksum_send_interval (p2p_session.rs:939-975) for every session at once: at call
 * frame_to_send + remote_latency + 1 (when last_confirmed_frame and last_saved_frame reach it) the
 * saved cell's checksum of frame_to_send = interval, 2 interval, ... enters a device-resident
 * local_checksum_history of MAX_CHECKSUM_HISTORY_SIZE = 32 reports (protocol.rs:27).  The host
 * exchanges reports between peers (UdpProtocol::send_checksum_report, protocol.rs:692-698) and
 * compares received ones (compare_local_checksums_against_peers, p2p_session.rs:904-937) with
 * ggrs_p2p_compare_checksums; ggrs_amd/desync.py holds the pending-report bookkeeping. */
/* interval 0 = Off.  Part of the session's configuration: only before the first call. */
int ggrs_p2p_set_desync_detection(ggrs_p2p_engine_t* eng, int32_t interval);
/* [num_sessions] u16: the local checksum report of `frame` (host or device destination);
 * GGRS_E_PRECONDITION when `frame` is not a report frame sent so far or left the history */
int ggrs_p2p_local_checksums(ggrs_p2p_engine_t* eng, int32_t frame, uint16_t* out, int32_t out_on_device);
/* compare the local report of `frame` with a peer's [num_sessions] report: bit s of mask
 * (ceil(num_sessions/64) u64, host) set where they differ -- a GgrsEvent::DesyncDetected
 * (src/lib.rs:158-167) for session s; *n_differ = number of such sessions */
int ggrs_p2p_compare_checksums(ggrs_p2p_engine_t* eng, int32_t frame, const uint16_t* remote,
                               int32_t remote_on_device, uint64_t* mask, int32_t* n_differ);
/* Sparse saving (SessionBuilder::with_sparse_saving_mode, builder.rs:160-169): rollbacks load the
 * last saved state and save only min_confirmed (adjust_gamestate, p2p_session.rs:666-702), the
 * current frame is saved only when the last save would leave the prediction window
 * (check_last_saved_state :819-843), last_confirmed_frame never passes the last save
 * (sync_layer.rs:323-326).  Part of the configuration: only before the first call. */
int ggrs_p2p_set_sparse_saving(ggrs_p2p_engine_t* eng, int32_t on);
/* kernel form (comparison and tests): 0 = default (each session's calls flattened into its own
 * step sequence, input rows staged in LDS, with or without sparse saving), 1 = calls in
 * lockstep with input rows read from global memory, 2 = calls in lockstep with staged rows,
 * 3 = the flattened form with the session rings in HBM (the default keeps a block's rings in LDS
 * for the launch when they fit beside the other blocks on the CU, else it runs this form),
 * 4 = chains: every call as the chain of remote_latency + 1 advances from the confirmed state that
 * the fixed-latency network makes it (LoadGameState(f - D), D frames replayed, the call's own
 * advance), (D + 1) x players lanes per session, for engines whose sessions would fill at most one
 * wave per CU in the flattened form (the default picks it there); plain launches only -- no desync
 * detection, trace, debug flip or sparse saving (GGRS_E_STATE when forced otherwise); the first D
 * calls run on the flattened form.  Same states, rings, statistics and queues as every other form.
 * 5 = the flattened form with LDS rings, stepping every remote InputQueue's bookkeeping per frame;
 * 6 = canonical flattened form (the default for plain launches that do not take the chains form):
 * the rollback decision of call f is the remote input of frame f - D against the prediction made
 * from frame f - D - 1, the replay's remote inputs the confirmed and then the predicted ones -- the
 * queue state the fixed-latency network implies, written back at the end; with sparse saving on
 * (no trace or debug flip) the same form replays from the last save and saves min_confirmed. */
int ggrs_p2p_set_unstaged(ggrs_p2p_engine_t* eng, int32_t form);
/* test hook: the AdvanceFrame from `frame` of `session` flips the lowest bit of player 0's x on
 * every (re)simulation -- a deterministic desync of this peer (session -1: off) */
int ggrs_p2p_debug_desync(ggrs_p2p_engine_t* eng, int32_t session, int32_t frame);

/* ---- Arrival schedules: the network of a real match, per session.
 * Replaces the fixed remote_latency model by each session's own remote-arrival table, so every
 * session rolls back to its own earliest misprediction (InputQueue::add_input_by_frame's
 * first_incorrect_frame, src/input_queue.rs:190-230 -> check_simulation_consistency,
 * src/sync_layer.rs:343-353) with its own depth, a call at the prediction threshold saves but does
 * not advance (frames_ahead >= max_prediction, p2p_session.rs:393-423), and a disconnected remote
 * player (handle_event Event::Disconnected :866-878 -> disconnect_player_at_frame :618-655) rolls
 * the session back to its last frame + 1 and is replayed with InputStatus::Disconnected (ex_game
 * input 4, src/sync_layer.rs:280-293).  Call c: (1) the remote frames (delivered, arrive_upto[c]]
 * arrive, in order, for every remote player not disconnected; (2) Event::Disconnected for each
 * remote player k with bit k of events[c] (ascending k); (3) add_local_input of every local player
 * with input row c's byte, for the session's current frame (a call that did not advance repeats its
 * frame, and InputQueue::add_input drops the repeat, input_queue.rs:170-186); (4) advance_frame.
 * Input row g (ggrs_p2p_add_inputs) = the local players' input of call g and the remote players'
 * input of frame g, as in the fixed-latency model.  max_prediction 0 is lockstep mode (no saves,
 * no rollbacks, a call advances only when last_confirmed_frame == current_frame, :301-304,
 * 393-397); sparse saving allowed in rollback mode; the display trace per call (trace_capacity > 0: the
 * checksum after the call's last AdvanceFrame, ggrs_p2p_read_trace indexed by call); peers' disconnect reports
 * (ggrs_p2p_add_peer_reports) after (2); desync detection (ggrs_p2p_set_desync_detection, without sparse
 * saving) per session: ggrs_p2p_read_reports; remote_latency is ignored.  A session whose
 * call would make the reference panic (a remote input no longer in the input rows or more than
 * 126 - max_prediction frames ahead of the session, a rollback to a frame that is not in the past
 * or older than the input queues hold, no connected player) or whose arrival row names a frame after its call (GGRS_E_INVALID) stops
 * there with that error (ggrs_p2p_read_sessions); the other sessions run on.  Kernel:
 * p2p_sched.hip. */
/* on = 1 switches the engine to arrival schedules; part of the configuration: before the first call */
int ggrs_p2p_set_arrival_schedule(ggrs_p2p_engine_t* eng, int32_t on);
/* arrive_upto [n_calls][num_sessions] i32: the newest remote frame delivered by each call (<= the
 * call's index; at or below what already arrived delivers nothing); events [n_calls][num_sessions]
 * u8 (NULL: none).  Calls in order from 0, at most input_capacity calls ahead of the next call. */
int ggrs_p2p_add_arrivals(ggrs_p2p_engine_t* eng, int32_t first_call, int32_t n_calls, const int32_t* arrive_upto,
                          const uint8_t* events);
/* A peer's connect status as its input messages carry it (peer_connect_status): remote player
 * `reporter`'s endpoint reports remote player `player` disconnected with last frame `frame`
 * (-1 <= frame <= the call).  0 = no report. */
#define GGRS_PEER_REPORT(player, reporter, frame) (16 | (player) | (reporter) << 2 | ((frame) + 1) << 5)
/* reports [n_calls][num_sessions] i32 (GGRS_PEER_REPORT or 0) received by calls first_call ..
 * first_call + n_calls - 1, after their arrivals (ggrs_p2p_add_arrivals; calls not yet run).  A
 * report stands until its reporter disconnects; each call runs update_player_disconnects
 * (p2p_session.rs:748-783) over the standing ones: player k is disconnected at queue_min_confirmed
 * -- the oldest frame a running reporter gives, and k's own last frame while it is connected here
 * (endpoints that do not report k are taken to have seen every reported frame) -- when it is
 * connected here or its last frame is newer (the rollback then repeats every call, as the
 * reference's).  The repeat-last predictor only. */
int ggrs_p2p_add_peer_reports(ggrs_p2p_engine_t* eng, int32_t first_call, int32_t n_calls, const int32_t* reports);
/* per session: SyncLayer::current_frame, the calls that did not advance (prediction threshold),
 * and the session's error (0, GGRS_E_PRECONDITION or GGRS_E_INVALID); any pointer may be NULL */
int ggrs_p2p_read_sessions(ggrs_p2p_engine_t* eng, int32_t* frames, int32_t* skipped, int32_t* errors);
/* Desync detection under arrival schedules (p2p_session.rs:281-291, 904-975): for calls
 * first_call .. first_call + n_calls - 1 (run, and among the last input_capacity calls), per call and
 * session [n_calls][num_sessions]: the frame of the checksum report check_checksum_send_interval
 * sent (NULL_FRAME: none) and its checksum (the cell's, as read when sent), the
 * last_confirmed_frame compare_local_checksums_against_peers compared against in that call, and
 * the local players' last queued frame after the call (the reports travel with those inputs).
 * The pending-report bookkeeping and comparison are the caller's (ggrs_amd/desync.py
 * SchedDesyncDetector: UdpProtocol::on_checksum_report, protocol.rs:663-682).  A session whose
 * report cell is gone (the reference panics, :951-954) stops with GGRS_E_PRECONDITION.  Any output
 * pointer may be NULL. */
int ggrs_p2p_read_reports(ggrs_p2p_engine_t* eng, int32_t first_call, int32_t n_calls, int32_t* frames,
                          uint16_t* checksums, int32_t* last_confirmed, int32_t* local_last);

/* ---- Input wire codec, batched (src/network/compression.rs:14-182; bitfield-rle 0.2.1 runs,
 * bincode 1.3 fixint framing of EncodedInputSequence).  Replaces compression::encode / decode as
 * called per endpoint by UdpProtocol::send_pending_output (protocol.rs:450-480) and on_input
 * (:580-642), for many packets per launch: one packet = a reference input and the pending inputs
 * encoded against it, every input input_bytes long (what a GGRS peer sends for a fixed-size
 * Config::Input).  All pointers are DEVICE pointers; `stream` is a hipStream_t (NULL: default).
 * Per-packet results are written to device memory (asynchronous with the host). */
#define GGRS_CODEC_OK 0
#define GGRS_CODEC_E_BINCODE -1   /* bincode::deserialize failed (bad tag, short buffer) */
#define GGRS_CODEC_E_RLE -2       /* bitfield_rle::decode failed (truncated header or literal) */
#define GGRS_CODEC_E_DELTA -3     /* delta_decode rejected the sizes (compression.rs:117-154) */
#define GGRS_CODEC_E_CAP -4       /* encode: out_stride too small; decode: more than max_inputs */
#define GGRS_CODEC_E_INVALID -5   /* count outside 0..max_inputs, length outside 0..stride */
#define GGRS_CODEC_UNSUPPORTED -6 /* valid packet whose inputs are not all input_bytes long */
/* encode: ref [n][input_bytes], pending [n][max_inputs][input_bytes], count [n] ->
 * out [n][out_stride] packet bytes, out_len [n] = packet length or a GGRS_CODEC_E_* code */
int ggrs_codec_encode(const uint8_t* ref, const uint8_t* pending, const int32_t* count, int64_t n_packets,
                      int32_t input_bytes, int32_t max_inputs, uint8_t* out, int32_t out_stride, int32_t* out_len,
                      void* stream);
/* decode: ref [n][input_bytes], packets [n][packet_stride] with packet_len [n] bytes ->
 * out [n][max_inputs][input_bytes], count [n], status [n] (GGRS_CODEC_OK or an error code;
 * never faults on hostile bytes -- decode_arbitrary_input_never_panics, compression.rs:205-213).
 * Every row of out is written whole: the slots past count, and a failed packet's row, are zero
 * (out needs no clearing beforehand). */
int ggrs_codec_decode(const uint8_t* ref, const uint8_t* packets, const int32_t* packet_len, int64_t n_packets,
                      int32_t packet_stride, int32_t input_bytes, int32_t max_inputs, uint8_t* out, int32_t* count,
                      int32_t* status, void* stream);
/* The same with the chunked packet layout: the packets of each block of 256 (packets
 * 256 b .. 256 b + 255) lie back to back from byte 256 * b * stride of out / packets, each padded to
 * a multiple of 4 bytes; a packet whose length is outside [1, stride] (an error code) takes no
 * bytes.  Packet i's offset is 256 * (i / 256) * stride plus the padded lengths of the block's
 * packets before it, so the lengths alone locate every packet; the kernels move exactly the
 * packets' bytes instead of whole stride-byte rows.  Requires input_bytes in {1, 2, 4},
 * max_inputs * input_bytes <= 64 and a multiple of 4, stride a multiple of 4, dword-aligned
 * buffers (GGRS_E_INVALID otherwise). */
int ggrs_codec_encode_chunked(const uint8_t* ref, const uint8_t* pending, const int32_t* count, int64_t n_packets,
                              int32_t input_bytes, int32_t max_inputs, uint8_t* out, int32_t out_stride,
                              int32_t* out_len, void* stream);
int ggrs_codec_decode_chunked(const uint8_t* ref, const uint8_t* packets, const int32_t* packet_len, int64_t n_packets,
                              int32_t packet_stride, int32_t input_bytes, int32_t max_inputs, uint8_t* out,
                              int32_t* count, int32_t* status, void* stream);
/* an out_stride that every packet of max_inputs inputs fits (a multiple of 16) */
int32_t ggrs_codec_max_packet_bytes(int32_t input_bytes, int32_t max_inputs);
/* kernel forms (for tests and comparison; process-wide): 0 = default (lane-cooperative where
 * max_inputs * input_bytes <= 64 and rows are whole dwords, else thread-per-packet LDS-staged where
 * rows are whole dwords, else direct), 1 = direct thread-per-packet, 2 = thread-per-packet
 * LDS-staged where it applies */
int ggrs_codec_set_direct(int32_t mode);

#ifdef __cplusplus
}
#endif

#endif /* GGRS_AMD_H */
