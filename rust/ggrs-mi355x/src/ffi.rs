//! Hand-written declarations of every symbol in include/ggrs_amd.h (no bindgen: the ABI is plain
//! C).  tests/test_rust_ffi.py parses this file against the header -- names, parameter counts and
//! types, struct field order and types, constants -- so the two cannot drift apart.
#![allow(non_camel_case_types)]
use std::os::raw::{c_char, c_void};

pub const GGRS_ABI_VERSION: i32 = 6;

pub const GGRS_OK: i32 = 0;
pub const GGRS_E_INVALID: i32 = -1;
pub const GGRS_E_PRECONDITION: i32 = -2;
pub const GGRS_E_HIP: i32 = -3;
pub const GGRS_E_STATE: i32 = -4;

pub const GGRS_NULL_FRAME: i32 = -1;

pub const GGRS_REQ_SAVE: i32 = 0;
pub const GGRS_REQ_LOAD: i32 = 1;
pub const GGRS_REQ_ADVANCE: i32 = 2;

pub const GGRS_STATUS_CONFIRMED: u8 = 0;
pub const GGRS_STATUS_PREDICTED: u8 = 1;
pub const GGRS_STATUS_DISCONNECTED: u8 = 2;

pub const GGRS_PATH_PIPELINED: i32 = 0;
pub const GGRS_PATH_SEQUENTIAL: i32 = 1;
pub const GGRS_PATH_PIPELINED_CHAINS: i32 = 2;
pub const GGRS_PATH_PIPELINED_BATCHED: i32 = 3;

pub const GGRS_LANE_RUNNING: i32 = 0;
pub const GGRS_LANE_MISMATCH: i32 = 1;

pub const GGRS_TOK_SAVE: u32 = 0;
pub const GGRS_TOK_ADVANCE: u32 = 1;
pub const GGRS_TOK_LOAD: u32 = 2;
pub const GGRS_TOK_END: u32 = 3;
pub const GGRS_TOKENS_PER_WORD: i32 = 16;

pub const GGRS_BATCH_STATUS: i32 = 1;

pub const GGRS_BATCH_MAX_WORDS: i32 = 32;
pub const GGRS_BATCH_MAX_LOADS: i32 = 8;
pub const GGRS_BATCH_MAX_ADV: i32 = 128;
pub const GGRS_BATCH_MAX_SAVES: i32 = 256;

pub const GGRS_CODEC_OK: i32 = 0;
pub const GGRS_CODEC_E_BINCODE: i32 = -1;
pub const GGRS_CODEC_E_RLE: i32 = -2;
pub const GGRS_CODEC_E_DELTA: i32 = -3;
pub const GGRS_CODEC_E_CAP: i32 = -4;
pub const GGRS_CODEC_E_INVALID: i32 = -5;
pub const GGRS_CODEC_UNSUPPORTED: i32 = -6;

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct ggrs_config_t {
    pub num_lanes: i32,
    pub num_players: i32,
    pub max_prediction: i32,
    pub check_distance: i32,
    pub input_delay: i32,
    pub input_capacity: i32,
    pub device: i32,
    pub trace_capacity: i32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct ggrs_request_t {
    pub kind: i32,
    pub frame: i32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct ggrs_lane_batch_t {
    pub token_words: i32,
    pub load_slots: i32,
    pub adv_rows: i32,
    pub save_rows: i32,
    pub tokens: *mut u32,
    pub load_frames: *mut i32,
    pub inputs: *mut u8,
    pub status: *mut u8,
    pub checksums: *mut u16,
    pub lane_result: *mut i32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct ggrs_branch_config_t {
    pub num_sessions: i32,
    pub num_players: i32,
    pub remote_mask: i32,
    pub window: i32,
    pub branches: i32,
    pub alphabet: i32,
    pub input_capacity: i32,
    pub device: i32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct ggrs_particle_config_t {
    pub num_sessions: i32,
    pub num_entities: i32,
    pub num_players: i32,
    pub max_prediction: i32,
    pub check_distance: i32,
    pub input_capacity: i32,
    pub device: i32,
    pub first_session_id: i32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct ggrs_p2p_config_t {
    pub num_sessions: i32,
    pub num_players: i32,
    pub local_mask: i32,
    pub input_delay: i32,
    pub max_prediction: i32,
    pub remote_latency: i32,
    pub predictor: i32,
    pub input_capacity: i32,
    pub trace_capacity: i32,
    pub device: i32,
}

#[repr(C)]
pub struct ggrs_engine_t {
    _private: [u8; 0],
}

#[repr(C)]
pub struct ggrs_branch_engine_t {
    _private: [u8; 0],
}

#[repr(C)]
pub struct ggrs_particle_engine_t {
    _private: [u8; 0],
}

#[repr(C)]
pub struct ggrs_p2p_engine_t {
    _private: [u8; 0],
}

extern "C" {
    pub fn ggrs_abi_version() -> i32;
    pub fn ggrs_last_error() -> *const c_char;

    // ---- the engine: SyncTest, lockstep and per-lane request lists
    pub fn ggrs_engine_create(cfg: *const ggrs_config_t, out: *mut *mut ggrs_engine_t) -> i32;
    pub fn ggrs_engine_destroy(eng: *mut ggrs_engine_t) -> i32;
    pub fn ggrs_engine_config(eng: *const ggrs_engine_t, out: *mut ggrs_config_t) -> i32;
    pub fn ggrs_add_local_inputs(eng: *mut ggrs_engine_t, first_frame: i32, n_frames: i32, inputs: *const u8) -> i32;
    pub fn ggrs_add_local_inputs_device(eng: *mut ggrs_engine_t, first_frame: i32, n_frames: i32,
                                        inputs_device: *const c_void) -> i32;
    pub fn ggrs_synctest_advance_frames(eng: *mut ggrs_engine_t, n_frames: i32) -> i32;
    pub fn ggrs_set_synctest_path(eng: *mut ggrs_engine_t, path: i32) -> i32;
    pub fn ggrs_handle_requests(eng: *mut ggrs_engine_t, reqs: *const ggrs_request_t, n_reqs: i32,
                                inputs: *const u8, status: *const u8) -> i32;
    pub fn ggrs_lane_batch_map(eng: *mut ggrs_engine_t, token_words: i32, load_slots: i32, adv_rows: i32,
                               save_rows: i32, out: *mut ggrs_lane_batch_t) -> i32;
    pub fn ggrs_lane_batch_run(eng: *mut ggrs_engine_t, batch: *const ggrs_lane_batch_t, flags: i32,
                               n_failed: *mut i32) -> i32;
    pub fn ggrs_handle_requests_lanes(eng: *mut ggrs_engine_t, reqs: *const ggrs_request_t, offsets: *const i32,
                                      inputs: *const u8, status: *const u8, save_checksums: *mut u16,
                                      lane_result: *mut i32) -> i32;
    pub fn ggrs_lane_batch_lds(eng: *mut ggrs_engine_t, token_words: i32, load_slots: i32, adv_rows: i32,
                               save_rows: i32, need_bytes: *mut i64, limit_bytes: *mut i64) -> i32;
    pub fn ggrs_lane_batch_submit(eng: *mut ggrs_engine_t, batch: *const ggrs_lane_batch_t, flags: i32) -> i32;
    pub fn ggrs_lane_batch_wait(eng: *mut ggrs_engine_t, n_failed: *mut i32) -> i32;
    pub fn ggrs_lane_encode(batch: *const ggrs_lane_batch_t, num_lanes: i64, num_players: i32, lane: i64,
                            reqs: *const ggrs_request_t, n_reqs: i32, inputs: *const u8, status: *const u8,
                            lane_frame: i32, bad_request: *mut i32) -> i32;
    pub fn ggrs_lane_shape(reqs: *const ggrs_request_t, n_reqs: i32, shape: *mut i32) -> i32;
    pub fn ggrs_lane_server(eng: *mut ggrs_engine_t, on: i32) -> i32;
    pub fn ggrs_read_lane_frames(eng: *mut ggrs_engine_t, frames: *mut i32) -> i32;
    pub fn ggrs_synchronize(eng: *mut ggrs_engine_t) -> i32;
    pub fn ggrs_current_frame(eng: *const ggrs_engine_t, out: *mut i32) -> i32;
    pub fn ggrs_read_mismatches(eng: *mut ggrs_engine_t, lane_status: *mut i32, mismatch_frame: *mut i32,
                                mismatch_mask: *mut u64) -> i32;
    pub fn ggrs_read_save_checksums(eng: *mut ggrs_engine_t, frame: i32, out: *mut u16) -> i32;
    pub fn ggrs_read_save_checksums_frames(eng: *mut ggrs_engine_t, frames: *const i32, n: i32, out: *mut u16) -> i32;
    pub fn ggrs_read_state(eng: *mut ggrs_engine_t, lane: i32, out: *mut u8) -> i32;
    pub fn ggrs_read_states(eng: *mut ggrs_engine_t, out: *mut u8) -> i32;
    pub fn ggrs_read_ring(eng: *mut ggrs_engine_t, lane: i32, frames: *mut i32, checksums: *mut u16,
                          states: *mut u8) -> i32;
    pub fn ggrs_read_trace(eng: *mut ggrs_engine_t, first_frame: i32, n_frames: i32, out: *mut u16) -> i32;
    pub fn ggrs_debug_corrupt_on_load(eng: *mut ggrs_engine_t, lane: i32, frame: i32) -> i32;
    pub fn ggrs_last_launch_ms(eng: *mut ggrs_engine_t, ms: *mut f32) -> i32;
    pub fn ggrs_timing_reset(eng: *mut ggrs_engine_t) -> i32;
    pub fn ggrs_timing_stop(eng: *mut ggrs_engine_t) -> i32;
    pub fn ggrs_timing_read(eng: *mut ggrs_engine_t, total_ms: *mut f32, launches: *mut i32) -> i32;

    // ---- speculative branch rollback (configs 3/4)
    pub fn ggrs_branch_engine_create(cfg: *const ggrs_branch_config_t, out: *mut *mut ggrs_branch_engine_t) -> i32;
    pub fn ggrs_branch_engine_destroy(eng: *mut ggrs_branch_engine_t) -> i32;
    pub fn ggrs_branch_engine_config(eng: *const ggrs_branch_engine_t, out: *mut ggrs_branch_config_t) -> i32;
    pub fn ggrs_branch_add_inputs(eng: *mut ggrs_branch_engine_t, first_frame: i32, n_frames: i32,
                                  inputs: *const u8) -> i32;
    pub fn ggrs_branch_speculate(eng: *mut ggrs_branch_engine_t) -> i32;
    pub fn ggrs_branch_confirm(eng: *mut ggrs_branch_engine_t, report_device: *mut c_void) -> i32;
    pub fn ggrs_branch_report_bytes(eng: *const ggrs_branch_engine_t, out: *mut i64) -> i32;
    pub fn ggrs_branch_synchronize(eng: *mut ggrs_branch_engine_t) -> i32;
    pub fn ggrs_branch_trunk_frame(eng: *const ggrs_branch_engine_t, out: *mut i32) -> i32;
    pub fn ggrs_branch_read_report(eng: *mut ggrs_branch_engine_t, checksums: *mut u16, survive_bits: *mut u64) -> i32;
    pub fn ggrs_branch_read_desync(eng: *mut ggrs_branch_engine_t, first_frame: *mut i32) -> i32;
    pub fn ggrs_branch_read_trunk(eng: *mut ggrs_branch_engine_t, session: i32, out: *mut u8) -> i32;
    pub fn ggrs_branch_read_lane(eng: *mut ggrs_branch_engine_t, lane: i64, frame: i32, checksum: *mut u16,
                                 out: *mut u8) -> i32;
    pub fn ggrs_branch_read_cells(eng: *mut ggrs_branch_engine_t, frame: i32, checksums: *mut u16, states: *mut u8)
                                  -> i32;
    pub fn ggrs_branch_timing_reset(eng: *mut ggrs_branch_engine_t) -> i32;
    pub fn ggrs_branch_timing_stop(eng: *mut ggrs_branch_engine_t) -> i32;
    pub fn ggrs_branch_timing_read(eng: *mut ggrs_branch_engine_t, total_ms: *mut f32, launches: *mut i32) -> i32;
    pub fn ggrs_branch_rounds(eng: *mut ggrs_branch_engine_t, n_rounds: i32) -> i32;
    pub fn ggrs_branch_set_round_launches(eng: *mut ggrs_branch_engine_t, on: i32) -> i32;
    pub fn ggrs_branch_set_stream(eng: *mut ggrs_branch_engine_t, stream: *mut c_void) -> i32;
    pub fn ggrs_branch_use_own_stream(eng: *mut ggrs_branch_engine_t) -> i32;
    pub fn ggrs_branch_round(eng: *mut ggrs_branch_engine_t, report_device: *mut c_void) -> i32;
    pub fn ggrs_branch_rounds_reports(eng: *mut ggrs_branch_engine_t, n_rounds: i32, reports_device: *mut c_void) -> i32;
    pub fn ggrs_branch_compare_peer_rows(eng: *mut ggrs_branch_engine_t, gathered: *const c_void, world: i32,
                                         rows_per_rank: i32, n_rows: i32, rank: i32, peer: i32, first_frame: i32,
                                         count_device: *mut i64, first_frame_device: *mut i64) -> i32;
    pub fn ggrs_branch_compare_peer(eng: *mut ggrs_branch_engine_t, gathered: *const c_void, world: i32, rank: i32,
                                    peer: i32, frame: i32, count_device: *mut i64,
                                    first_frame_device: *mut i64) -> i32;

    // ---- config-5 large-state stress game
    pub fn ggrs_particle_engine_create(cfg: *const ggrs_particle_config_t,
                                       out: *mut *mut ggrs_particle_engine_t) -> i32;
    pub fn ggrs_particle_engine_destroy(eng: *mut ggrs_particle_engine_t) -> i32;
    pub fn ggrs_particle_add_local_inputs(eng: *mut ggrs_particle_engine_t, first_frame: i32, n_frames: i32,
                                          inputs: *const u8) -> i32;
    pub fn ggrs_particle_synctest_advance_frames(eng: *mut ggrs_particle_engine_t, n_frames: i32) -> i32;
    pub fn ggrs_particle_synchronize(eng: *mut ggrs_particle_engine_t) -> i32;
    pub fn ggrs_particle_current_frame(eng: *const ggrs_particle_engine_t, out: *mut i32) -> i32;
    pub fn ggrs_particle_read_mismatches(eng: *mut ggrs_particle_engine_t, status: *mut i32, mismatch_frame: *mut i32,
                                         mismatch_mask: *mut u64) -> i32;
    pub fn ggrs_particle_read_state(eng: *mut ggrs_particle_engine_t, session: i32, out: *mut u8) -> i32;
    pub fn ggrs_particle_read_saved(eng: *mut ggrs_particle_engine_t, session: i32, frame: i32, checksum: *mut u16,
                                    out: *mut u8) -> i32;
    pub fn ggrs_particle_debug_corrupt_on_load(eng: *mut ggrs_particle_engine_t, session: i32, frame: i32) -> i32;
    pub fn ggrs_particle_timing_reset(eng: *mut ggrs_particle_engine_t) -> i32;
    pub fn ggrs_particle_timing_stop(eng: *mut ggrs_particle_engine_t) -> i32;
    pub fn ggrs_particle_timing_read(eng: *mut ggrs_particle_engine_t, total_ms: *mut f32, launches: *mut i32) -> i32;

    // ---- P2P sessions on the device
    pub fn ggrs_p2p_engine_create(cfg: *const ggrs_p2p_config_t, out: *mut *mut ggrs_p2p_engine_t) -> i32;
    pub fn ggrs_p2p_engine_destroy(eng: *mut ggrs_p2p_engine_t) -> i32;
    pub fn ggrs_p2p_engine_config(eng: *const ggrs_p2p_engine_t, out: *mut ggrs_p2p_config_t) -> i32;
    pub fn ggrs_p2p_add_inputs(eng: *mut ggrs_p2p_engine_t, first_frame: i32, n_frames: i32, inputs: *const u8) -> i32;
    pub fn ggrs_p2p_advance_frames(eng: *mut ggrs_p2p_engine_t, n_frames: i32) -> i32;
    pub fn ggrs_p2p_current_frame(eng: *const ggrs_p2p_engine_t, out: *mut i32) -> i32;
    pub fn ggrs_p2p_calls(eng: *const ggrs_p2p_engine_t, out: *mut i32) -> i32;
    pub fn ggrs_p2p_synchronize(eng: *mut ggrs_p2p_engine_t) -> i32;
    pub fn ggrs_p2p_read_state(eng: *mut ggrs_p2p_engine_t, session: i32, out: *mut u8) -> i32;
    pub fn ggrs_p2p_read_states(eng: *mut ggrs_p2p_engine_t, out: *mut u8) -> i32;
    pub fn ggrs_p2p_add_peer_reports(eng: *mut ggrs_p2p_engine_t, first_call: i32, n_calls: i32, reports: *const i32)
                                     -> i32;
    pub fn ggrs_p2p_read_ring(eng: *mut ggrs_p2p_engine_t, session: i32, frames: *mut i32, checksums: *mut u16,
                              states: *mut u8) -> i32;
    pub fn ggrs_p2p_read_stats(eng: *mut ggrs_p2p_engine_t, rollbacks: *mut i32, resim_frames: *mut i64) -> i32;
    pub fn ggrs_p2p_read_queues(eng: *mut ggrs_p2p_engine_t, out: *mut i32) -> i32;
    pub fn ggrs_p2p_read_trace(eng: *mut ggrs_p2p_engine_t, first_frame: i32, n: i32, out: *mut u16) -> i32;
    pub fn ggrs_p2p_timing_reset(eng: *mut ggrs_p2p_engine_t) -> i32;
    pub fn ggrs_p2p_timing_stop(eng: *mut ggrs_p2p_engine_t) -> i32;
    pub fn ggrs_p2p_timing_read(eng: *mut ggrs_p2p_engine_t, total_ms: *mut f32, launches: *mut i32) -> i32;
    pub fn ggrs_p2p_set_desync_detection(eng: *mut ggrs_p2p_engine_t, interval: i32) -> i32;
    pub fn ggrs_p2p_local_checksums(eng: *mut ggrs_p2p_engine_t, frame: i32, out: *mut u16, out_on_device: i32) -> i32;
    pub fn ggrs_p2p_compare_checksums(eng: *mut ggrs_p2p_engine_t, frame: i32, remote: *const u16,
                                      remote_on_device: i32, mask: *mut u64, n_differ: *mut i32) -> i32;
    pub fn ggrs_p2p_set_sparse_saving(eng: *mut ggrs_p2p_engine_t, on: i32) -> i32;
    pub fn ggrs_p2p_set_unstaged(eng: *mut ggrs_p2p_engine_t, form: i32) -> i32;
    pub fn ggrs_p2p_debug_desync(eng: *mut ggrs_p2p_engine_t, session: i32, frame: i32) -> i32;
    pub fn ggrs_p2p_set_arrival_schedule(eng: *mut ggrs_p2p_engine_t, on: i32) -> i32;
    pub fn ggrs_p2p_add_arrivals(
        eng: *mut ggrs_p2p_engine_t,
        first_call: i32,
        n_calls: i32,
        arrive_upto: *const i32,
        events: *const u8,
    ) -> i32;
    pub fn ggrs_p2p_read_sessions(
        eng: *mut ggrs_p2p_engine_t,
        frames: *mut i32,
        skipped: *mut i32,
        errors: *mut i32,
    ) -> i32;
    pub fn ggrs_p2p_read_reports(
        eng: *mut ggrs_p2p_engine_t,
        first_call: i32,
        n_calls: i32,
        frames: *mut i32,
        checksums: *mut u16,
        last_confirmed: *mut i32,
        local_last: *mut i32,
    ) -> i32;

    // ---- input wire codec, batched (src/network/compression.rs:14-182); device pointers
    pub fn ggrs_codec_encode(ref_: *const u8, pending: *const u8, count: *const i32, n_packets: i64,
                             input_bytes: i32, max_inputs: i32, out: *mut u8, out_stride: i32,
                             out_len: *mut i32, stream: *mut c_void) -> i32;
    pub fn ggrs_codec_decode(ref_: *const u8, packets: *const u8, packet_len: *const i32, n_packets: i64,
                             packet_stride: i32, input_bytes: i32, max_inputs: i32, out: *mut u8,
                             count: *mut i32, status: *mut i32, stream: *mut c_void) -> i32;
    pub fn ggrs_codec_encode_chunked(ref_: *const u8, pending: *const u8, count: *const i32, n_packets: i64,
                                     input_bytes: i32, max_inputs: i32, out: *mut u8, out_stride: i32,
                                     out_len: *mut i32, stream: *mut c_void) -> i32;
    pub fn ggrs_codec_decode_chunked(ref_: *const u8, packets: *const u8, packet_len: *const i32, n_packets: i64,
                                     packet_stride: i32, input_bytes: i32, max_inputs: i32, out: *mut u8,
                                     count: *mut i32, status: *mut i32, stream: *mut c_void) -> i32;
    pub fn ggrs_codec_max_packet_bytes(input_bytes: i32, max_inputs: i32) -> i32;
    pub fn ggrs_codec_set_direct(mode: i32) -> i32;
}

/// The engine's last error message on this thread.
pub fn last_error() -> String {
    unsafe { std::ffi::CStr::from_ptr(ggrs_last_error()) }.to_string_lossy().into_owned()
}
