//! Hand-written declarations of include/ggrs_amd.h (no bindgen: the ABI is plain C).
#![allow(non_camel_case_types)]
use std::os::raw::{c_char, c_void};

pub const GGRS_OK: i32 = 0;
pub const GGRS_REQ_SAVE: i32 = 0;
pub const GGRS_REQ_LOAD: i32 = 1;
pub const GGRS_REQ_ADVANCE: i32 = 2;
pub const GGRS_STATUS_CONFIRMED: u8 = 0;
pub const GGRS_STATUS_PREDICTED: u8 = 1;
pub const GGRS_STATUS_DISCONNECTED: u8 = 2;
pub const GGRS_LANE_MISMATCH: i32 = 1;

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
pub struct ggrs_engine_t {
    _private: [u8; 0],
}

extern "C" {
    pub fn ggrs_abi_version() -> i32;
    pub fn ggrs_last_error() -> *const c_char;
    pub fn ggrs_engine_create(cfg: *const ggrs_config_t, out: *mut *mut ggrs_engine_t) -> i32;
    pub fn ggrs_engine_destroy(eng: *mut ggrs_engine_t) -> i32;
    pub fn ggrs_add_local_inputs(eng: *mut ggrs_engine_t, first_frame: i32, n_frames: i32, inputs: *const u8) -> i32;
    pub fn ggrs_add_local_inputs_device(eng: *mut ggrs_engine_t, first_frame: i32, n_frames: i32,
                                        inputs_device: *const c_void) -> i32;
    pub fn ggrs_synctest_advance_frames(eng: *mut ggrs_engine_t, n_frames: i32) -> i32;
    pub fn ggrs_handle_requests(eng: *mut ggrs_engine_t, reqs: *const ggrs_request_t, n_reqs: i32,
                                inputs: *const u8, status: *const u8) -> i32;
    pub fn ggrs_synchronize(eng: *mut ggrs_engine_t) -> i32;
    pub fn ggrs_current_frame(eng: *const ggrs_engine_t, out: *mut i32) -> i32;
    pub fn ggrs_read_mismatches(eng: *mut ggrs_engine_t, lane_status: *mut i32, mismatch_frame: *mut i32,
                                mismatch_mask: *mut u64) -> i32;
    pub fn ggrs_read_save_checksums(eng: *mut ggrs_engine_t, frame: i32, out: *mut u16) -> i32;
    pub fn ggrs_read_state(eng: *mut ggrs_engine_t, lane: i32, out: *mut u8) -> i32;

    // input wire codec, batched (src/network/compression.rs:14-182); device pointers
    pub fn ggrs_codec_encode(ref_: *const u8, pending: *const u8, count: *const i32, n_packets: i64,
                             input_bytes: i32, max_inputs: i32, out: *mut u8, out_stride: i32,
                             out_len: *mut i32, stream: *mut c_void) -> i32;
    pub fn ggrs_codec_decode(ref_: *const u8, packets: *const u8, packet_len: *const i32, n_packets: i64,
                             packet_stride: i32, input_bytes: i32, max_inputs: i32, out: *mut u8,
                             count: *mut i32, status: *mut i32, stream: *mut c_void) -> i32;
    pub fn ggrs_codec_max_packet_bytes(input_bytes: i32, max_inputs: i32) -> i32;
}

/// The engine's last error message on this thread.
pub fn last_error() -> String {
    unsafe { std::ffi::CStr::from_ptr(ggrs_last_error()) }.to_string_lossy().into_owned()
}
