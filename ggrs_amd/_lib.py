"""ctypes binding of the engine's C ABI (include/ggrs_amd.h) -- libggrs_amd.so, built in-tree.

There is no fallback: if the HIP library is missing or fails to load, every entry point raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libggrs_amd.so")
# timing-experiment builds (tools/exp_build.sh) live in ggrs_amd/exp/; only those may replace the library
_EXP = os.environ.get("GGRS_AMD_EXP_LIB")
if _EXP:
    LIB_PATH = os.path.join(HERE, "exp", os.path.basename(_EXP))

ABI_VERSION = 6  # include/ggrs_amd.h GGRS_ABI_VERSION
GGRS_OK = 0
GGRS_E_INVALID = -1
GGRS_E_PRECONDITION = -2
GGRS_E_HIP = -3
GGRS_E_STATE = -4
NULL_FRAME = -1
REQ_SAVE, REQ_LOAD, REQ_ADVANCE = 0, 1, 2
STATUS_CONFIRMED, STATUS_PREDICTED, STATUS_DISCONNECTED = 0, 1, 2
LANE_RUNNING, LANE_MISMATCH = 0, 1
PATH_PIPELINED, PATH_SEQUENTIAL, PATH_PIPELINED_CHAINS, PATH_PIPELINED_BATCHED = 0, 1, 2, 3
TOK_SAVE, TOK_ADVANCE, TOK_LOAD, TOK_END = 0, 1, 2, 3
TOKENS_PER_WORD = 16
BATCH_STATUS = 1

# every symbol include/ggrs_amd.h declares (tests check the library exports all of them)
EXPORTS = (
    "ggrs_abi_version", "ggrs_last_error", "ggrs_engine_create", "ggrs_engine_destroy",
    "ggrs_engine_config", "ggrs_add_local_inputs", "ggrs_add_local_inputs_device",
    "ggrs_synctest_advance_frames", "ggrs_handle_requests", "ggrs_synchronize",
    "ggrs_current_frame", "ggrs_read_mismatches", "ggrs_read_save_checksums", "ggrs_read_save_checksums_frames", "ggrs_read_state", "ggrs_read_states",
    "ggrs_read_ring", "ggrs_read_trace", "ggrs_debug_corrupt_on_load", "ggrs_last_launch_ms",
    "ggrs_timing_reset", "ggrs_timing_stop", "ggrs_timing_read", "ggrs_set_synctest_path",
    "ggrs_lane_batch_map", "ggrs_lane_batch_run", "ggrs_handle_requests_lanes", "ggrs_read_lane_frames",
    "ggrs_lane_server", "ggrs_lane_batch_submit", "ggrs_lane_batch_wait", "ggrs_lane_encode", "ggrs_lane_shape",
    "ggrs_lane_batch_lds",
    "ggrs_branch_engine_create", "ggrs_branch_engine_destroy", "ggrs_branch_engine_config",
    "ggrs_branch_add_inputs", "ggrs_branch_speculate", "ggrs_branch_confirm",
    "ggrs_branch_report_bytes", "ggrs_branch_synchronize", "ggrs_branch_trunk_frame",
    "ggrs_branch_read_report", "ggrs_branch_read_desync", "ggrs_branch_read_trunk",
    "ggrs_branch_read_lane", "ggrs_branch_read_cells", "ggrs_branch_timing_reset", "ggrs_branch_timing_stop", "ggrs_branch_timing_read",
    "ggrs_branch_rounds", "ggrs_branch_set_round_launches", "ggrs_branch_set_stream", "ggrs_branch_use_own_stream",
    "ggrs_branch_round", "ggrs_branch_rounds_reports", "ggrs_branch_compare_peer", "ggrs_branch_compare_peer_rows",
    "ggrs_particle_engine_create", "ggrs_particle_engine_destroy", "ggrs_particle_add_local_inputs",
    "ggrs_particle_synctest_advance_frames", "ggrs_particle_synchronize",
    "ggrs_particle_current_frame", "ggrs_particle_read_mismatches", "ggrs_particle_read_state",
    "ggrs_particle_read_saved", "ggrs_particle_debug_corrupt_on_load",
    "ggrs_particle_timing_reset", "ggrs_particle_timing_stop", "ggrs_particle_timing_read",
    "ggrs_p2p_engine_create", "ggrs_p2p_engine_destroy", "ggrs_p2p_engine_config",
    "ggrs_p2p_add_inputs", "ggrs_p2p_advance_frames", "ggrs_p2p_current_frame", "ggrs_p2p_calls",
    "ggrs_p2p_synchronize", "ggrs_p2p_read_state", "ggrs_p2p_read_ring", "ggrs_p2p_read_stats", "ggrs_p2p_read_queues",
    "ggrs_p2p_read_trace", "ggrs_p2p_timing_reset", "ggrs_p2p_timing_stop", "ggrs_p2p_timing_read",
    "ggrs_p2p_set_desync_detection", "ggrs_p2p_local_checksums", "ggrs_p2p_compare_checksums",
    "ggrs_p2p_debug_desync", "ggrs_p2p_set_sparse_saving", "ggrs_p2p_set_unstaged",
    "ggrs_p2p_set_arrival_schedule", "ggrs_p2p_add_arrivals", "ggrs_p2p_read_sessions", "ggrs_p2p_read_reports", "ggrs_p2p_read_states", "ggrs_p2p_add_peer_reports",
    "ggrs_codec_encode", "ggrs_codec_decode", "ggrs_codec_encode_chunked", "ggrs_codec_decode_chunked", "ggrs_codec_max_packet_bytes", "ggrs_codec_set_direct",
)


class Config(ctypes.Structure):
    _fields_ = [
        ("num_lanes", ctypes.c_int32),
        ("num_players", ctypes.c_int32),
        ("max_prediction", ctypes.c_int32),
        ("check_distance", ctypes.c_int32),
        ("input_delay", ctypes.c_int32),
        ("input_capacity", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("trace_capacity", ctypes.c_int32),
    ]


class Request(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("frame", ctypes.c_int32)]


class LaneBatch(ctypes.Structure):
    """ggrs_lane_batch_t"""
    _fields_ = [
        ("token_words", ctypes.c_int32),
        ("load_slots", ctypes.c_int32),
        ("adv_rows", ctypes.c_int32),
        ("save_rows", ctypes.c_int32),
        ("tokens", ctypes.POINTER(ctypes.c_uint32)),
        ("load_frames", ctypes.POINTER(ctypes.c_int32)),
        ("inputs", ctypes.POINTER(ctypes.c_uint8)),
        ("status", ctypes.POINTER(ctypes.c_uint8)),
        ("checksums", ctypes.POINTER(ctypes.c_uint16)),
        ("lane_result", ctypes.POINTER(ctypes.c_int32)),
    ]


class GgrsError(Exception):
    """Mirror of GgrsError (src/error.rs:31-57) for errors the engine reports."""

    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class InvalidRequest(GgrsError):
    """GgrsError::InvalidRequest (error.rs:39-43)."""


class PreconditionError(GgrsError):
    """A condition on which the reference panics (assert!), reported instead of unwinding."""


_lib = None


def lib():
    """Load libggrs_amd.so (raises OSError if it has not been built: no CPU fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} not built: run `python -m ggrs_amd.build` "
                          "(the engine has no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER
        vp = ctypes.c_void_p
        L.ggrs_abi_version.restype = ctypes.c_int32
        L.ggrs_last_error.restype = ctypes.c_char_p
        if L.ggrs_abi_version() != ABI_VERSION:  # a stale build: fail loudly, never misread a signature
            raise OSError(f"{LIB_PATH} implements ABI {L.ggrs_abi_version()}, this package binds ABI "
                          f"{ABI_VERSION}: rebuild with `python -m ggrs_amd.build`")
        L.ggrs_engine_create.argtypes = [P(Config), P(vp)]
        L.ggrs_engine_destroy.argtypes = [vp]
        L.ggrs_engine_config.argtypes = [vp, P(Config)]
        L.ggrs_add_local_inputs.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp]
        L.ggrs_add_local_inputs_device.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp]
        L.ggrs_synctest_advance_frames.argtypes = [vp, ctypes.c_int32]
        L.ggrs_handle_requests.argtypes = [vp, P(Request), ctypes.c_int32, vp, vp]
        L.ggrs_synchronize.argtypes = [vp]
        L.ggrs_current_frame.argtypes = [vp, P(ctypes.c_int32)]
        L.ggrs_read_mismatches.argtypes = [vp, vp, vp, vp]
        L.ggrs_read_save_checksums.argtypes = [vp, ctypes.c_int32, vp]
        L.ggrs_read_save_checksums_frames.argtypes = [vp, vp, ctypes.c_int32, vp]
        L.ggrs_read_state.argtypes = [vp, ctypes.c_int32, vp]
        L.ggrs_read_states.argtypes = [vp, vp]
        L.ggrs_read_ring.argtypes = [vp, ctypes.c_int32, vp, vp, vp]
        L.ggrs_read_trace.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp]
        L.ggrs_debug_corrupt_on_load.argtypes = [vp, ctypes.c_int32, ctypes.c_int32]
        L.ggrs_last_launch_ms.argtypes = [vp, P(ctypes.c_float)]
        L.ggrs_timing_reset.argtypes = [vp]
        L.ggrs_timing_stop.argtypes = [vp]
        L.ggrs_set_synctest_path.argtypes = [vp, ctypes.c_int32]
        L.ggrs_timing_read.argtypes = [vp, P(ctypes.c_float), P(ctypes.c_int32)]
        i32 = ctypes.c_int32
        L.ggrs_lane_batch_map.argtypes = [vp, i32, i32, i32, i32, P(LaneBatch)]
        L.ggrs_lane_batch_run.argtypes = [vp, P(LaneBatch), i32, P(i32)]
        L.ggrs_lane_batch_submit.argtypes = [vp, P(LaneBatch), i32]
        L.ggrs_lane_batch_wait.argtypes = [vp, P(i32)]
        L.ggrs_lane_encode.argtypes = [P(LaneBatch), ctypes.c_int64, i32, ctypes.c_int64, vp, i32, vp, vp, i32, P(i32)]
        L.ggrs_lane_shape.argtypes = [vp, i32, vp]
        L.ggrs_lane_batch_lds.argtypes = [vp, i32, i32, i32, i32, P(ctypes.c_int64), P(ctypes.c_int64)]
        L.ggrs_handle_requests_lanes.argtypes = [vp, vp, vp, vp, vp, vp, vp]
        L.ggrs_read_lane_frames.argtypes = [vp, vp]
        L.ggrs_lane_server.argtypes = [vp, i32]
        for name in EXPORTS:
            if name not in ("ggrs_abi_version", "ggrs_last_error", "ggrs_codec_max_packet_bytes"):
                getattr(L, name).restype = ctypes.c_int
        _lib = L
    return _lib


def check(rc):
    if rc == GGRS_OK:
        return
    msg = lib().ggrs_last_error().decode(errors="replace")
    if rc == GGRS_E_INVALID:
        raise InvalidRequest(rc, msg)
    if rc == GGRS_E_PRECONDITION:
        raise PreconditionError(rc, msg)
    raise GgrsError(rc, msg)
