//! A GGRS request handler for L box-game sessions that run in lockstep (same request kinds and
//! frames, different inputs): it replaces `Game::handle_requests` of examples/ex_game/ex_game.rs
//! (:79-127).  Saves keep the state in HBM and hand GGRS `cell.save(frame, None, Some(checksum))`
//! (data = None is legal; GGRS only reads frame() and checksum(), src/sync_layer.rs:72-78).
pub mod ffi;

use ffi::*;
use ggrs::{Config, GgrsRequest, InputStatus};

#[derive(Debug)]
pub struct EngineError(pub i32, pub String);

fn check(rc: i32) -> Result<(), EngineError> {
    if rc == GGRS_OK { Ok(()) } else { Err(EngineError(rc, last_error())) }
}

/// Turns a game input into the byte the box game reads (`Input.inp`, ex_game.rs:28-32).
pub trait InputByte {
    fn input_byte(&self) -> u8;
}

pub struct BatchedBoxGame {
    eng: *mut ggrs_engine_t,
    lanes: usize,
    players: usize,
}

impl BatchedBoxGame {
    /// One engine lane per session: SessionBuilder's max_prediction / check_distance / input delay.
    pub fn new(lanes: usize, players: usize, max_prediction: usize, check_distance: usize,
               input_delay: usize, device: i32) -> Result<Self, EngineError> {
        let cfg = ggrs_config_t {
            num_lanes: lanes as i32,
            num_players: players as i32,
            max_prediction: max_prediction as i32,
            check_distance: check_distance as i32,
            input_delay: input_delay as i32,
            input_capacity: 0,
            device,
            trace_capacity: 0,
        };
        let mut eng = std::ptr::null_mut();
        check(unsafe { ggrs_engine_create(&cfg, &mut eng) })?;
        Ok(Self { eng, lanes, players })
    }

    /// `requests[l]` is session l's request list from its `advance_frame()`.
    pub fn handle_requests<T>(&mut self, requests: &[Vec<GgrsRequest<T>>]) -> Result<(), EngineError>
    where
        T: Config,
        T::Input: InputByte,
    {
        assert_eq!(requests.len(), self.lanes);
        let mut reqs = Vec::new();
        let mut inputs = Vec::new();
        let mut status = Vec::new();
        let mut saves = Vec::new();
        for (k, r) in requests[0].iter().enumerate() {
            match r {
                GgrsRequest::SaveGameState { frame, .. } => {
                    reqs.push(ggrs_request_t { kind: GGRS_REQ_SAVE, frame: *frame });
                    saves.push((k, *frame));
                }
                GgrsRequest::LoadGameState { frame, .. } => {
                    reqs.push(ggrs_request_t { kind: GGRS_REQ_LOAD, frame: *frame })
                }
                GgrsRequest::AdvanceFrame { .. } => {
                    reqs.push(ggrs_request_t { kind: GGRS_REQ_ADVANCE, frame: 0 });
                    for lane in requests {
                        if let GgrsRequest::AdvanceFrame { inputs: v } = &lane[k] {
                            for (inp, st) in v {
                                inputs.push(inp.input_byte());
                                status.push(match st {
                                    InputStatus::Confirmed => GGRS_STATUS_CONFIRMED,
                                    InputStatus::Predicted => GGRS_STATUS_PREDICTED,
                                    InputStatus::Disconnected => GGRS_STATUS_DISCONNECTED,
                                });
                            }
                        }
                    }
                }
            }
        }
        debug_assert_eq!(inputs.len() % (self.lanes * self.players), 0);
        check(unsafe {
            ggrs_handle_requests(self.eng, reqs.as_ptr(), reqs.len() as i32, inputs.as_ptr(), status.as_ptr())
        })?;
        let mut cs = vec![0u16; self.lanes];
        for (k, frame) in saves {
            check(unsafe { ggrs_read_save_checksums(self.eng, frame, cs.as_mut_ptr()) })?;
            for (lane, reqs) in requests.iter().enumerate() {
                if let GgrsRequest::SaveGameState { cell, frame } = &reqs[k] {
                    cell.save(*frame, None, Some(cs[lane] as u128));
                }
            }
        }
        Ok(())
    }

    /// Fused SyncTest: n x (SyncTestSession::advance_frame + handle_requests) on every lane, for
    /// callers that do not need GGRS session objects at all.  inputs: [n][lanes][players].
    pub fn synctest(&mut self, first_frame: i32, inputs: &[u8], n: i32) -> Result<Vec<(usize, i32, u64)>, EngineError> {
        check(unsafe { ggrs_add_local_inputs(self.eng, first_frame, n, inputs.as_ptr()) })?;
        check(unsafe { ggrs_synctest_advance_frames(self.eng, n) })?;
        let mut st = vec![0i32; self.lanes];
        let mut fr = vec![0i32; self.lanes];
        let mut mask = vec![0u64; self.lanes];
        check(unsafe { ggrs_read_mismatches(self.eng, st.as_mut_ptr(), fr.as_mut_ptr(), mask.as_mut_ptr()) })?;
        // GgrsError::MismatchedChecksum per halted lane: (lane, current_frame, mismatched mask)
        Ok((0..self.lanes).filter(|&l| st[l] == GGRS_LANE_MISMATCH).map(|l| (l, fr[l], mask[l])).collect())
    }
}

impl Drop for BatchedBoxGame {
    fn drop(&mut self) {
        unsafe { ggrs_engine_destroy(self.eng) };
    }
}
