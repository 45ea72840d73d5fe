//! A GGRS request handler for L box-game sessions on one MI355X: it replaces `Game::handle_requests`
//! of examples/ex_game/ex_game.rs (:79-127) for every session at once.  Saves keep the state in HBM
//! and hand GGRS `cell.save(frame, None, Some(checksum))` (data = None is legal; GGRS only reads
//! frame() and checksum(), src/sync_layer.rs:72-78).
//!
//! Every session's request list is its own (P2PSession::advance_frame rolls back to each session's
//! own first_incorrect frame, p2p_session.rs:322-337,658-714), so `handle_requests` hands the engine
//! one list per lane: encoded into the engine's mapped lane batch (ggrs_lane_batch_run: request
//! kinds as 2-bit tokens, Load frames, input rows, checksums back in the same pinned memory), or,
//! when a list exceeds the batch limits, through the generic CSR form (ggrs_handle_requests_lanes).
//! `handle_requests_lockstep` is the one-list-for-all form for sessions known to be in lockstep; it
//! checks that assumption and returns an error instead of misaligning lanes when it does not hold.
//! `handle_requests_deferred` (P2PSessions only) returns before the device does: checksums reach
//! their cells on the next call, so the PCIe round trip overlaps the caller's session logic.
pub mod ffi;

use ffi::*;
use ggrs::{Config, GgrsRequest, InputStatus};

#[derive(Debug)]
pub struct EngineError(pub i32, pub String);

fn check(rc: i32) -> Result<(), EngineError> {
    if rc == GGRS_OK { Ok(()) } else { Err(EngineError(rc, last_error())) }
}

/// The library this crate links must implement the ABI its declarations describe (ffi.rs); checked
/// before any engine is created, so a stale libggrs_amd.so fails loudly instead of misreading a
/// changed signature (ABI 3 changed what ggrs_branch_set_stream(NULL) means).
fn check_abi() -> Result<(), EngineError> {
    let v = unsafe { ggrs_abi_version() };
    if v == GGRS_ABI_VERSION {
        Ok(())
    } else {
        Err(EngineError(GGRS_E_STATE, format!("libggrs_amd ABI {} but this crate declares ABI {}", v, GGRS_ABI_VERSION)))
    }
}

/// Turns a game input into the byte the box game reads (`Input.inp`, ex_game.rs:28-32).
pub trait InputByte {
    fn input_byte(&self) -> u8;
}

fn status_byte(st: &InputStatus) -> u8 {
    match st {
        InputStatus::Confirmed => GGRS_STATUS_CONFIRMED,
        InputStatus::Predicted => GGRS_STATUS_PREDICTED,
        InputStatus::Disconnected => GGRS_STATUS_DISCONNECTED,
    }
}

/// Lanes whose request list failed the engine's validation (a Load of a frame its cell does not
/// hold, a Save of a frame other than the state's: where the reference panics).  Those lanes were
/// left untouched; every other lane ran and its saves were delivered.
#[derive(Debug)]
pub struct FailedLanes {
    /// (lane, index of the first rejected request in its list)
    pub lanes: Vec<(usize, usize)>,
}

/// Deferred mode: the submitted batch's SaveGameStates, per lane in request order, each a closure
/// that hands the cell its checksum (`cell.save(frame, None, Some(checksum))`).
type PendingSaves = Vec<(usize, Vec<Box<dyn FnOnce(u128)>>)>;

pub struct BatchedBoxGame {
    eng: *mut ggrs_engine_t,
    lanes: usize,
    players: usize,
    /// every lane's frame after its last list (lane_result): the start frame the Save frames of
    /// its next list are checked against (ex_game.rs:104), since the batch carries no Save frames
    lane_frames: Vec<i32>,
    /// deferred mode: the batch submitted by the last call and its saves, collected by the next
    /// call (or flush)
    pending: Option<(ggrs_lane_batch_t, PendingSaves)>,
}

/// One lane's list as the C ABI takes it: requests, and one input / status row per AdvanceFrame.
fn lane_list<T>(list: &[GgrsRequest<T>], reqs: &mut Vec<ggrs_request_t>, inputs: &mut Vec<u8>, status: &mut Vec<u8>)
where
    T: Config,
    T::Input: InputByte,
{
    reqs.clear();
    inputs.clear();
    status.clear();
    for r in list {
        match r {
            GgrsRequest::SaveGameState { frame, .. } => reqs.push(ggrs_request_t { kind: GGRS_REQ_SAVE, frame: *frame }),
            GgrsRequest::LoadGameState { frame, .. } => reqs.push(ggrs_request_t { kind: GGRS_REQ_LOAD, frame: *frame }),
            GgrsRequest::AdvanceFrame { inputs: v } => {
                reqs.push(ggrs_request_t { kind: GGRS_REQ_ADVANCE, frame: 0 });
                for (inp, st) in v {
                    inputs.push(inp.input_byte());
                    status.push(status_byte(st));
                }
            }
        }
    }
}

impl BatchedBoxGame {
    /// One engine lane per session: SessionBuilder's max_prediction / check_distance / input delay.
    pub fn new(lanes: usize, players: usize, max_prediction: usize, check_distance: usize,
               input_delay: usize, device: i32) -> Result<Self, EngineError> {
        check_abi()?;
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
        Ok(Self { eng, lanes, players, lane_frames: vec![0; lanes], pending: None })
    }

    /// Every lane's list encoded into the engine's mapped batch: Ok(None) when some list exceeds the
    /// batch limits (the caller takes the CSR form), else the batch with the call's row counts and
    /// the lanes the encoder rejected (a SaveGameState of a frame other than the one the list has
    /// reached, ggrs_lane_encode).
    fn encode_batch<T>(&mut self, requests: &[Vec<GgrsRequest<T>>])
        -> Result<Option<(ggrs_lane_batch_t, Vec<(usize, usize)>)>, EngineError>
    where
        T: Config,
        T::Input: InputByte,
    {
        assert_eq!(requests.len(), self.lanes);
        // every lane's list in the ABI's form, and the batch shape: the largest per-lane counts
        let mut lists = Vec::with_capacity(self.lanes);
        let mut shape = [0i32; 4];
        for list in requests {
            let (mut reqs, mut inputs, mut status) = (Vec::new(), Vec::new(), Vec::new());
            lane_list(list, &mut reqs, &mut inputs, &mut status);
            let mut s = [0i32; 4];
            check(unsafe { ggrs_lane_shape(reqs.as_ptr(), reqs.len() as i32, s.as_mut_ptr()) })?;
            for k in 0..4 {
                shape[k] = shape[k].max(s[k]);
            }
            lists.push((reqs, inputs, status));
        }
        if shape[0] > GGRS_BATCH_MAX_WORDS || shape[1] > GGRS_BATCH_MAX_LOADS || shape[2] > GGRS_BATCH_MAX_ADV
            || shape[3] > GGRS_BATCH_MAX_SAVES {
            return Ok(None);
        }
        let (w, ld, a, s) = (shape[0].max(1), shape[1].max(1), shape[2].max(1), shape[3].max(1));
        // mapped afresh on every call: a CSR call may have grown (and freed) the previous mapping
        let mut b = ggrs_lane_batch_t {
            token_words: 0, load_slots: 0, adv_rows: 0, save_rows: 0,
            tokens: std::ptr::null_mut(), load_frames: std::ptr::null_mut(), inputs: std::ptr::null_mut(),
            status: std::ptr::null_mut(), checksums: std::ptr::null_mut(), lane_result: std::ptr::null_mut(),
        };
        check(unsafe { ggrs_lane_batch_map(self.eng, w, ld, a, s, &mut b) })?;
        let mut failed = Vec::new();
        for (lane, (reqs, inputs, status)) in lists.iter().enumerate() {
            let mut bad = -1i32;
            let rc = unsafe {
                ggrs_lane_encode(&b, self.lanes as i64, self.players as i32, lane as i64, reqs.as_ptr(),
                                 reqs.len() as i32, inputs.as_ptr(), status.as_ptr(), self.lane_frames[lane], &mut bad)
            };
            match rc {
                GGRS_OK => {}
                GGRS_E_PRECONDITION => failed.push((lane, bad as usize)),
                _ => return Err(EngineError(rc, last_error())),
            }
        }
        let mut run = b;
        run.token_words = w;
        run.load_slots = ld;
        run.adv_rows = a;
        run.save_rows = s;
        Ok(Some((run, failed)))
    }

    /// `requests[l]` is session l's request list from its `advance_frame()`; lists may differ in
    /// kinds, frames and length.  Ok(None) when every lane ran; Ok(Some(failed)) when some lanes'
    /// lists were rejected (those lanes did not run): a SaveGameState of a frame other than the one
    /// the list has reached (checked while encoding, ggrs_lane_encode), or a Load of a frame the
    /// lane's cell does not hold (checked on the device).  Returns with every checksum in its cell.
    pub fn handle_requests<T>(&mut self, requests: &[Vec<GgrsRequest<T>>]) -> Result<Option<FailedLanes>, EngineError>
    where
        T: Config,
        T::Input: InputByte,
    {
        let mut failed = self.flush()?.map(|f| f.lanes).unwrap_or_default();
        let Some((b, enc_failed)) = self.encode_batch(requests)? else {
            return Ok(merge_failed(failed, self.handle_requests_csr(requests)?));
        };
        let mut n_failed = 0i32;
        let rc = unsafe { ggrs_lane_batch_run(self.eng, &b, GGRS_BATCH_STATUS, &mut n_failed) };
        if rc != GGRS_OK && rc != GGRS_E_PRECONDITION {
            return Err(EngineError(rc, last_error()));
        }
        // every Save's checksum back to its GameStateCell, lane by lane; failed lanes report
        let rejected: std::collections::HashSet<usize> = enc_failed.iter().map(|&(l, _)| l).collect();
        failed.extend(enc_failed);
        for (lane, list) in requests.iter().enumerate() {
            let res = unsafe { *b.lane_result.add(lane) };
            if res < 0 {
                failed.push((lane, (-res - 1) as usize));
                continue;
            }
            self.lane_frames[lane] = res;
            if rejected.contains(&lane) {
                continue;
            }
            let mut si = 0usize;
            for r in list {
                if let GgrsRequest::SaveGameState { cell, frame } = r {
                    let cs = unsafe { *b.checksums.add(si * self.lanes + lane) };
                    cell.save(*frame, None, Some(cs as u128));
                    si += 1;
                }
            }
        }
        Ok(if failed.is_empty() { None } else { Some(FailedLanes { lanes: failed }) })
    }

    /// Deferred hand-back, for P2PSessions only: encodes and submits the batch, saves every cell as
    /// `cell.save(frame, None, None)` and returns at once, so the device round trip overlaps the
    /// caller's session logic until the next call; that call (or `flush`) waits for the batch and
    /// fills `Some(checksum)` into these cells in request order.  A P2PSession reads a cell's
    /// checksum only for confirmed frames at its desync interval and retries on a later call while
    /// it is None (check_checksum_send_interval, p2p_session.rs:939-963); a confirmed frame is never
    /// re-saved, so the report it sends is the same.  Not for SyncTestSessions: checksums_consistent
    /// reads the previous call's cells (sync_test_session.rs:173-190).  Lanes the device rejects
    /// are reported by the call that collects their batch.
    pub fn handle_requests_deferred<T>(&mut self, requests: &[Vec<GgrsRequest<T>>])
        -> Result<Option<FailedLanes>, EngineError>
    where
        T: Config,
        T::Input: InputByte,
        T::State: 'static,
    {
        let mut failed = self.flush()?.map(|f| f.lanes).unwrap_or_default();
        let Some((b, enc_failed)) = self.encode_batch(requests)? else {
            return Ok(merge_failed(failed, self.handle_requests_csr(requests)?));
        };
        check(unsafe { ggrs_lane_batch_submit(self.eng, &b, GGRS_BATCH_STATUS) })?;
        let rejected: std::collections::HashSet<usize> = enc_failed.iter().map(|&(l, _)| l).collect();
        failed.extend(enc_failed);
        let mut pending: PendingSaves = Vec::with_capacity(self.lanes);
        for (lane, list) in requests.iter().enumerate() {
            if rejected.contains(&lane) {
                continue;
            }
            let mut saves: Vec<Box<dyn FnOnce(u128)>> = Vec::new();
            for r in list {
                if let GgrsRequest::SaveGameState { cell, frame } = r {
                    cell.save(*frame, None, None);
                    let (c, f) = (cell.clone(), *frame);
                    saves.push(Box::new(move |cs| c.save(f, None, Some(cs))));
                }
            }
            pending.push((lane, saves));
        }
        self.pending = Some((b, pending));
        Ok(if failed.is_empty() { None } else { Some(FailedLanes { lanes: failed }) })
    }

    /// Collects the batch a deferred call submitted, if any: waits for it, hands every Save's
    /// checksum to its cell in request order and records every lane's frame.  Ok(Some(failed)):
    /// the lanes the device rejected in that batch.
    pub fn flush(&mut self) -> Result<Option<FailedLanes>, EngineError> {
        let Some((b, pending)) = self.pending.take() else {
            return Ok(None);
        };
        let mut n_failed = 0i32;
        let rc = unsafe { ggrs_lane_batch_wait(self.eng, &mut n_failed) };
        if rc != GGRS_OK && rc != GGRS_E_PRECONDITION {
            return Err(EngineError(rc, last_error()));
        }
        let mut failed = Vec::new();
        for (lane, saves) in pending {
            let res = unsafe { *b.lane_result.add(lane) };
            if res < 0 {
                failed.push((lane, (-res - 1) as usize));
                continue;
            }
            self.lane_frames[lane] = res;
            for (si, save) in saves.into_iter().enumerate() {
                save(unsafe { *b.checksums.add(si * self.lanes + lane) } as u128);
            }
        }
        Ok(if failed.is_empty() { None } else { Some(FailedLanes { lanes: failed }) })
    }

    /// The generic per-lane form (ggrs_handle_requests_lanes): any list length.
    pub fn handle_requests_csr<T>(&mut self, requests: &[Vec<GgrsRequest<T>>]) -> Result<Option<FailedLanes>, EngineError>
    where
        T: Config,
        T::Input: InputByte,
    {
        assert_eq!(requests.len(), self.lanes);
        let earlier = self.flush()?;
        let mut reqs = Vec::new();
        let mut offsets = vec![0i32];
        let mut inputs = Vec::new();
        let mut status = Vec::new();
        let mut n_saves = 0usize;
        for list in requests {
            for r in list {
                match r {
                    GgrsRequest::SaveGameState { frame, .. } => {
                        reqs.push(ggrs_request_t { kind: GGRS_REQ_SAVE, frame: *frame });
                        n_saves += 1;
                    }
                    GgrsRequest::LoadGameState { frame, .. } => {
                        reqs.push(ggrs_request_t { kind: GGRS_REQ_LOAD, frame: *frame })
                    }
                    GgrsRequest::AdvanceFrame { inputs: v } => {
                        reqs.push(ggrs_request_t { kind: GGRS_REQ_ADVANCE, frame: 0 });
                        for (inp, st) in v {
                            inputs.push(inp.input_byte());
                            status.push(status_byte(st));
                        }
                    }
                }
            }
            offsets.push(reqs.len() as i32);
        }
        let mut cks = vec![0u16; n_saves.max(1)];
        let mut result = vec![0i32; self.lanes];
        let rc = unsafe {
            ggrs_handle_requests_lanes(self.eng, reqs.as_ptr(), offsets.as_ptr(), inputs.as_ptr(), status.as_ptr(),
                                       cks.as_mut_ptr(), result.as_mut_ptr())
        };
        if rc != GGRS_OK && rc != GGRS_E_PRECONDITION {
            return Err(EngineError(rc, last_error()));
        }
        let mut failed = Vec::new();
        let mut k = 0usize;
        for (lane, list) in requests.iter().enumerate() {
            let ok = result[lane] >= 0;
            if !ok {
                failed.push((lane, (-result[lane] - 1) as usize));
            } else {
                self.lane_frames[lane] = result[lane];
            }
            for r in list {
                if let GgrsRequest::SaveGameState { cell, frame } = r {
                    if ok {
                        cell.save(*frame, None, Some(cks[k] as u128));
                    }
                    k += 1;
                }
            }
        }
        Ok(merge_failed(earlier.map(|f| f.lanes).unwrap_or_default(),
                        if failed.is_empty() { None } else { Some(FailedLanes { lanes: failed }) }))
    }

    /// One list for every lane (ggrs_handle_requests: one launch, the lists' kinds and frames
    /// shared).  Valid only for sessions in lockstep: a lane whose kinds or frames differ from
    /// lane 0's is an error (GGRS_E_INVALID), nothing runs.  An engine that has run per-lane lists
    /// keeps per-lane frames and refuses this form (GGRS_E_STATE).
    pub fn handle_requests_lockstep<T>(&mut self, requests: &[Vec<GgrsRequest<T>>]) -> Result<(), EngineError>
    where
        T: Config,
        T::Input: InputByte,
    {
        assert_eq!(requests.len(), self.lanes);
        if let Some(f) = self.flush()? {
            return Err(EngineError(GGRS_E_PRECONDITION, format!("lanes {:?} of the previous deferred batch failed", f.lanes)));
        }
        let shape = |r: &GgrsRequest<T>| match r {
            GgrsRequest::SaveGameState { frame, .. } => (GGRS_REQ_SAVE, *frame),
            GgrsRequest::LoadGameState { frame, .. } => (GGRS_REQ_LOAD, *frame),
            GgrsRequest::AdvanceFrame { .. } => (GGRS_REQ_ADVANCE, 0),
        };
        let lead: Vec<(i32, i32)> = requests[0].iter().map(shape).collect();
        for (lane, list) in requests.iter().enumerate().skip(1) {
            if list.len() != lead.len() || list.iter().map(shape).zip(lead.iter()).any(|(a, b)| a != *b) {
                return Err(EngineError(GGRS_E_INVALID,
                                       format!("lane {lane}'s request list differs from lane 0's: not in lockstep")));
            }
        }
        let mut reqs = Vec::new();
        let mut inputs = Vec::new();
        let mut status = Vec::new();
        let mut saves = Vec::new();
        for (k, &(kind, frame)) in lead.iter().enumerate() {
            reqs.push(ggrs_request_t { kind, frame });
            if kind == GGRS_REQ_SAVE {
                saves.push((k, frame));
            } else if kind == GGRS_REQ_ADVANCE {
                for lane in requests {
                    if let GgrsRequest::AdvanceFrame { inputs: v } = &lane[k] {
                        for (inp, st) in v {
                            inputs.push(inp.input_byte());
                            status.push(status_byte(st));
                        }
                    }
                }
            }
        }
        check(unsafe {
            ggrs_handle_requests(self.eng, reqs.as_ptr(), reqs.len() as i32, inputs.as_ptr(), status.as_ptr())
        })?;
        // every save's checksums in one transfer wait: [saves][lanes]
        let frames: Vec<i32> = saves.iter().map(|&(_, f)| f).collect();
        let mut cs = vec![0u16; self.lanes * frames.len()];
        if !frames.is_empty() {
            check(unsafe {
                ggrs_read_save_checksums_frames(self.eng, frames.as_ptr(), frames.len() as i32, cs.as_mut_ptr())
            })?;
        }
        for (j, &(k, _)) in saves.iter().enumerate() {
            for (lane, reqs) in requests.iter().enumerate() {
                if let GgrsRequest::SaveGameState { cell, frame } = &reqs[k] {
                    cell.save(*frame, None, Some(cs[j * self.lanes + lane] as u128));
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

    /// Every lane's current frame (after per-lane lists).
    pub fn lane_frames(&mut self) -> Result<Vec<i32>, EngineError> {
        let mut out = vec![0i32; self.lanes];
        check(unsafe { ggrs_read_lane_frames(self.eng, out.as_mut_ptr()) })?;
        Ok(out)
    }
}

/// The failures collected from an earlier deferred batch followed by this call's.
fn merge_failed(mut earlier: Vec<(usize, usize)>, now: Option<FailedLanes>) -> Option<FailedLanes> {
    if let Some(f) = now {
        earlier.extend(f.lanes);
    }
    if earlier.is_empty() { None } else { Some(FailedLanes { lanes: earlier }) }
}

impl Drop for BatchedBoxGame {
    fn drop(&mut self) {
        let _ = self.flush();  // a deferred batch's checksums still reach their cells
        unsafe { ggrs_engine_destroy(self.eng) };
    }
}
