// lane_encode.cpp -- host-side encoding of one session's ordered request list into a lane batch
// (ggrs_lane_encode / ggrs_lane_shape, include/ggrs_amd.h).  This is the per-session work of a GGRS
// request handler in front of ggrs_lane_batch_run: GGRS hands the handler one Vec<GgrsRequest> per
// session per advance_frame (src/lib.rs:171-195; P2PSession::advance_frame, p2p_session.rs:265-426),
// and the handler writes its kinds, Load frames and AdvanceFrame input rows into the session's
// column of the batch.  One C implementation shared by every caller: the Rust handler crate
// (rust/ggrs-mi355x/src/lib.rs), the bench's C driver (bench_native/handler_driver.c) and tests.
//
// The batch carries no Save frames (the kernel saves the state the list has reached), so the one
// assert of Game::handle_requests the device cannot check -- `assert_eq!(self.state.frame, frame)`
// on SaveGameState, examples/ex_game/ex_game.rs:104 -- is checked here against the frame the list
// reaches from the lane's current frame (its last lane_result).  The Load asserts
// (sync_layer.rs:231-248) are checked on the device against the lane's cell tags.
// Pure host code: no HIP call, usable without a GPU.
#include <stdint.h>

#include "ggrs_amd.h"

namespace {

inline uint32_t token_of(int32_t kind) {
  return kind == GGRS_REQ_SAVE ? GGRS_TOK_SAVE : (kind == GGRS_REQ_LOAD ? GGRS_TOK_LOAD : GGRS_TOK_ADVANCE);
}

}  // namespace

namespace ggrs {
int set_error(int code, const char* fmt, ...);
}

extern "C" {

int ggrs_lane_shape(const ggrs_request_t* reqs, int32_t n_reqs, int32_t* shape) {
  if (!shape || n_reqs < 0 || (n_reqs > 0 && !reqs)) return ggrs::set_error(GGRS_E_INVALID, "bad request list");
  int32_t ld = 0, adv = 0, sv = 0;
  for (int32_t k = 0; k < n_reqs; k++) {
    const int32_t kind = reqs[k].kind;
    if (kind == GGRS_REQ_LOAD) ld++;
    else if (kind == GGRS_REQ_ADVANCE) adv++;
    else if (kind == GGRS_REQ_SAVE) sv++;
    else return ggrs::set_error(GGRS_E_INVALID, "request %d: unknown kind %d", k, kind);
  }
  // a list of exactly W * 16 requests needs no END token: the kernel stops after W words
  shape[0] = (n_reqs + GGRS_TOKENS_PER_WORD - 1) / GGRS_TOKENS_PER_WORD;
  shape[1] = ld;
  shape[2] = adv;
  shape[3] = sv;
  return GGRS_OK;
}

int ggrs_lane_encode(const ggrs_lane_batch_t* b, int64_t num_lanes, int32_t num_players, int64_t lane,
                     const ggrs_request_t* reqs, int32_t n_reqs, const uint8_t* inputs, const uint8_t* status,
                     int32_t lane_frame, int32_t* bad_request) {
  if (bad_request) *bad_request = -1;
  if (!b || !b->tokens || !b->load_frames || !b->inputs || !b->status)
    return ggrs::set_error(GGRS_E_INVALID, "null batch");
  if (num_lanes < 1 || lane < 0 || lane >= num_lanes || num_players < 1 || num_players > 4)
    return ggrs::set_error(GGRS_E_INVALID, "lane %lld of %lld lanes, %d players", (long long)lane,
                           (long long)num_lanes, num_players);
  if (n_reqs < 0 || (n_reqs > 0 && !reqs)) return ggrs::set_error(GGRS_E_INVALID, "bad request list");
  // one pass: the list's shape (ggrs_lane_shape) and the Save frames against the frame the list
  // reaches (ex_game.rs:104; a Save of NULL_FRAME is the assert of GameStateCell::save,
  // sync_layer.rs:20) -- a GGRS list is a handful of requests, so a pass per check cost more than
  // the checks
  int32_t ld = 0, adv = 0, sv = 0, bad = -1, f = lane_frame;
  const bool check_saves = lane_frame != GGRS_NULL_FRAME;
  for (int32_t k = 0; k < n_reqs; k++) {
    const int32_t kind = reqs[k].kind;
    if (kind == GGRS_REQ_LOAD) {
      ld++;
      f = reqs[k].frame;
    } else if (kind == GGRS_REQ_ADVANCE) {
      adv++;
      f += 1;
    } else if (kind == GGRS_REQ_SAVE) {
      sv++;
      if (check_saves && bad < 0 && (reqs[k].frame == GGRS_NULL_FRAME || reqs[k].frame != f)) bad = k;
    } else {
      return ggrs::set_error(GGRS_E_INVALID, "request %d: unknown kind %d", k, kind);
    }
  }
  const int32_t words = (n_reqs + GGRS_TOKENS_PER_WORD - 1) / GGRS_TOKENS_PER_WORD;
  if (adv > 0 && !inputs) return ggrs::set_error(GGRS_E_INVALID, "null inputs for %d AdvanceFrames", adv);
  if (words > b->token_words || ld > b->load_slots || adv > b->adv_rows || sv > b->save_rows)
    return ggrs::set_error(GGRS_E_INVALID, "lane %lld's list (%d words, %d loads, %d advances, %d saves) exceeds the "
                           "batch (%d, %d, %d, %d)", (long long)lane, words, ld, adv, sv, b->token_words,
                           b->load_slots, b->adv_rows, b->save_rows);
  const int64_t L = num_lanes;
  const int P = num_players;
  const int32_t n = bad >= 0 ? 0 : n_reqs;  // a rejected lane gets an empty list: it does not run
  // token words: every slot END (all ones) unless a request fills it
  int32_t k = 0, li = 0, ai = 0;
  for (int32_t w = 0; w < b->token_words; w++) {
    uint32_t word = 0xFFFFFFFFu;
    for (int t = 0; t < GGRS_TOKENS_PER_WORD && k < n; t++, k++) {
      const ggrs_request_t& r = reqs[k];
      word &= ~(3u << (2 * t));
      word |= token_of(r.kind) << (2 * t);
      if (r.kind == GGRS_REQ_LOAD) {
        b->load_frames[(int64_t)li * L + lane] = r.frame;
        li++;
      } else if (r.kind == GGRS_REQ_ADVANCE) {
        uint8_t* in = b->inputs + ((int64_t)ai * L + lane) * P;
        uint8_t* st = b->status + ((int64_t)ai * L + lane) * P;
        const uint8_t* src_in = inputs + (int64_t)ai * P;
        if (P == 2) {  // the two-player row as one 16-bit store
          uint16_t v;
          __builtin_memcpy(&v, src_in, 2);
          __builtin_memcpy(in, &v, 2);
          if (status) __builtin_memcpy(&v, status + (int64_t)ai * P, 2);
          else v = (uint16_t)(GGRS_STATUS_CONFIRMED | (GGRS_STATUS_CONFIRMED << 8));
          __builtin_memcpy(st, &v, 2);
        } else {
          for (int p = 0; p < P; p++) {
            in[p] = src_in[p];
            st[p] = status ? status[(int64_t)ai * P + p] : (uint8_t)GGRS_STATUS_CONFIRMED;
          }
        }
        ai++;
      }
    }
    b->tokens[(int64_t)w * L + lane] = word;
  }
  if (bad >= 0) {
    if (bad_request) *bad_request = bad;
    return ggrs::set_error(GGRS_E_PRECONDITION, "lane %lld: SaveGameState of frame %d at request %d, but the list "
                           "has reached frame %d there (ex_game.rs:104)", (long long)lane, reqs[bad].frame, bad,
                           [&] {
                             int32_t fr = lane_frame;
                             for (int32_t q = 0; q < bad; q++)
                               fr = reqs[q].kind == GGRS_REQ_LOAD ? reqs[q].frame
                                                                  : (reqs[q].kind == GGRS_REQ_ADVANCE ? fr + 1 : fr);
                             return fr;
                           }());
  }
  return GGRS_OK;
}

}  // extern "C"
