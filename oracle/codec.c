/* codec.c -- CPU restatement of GGRS's input wire codec (TEST INFRASTRUCTURE: the checker of the
 * GPU codec in ggrs_amd/csrc/codec.hip; never the product path).
 *
 * Reference: src/network/compression.rs (caspark/ggrs 0.10.2)
 *   encode        :14-24   delta_encode -> bitfield_rle::encode -> bincode::serialize
 *   delta_encode  :26-81   XOR against the reference / the previous input, sizes when they vary
 *   decode        :83-95   bincode::deserialize -> bitfield_rle::decode -> delta_decode
 *   delta_decode  :97-182  size checks returning errors (never panics on hostile input)
 * Third-party algorithms restated (not vendored in /root/reference):
 *   bitfield-rle 0.2.1 (Cargo.toml:20): a sequence of runs, each introduced by an unsigned LEB128
 *     varint header h: h odd  -> compressed run of (h >> 2) bytes, all 0xFF if (h & 2) else 0x00;
 *                      h even -> literal run of (h >> 1) bytes that follow the header.
 *     Encoder run choice: every maximal run of identical 0x00 or 0xFF bytes is a compressed run,
 *     every maximal stretch of other bytes a literal run.  The wire format is pinned by the
 *     format; the encoder's exact run choice is this restatement's (parity of encoded BYTES with
 *     the crate is unpinned; decode of any valid stream and encode->decode round trips are).
 *   bincode 1.3 top-level serialize/deserialize (fixint, little endian, trailing bytes allowed):
 *     EncodedInputSequence { input_sizes: Option<Vec<i32>>, encoded_bytes: Vec<u8> } =
 *     u8 tag (0 None / 1 Some) [u64 n, n x i32] u64 m, m bytes; any other tag or a short buffer is
 *     an error.
 * Deviation guarded: a decoded buffer larger than CODEC_MAX_DECODED bytes is rejected (the crate
 * would attempt the allocation); GGRS input packets are orders of magnitude smaller. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define CODEC_MAX_DECODED (1 << 24)

enum { CODEC_OK = 0, CODEC_E_BINCODE = -1, CODEC_E_RLE = -2, CODEC_E_DELTA = -3, CODEC_E_CAP = -4 };

static int put_varint(uint8_t* out, int64_t cap, int64_t* pos, uint64_t v) {
  do {
    if (*pos >= cap) return -1;
    uint8_t b = v & 0x7f;
    v >>= 7;
    out[(*pos)++] = b | (v ? 0x80 : 0);
  } while (v);
  return 0;
}

/* bitfield_rle::encode */
int64_t oracle_rle_encode(const uint8_t* in, int64_t n, uint8_t* out, int64_t cap) {
  int64_t pos = 0, i = 0;
  while (i < n) {
    int64_t j = i;
    if (in[i] == 0x00 || in[i] == 0xFF) {
      while (j < n && in[j] == in[i]) j++;
      if (put_varint(out, cap, &pos, ((uint64_t)(j - i) << 2) | (in[i] == 0xFF ? 2u : 0u) | 1u)) return -1;
    } else {
      while (j < n && in[j] != 0x00 && in[j] != 0xFF) j++;
      if (put_varint(out, cap, &pos, (uint64_t)(j - i) << 1)) return -1;
      if (pos + (j - i) > cap) return -1;
      memcpy(out + pos, in + i, (size_t)(j - i));
      pos += j - i;
    }
    i = j;
  }
  return pos;
}

static int get_varint(const uint8_t* in, int64_t n, int64_t* pos, uint64_t* v) {
  uint64_t r = 0;
  for (int shift = 0; shift < 64; shift += 7) {
    if (*pos >= n) return -1;
    const uint8_t b = in[(*pos)++];
    r |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) { *v = r; return 0; }
  }
  return -1; /* more than 10 bytes */
}

/* bitfield_rle::decode: decoded length, or CODEC_E_RLE / CODEC_E_CAP */
int64_t oracle_rle_decode(const uint8_t* in, int64_t n, uint8_t* out, int64_t cap) {
  int64_t pos = 0, o = 0;
  while (pos < n) {
    uint64_t h;
    if (get_varint(in, n, &pos, &h)) return CODEC_E_RLE;
    const uint64_t len = (h & 1) ? h >> 2 : h >> 1;
    if (len > CODEC_MAX_DECODED || (uint64_t)o + len > CODEC_MAX_DECODED) return CODEC_E_RLE;
    if ((uint64_t)o + len > (uint64_t)cap) return CODEC_E_CAP;
    if (h & 1) {
      memset(out + o, (h & 2) ? 0xFF : 0x00, (size_t)len);
    } else {
      if ((uint64_t)(n - pos) < len) return CODEC_E_RLE;
      memcpy(out + o, in + pos, (size_t)len);
      pos += (int64_t)len;
    }
    o += (int64_t)len;
  }
  return o;
}

/* compression::encode.  inputs: n inputs back to back, lens[k] bytes each.  Returns the packet
 * length, or CODEC_E_CAP. */
int64_t oracle_codec_encode(const uint8_t* ref, int32_t ref_len, const uint8_t* inputs, const int32_t* lens,
                            int32_t n, uint8_t* out, int64_t cap) {
  int all_ref = ref_len > 0;
  int64_t total = 0;
  for (int32_t k = 0; k < n; k++) { all_ref &= lens[k] == ref_len; total += lens[k]; }
  uint8_t* x = (uint8_t*)malloc(total > 0 ? (size_t)total : 1);
  /* delta_encode (:55-75) */
  const uint8_t* base = ref; int32_t base_len = ref_len;
  int64_t p = 0, off = 0;
  for (int32_t k = 0; k < n; k++) {
    const uint8_t* in = inputs + off;
    const int32_t m = lens[k] < base_len ? lens[k] : base_len;
    for (int32_t b = 0; b < m; b++) x[p++] = base[b] ^ in[b];
    for (int32_t b = m; b < lens[k]; b++) x[p++] = in[b];
    base = in; base_len = lens[k];
    off += lens[k];
  }
  /* bincode: tag, [sizes], u64 len, rle bytes */
  int64_t pos = 0;
  const int64_t hdr = 1 + (all_ref ? 0 : 8 + 4 * (int64_t)n) + 8;
  if (cap < hdr) { free(x); return CODEC_E_CAP; }
  out[pos++] = all_ref ? 0 : 1;
  if (!all_ref) {
    uint64_t nn = (uint64_t)n;
    for (int b = 0; b < 8; b++) out[pos++] = (uint8_t)(nn >> (8 * b));
    int32_t bs = ref_len;
    for (int32_t k = 0; k < n; k++) { /* :42-51 */
      const uint32_t d = (uint32_t)(lens[k] - bs);
      for (int b = 0; b < 4; b++) out[pos++] = (uint8_t)(d >> (8 * b));
      bs = lens[k];
    }
  }
  const int64_t len_at = pos;
  pos += 8;
  const int64_t r = oracle_rle_encode(x, total, out + pos, cap - pos);
  free(x);
  if (r < 0) return CODEC_E_CAP;
  for (int b = 0; b < 8; b++) out[len_at + b] = (uint8_t)((uint64_t)r >> (8 * b));
  return pos + r;
}

/* compression::decode.  On success writes the decoded inputs back to back into out (cap bytes),
 * their sizes into lens (lens_cap entries), *n_out, and returns 0; else a negative CODEC_E_*. */
int oracle_codec_decode(const uint8_t* ref, int32_t ref_len, const uint8_t* data, int64_t len, uint8_t* out,
                        int64_t cap, int32_t* lens, int32_t lens_cap, int32_t* n_out) {
  *n_out = 0;
  int64_t pos = 0;
  if (len < 1) return CODEC_E_BINCODE;
  const uint8_t tag = data[pos++];
  if (tag > 1) return CODEC_E_BINCODE;
  uint64_t n_sizes = 0;
  int64_t sizes_at = 0;
  if (tag == 1) {
    if (len - pos < 8) return CODEC_E_BINCODE;
    for (int b = 0; b < 8; b++) n_sizes |= (uint64_t)data[pos + b] << (8 * b);
    pos += 8;
    if (n_sizes > (uint64_t)(len - pos) / 4) return CODEC_E_BINCODE; /* runs out of bytes */
    sizes_at = pos;
    pos += 4 * (int64_t)n_sizes;
  }
  if (len - pos < 8) return CODEC_E_BINCODE;
  uint64_t m = 0;
  for (int b = 0; b < 8; b++) m |= (uint64_t)data[pos + b] << (8 * b);
  pos += 8;
  if (m > (uint64_t)(len - pos)) return CODEC_E_BINCODE;
  /* the decoded bytes: a per-thread scratch of the decode cap, allocated once (a 16 MiB malloc per
   * packet is an mmap + munmap: page faults that serialise threads) */
  static __thread uint8_t* scratch;
  if (!scratch) scratch = (uint8_t*)malloc(CODEC_MAX_DECODED);
  uint8_t* x = scratch;
  const int64_t xl = oracle_rle_decode(data + pos, (int64_t)m, x, CODEC_MAX_DECODED);
  if (xl < 0) { return CODEC_E_RLE; }
  /* delta_decode (:97-182): the sizes first */
  int64_t count;
  if (tag == 1) {
    count = (int64_t)n_sizes;
    int64_t bs = ref_len, sum = 0;
    for (int64_t k = 0; k < count; k++) {
      uint32_t u = 0;
      for (int b = 0; b < 4; b++) u |= (uint32_t)data[sizes_at + 4 * k + b] << (8 * b);
      const int32_t rel = (int32_t)u;
      const int64_t sz = (int64_t)(int32_t)((uint32_t)bs + (uint32_t)rel); /* i32 arithmetic (:118) */
      if (sz < 0) { return CODEC_E_DELTA; }
      if (k < lens_cap) lens[k] = (int32_t)sz;
      bs = sz;
      sum += sz;
      if (sum > xl) { return CODEC_E_DELTA; }
    }
    if (sum != xl) { return CODEC_E_DELTA; }
  } else {
    if (ref_len == 0) { return CODEC_E_DELTA; }
    count = xl / ref_len;
    for (int64_t k = 0; k < count && k < lens_cap; k++) lens[k] = ref_len;
    if (count * ref_len != xl) { return CODEC_E_DELTA; }
  }
  if (count > lens_cap || xl > cap) { return CODEC_E_CAP; }
  const uint8_t* base = ref; int64_t base_len = ref_len;
  int64_t p = 0;
  for (int64_t k = 0; k < count; k++) {
    const int64_t sz = lens[k];
    for (int64_t b = 0; b < sz; b++) out[p + b] = x[p + b] ^ (b < base_len ? base[b] : 0);
    base = out + p; base_len = sz;
    p += sz;
  }
  *n_out = (int32_t)count;
  return CODEC_OK;
}

/* CPU baseline of the batched codec (bench.py --workload codec): encode then decode every packet
 * (one thread, the reference's per-endpoint call pattern), `passes` times.  Returns packets
 * round-tripped; *wall = seconds; -1 on a round-trip mismatch. */
#include <time.h>
int64_t oracle_codec_bench(const uint8_t* ref, const uint8_t* pending, const int32_t* count, int64_t n_packets,
                           int32_t B, int32_t W, int32_t passes, double* wall) {
  const int64_t cap = 64 + 4 * (int64_t)W + 2 * (int64_t)W * B;
  uint8_t* pkt = (uint8_t*)malloc((size_t)cap);
  uint8_t* dec = (uint8_t*)malloc((size_t)W * B + 1);
  int32_t* lens = (int32_t*)malloc(sizeof(int32_t) * ((size_t)W + 1));
  for (int32_t k = 0; k <= W; k++) lens[k] = B;
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  int64_t done = 0;
  for (int32_t it = 0; it < passes; it++)
    for (int64_t p = 0; p < n_packets; p++) {
      const int64_t n = oracle_codec_encode(ref + p * B, B, pending + p * (int64_t)W * B, lens, count[p], pkt, cap);
      int32_t got = 0;
      int32_t dl[256];
      if (n < 0 || oracle_codec_decode(ref + p * B, B, pkt, n, dec, (int64_t)W * B + 1, dl, 256, &got) != 0 ||
          got != count[p]) {
        free(pkt); free(dec); free(lens);
        return -1;
      }
      done++;
    }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  *wall = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
  free(pkt); free(dec); free(lens);
  return done;
}

/* oracle_codec_bench on `threads` threads, each its own slice of the packets (the endpoints a game
 * server's threads would serve), `passes` times.  Returns packets round-tripped (-1 on a mismatch);
 * *wall = seconds from the first start to the last end. */
#include <pthread.h>
typedef struct {
  const uint8_t *ref, *pending;
  const int32_t* count;
  int64_t n;
  int32_t B, W, passes;
  int64_t done;
  double wall;
} CodecJob;
static void* codec_worker(void* arg) {
  CodecJob* j = (CodecJob*)arg;
  j->done = oracle_codec_bench(j->ref, j->pending, j->count, j->n, j->B, j->W, j->passes, &j->wall);
  return NULL;
}
int64_t oracle_codec_bench_mt(const uint8_t* ref, const uint8_t* pending, const int32_t* count, int64_t n_packets,
                              int32_t B, int32_t W, int32_t passes, int32_t threads, double* wall) {
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  pthread_t th[64];
  CodecJob jobs[64];
  const int64_t per = (n_packets + threads - 1) / threads;
  int used = 0;
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < threads; t++) {
    const int64_t a = (int64_t)t * per, b = a + per < n_packets ? a + per : n_packets;
    if (a >= b) break;
    jobs[t] = (CodecJob){ref + a * B, pending + a * (int64_t)W * B, count + a, b - a, B, W, passes, 0, 0};
    pthread_create(&th[t], NULL, codec_worker, &jobs[t]);
    used++;
  }
  int64_t done = 0;
  int bad = 0;
  for (int t = 0; t < used; t++) {
    pthread_join(th[t], NULL);
    if (jobs[t].done < 0) bad = 1;
    else done += jobs[t].done;
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  *wall = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
  return bad ? -1 : done;
}
