// Host-side KAT of the product sincosf restatement (ggrs_amd/csrc/glibc_sincosf.h) against this
// image's glibc libm sinf/cosf.  Test infrastructure: compiled by tests/test_sincosf_kat.py.
// usage: sincosf_kat_host <lo_bits_hex> <hi_bits_hex> [threads]   (inclusive f32 bit range)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include <atomic>
#include "glibc_sincosf.h"

static uint32_t bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

int main(int argc, char** argv) {
  uint64_t lo = strtoull(argv[1], nullptr, 16), hi = strtoull(argv[2], nullptr, 16);
  int nt = argc > 3 ? atoi(argv[3]) : 8;
  std::atomic<uint64_t> bad_s{0}, bad_c{0}, bad_f{0}, bad_d{0};
  std::vector<std::thread> th;
  for (int t = 0; t < nt; t++) th.emplace_back([&, t] {
    uint64_t bs = 0, bc = 0, bf = 0, bd = 0;
    for (uint64_t u = lo + t; u <= hi; u += nt) {
      float f; uint32_t w = (uint32_t)u; std::memcpy(&f, &w, 4);
      float a = sinf(f), b = ggrs::glibc_sinf(f);
      float c = cosf(f), d = ggrs::glibc_cosf(f);
      if (bits(a) != bits(b) && !(std::isnan(a) && std::isnan(b))) { if (bs < 3) printf("sin %a libm %a port %a\n", f, a, b); bs++; }
      if (bits(c) != bits(d) && !(std::isnan(c) && std::isnan(d))) { if (bc < 3) printf("cos %a libm %a port %a\n", f, c, d); bc++; }
      if (std::fabs(f) < 120.0f) {
        float s2, c2; ggrs::glibc_sincosf_small(f, &s2, &c2);
        if (bits(s2) != bits(a) || bits(c2) != bits(c)) bf++;
      }
      if (w <= ggrs::kTwoPiBits) {
        float s3, c3; ggrs::glibc_sincosf_domain(f, &s3, &c3);
        if (bits(s3) != bits(a) || bits(c3) != bits(c)) { if (bd < 3) printf("domain %a\n", f); bd++; }
        float s5, c5; uint32_t q5s, q5c; ggrs::glibc_sincosf_domain_raw(f, &s5, &c5, &q5s, &q5c);
        if ((bits(s5) ^ q5s) != bits(a) || (bits(c5) ^ q5c) != bits(c)) { if (bd < 3) printf("domain_raw %a\n", f); bd++; }
        float s4, c4; ggrs::glibc_sincosf_domain_k(f, &s4, &c4, ggrs::sincos_consts_vgpr());
        if (bits(s4) != bits(a) || bits(c4) != bits(c)) { if (bd < 3) printf("domain_k %a\n", f); bd++; }
      }
    }
    bad_s += bs; bad_c += bc; bad_f += bf; bad_d += bd;
  });
  for (auto& x : th) x.join();
  printf("range %08llx..%08llx bad_sin %llu bad_cos %llu bad_fused %llu bad_domain %llu\n", (unsigned long long)lo,
         (unsigned long long)hi, (unsigned long long)bad_s.load(), (unsigned long long)bad_c.load(),
         (unsigned long long)bad_f.load(), (unsigned long long)bad_d.load());
  return (bad_s || bad_c || bad_f || bad_d) ? 1 : 0;
}
