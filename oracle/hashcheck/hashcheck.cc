// hashcheck.cc -- TEST INFRASTRUCTURE ONLY.  Pins the oracle's gram hashes to
// the reference's own implementation: this driver is linked with
// /root/reference/cld2/internal/cldutil_shared.cc compiled from where it lies
// (oracle/hashcheck/Makefile; that translation unit needs no table and no
// stand-in), and with oracle/cld_oracle.c.  It compares, on seeded random
// byte spans of every length class 0..40 with and without a space before /
// after the gram (the pre/post-space indicator bits):
//   QuadHashV2 (cldutil_shared.cc:196)  vs cldo_gram_hash(0)
//   BiHashV2   (cldutil_shared.cc:107)  vs cldo_gram_hash(1)
//   OctaHash40 (cldutil_shared.cc:348)  vs cldo_gram_hash(2)
//   PairHash   (cldutil_shared.cc:384)  vs cldo_pair_hash
// Usage: hashcheck [n_spans]  -> prints one JSON line, exit 0 iff all equal.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../cld_oracle.h"

namespace CLD2 {   // the reference's signatures (cldutil_shared.h:60-120, integral_types.h)
typedef unsigned int uint32;
typedef unsigned long long uint64;
uint32 BiHashV2(const char* word_ptr, int bytecount);
uint32 QuadHashV2(const char* word_ptr, int bytecount);
uint64 OctaHash40(const char* word_ptr, int bytecount);
uint64 PairHash(uint64 worda_hash, uint64 wordb_hash);
}  // namespace CLD2

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next64() {   // splitmix64
  uint64_t z = (rng += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 1000000;
  long bad[4] = {0, 0, 0, 0}, per_len[41] = {0};
  char buf[64];
  for (long i = 0; i < n; ++i) {
    const int len = (int)(i % 41);                // every length class, evenly
    for (int k = 0; k < 64; ++k) {
      const uint64_t r = next64();
      // mostly letters (ASCII and UTF-8 lead/continuation bytes), some spaces
      const int c = (int)(r & 7);
      buf[k] = (char)(c == 0 ? ' ' : c < 4 ? 'a' + (int)((r >> 8) % 26) : 0x80 + (int)((r >> 8) % 0x7F));
    }
    const uint64_t sel = next64();
    char* w = buf + 8;
    w[-1] = (sel & 1) ? ' ' : 'x';                // pre-space bit both ways
    w[len] = (sel & 2) ? ' ' : 'y';               // post-space bit both ways
    ++per_len[len];
    if ((uint64_t)CLD2::QuadHashV2(w, len) != cldo_gram_hash(0, w, len)) ++bad[0];
    if ((uint64_t)CLD2::BiHashV2(w, len) != cldo_gram_hash(1, w, len)) ++bad[1];
    if ((uint64_t)CLD2::OctaHash40(w, len) != cldo_gram_hash(2, w, len)) ++bad[2];
    const uint64_t a = next64(), b = next64();
    if ((uint64_t)CLD2::PairHash(a, b) != cldo_pair_hash(a, b)) ++bad[3];
  }
  printf("{\"spans\": %ld, \"lengths\": \"0..40\", \"quad_mismatch\": %ld, \"bi_mismatch\": %ld, "
         "\"octa_mismatch\": %ld, \"pair_mismatch\": %ld}\n", n, bad[0], bad[1], bad[2], bad[3]);
  return (bad[0] | bad[1] | bad[2] | bad[3]) ? 1 : 0;
}
