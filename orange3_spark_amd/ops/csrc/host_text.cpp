// Host-side text runtime (C ABI, libo3s_host.so): the same MurmurHash3_x86_32 as the
// device kernel for CPU sessions, and a UTF-8 aware whitespace/lowercase tokenizer used by
// Tokenizer on large columns (Python's str.split per row is the bottleneck otherwise).
#include <stdint.h>
#include <string.h>

#include "murmur3.h"

extern "C" {

__attribute__((visibility("default"))) void o3s_host_murmur3(const int64_t* offs, const uint8_t* bytes,
                                                             int64_t n, uint32_t seed, int64_t num_buckets,
                                                             int32_t* hash_out, int64_t* bucket_out) {
  for (int64_t t = 0; t < n; ++t) {
    const uint32_t h = o3s_murmur3_32(bytes + offs[t], offs[t + 1] - offs[t], seed);
    if (hash_out) hash_out[t] = (int32_t)h;
    if (bucket_out && num_buckets > 0) {
      const int64_t raw = (int64_t)(int32_t)h % num_buckets;
      bucket_out[t] = raw < 0 ? raw + num_buckets : raw;
    }
  }
}

// Spark Tokenizer semantics (Tokenizer.createTransformFunc: toLowerCase + split("\\s")):
// ASCII lower-case, then split on EVERY single whitespace character [ \t\n\v\f\r] --
// runs of whitespace yield empty tokens, a leading separator yields a leading empty token,
// trailing empty tokens are dropped (Java String.split), an empty string is one empty
// token and an all-whitespace string has none.  Writes token byte ranges into
// tok_start/tok_end (capacity cap) and per-string token counts; returns the total or -1
// if cap is too small.  Bytes are lower-cased into `out_bytes`.
static inline bool o3s_ws(uint8_t c) { return c == ' ' || (c >= 9 && c <= 13); }

__attribute__((visibility("default"))) int64_t o3s_host_tokenize(const int64_t* offs, const uint8_t* bytes,
                                                                 int64_t n, uint8_t* out_bytes, int64_t* tok_start,
                                                                 int64_t* tok_end, int64_t cap,
                                                                 int64_t* counts) {
  int64_t k = 0;
  for (int64_t s = 0; s < n; ++s) {
    const int64_t a = offs[s], b = offs[s + 1];
    int64_t last = -1;
    for (int64_t i = a; i < b; ++i) {
      const uint8_t ch = bytes[i];
      out_bytes[i] = (ch >= 'A' && ch <= 'Z') ? (uint8_t)(ch + 32) : ch;
      if (!o3s_ws(ch)) last = i;
    }
    int64_t c = 0;
    if (a == b) {                                   // "" -> [""]
      if (k >= cap) return -1;
      tok_start[k] = a; tok_end[k] = a; ++k; ++c;
    } else if (last >= 0) {
      int64_t st = a;
      for (int64_t i = a; i <= last; ++i) {
        if (o3s_ws(bytes[i])) {
          if (k >= cap) return -1;
          tok_start[k] = st; tok_end[k] = i; ++k; ++c;
          st = i + 1;
        }
      }
      if (k >= cap) return -1;
      tok_start[k] = st; tok_end[k] = last + 1; ++k; ++c;
    }
    counts[s] = c;
  }
  return k;
}
}
