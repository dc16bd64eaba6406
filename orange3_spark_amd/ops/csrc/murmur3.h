// MurmurHash3_x86_32 (public-domain algorithm by Austin Appleby), shared by the device
// kernel and the host library so both paths hash identically.  Spark's HashingTF /
// FeatureHasher hash a term's UTF-8 bytes with seed 42 and take nonNegativeMod.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define O3S_HD __host__ __device__ __forceinline__
#else
#define O3S_HD inline
#endif

O3S_HD uint32_t o3s_rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

O3S_HD uint32_t o3s_murmur3_32(const uint8_t* data, int64_t len, uint32_t seed) {
  const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  uint32_t h1 = seed;
  const int64_t nblocks = len / 4;
  for (int64_t i = 0; i < nblocks; ++i) {
    uint32_t k1 = (uint32_t)data[4 * i] | ((uint32_t)data[4 * i + 1] << 8) | ((uint32_t)data[4 * i + 2] << 16) |
                  ((uint32_t)data[4 * i + 3] << 24);
    k1 *= c1; k1 = o3s_rotl32(k1, 15); k1 *= c2;
    h1 ^= k1; h1 = o3s_rotl32(h1, 13); h1 = h1 * 5 + 0xe6546b64u;
  }
  const uint8_t* tail = data + nblocks * 4;
  uint32_t k1 = 0;
  switch (len & 3) {
    case 3: k1 ^= (uint32_t)tail[2] << 16; [[fallthrough]];
    case 2: k1 ^= (uint32_t)tail[1] << 8; [[fallthrough]];
    case 1: k1 ^= tail[0]; k1 *= c1; k1 = o3s_rotl32(k1, 15); k1 *= c2; h1 ^= k1;
  }
  h1 ^= (uint32_t)len;
  h1 ^= h1 >> 16; h1 *= 0x85ebca6bu; h1 ^= h1 >> 13; h1 *= 0xc2b2ae35u; h1 ^= h1 >> 16;
  return h1;
}
