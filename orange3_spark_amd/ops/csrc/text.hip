// HashingTF / FeatureHasher term hashing on device (gfx950).
//
// Replaces the per-row term hashing of Spark's HashingTF.transform (reached through the
// Feature widget, orangecontrib/spark/widgets/ml/spark_ml_feature.py:15).  Input is a
// device string column as (offsets, bytes); one thread hashes one term
// (MurmurHash3_x86_32 of its UTF-8 bytes, seed 42), then maps it to a bucket with
// Spark's nonNegativeMod.  Term -> (row, bucket) counting into CSR is done by the caller
// with a device sort/unique (terms per row are few; the hash is the hot part).
#include "common.h"
#include "murmur3.h"

namespace {

__global__ void murmur3_bucket_kernel(const int64_t* __restrict__ offs, const uint8_t* __restrict__ bytes,
                                      int64_t nterms, uint32_t seed, int64_t num_buckets,
                                      int32_t* __restrict__ hash_out, int64_t* __restrict__ bucket_out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nterms) return;
  const int64_t a = offs[t], b = offs[t + 1];
  const uint32_t h = o3s_murmur3_32(bytes + a, b - a, seed);
  if (hash_out) hash_out[t] = (int32_t)h;
  if (bucket_out && num_buckets > 0) {
    const int64_t raw = (int64_t)(int32_t)h % num_buckets;       // Spark Utils.nonNegativeMod
    bucket_out[t] = raw < 0 ? raw + num_buckets : raw;
  }
}

}  // namespace

O3S_API int o3s_murmur3_terms(const int64_t* offs, const uint8_t* bytes, int64_t nterms, uint32_t seed,
                              int64_t num_buckets, int32_t* hash_out, int64_t* bucket_out, hipStream_t st) {
  if (nterms <= 0) return 0;
  hipLaunchKernelGGL(murmur3_bucket_kernel, dim3((unsigned)((nterms + 255) / 256)), dim3(256), 0, st, offs, bytes,
                     nterms, seed, num_buckets, hash_out, bucket_out);
  O3S_CHECK_LAUNCH();
  return 0;
}
