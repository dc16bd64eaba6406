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

// ---------------------------------------------------------------------------------
// Device Tokenizer (Spark semantics, ASCII columns): toLowerCase + split on every single
// whitespace char [ \t\n\v\f\r]; runs give empty tokens, trailing empties dropped, ""
// -> [""], all-whitespace -> [] (see host_text.cpp).  Input = an Arrow-layout string
// column (int64 offsets + UTF-8 bytes, straight from pyarrow's buffers).  One thread per
// document: pass 1 counts tokens, the caller scans the counts, pass 2 writes the
// lower-cased bytes and the token spans.
__device__ __forceinline__ bool tok_ws(uint8_t c) { return c == ' ' || (c >= 9 && c <= 13); }

__global__ void tokenize_count_kernel(const int64_t* __restrict__ offs, const uint8_t* __restrict__ bytes,
                                      int64_t ndocs, int64_t* __restrict__ counts) {
  const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= ndocs) return;
  const int64_t a = offs[d], b = offs[d + 1];
  int64_t c = 0, nws_before_last = 0, last = -1;
  for (int64_t i = a; i < b; ++i) {
    if (tok_ws(bytes[i])) ++c;
    else { last = i; nws_before_last = c; }
  }
  counts[d] = (a == b) ? 1 : (last < 0 ? 0 : nws_before_last + 1);
}

__global__ void tokenize_emit_kernel(const int64_t* __restrict__ offs, const uint8_t* __restrict__ bytes,
                                     int64_t ndocs, const int64_t* __restrict__ tok_base,
                                     uint8_t* __restrict__ out_bytes, int64_t* __restrict__ tok_start,
                                     int64_t* __restrict__ tok_end) {
  const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= ndocs) return;
  const int64_t a = offs[d], b = offs[d + 1];
  int64_t last = -1;
  for (int64_t i = a; i < b; ++i) {
    const uint8_t ch = bytes[i];
    out_bytes[i] = (ch >= 'A' && ch <= 'Z') ? (uint8_t)(ch + 32) : ch;
    if (!tok_ws(ch)) last = i;
  }
  int64_t k = tok_base[d];
  if (k == tok_base[d + 1]) return;               // no tokens (all whitespace, or a null row)
  if (a == b) { tok_start[k] = a; tok_end[k] = a; return; }
  if (last < 0) return;
  int64_t st = a;
  for (int64_t i = a; i <= last; ++i)
    if (tok_ws(bytes[i])) { tok_start[k] = st; tok_end[k] = i; ++k; st = i + 1; }
  tok_start[k] = st;
  tok_end[k] = last + 1;
}

// MurmurHash3 buckets of token spans [start, end) of a byte buffer (HashingTF over the
// device tokens, no re-packing).
__global__ void murmur3_span_kernel(const int64_t* __restrict__ starts, const int64_t* __restrict__ ends,
                                    const uint8_t* __restrict__ bytes, int64_t nterms, uint32_t seed,
                                    int64_t num_buckets, int64_t* __restrict__ bucket_out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nterms) return;
  const int64_t a = starts[t], b = ends[t];
  const uint32_t h = o3s_murmur3_32(bytes + a, b - a, seed);
  const int64_t raw = (int64_t)(int32_t)h % num_buckets;
  bucket_out[t] = raw < 0 ? raw + num_buckets : raw;
}

}  // namespace

// pass 0: counts[d] = #tokens of document d; pass 1: lower-cased bytes + spans (tok_base =
// [ndocs+1] prefix sums of the (possibly null-masked) counts).
O3S_API int o3s_tokenize(int pass, const int64_t* offs, const uint8_t* bytes, int64_t ndocs, int64_t* counts,
                         const int64_t* tok_base, uint8_t* out_bytes, int64_t* tok_start, int64_t* tok_end,
                         hipStream_t st) {
  if (ndocs <= 0) return 0;
  const dim3 grid((unsigned)((ndocs + 255) / 256));
  if (pass == 0)
    hipLaunchKernelGGL(tokenize_count_kernel, grid, dim3(256), 0, st, offs, bytes, ndocs, counts);
  else
    hipLaunchKernelGGL(tokenize_emit_kernel, grid, dim3(256), 0, st, offs, bytes, ndocs, tok_base, out_bytes,
                       tok_start, tok_end);
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_API int o3s_murmur3_spans(const int64_t* starts, const int64_t* ends, const uint8_t* bytes, int64_t nterms,
                              uint32_t seed, int64_t num_buckets, int64_t* bucket_out, hipStream_t st) {
  if (nterms <= 0) return 0;
  if (num_buckets <= 0) return -1;
  hipLaunchKernelGGL(murmur3_span_kernel, dim3((unsigned)((nterms + 255) / 256)), dim3(256), 0, st, starts, ends,
                     bytes, nterms, seed, num_buckets, bucket_out);
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_API int o3s_murmur3_terms(const int64_t* offs, const uint8_t* bytes, int64_t nterms, uint32_t seed,
                              int64_t num_buckets, int32_t* hash_out, int64_t* bucket_out, hipStream_t st) {
  if (nterms <= 0) return 0;
  hipLaunchKernelGGL(murmur3_bucket_kernel, dim3((unsigned)((nterms + 255) / 256)), dim3(256), 0, st, offs, bytes,
                     nterms, seed, num_buckets, hash_out, bucket_out);
  O3S_CHECK_LAUNCH();
  return 0;
}
