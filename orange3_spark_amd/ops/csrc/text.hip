// HashingTF / FeatureHasher term hashing on device (gfx950).
//
// Replaces the per-row term hashing of Spark's HashingTF.transform (reached through the
// Feature widget, orangecontrib/spark/widgets/ml/spark_ml_feature.py:15).  Input is a
// device string column as (offsets, bytes); one thread hashes one term
// (MurmurHash3_x86_32 of its UTF-8 bytes, seed 42), then maps it to a bucket with
// Spark's nonNegativeMod.  Device token columns go straight to CSR per document
// (hashing_tf_*_kernel below: one wave per document, no global sort).
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

// ---------------------------------------------------------------------------------
// HashingTF -> CSR per document (Spark HashingTF.transform: per row, hash every term,
// nonNegativeMod numFeatures, count per bucket -> a sparse vector with sorted indices).
// No global sort: each document is one wave.
//   hashing_tf_small_kernel (<= 64 tokens: one token per lane) -- murmur3 + bucket, a
//     bitonic sort of the 64 keys across the wave (__shfl_xor), run starts by ballot,
//     ranks by popcount, run lengths from the next set bit;
//   hashing_tf_large_kernel (65..4096 tokens, listed by the caller) -- the same on a
//     per-wave LDS buffer (bitonic network in LDS, runs scanned 64 keys at a time, the
//     run start positions parked in the already-consumed key slots).
// Both write the row's unique buckets / counts at its token base (tmp, unique <= tokens)
// and nnz[d]; hashing_tf_compact_kernel moves them to the CSR once nnz is scanned.
// Documents with more than 4096 tokens get nnz = -2 (the caller's fallback).
constexpr int kTfLarge = 4096;

__device__ __forceinline__ int tf_bucket(const int64_t* ts, const int64_t* te, const uint8_t* bytes, int64_t t,
                                         uint32_t seed, int64_t nb) {
  const int64_t a = ts[t], b = te[t];
  const uint32_t h = o3s_murmur3_32(bytes + a, b - a, seed);
  const int64_t raw = (int64_t)(int32_t)h % nb;
  return (int)(raw < 0 ? raw + nb : raw);
}

__global__ __launch_bounds__(256) void hashing_tf_small_kernel(
    const int64_t* __restrict__ doc_offs, const int64_t* __restrict__ ts, const int64_t* __restrict__ te,
    const uint8_t* __restrict__ bytes, int64_t ndocs, uint32_t seed, int64_t nb, int32_t* __restrict__ tmp_idx,
    int32_t* __restrict__ tmp_cnt, int64_t* __restrict__ nnz) {
  const int64_t d = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (d >= ndocs) return;                       // wave-uniform
  const int lane = threadIdx.x & 63;
  const int64_t a = doc_offs[d];
  const int64_t n = doc_offs[d + 1] - a;
  if (n > 64) {
    if (lane == 0) nnz[d] = n > kTfLarge ? -2 : -1;
    return;
  }
  int key = 0x7fffffff;                         // padding sorts last
  if (lane < n) key = tf_bucket(ts, te, bytes, a + lane, seed, nb);
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int o = __shfl_xor(key, j, 64);
      const bool up = (lane & k) == 0, low = (lane & j) == 0;
      key = (low == up) ? min(key, o) : max(key, o);
    }
  const int prev = __shfl(key, lane > 0 ? lane - 1 : 0, 64);
  const bool start = lane < n && (lane == 0 || key != prev);
  const uint64_t mask = __ballot(start);
  if (start) {
    const int rank = __popcll(mask & ((1ull << lane) - 1));
    const uint64_t after = lane == 63 ? 0ull : mask >> (lane + 1);
    const int nxt = after ? lane + __ffsll((long long)after) : (int)n;
    tmp_idx[a + rank] = key;
    tmp_cnt[a + rank] = nxt - lane;
  }
  if (lane == 0) nnz[d] = __popcll(mask);
}

__global__ __launch_bounds__(256) void hashing_tf_large_kernel(
    const int64_t* __restrict__ doc_offs, const int64_t* __restrict__ ts, const int64_t* __restrict__ te,
    const uint8_t* __restrict__ bytes, const int64_t* __restrict__ docs, int64_t ndocs, uint32_t seed, int64_t nb,
    int32_t* __restrict__ tmp_idx, int32_t* __restrict__ tmp_cnt, int64_t* __restrict__ nnz) {
  __shared__ int sbuf[4][kTfLarge];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + w;
  if (q >= ndocs) return;
  const int64_t d = docs[q];
  const int64_t a = doc_offs[d];
  const int n = (int)(doc_offs[d + 1] - a);     // 65..kTfLarge (the caller's list)
  int* const s = sbuf[w];
  int P = 128;
  while (P < n) P <<= 1;
  // (the wave's LDS instructions run in order; the empty asm barriers keep the compiler from
  // moving a lane's load past another lane's store between network steps)
  for (int i = lane; i < P; i += 64) s[i] = i < n ? tf_bucket(ts, te, bytes, a + i, seed, nb) : 0x7fffffff;
  asm volatile("" ::: "memory");
  for (int k = 2; k <= P; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = lane; i < P; i += 64) {
        const int l = i ^ j;
        if (l > i) {
          const int x = s[i], y = s[l];
          if ((x > y) == ((i & k) == 0)) { s[i] = y; s[l] = x; }
        }
      }
      asm volatile("" ::: "memory");
    }
  // runs: starts (rank r -> its position parked in s[r], a slot whose key was consumed)
  // (the previous chunk's last key travels in a register: its slot may already hold a
  // parked start position)
  int nstart = 0, nend = 0, lastkey = 0;
  for (int c = 0; c < n; c += 64) {
    const int i = c + lane;
    const int key = i < n ? s[i] : 0;
    const int up = __shfl(key, lane > 0 ? lane - 1 : 0, 64);
    const int prev = lane > 0 ? up : lastkey;
    const int dn = __shfl(key, lane < 63 ? lane + 1 : 63, 64);
    const int next = lane < 63 ? dn : (i + 1 < n ? s[i + 1] : 0);
    lastkey = __shfl(key, 63, 64);
    const bool start = i < n && (i == 0 || key != prev);
    const bool end = i < n && (i + 1 == n || key != next);
    const uint64_t smask = __ballot(start), emask = __ballot(end);
    const uint64_t below = (1ull << lane) - 1;
    asm volatile("" ::: "memory");           // every lane's key reads before the parked writes
    if (start) {
      const int r = nstart + __popcll(smask & below);
      tmp_idx[a + r] = key;
      s[r] = i;
    }
    asm volatile("" ::: "memory");
    if (end) {
      const int r = nend + __popcll(emask & below);
      tmp_cnt[a + r] = i - s[r] + 1;
    }
    nstart += __popcll(smask);
    nend += __popcll(emask);
    asm volatile("" ::: "memory");
  }
  if (lane == 0) nnz[d] = nstart;
}

__global__ __launch_bounds__(256) void hashing_tf_compact_kernel(
    const int64_t* __restrict__ doc_offs, const int64_t* __restrict__ indptr, const int32_t* __restrict__ tmp_idx,
    const int32_t* __restrict__ tmp_cnt, int64_t ndocs, int binary, int32_t* __restrict__ out_idx,
    double* __restrict__ out_val) {
  const int64_t d = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (d >= ndocs) return;
  const int lane = threadIdx.x & 63;
  const int64_t a = doc_offs[d], o = indptr[d], m = indptr[d + 1] - o;
  for (int64_t i = lane; i < m; i += 64) {
    out_idx[o + i] = tmp_idx[a + i];
    out_val[o + i] = binary ? 1.0 : (double)tmp_cnt[a + i];
  }
}

}  // namespace

// HashingTF per-document CSR (see the kernels above).  pass 0: small kernel over every
// document; pass 1: large kernel over ``docs`` [ndocs]; pass 2: compaction into
// (out_idx, out_val) at ``indptr``.
O3S_API int o3s_hashing_tf(int pass, const int64_t* doc_offs, const int64_t* ts, const int64_t* te,
                           const uint8_t* bytes, const int64_t* docs, int64_t ndocs, uint32_t seed, int64_t nb,
                           int32_t* tmp_idx, int32_t* tmp_cnt, int64_t* nnz, const int64_t* indptr, int binary,
                           int32_t* out_idx, double* out_val, hipStream_t st) {
  if (ndocs <= 0) return 0;
  if (nb <= 0 || nb > 0x7fffffffll) return -1;
  const dim3 grid((unsigned)((ndocs + 3) / 4));
  if (pass == 0)
    hipLaunchKernelGGL(hashing_tf_small_kernel, grid, dim3(256), 0, st, doc_offs, ts, te, bytes, ndocs, seed, nb,
                       tmp_idx, tmp_cnt, nnz);
  else if (pass == 1)
    hipLaunchKernelGGL(hashing_tf_large_kernel, grid, dim3(256), 0, st, doc_offs, ts, te, bytes, docs, ndocs, seed,
                       nb, tmp_idx, tmp_cnt, nnz);
  else
    hipLaunchKernelGGL(hashing_tf_compact_kernel, grid, dim3(256), 0, st, doc_offs, indptr, tmp_idx, tmp_cnt, ndocs,
                       binary, out_idx, out_val);
  O3S_CHECK_LAUNCH();
  return 0;
}

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

O3S_PRELOAD(text)
