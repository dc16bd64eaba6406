// Evaluator kernels (gfx950): one streaming pass over the prediction columns each.
//
//   o3s_regression_stats : 7 fp64 sums {w, w e^2, w |e|, w y, w y^2, w p, w p^2} with
//                          e = p - y (RegressionEvaluator; rmse/mse/mae/r2/var).
//   o3s_confusion        : k x k weighted confusion matrix, rows = label, cols = prediction,
//                          privatised in LDS per block (MulticlassClassificationEvaluator).
//   o3s_score_hist       : per-class weighted histogram of a score over [lo, lo + span]
//                          in `bins` bins (BinaryClassificationEvaluator ROC / PR).
//
// The torch formulation of each is 6-12 separate elementwise/reduction launches that
// re-read the columns (and index_add over boolean-masked copies for the histogram);
// here each column is read once (coalesced, lane-consecutive rows), values are
// converted in registers, and the block results go to slab rows that a fixed-order
// reduction combines (deterministic; the histogram uses fp64 global atomics into
// 2 x bins cells -- unit weights give exact integer counts, so it is deterministic
// for the unweighted case Spark's evaluator uses by default).
//
// Column dtypes are passed as codes (0 = f32, 1 = f64, 2 = i64, 3 = i32); a null weight
// pointer means unit weights.  `pstride` lets the score come straight out of a
// [n, 2] rawPrediction matrix (column 1) without a strided copy.
#include "common.h"

namespace o3s {

__device__ __forceinline__ double ld_num(const void* p, int dt, int64_t i) {
  switch (dt) {
    case 0: return (double)reinterpret_cast<const float*>(p)[i];
    case 1: return reinterpret_cast<const double*>(p)[i];
    case 2: return (double)reinterpret_cast<const int64_t*>(p)[i];
    default: return (double)reinterpret_cast<const int32_t*>(p)[i];
  }
}

constexpr int kEvalThreads = 256;

__global__ __launch_bounds__(kEvalThreads) void regression_stats_kernel(
    const void* __restrict__ y, int ydt, const void* __restrict__ p, int pdt, const void* __restrict__ w, int wdt,
    int64_t n, double* __restrict__ slab) {
  double acc[7] = {0, 0, 0, 0, 0, 0, 0};
  const int64_t stride = (int64_t)gridDim.x * kEvalThreads;
  for (int64_t i = (int64_t)blockIdx.x * kEvalThreads + threadIdx.x; i < n; i += stride) {
    const double yy = ld_num(y, ydt, i), pp = ld_num(p, pdt, i);
    const double ww = w ? ld_num(w, wdt, i) : 1.0;
    const double e = pp - yy;
    acc[0] += ww;
    acc[1] += ww * e * e;
    acc[2] += ww * fabs(e);
    acc[3] += ww * yy;
    acc[4] += ww * yy * yy;
    acc[5] += ww * pp;
    acc[6] += ww * pp * pp;
  }
  __shared__ double red[kEvalThreads / kWave][7];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    double v = wave_sum_d(acc[j]);
    if (lane == 0) red[wv][j] = v;
  }
  __syncthreads();
  if (threadIdx.x < 7) {
    double v = 0;
#pragma unroll
    for (int k = 0; k < kEvalThreads / kWave; ++k) v += red[k][threadIdx.x];
    slab[(int64_t)blockIdx.x * 8 + threadIdx.x] = v;
  }
}

// LDS-privatised confusion matrix: k*k fp64 cells (k <= 64 -> 32 KB).  Lanes of a wave
// hitting the same cell serialise in the LDS atomic unit, which is fine: the number of
// distinct (label, prediction) pairs is small and cells are spread over 32 banks.
__global__ __launch_bounds__(kEvalThreads) void confusion_kernel(
    const void* __restrict__ y, int ydt, const void* __restrict__ p, int pdt, const void* __restrict__ w, int wdt,
    int64_t n, int k, double* __restrict__ slab) {
  extern __shared__ double cm[];
  const int kk = k * k;
  for (int c = threadIdx.x; c < kk; c += kEvalThreads) cm[c] = 0.0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * kEvalThreads;
  for (int64_t i = (int64_t)blockIdx.x * kEvalThreads + threadIdx.x; i < n; i += stride) {
    int a = (int)ld_num(y, ydt, i), b = (int)ld_num(p, pdt, i);
    a = min(max(a, 0), k - 1);
    b = min(max(b, 0), k - 1);
    const double ww = w ? ld_num(w, wdt, i) : 1.0;
    atomicAdd(&cm[a * k + b], ww);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < kk; c += kEvalThreads) slab[(int64_t)blockIdx.x * kk + c] = cm[c];
}

__global__ __launch_bounds__(kEvalThreads) void score_hist_kernel(
    const void* __restrict__ s, int sdt, int64_t pstride, const void* __restrict__ y, int ydt,
    const void* __restrict__ w, int wdt, int64_t n, double lo, double scale, int bins, double* __restrict__ hist) {
  const int64_t stride = (int64_t)gridDim.x * kEvalThreads;
  for (int64_t i = (int64_t)blockIdx.x * kEvalThreads + threadIdx.x; i < n; i += stride) {
    const double sc = ld_num(s, sdt, i * pstride);
    const double yy = ld_num(y, ydt, i);
    const double ww = w ? ld_num(w, wdt, i) : 1.0;
    int b = (int)((sc - lo) * scale);
    b = min(max(b, 0), bins - 1);
    // class 0 = positive (label > 0.5), 1 = negative
    atomicAdd(&hist[(yy > 0.5 ? 0 : bins) + b], ww);
  }
}

__global__ void slab_sum_kernel(const double* __restrict__ slab, int rows, int width, int ld, double* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= width) return;
  double v = 0;
  for (int r = 0; r < rows; ++r) v += slab[(int64_t)r * ld + c];
  out[c] = v;
}

}  // namespace o3s

using namespace o3s;

static int eval_grid(int64_t n) {
  int64_t g = (n + kEvalThreads * 8 - 1) / (kEvalThreads * 8);
  return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

// slab: >= grid * 8 doubles (grid = o3s_eval_grid(n)); out: 7 doubles.
O3S_API int o3s_eval_grid(int64_t n) { return eval_grid(n); }

O3S_API int o3s_regression_stats(const void* y, int ydt, const void* p, int pdt, const void* w, int wdt, int64_t n,
                                 double* slab, double* out, hipStream_t st) {
  if (n < 0 || !y || !p || !slab || !out) return -1;
  const int g = eval_grid(n);
  regression_stats_kernel<<<g, kEvalThreads, 0, st>>>(y, ydt, p, pdt, w, wdt, n, slab);
  slab_sum_kernel<<<1, 64, 0, st>>>(slab, g, 7, 8, out);
  return (int)hipGetLastError();
}

// slab: >= grid * k * k doubles; out: k * k doubles.  k <= 64.
O3S_API int o3s_confusion(const void* y, int ydt, const void* p, int pdt, const void* w, int wdt, int64_t n, int k,
                          double* slab, double* out, hipStream_t st) {
  if (n < 0 || k < 1 || k > 64 || !y || !p || !slab || !out) return -1;
  const int g = eval_grid(n);
  confusion_kernel<<<g, kEvalThreads, (size_t)k * k * sizeof(double), st>>>(y, ydt, p, pdt, w, wdt, n, k, slab);
  const int kk = k * k;
  slab_sum_kernel<<<(kk + 255) / 256, 256, 0, st>>>(slab, g, kk, kk, out);
  return (int)hipGetLastError();
}

// hist: 2 * bins doubles, zeroed by the caller (positives first, then negatives).
O3S_API int o3s_score_hist(const void* s, int sdt, int64_t pstride, const void* y, int ydt, const void* w, int wdt,
                           int64_t n, double lo, double span, int bins, double* hist, hipStream_t st) {
  if (n < 0 || bins < 1 || !s || !y || !hist || !(span > 0)) return -1;
  const double scale = (double)(bins - 1) / span;
  score_hist_kernel<<<eval_grid(n), kEvalThreads, 0, st>>>(s, sdt, pstride, y, ydt, w, wdt, n, lo, scale, bins, hist);
  return (int)hipGetLastError();
}

O3S_PRELOAD(eval)
