// Decision-tree histogram build (gfx950): DecisionTree / RandomForest / GBT.
//
// Replaces Spark's per-level DTStatsAggregator pass (binned features -> per (node,
// feature, bin) label statistics, reduced with reduceByKey; reached through the
// Classification/Regression widgets -> fit, orangecontrib/spark/base/spark_ml_estimator.py:22).
//
// Data layout: binned features uint8 [n][F] (row-major, one 64-B line per row at F=64),
// rows grouped by tree node through a permutation `order` (the engine re-partitions it
// after every level), so a work item = one contiguous run of rows of ONE node.
//
// LDS-privatised histograms with NO atomics and NO bank conflicts: lane (rs, f) of a
// wave owns feature f of row-slot rs, so each lane writes only its own columns of an LDS
// image laid out [rs][bin][stat][f] (f fastest: 64 lanes -> 64 banks), and every wave
// has its own image.  At the end the block sums its waves' images in a fixed order
// and writes ONE fp32 slab row per work item; the engine sums slab rows per node in a
// fixed order (deterministic).
//
// Stat modes: REG (S = 3: w, w*y, w*y^2 -- variance impurity, GBT residual trees) and
// CLS (S = #classes: weighted class counts -- gini/entropy).
#include "common.h"

using namespace o3s;

namespace {

constexpr int kHistWaves = 4;
constexpr int kHistThreads = kHistWaves * kWave;

// FP: features per row-slot (power of 2, <= 64); RS = 64 / FP row-slots per wave.
template <int FP, bool CLS>
__global__ __launch_bounds__(kHistThreads) void tree_hist_kernel(
    const uint8_t* __restrict__ bins, int F, int fg0, int B, int S, const int32_t* __restrict__ order,
    const float* __restrict__ y, const float* __restrict__ w, const int64_t* __restrict__ item_lo,
    const int64_t* __restrict__ item_hi, float* __restrict__ slab, int64_t slab_stride) {
  constexpr int RS = kWave / FP;
  extern __shared__ __attribute__((aligned(16))) float hist[];   // [wave][rs][B][S][FP] (+pad)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int rs = lane / FP, f = lane % FP;
  const int region = B * S * FP + 16;                             // +16: rs-regions on distinct banks
  const int per_wave = RS * region;
  float* my = hist + wid * per_wave + rs * region;
  for (int i = threadIdx.x; i < kHistWaves * per_wave; i += kHistThreads) hist[i] = 0.f;
  __syncthreads();
  const int fcol = fg0 + f;
  const bool fok = fcol < F;
  const int64_t lo = item_lo[blockIdx.x], hi = item_hi[blockIdx.x];
  // rows of the item are dealt round-robin to (wave, row-slot) pairs, 4 rows in flight
  constexpr int U = 4;
  const int64_t stride = (int64_t)kHistWaves * RS;
  for (int64_t p0 = lo + wid * RS + rs; p0 < hi; p0 += stride * U) {
    int b[U];
    float yy[U], ww[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = p0 + u * stride;
      ok[u] = p < hi;
      const int64_t pc = ok[u] ? p : lo;
      const int64_t row = order[pc];
      b[u] = fok ? bins[row * F + fcol] : 0;
      yy[u] = y[row];
      ww[u] = w ? w[row] : 1.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!(ok[u] && fok)) continue;
      float* cell = my + b[u] * S * FP + f;
      if (CLS) {
        cell[(int)yy[u] * FP] += ww[u];
      } else {
        cell[0] += ww[u];
        cell[FP] += ww[u] * yy[u];
        cell[2 * FP] += ww[u] * yy[u] * yy[u];
      }
    }
  }
  __syncthreads();
  // fixed-order block reduction -> slab[item][f][b][s] (features of this group only)
  float* out = slab + (int64_t)blockIdx.x * slab_stride;
  const int cells = FP * B * S;
  for (int i = threadIdx.x; i < cells; i += kHistThreads) {
    const int ff = i / (B * S), rem = i % (B * S);
    const int bb = rem / S, ss = rem % S;
    if (fg0 + ff >= F) continue;
    float acc = 0.f;
    for (int q = 0; q < kHistWaves; ++q)
      for (int r = 0; r < RS; ++r) acc += hist[q * per_wave + r * region + (bb * S + ss) * FP + ff];
    out[((int64_t)(fg0 + ff) * B + bb) * S + ss] = acc;
  }
}

}  // namespace

// Shared-memory bytes needed for (F-group width fp, B bins, S stats); 0 if it cannot fit.
O3S_API int o3s_tree_hist_lds(int fp, int B, int S) {
  const int RS = 64 / fp;
  const int64_t bytes = (int64_t)kHistWaves * RS * (B * S * fp + 16) * 4;
  return bytes <= 160 * 1024 ? (int)bytes : 0;
}

// One launch per feature group of 64: items = contiguous position ranges of `order`.
// slab: [n_items][F*B*S] fp32 (every cell written).  cls: 0 = REG (S must be 3), 1 = CLS.
O3S_API int o3s_tree_hist(const uint8_t* bins, int64_t n, int F, int B, int S, int cls, const int32_t* order,
                          const float* y, const float* w, const int64_t* item_lo, const int64_t* item_hi,
                          int n_items, float* slab, hipStream_t st) {
  if (n_items <= 0) return 0;
  if (!cls && S != 3) return -1;
  int fp = 1;
  while (fp < F && fp < 64) fp <<= 1;
  if (fp < 4) fp = 4;
  const int lds = o3s_tree_hist_lds(fp, B, S);
  if (lds == 0) return -2;
  const int64_t stride = (int64_t)F * B * S;
  for (int fg0 = 0; fg0 < F; fg0 += fp) {
#define O3S_TH(FPV)                                                                                     \
  if (fp == FPV) {                                                                                      \
    if (cls)                                                                                            \
      hipLaunchKernelGGL((tree_hist_kernel<FPV, true>), dim3(n_items), dim3(kHistThreads), lds, st, bins, \
                         F, fg0, B, S, order, y, w, item_lo, item_hi, slab, stride);                    \
    else                                                                                                \
      hipLaunchKernelGGL((tree_hist_kernel<FPV, false>), dim3(n_items), dim3(kHistThreads), lds, st, bins, \
                         F, fg0, B, S, order, y, w, item_lo, item_hi, slab, stride);                    \
  }
    O3S_TH(4) O3S_TH(8) O3S_TH(16) O3S_TH(32) O3S_TH(64)
#undef O3S_TH
    O3S_CHECK_LAUNCH();
  }
  (void)n;
  return 0;
}
