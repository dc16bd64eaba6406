// Per-bin row sums: out[b] = [sum_{i: bin_i = b} w_i x_i (D) | sum w_i | sum w_i ||x_i||^2]
// for a handful of bins -- the sufficient statistics of bisecting k-means splits, GMM /
// clustering-evaluator cluster sums, class sums, etc.
//
// torch's index_add_ on a few bins serialises on global fp64 atomics (every row of a
// 4M x 64 table adding into the same 64 addresses: minutes), and a one-hot GEMM with a
// tiny output and a 4M-deep K runs on one or two workgroups.  Here each wave owns a
// private fp64 copy of the bins in LDS: it walks its rows one at a time (the row's bin is
// wave-uniform, a scalar load), every lane adds its columns (no two lanes share an
// address, no atomics), the row's ||x||^2 is a wave sum.  Waves then fold into one
// slab row per block and glm-style fixed-order fp64 finishing sums the slabs: the result
// is deterministic for a given grid.
#include "common.h"

using namespace o3s;

namespace {

constexpr int kBsWaves = 4;
constexpr int kBsThreads = kBsWaves * kWave;

template <typename T>
__device__ __forceinline__ double load_val(const T* p);
template <>
__device__ __forceinline__ double load_val<double>(const double* p) { return *p; }
template <>
__device__ __forceinline__ double load_val<float>(const float* p) { return (double)*p; }
template <>
__device__ __forceinline__ double load_val<uint16_t>(const uint16_t* p) { return (double)bf16_to_f32(*p); }

// CPL columns per lane (D <= 64 CPL); W = stats per bin (D + 2), padded.
template <typename T, int CPL>
__global__ __launch_bounds__(kBsThreads) void bin_sums_kernel(const T* __restrict__ X, int64_t n, int64_t ldx,
                                                              int D, const int64_t* __restrict__ bins,
                                                              int64_t bin0, const float* __restrict__ w,
                                                              int nbins,
                                                              double* __restrict__ partial, int pstride) {
  extern __shared__ double acc[];                      // [kBsWaves][nbins][pstride_b]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int W = D + 2;
  for (int i = threadIdx.x; i < kBsWaves * nbins * W; i += kBsThreads) acc[i] = 0.0;
  __syncthreads();
  double* mine = acc + (int64_t)wid * nbins * W;
  const int64_t per = (n + (int64_t)gridDim.x * kBsWaves - 1) / ((int64_t)gridDim.x * kBsWaves);
  const int64_t r0 = ((int64_t)blockIdx.x * kBsWaves + wid) * per;
  const int64_t r1 = r0 + per < n ? r0 + per : n;
  for (int64_t row = r0; row < r1; ++row) {
    const int64_t bv = bins[row] - bin0;
    const int b = __builtin_amdgcn_readfirstlane((bv < 0 || bv >= nbins) ? -1 : (int)bv);
    if (b < 0) continue;                               // rows outside this bin range are skipped
    const double wr = w ? (double)w[row] : 1.0;
    double sq = 0.0;
    double* dst = mine + (int64_t)b * W;
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int c = lane + 64 * q;
      if (c < D) {
        const double v = load_val<T>(X + row * ldx + c);
        sq = fma(v, v, sq);
        dst[c] += wr * v;
      }
    }
    const double tot = wave_sum_d(sq);
    if (lane == 0) {
      dst[D] += wr;
      dst[D + 1] += wr * tot;
    }
  }
  __syncthreads();
  // fold the waves (fixed order) into this block's slab row
  for (int i = threadIdx.x; i < nbins * W; i += kBsThreads) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < kBsWaves; ++q) s += acc[(int64_t)q * nbins * W + i];
    partial[(int64_t)blockIdx.x * pstride + i] = s;
  }
}

// out[i] = sum over blocks of partial[b][i], fixed order
__global__ __launch_bounds__(256) void bin_sums_finish_kernel(const double* __restrict__ partial, int nblocks,
                                                              int pstride, int ncols, double* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= ncols) return;
  double s = 0.0;
  for (int b = 0; b < nblocks; ++b) s += partial[(int64_t)b * pstride + i];
  out[i] = s;
}

}  // namespace

// dtype: 0 = fp32, 1 = bf16, 2 = fp64.  bins: int64 [n]; rows whose bin - bin0 is
// outside [0, nbins) are skipped (callers cover many bins in groups of nbins);
// w: fp32 [n] or null.  partial: fp64 [grid][nbins * (D + 2)]; out: fp64 [nbins][D + 2].
O3S_API int o3s_bin_sums(const void* X, int dtype, int64_t n, int64_t ldx, int D, const int64_t* bins,
                         int64_t bin0, const float* w, int nbins, double* partial, int grid, double* out, hipStream_t st) {
  const int W = D + 2;
  const size_t lds = sizeof(double) * (size_t)kBsWaves * nbins * W;
  if (D < 1 || D > 256 || nbins < 1 || grid < 1 || lds > 64 * 1024) return -1;
  const int cpl = (D + 63) / 64;
  const int pstride = nbins * W;
  if (n > 0) {
#define O3S_BS(T, C)                                                                                          \
  hipLaunchKernelGGL((bin_sums_kernel<T, C>), dim3(grid), dim3(kBsThreads), lds, st, (const T*)X, n, ldx, D, bins, \
                     bin0, w, nbins, partial, pstride)
    if (dtype == 0) {
      if (cpl == 1) O3S_BS(float, 1); else if (cpl == 2) O3S_BS(float, 2); else if (cpl == 3) O3S_BS(float, 3);
      else O3S_BS(float, 4);
    } else if (dtype == 1) {
      if (cpl == 1) O3S_BS(uint16_t, 1); else if (cpl == 2) O3S_BS(uint16_t, 2);
      else if (cpl == 3) O3S_BS(uint16_t, 3); else O3S_BS(uint16_t, 4);
    } else if (dtype == 2) {
      if (cpl == 1) O3S_BS(double, 1); else if (cpl == 2) O3S_BS(double, 2); else if (cpl == 3) O3S_BS(double, 3);
      else O3S_BS(double, 4);
    } else {
      return -1;
    }
#undef O3S_BS
  } else {
    if (hipMemsetAsync(partial, 0, sizeof(double) * pstride * (size_t)grid, st) != hipSuccess) return -1;
  }
  O3S_CHECK_LAUNCH();
  hipLaunchKernelGGL(bin_sums_finish_kernel, dim3((pstride + 255) / 256), dim3(256), 0, st, partial, grid, pstride,
                     pstride, out);
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_PRELOAD(binsum)
