// Diagnostic: the random-row gather rate of the device (tools/bench_gather.py).  The exact
// ALS solves gather one factor row (R fp32 = 512 B at rank 128) per rating, two sides per
// iteration -- 1 TB per iteration of the 50M x 5M x 1B config -- so this rate is the floor
// of an ALS iteration.  Each wave gathers the listed rows of an [n][R] fp32 table, 64 / (R/4)
// rows per load instruction (16 B per lane), UNR loads in flight, and folds them into one
// float4 per lane (written per wave so nothing is optimised away).
#include "common.h"

using namespace o3s;

namespace {
typedef float float4v __attribute__((ext_vector_type(4)));

template <int R, int UNR>
__global__ __launch_bounds__(256) void gather_probe_kernel(const float* __restrict__ F, const int32_t* __restrict__ idx,
                                                           int64_t nidx, float* __restrict__ out) {
  constexpr int LPR = R / 4;                   // lanes per row
  constexpr int RPI = 64 / LPR;                // rows per load instruction
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * 256) >> 6;
  const int sub = lane / LPR, col = lane % LPR;
  float4v acc = {0.f, 0.f, 0.f, 0.f};
  const int64_t per = RPI * UNR;               // rows per wave per round
  for (int64_t base = wave * per; base < nidx; base += nwaves * per) {
    float4v v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t j = base + (int64_t)u * RPI + sub;
      const int32_t r = idx[j < nidx ? j : nidx - 1];
      v[u] = *reinterpret_cast<const float4v*>(F + (int64_t)r * R + 4 * col);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc += v[u];
  }
  reinterpret_cast<float4v*>(out)[wave * 64 + lane] = acc;
}
}  // namespace

// out: [grid * 4][64] float4 (per-wave sums).  R: 64 or 128.
O3S_API int o3s_gather_probe(const float* F, int R, const int32_t* idx, int64_t nidx, int grid, float* out,
                             hipStream_t st) {
  if (nidx <= 0 || grid <= 0) return -1;
  if (R == 128)
    hipLaunchKernelGGL((gather_probe_kernel<128, 8>), dim3(grid), dim3(256), 0, st, F, idx, nidx, out);
  else if (R == 64)
    hipLaunchKernelGGL((gather_probe_kernel<64, 8>), dim3(grid), dim3(256), 0, st, F, idx, nidx, out);
  else
    return -2;
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_PRELOAD(probe)
