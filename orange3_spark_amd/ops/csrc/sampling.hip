// Counter-hash random draws keyed on (seed, stream, global row) (gfx950).  Replaces the
// ~15 int64 torch passes per draw of ops/sampling.py::uniform on device tensors --
// Spark's per-partition seeded samplers (DataFrame.sample, RandomForest bootstrap,
// k-means|| oversampling, tree split-candidate sampling) made partition-invariant.
// Bitwise the same values as the torch path (common.h::hash_uniform).
#include "common.h"

using namespace o3s;

namespace {

// mode 0: out_f64[i] = U(row_i); mode 1: out_u8[i] = U(row_i) < p (Bernoulli mask).
// Rows: rows[i] if rows != null, else row0 + i.
__global__ __launch_bounds__(256) void hash_uniform_kernel(const int64_t* __restrict__ rows, int64_t row0, int64_t n,
                                                           uint32_t seed, uint32_t stream, int mode, double p,
                                                           double* __restrict__ out_f64, uint8_t* __restrict__ out_u8) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const int64_t r = rows ? rows[i] : row0 + i;
    const double u = hash_uniform(seed, stream, r);
    if (mode == 0) out_f64[i] = u;
    else out_u8[i] = u < p ? 1 : 0;
  }
}

}  // namespace

O3S_API int o3s_hash_uniform(const int64_t* rows, int64_t row0, int64_t n, uint32_t seed, uint32_t stream, int mode,
                             double p, double* out_f64, uint8_t* out_u8, hipStream_t st) {
  if (n <= 0) return 0;
  if ((mode == 0 && !out_f64) || (mode == 1 && !out_u8) || mode < 0 || mode > 1) return -1;
  const int64_t blocks = (n + 255) / 256;
  const unsigned grid = (unsigned)(blocks < 8192 ? blocks : 8192);
  hipLaunchKernelGGL(hash_uniform_kernel, dim3(grid), dim3(256), 0, st, rows, row0, n, seed, stream, mode, p, out_f64,
                     out_u8);
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_PRELOAD(sampling)
