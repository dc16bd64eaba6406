// Sparse (CSR) generalized-linear passes (gfx950): LogisticRegression / LinearSVC /
// LinearRegression on HashingTF / CountVectorizer features without densifying.
//
// Spark's LogisticAggregator iterates over the ACTIVE entries of each sparse instance
// (reached through the Classification widget -> fit, spark_ml_estimator.py:22); this is
// the same computation, split in two deterministic passes over this rank's rows:
//
//  * csr_glm_kernel: 8 lanes per CSR row gather coef[idx] for the row's entries
//    (coalesced over the entries, the coefficient vector lives in L2), fold the margin
//    with DPP-free xor shuffles, apply the loss, write the residual r_i (or, in margin
//    mode, the margin) and accumulate (sum r, loss, weight) in registers -> one fp32 slab
//    row per block (no atomics; the host sums the slab).
//  * csc_piece_kernel + csc_combine_kernel: the gradient X^T r over a CSC copy built
//    once per fit; every column is cut into pieces of <= kPiece entries, 8 lanes reduce a
//    piece (r gathered by row), and each column sums its pieces in order in fp64 -- a
//    long (frequent-term) column is spread over many waves yet the sum is bitwise
//    reproducible.  The same pair computes the column moments (sum w x, sum w x^2).
#include "common.h"

using namespace o3s;

namespace {

constexpr int kPiece = 256;     // CSC entries per piece
constexpr int kGroup = 8;       // lanes per row / piece

__device__ __forceinline__ float group8_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v;
}

__device__ __forceinline__ float softplusf(float m) {      // log(1 + e^m), stable
  return fmaxf(m, 0.f) + log1pf(expf(-fabsf(m)));
}

// LOSS: 0 logistic, 1 hinge, 2 squared, -1 margin only (out = margin).
template <int LOSS>
__global__ __launch_bounds__(256) void csr_glm_kernel(const int64_t* __restrict__ indptr,
                                                      const int32_t* __restrict__ idx,
                                                      const float* __restrict__ val, int64_t n,
                                                      const float* __restrict__ coef, float intercept,
                                                      const float* __restrict__ y, const float* __restrict__ w,
                                                      float* __restrict__ out, float* __restrict__ slab) {
  const int g = threadIdx.x & (kGroup - 1);
  const int64_t rows_per_block = 256 / kGroup;
  float sr = 0.f, sl = 0.f, sw = 0.f;
  for (int64_t row = (int64_t)blockIdx.x * rows_per_block + threadIdx.x / kGroup; row < n;
       row += (int64_t)gridDim.x * rows_per_block) {
    const int64_t p0 = indptr[row], p1 = indptr[row + 1];
    float s = 0.f;
    for (int64_t p = p0 + g; p < p1; p += kGroup) s = fmaf(val[p], coef[idx[p]], s);
    const float m = group8_sum(s) + intercept;
    if (LOSS < 0) {
      if (g == 0) out[row] = m;
      continue;
    }
    const float yi = y[row], wi = w ? w[row] : 1.f;
    float r, l;
    if (LOSS == 0) {
      r = (1.f / (1.f + expf(-m)) - yi) * wi;
      l = wi * (softplusf(m) - yi * m);
    } else if (LOSS == 1) {
      const float sgn = 2.f * yi - 1.f, mg = 1.f - sgn * m;
      const float act = mg > 0.f ? 1.f : 0.f;
      r = -sgn * wi * act;
      l = wi * mg * act;
    } else {
      const float e = m - yi;
      r = e * wi;
      l = 0.5f * wi * e * e;
    }
    if (g == 0) {
      out[row] = r;
      sr += r; sl += l; sw += wi;
    }
  }
  if (LOSS < 0) return;
  // fixed-order block reduction of (sum r, loss, weight) -> slab[block][3]
  __shared__ float red[3][256];
  red[0][threadIdx.x] = sr; red[1][threadIdx.x] = sl; red[2][threadIdx.x] = sw;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off)
      for (int q = 0; q < 3; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x < 3) slab[(int64_t)blockIdx.x * 3 + threadIdx.x] = red[threadIdx.x][0];
}

// piece p covers CSC entries [plo[p], plo[p] + pcnt[p]); psum[p] = sum r[row] * val (val^2 if SQ)
template <bool SQ>
__global__ __launch_bounds__(256) void csc_piece_kernel(const int64_t* __restrict__ plo,
                                                        const int32_t* __restrict__ pcnt, int64_t npieces,
                                                        const int32_t* __restrict__ rows,
                                                        const float* __restrict__ val, const float* __restrict__ r,
                                                        float* __restrict__ psum) {
  const int g = threadIdx.x & (kGroup - 1);
  const int64_t p = (int64_t)blockIdx.x * (256 / kGroup) + threadIdx.x / kGroup;
  if (p >= npieces) return;                      // whole 8-lane groups exit together
  const int64_t a = plo[p], b = a + pcnt[p];
  float s = 0.f;
  for (int64_t k = a + g; k < b; k += kGroup) {
    const float v = val[k];
    s = fmaf(SQ ? v * v : v, r ? r[rows[k]] : 1.f, s);
  }
  s = group8_sum(s);
  if (g == 0) psum[p] = s;
}

// out[c] = sum of pieces [cp[c], cp[c+1]) in order (fp64)
__global__ __launch_bounds__(256) void csc_combine_kernel(const int64_t* __restrict__ cp, int64_t d,
                                                          const float* __restrict__ psum, double* __restrict__ out) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= d) return;
  double s = 0.0;
  for (int64_t q = cp[c]; q < cp[c + 1]; ++q) s += (double)psum[q];
  out[c] = s;
}

}  // namespace

// mode: LOSS (0 logistic, 1 hinge, 2 squared) or -1 (margins into out).  slab: [grid][3].
O3S_API int o3s_csr_glm(int mode, const int64_t* indptr, const int32_t* idx, const float* val, int64_t n,
                        const float* coef, float intercept, const float* y, const float* w, float* out, float* slab,
                        int grid, hipStream_t st) {
  if (n <= 0) return 0;
  if (grid <= 0 || mode < -1 || mode > 2 || (mode >= 0 && (!y || !slab))) return -1;
#define O3S_CG(M)                                                                                     \
  hipLaunchKernelGGL((csr_glm_kernel<M>), dim3(grid), dim3(256), 0, st, indptr, idx, val, n, coef, intercept, y, \
                     w, out, slab);
  switch (mode) {
    case -1: O3S_CG(-1) break;
    case 0: O3S_CG(0) break;
    case 1: O3S_CG(1) break;
    default: O3S_CG(2) break;
  }
#undef O3S_CG
  O3S_CHECK_LAUNCH();
  return 0;
}

// out[c] = sum over column c's CSC entries of r[row] * val (val^2 when sq; r may be null = 1).
O3S_API int o3s_csc_colsum(const int64_t* plo, const int32_t* pcnt, int64_t npieces, const int64_t* col_pieces,
                           int64_t d, const int32_t* rows, const float* val, const float* r, int sq, float* psum,
                           double* out, hipStream_t st) {
  if (d <= 0) return 0;
  if (npieces > 0) {
    const dim3 g((unsigned)((npieces + 31) / 32));
    if (sq)
      hipLaunchKernelGGL(csc_piece_kernel<true>, g, dim3(256), 0, st, plo, pcnt, npieces, rows, val, r, psum);
    else
      hipLaunchKernelGGL(csc_piece_kernel<false>, g, dim3(256), 0, st, plo, pcnt, npieces, rows, val, r, psum);
    O3S_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(csc_combine_kernel, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, st, col_pieces, d, psum,
                     out);
  O3S_CHECK_LAUNCH();
  return 0;
}

// CSC piece size used by the host planner.
O3S_API int o3s_csc_piece() { return kPiece; }

O3S_PRELOAD(sparse)
