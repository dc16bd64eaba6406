// Exact ALS solves on gfx950: every row's normal equations solved directly (Spark's
// per-row Cholesky, reached through the Recommendation widget -> ALS.fit,
// orangecontrib/spark/widgets/ml/spark_ml_recommendation.py:15), never materialising the
// rank x rank systems in HBM.
//
//   A_u = G + Y_u^T W_u Y_u + lam_u I,   b_u = Y_u^T c_u,   x_u = A_u^{-1} b_u
//
// (implicit: G = Y^T Y, W = diag(alpha |r|), c = (1 + alpha |r|)[r > 0]; explicit: G = 0,
// W = I, c = r; lam_u = regParam * n_u).  Two kernels by row length n_u:
//
// * als_wood_kernel (n_u <= 32, lam_u > 0; the user side of the ALS config averages 20
//   ratings): with G = Q diag(e) Q^T (one eigendecomposition per half-iteration, host) and
//   P = Y_u Q (n x R), Woodbury gives
//       x_u = Q D P^T z,   D = diag(1 / (e + lam_u)),   S z = W^{-1} c,
//       S = W^{-1} + P D P^T   (n x n, SPD)
//   so the only factorisation is an n x n Cholesky -- no 128-step pivot chain per row.
//   One wave per row: P lives in registers (lane l holds columns l, l + 64 as float2 ->
//   v_pk_fma), S in LDS (lane i owns row i), triangular solves broadcast with readlane.
//   Cost ~ n R^2 FMA per row (the P transform), the same as forming the Gram matrix.
// * als_dense_kernel (longer rows: the item side, ~200 ratings): one block per row; the
//   Gram matrix accumulates in registers (8 x 8 tile per thread) from factor rows staged
//   through LDS, then A sits in LDS for a blocked right-looking Cholesky (8-wide panels:
//   wave 0 factors the diagonal block and the panel, all threads do the trailing update
//   over the lower triangle), followed by the two triangular solves.
//
// Both write x_u straight into the factor table.  fp32 throughout (the Gram / S sums are
// short: n_u terms).
#include "common.h"

using namespace o3s;

namespace {

constexpr int kNW = 32;   // Woodbury path: rows with at most this many ratings
constexpr int kWW = 2;    // waves (rows) per Woodbury block

__device__ __forceinline__ float rl(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}

template <int R, bool IMPL>
__global__ __launch_bounds__(kWW * 64) void als_wood_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ cols, const float* __restrict__ w,
    const float* __restrict__ b, const float* __restrict__ F, const float* __restrict__ Q,
    const float* __restrict__ QT, const float* __restrict__ eig, const float* __restrict__ lam,
    const int32_t* __restrict__ rows, int64_t nlist, float* __restrict__ X) {
  static_assert(R % 32 == 0 && R <= 128, "rank must be a multiple of 32, at most 128");
  constexpr int RV = (R + 63) / 64;              // columns per lane (1 or 2)
  __shared__ float sY[kWW][kNW][R];              // staged factor rows (IMPL)
  __shared__ float sS[kWW][kNW][kNW + 1];        // S, then its Cholesky factor (lower)
  __shared__ float sv[kWW][R];                   // y = D u, for x = Q y
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t li = (int64_t)blockIdx.x * kWW + wv;
  if (li >= nlist) return;                       // wave-uniform; the kernel has no block barrier
  const int64_t u = rows[li];
  const int64_t p0 = indptr[u];
  const int n = (int)(indptr[u + 1] - p0);       // <= kNW (host routing)
  const float lu = lam[u];
  float (*S)[kNW + 1] = sS[wv];

  // per-rating W^{-1} c (lane i < n holds rating i); w = 0 (r = 0 implicit): no term
  float t = 0.f, winv = 0.f;
  if (lane < n) {
    const float wi = w[p0 + lane], bi = b[p0 + lane];
    winv = wi > 0.f ? 1.f / wi : 1e30f;
    t = wi > 0.f ? bi * winv : 0.f;
  }
  float dinv[RV];
#pragma unroll
  for (int k = 0; k < RV; ++k) {
    const int d = lane + 64 * k;
    dinv[k] = d < R ? 1.f / ((IMPL ? eig[d] : 0.f) + lu) : 0.f;
  }

  // P = Y_u Q (implicit) or Y_u (explicit), rows of P in registers: acc[i] = (P[i][lane],
  // P[i][lane + 64]).  Every loop over rows is unrolled to kNW with a uniform guard, so
  // acc stays in registers (a runtime index would move it to scratch).
  const bool c0ok = lane < R, c1ok = RV > 1 && lane + 64 < R;
  float2_ acc[kNW];
#pragma unroll
  for (int i = 0; i < kNW; ++i) acc[i] = float2_{0.f, 0.f};
  if (IMPL) {
    for (int i = 0; i < n; ++i) {
      const int64_t c = cols[p0 + i];
      if (c0ok) sY[wv][i][lane] = F[c * R + lane];
      if (c1ok) sY[wv][i][lane + 64] = F[c * R + lane + 64];
    }
    for (int kk = 0; kk < R; kk += 4) {
      float2_ q[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        q[s].x = c0ok ? Q[(kk + s) * R + lane] : 0.f;
        q[s].y = c1ok ? Q[(kk + s) * R + lane + 64] : 0.f;
      }
#pragma unroll
      for (int ib = 0; ib < kNW; ib += 8) {
        if (ib < n) {                            // uniform: rows in blocks of 8
#pragma unroll
          for (int i = ib; i < ib + 8; ++i) {
            const float4_ y = *reinterpret_cast<const float4_*>(&sY[wv][i][kk]);
            acc[i] = __builtin_elementwise_fma(float2_{y.x, y.x}, q[0], acc[i]);
            acc[i] = __builtin_elementwise_fma(float2_{y.y, y.y}, q[1], acc[i]);
            acc[i] = __builtin_elementwise_fma(float2_{y.z, y.z}, q[2], acc[i]);
            acc[i] = __builtin_elementwise_fma(float2_{y.w, y.w}, q[3], acc[i]);
          }
        }
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < kNW; ++i) {
      if (i < n) {
        const int64_t c = cols[p0 + i];
        acc[i].x = c0ok ? F[c * R + lane] : 0.f;
        acc[i].y = c1ok ? F[c * R + lane + 64] : 0.f;
      }
    }
  }

  // S = diag(W^{-1}) + P D P^T (lower triangle): per-lane partial over its columns, DPP
  // wave sum per entry
  const float2_ dd = {dinv[0], RV > 1 ? dinv[RV - 1] : 0.f};
#pragma unroll
  for (int i = 0; i < kNW; ++i) {
    if (i < n) {
      const float2_ pi = acc[i] * dd;
#pragma unroll
      for (int m = 0; m <= i; ++m) {
        const float sm = wave_sum_dpp(pi.x * acc[m].x + pi.y * acc[m].y);
        if (lane == 0) S[i][m] = sm;
      }
    }
  }
  if (lane < n) S[lane][lane] += winv;

  // Cholesky of S in LDS (lane i owns row i), right-looking
  for (int k = 0; k < n; ++k) {
    const float dk = sqrtf(fmaxf(S[k][k], 1e-30f));
    const bool own = lane > k && lane < n;
    float lik = 0.f;
    if (own) {
      lik = S[lane][k] / dk;
      S[lane][k] = lik;
    }
    if (lane == k) S[k][k] = dk;
    if (own)
      for (int j = k + 1; j <= lane; ++j) S[lane][j] -= lik * S[j][k];
  }
  // S z = W^{-1} c: forward (L y = t), backward (L^T z = y); lane i holds entry i
  float v = t;
  for (int k = 0; k < n; ++k) {
    const float yk = rl(v, k) / S[k][k];
    if (lane == k) v = yk;
    else if (lane > k && lane < n) v -= S[lane][k] * yk;
  }
  for (int k = n - 1; k >= 0; --k) {
    const float zk = rl(v, k) / S[k][k];
    if (lane == k) v = zk;
    else if (lane < k) v -= S[k][lane] * zk;
  }
  // y = D P^T z
  float2_ uu = {0.f, 0.f};
#pragma unroll
  for (int i = 0; i < kNW; ++i) {
    if (i < n) {
      const float zi = rl(v, i);
      uu = __builtin_elementwise_fma(float2_{zi, zi}, acc[i], uu);
    }
  }
  uu = uu * dd;
  float* xo = X + u * R;
  if (!IMPL) {
    if (c0ok) xo[lane] = uu.x;
    if (c1ok) xo[lane + 64] = uu.y;
    return;
  }
  // x = Q y
  if (c0ok) sv[wv][lane] = uu.x;
  if (c1ok) sv[wv][lane + 64] = uu.y;
  float2_ xx = {0.f, 0.f};
  for (int j = 0; j < R; ++j) {
    const float yj = sv[wv][j];
    const float2_ qt = {c0ok ? QT[j * R + lane] : 0.f, c1ok ? QT[j * R + lane + 64] : 0.f};
    xx = __builtin_elementwise_fma(float2_{yj, yj}, qt, xx);
  }
  if (c0ok) xo[lane] = xx.x;
  if (c1ok) xo[lane + 64] = xx.y;
}

template <int R>
struct Dense {
  static constexpr int NT = R / 8;                       // 8 x 8 tiles per side
  static constexpr int NTH = NT * NT < 64 ? 64 : NT * NT;
  static constexpr int LDA = R + 4;                      // 16-B aligned rows, bank spread
  static constexpr int CH = 16;                          // ratings staged per round
};

template <int R, bool IMPL>
__global__ __launch_bounds__(Dense<R>::NTH) void als_dense_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ cols, const float* __restrict__ w,
    const float* __restrict__ b, const float* __restrict__ F, const float* __restrict__ G,
    const float* __restrict__ lam, const int32_t* __restrict__ rows, float* __restrict__ X) {
  using D = Dense<R>;
  constexpr int NT = D::NT, NTH = D::NTH, LDA = D::LDA, CH = D::CH;
  __shared__ float sA[R * LDA];
  __shared__ float sY[CH][R];
  __shared__ float sW[CH], sB[CH];
  __shared__ float sr[R];
  const int tid = threadIdx.x;
  const int64_t u = rows[blockIdx.x];
  const int64_t p0 = indptr[u], p1 = indptr[u + 1];
  const float lu = lam[u];
  const bool act = tid < NT * NT;
  const int ti = tid / NT, tj = tid % NT;
  float acc[8][8];
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[r][c] = 0.f;
  float rhs = 0.f;
  for (int64_t c0 = p0; c0 < p1; c0 += CH) {
    const int m = (int)(p1 - c0 < CH ? p1 - c0 : CH);
    for (int e = tid; e < m * R; e += NTH) {
      const int c = e / R, d = e % R;
      sY[c][d] = F[(int64_t)cols[c0 + c] * R + d];
    }
    if (tid < m) {
      sW[tid] = w[c0 + tid];
      sB[tid] = b[c0 + tid];
    }
    __syncthreads();
    if (act) {
      for (int c = 0; c < m; ++c) {
        const float wc = sW[c];
        float a[8], bb[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          a[r] = sY[c][8 * ti + r];
          bb[r] = wc * sY[c][8 * tj + r];
        }
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[r][q] = fmaf(a[r], bb[q], acc[r][q]);
      }
    }
    if (tid < R)
      for (int c = 0; c < m; ++c) rhs = fmaf(sB[c], sY[c][tid], rhs);
    __syncthreads();
  }
  if (act) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int i = 8 * ti + r, j = 8 * tj + q;
        sA[i * LDA + j] = acc[r][q] + (IMPL ? G[i * R + j] : 0.f) + (i == j ? lu : 0.f);
      }
  }
  if (tid < R) sr[tid] = rhs;
  __syncthreads();

  const int lane = tid & 63;
  for (int p = 0; p < NT; ++p) {
    const int k0 = 8 * p;
    if (tid < 64) {
      // diagonal 8 x 8 factor, computed redundantly by every lane of wave 0
      float L[8][8];
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int c = 0; c < 8; ++c) L[r][c] = c <= r ? sA[(k0 + r) * LDA + k0 + c] : 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float s = L[c][c];
#pragma unroll
        for (int q = 0; q < c; ++q) s -= L[c][q] * L[c][q];
        const float dc = sqrtf(fmaxf(s, 1e-30f));
        L[c][c] = dc;
#pragma unroll
        for (int r = c + 1; r < 8; ++r) {
          float v = L[r][c];
#pragma unroll
          for (int q = 0; q < c; ++q) v -= L[r][q] * L[c][q];
          L[r][c] = v / dc;
        }
      }
      // panel rows (TRSM l = a L^-T).  For a row r of the diagonal block the same
      // recursion reproduces L[r][0..r] (its c = r step gives (A_rr - sum L_rq^2) / L_rr =
      // L_rr); what it writes right of the diagonal is upper triangle, never read.
      for (int i = k0 + lane; i < R; i += 64) {
        float a[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) a[c] = sA[i * LDA + k0 + c];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          float v = a[c];
#pragma unroll
          for (int q = 0; q < c; ++q) v -= a[q] * L[c][q];
          a[c] = v / L[c][c];
        }
        // a clamped pivot (singular row, e.g. no ratings and lam = 0) breaks that identity:
        // store the diagonal itself so the solves never divide by zero
#pragma unroll
        for (int c = 0; c < 8; ++c)
          if (i == k0 + c) a[c] = L[c][c];
#pragma unroll
        for (int c = 0; c < 8; ++c) sA[i * LDA + k0 + c] = a[c];
      }
    }
    __syncthreads();
    // trailing update of the lower triangle: A_ij -= L_i,panel . L_j,panel
    const int T = R - k0 - 8;
    const int ntri = T * (T + 1) / 2;
    for (int e = tid; e < ntri; e += NTH) {
      int ii = (int)((sqrtf(8.f * (float)e + 1.f) - 1.f) * 0.5f);
      while (ii * (ii + 1) / 2 > e) --ii;
      while ((ii + 1) * (ii + 2) / 2 <= e) ++ii;
      const int jj = e - ii * (ii + 1) / 2;
      const int i = k0 + 8 + ii, j = k0 + 8 + jj;
      const float4_ a0 = *reinterpret_cast<const float4_*>(&sA[i * LDA + k0]);
      const float4_ a1 = *reinterpret_cast<const float4_*>(&sA[i * LDA + k0 + 4]);
      const float4_ b0 = *reinterpret_cast<const float4_*>(&sA[j * LDA + k0]);
      const float4_ b1 = *reinterpret_cast<const float4_*>(&sA[j * LDA + k0 + 4]);
      float s = a0.x * b0.x + a0.y * b0.y + a0.z * b0.z + a0.w * b0.w + a1.x * b1.x + a1.y * b1.y +
                a1.z * b1.z + a1.w * b1.w;
      sA[i * LDA + j] -= s;
    }
    __syncthreads();
  }
  // triangular solves on wave 0 (lane holds rows lane, lane + 64)
  if (tid < 64) {
    constexpr int RV = (R + 63) / 64;
    float v[RV];
#pragma unroll
    for (int k = 0; k < RV; ++k) v[k] = lane + 64 * k < R ? sr[lane + 64 * k] : 0.f;
    for (int k = 0; k < R; ++k) {
      const float zk = rl(k < 64 ? v[0] : v[RV - 1], k & 63) / sA[k * LDA + k];
#pragma unroll
      for (int q = 0; q < RV; ++q) {
        const int i = lane + 64 * q;
        if (i == k) v[q] = zk;
        else if (i > k && i < R) v[q] -= sA[i * LDA + k] * zk;
      }
    }
    for (int k = R - 1; k >= 0; --k) {
      const float xk = rl(k < 64 ? v[0] : v[RV - 1], k & 63) / sA[k * LDA + k];
#pragma unroll
      for (int q = 0; q < RV; ++q) {
        const int i = lane + 64 * q;
        if (i == k) v[q] = xk;
        else if (i < k) v[q] -= sA[k * LDA + i] * xk;
      }
    }
#pragma unroll
    for (int q = 0; q < RV; ++q)
      if (lane + 64 * q < R) X[u * R + lane + 64 * q] = v[q];
  }
}

template <int R, bool IMPL>
void launch_exact(const int64_t* indptr, const int32_t* cols, const float* w, const float* b, const float* F,
                  const float* G, const float* Q, const float* QT, const float* eig, const float* lam,
                  const int32_t* small, int64_t nsmall, const int32_t* dense, int64_t ndense, float* X,
                  hipStream_t st) {
  if (nsmall > 0)
    hipLaunchKernelGGL((als_wood_kernel<R, IMPL>), dim3((unsigned)((nsmall + kWW - 1) / kWW)), dim3(kWW * 64), 0, st,
                       indptr, cols, w, b, F, Q, QT, eig, lam, small, nsmall, X);
  if (ndense > 0)
    hipLaunchKernelGGL((als_dense_kernel<R, IMPL>), dim3((unsigned)ndense), dim3(Dense<R>::NTH), 0, st, indptr, cols,
                       w, b, F, G, lam, dense, X);
}

}  // namespace

// Exact per-row solves of one ALS half-iteration.  small / dense: row indices (int32) for
// the Woodbury (n_u <= 32, lam_u > 0) and the dense-Cholesky kernels; implicit: G = Y^T Y
// (fp32 R x R) with its eigendecomposition G = Q diag(eig) Q^T (Q row-major, QT = Q^T).
// X (fp32 [rows, R]) receives x_u for every listed row.
O3S_API int o3s_als_exact(int implicit, int R, const int64_t* indptr, const int32_t* cols, const float* w,
                          const float* b, const float* F, const float* G, const float* Q, const float* QT,
                          const float* eig, const float* lam, const int32_t* small, int64_t nsmall,
                          const int32_t* dense, int64_t ndense, float* X, hipStream_t st) {
  if (nsmall < 0 || ndense < 0 || (nsmall > 0 && implicit && (!Q || !QT || !eig)) || (implicit && ndense > 0 && !G))
    return -1;
#define O3S_EX(RR)                                                                                          \
  if (R == RR) {                                                                                            \
    if (implicit)                                                                                           \
      launch_exact<RR, true>(indptr, cols, w, b, F, G, Q, QT, eig, lam, small, nsmall, dense, ndense, X, st); \
    else                                                                                                    \
      launch_exact<RR, false>(indptr, cols, w, b, F, G, Q, QT, eig, lam, small, nsmall, dense, ndense, X, st); \
    O3S_CHECK_LAUNCH();                                                                                     \
    return 0;                                                                                               \
  }
  O3S_EX(32) O3S_EX(64) O3S_EX(96) O3S_EX(128)
#undef O3S_EX
  return -2;
}

O3S_API int o3s_als_exact_max_small() { return kNW; }
