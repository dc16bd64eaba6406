// ALS ratings passes (gfx950).  Replaces the per-block normal-equation assembly of
// Spark's ALS (reached through the Recommendation widget -> fit,
// orangecontrib/spark/widgets/ml/spark_ml_recommendation.py:15).
//
// The solver is conjugate gradient on each user's (item's) normal equations, so the
// rank x rank systems are never formed: every CG step needs only
//     out[u] = sum_{j in row u} w_j * (F[col_j] . V[u]) * F[col_j]          (MATVEC)
// and once per half-iteration the right-hand side
//     out[u] = sum_{j in row u} b_j * F[col_j]                              (RHS)
// over the CSR ratings of this rank (rows = users for the user half, items for the item
// half; F = the all-gathered factor table of the other side).  The dense parts
// (implicit Y^T Y . v, lambda * n_u * v) are batched GEMMs done by the caller.
//
// One wave per CSR row: lane l holds dims l, l+64, ... (R/64 per lane) of V[u] and of
// the accumulator in registers; F rows are streamed 16 B... per lane-pair coalesced
// (R*4 bytes contiguous per rating); the per-rating dot product is one wave
// reduction.  4 ratings are kept in flight per wave to hide gather latency.
#include "common.h"

using namespace o3s;

namespace {

constexpr int kAlsWaves = 4;

// MODE 0 = MATVEC, 1 = RHS, 2 = both in one gather pass (out = matvec, out2 = rhs with
// coefficients coef2): CG's first residual needs rhs - A x0, and both sum the same rows.
template <int RV, int MODE>   // RV = dims per lane (R = 64*RV)
__global__ __launch_bounds__(kAlsWaves * 64) void als_pass_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ cols, const float* __restrict__ coef,
    int64_t nrows, const float* __restrict__ F, int R, const float* __restrict__ V, float* __restrict__ out,
    const float* __restrict__ coef2, float* __restrict__ out2) {
  const int lane = threadIdx.x & 63;
  const int64_t u = (int64_t)blockIdx.x * kAlsWaves + (threadIdx.x >> 6);
  if (u >= nrows) return;
  float v[RV], acc[RV], acc2[RV];
#pragma unroll
  for (int k = 0; k < RV; ++k) {
    const int d = lane + 64 * k;
    v[k] = (MODE != 1 && d < R) ? V[u * R + d] : 0.f;
    acc[k] = 0.f;
    acc2[k] = 0.f;
  }
  const int64_t s0 = indptr[u], s1 = indptr[u + 1];
  constexpr int U = 4;
  for (int64_t j0 = s0; j0 < s1; j0 += U) {
    float f[U][RV], cj[U], cj2[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int64_t j = j0 + q;
      const bool ok = j < s1;
      const int64_t jc = ok ? j : s0;
      const int64_t c = cols[jc];
      cj[q] = ok ? coef[jc] : 0.f;
      cj2[q] = (MODE == 2 && ok) ? coef2[jc] : 0.f;
#pragma unroll
      for (int k = 0; k < RV; ++k) {
        const int d = lane + 64 * k;
        f[q][k] = d < R ? F[c * R + d] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      float s = cj[q];
      if (MODE != 1) {
        float dot = 0.f;
#pragma unroll
        for (int k = 0; k < RV; ++k) dot = fmaf(f[q][k], v[k], dot);
        s *= wave_sum_dpp(dot);             // DPP: no LDS round trips in the per-rating chain
      }
#pragma unroll
      for (int k = 0; k < RV; ++k) acc[k] = fmaf(s, f[q][k], acc[k]);
      if (MODE == 2) {
#pragma unroll
        for (int k = 0; k < RV; ++k) acc2[k] = fmaf(cj2[q], f[q][k], acc2[k]);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < RV; ++k) {
    const int d = lane + 64 * k;
    if (d < R) out[u * R + d] = acc[k];
    if (MODE == 2 && d < R) out2[u * R + d] = acc2[k];
  }
}

// ---------------------------------------------------------------------------------
// Fused per-row CG vector work of the normal-equation solves (one wave per row; every
// user's / item's system is independent, so the whole CG bookkeeping is row-local).
// INIT (mode 0): q = ax + pf + lam*x;  r = rhs - q;  p = r;  rs = r.r
// STEP (mode 1): q = ap + pf + lam*p;  a = rs / p.q;  x += a p;  r -= a q;
//                rs' = r.r;  p = r + (rs'/rs) p;  rs = rs'
// (pf = v @ FtF from hipBLASLt, may be null).  Replaces ~15 separate torch element-wise
// passes over [n, R] per CG step with one read of x, r, p, ap, pf and one write of x, r, p.
template <int RV, int MODE>
__global__ __launch_bounds__(kAlsWaves * 64) void als_cg_kernel(int64_t nrows, int R, float* __restrict__ x,
                                                                 float* __restrict__ r, float* __restrict__ p,
                                                                 const float* __restrict__ av,
                                                                 const float* __restrict__ pf,
                                                                 const float* __restrict__ rhs,
                                                                 const float* __restrict__ lam,
                                                                 float* __restrict__ rs) {
  const int lane = threadIdx.x & 63;
  const int64_t u = (int64_t)blockIdx.x * kAlsWaves + (threadIdx.x >> 6);
  if (u >= nrows) return;                               // whole waves exit together
  const float l = lam[u];
  const int64_t base = u * R;
  float q[RV], vv[RV];
  float dot = 0.f;
#pragma unroll
  for (int k = 0; k < RV; ++k) {
    const int d = lane + 64 * k;
    if (d < R) {
      vv[k] = MODE == 0 ? x[base + d] : p[base + d];
      q[k] = av[base + d] + (pf ? pf[base + d] : 0.f) + l * vv[k];
    } else {
      vv[k] = 0.f;
      q[k] = 0.f;
    }
  }
  if (MODE == 0) {
#pragma unroll
    for (int k = 0; k < RV; ++k) {
      const int d = lane + 64 * k;
      if (d < R) {
        const float rr = rhs[base + d] - q[k];
        r[base + d] = rr;
        p[base + d] = rr;
        dot = fmaf(rr, rr, dot);
      }
    }
    dot = wave_sum_dpp(dot);
    if (lane == 0) rs[u] = dot;
    return;
  }
#pragma unroll
  for (int k = 0; k < RV; ++k) dot = fmaf(vv[k], q[k], dot);
  const float den = wave_sum_dpp(dot);
  const float rs0 = rs[u];
  const float a = den > 0.f ? rs0 / fmaxf(den, 1e-30f) : 0.f;
  float rr[RV];
  float nr = 0.f;
#pragma unroll
  for (int k = 0; k < RV; ++k) {
    const int d = lane + 64 * k;
    rr[k] = 0.f;
    if (d < R) {
      x[base + d] = fmaf(a, vv[k], x[base + d]);
      rr[k] = fmaf(-a, q[k], r[base + d]);
      r[base + d] = rr[k];
      nr = fmaf(rr[k], rr[k], nr);
    }
  }
  const float rs1 = wave_sum_dpp(nr);
  const float beta = rs0 > 0.f ? rs1 / fmaxf(rs0, 1e-30f) : 0.f;
#pragma unroll
  for (int k = 0; k < RV; ++k) {
    const int d = lane + 64 * k;
    if (d < R) p[base + d] = fmaf(beta, vv[k], rr[k]);
  }
  if (lane == 0) rs[u] = rs1;
}

}  // namespace

// mode 0: CG init (x, av = A-part of A x, rhs -> r, p, rs); mode 1: CG step (p, av = A-part of A p).
// All [nrows, R] fp32 row-major; pf / rhs may be null where unused.
O3S_API int o3s_als_cg(int mode, int64_t nrows, int R, float* x, float* r, float* p, const float* av,
                       const float* pf, const float* rhs, const float* lam, float* rs, hipStream_t st) {
  if (nrows <= 0) return 0;
  if (R <= 0 || R > 512 || (mode == 0 && !rhs)) return -1;
  const int rv = (R + 63) / 64;
  const unsigned grid = (unsigned)((nrows + kAlsWaves - 1) / kAlsWaves);
#define O3S_CG(RVV)                                                                                        \
  if (rv == RVV) {                                                                                         \
    if (mode == 0)                                                                                         \
      hipLaunchKernelGGL((als_cg_kernel<RVV, 0>), dim3(grid), dim3(kAlsWaves * 64), 0, st, nrows, R, x, r, p, \
                         av, pf, rhs, lam, rs);                                                            \
    else                                                                                                   \
      hipLaunchKernelGGL((als_cg_kernel<RVV, 1>), dim3(grid), dim3(kAlsWaves * 64), 0, st, nrows, R, x, r, p, \
                         av, pf, rhs, lam, rs);                                                            \
  }
  O3S_CG(1) O3S_CG(2) O3S_CG(3) O3S_CG(4) O3S_CG(5) O3S_CG(6) O3S_CG(7) O3S_CG(8)
#undef O3S_CG
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_API int o3s_als_pass(int mode, const int64_t* indptr, const int32_t* cols, const float* coef, int64_t nrows,
                         const float* F, int R, const float* V, float* out, const float* coef2, float* out2,
                         hipStream_t st) {
  if (nrows <= 0) return 0;
  if (R <= 0 || R > 512) return -1;
  const int rv = (R + 63) / 64;
  const unsigned grid = (unsigned)((nrows + kAlsWaves - 1) / kAlsWaves);
#define O3S_AL(RVV)                                                                                      \
  if (rv == RVV) {                                                                                       \
    if (mode == 0)                                                                                       \
      hipLaunchKernelGGL((als_pass_kernel<RVV, 0>), dim3(grid), dim3(kAlsWaves * 64), 0, st, indptr, cols, \
                         coef, nrows, F, R, V, out, coef2, out2);                                        \
    else if (mode == 1)                                                                                  \
      hipLaunchKernelGGL((als_pass_kernel<RVV, 1>), dim3(grid), dim3(kAlsWaves * 64), 0, st, indptr, cols, \
                         coef, nrows, F, R, V, out, coef2, out2);                                        \
    else                                                                                                 \
      hipLaunchKernelGGL((als_pass_kernel<RVV, 2>), dim3(grid), dim3(kAlsWaves * 64), 0, st, indptr, cols, \
                         coef, nrows, F, R, V, out, coef2, out2);                                        \
  }
  O3S_AL(1) O3S_AL(2) O3S_AL(3) O3S_AL(4) O3S_AL(5) O3S_AL(6) O3S_AL(7) O3S_AL(8)
#undef O3S_AL
  O3S_CHECK_LAUNCH();
  return 0;
}
