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


// ---------------------------------------------------------------------------------
// Exact normal equations on MFMA (rows with many ratings, e.g. the item side):
//     A_u = FtF[implicit] + sum_j w_j y_j y_j^T + lam_u I,      b_u = sum_j b_j y_j
// for a batch of CSR rows, written densely (A: [batch][R][R] fp32, b: [batch][R]) for a
// batched Cholesky solve -- Spark's exact per-row solve instead of warm-started CG.
// One 256-thread workgroup per row.  Each 16-rating k-step the block gathers the 16
// factor rows (R fp32 each), scales them by sqrt(w_j) (w >= 0: alpha|r| or 1), splits
// them into bf16 hi + lo and stores them TRANSPOSED ([R][16], rating index fastest) in
// LDS, so an MFMA fragment (8 consecutive ratings of one factor component) is one 16-B
// read.  Wave I (< R/32) owns output rows [32I, 32I+32) and all R/32 column tiles:
// 3 v_mfma_f32_32x32x16_bf16 per tile (hi.hi + lo.hi + hi.lo: ~2^-16 relative, fp32-level
// Gram entries).  The gathers of step s+1 are in flight while step s's MFMAs run
// (double-buffered LDS, one barrier per step).  The rhs is accumulated in fp32 by the
// staging threads and reduced through LDS at the end.
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
constexpr int kGramKS = 16;                 // ratings per k-step
constexpr int kGramLd = kGramKS + 8;        // LDS row stride (bf16): 48 B, spreads banks

template <int RT>   // R = 32 * RT
__global__ __launch_bounds__(256) void als_gram_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ cols, const float* __restrict__ w,
    const float* __restrict__ b, const float* __restrict__ F, const float* __restrict__ FtF,
    const float* __restrict__ lam, int64_t row0, float* __restrict__ Aout, float* __restrict__ bout) {
  constexpr int R = 32 * RT;
  constexpr int EPT = R / 16;               // elements per staging thread (16 threads per rating)
  __shared__ __attribute__((aligned(16))) uint16_t T[2][2][R * kGramLd];   // [buf][hi|lo][r][k]
  __shared__ float rpart[kGramKS][R];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t u = row0 + blockIdx.x;
  const int64_t j0 = indptr[u], j1 = indptr[u + 1];
  const int sk = tid >> 4, sseg = tid & 15;         // staging: rating sk of the step, elements sseg*EPT..
  float rhs[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) rhs[e] = 0.f;
  float yv[EPT], wv = 0.f, bv = 0.f;
  auto load = [&](int64_t jb) {                     // gather this thread's slice of rating jb + sk
    const int64_t j = jb + sk;
    const bool ok = j < j1;
    const int64_t c = ok ? (int64_t)cols[j] : 0;
    wv = ok ? w[j] : 0.f;
    bv = ok ? b[j] : 0.f;
    const float* fp = F + c * R + sseg * EPT;
#pragma unroll
    for (int e = 0; e < EPT; ++e) yv[e] = ok ? fp[e] : 0.f;
  };
  auto store = [&](int buf) {
    const float sw = sqrtf(fmaxf(wv, 0.f));
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      rhs[e] = fmaf(bv, yv[e], rhs[e]);
      const float z = sw * yv[e];
      const uint16_t hi = f32_to_bf16(z);
      const uint16_t lo = f32_to_bf16(z - bf16_to_f32(hi));
      const int r = sseg * EPT + e;
      T[buf][0][r * kGramLd + sk] = hi;
      T[buf][1][r * kGramLd + sk] = lo;
    }
  };
  f32x16 acc[RT];
#pragma unroll
  for (int J = 0; J < RT; ++J)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[J][i] = 0.f;
  const int r = lane & 31, h = lane >> 5;
  const int nsteps = (int)((j1 - j0 + kGramKS - 1) / kGramKS);
  if (nsteps > 0) {
    load(j0);
    store(0);
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    const bool more = s + 1 < nsteps;
    if (more) load(j0 + (int64_t)(s + 1) * kGramKS);          // next step's gathers in flight
    if (wid < RT) {
      const uint16_t* Th = T[buf][0];
      const uint16_t* Tl = T[buf][1];
      const bf16x8 ah = *reinterpret_cast<const bf16x8*>(Th + (32 * wid + r) * kGramLd + 8 * h);
      const bf16x8 al = *reinterpret_cast<const bf16x8*>(Tl + (32 * wid + r) * kGramLd + 8 * h);
#pragma unroll
      for (int J = 0; J < RT; ++J) {
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(Th + (32 * J + r) * kGramLd + 8 * h);
        const bf16x8 bl = *reinterpret_cast<const bf16x8*>(Tl + (32 * J + r) * kGramLd + 8 * h);
        acc[J] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[J], 0, 0, 0);
        acc[J] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[J], 0, 0, 0);
        acc[J] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[J], 0, 0, 0);
      }
    }
    if (more) store(buf ^ 1);
    __syncthreads();
  }
  // A_u = acc + FtF + lam I, written straight from the accumulators (lanes -> columns)
  float* Ab = Aout + (int64_t)blockIdx.x * R * R;
  if (wid < RT) {
    const float lu = lam[u];
#pragma unroll
    for (int J = 0; J < RT; ++J) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = 32 * wid + 4 * h + (i & 3) + 8 * (i >> 2);
        const int nn = 32 * J + r;
        float v = acc[J][i];
        if (FtF) v += FtF[m * R + nn];
        if (m == nn) v += lu;
        Ab[m * R + nn] = v;
      }
    }
  }
  // rhs: the 16 staging threads of each element slice hold partial sums over their ratings
  if (nsteps == 0) {
#pragma unroll
    for (int e = 0; e < EPT; ++e) rhs[e] = 0.f;
  }
#pragma unroll
  for (int e = 0; e < EPT; ++e) rpart[sk][sseg * EPT + e] = rhs[e];
  __syncthreads();
  for (int c = tid; c < R; c += 256) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < kGramKS; ++k) t += rpart[k][c];
    bout[(int64_t)blockIdx.x * R + c] = t;
  }
}

// ---------------------------------------------------------------------------------
// Factor initialisation (unit-norm gaussian rows keyed on (seed, global row), so the
// result does not depend on the sharding): element (u, k) = Box-Muller of two
// counter-hash uniforms of streams 2k+11 / 2k+12 -- the same draws as
// ops/sampling.py::uniform, in fp64 -- then each row scaled to unit norm.  One wave
// per row; replaces ~15 torch passes over int64 [rows, rank] temporaries.
template <int RV>
__global__ __launch_bounds__(256) void als_init_kernel(int64_t row0, int64_t n, int R, uint32_t seed, int nonneg,
                                                      float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= n) return;
  float v[RV];
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < RV; ++q) {
    const int k = lane + 64 * q;
    v[q] = 0.f;
    if (k < R) {
      double u1 = hash_uniform(seed, 2u * k + 11u, row0 + u);
      u1 = u1 > 1e-12 ? u1 : 1e-12;
      const double u2 = hash_uniform(seed, 2u * k + 12u, row0 + u);
      v[q] = (float)(sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
      ss = fmaf(v[q], v[q], ss);
    }
  }
  ss = wave_sum_dpp(ss);
  const float inv = 1.f / fmaxf(sqrtf(ss), 1e-12f);
#pragma unroll
  for (int q = 0; q < RV; ++q) {
    const int k = lane + 64 * q;
    if (k < R) {
      const float x = v[q] * inv;
      out[u * R + k] = nonneg ? fabsf(x) : x;
    }
  }
}


// ---------------------------------------------------------------------------------
// F^T F of an [n][ld] fp32 factor table (the implicit-ALS Gram Y^T Y, once per
// half-iteration over all rows of one side).  Exact fp32 products on
// v_mfma_f32_32x32x2_f32 with the K index running over rows: each wave owns a contiguous
// row range and ALL NT (NT + 1) / 2 upper 32 x 32 tiles of the result in its accumulators
// (NT = 4: 10 tiles, 160 registers), so no operand is shared between waves and no LDS is
// touched -- per row pair a lane loads one float per 32-column block,
// F[r + (lane >> 5)][32 cb + (lane & 31)] (coalesced 128-B half-wave runs), which is at once
// the A operand (rows i of the tile) and the B operand (columns j) of every tile using
// block cb.  PF row pairs are in flight per wave.  Partials go to slab[wave][tile][16][64]
// in accumulator order; ftf_reduce_kernel sums them per element in wave order in fp64
// (bitwise reproducible).  hipBLASLt's GEMM for this shape (K = millions, M = N = 128)
// ran a handful of 32 x 32 output tiles on a few CUs: ~1.8 ms per 1M rows.
typedef float f32x16_ __attribute__((ext_vector_type(16)));
constexpr int kFtfWaves = 4;

template <int NT>
__global__ __launch_bounds__(kFtfWaves * 64, 2) void ftf_kernel(const float* __restrict__ F, int64_t n, int64_t ld,
                                                                int R, int64_t rows_per_wave,
                                                                float* __restrict__ slab) {
  constexpr int NL = NT * (NT + 1) / 2;
  constexpr int PF = NT == 4 ? 6 : 8;                    // row pairs in flight (register budget)
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * kFtfWaves + (threadIdx.x >> 6);
  const int64_t r0 = gw * rows_per_wave;
  const int64_t r1 = r0 + rows_per_wave < n ? r0 + rows_per_wave : n;
  const int kr = lane >> 5, c = lane & 31;
  float cm[NT];                                          // column mask (columns >= R read as 0)
  int col[NT];
#pragma unroll
  for (int cb = 0; cb < NT; ++cb) {
    cm[cb] = 32 * cb + c < R ? 1.f : 0.f;
    col[cb] = 32 * cb + c < R ? 32 * cb + c : 0;
  }
  f32x16_ acc[NL];
#pragma unroll
  for (int t = 0; t < NL; ++t)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[t][v] = 0.f;
  auto load = [&](int64_t pr, float (&o)[NT]) {         // row pair pr of the range (clamped row)
    int64_t r = r0 + 2 * pr + kr;
    r = r < n ? r : n - 1;
#pragma unroll
    for (int cb = 0; cb < NT; ++cb) o[cb] = F[r * ld + col[cb]];
  };
  auto consume = [&](const float (&o)[NT], float rm) {  // rm: this lane's row weight (0 / 1)
    float a[NT];
#pragma unroll
    for (int cb = 0; cb < NT; ++cb) a[cb] = o[cb] * cm[cb] * rm;
    int t = 0;
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int j = i; j < NT; ++j, ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], a[j], acc[t], 0, 0, 0);
  };
  const int64_t nrows = r1 > r0 ? r1 - r0 : 0;
  const int64_t full = nrows / 2 / PF * PF;              // whole ring rounds of full pairs
  float v[PF][NT];
#pragma unroll
  for (int u = 0; u < PF; ++u) load(u, v[u]);
  for (int64_t pr = 0; pr < full; pr += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      consume(v[u], 1.f);
      load(pr + PF + u, v[u]);                           // next round (clamped past the range)
    }
  }
  // tail: the remaining rows one pair at a time, rows past the range weighted 0
  for (int64_t pr = full; 2 * pr < nrows; ++pr) {
    float o[NT];
    load(pr, o);
    consume(o, r0 + 2 * pr + kr < r1 ? 1.f : 0.f);
  }
  float* out = slab + gw * NL * 1024;
#pragma unroll
  for (int t = 0; t < NL; ++t)
#pragma unroll
    for (int v2 = 0; v2 < 16; ++v2) out[(t * 16 + v2) * 64 + lane] = acc[t][v2];
}

// out[i][j] (fp64 R x R, both triangles) = sum over waves, in wave order, of the slab
// element holding (i, j) of the upper tile (i / 32, j / 32) (i <= j; (j, i) otherwise)
__global__ __launch_bounds__(256) void ftf_reduce_kernel(const float* __restrict__ slab, int64_t nwaves, int NT,
                                                         int R, double* __restrict__ out) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= R * R) return;
  int i = e / R, j = e % R;
  if (i > j) { const int tmp = i; i = j; j = tmp; }
  const int ib = i >> 5, jb = j >> 5, ri = i & 31, cj = j & 31;
  const int t = ib * NT - ib * (ib - 1) / 2 + (jb - ib);  // upper-triangle tile index
  const int v = (ri & 3) + 4 * (ri >> 3), l = cj + 32 * ((ri >> 2) & 1);
  const int NL = NT * (NT + 1) / 2;
  double s = 0.0;
  for (int64_t g = 0; g < nwaves; ++g) s += (double)slab[(g * NL + t) * 1024 + v * 64 + l];
  out[e] = s;
}

}  // namespace

// F^T F (fp64 [R][R]) of an [n][ld] fp32 table, R <= 128.  slab: >= nwaves * NL * 1024
// floats, NL = NT (NT + 1) / 2, NT = ceil(R / 32); nwaves = a multiple of 4.
O3S_API int o3s_ftf(const float* F, int64_t n, int64_t ld, int R, int64_t nwaves, float* slab, double* out,
                    hipStream_t st) {
  if (n < 0 || R <= 0 || R > 128 || ld < R || nwaves <= 0 || nwaves % kFtfWaves) return -1;
  const int NT = (R + 31) / 32;
  int64_t rpw = (n + nwaves - 1) / nwaves;
  rpw += rpw & 1;                                        // even: whole row pairs per wave
  const dim3 grid((unsigned)(nwaves / kFtfWaves));
  if (n > 0) {
    switch (NT) {
      case 1: hipLaunchKernelGGL((ftf_kernel<1>), grid, dim3(kFtfWaves * 64), 0, st, F, n, ld, R, rpw, slab); break;
      case 2: hipLaunchKernelGGL((ftf_kernel<2>), grid, dim3(kFtfWaves * 64), 0, st, F, n, ld, R, rpw, slab); break;
      case 3: hipLaunchKernelGGL((ftf_kernel<3>), grid, dim3(kFtfWaves * 64), 0, st, F, n, ld, R, rpw, slab); break;
      default: hipLaunchKernelGGL((ftf_kernel<4>), grid, dim3(kFtfWaves * 64), 0, st, F, n, ld, R, rpw, slab); break;
    }
    O3S_CHECK_LAUNCH();
  } else {
    if (hipMemsetAsync(slab, 0, sizeof(float) * (size_t)nwaves * (NT * (NT + 1) / 2) * 1024, st) != hipSuccess)
      return -3;
  }
  hipLaunchKernelGGL(ftf_reduce_kernel, dim3((unsigned)((R * R + 255) / 256)), dim3(256), 0, st, slab, nwaves, NT, R,
                     out);
  O3S_CHECK_LAUNCH();
  return 0;
}

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

// Dense normal equations for CSR rows [row0, row0 + nrows) (R = 32, 64, 96 or 128):
// A: [nrows][R][R], b: [nrows][R] fp32.  FtF may be null (explicit feedback).
O3S_API int o3s_als_gram(const int64_t* indptr, const int32_t* cols, const float* w, const float* b, const float* F,
                         int R, const float* FtF, const float* lam, int64_t row0, int64_t nrows, float* A,
                         float* bout, hipStream_t st) {
  if (nrows <= 0) return 0;
  if (R % 32 != 0 || R < 32 || R > 128 || nrows > 0x7fffffff) return -1;
#define O3S_G(RTV)                                                                                        \
  case RTV:                                                                                               \
    hipLaunchKernelGGL((als_gram_kernel<RTV>), dim3((unsigned)nrows), dim3(256), 0, st, indptr, cols, w, b, F, \
                       FtF, lam, row0, A, bout);                                                          \
    break;
  switch (R / 32) {
    O3S_G(1) O3S_G(2) O3S_G(3) O3S_G(4)
    default: return -1;
  }
#undef O3S_G
  O3S_CHECK_LAUNCH();
  return 0;
}

// out: fp32 [n][R] rows row0 .. row0+n-1 of the factor table (R <= 512).
O3S_API int o3s_als_init(int64_t row0, int64_t n, int R, uint32_t seed, int nonneg, float* out, hipStream_t st) {
  if (n <= 0) return 0;
  if (R <= 0 || R > 512) return -1;
  const int rv = (R + 63) / 64;
  const unsigned grid = (unsigned)((n + 3) / 4);
#define O3S_AI(RVV) \
  if (rv == RVV) hipLaunchKernelGGL((als_init_kernel<RVV>), dim3(grid), dim3(256), 0, st, row0, n, R, seed, nonneg, out);
  O3S_AI(1) O3S_AI(2) O3S_AI(3) O3S_AI(4) O3S_AI(5) O3S_AI(6) O3S_AI(7) O3S_AI(8)
#undef O3S_AI
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_PRELOAD(als)
