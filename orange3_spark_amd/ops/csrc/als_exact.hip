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
//   P = Y_u Q (n x R: rows of the table F Q, rotated once per half-iteration by one GEMM),
//   Woodbury gives
//       x_u = Q D P^T z,   D = diag(1 / (e + lam_u)),   S z = W^{-1} c,
//       S = W^{-1} + P D P^T   (n x n, SPD)
//   so the only factorisation is an n x n Cholesky -- no 128-step pivot chain per row.
//   One wave per row: P lives in registers (lane l holds columns l, l + 64 as float2 ->
//   v_pk_fma), S in LDS (lane i owns row i), triangular solves broadcast with readlane.
//   Per row: a gather of n factor rows and n^2 R / 2 FMA -- no rank x rank work at all
//   (the rotation back, x = Q y, is one GEMM over all Woodbury rows on the host side).
// * als_dense_kernel (longer rows: the item side, ~200 ratings): one block per row, thread
//   (i, j) of an (R/8)^2 grid owns the 8 x 8 tile A_ij (lower triangle) in registers for
//   the whole solve: the Gram matrix accumulates there (packed FMA over factor rows staged
//   through LDS), then a blocked right-looking Cholesky runs on the tiles -- per 8-wide
//   panel the diagonal owner factors and inverts its tile, the panel owners form
//   L_ip = A_ip inv(L_pp)^T and publish it through LDS, every trailing owner subtracts
//   L_ip L_jp^T -- and the two triangular solves walk the same tiles.  A never touches
//   LDS; the per-row LDS is the staging buffer, one panel and the 8 x 8 inverses.
//
// Both write x_u straight into the factor table.  fp32 throughout (the Gram / S sums are
// short: n_u terms).
#include "common.h"

using namespace o3s;

namespace {

typedef float f32x16_ __attribute__((ext_vector_type(16)));
constexpr int kNW = 32;   // Woodbury path: rows with at most this many ratings
constexpr int kWW = 2;    // waves (rows) per Woodbury block
constexpr int kPS = 72;   // LDS row stride of a P' half tile (features 32 h + s at [36 h + s])

__device__ __forceinline__ float rl(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}

template <int R>
__global__ __launch_bounds__(kWW * 64) void als_wood_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ cols, const float* __restrict__ w,
    const float* __restrict__ b, const float* __restrict__ P, const float* __restrict__ eig,
    const float* __restrict__ lam, const int32_t* __restrict__ rows, int64_t nlist, float* __restrict__ X) {
  static_assert(R % 32 == 0 && R <= 128, "rank must be a multiple of 32, at most 128");
  constexpr int RV = (R + 63) / 64;              // columns per lane (1 or 2)
  // per wave: the sqrt(D)-scaled rows P' for the MFMA (32 x kPS floats), later reused for
  // the S image and L by columns (Lc[k][i] = L_ik)
  __shared__ __attribute__((aligned(16))) float sP[kWW][kNW * kPS];
  __shared__ __attribute__((aligned(16))) float sColb[kWW][kNW + 4];   // step k's column, packed
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t li = (int64_t)blockIdx.x * kWW + wv;
  if (li >= nlist) return;                       // wave-uniform; the kernel has no block barrier
  const int64_t u = rows[li];
  const int64_t p0 = indptr[u];
  const int n = (int)(indptr[u + 1] - p0);       // <= kNW (host routing)
  const float lu = lam[u];
  float (*S)[kNW + 1] = reinterpret_cast<float (*)[kNW + 1]>(sP[wv]);

  // per-rating W^{-1} c (lane i < n holds rating i); w = 0 (r = 0 implicit): no term
  float t = 0.f, winv = 0.f;
  if (lane < n) {
    const float wi = w[p0 + lane], bi = b[p0 + lane];
    winv = wi > 0.f ? 1.f / wi : 1e30f;
    t = wi > 0.f ? bi * winv : 0.f;
  }
  const bool c0ok = lane < R, c1ok = RV > 1 && lane + 64 < R;
  const float2_ dd = {c0ok ? 1.f / (eig[lane] + lu) : 0.f, c1ok ? 1.f / (eig[lane + 64] + lu) : 0.f};

  // rows of P = Y_u Q gathered from the pre-rotated table (F Q, one GEMM per
  // half-iteration; F itself when explicit): acc[i] = (P[i][lane], P[i][lane + 64]).
  // Every loop over rows is unrolled to kNW with a uniform guard, so acc stays in
  // registers (a runtime index would move it to scratch) and all n row loads are in
  // flight together.
  // the row's rating indices arrive in ONE vector load (lane i holds index i) and are
  // broadcast by v_readlane, so the n row gathers issue back to back (a scalar load per
  // index would serialise n load latencies behind the per-row guards)
  const int myc = lane < n ? cols[p0 + lane] : 0;
  int ci[kNW];                                   // all broadcasts before the first gather
#pragma unroll
  for (int i = 0; i < kNW; ++i) ci[i] = __builtin_amdgcn_readlane(myc, i);
  float2_ acc[kNW];
#pragma unroll
  for (int i = 0; i < kNW; ++i) {
    acc[i] = float2_{0.f, 0.f};
    if (i < n) {
      const int64_t c = ci[i];
      acc[i].x = c0ok ? P[c * R + lane] : 0.f;
      acc[i].y = c1ok ? P[c * R + lane + 64] : 0.f;
    }
  }

  // S = P D P^T = P' P'^T with P' = P sqrt(D), on the matrix cores: each 64-feature half of
  // the rows goes through a 9 KB LDS tile (lane l of the MFMA needs row l & 31), then 32
  // v_mfma_f32_32x32x2_f32 per half accumulate the 32 x 32 product in fp32 (feature
  // 32 h + s in k-slot h of step s -- the same value for the A and B operands), on two
  // accumulator chains.  Rows >= n are zero.
  const float2_ sq = {sqrtf(dd.x), sqrtf(dd.y)};
  float* sp = sP[wv];
  f32x16_ sa0, sa1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    sa0[r] = 0.f;
    sa1[r] = 0.f;
  }
  const int wcol = lane < 32 ? lane : lane + 4;
  const float* rp = sp + (lane & 31) * kPS + (lane >> 5) * 36;
#pragma unroll
  for (int hf = 0; hf < RV; ++hf) {
#pragma unroll
    for (int i = 0; i < kNW; ++i) sp[i * kPS + wcol] = hf == 0 ? acc[i].x * sq.x : acc[i].y * sq.y;
#pragma unroll
    for (int s4 = 0; s4 < 32; s4 += 4) {
      const float4_ v = *reinterpret_cast<const float4_*>(rp + s4);
      sa0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v.x, v.x, sa0, 0, 0, 0);
      sa1 = __builtin_amdgcn_mfma_f32_32x32x2f32(v.y, v.y, sa1, 0, 0, 0);
      sa0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v.z, v.z, sa0, 0, 0, 0);
      sa1 = __builtin_amdgcn_mfma_f32_32x32x2f32(v.w, v.w, sa1, 0, 0, 0);
    }
  }
  const f32x16_ sacc = sa0 + sa1;
  // S image in LDS (C/D map: column lane & 31, row (r & 3) + 8 (r >> 2) + 4 (lane >> 5)),
  // then every lane takes its row: srow[m] = S_lane,m (the upper part is the symmetric
  // half, which the Cholesky below never reads)
#pragma unroll
  for (int r = 0; r < 16; ++r) S[(r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)][lane & 31] = sacc[r];
  if (lane < kNW) S[lane][lane] += winv;         // W^{-1} on the diagonal, in the image
  float srow[kNW];
#pragma unroll
  for (int m = 0; m < kNW; ++m) srow[m] = S[lane & 31][m];

  // Cholesky in registers, right-looking, with a SHIFTING row window: after step k lane i
  // holds S_{i, k+1+j} in srow[j], so the active column is always srow[0] and every
  // register index is a constant although k runs in an ordinary loop.  Step k: pivot from
  // lane k (readlane), column k of L published to LDS twice -- packed at [0, n-k-1) for
  // the rank-1 update (aligned float4 reads) and at Lc[k][i] for the solves.  About
  // n^2 / 2 FMAs per lane in all.
  float (*Lc)[kNW + 1] = S;                      // Lc[k][i] = L_ik
  float* colb = sColb[wv];
  if (lane < kNW + 4) colb[lane] = 0.f;          // never-written slots read as 0, not junk
  for (int k = 0; k < n; ++k) {
    const float piv = fmaxf(rl(srow[0], k), 1e-30f);
    const float id = __builtin_amdgcn_rsqf(piv);
    const float lik = lane > k ? srow[0] * id : (lane == k ? piv * id : 0.f);
    if (lane < kNW) Lc[k][lane] = lik;
    if (lane > k && lane < kNW) colb[lane - k - 1] = lik;
    // rank-1 update + shift.  Entries right of the diagonal (column > lane) and columns
    // >= n take garbage-free but unused values (lik = 0 above the diagonal), so there is
    // no per-entry predicate; blocks past column n are skipped whole (uniform branch).
    const int live = n - k - 1;
#pragma unroll
    for (int j4 = 0; j4 < kNW; j4 += 4) {
      if (j4 < live) {
        const float4_ c4 = *reinterpret_cast<const float4_*>(&colb[j4]);
        const float cj[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = j4 + q;                  // srow[j + 1] = S_{i, k+1+j} before the shift
          srow[j] = fmaf(-lik, cj[q], j + 1 < kNW ? srow[j + 1] : 0.f);
        }
      }
    }
  }
  // S z = W^{-1} c: forward L y = t, backward L^T z = y, both reading L by columns from
  // LDS (lane i holds entry i)
  float v = t;
  for (int k = 0; k < n; ++k) {
    const float lik = Lc[k][lane < kNW ? lane : 0];
    const float yk = rl(v, k) * __builtin_amdgcn_rcpf(Lc[k][k]);
    v = lane == k ? yk : (lane > k ? fmaf(-lik, yk, v) : v);
  }
  for (int k = n - 1; k >= 0; --k) {
    // L^T row k = L column k: z_k = (y_k - sum_{i > k} L_ik z_i) / L_kk, right-looking:
    // v_i -= L_ki z_k for i < k (row k of L = entries Lc[i][k])
    const float lki = Lc[lane < kNW ? lane : 0][k];
    const float zk = rl(v, k) * __builtin_amdgcn_rcpf(Lc[k][k]);
    v = lane == k ? zk : (lane < k ? fmaf(-lki, zk, v) : v);
  }
  // y = D P^T z: the solution in the eigenbasis (implicit; the host rotates x = Q y for all
  // Woodbury rows) or x itself (explicit, Q = I)
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
  if (c0ok) xo[lane] = uu.x;
  if (c1ok) xo[lane + 64] = uu.y;
}

template <int R>
struct Dense {
  static constexpr int NT = R / 8;                       // 8 x 8 tiles per side
  static constexpr int NL = NT * (NT + 1) / 2;            // lower-triangle tiles, one per thread
  static constexpr int NTH = NL <= 64 ? 64 : (NL + 63) / 64 * 64;
  static constexpr int CH = 16;                          // ratings staged per round
  static constexpr int PS = 68;                          // panel tile stride (floats): 16-B aligned, banks spread
  static constexpr int MINW = R == 128 ? 3 : 2;          // waves per SIMD the register budget must allow
};

// element (r, c) of a register tile held as 8 rows x 4 float2 (pairs of columns)
#define T_(a, r, c) a[r][(c) >> 1][(c)&1]

template <int R, bool IMPL>
__global__ __launch_bounds__(Dense<R>::NTH, Dense<R>::MINW) void als_dense_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ cols, const float* __restrict__ w,
    const float* __restrict__ b, const float* __restrict__ F, const float* __restrict__ G,
    const float* __restrict__ lam, const int32_t* __restrict__ rows, float* __restrict__ X) {
  using D = Dense<R>;
  constexpr int NT = D::NT, NTH = D::NTH, CH = D::CH, PS = D::PS;
  __shared__ float sY[CH][R];
  __shared__ float sW[CH], sB[CH];
  __shared__ float sPT[NT][PS];     // current panel: L_ip transposed (column k at [8k .. 8k+7])
  __shared__ float sI[NT][64];      // L_pp, row-major (zeros above the diagonal), every p
  __shared__ float sIdv[NT][8];     // 1 / L_cc of every diagonal tile
  __shared__ float sr[R];           // rhs -> y -> x
  const int tid = threadIdx.x;
  const int64_t u = rows[blockIdx.x];
  const int64_t p0 = indptr[u], p1 = indptr[u + 1];
  const float lu = lam[u];
  // thread t < NL owns lower tile t = ti (ti + 1) / 2 + tj: the working lanes are packed
  // into the first waves (no lanes parked on upper tiles); idle threads own no tile
  const bool act = tid < D::NL;
  int ti = NT, tj = NT;
  if (act) {
    ti = 0;
    while ((ti + 1) * (ti + 2) / 2 <= tid) ++ti;
    tj = tid - ti * (ti + 1) / 2;
  }
  float2_ acc[8][4];
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int h = 0; h < 4; ++h) acc[r][h] = float2_{0.f, 0.f};

  // ---- Gram sum_c w_c y_c y_c^T: tile (ti, tj) in registers, packed FMA ----
  // Staging is software-pipelined: round k + 1's factor rows are loaded into registers
  // (PF per thread) while round k is multiplied out of LDS, so the gather latency of a
  // long row is paid once, not once per 16 ratings.
  constexpr int PF = (CH * R + NTH - 1) / NTH;
  float pf[PF];
  float pw = 0.f, pb = 0.f;
  auto issue = [&](int64_t c0) {
    const int m = (int)(p1 - c0 < CH ? p1 - c0 : CH);
    // all index loads first, then all factor loads: PF independent gathers in flight
    // (a loop of dependent index -> row loads would pay one memory latency per element)
    // out-of-round slots read a valid element (the round's last rating) and are zeroed
    // by a select: no branches, so every load issues back to back
    int cidx[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int e = tid + q * NTH;
      const int c = e / R < m ? e / R : m - 1;
      cidx[q] = cols[c0 + c];
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int e = tid + q * NTH;
      const int d = e % R;
      const float v = F[(int64_t)cidx[q] * R + d];
      pf[q] = e < m * R ? v : 0.f;
    }
    if (tid < m) {
      pw = w[c0 + tid];
      pb = b[c0 + tid];
    }
  };
  float rhs = 0.f;
  if (p0 < p1) issue(p0);
  for (int64_t c0 = p0; c0 < p1; c0 += CH) {
    const int m = (int)(p1 - c0 < CH ? p1 - c0 : CH);
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int e = tid + q * NTH;
      if (e < m * R) sY[e / R][e % R] = pf[q];
    }
    if (tid < m) {
      sW[tid] = pw;
      sB[tid] = pb;
    }
    __syncthreads();
    if (c0 + CH < p1) issue(c0 + CH);
    if (act && ti >= tj) {
      for (int c = 0; c < m; ++c) {
        const float wc = sW[c];
        const float4_ a0 = *reinterpret_cast<const float4_*>(&sY[c][8 * ti]);
        const float4_ a1 = *reinterpret_cast<const float4_*>(&sY[c][8 * ti + 4]);
        const float4_ b0 = *reinterpret_cast<const float4_*>(&sY[c][8 * tj]);
        const float4_ b1 = *reinterpret_cast<const float4_*>(&sY[c][8 * tj + 4]);
        const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const float2_ bp[4] = {float2_{b0.x, b0.y} * wc, float2_{b0.z, b0.w} * wc, float2_{b1.x, b1.y} * wc,
                               float2_{b1.z, b1.w} * wc};
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
          for (int h = 0; h < 4; ++h) acc[r][h] = __builtin_elementwise_fma(float2_{av[r], av[r]}, bp[h], acc[r][h]);
      }
    }
    if (tid < R)
      for (int c = 0; c < m; ++c) rhs = fmaf(sB[c], sY[c][tid], rhs);
    __syncthreads();
  }
  if (act && ti >= tj) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float v = T_(acc, r, c);
        if (IMPL) v += G[(8 * ti + r) * R + 8 * tj + c];
        if (ti == tj && r == c) v += lu;
        T_(acc, r, c) = v;
      }
  }
  if (tid < R) sr[tid] = rhs;
  __syncthreads();

  // ---- blocked right-looking Cholesky over the register tiles (the forward solve
  // L y = rhs rides along: diagonal owners finish y_p, panel owners update r_i) ----
  for (int p = 0; p < NT; ++p) {
    if (ti == p && tj == p) {
      // factor the diagonal tile in place (lower; v_rsq, no divisions), invert the factor
      // into sI[p], and take this block of the forward solve: y_p = inv(L_pp) r_p (r_p
      // already carries every earlier panel's update)
      float idv[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float s = T_(acc, c, c);
#pragma unroll
        for (int k = 0; k < c; ++k) s -= T_(acc, c, k) * T_(acc, c, k);
        s = fmaxf(s, 1e-30f);
        const float id = __builtin_amdgcn_rsqf(s);
        idv[c] = id;
        T_(acc, c, c) = s * id;
#pragma unroll
        for (int r = c + 1; r < 8; ++r) {
          float v = T_(acc, r, c);
#pragma unroll
          for (int k = 0; k < c; ++k) v -= T_(acc, r, k) * T_(acc, c, k);
          T_(acc, r, c) = v * id;
        }
      }
      // publish L_pp (row-major, zeros above the diagonal) and 1 / L_cc; forward
      // substitution y_p = L_pp^-1 r_p (r_p already carries every earlier panel's update)
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        float lr[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) lr[c] = c <= r ? T_(acc, r, c) : 0.f;
        *reinterpret_cast<float4_*>(&sI[p][8 * r]) = float4_{lr[0], lr[1], lr[2], lr[3]};
        *reinterpret_cast<float4_*>(&sI[p][8 * r + 4]) = float4_{lr[4], lr[5], lr[6], lr[7]};
      }
      *reinterpret_cast<float4_*>(&sIdv[p][0]) = float4_{idv[0], idv[1], idv[2], idv[3]};
      *reinterpret_cast<float4_*>(&sIdv[p][4]) = float4_{idv[4], idv[5], idv[6], idv[7]};
      float y[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        float v = sr[8 * p + r];
#pragma unroll
        for (int k = 0; k < r; ++k) v = fmaf(-T_(acc, r, k), y[k], v);
        y[r] = v * idv[r];
      }
#pragma unroll
      for (int r = 0; r < 8; ++r) sr[8 * p + r] = y[r];
    }
    __syncthreads();
    if (tj == p && ti > p && ti < NT) {
      // panel: L_ip = A_ip L_pp^-T by forward substitution along each row (the 8 rows are
      // independent chains), L_pp and 1 / L_cc loaded once into registers
      float lp[8][8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const float4_ l0 = *reinterpret_cast<const float4_*>(&sI[p][8 * r]);
        const float4_ l1 = *reinterpret_cast<const float4_*>(&sI[p][8 * r + 4]);
        lp[r][0] = l0.x; lp[r][1] = l0.y; lp[r][2] = l0.z; lp[r][3] = l0.w;
        lp[r][4] = l1.x; lp[r][5] = l1.y; lp[r][6] = l1.z; lp[r][7] = l1.w;
      }
      const float4_ d0 = *reinterpret_cast<const float4_*>(&sIdv[p][0]);
      const float4_ d1 = *reinterpret_cast<const float4_*>(&sIdv[p][4]);
      const float dv[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
      for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          float v = T_(acc, r, c);
#pragma unroll
          for (int k = 0; k < c; ++k) v = fmaf(-T_(acc, r, k), lp[c][k], v);
          T_(acc, r, c) = v * dv[c];
        }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        *reinterpret_cast<float4_*>(&sPT[ti][8 * k]) =
            float4_{T_(acc, 0, k), T_(acc, 1, k), T_(acc, 2, k), T_(acc, 3, k)};
        *reinterpret_cast<float4_*>(&sPT[ti][8 * k + 4]) =
            float4_{T_(acc, 4, k), T_(acc, 5, k), T_(acc, 6, k), T_(acc, 7, k)};
      }
      // forward solve, right-looking: r_i -= L_ip y_p (one writer of r_i per panel)
      float yv[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) yv[k] = sr[8 * p + k];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) v = fmaf(T_(acc, r, k), yv[k], v);
        sr[8 * ti + r] -= v;
      }
    }
    __syncthreads();
    if (tj > p && ti >= tj && ti < NT) {
      // trailing update A_ij -= L_ip L_jp^T (two k-steps per iteration: the next step's
      // LDS reads overlap this step's FMAs)
#pragma unroll 2
      for (int k = 0; k < 8; ++k) {
        const float4_ a0 = *reinterpret_cast<const float4_*>(&sPT[ti][8 * k]);
        const float4_ a1 = *reinterpret_cast<const float4_*>(&sPT[ti][8 * k + 4]);
        const float4_ b0 = *reinterpret_cast<const float4_*>(&sPT[tj][8 * k]);
        const float4_ b1 = *reinterpret_cast<const float4_*>(&sPT[tj][8 * k + 4]);
        const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const float2_ bp[4] = {float2_{b0.x, b0.y}, float2_{b0.z, b0.w}, float2_{b1.x, b1.y}, float2_{b1.z, b1.w}};
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
          for (int h = 0; h < 4; ++h)
            acc[r][h] = __builtin_elementwise_fma(float2_{-av[r], -av[r]}, bp[h], acc[r][h]);
      }
    }
  }

  __syncthreads();
  // ---- L^T x = y (backward) ----
  for (int p = NT - 1; p >= 0; --p) {
    if (ti == p && tj == p) {
      // back substitution L_pp^T x_p = r_p (L_pp is still in this thread's registers)
      float x[8];
#pragma unroll
      for (int c = 7; c >= 0; --c) {
        float v = sr[8 * p + c];
#pragma unroll
        for (int k = c + 1; k < 8; ++k) v = fmaf(-T_(acc, k, c), x[k], v);
        x[c] = v * sIdv[p][c];
      }
#pragma unroll
      for (int c = 0; c < 8; ++c) sr[8 * p + c] = x[c];
    }
    __syncthreads();
    if (ti == p && tj < p) {
      float xv[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) xv[k] = sr[8 * p + k];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float v = 0.f;
#pragma unroll
        for (int r = 0; r < 8; ++r) v = fmaf(T_(acc, r, c), xv[r], v);
        sr[8 * tj + c] -= v;
      }
    }
    __syncthreads();
  }
  if (tid < R) X[u * R + tid] = sr[tid];
}
#undef T_

// x = Q y for every listed row, in place (the Woodbury rows of an implicit half-iteration
// come out in the eigenbasis).  Q^T is staged once per block in LDS; each wave rotates 8
// rows at a time (rows staged in its LDS slice, lane l owns outputs l and l + 64), so
// every row is computed by the same instruction sequence whatever the row list holds --
// chunked (multi-rank) and whole-table solves give bit-identical factors.
constexpr int kRotRows = 8;

template <int R>
__global__ __launch_bounds__(256) void als_rotate_kernel(const float* __restrict__ QT, const int32_t* __restrict__ rows,
                                                         int64_t nrows, float* __restrict__ X) {
  constexpr int RV = (R + 63) / 64;
  __shared__ float sQ[R * R];                       // sQ[j R + c] = Q[c][j]
  __shared__ float sYb[4][kRotRows][R];
  for (int i = threadIdx.x; i < R * R; i += 256) sQ[i] = QT[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int64_t base = ((int64_t)blockIdx.x * 4 + wv) * kRotRows; base < nrows;
       base += (int64_t)gridDim.x * 4 * kRotRows) {
    int64_t rid[kRotRows];
#pragma unroll
    for (int r = 0; r < kRotRows; ++r) {
      const int64_t i = base + r;
      rid[r] = i < nrows ? (int64_t)rows[i] : -1;
#pragma unroll
      for (int h = 0; h < RV; ++h) {
        const int c = lane + 64 * h;
        if (c < R) sYb[wv][r][c] = rid[r] >= 0 ? X[rid[r] * R + c] : 0.f;
      }
    }
    float acc[kRotRows][RV];
#pragma unroll
    for (int r = 0; r < kRotRows; ++r)
#pragma unroll
      for (int h = 0; h < RV; ++h) acc[r][h] = 0.f;
    for (int j = 0; j < R; j += 4) {
      float q[4][RV];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int h = 0; h < RV; ++h) {
          const int c = lane + 64 * h;
          q[s4][h] = c < R ? sQ[(j + s4) * R + c] : 0.f;
        }
#pragma unroll
      for (int r = 0; r < kRotRows; ++r) {
        const float4_ y = *reinterpret_cast<const float4_*>(&sYb[wv][r][j]);
#pragma unroll
        for (int h = 0; h < RV; ++h)
          acc[r][h] = fmaf(y.w, q[3][h], fmaf(y.z, q[2][h], fmaf(y.y, q[1][h], fmaf(y.x, q[0][h], acc[r][h]))));
      }
    }
#pragma unroll
    for (int r = 0; r < kRotRows; ++r) {
      if (rid[r] < 0) continue;
#pragma unroll
      for (int h = 0; h < RV; ++h) {
        const int c = lane + 64 * h;
        if (c < R) X[rid[r] * R + c] = acc[r][h];
      }
    }
  }
}

}  // namespace

// Woodbury solves (rows with n_u <= 32 ratings and lam_u > 0).  P: the factor table
// rotated into the eigenbasis of G (F Q, implicit) or F itself (explicit, eig = 0);
// eig: the eigenvalues of G (zeros when explicit).  X row u receives y_u = D P_u^T z
// (implicit: the caller applies x = Q y) or x_u (explicit).
O3S_API int o3s_als_wood(int R, const int64_t* indptr, const int32_t* cols, const float* w, const float* b,
                         const float* P, const float* eig, const float* lam, const int32_t* small, int64_t nsmall,
                         float* X, hipStream_t st) {
  if (nsmall < 0 || !eig || !P) return -1;
  if (nsmall == 0) return 0;
  const dim3 grid((unsigned)((nsmall + kWW - 1) / kWW));
#define O3S_WD(RR)                                                                                          \
  if (R == RR) {                                                                                            \
    hipLaunchKernelGGL((als_wood_kernel<RR>), grid, dim3(kWW * 64), 0, st, indptr, cols, w, b, P, eig, lam, \
                       small, nsmall, X);                                                                   \
    O3S_CHECK_LAUNCH();                                                                                     \
    return 0;                                                                                               \
  }
  O3S_WD(32) O3S_WD(64) O3S_WD(96) O3S_WD(128)
#undef O3S_WD
  return -2;
}

// x = Q y in place for the listed rows (QT = Q^T row-major, R x R).
O3S_API int o3s_als_rotate(int R, const float* QT, const int32_t* rows, int64_t nrows, float* X, int grid,
                           hipStream_t st) {
  if (nrows < 0 || !QT || grid <= 0) return -1;
  if (nrows == 0) return 0;
#define O3S_RT(RR)                                                                                       \
  if (R == RR) {                                                                                         \
    hipLaunchKernelGGL((als_rotate_kernel<RR>), dim3(grid), dim3(256), 0, st, QT, rows, nrows, X);       \
    O3S_CHECK_LAUNCH();                                                                                  \
    return 0;                                                                                            \
  }
  O3S_RT(32) O3S_RT(64) O3S_RT(96) O3S_RT(128)
#undef O3S_RT
  return -2;
}

// Dense solves (any row): register Gram + LDS Cholesky.  implicit: G = Y^T Y (fp32 R x R).
O3S_API int o3s_als_dense(int implicit, int R, const int64_t* indptr, const int32_t* cols, const float* w,
                          const float* b, const float* F, const float* G, const float* lam, const int32_t* dense,
                          int64_t ndense, float* X, hipStream_t st) {
  if (ndense < 0 || (implicit && !G)) return -1;
  if (ndense == 0) return 0;
#define O3S_DN(RR)                                                                                            \
  if (R == RR) {                                                                                              \
    if (implicit)                                                                                             \
      hipLaunchKernelGGL((als_dense_kernel<RR, true>), dim3((unsigned)ndense), dim3(Dense<RR>::NTH), 0, st,   \
                         indptr, cols, w, b, F, G, lam, dense, X);                                            \
    else                                                                                                      \
      hipLaunchKernelGGL((als_dense_kernel<RR, false>), dim3((unsigned)ndense), dim3(Dense<RR>::NTH), 0, st,  \
                         indptr, cols, w, b, F, G, lam, dense, X);                                            \
    O3S_CHECK_LAUNCH();                                                                                       \
    return 0;                                                                                                 \
  }
  O3S_DN(32) O3S_DN(64) O3S_DN(96) O3S_DN(128)
#undef O3S_DN
  return -2;
}

O3S_API int o3s_als_exact_max_small() { return kNW; }
