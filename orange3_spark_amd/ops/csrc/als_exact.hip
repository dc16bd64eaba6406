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
//   v_pk_fma), S in registers (lane i owns row i), the Cholesky in 8-column panels (readlane
//   broadcasts inside a panel, the trailing rank-8 update on MFMA), solves by readlane.
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
// * als_dense_mfma_kernel (the default for long rows, ops/als.py DENSE_KERNEL): the same
//   solve on 32 x 32 tiles in MFMA accumulator layout -- Gram, panel products and trailing
//   updates on v_mfma_f32_32x32x2_f32, one wave per diagonal factorisation (see the
//   kernel's own comment).
//
// Both write x_u straight into the factor table.  fp32 throughout (the Gram / S sums are
// short: n_u terms).
#include "common.h"

using namespace o3s;

namespace {

typedef float f32x16_ __attribute__((ext_vector_type(16)));
typedef short bf16x8_ __attribute__((ext_vector_type(8)));
constexpr int kNW = 32;   // Woodbury path: rows with at most this many ratings
constexpr int kWW = 2;    // waves (rows) per Woodbury block
constexpr int kPS = 72;   // LDS row stride of a P' half tile (features 32 h + s at [36 h + s])

__device__ __forceinline__ float rl(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}

// S z = t for one Woodbury row (lane i holds row i of S in srow, t_i in t; n <= NM):
// right-looking Cholesky S = L L^T where step k needs only broadcasts -- the pivot and L's
// column k (L_mk, m > k) come from v_readlane, so the factorisation has no LDS round trip
// (publishing the column through LDS cost ~880 cycles per step: tools/als_wood_phases.py,
// profiles/als_wood_phases_r4.json); the forward solve L y = t rides along, column k of L
// goes to LDS (Lc[k][i] = L_ik) for the backward solve L^T z = y.  Steps k >= n are exact
// no-ops (rows and columns >= n of S are zero and t_i = 0 there: the clamped pivot gives
// L_kk = 1e-15, every other L entry and y_k are 0), so NM steps run with no branches.
// Returns z (lane i holds z_i).
// BLK: 8-column panels -- inside a panel the v_readlane rank-1 updates above, then the
// trailing columns take the panel's whole rank-8 update P = L21 L21^T from 4
// v_mfma_f32_32x32x2_f32 (A = B = the panel's L entries, lane l holding row l & 31 and
// k-slot l >> 5); P is symmetric, so the accumulator's column l & 31 is row l & 31 of P,
// split between lanes l and l ^ 32 (one ds_bpermute exchange per register).  Per trailing
// column: 2 VALU ops per panel instead of 16.  Lanes l >= 32 mirror rows l & 31 exactly
// (the MFMA reads their L entries).
template <int NM, bool BLK = false, int KN = kNW>
__device__ __forceinline__ float wood_factor_solve(float (&srow)[KN], float v, float (*Lc)[kNW + 1], int lane) {
  const int r = lane & 31;
  const int h = lane >> 5;
#pragma unroll
  for (int p = 0; p < NM / 8; ++p) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * p + j;
      const float piv = fmaxf(rl(srow[k], k), 1e-30f);
      const float id = __builtin_amdgcn_rsqf(piv);
      const float lik = r > k ? srow[k] * id : (r == k ? piv * id : 0.f);
      if (lane < kNW) Lc[k][lane] = lik;
      const float yk = rl(v, k) * id;
      v = r == k ? yk : (r > k ? fmaf(-lik, yk, v) : v);
#pragma unroll
      for (int m = k + 1; m < (BLK ? 8 * p + 8 : NM); ++m) srow[m] = fmaf(-lik, rl(lik, m), srow[m]);
    }
    if constexpr (BLK) {
      if (8 * p + 8 < NM) {
        f32x16_ acc;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const float a = Lc[8 * p + 2 * s2 + h][r];      // the panel's L, back from LDS
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, a, acc, 0, 0, 0);
        }
        // register q holds P[r][(q & 3) + 8 (q >> 2) + 4 h]; its partner lane the other half
#pragma unroll
        for (int q = 4 * (p + 1); q < 4 * (NM / 8); ++q) {
          const float mine = acc[q];
          const float other = __shfl_xor(mine, 32, 64);
          const int m0 = (q & 3) + 8 * (q >> 2);
          srow[m0] -= h ? other : mine;
          srow[m0 + 4] -= h ? mine : other;
        }
      }
    }
  }
  // backward, right-looking: z_k = v_k / L_kk, then v_i -= L_ki z_k for i < k (row k of L =
  // entries Lc[i][k]: lane i's column read, conflict-free at stride kNW + 1); the L entries
  // and the reciprocal diagonal are loaded up front, off the z chain
#pragma unroll
  for (int k = NM - 1; k >= 0; --k) {
    const float lki = Lc[r][k];
    const float zk = rl(v, k) * __builtin_amdgcn_rcpf(Lc[k][k]);
    v = r == k ? zk : (r < k ? fmaf(-lki, zk, v) : v);
  }
  return v;
}

// TIM (diagnostic build, o3s_als_wood_timed): lane 0 stamps the shader clock at the phase
// boundaries of each row -> timing[row][0..4] = gathers landed, S built (MFMA + LDS image),
// Cholesky, both solves, output (cycles; the gathers are waited for with vmcnt(0) there)
// WOCC: waves per SIMD the register budget must allow (3: 168 VGPRs, no spill).
// (a 4-waves-per-SIMD build spilled and measured 8.6% slower; S = P D P^T as bf16x3 on
// 32x32x16 MFMAs measured 4% slower; persistent waves prefetching the next row's metadata
// measured 14% slower: profiles/kernel_experiments_r4.json)
// KN: the longest row of the launch (32, or 16 for the launch of the short rows: half the
// P registers, and S on v_mfma_f32_16x16x4_f32 -- a quarter of the matrix-pipe cycles)
template <int R, bool TIM = false, int WOCC = 3, bool BLK = false, int KN = kNW>
__global__ __launch_bounds__(kWW * 64, WOCC) void als_wood_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ cols, const float* __restrict__ w,
    const float* __restrict__ b, const float* __restrict__ P, const float* __restrict__ eig,
    const float* __restrict__ lam, const int32_t* __restrict__ rows, int64_t nlist, float* __restrict__ X,
    int64_t* __restrict__ timing = nullptr) {
  int64_t tm[6] = {0, 0, 0, 0, 0, 0};
  if constexpr (TIM) tm[0] = clock64();
  static_assert(R % 32 == 0 && R <= 128, "rank must be a multiple of 32, at most 128");
  constexpr int RV = (R + 63) / 64;              // columns per lane (1 or 2)
  // per wave: the sqrt(D)-scaled rows P' for the MFMA (32 x kPS floats), later reused for
  // the S image and L by columns (Lc[k][i] = L_ik)
  // (KN = 16: 16 staged rows; the 32 x 33 S / L image, 1056 floats, still fits in 16 x kPS)
  __shared__ __attribute__((aligned(16))) float sP[kWW][(KN == 16 ? 16 : kNW) * kPS];
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
  int ci[KN];                                    // all broadcasts before the first gather
#pragma unroll
  for (int i = 0; i < KN; ++i) ci[i] = __builtin_amdgcn_readlane(myc, i);
  float2_ acc[KN];
#pragma unroll
  for (int i = 0; i < KN; ++i) {
    acc[i] = float2_{0.f, 0.f};
    if (i < n) {
      const int64_t c = ci[i];
      acc[i].x = c0ok ? P[c * R + lane] : 0.f;
      acc[i].y = c1ok ? P[c * R + lane + 64] : 0.f;
    }
  }

  if constexpr (TIM) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tm[1] = clock64();
  }
  // S = P D P^T = P' P'^T with P' = P sqrt(D), on the matrix cores: each 64-feature half of
  // the rows goes through a 9 KB LDS tile (lane l of the MFMA needs row l & 31), then 32
  // v_mfma_f32_32x32x2_f32 per half accumulate the 32 x 32 product in fp32 (feature
  // 32 h + s in k-slot h of step s -- the same value for the A and B operands), on two
  // accumulator chains.  Rows >= n are zero.
  const float2_ sq = {sqrtf(dd.x), sqrtf(dd.y)};
  float* sp = sP[wv];
  const int wcol = lane < 32 ? lane : lane + 4;
  float srow[KN];
  if constexpr (KN == 16) {
    // 16 x 16 S: lane l feeds row l & 15, k-slot g = l >> 4 = features 16 g + s of the half
    // (s = 0..15); rows 16..31 of the image are never read (those lanes' srow is zero, so
    // their L entries are exact zeros)
    const int g = lane >> 4;
    const float* rq = sp + (lane & 15) * kPS + 16 * g + (g >> 1) * 4;
    float4_ sb0 = {0.f, 0.f, 0.f, 0.f}, sb1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int hf = 0; hf < RV; ++hf) {
#pragma unroll
      for (int i = 0; i < 16; ++i) sp[i * kPS + wcol] = hf == 0 ? acc[i].x * sq.x : acc[i].y * sq.y;
#pragma unroll
      for (int s4 = 0; s4 < 16; s4 += 4) {
        const float4_ x = *reinterpret_cast<const float4_*>(rq + s4);
        sb0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, x.x, sb0, 0, 0, 0);
        sb1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, x.y, sb1, 0, 0, 0);
        sb0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, x.z, sb0, 0, 0, 0);
        sb1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, x.w, sb1, 0, 0, 0);
      }
    }
    const float4_ sc = sb0 + sb1;
#pragma unroll
    for (int q = 0; q < 4; ++q) S[4 * g + q][lane & 15] = sc[q];   // column lane & 15, row 4 g + q
    if (lane < 16) S[lane][lane] += winv;
    const bool rok = (lane & 31) < 16;
#pragma unroll
    for (int m = 0; m < 16; ++m) srow[m] = rok ? S[lane & 31][m] : 0.f;
  } else {
  f32x16_ sa0, sa1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    sa0[r] = 0.f;
    sa1[r] = 0.f;
  }
  const float* rp = sp + (lane & 31) * kPS + (lane >> 5) * 36;
#pragma unroll
  for (int hf = 0; hf < RV; ++hf) {
#pragma unroll
    for (int i = 0; i < kNW; ++i)
      sp[i * kPS + wcol] = i >= KN ? 0.f : (hf == 0 ? acc[i < KN ? i : 0].x * sq.x : acc[i < KN ? i : 0].y * sq.y);
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
#pragma unroll
  for (int m = 0; m < KN; ++m) srow[m] = S[lane & 31][m];
  }
  if constexpr (TIM) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    tm[2] = clock64();
  }

  // Cholesky + both triangular solves in registers (wood_factor_solve): NM = the row length
  // rounded up to 8, so the fully unrolled steps keep every register index constant and
  // carry no per-step branches
  float (*Lc)[kNW + 1] = S;                      // Lc[k][i] = L_ik
  float v = t;
  if (n <= 8) v = wood_factor_solve<8, BLK, KN>(srow, t, Lc, lane);
  else if (KN == 16 || n <= 16) v = wood_factor_solve<16, BLK, KN>(srow, t, Lc, lane);
  else if constexpr (KN == 24) {
    v = wood_factor_solve<24, BLK, KN>(srow, t, Lc, lane);
  } else if constexpr (KN == 32) {
    if (n <= 24) v = wood_factor_solve<24, BLK, KN>(srow, t, Lc, lane);
    else v = wood_factor_solve<32, BLK, KN>(srow, t, Lc, lane);
  }
  if constexpr (TIM) tm[3] = clock64();
  if constexpr (TIM) tm[4] = clock64();
  // y = D P^T z: the solution in the eigenbasis (implicit; the host rotates x = Q y for all
  // Woodbury rows) or x itself (explicit, Q = I)
  float2_ uu = {0.f, 0.f};
#pragma unroll
  for (int i = 0; i < KN; ++i) {
    if (i < n) {
      const float zi = rl(v, i);
      uu = __builtin_elementwise_fma(float2_{zi, zi}, acc[i], uu);
    }
  }
  uu = uu * dd;
  float* xo = X + u * R;
  if (c0ok) xo[lane] = uu.x;
  if (c1ok) xo[lane + 64] = uu.y;
  if constexpr (TIM) {
    tm[5] = clock64();
    if (lane == 0)
      for (int k = 0; k < 5; ++k) timing[li * 5 + k] = tm[k + 1] - tm[k];
  }
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

// x = Q y on the matrix cores (R = 128): a block takes 32 listed rows at a time, stages
// them in LDS (row stride 130 floats: the MFMA operand reads of 32 rows x 2 columns fall
// on 64 different banks), and wave w computes output columns [32 w, 32 w + 32) as 64
// v_mfma_f32_32x32x2_f32 steps (exact fp32 products) with its B operand -- column block w
// of Q^T, 64 values per lane -- held in registers for the whole launch.  The next tile's
// rows are loaded into registers while the current tile's MFMAs run.  Every row is computed
// by the same instruction sequence whatever the list holds (chunked and whole-table solves
// agree bitwise).  Rows are rewritten in place: a tile's rows are all staged before any is
// written.
constexpr int kRotStride = 130;
// Y: the source rows (Y == X: in place; the rotated table F Q reads F, writes FQ).
__global__ __launch_bounds__(256, 2) void als_rotate_mfma_kernel(const float* __restrict__ QT,
                                                                 const int32_t* __restrict__ rows, int64_t nrows,
                                                                 const float* Y, float* X) {
  __shared__ __attribute__((aligned(16))) float sY[32 * kRotStride];
  __shared__ int64_t sRid[32];                          // the tile's row ids (-1: past the list)
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 31, h = lane >> 5;
  float bq[64];                                         // B operand: Q^T[2 s + h][32 wid + c]
#pragma unroll
  for (int st = 0; st < 64; ++st) bq[st] = QT[(2 * st + h) * 128 + 32 * wid + c];
  // tile staging: thread t loads row t >> 3, columns 16 (t & 7) .. + 16 (4 float4)
  const int lr = threadIdx.x >> 3, lc = 16 * (threadIdx.x & 7);
  const int64_t ntiles = (nrows + 31) / 32;
  auto load = [&](int64_t tile, float4_ (&o)[4], int64_t& rid) {
    const int64_t i = tile * 32 + lr;
    rid = i < nrows ? (int64_t)rows[i] : -1;
    const int64_t rr = rid >= 0 ? rid : (int64_t)rows[nrows - 1];   // in bounds; never written
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = *reinterpret_cast<const float4_*>(Y + rr * 128 + lc + 4 * k);
  };
  float4_ nx[4];
  int64_t nrid = -1;
  int64_t tile = blockIdx.x;
  if (tile < ntiles) load(tile, nx, nrid);
  for (; tile < ntiles; tile += gridDim.x) {
    // stage this tile (float2 stores: rows start 8-B aligned at stride 130)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float2_* d = reinterpret_cast<float2_*>(sY + lr * kRotStride + lc + 4 * k);
      d[0] = float2_{nx[k].x, nx[k].y};
      d[1] = float2_{nx[k].z, nx[k].w};
    }
    if ((threadIdx.x & 7) == 0) sRid[lr] = nrid;
    __syncthreads();
    if (tile + gridDim.x < ntiles) load(tile + gridDim.x, nx, nrid);
    f32x16_ acc;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = 0.f;
    const float* ya = sY + c * kRotStride + h;
#pragma unroll
    for (int st = 0; st < 64; ++st) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ya[2 * st], bq[st], acc, 0, 0, 0);
    // outputs: register v -> row (v & 3) + 8 (v >> 2) + 4 h of the tile, column 32 wid + c
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int64_t ri = sRid[(v & 3) + 8 * (v >> 2) + 4 * h];
      if (ri >= 0) X[ri * 128 + 32 * wid + c] = acc[v];
    }
    __syncthreads();                                    // sY reused by the next tile
  }
}

template <int R>
__global__ __launch_bounds__(256) void als_rotate_kernel(const float* __restrict__ QT, const int32_t* __restrict__ rows,
                                                         int64_t nrows, const float* Y, float* X) {
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
        if (c < R) sYb[wv][r][c] = rid[r] >= 0 ? Y[rid[r] * R + c] : 0.f;
      }
    }
    if constexpr (RV == 2) {
      // lane l owns the output pair (l, l + 64): one v_pk_fma_f32 per (row, j) with the
      // row's y_j broadcast -- half the FMA issue of the scalar form below
      float2_ acc2[kRotRows];
#pragma unroll
      for (int r = 0; r < kRotRows; ++r) acc2[r] = float2_{0.f, 0.f};
      for (int j = 0; j < R; j += 4) {
        float2_ q2[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
          q2[s4] = float2_{sQ[(j + s4) * R + lane], lane + 64 < R ? sQ[(j + s4) * R + lane + 64] : 0.f};
#pragma unroll
        for (int r = 0; r < kRotRows; ++r) {
          const float4_ y = *reinterpret_cast<const float4_*>(&sYb[wv][r][j]);
          float2_ a = acc2[r];
          a = __builtin_elementwise_fma(float2_{y.x, y.x}, q2[0], a);
          a = __builtin_elementwise_fma(float2_{y.y, y.y}, q2[1], a);
          a = __builtin_elementwise_fma(float2_{y.z, y.z}, q2[2], a);
          a = __builtin_elementwise_fma(float2_{y.w, y.w}, q2[3], a);
          acc2[r] = a;
        }
      }
#pragma unroll
      for (int r = 0; r < kRotRows; ++r) {
        if (rid[r] < 0) continue;
        X[rid[r] * R + lane] = acc2[r].x;
        if (lane + 64 < R) X[rid[r] * R + lane + 64] = acc2[r].y;
      }
      continue;
    }
    float acc[kRotRows][RV];
#pragma unroll
    for (int r = 0; r < kRotRows; ++r)
#pragma unroll
      for (int h = 0; h < RV; ++h) acc[r][h] = 0.f;
    // (bounded unroll: the fully unrolled loop hoisted every LDS read and spilled at R = 64)
#pragma unroll 2
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

// ---------------------------------------------------------------------------------
// als_dense_mfma_kernel: the dense solve of als_dense_kernel on the matrix cores, for
// long rows (the item side: ~200 ratings per row at rank 128).  The VALU kernel above is
// issue-bound -- its 8 x 8 register tiles leave most lanes idle in the panel and diagonal
// steps, and the Gram costs ~R^2/64 packed FMAs per rating per thread.  Here the system is
// held as 32 x 32 tiles in MFMA accumulator layout (lane l: column l & 31, rows
// (v & 3) + 8 (v >> 2) + 4 (l >> 5) in register v), upper triangle only (tile (j, i),
// j <= i, holds A[32 j.., 32 i..]), dealt round robin to min(4, #tiles) waves:
//   Gram   S_ji += sum_c w_c y_c[j] y_c[i]^T      v_mfma_f32_32x32x2_f32, two ratings per
//          instruction (exact fp32 products, the fmaf-chain numerics of the VALU kernel),
//          both operands one LDS read of the staged factor rows;
//   per 32-wide panel p (block Cholesky A = U^T U, U_pp = L_pp^T):
//     A  the owner of (p, p) stages it through LDS and factors it with one wave (lane i
//        holds row i; column c's multipliers broadcast by v_readlane).  The SAME
//        right-looking recurrence run on an identity right-hand side (lanes 0-31) and on
//        the current rhs block (lanes 32-63) yields X_p = L_pp^-1 (column q on lane q) and
//        y_p = L_pp^-1 r_p at no extra broadcast cost;
//     B  U_pi = X_p S_pi: 16 MFMAs whose B operand is the owner's own accumulator
//        register v (the k index pairs rows (v&3)+8(v>>2) and +4 -- any pairing works if
//        both operands agree), A operand X_p from LDS; U_pi is published as a row panel
//        and r_i -= U_pi^T y_p (a sum over the tile's own registers + one lane swap);
//     C  trailing S_ji -= U_pj^T U_pi: 16 MFMAs with both operands read from the panel;
//   backward U x = y: per p, owners of (p, i > p) form U_pi x_i (row sums through a
//   per-wave LDS transpose), the diagonal owner applies x_p = X_p^T (y_p - sum).
// Two block barriers per panel; R = 32 NT, NT <= 4.
template <int R>
struct DenseM {
  static constexpr int NT = R / 32;
  static constexpr int NL = NT * (NT + 1) / 2;          // upper-triangle tiles
  static constexpr int W = NL < 4 ? NL : 4;              // waves per block
  static constexpr int MT = (NL + W - 1) / W;            // tiles per wave
  static constexpr int NTH = 64 * W;
  static constexpr int CH = 16;                          // ratings staged per round
  static constexpr int PNS = R == 32 ? 32 : (R == 96 ? 96 : R - 32);   // panel row stride (floats)
  static constexpr int TS = 32 * 33;                     // one padded 32 x 32 tile in LDS
  static constexpr int SA0 = CH * R > 32 * PNS ? CH * R : 32 * PNS;
  static constexpr int SA1 = SA0 > W * TS ? SA0 : W * TS;
  static constexpr int SA = SA1 > R * 48 ? SA1 : R * 48;   // staging / panel / backward scratch
  static constexpr int LDS = SA + TS + NT * TS + R + 2 * CH + W * 32;
  // glds ring layout (GL, R = 128): the factor rows of DEP Gram steps land in LDS by
  // LDS-DMA (no VGPRs hold in-flight gathers); the ring shares its region with the diagonal
  // staging / X_p images, which are only used after the Gram.  IC = rating indices staged
  // per chunk (one refill per IC ratings).
  static constexpr int DEP = 3, IC = 128;
  static constexpr int XR = TS + NT * TS > DEP * CH * R ? TS + NT * TS : DEP * CH * R;
  static constexpr int LDSG = SA + XR + R + 2 * CH + W * 32 + 3 * IC + 2 * DEP * CH;
};

template <int R, bool IMPL, bool BLK, bool TIM = false, bool GL = false>
__global__ __launch_bounds__(DenseM<R>::NTH, BLK ? 3 : 1) void als_dense_mfma_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ cols, const float* __restrict__ w,
    const float* __restrict__ b, const float* __restrict__ F, const float* __restrict__ G,
    const float* __restrict__ lam, const int32_t* __restrict__ rows, float* __restrict__ X,
    int64_t* __restrict__ timing = nullptr) {
  // TIM (diagnostic build, o3s_als_dense_mfma_timed): thread 0 stamps the shader clock at
  // the block-synchronised phase boundaries -> timing[block][0..5] = Gram, diagonal
  // factors, panel products, trailing updates (wave 0's share), backward, total (cycles)
  int64_t tm0 = 0, tmA = 0, tmB = 0, tmC = 0, tmG = 0, tmP = 0;
  if constexpr (TIM) tm0 = tmP = clock64();
  using D = DenseM<R>;
  constexpr int NT = D::NT, NL = D::NL, W = D::W, MT = D::MT, NTH = D::NTH, CH = D::CH, PNS = D::PNS,
                TS = D::TS;
  constexpr bool G3 = BLK && W == 4;     // bf16x3 Gram (16 staging threads per rating)
  constexpr bool GLP = GL && G3 && R == 128;   // factor-row gathers by LDS-DMA into a ring
  __shared__ __attribute__((aligned(16))) float lds[GLP ? D::LDSG : D::LDS];
  float* const sY = lds;                 // Gram: staged factor rows [CH][R]
  float* const sPn = lds;                // factor: row panel [32][PNS]
  float* const sScr = lds;               // backward: per-wave transpose [W][32][33]
  float* const sD = lds + D::SA;         // diagonal tile staging [32][33]
  float* const sX = sD + TS;             // X_p = L_pp^-1, every p: [NT][32][33]
  float* const sr = GLP ? lds + D::SA + D::XR : sX + NT * TS;   // rhs -> y -> x
  float* const sW = sr + R;
  float* const sB = sW + CH;
  float* const sWp = sB + CH;            // backward partial sums [W][32]
  const int tid = threadIdx.x;
  const int lane = tid & 63, h = lane >> 5, q = lane & 31;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t u = rows[blockIdx.x];
  const int64_t p0 = indptr[u], p1 = indptr[u + 1];
  const float lu = lam[u];

  // this wave's tiles: t = wid + s W, upper-triangle order (0,0), (0,1), .., (1,1), ..
  int tj[MT], ti[MT];
#pragma unroll
  for (int s = 0; s < MT; ++s) {
    int t = wid + s * W, j = 0;
    if (t < NL) {
      while (t >= NT - j) { t -= NT - j; ++j; }
      tj[s] = j;
      ti[s] = j + t;
    } else {
      tj[s] = ti[s] = NT;                  // no tile
    }
  }
  f32x16_ acc[MT];
#pragma unroll
  for (int s = 0; s < MT; ++s)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[s][v] = 0.f;

  // ---- Gram ----
  // G3 (blocked variant, 4-wave blocks): sqrt(w_c) y_c split into bf16 hi + lo, staged
  // TRANSPOSED ([R][24] bf16, rating fastest, double-buffered) so one 16-B LDS read is an
  // MFMA fragment; per 16 ratings and tile 3 v_mfma_f32_32x32x16_bf16 (hi.hi + lo.hi +
  // hi.lo, ~2^-16 relative: the als_gram_kernel numerics) -- 96 MFMA cycles where the f32
  // path spends 8 x 64.  The staging threads (16 per rating, R/16 elements each) also
  // accumulate the rhs in fp32.
  float rhs_t = 0.f;
  if constexpr (G3) {
    // staging map (conflict-free transposed stores): lane = (r_low = dim within a 16-dim
    // block, kp_low = rating pair 0..3); a thread owns ITEMS (dim block, pair group) items
    // and writes each item as ONE dword (ratings 2kp, 2kp + 1 of dim r) at dword 12 r + kp:
    // banks 12 r_low + kp_low (+ 0 mod 64) are all different across the wave.  Its global
    // loads are 64-B runs of one factor row per 16 lanes.
    constexpr int LDT = 24, NRB = R / 16, ITEMS = NRB / 2;   // 2 NRB items over 4 waves
    uint16_t* const sT = reinterpret_cast<uint16_t*>(lds);    // [buf][hi|lo][R][LDT]
    const int r_low = lane & 15, kp_low = lane >> 4;
    float y0[ITEMS], y1[ITEMS], rh[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) rh[i] = 0.f;
    auto item_r = [&](int i) { return 16 * ((wid + 4 * i) % NRB) + r_low; };
    // item i's rating-pair group, as a wave-uniform bool: indexing the [2] arrays with a
    // runtime subscript puts them in scratch memory
    auto item_k1 = [&](int i) { return (wid + 4 * i) >= NRB; };
    // A step's rating indices / weights are loaded with the index clamped to the row's last
    // rating, so every load is unconditional and in bounds; ratings past the end are zeroed
    // in store() through their weights (w = b = 0 -> z = 0, no rhs term), not by selecting
    // on the loaded values -- a select right after a gather makes the compiler wait for it
    // there, before the step's MFMAs.  The indices run one step ahead of their gathers.
    struct Idx { int32_t c[2][2]; float w[2][2], b[2][2]; };
    auto load_idx = [&](int64_t jb, Idx& o) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int par = 0; par < 2; ++par) {
          const int64_t j = jb + 2 * (4 * kb + kp_low) + par;
          const int64_t jc = j < p1 ? j : p1 - 1;
          o.c[kb][par] = cols[jc];
          o.w[kb][par] = w[jc];
          o.b[kb][par] = b[jc];
        }
    };
    auto load_f = [&](const Idx& o) {
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const bool k1 = item_k1(i);
        const int r = item_r(i);
        const int64_t c0 = k1 ? o.c[1][0] : o.c[0][0], c1 = k1 ? o.c[1][1] : o.c[0][1];
        y0[i] = F[c0 * R + r];
        y1[i] = F[c1 * R + r];
      }
    };
    auto store = [&](int buf, const Idx& o, int64_t jb) {
      uint32_t* const th = reinterpret_cast<uint32_t*>(sT + buf * 2 * R * LDT);
      uint32_t* const tl = th + R * LDT / 2;
      float sq[2][2], bv[2][2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int par = 0; par < 2; ++par) {
          const bool ok = jb + 2 * (4 * kb + kp_low) + par < p1;
          sq[kb][par] = ok ? sqrtf(fmaxf(o.w[kb][par], 0.f)) : 0.f;
          bv[kb][par] = ok ? o.b[kb][par] : 0.f;
        }
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const bool k1 = item_k1(i);
        const int kb = k1 ? 1 : 0, r = item_r(i);
        const float s0 = k1 ? sq[1][0] : sq[0][0], s1 = k1 ? sq[1][1] : sq[0][1];
        const float b0 = k1 ? bv[1][0] : bv[0][0], b1 = k1 ? bv[1][1] : bv[0][1];
        rh[i] = fmaf(b1, y1[i], fmaf(b0, y0[i], rh[i]));
        const float z0 = s0 * y0[i], z1 = s1 * y1[i];
        const uint16_t h0 = f32_to_bf16(z0), h1 = f32_to_bf16(z1);
        const uint16_t l0 = f32_to_bf16(z0 - bf16_to_f32(h0)), l1 = f32_to_bf16(z1 - bf16_to_f32(h1));
        const int dw = r * (LDT / 2) + 4 * kb + kp_low;
        th[dw] = (uint32_t)h0 | ((uint32_t)h1 << 16);
        tl[dw] = (uint32_t)l0 | ((uint32_t)l1 << 16);
      }
    };
    const int nsteps = (int)((p1 - p0 + CH - 1) / CH);
    auto gram_step = [&](int buf) {
      const uint16_t* th = sT + buf * 2 * R * LDT + q * LDT + 8 * h;
      const uint16_t* tl = th + R * LDT;
#pragma unroll
      for (int s = 0; s < MT; ++s) {
        if (tj[s] >= NT) continue;
        const bf16x8_ ah = *reinterpret_cast<const bf16x8_*>(th + 32 * tj[s] * LDT);
        const bf16x8_ al = *reinterpret_cast<const bf16x8_*>(tl + 32 * tj[s] * LDT);
        const bf16x8_ bh = *reinterpret_cast<const bf16x8_*>(th + 32 * ti[s] * LDT);
        const bf16x8_ bl = *reinterpret_cast<const bf16x8_*>(tl + 32 * ti[s] * LDT);
        acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[s], 0, 0, 0);
        acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[s], 0, 0, 0);
        acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[s], 0, 0, 0);
      }
    };
    // (gathers issued two steps ahead with two register sets measured no faster: 0.1233 vs
    // 0.1224 s per rank-of-8 iteration, profiles/kernel_experiments_r4.json)
    if constexpr (GLP) {
      // ---- LDS-DMA ring: the gathers of step s + DEP are issued while step s's MFMAs and
      // step s + 1's conversion run, so DEP - 1 steps of factor rows (16 KB per block) stay
      // in flight across the barriers with no VGPR holding them.  Each wave gathers 4 of a
      // step's 16 rows as 2 global_load_lds_dwordx4 (one row = 32 lanes x 16 B; the DMA image
      // is lane-linear, rows contiguous).  The rating indices come from an LDS chunk, so no
      // ordinary global load is consumed while a DMA is outstanding (hipcc would drain the
      // ring with vmcnt(0) there); only the chunk refill, once per IC ratings, drains it.
      // Barriers are raw s_barrier + lgkmcnt(0): __syncthreads()' fence would wait vmcnt(0).
      constexpr int DEP = D::DEP, IC = D::IC;
      float* const ring = lds + D::SA;                                  // [DEP][CH][R]
      int32_t* const sCi = reinterpret_cast<int32_t*>(sWp + W * 32);    // index chunk [IC]
      float* const sWc = reinterpret_cast<float*>(sCi + IC);            // w of the chunk
      float* const sBc = sWc + IC;                                      // b of the chunk
      float* const sWs = sBc + IC;                                      // per slot: sqrt(w), 0 past the row
      float* const sBs = sWs + DEP * CH;                                // per slot: b, 0 past the row
      auto bar = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      };
      int64_t cb = -(int64_t)IC - 1;       // first rating of the staged chunk (block-uniform)
      auto issue = [&](int s) {
        const int64_t j0 = p0 + (int64_t)s * CH;
        if (j0 >= cb + IC) {               // chunks start at step boundaries (IC % CH == 0)
          cb = j0;
          if (tid < IC) {
            const int64_t j = j0 + tid < p1 ? j0 + tid : p1 - 1;
            sCi[tid] = cols[j];
            sWc[tid] = w[j];
            sBc[tid] = b[j];
          }
          bar();
        }
        const int slot = s % DEP, o = (int)(j0 - cb);
        if (tid < CH) {
          const bool ok = j0 + tid < p1;
          sWs[slot * CH + tid] = ok ? sqrtf(fmaxf(sWc[o + tid], 0.f)) : 0.f;
          sBs[slot * CH + tid] = ok ? sBc[o + tid] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int rr = 4 * wid + 2 * k;                               // wave-uniform
          const int64_t c = sCi[o + rr + h];                            // clamped at refill
          __builtin_amdgcn_global_load_lds(F + c * R + 4 * q, ring + (slot * CH + rr) * R, 16, 0, 0);
        }
      };
      auto convert = [&](const float* __restrict__ rg, const float* __restrict__ ws,
                         const float* __restrict__ bs, uint16_t* __restrict__ dst) {
        uint32_t* const th = reinterpret_cast<uint32_t*>(dst);
        uint32_t* const tl = th + R * LDT / 2;
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
          const int kb = item_k1(i) ? 1 : 0, r = item_r(i);
          const int c0 = 2 * (4 * kb + kp_low);
          const float u0 = rg[c0 * R + r], u1 = rg[(c0 + 1) * R + r];
          const float s0 = ws[c0], s1 = ws[c0 + 1];
          rh[i] = fmaf(bs[c0 + 1], u1, fmaf(bs[c0], u0, rh[i]));
          const float z0 = s0 * u0, z1 = s1 * u1;
          const uint16_t h0 = f32_to_bf16(z0), h1 = f32_to_bf16(z1);
          const uint16_t l0 = f32_to_bf16(z0 - bf16_to_f32(h0)), l1 = f32_to_bf16(z1 - bf16_to_f32(h1));
          const int dw = r * (LDT / 2) + 4 * kb + kp_low;
          th[dw] = (uint32_t)h0 | ((uint32_t)h1 << 16);
          tl[dw] = (uint32_t)l0 | ((uint32_t)l1 << 16);
        }
      };
      auto conv = [&](int s) {
        const int slot = s % DEP;
        convert(ring + slot * CH * R, sWs + slot * CH, sBs + slot * CH, sT + (s & 1) * 2 * R * LDT);
      };
      if (nsteps > 0) {
        issue(0);
        if (nsteps > 1) issue(1);
        if (nsteps > 2) issue(2);
        if (nsteps > 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if (nsteps > 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();                                                          // step 0 landed
        conv(0);
        if (nsteps > 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();                                                          // step 1 landed, sT[0] ready
      }
      for (int st = 0; st < nsteps; ++st) {
        gram_step(st & 1);
        if (st + 1 < nsteps) conv(st + 1);
        if (st + DEP < nsteps) {
          issue(st + DEP);                 // into the slot step st vacated
          asm volatile("s_waitcnt vmcnt(2)" ::: "memory");             // step st + 2 landed
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar();
      }
    } else {
    Idx nxt;
    if (nsteps > 0) {
      Idx o;
      load_idx(p0, o);
      load_f(o);
      load_idx(p0 + CH, nxt);
      store(0, o, p0);
    }
    __syncthreads();
    for (int st = 0; st < nsteps; ++st) {
      const int buf = st & 1;
      const bool more = st + 1 < nsteps;
      const int64_t jn = p0 + (int64_t)(st + 1) * CH;
      const Idx cur = nxt;                 // step st + 1's indices (loaded a step ago)
      if (more) {
        load_f(cur);
        load_idx(jn + CH, nxt);
      }
      gram_step(buf);
      if (more) store(buf ^ 1, cur, jn);
      __syncthreads();
    }
    }
    // rhs: sum the item partials over the 4 rating-pair lanes, then over the 2 pair groups
    float* const rpart = lds;                                  // [2][R], staging is done
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      float t = rh[i];
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      if (kp_low == 0) rpart[(item_k1(i) ? R : 0) + item_r(i)] = t;
    }
    __syncthreads();
    if (tid < R) rhs_t = rpart[tid] + rpart[R + tid];
  } else {
    // f32 path: rounds of CH ratings staged through LDS, next round in registers
    constexpr int PF = (CH * R + NTH - 1) / NTH;
    float pf[PF];
    float pw = 0.f, pb = 0.f;
    auto issue = [&](int64_t c0) {
      const int m = (int)(p1 - c0 < CH ? p1 - c0 : CH);
      int cidx[PF];
  #pragma unroll
      for (int k = 0; k < PF; ++k) {
        const int e = tid + k * NTH;
        const int c = e / R < m ? e / R : m - 1;
        cidx[k] = cols[c0 + c];
      }
      // rows >= m hold a copy of row m - 1 (finite), not zeros: their weights are 0, and a
      // select on the loaded value would make the compiler wait for the gather right here
      // instead of after the round's MFMAs
  #pragma unroll
      for (int k = 0; k < PF; ++k) {
        const int e = tid + k * NTH;
        pf[k] = F[(int64_t)cidx[k] * R + e % R];
      }
      pw = 0.f;
      pb = 0.f;
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
      for (int k = 0; k < PF; ++k) {
        const int e = tid + k * NTH;
        if (e < CH * R) sY[e] = pf[k];         // rows >= m: zero weight
      }
      if (tid < CH) {
        sW[tid] = pw;
        sB[tid] = pb;
      }
      __syncthreads();
      if (c0 + CH < p1) issue(c0 + CH);
  #pragma unroll 2
      for (int k = 0; k < (m + 1) >> 1; ++k) {
        const int c = 2 * k + h;               // ratings 2k (lanes 0-31) and 2k + 1 (lanes 32-63)
        const float wc = sW[c];
        const float* yc = sY + c * R + q;
  #pragma unroll
        for (int s = 0; s < MT; ++s)
          if (tj[s] < NT) acc[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(yc[32 * tj[s]], yc[32 * ti[s]] * wc, acc[s], 0, 0, 0);
      }
      if (tid < R)
        for (int c = 0; c < m; ++c) rhs = fmaf(sB[c], sY[c * R + tid], rhs);
      __syncthreads();
    }
    rhs_t = rhs;
  }
#pragma unroll
  for (int s = 0; s < MT; ++s) {
    if (tj[s] >= NT) continue;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int r = (v & 3) + 8 * (v >> 2) + 4 * h;
      float a = acc[s][v];
      if (IMPL) a += G[(32 * tj[s] + r) * R + 32 * ti[s] + q];
      if (tj[s] == ti[s] && r == q) a += lu;
      acc[s][v] = a;
    }
  }
  if (tid < R) sr[tid] = rhs_t;
  __syncthreads();
  if constexpr (TIM) { const int64_t t = clock64(); tmG = t - tm0; tmP = t; }

  // ---- block Cholesky A = U^T U with the forward solve U^T y = rhs riding along ----
  for (int p = 0; p < NT; ++p) {
    // A: factor the diagonal tile (one wave; lane i and i + 32 hold row i).  The slot is
    // resolved first so the factorisation is emitted once, not once per tile slot.
    int ds = -1;
#pragma unroll
    for (int s = 0; s < MT; ++s)
      if (tj[s] == p && ti[s] == p) ds = s;
    if (ds >= 0) {
#pragma unroll
      for (int s = 0; s < MT; ++s)
        if (s == ds)
#pragma unroll
          for (int v = 0; v < 16; ++v) sD[((v & 3) + 8 * (v >> 2) + 4 * h) * 33 + q] = acc[s][v];
      if constexpr (BLK) {
        // lanes 0-31: row q of the tile (-> row q of L); lanes 32-63: column q of the
        // identity (-> column q of X_p = L_pp^-1) -- ONE register array for both, since
        // the right-looking updates of a row of A and of a column of X are the same FMA
        // with the lane's own multiplier (L[q][c], resp. x_c) times L[j][c].  Columns go in
        // blocks of 4: inside a block the multipliers L[j][c] of the block's rows come
        // from v_readlane, the update of the later columns is deferred to one rank-4 step
        // whose multipliers arrive as one float4 LDS broadcast per row (8 LDS round trips
        // per tile instead of 32).  y_p = X_p r_p afterwards, from the X image in LDS.
        float v[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) v[k] = h ? (k == q ? 1.f : 0.f) : sD[q * 33 + k];
        float4_* const sC4 = reinterpret_cast<float4_*>(sD);   // free once the rows are loaded
#pragma unroll
        for (int c0 = 0; c0 < 32; c0 += 4) {
#pragma unroll
          for (int c = c0; c < c0 + 4; ++c) {
            const float piv = fmaxf(rl(v[c], c), 1e-30f);
            const float t = v[c] * __builtin_amdgcn_rsqf(piv);   // L[q][c] / x_c
            v[c] = t;
#pragma unroll
            for (int j = c + 1; j < c0 + 4; ++j) v[j] = fmaf(-t, rl(t, j), v[j]);
          }
          if (c0 + 4 < 32) {
            // every lane stores (an exec-masked store makes the compiler keep all 28 rows'
            // broadcasts live across the block: 234 instead of 64 VGPRs); lanes 32-63 hold
            // x values and park them in slots 32-63, which are never read
            sC4[lane] = float4_{v[c0], v[c0 + 1], v[c0 + 2], v[c0 + 3]};
#pragma unroll
            for (int j = c0 + 4; j < 32; ++j) {
              const float4_ l4 = sC4[j];
              v[j] = fmaf(-v[c0 + 3], l4.w, fmaf(-v[c0 + 2], l4.z, fmaf(-v[c0 + 1], l4.y, fmaf(-v[c0], l4.x, v[j]))));
              // at most 8 broadcasts in flight: without a fence the scheduler hoists all 28
              // float4 reads of a block (112 VGPRs) above the first FMA
              if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
        float* Xp = sX + p * TS;
        if (h == 1) {
#pragma unroll
          for (int k = 0; k < 32; ++k) Xp[k * 33 + q] = v[k];       // X_p[k][q]
        }
        __builtin_amdgcn_sched_barrier(0);
        if (h == 0) {
          float yq = 0.f;
#pragma unroll
          for (int j = 0; j < 32; ++j) {
            yq = fmaf(Xp[q * 33 + j], sr[32 * p + j], yq);
            if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);
          }
          sr[32 * p + q] = yq;                                       // y_p = X_p r_p
        }
      } else {
        float a[32], x[32];
  #pragma unroll
        for (int k = 0; k < 32; ++k) {
          a[k] = sD[q * 33 + k];
          x[k] = h ? sr[32 * p + k] : (k == q ? 1.f : 0.f);
        }
        // column c's multipliers L[j][c] go through a 32-float LDS vector (sD is free once
        // the rows are in registers; LDS ops of one wave complete in order) and come back as
        // float4 broadcasts: VGPR operands, no per-element v_readlane into SGPRs
        float* const sCol = sD;
  #pragma unroll
        for (int c = 0; c < 32; ++c) {
          const float piv = fmaxf(rl(a[c], c), 1e-30f);
          const float rs = __builtin_amdgcn_rsqf(piv);
          const float lc = a[c] * rs;          // L[row][c] (rows >= c)
          const float xc = x[c] * rs;
          x[c] = xc;
          sCol[q] = lc;
  #pragma unroll
          for (int g = (c + 1) >> 2; g < 8; ++g) {
            const float4_ l4 = *reinterpret_cast<const float4_*>(&sCol[4 * g]);
            const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
  #pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int j = 4 * g + e;
              if (j > c) {
                a[j] = fmaf(-lc, lv[e], a[j]);
                x[j] = fmaf(-lv[e], xc, x[j]);
              }
            }
          }
        }
        float* Xp = sX + p * TS;
        if (h == 0) {
  #pragma unroll
          for (int k = 0; k < 32; ++k) Xp[k * 33 + q] = x[k];       // X_p[k][q]
        } else if (q == 0) {
  #pragma unroll
          for (int k = 0; k < 32; ++k) sr[32 * p + k] = x[k];       // y_p
        }
      }
    }
    __syncthreads();
    if constexpr (TIM) { const int64_t t = clock64(); tmA += t - tmP; tmP = t; }
#pragma unroll
    for (int s = 0; s < MT; ++s) {
      if (tj[s] != p || ti[s] <= p) continue;
      // B: U_pi = X_p S_pi; publish it; r_i -= U_pi^T y_p
      const float* Xp = sX + p * TS + q * 33 + 4 * h;
      f32x16_ z;
#pragma unroll
      for (int v = 0; v < 16; ++v) z[v] = 0.f;
#pragma unroll
      for (int v = 0; v < 16; ++v) z = __builtin_amdgcn_mfma_f32_32x32x2f32(Xp[(v & 3) + 8 * (v >> 2)], acc[s][v], z, 0, 0, 0);
      acc[s] = z;
      const int off = 32 * (ti[s] - p - 1);
      float part = 0.f;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int r = (v & 3) + 8 * (v >> 2) + 4 * h;
        sPn[r * PNS + off + q] = z[v];
        part = fmaf(z[v], sr[32 * p + r], part);
      }
      part += __shfl_xor(part, 32, 64);
      if (h == 0) sr[32 * ti[s] + q] -= part;
    }
    __syncthreads();
    if constexpr (TIM) { const int64_t t = clock64(); tmB += t - tmP; tmP = t; }
#pragma unroll
    for (int s = 0; s < MT; ++s) {
      if (tj[s] >= NT || tj[s] <= p) continue;
      // C: trailing update S_ji -= U_pj^T U_pi
      const float* aj = sPn + 32 * (tj[s] - p - 1) + q;
      const float* bi = sPn + 32 * (ti[s] - p - 1) + q;
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const int k = 2 * st + h;
        acc[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(-aj[k * PNS], bi[k * PNS], acc[s], 0, 0, 0);
      }
    }
    if constexpr (TIM) { const int64_t t = clock64(); tmC += t - tmP; tmP = t; }
  }
  __syncthreads();
  if constexpr (TIM) tmP = clock64();

  // ---- backward U x = y ----
  for (int p = NT - 1; p >= 0; --p) {
    float prod[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) prod[v] = 0.f;
    bool any = false;
#pragma unroll
    for (int s = 0; s < MT; ++s) {
      if (tj[s] != p || ti[s] <= p) continue;
      any = true;
      const float xi = sr[32 * ti[s] + q];
#pragma unroll
      for (int v = 0; v < 16; ++v) prod[v] = fmaf(acc[s][v], xi, prod[v]);
    }
    float* scr = sScr + wid * TS;
    if (any) {
#pragma unroll
      for (int v = 0; v < 16; ++v) scr[((v & 3) + 8 * (v >> 2) + 4 * h) * 33 + q] = prod[v];
    }
    if (h == 0) {
      float t = 0.f;
      if (any)
#pragma unroll
        for (int k = 0; k < 32; ++k) t += scr[q * 33 + k];
      sWp[wid * 32 + q] = t;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < MT; ++s) {
      if (tj[s] != p || ti[s] != p || h != 0) continue;
      const float* Xp = sX + p * TS + q;
      float xq = 0.f;
#pragma unroll
      for (int k = 0; k < 32; ++k) {
        float tk = sr[32 * p + k];
#pragma unroll
        for (int w2 = 0; w2 < W; ++w2) tk -= sWp[w2 * 32 + k];
        xq = fmaf(Xp[k * 33], tk, xq);
      }
      sr[32 * p + q] = xq;
    }
    __syncthreads();
  }
  if (tid < R) X[u * R + tid] = sr[tid];
  if constexpr (TIM) {
    if (tid == 0) {
      const int64_t t = clock64();
      int64_t* o = timing + (int64_t)blockIdx.x * 6;
      o[0] = tmG; o[1] = tmA; o[2] = tmB; o[3] = tmC; o[4] = t - tmP; o[5] = t - tm0;
    }
  }
}

}  // namespace

// Woodbury solves (rows with n_u <= 32 ratings and lam_u > 0).  P: the factor table
// rotated into the eigenbasis of G (F Q, implicit) or F itself (explicit, eig = 0);
// eig: the eigenvalues of G (zeros when explicit).  X row u receives y_u = D P_u^T z
// (implicit: the caller applies x = Q y) or x_u (explicit).
// Diagnostic: als_wood_kernel<128> with per-row phase cycles in timing [nsmall][5].
O3S_API int o3s_als_wood_timed(const int64_t* indptr, const int32_t* cols, const float* w, const float* b,
                               const float* P, const float* eig, const float* lam, const int32_t* small,
                               int64_t nsmall, float* X, int64_t* timing, hipStream_t st) {
  if (nsmall <= 0 || !eig || !P || !timing) return -1;
  hipLaunchKernelGGL((als_wood_kernel<128, true>), dim3((unsigned)((nsmall + kWW - 1) / kWW)), dim3(kWW * 64), 0, st,
                     indptr, cols, w, b, P, eig, lam, small, nsmall, X, timing);
  O3S_CHECK_LAUNCH();
  return 0;
}

namespace {
int g_wood_blk = 1;         // o3s_als_wood_blocked: panel-blocked Woodbury Cholesky (MFMA trailing updates)
}
O3S_API int o3s_als_wood_blocked(int on) {
  g_wood_blk = on ? 1 : 0;
  return 0;
}

// Woodbury rows of at most kn ratings (kn = 16: the short-row build, 16 x 16 S; 32: as
// o3s_als_wood), panel-blocked Cholesky.
O3S_API int o3s_als_wood_kn(int R, int kn, const int64_t* indptr, const int32_t* cols, const float* w,
                            const float* b, const float* P, const float* eig, const float* lam, const int32_t* small,
                            int64_t nsmall, float* X, hipStream_t st) {
  if (nsmall < 0 || !eig || !P || (kn != 16 && kn != 24 && kn != 32)) return -1;
  if (nsmall == 0) return 0;
  const dim3 grid((unsigned)((nsmall + kWW - 1) / kWW));
#define O3S_WK(RR)                                                                                          \
  if (R == RR) {                                                                                            \
    if (kn == 16)                                                                                           \
      hipLaunchKernelGGL((als_wood_kernel<RR, false, 3, true, 16>), grid, dim3(kWW * 64), 0, st, indptr,    \
                         cols, w, b, P, eig, lam, small, nsmall, X, nullptr);                               \
    else if (kn == 24)                                                                                      \
      hipLaunchKernelGGL((als_wood_kernel<RR, false, 3, true, 24>), grid, dim3(kWW * 64), 0, st, indptr,    \
                         cols, w, b, P, eig, lam, small, nsmall, X, nullptr);                               \
    else                                                                                                    \
      hipLaunchKernelGGL((als_wood_kernel<RR, false, 3, true>), grid, dim3(kWW * 64), 0, st, indptr, cols, w, \
                         b, P, eig, lam, small, nsmall, X, nullptr);                                        \
    O3S_CHECK_LAUNCH();                                                                                     \
    return 0;                                                                                               \
  }
  O3S_WK(32) O3S_WK(64) O3S_WK(96) O3S_WK(128)
#undef O3S_WK
  return -2;
}

O3S_API int o3s_als_wood(int R, const int64_t* indptr, const int32_t* cols, const float* w, const float* b,
                         const float* P, const float* eig, const float* lam, const int32_t* small, int64_t nsmall,
                         float* X, hipStream_t st) {
  if (nsmall < 0 || !eig || !P) return -1;
  if (nsmall == 0) return 0;
  const dim3 grid((unsigned)((nsmall + kWW - 1) / kWW));
#define O3S_WD(RR)                                                                                          \
  if (R == RR) {                                                                                            \
    if (g_wood_blk)                                                                                         \
      hipLaunchKernelGGL((als_wood_kernel<RR, false, 3, true>), grid, dim3(kWW * 64), 0, st, indptr, cols, w, \
                         b, P, eig, lam, small, nsmall, X, nullptr);                                        \
    else                                                                                                    \
      hipLaunchKernelGGL((als_wood_kernel<RR>), grid, dim3(kWW * 64), 0, st, indptr, cols, w, b, P, eig,    \
                         lam, small, nsmall, X, nullptr);                                                   \
    O3S_CHECK_LAUNCH();                                                                                     \
    return 0;                                                                                               \
  }
  O3S_WD(32) O3S_WD(64) O3S_WD(96) O3S_WD(128)
#undef O3S_WD
  return -2;
}

// x = Q y in place for the listed rows (QT = Q^T row-major, R x R).
namespace {
int g_rotate_mfma = 0;      // o3s_als_rotate_mfma: x = Q y on the matrix cores (R = 128)
}
O3S_API int o3s_als_rotate_mfma(int on) {
  g_rotate_mfma = on ? 1 : 0;
  return 0;
}

// x = Q y for the listed rows: read from Y, written to X (Y == X: in place).
O3S_API int o3s_als_rotate_to(int R, const float* QT, const int32_t* rows, int64_t nrows, const float* Y,
                              float* X, int grid, hipStream_t st) {
  if (nrows < 0 || !QT || !Y || grid <= 0) return -1;
  if (nrows == 0) return 0;
  if (R == 128 && g_rotate_mfma) {
    const int64_t tiles = (nrows + 31) / 32;
    const int g = (int)(tiles < 4096 ? tiles : 4096);
    hipLaunchKernelGGL(als_rotate_mfma_kernel, dim3(g), dim3(256), 0, st, QT, rows, nrows, Y, X);
    O3S_CHECK_LAUNCH();
    return 0;
  }
#define O3S_RT(RR)                                                                                       \
  if (R == RR) {                                                                                         \
    hipLaunchKernelGGL((als_rotate_kernel<RR>), dim3(grid), dim3(256), 0, st, QT, rows, nrows, Y, X);    \
    O3S_CHECK_LAUNCH();                                                                                  \
    return 0;                                                                                            \
  }
  O3S_RT(32) O3S_RT(64) O3S_RT(96) O3S_RT(128)
#undef O3S_RT
  return -2;
}

O3S_API int o3s_als_rotate(int R, const float* QT, const int32_t* rows, int64_t nrows, float* X, int grid,
                           hipStream_t st) {
  return o3s_als_rotate_to(R, QT, rows, nrows, X, X, grid, st);
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

namespace {
template <bool BLK, bool GL = false>
int launch_dense_mfma(int implicit, int R, const int64_t* indptr, const int32_t* cols, const float* w,
                      const float* b, const float* F, const float* G, const float* lam, const int32_t* dense,
                      int64_t ndense, float* X, hipStream_t st) {
  if (ndense < 0 || (implicit && !G)) return -1;
  if (ndense == 0) return 0;
#define O3S_DM(RR)                                                                                              \
  if (R == RR) {                                                                                                \
    if (implicit)                                                                                               \
      hipLaunchKernelGGL((als_dense_mfma_kernel<RR, true, BLK, false, GL>), dim3((unsigned)ndense),             \
                         dim3(DenseM<RR>::NTH), 0, st, indptr, cols, w, b, F, G, lam, dense, X, nullptr);       \
    else                                                                                                        \
      hipLaunchKernelGGL((als_dense_mfma_kernel<RR, false, BLK, false, GL>), dim3((unsigned)ndense),            \
                         dim3(DenseM<RR>::NTH), 0, st, indptr, cols, w, b, F, G, lam, dense, X, nullptr);       \
    O3S_CHECK_LAUNCH();                                                                                         \
    return 0;                                                                                                   \
  }
  O3S_DM(32) O3S_DM(64) O3S_DM(96) O3S_DM(128)
#undef O3S_DM
  return -2;
}
}  // namespace

// Dense solves on the matrix cores (als_dense_mfma_kernel); same contract as o3s_als_dense.
// o3s_als_dense_mfma: diagonal tiles factored column by column (32 LDS broadcasts per
// tile); o3s_als_dense_mfma_blk: 4-column blocks, row and X column sharing one register array;
// o3s_als_dense_mfma_gl: _blk with the R = 128 Gram fed by the LDS-DMA gather ring.
O3S_API int o3s_als_dense_mfma(int implicit, int R, const int64_t* indptr, const int32_t* cols, const float* w,
                               const float* b, const float* F, const float* G, const float* lam, const int32_t* dense,
                               int64_t ndense, float* X, hipStream_t st) {
  return launch_dense_mfma<false>(implicit, R, indptr, cols, w, b, F, G, lam, dense, ndense, X, st);
}
O3S_API int o3s_als_dense_mfma_blk(int implicit, int R, const int64_t* indptr, const int32_t* cols, const float* w,
                                   const float* b, const float* F, const float* G, const float* lam,
                                   const int32_t* dense, int64_t ndense, float* X, hipStream_t st) {
  return launch_dense_mfma<true>(implicit, R, indptr, cols, w, b, F, G, lam, dense, ndense, X, st);
}
O3S_API int o3s_als_dense_mfma_gl(int implicit, int R, const int64_t* indptr, const int32_t* cols, const float* w,
                                  const float* b, const float* F, const float* G, const float* lam,
                                  const int32_t* dense, int64_t ndense, float* X, hipStream_t st) {
  return launch_dense_mfma<true, true>(implicit, R, indptr, cols, w, b, F, G, lam, dense, ndense, X, st);
}

// Diagnostic: the dense kernel (BLK, implicit, R = 128; gl != 0: with the LDS-DMA gather
// ring) with per-block phase cycle counts in timing [ndense][6] (see the kernel's TIM comment).
O3S_API int o3s_als_dense_mfma_timed(int gl, const int64_t* indptr, const int32_t* cols, const float* w,
                                     const float* b, const float* F, const float* G, const float* lam,
                                     const int32_t* dense, int64_t ndense, float* X, int64_t* timing, hipStream_t st) {
  if (ndense <= 0 || !G || !timing) return -1;
  if (gl)
    hipLaunchKernelGGL((als_dense_mfma_kernel<128, true, true, true, true>), dim3((unsigned)ndense),
                       dim3(DenseM<128>::NTH), 0, st, indptr, cols, w, b, F, G, lam, dense, X, timing);
  else
    hipLaunchKernelGGL((als_dense_mfma_kernel<128, true, true, true>), dim3((unsigned)ndense),
                       dim3(DenseM<128>::NTH), 0, st, indptr, cols, w, b, F, G, lam, dense, X, timing);
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_API int o3s_als_exact_max_small() { return kNW; }
