// Exact ALS solves on gfx950: every row's normal equations solved directly (Spark's
// per-row Cholesky, reached through the Recommendation widget -> ALS.fit,
// orangecontrib/spark/widgets/ml/spark_ml_recommendation.py:15), never materialising the
// rank x rank systems in HBM.
//
//   A_u = G + Y_u^T W_u Y_u + lam_u I,   b_u = Y_u^T c_u,   x_u = A_u^{-1} b_u
//
// (implicit: G = Y^T Y, W = diag(alpha |r|), c = (1 + alpha |r|)[r > 0]; explicit: G = 0,
// W = I, c = r; lam_u = regParam * n_u).  Two solvers by row length n_u:
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
//   (the rotation back, x = Q y, runs over all Woodbury rows afterwards).
// * longer rows (the item side, ~200 ratings): als_dense_wave_kernel in als_dense.hip --
//   one wave per row, bf16x3 Gram on the matrix cores fed by an LDS-DMA gather ring, blocked
//   Cholesky in MFMA accumulator layout.
//
// This file also holds the rotations x = Q y (als_rotate_mfma_kernel at R = 128,
// als_rotate_kernel below it).  The solvers write x_u straight into the factor table;
// fp32 throughout (the S sums are short: n_u terms).
#include "common.h"

#include <stdlib.h>

using namespace o3s;

namespace {

typedef float f32x16_ __attribute__((ext_vector_type(16)));
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
// In 8-column panels: inside a panel the v_readlane rank-1 updates above, then the
// trailing columns take the panel's whole rank-8 update P = L21 L21^T from 4
// v_mfma_f32_32x32x2_f32 (A = B = the panel's L entries, lane l holding row l & 31 and
// k-slot l >> 5); P is symmetric, so the accumulator's column l & 31 is row l & 31 of P,
// split between lanes l and l ^ 32 (one ds_bpermute exchange per register).  Per trailing
// column: 2 VALU ops per panel instead of 16.  Lanes l >= 32 mirror rows l & 31 exactly
// (the MFMA reads their L entries).
template <int NM, int KN = kNW>
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
      for (int m = k + 1; m < 8 * p + 8; ++m) srow[m] = fmaf(-lik, rl(lik, m), srow[m]);
    }
    {
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
// Three waves per SIMD (168 VGPRs, no spill).
// (a 4-waves-per-SIMD build spilled and measured 8.6% slower; S = P D P^T as bf16x3 on
// 32x32x16 MFMAs measured 4% slower; persistent waves prefetching the next row's metadata
// measured 14% slower: profiles/kernel_experiments_r4.json)
// KN: the longest row of the launch (32, or 16 for the launch of the short rows: half the
// P registers, and S on v_mfma_f32_16x16x4_f32 -- a quarter of the matrix-pipe cycles)
// WOOD24_16: the 17..24- and 25..32-rating launches build S on 16 x 16 tiles (see the S build)
template <int R, int KN = kNW, bool TIM = false, bool WOOD24_16 = true>
__global__ __launch_bounds__(kWW * 64, 3) void als_wood_kernel(
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
  } else if (WOOD24_16) {
    // S (24 or 32 rows) as three 16 x 16 tiles (rows 0-15 / 16-31 of the image; rows >= n
    // are zero): S00, S01, S11 on v_mfma_f32_16x16x4_f32 -- 96 MFMAs of 8 passes instead of
    // the 32 x 32 tile's 64 of 16: the upper blocks only, a quarter of the matrix-pipe
    // cycles saved (17..24-rating launch: 7.5 -> 6.8-7.4 ms per 2M rows, tools/als_wood_phases.py)
    const int g = lane >> 4;
    const float* rq0 = sp + (lane & 15) * kPS + 16 * g + (g >> 1) * 4;
    const float* rq1 = rq0 + 16 * kPS;
    float4_ s00 = {0.f, 0.f, 0.f, 0.f}, s01 = {0.f, 0.f, 0.f, 0.f}, s11 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int hf = 0; hf < RV; ++hf) {
#pragma unroll
      for (int i = 0; i < kNW; ++i)
        sp[i * kPS + wcol] = i >= KN ? 0.f : (hf == 0 ? acc[i < KN ? i : 0].x * sq.x : acc[i < KN ? i : 0].y * sq.y);
#pragma unroll
      for (int s4 = 0; s4 < 16; s4 += 4) {
        const float4_ x0 = *reinterpret_cast<const float4_*>(rq0 + s4);
        const float4_ x1 = *reinterpret_cast<const float4_*>(rq1 + s4);
        const float a0[4] = {x0.x, x0.y, x0.z, x0.w}, a1[4] = {x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          s00 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[c], a0[c], s00, 0, 0, 0);
          s01 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[c], a1[c], s01, 0, 0, 0);
          s11 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[c], a1[c], s11, 0, 0, 0);
        }
      }
    }
    // register q of lane l: row 4 (l >> 4) + q, column l & 15 of its tile; S01 also as the
    // lower block S10 = S01^T
    const int c = lane & 15;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      S[4 * g + q][c] = s00[q];
      S[4 * g + q][16 + c] = s01[q];
      S[16 + c][4 * g + q] = s01[q];
      S[16 + 4 * g + q][16 + c] = s11[q];
    }
    asm volatile("" ::: "memory");
    if (lane < kNW) S[lane][lane] += winv;
    asm volatile("" ::: "memory");
#pragma unroll
    for (int m = 0; m < KN; ++m) srow[m] = S[lane & 31][m];
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
  if (n <= 8) v = wood_factor_solve<8, KN>(srow, t, Lc, lane);
  else if (KN == 16 || n <= 16) v = wood_factor_solve<16, KN>(srow, t, Lc, lane);
  else if constexpr (KN == 24) {
    v = wood_factor_solve<24, KN>(srow, t, Lc, lane);
  } else if constexpr (KN == 32) {
    if (n <= 24) v = wood_factor_solve<24, KN>(srow, t, Lc, lane);
    else v = wood_factor_solve<32, KN>(srow, t, Lc, lane);
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

}  // namespace

// Woodbury solves (rows with n_u <= 32 ratings and lam_u > 0).  P: the factor table
// rotated into the eigenbasis of G (F Q, implicit) or F itself (explicit, eig = 0);
// eig: the eigenvalues of G (zeros when explicit).  X row u receives y_u = D P_u^T z
// (implicit: the caller applies x = Q y) or x_u (explicit).
// Diagnostic: als_wood_kernel<128, kn> (kn = 16 / 24 / 32, as o3s_als_wood_kn) with
// per-row phase cycles in timing [nsmall][5].
O3S_API int o3s_als_wood_timed(int kn, const int64_t* indptr, const int32_t* cols, const float* w, const float* b,
                               const float* P, const float* eig, const float* lam, const int32_t* small,
                               int64_t nsmall, float* X, int64_t* timing, hipStream_t st) {
  if (nsmall <= 0 || !eig || !P || !timing) return -1;
  const dim3 grid((unsigned)((nsmall + kWW - 1) / kWW)), block(kWW * 64);
  if (kn == 16)
    hipLaunchKernelGGL((als_wood_kernel<128, 16, true>), grid, block, 0, st, indptr, cols, w, b, P, eig, lam, small,
                       nsmall, X, timing);
  else if (kn == 24)
    hipLaunchKernelGGL((als_wood_kernel<128, 24, true>), grid, block, 0, st, indptr, cols, w, b, P, eig, lam, small,
                       nsmall, X, timing);
  else if (kn == 32)
    hipLaunchKernelGGL((als_wood_kernel<128, kNW, true>), grid, block, 0, st, indptr, cols, w, b, P, eig, lam, small,
                       nsmall, X, timing);
  else
    return -2;
  O3S_CHECK_LAUNCH();
  return 0;
}

// A/B switch, read per call so a benchmark can flip it between launches:
// O3S_ALS_WOOD24_16=0 -- the 17..32-rating launches build S as one 32 x 32 tile.
// (Rejected, profiles/kernel_experiments_r6.json: rank-128 rows gathered as float2
// (features 2 l, 2 l + 1: one load per factor row instead of two) -- neutral.)
static bool env_on(const char* name) {
  const char* e = getenv(name);
  return !(e && e[0] == '0');
}

template <int RR, int KN, bool S16>
void wood_launch(dim3 grid, hipStream_t st, const int64_t* indptr, const int32_t* cols, const float* w,
                 const float* b, const float* P, const float* eig, const float* lam, const int32_t* small,
                 int64_t nsmall, float* X) {
  hipLaunchKernelGGL((als_wood_kernel<RR, KN, false, S16>), grid, dim3(kWW * 64), 0, st, indptr, cols, w, b, P,
                     eig, lam, small, nsmall, X, nullptr);
}

template <int RR>
void wood_dispatch(int kn, dim3 grid, hipStream_t st, const int64_t* indptr, const int32_t* cols, const float* w,
                   const float* b, const float* P, const float* eig, const float* lam, const int32_t* small,
                   int64_t nsmall, float* X) {
  const bool s16 = env_on("O3S_ALS_WOOD24_16");
#define O3S_WL(KN, S) wood_launch<RR, KN, S>(grid, st, indptr, cols, w, b, P, eig, lam, small, nsmall, X)
  if (kn == 16) O3S_WL(16, true);
  else if (kn == 24) { if (s16) O3S_WL(24, true); else O3S_WL(24, false); }
  else { if (s16) O3S_WL(kNW, true); else O3S_WL(kNW, false); }
#undef O3S_WL
}

// Woodbury rows of at most kn ratings (kn = 16: the short-row build, 16 x 16 S on
// v_mfma_f32_16x16x4_f32; 24 / 32: S on three 16 x 16 tiles), panel-blocked Cholesky.
O3S_API int o3s_als_wood_kn(int R, int kn, const int64_t* indptr, const int32_t* cols, const float* w,
                            const float* b, const float* P, const float* eig, const float* lam, const int32_t* small,
                            int64_t nsmall, float* X, hipStream_t st) {
  if (nsmall < 0 || !eig || !P || (kn != 16 && kn != 24 && kn != 32)) return -1;
  if (nsmall == 0) return 0;
  const dim3 grid((unsigned)((nsmall + kWW - 1) / kWW));
  switch (R) {
    case 32: wood_dispatch<32>(kn, grid, st, indptr, cols, w, b, P, eig, lam, small, nsmall, X); break;
    case 64: wood_dispatch<64>(kn, grid, st, indptr, cols, w, b, P, eig, lam, small, nsmall, X); break;
    case 96: wood_dispatch<96>(kn, grid, st, indptr, cols, w, b, P, eig, lam, small, nsmall, X); break;
    case 128: wood_dispatch<128>(kn, grid, st, indptr, cols, w, b, P, eig, lam, small, nsmall, X); break;
    default: return -2;
  }
  O3S_CHECK_LAUNCH();
  return 0;
}

// x = Q y for the listed rows: read from Y, written to X (Y == X: in place).
O3S_API int o3s_als_rotate_to(int R, const float* QT, const int32_t* rows, int64_t nrows, const float* Y,
                              float* X, int grid, hipStream_t st) {
  if (nrows < 0 || !QT || !Y || grid <= 0) return -1;
  if (nrows == 0) return 0;
  if (R == 128) {
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

O3S_API int o3s_als_exact_max_small() { return kNW; }

O3S_PRELOAD(als_exact)
