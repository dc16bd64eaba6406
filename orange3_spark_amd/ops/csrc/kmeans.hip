// KMeans assign + update (gfx950).  Replaces the per-partition closest-centre search
// and per-cluster sums that Spark's KMeans runs per iteration (reached through the
// Clustering widget -> fit, orangecontrib/spark/widgets/ml/spark_ml_clustering.py:14).
//
// ---------------------------------------------------------------------------------
// kmeans_assign: argmin_c ||x - c||^2 = argmin_c (||c||^2 - 2 x.c) as an MFMA GEMM
// with a fused arg-min epilogue -- the N x K distance matrix is never materialised.
//
//  * D' = C . X^T with v_mfma_f32_32x32x16_bf16: A = a 32-centroid chunk (from LDS),
//    B = X^T of a 32-row tile (registers).  In this orientation each lane's 16
//    accumulators belong to ONE data row (its column) and 16 centroids, so the running
//    (min, argmin) is lane-local: no cross-lane work until one final half-wave merge.
//  * split precision: x = xh + xl, c = ch + cl (bf16 hi/lo); x.c ~ xh.ch + xl.ch + xh.cl
//    (3 bf16 MFMAs, ~2^-16 relative error, i.e. fp32-level distance accuracy at the
//    bf16 MFMA rate; a 1-pass bf16 product would mis-assign near ties).  The -2 factor
//    is folded into the centre split on the host.
//  * each wave owns one 32-row tile (X fragments hi/lo: 64 VGPRs at D=128, held for the
//    whole centroid sweep); 8 waves share each centroid chunk through LDS, staged by
//    LDS-DMA (global_load_lds_dwordx4) double-buffered so chunk j+1 lands under chunk
//    j's MFMAs; the 16-B slot XOR-swizzle (slot ^= row & 15, applied to the DMA SOURCE
//    address since the DMA image is lane-linear) makes the 32-row ds_read_b128
//    fragment reads bank-conflict free (CDNA guide §5.5 T2, §5.4 rule 21).
//
// kmeans_update: per-cluster sums without float atomics.  Each block takes chunks of
// R rows, counting-sorts their indices by cluster in LDS, then each wave owns a contiguous
// cluster range and streams its rows (coalesced 512-B row reads) accumulating in
// registers; a cluster's sum is flushed once per chunk into the block's private slab.
// (The bucket order is row order, produced by a stable ballot-ranked scatter.)
// Slabs are summed by kmeans_reduce in a fixed order (bitwise deterministic).
#include "common.h"

using namespace o3s;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kAssignWaves = 8;   // 8 waves x one 32-row tile share each centroid chunk
constexpr int kAssignThreads = kAssignWaves * kWave;

__device__ __forceinline__ void split_bf16(float v, short& hi, short& lo) {
  const uint16_t h = f32_to_bf16(v);
  hi = (short)h;
  lo = (short)f32_to_bf16(v - bf16_to_f32(h));
}

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// x * scale split into two fp16 halves (hi + lo carries ~22 significant bits); the caller
// picks the power-of-two scale so |x * scale| <= 2^15 (no fp16 overflow)
__device__ __forceinline__ void split_f16(float v, float scale, short& hi, short& lo) {
  const float sv = v * scale;
  const _Float16 h = (_Float16)sv;
  hi = __builtin_bit_cast(short, h);
  lo = __builtin_bit_cast(short, (_Float16)(sv - (float)h));
}

// as split_f16, also returning the scaled rounding error of the hi half (exact in fp32:
// the hi half is the fp16 rounding of sv, so sv - hi is representable)
__device__ __forceinline__ float split_f16e(float v, float scale, short& hi, short& lo) {
  const float sv = v * scale;
  const _Float16 h = (_Float16)sv;
  const float d = sv - (float)h;
  hi = __builtin_bit_cast(short, h);
  lo = __builtin_bit_cast(short, (_Float16)d);
  return d;
}

__device__ __forceinline__ float f16_bits_to_f32(uint32_t bits16) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)bits16);
}

// KS = D / 16 k-steps, TT = 32-row tiles per wave.  Cpad: centroids padded to 32
// (padding rows carry cn = +inf).  CNL: ||c||^2 staged in LDS (when Cpad floats fit beside
// the chunk buffers) and folded into the accumulator init; else read per chunk.  The
// epilogue keeps explicit indices (exact ties resolve to the lowest index: the screen's
// slot-coded keys would order exact ties of negative partial distances backwards), which
// costs little here: three MFMAs per k-step leave the VALU mostly idle.
template <int KS, int TT, bool CNL>
__global__ __launch_bounds__(kAssignThreads, 2) void kmeans_assign_kernel(
    const float* __restrict__ X, int64_t n, int64_t ldx, const uint16_t* __restrict__ Chi,
    const uint16_t* __restrict__ Clo, const float* __restrict__ cn, int Cpad,
    int32_t* __restrict__ assign, float* __restrict__ mind, int Dx, const int32_t* __restrict__ rowlist) {
  constexpr int D = KS * 16;
  constexpr int SLOTS = D / 8;                 // 16-B slots per centroid row
  constexpr int CH_ELEMS = 32 * D;             // bf16 per chunk (hi or lo)
  constexpr int PIECES = 2 * 32 * SLOTS;       // 16-B pieces per chunk (hi + lo)
  // G centroid chunks per LDS stage (one barrier per G chunks), double-buffered
  constexpr int G = D <= 128 ? 4 : 2;
  constexpr int PER_THREAD = (G * PIECES + kAssignThreads - 1) / kAssignThreads;
  static_assert(PIECES % kWave == 0, "whole waves per DMA instruction");
  constexpr int ROWS_PER_WAVE = 32 * TT;
  constexpr int ROWS_PER_BLOCK = kAssignWaves * ROWS_PER_WAVE;
  // ONE __shared__ array (guide §5 item 4a): [buf][hi|lo][32][D] bf16, slot-swizzled rows,
  // then (CNL) Cpad floats of ||c||^2
  constexpr int STAGE_ELEMS = 2 * G * 2 * CH_ELEMS;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  float* const scn = reinterpret_cast<float*>(lds + STAGE_ELEMS);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t row_base = (int64_t)blockIdx.x * ROWS_PER_BLOCK + wid * ROWS_PER_WAVE;

  // ---- X^T fragments (B operand) for the wave's rows, split hi/lo, + ||x||^2.
  // The fragment layout wants 32 rows per load instruction (lane r <- row r), which
  // touches 32 rows x 32 B per wave-instruction; instead the wave streams its 32-row
  // tile row-contiguously (1 KiB per instruction) into its slice of the (not yet used)
  // centroid LDS buffer and reads the fragments back transposed.  16-B slots are
  // XOR-swizzled by row so the 32-row column reads are conflict free.
  // (D > 128: the tile does not fit the stage buffer; load the fragments directly.)
  constexpr int XS = D / 4;                    // 16-B slots per staged row
  constexpr bool kStageX = kAssignWaves * ROWS_PER_WAVE * D * 4 <= STAGE_ELEMS * 2;
  if constexpr (CNL) {
    for (int i = threadIdx.x; i < Cpad; i += kAssignThreads) scn[i] = cn[i];
  }
  float* xt = reinterpret_cast<float*>(lds) + wid * ROWS_PER_WAVE * D;
  bf16x8 bh[TT][KS], bl[TT][KS];
  float xn[TT];
  if constexpr (kStageX) {
    constexpr int PIECES_X = ROWS_PER_WAVE * XS;
#pragma unroll 4
    for (int P = lane; P < PIECES_X; P += kWave) {
      const int rr = P / XS, sl = P % XS;
      const int64_t row = row_base + rr;
      int64_t rowc = row < n ? row : n - 1;
      if (rowlist) rowc = rowlist[rowc];        // recheck pass: rows gathered by index
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 v = 4 * sl < Dx ? *reinterpret_cast<const float4*>(X + rowc * ldx + 4 * sl) : z;
      *reinterpret_cast<float4*>(xt + rr * D + 4 * (sl ^ (rr & (XS - 1) & 31))) = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the wave reads back only its own slice
  }
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    const int rr = t * 32 + r;
    float s = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      float4 a, b;
      if constexpr (kStageX) {
        const int s0 = (ks * 16 + 8 * h) / 4;
        const int sw = rr & (XS - 1) & 31;
        a = *reinterpret_cast<const float4*>(xt + rr * D + 4 * (s0 ^ sw));
        b = *reinterpret_cast<const float4*>(xt + rr * D + 4 * ((s0 + 1) ^ sw));
      } else {
        const int64_t row = row_base + rr;
        int64_t rowc = row < n ? row : n - 1;
        if (rowlist) rowc = rowlist[rowc];
        const float* xp = X + rowc * ldx;
        const int c0 = ks * 16 + 8 * h;        // Dx % 4 == 0: whole float4s are in or out
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        a = c0 < Dx ? *reinterpret_cast<const float4*>(xp + c0) : z;
        b = c0 + 4 < Dx ? *reinterpret_cast<const float4*>(xp + c0 + 4) : z;
      }
      const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      // pack pairs into dwords explicitly and pin the packed registers: left as 16 separate
      // shorts, hipcc keeps one bf16 per VGPR and re-packs every fragment (4 v_perm) for
      // every chunk of the centroid sweep
      uint32_t ph[4], pl[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        short h0, l0, h1, l1;
        split_bf16(v[2 * j], h0, l0);
        split_bf16(v[2 * j + 1], h1, l1);
        ph[j] = (uint32_t)(uint16_t)h0 | ((uint32_t)(uint16_t)h1 << 16);
        pl[j] = (uint32_t)(uint16_t)l0 | ((uint32_t)(uint16_t)l1 << 16);
        s = fmaf(v[2 * j], v[2 * j], s);
        s = fmaf(v[2 * j + 1], v[2 * j + 1], s);
      }
      bh[t][ks] = __builtin_bit_cast(bf16x8, ph);
      bl[t][ks] = __builtin_bit_cast(bf16x8, pl);
      asm volatile("" : "+v"(bh[t][ks]), "+v"(bl[t][ks]));
    }
    xn[t] = s + __shfl_xor(s, 32, 64);
  }
  __syncthreads();                             // every wave done with the staging area

  // ---- chunk staging by LDS-DMA (global_load_lds_dwordx4): the LDS image is lane-linear,
  // so the XOR swizzle is applied to the SOURCE slot (guide §5.4 rule 21).
  const int nchunks = Cpad / 32;
  const int nchunks_ = Cpad / 32;
  auto stage = [&](int stg, uint16_t* __restrict__ dbuf) {
#pragma unroll
    for (int k = 0; k < PER_THREAD; ++k) {
      const int P = threadIdx.x + k * kAssignThreads;      // linear 16-B piece index in the stage
      const int g = P / PIECES;                            // wave-uniform (PIECES % 64 == 0)
      const int chunk = stg * G + g;
      if (P >= G * PIECES || chunk >= nchunks_) continue;  // the DMA image stays lane-linear
      const int Q = P % PIECES;
      const int which = Q / (32 * SLOTS);
      const int rem = Q % (32 * SLOTS);
      const int cr = rem / SLOTS, sw = rem % SLOTS;
      const int sl = sw ^ (cr & 15 & (SLOTS - 1));
      const uint16_t* src = (which ? Clo : Chi) + ((int64_t)(chunk * 32 + cr)) * D + sl * 8;
      __builtin_amdgcn_global_load_lds(src, dbuf + (wid * kWave + k * kAssignThreads) * 8, 16, 0, 0);   // wave-uniform
    }
  };

  float bestv[TT], xnv[TT];
  int besti[TT];
#pragma unroll
  for (int t = 0; t < TT; ++t) { bestv[t] = INFINITY; besti[t] = 0; xnv[t] = xn[t]; }
  stage(0, lds);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // Software pipeline: the MFMAs of chunk ch are issued, then the arg-min epilogue of
  // chunk ch-1 (independent VALU work) fills the MFMA issue gaps instead of running in
  // a separate phase after every barrier.
  f32x16 accp[TT];
  auto epilogue = [&](const f32x16 (&a)[TT], int chp) {
    const int cbase = chp * 32 + 4 * h;      // acc reg i -> centroid cbase + (i&3) + 8*(i>>2)
    float cv[16];
    if constexpr (!CNL) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 c4 = *reinterpret_cast<const float4*>(cn + cbase + 8 * q);
        cv[4 * q + 0] = c4.x; cv[4 * q + 1] = c4.y; cv[4 * q + 2] = c4.z; cv[4 * q + 3] = c4.w;
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int idx = cbase + (i & 3) + 8 * (i >> 2);
#pragma unroll
      for (int t = 0; t < TT; ++t) {
        const float dv = CNL ? a[t][i] : a[t][i] + cv[i];
        const bool better = dv < bestv[t];
        bestv[t] = better ? dv : bestv[t];
        besti[t] = better ? idx : besti[t];
      }
    }
  };
  const int nstages = (nchunks + G - 1) / G;
  // One stage's body with its LDS regions as __restrict__ pointers: the scoped no-alias
  // info keeps hipcc from draining the next stage's in-flight DMA (vmcnt(0)) before the
  // first LDS read of every chunk.
  auto run_stage = [&](int stg, const uint16_t* __restrict__ cur, uint16_t* __restrict__ nxt,
                       const float* __restrict__ sc) {
    if (stg + 1 < nstages) stage(stg + 1, nxt);         // DMA in flight under the MFMAs
    for (int g = 0; g < G; ++g) {
      const int ch = stg * G + g;
      if (ch >= nchunks) break;
      const uint16_t* Lh = cur + g * 2 * CH_ELEMS;
      const uint16_t* Ll = Lh + CH_ELEMS;
      f32x16 acc[TT];
      if constexpr (CNL) {                             // accumulators start at ||c||^2
        const int cbase = ch * 32 + 4 * h;
        f32x16 c0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 c4 = *reinterpret_cast<const float4*>(sc + cbase + 8 * q);
          c0[4 * q + 0] = c4.x; c0[4 * q + 1] = c4.y; c0[4 * q + 2] = c4.z; c0[4 * q + 3] = c4.w;
        }
#pragma unroll
        for (int t = 0; t < TT; ++t) acc[t] = c0;
      } else {
#pragma unroll
        for (int t = 0; t < TT; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
      }
      // A fragments are read one k-step ahead of the MFMAs that consume them, so the LDS
      // latency hides under the previous step's three MFMAs
      auto afrag = [&](const uint16_t* L, int ks) {
        const int sw = (ks * 2 + h) ^ (r & 15 & (SLOTS - 1));
        return *reinterpret_cast<const bf16x8*>(L + r * D + sw * 8);
      };
      bf16x8 nh = afrag(Lh, 0), nl = afrag(Ll, 0);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 ah = nh, al = nl;
        if (ks + 1 < KS) { nh = afrag(Lh, ks + 1); nl = afrag(Ll, ks + 1); }
#pragma unroll
        for (int t = 0; t < TT; ++t) {
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[t][ks], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[t][ks], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[t][ks], acc[t], 0, 0, 0);
        }
      }
      if (ch > 0) epilogue(accp, ch - 1);
#pragma unroll
      for (int t = 0; t < TT; ++t) accp[t] = acc[t];
    }
  };
  for (int stg = 0; stg < nstages; ++stg) {
    const int buf = stg & 1;
    run_stage(stg, lds + buf * G * 2 * CH_ELEMS, lds + (buf ^ 1) * G * 2 * CH_ELEMS, scn);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // next stage landed
    __syncthreads();                                    // ... for every wave; buf free again
  }
  if (nchunks > 0) epilogue(accp, nchunks - 1);
  // merge the two half-waves (different centroid subsets of the same row)
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    const float ov = __shfl_xor(bestv[t], 32, 64);
    const int oi = __shfl_xor(besti[t], 32, 64);
    if (ov < bestv[t] || (ov == bestv[t] && oi < besti[t])) { bestv[t] = ov; besti[t] = oi; }
    const int64_t row = row_base + t * 32 + r;
    if (h == 0 && row < n) {
      const int64_t orow = rowlist ? (int64_t)rowlist[row] : row;
      assign[orow] = besti[t];
      if (mind) mind[orow] = fmaxf(bestv[t] + xnv[t], 0.f);
    }
  }
}

// ---------------------------------------------------------------------------------
// kmeans_screen: ONE fp16 MFMA per k-step plus a rigorous error bound.
//
// x and m = -2c are scaled by powers of two (xs, ms: |x xs|, |m ms| <= 2^15, chosen on the
// host) and rounded to fp16 (11 significant bits, 8x finer than bf16), so the screened
// distance S d~_c = S ||c||^2 + (m ms)~.(x xs)~ with S = xs ms differs from S (||c||^2 -
// 2 x.c) by at most S E, where (derivation in ops/kmeans.py::screen_bound)
//   E = eps_x ||x|| + eps_e' ||dx|| + eps0,   dx = fp16(x xs)/xs - x: the row's ACTUAL
//   rounding error (its norm comes with ||x||^2 from the prologue / the pre-split rows),
//   eps_x = max_c ||fp16(m_c ms)/ms - m_c|| (+ fp32 accumulation), eps_e' ~ max||m||
// -- Cauchy-Schwarz on the actual rounding errors instead of 2^-11 per element: ~5x
// tighter on data with full mantissas (profiles/kernel_experiments_r6.json)
// Each lane tracks best, index and SECOND best (one v_med3: the new
// second is med3(old best, v, old second)); a row whose margin (second - best) exceeds
// 2E has provably the same arg-min as the exact product and is finished here: its
// squared distance is recomputed exactly in fp32 from the register-resident split x
// (fp16 hi + lo, ~22 bits) and the fp32 centre row.  Other rows (near-ties) are appended
// to a compacted list (one atomic per wave) and re-solved by the split-precision kernel
// above.  This is 1/3 of the MFMAs of the split kernel; the S ||c||^2 bias is folded
// into the accumulator init (read from LDS).  The epilogue is 2.5 VALU per distance and
// touches no VCC: the candidate's slot in its chunk (0..15) replaces the low 4 mantissa
// bits of the distance (v_and_or: a perturbation below 2^-19 of its magnitude, added to
// the bound), so best = v_min and second = v_med3 carry the index with them; the chunk
// of the best is recorded once per chunk.  On structureless data (uniform in a cube) the
// fp16 bound leaves ~10% of the rows as near ties where the bf16 one flagged nearly all.
// All LDS (staging + ||c||^2) is ONE dynamic __shared__ array, and each stage's body sees
// its three regions as __restrict__ pointers (see run_stage).
//
// 4 waves (one per SIMD) x TT 32-row tiles per block, 2 blocks per CU: one block's X
// staging and DMA prologue overlaps the other's MFMA sweep.
constexpr int kScrWaves = 4;
#ifndef O3S_SCR_FRAG_AHEAD
#define O3S_SCR_FRAG_AHEAD 1
#endif
constexpr bool kScrFragAhead = O3S_SCR_FRAG_AHEAD;
constexpr int kScrThreads = kScrWaves * kWave;

template <int KS>
struct ScrLds {
  static constexpr int D = KS * 16;
  static constexpr int G = D <= 128 ? 4 : 2;                    // centroid chunks per stage
  static constexpr int CHUNK_BYTES = 2 * 32 * D;                // hi only
  static constexpr int STAGE_BYTES = 2 * G * CHUNK_BYTES;       // double buffered
  static constexpr int X_BYTES = kScrWaves * 32 * D * 4;        // one 32-row tile per wave
  static constexpr int BYTES = STAGE_BYTES > X_BYTES ? STAGE_BYTES : X_BYTES;
};

// NOD (plain screen, mind == nullptr: the Lloyd iterations, whose cost comes from the
// cluster sums -- models/kmeans.py): no per-row distance, so neither the lo half of x (the
// pre-split rows' second 16 B: half the prologue's HBM bytes) nor the chosen centre's fp32
// row (an L2 gather of D floats per row) is read.
// (a lean build -- 2-chunk stages, 3 blocks per CU at 168 VGPRs -- measured slower: 44.4 vs
// 39.2 ms per iteration, profiles/kernel_experiments_r4.json)
template <int KS, int TT, bool PAIR, bool PS = false, bool NOD = false>
__global__ __launch_bounds__(kScrThreads, 2) void kmeans_screen_kernel(
    const float* __restrict__ X, int64_t n, int64_t ldx, const uint16_t* __restrict__ Chi,
    const float* __restrict__ cn, const float* __restrict__ C32, int ldc, int Cpad, float eps_x, float eps0,
    float eps_e, float xscale, float sscale, int32_t* __restrict__ assign, float* __restrict__ mind,
    int32_t* __restrict__ flag_cnt, int32_t* __restrict__ flag_rows, int Dx,
    const uint4* __restrict__ XP = nullptr, const float2* __restrict__ XN = nullptr,
    const int32_t* __restrict__ rowlist = nullptr, float2* __restrict__ bnd = nullptr) {
  using L = ScrLds<KS>;
  constexpr int D = L::D;
  constexpr int G = L::G;
  constexpr int SLOTS = D / 8;
  constexpr int CH_ELEMS = 32 * D;
  constexpr int PIECES = 32 * SLOTS;
  constexpr int PER_THREAD = (G * PIECES + kScrThreads - 1) / kScrThreads;
  static_assert(PIECES % kWave == 0, "whole waves per DMA instruction");
  static_assert(G % 2 == 0, "chunks are processed in ping-pong pairs");
  constexpr int XS = D / 4;
  constexpr int XL = 32 * XS / kWave;          // float4 loads per lane per 32-row tile
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];   // [L::BYTES staging | Cpad floats]
  float* const scn = reinterpret_cast<float*>(lds + L::BYTES / 2);  // S ||c||^2 (padding: 2^125)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t row_base = (int64_t)blockIdx.x * (kScrWaves * 32 * TT) + (int64_t)wid * 32 * TT;

  // padded centres (+inf) become 2^125: finite, so a slot code in the low bits never
  // turns a key into a NaN, and still farther than any real centre
  for (int i = threadIdx.x; i < Cpad; i += kScrThreads) scn[i] = fminf(cn[i] * sscale, 0x1p125f);
  // ---- X tiles -> split fp16 fragments (hi: B operand) + ||x||^2.  All XL loads of a tile
  // are issued before any is consumed (one HBM round trip per tile), then staged
  // row-contiguously through this wave's LDS slice (slot XOR swizzle: conflict-free
  // transposed reads).
  float* xt = reinterpret_cast<float*>(lds) + wid * 32 * D;
  bf16x8 bh[TT][KS], bl[TT][KS];
  float xn[TT], xe[TT];                    // ||x||^2 and ||x xs - fp16(x xs)||^2 per row
  if constexpr (PS) {
    // pre-split rows (kmeans_presplit_kernel, once per data version): per row and
    // (k-step, half) group 16 B of scaled fp16 hi then 16 B of lo, loaded straight into the
    // MFMA B fragments -- no fp32 staging, no conversion VALU in the prologue
#pragma unroll
    for (int t = 0; t < TT; ++t) {
      const int64_t row = row_base + t * 32 + r;
      const int64_t rowc = rowlist ? (int64_t)rowlist[row < n ? row : n - 1] : (row < n ? row : n - 1);
      const uint4* src = XP + rowc * (D / 4);
      uint4 hv[KS], lv[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        hv[ks] = src[(ks * 2 + h) * 2];
        if constexpr (!NOD) lv[ks] = src[(ks * 2 + h) * 2 + 1];
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bh[t][ks] = __builtin_bit_cast(bf16x8, hv[ks]);
        if constexpr (!NOD) bl[t][ks] = __builtin_bit_cast(bf16x8, lv[ks]);
      }
      const float2 ne = XN[rowc];
      xn[t] = ne.x;
      xe[t] = ne.y;
    }
  } else {
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    float4 xv[XL];
#pragma unroll
    for (int q = 0; q < XL; ++q) {
      const int P = lane + q * kWave;
      const int rr = P / XS, sl = P % XS;
      const int64_t row = row_base + t * 32 + rr;
      const int64_t rowc = rowlist ? (int64_t)rowlist[row < n ? row : n - 1] : (row < n ? row : n - 1);
      const int slc = 4 * sl < Dx ? sl : 0;
      xv[q] = *reinterpret_cast<const float4*>(X + rowc * ldx + 4 * slc);
      if (4 * sl >= Dx) xv[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < XL; ++q) {
      const int P = lane + q * kWave;
      const int rr = P / XS, sl = P % XS;
      *reinterpret_cast<float4*>(xt + rr * D + 4 * (sl ^ (rr & (XS - 1) & 31))) = xv[q];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    float s = 0.f, e = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int s0 = (ks * 16 + 8 * h) / 4;
      const int sw = r & (XS - 1) & 31;
      const float4 a = *reinterpret_cast<const float4*>(xt + r * D + 4 * (s0 ^ sw));
      const float4 b = *reinterpret_cast<const float4*>(xt + r * D + 4 * ((s0 + 1) ^ sw));
      const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      uint32_t ph[4], pl[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        short h0, l0, h1, l1;
        const float d0 = split_f16e(v[2 * j], xscale, h0, l0);
        const float d1 = split_f16e(v[2 * j + 1], xscale, h1, l1);
        ph[j] = (uint32_t)(uint16_t)h0 | ((uint32_t)(uint16_t)h1 << 16);
        pl[j] = (uint32_t)(uint16_t)l0 | ((uint32_t)(uint16_t)l1 << 16);
        s = fmaf(v[2 * j], v[2 * j], s);
        s = fmaf(v[2 * j + 1], v[2 * j + 1], s);
        e = fmaf(d0, d0, e);
        e = fmaf(d1, d1, e);
      }
      bh[t][ks] = __builtin_bit_cast(bf16x8, ph);
      bl[t][ks] = __builtin_bit_cast(bf16x8, pl);
      if constexpr (NOD) asm volatile("" : "+v"(bh[t][ks]));
      else asm volatile("" : "+v"(bh[t][ks]), "+v"(bl[t][ks]));
    }
    xn[t] = s + __shfl_xor(s, 32, 64);
    xe[t] = e + __shfl_xor(e, 32, 64);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // slice reads done before the next tile
  }
  }
  __syncthreads();                                         // staging area free; scn visible

  const int nchunks = Cpad / 32;
  // one stage = G centroid chunks, DMA'd into dbuf (per-thread offsets from a uniform stage base)
  auto stage = [&](int stg, uint16_t* __restrict__ dbuf) __attribute__((always_inline)) {
    const uint16_t* sbase = Chi + (int64_t)stg * G * CH_ELEMS;
#pragma unroll
    for (int k = 0; k < PER_THREAD; ++k) {
      const int P = threadIdx.x + k * kScrThreads;
      const int g = P / PIECES;
      if (P >= G * PIECES || stg * G + g >= nchunks) continue;
      const int Q = P % PIECES;
      const int cr = Q / SLOTS, sw = Q % SLOTS;
      const int sl = sw ^ (cr & 15 & (SLOTS - 1));
      __builtin_amdgcn_global_load_lds(sbase + ((g * 32 + cr) * D + sl * 8),
                                       dbuf + (wid * kWave + k * kScrThreads) * 8, 16, 0, 0);   // wave-uniform dst
    }
  };
  // Running (best, second) per row.  PAIR keeps explicit indices RELATIVE to the current
  // chunk base (ch*32 + 4h): candidates are the inline constants (i&3) + 8*(i>>2) and a new
  // chunk costs one subtract; it also keeps the second's index and the THIRD value
  // (v_med3 again): a row whose third is clear of the best by the bound has its arg-min
  // among {best, second} and is settled by two exact distances instead of the split
  // re-solve (8 VALU per distance).  The plain screen carries the slot in the key's low
  // mantissa bits (3 VALU per distance, epi_step) and the chunk of the best in bch.
  float best[TT], second[TT], third[TT];
  int bidx[TT], sidx[TT], bch[TT];
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    best[t] = INFINITY; second[t] = INFINITY; third[t] = INFINITY; bidx[t] = 0; sidx[t] = 0; bch[t] = 0;
  }
  auto epilogue = [&](const f32x16 (&a)[TT], int ch) __attribute__((always_inline)) {
    if constexpr (PAIR) {
#pragma unroll
      for (int t = 0; t < TT; ++t) {                     // re-base onto this chunk
        bidx[t] -= 32;
        sidx[t] -= 32;
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int k = (i & 3) + 8 * (i >> 2);
#pragma unroll
        for (int t = 0; t < TT; ++t) {
          const float dv = a[t][i];
          const bool better = dv < best[t];
          const bool better2 = dv < second[t];
          third[t] = __builtin_amdgcn_fmed3f(second[t], dv, third[t]);
          sidx[t] = better ? bidx[t] : (better2 ? k : sidx[t]);
          second[t] = __builtin_amdgcn_fmed3f(best[t], dv, second[t]);
          bidx[t] = better ? k : bidx[t];
          best[t] = better ? dv : best[t];
        }
      }
    }
  };
  // plain screen: two distances of the previous chunk (pair e of E = 8 TT, tiles
  // interleaved) folded into the running (best, second) keys.  With best <= second, the
  // second smallest of {best, second, ka, kb} is min(second, med3(best, ka, kb)): 3 VALU
  // per PAIR (med3, min3, min) plus the two slot codes -- 2.5 VALU per distance where one
  // distance at a time took 3 (med3, min, slot), which left the SIMD's issue port, not
  // the matrix core, setting the pace (103 VALU per 16 MFMAs of a chunk).
  auto epi_step = [&](const f32x16 (&a)[TT], int e) __attribute__((always_inline)) {
    const int t = e % TT, i = 2 * (e / TT);
    const float ka = __uint_as_float((__float_as_uint(a[t][i]) & 0xfffffff0u) | (uint32_t)i);
    const float kb = __uint_as_float((__float_as_uint(a[t][i + 1]) & 0xfffffff0u) | (uint32_t)(i + 1));
    float m3, b3, s2;
    // the instructions themselves: fminf / fmed3 would canonicalise the (bit-built) keys
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(m3) : "v"(best[t]), "v"(ka), "v"(kb));
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(b3) : "v"(best[t]), "v"(ka), "v"(kb));
    asm("v_min_f32 %0, %1, %2" : "=v"(s2) : "v"(second[t]), "v"(m3));
    best[t] = b3;
    second[t] = s2;
  };
  // one chunk's MFMAs: accumulators start at ||c||^2 (bias folded into the first MFMA's C)
  // One chunk's MFMAs (accumulators start at S ||c||^2, the bias folded into the first
  // MFMA's C).  EPI: the previous chunk's epilogue (accumulator old, chunk ch_old) is
  // spread over the k-steps, E/KS distance pairs after each step's MFMAs, so the wave issues
  // that VALU work while its own MFMAs occupy the matrix pipe.
  auto sweep = [&](auto epi_tag, const uint16_t* Lh, const float* sc, int ch, f32x16 (&acc)[TT],
                   const f32x16 (&old)[TT], int ch_old) __attribute__((always_inline)) {
    constexpr bool EPI = decltype(epi_tag)::value;
    constexpr int E = 8 * TT;                                     // distance pairs
    const int cbase = ch * 32 + 4 * h;
    f32x16 c0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 c4 = *reinterpret_cast<const float4*>(sc + cbase + 8 * q);
      c0[4 * q + 0] = c4.x; c0[4 * q + 1] = c4.y; c0[4 * q + 2] = c4.z; c0[4 * q + 3] = c4.w;
    }
    auto afrag = [&](int ks) __attribute__((always_inline)) {
      const int sw = (ks * 2 + h) ^ (r & 15 & (SLOTS - 1));
      return *reinterpret_cast<const bf16x8*>(Lh + r * D + sw * 8);
    };
    float b0[TT];
#pragma unroll
    for (int t = 0; t < TT; ++t) b0[t] = best[t];
    bf16x8 nh = afrag(0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const bf16x8 ah = nh;
      if (ks + 1 < KS) nh = afrag(ks + 1);
#pragma unroll
      for (int t = 0; t < TT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, ah),
                                                         __builtin_bit_cast(f16x8, bh[t][ks]),
                                                         ks == 0 ? c0 : acc[t], 0, 0, 0);
      if constexpr (EPI) {
#pragma unroll
        for (int e = ks * E / KS; e < (ks + 1) * E / KS; ++e) epi_step(old, e);
      }
    }
    if constexpr (EPI) {
#pragma unroll
      for (int t = 0; t < TT; ++t) bch[t] = best[t] != b0[t] ? ch_old : bch[t];
    }
  };
  // The plain screen's chunk sweep with its centre fragments loaded one chunk AHEAD (all KS
  // of them, double-buffered in registers): the next chunk's LDS reads are issued at the
  // top of this chunk's sweep, so no MFMA waits on a fragment read (the one-step-ahead
  // read of the loop above left a lgkmcnt wait every other k-step).
  auto load_frags = [&](const uint16_t* Lh, bf16x8 (&F)[KS]) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int sw = (ks * 2 + h) ^ (r & 15 & (SLOTS - 1));
      F[ks] = *reinterpret_cast<const bf16x8*>(Lh + r * D + sw * 8);
    }
  };
  auto sweep_f = [&](const bf16x8 (&F)[KS], const uint16_t* Lnext, bf16x8 (&Fn)[KS], const float* sc, int ch,
                     f32x16 (&acc)[TT], const f32x16 (&old)[TT], int ch_old) __attribute__((always_inline)) {
    constexpr int E = 8 * TT;
    const int cbase = ch * 32 + 4 * h;
    f32x16 c0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 c4 = *reinterpret_cast<const float4*>(sc + cbase + 8 * q);
      c0[4 * q + 0] = c4.x; c0[4 * q + 1] = c4.y; c0[4 * q + 2] = c4.z; c0[4 * q + 3] = c4.w;
    }
    if (Lnext) load_frags(Lnext, Fn);
    float b0[TT];
#pragma unroll
    for (int t = 0; t < TT; ++t) b0[t] = best[t];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int t = 0; t < TT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, F[ks]),
                                                         __builtin_bit_cast(f16x8, bh[t][ks]),
                                                         ks == 0 ? c0 : acc[t], 0, 0, 0);
#pragma unroll
      for (int e = ks * E / KS; e < (ks + 1) * E / KS; ++e) epi_step(old, e);
    }
#pragma unroll
    for (int t = 0; t < TT; ++t) bch[t] = best[t] != b0[t] ? ch_old : bch[t];
  };
  stage(0, lds);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // ping-pong accumulators: the epilogue of one chunk runs beside the next chunk's MFMAs
  f32x16 accA[TT], accB[TT];
  const int nstages = (nchunks + G - 1) / G;
  using Yes = std::integral_constant<bool, true>;
  using No = std::integral_constant<bool, false>;
  if constexpr (!PAIR) {
    // sentinel 2^126: the first chunk's "previous" epilogue cannot beat a real distance
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
      for (int j = 0; j < 16; ++j) accB[t][j] = 0x1p126f;
  }
  bool pendA = false, pendB = false;
  bf16x8 FA[KS], FB[KS];
  // One stage's body with its three LDS regions as __restrict__ pointers: the scoped
  // no-alias info lets hipcc's wait insertion see that the chunk / ||c||^2 reads do not
  // touch the next stage's in-flight DMA (otherwise it drains that DMA, vmcnt(0), before
  // the first read of every chunk).  G is even, so chunk pairs never straddle stages.
  auto run_stage = [&](int stg, const uint16_t* __restrict__ cur, uint16_t* __restrict__ nxt,
                       const float* __restrict__ sc) __attribute__((always_inline)) {
    if (stg + 1 < nstages) stage(stg + 1, nxt);
#pragma unroll
    for (int g = 0; g < G; g += 2) {
      const int ch = stg * G + g;
      if constexpr (PAIR) {
        if (ch < nchunks) {
          sweep(No{}, cur + g * CH_ELEMS, sc, ch, accA, accB, 0);
          if (pendB) epilogue(accB, ch - 1);
          pendA = true; pendB = false;
        }
        if (ch + 1 < nchunks) {
          sweep(No{}, cur + (g + 1) * CH_ELEMS, sc, ch + 1, accB, accA, 0);
          if (pendA) epilogue(accA, ch);
          pendB = true; pendA = false;
        }
      } else if constexpr (!(kScrFragAhead && NOD)) {   // (with lo halves held: too many registers)
        if (ch < nchunks) sweep(Yes{}, cur + g * CH_ELEMS, sc, ch, accA, accB, ch - 1);
        if (ch + 1 < nchunks) sweep(Yes{}, cur + (g + 1) * CH_ELEMS, sc, ch + 1, accB, accA, ch);
      } else {
        // fragments of chunk g in FA (g even) / FB (g odd); the stage's first chunk loads
        // its own after the stage barrier, every later one was loaded by its predecessor
        // (a chunk index past nchunks reads stale LDS that no MFMA uses)
        if (g == 0) load_frags(cur, FA);
        if (ch < nchunks) sweep_f(FA, cur + (g + 1) * CH_ELEMS, FB, sc, ch, accA, accB, ch - 1);
        if (ch + 1 < nchunks)
          sweep_f(FB, g + 2 < G ? cur + (g + 2) * CH_ELEMS : nullptr, FA, sc, ch + 1, accB, accA, ch);
      }
    }
  };
  for (int stg = 0; stg < nstages; ++stg) {
    const int buf = stg & 1;
    run_stage(stg, lds + buf * G * CH_ELEMS, lds + (buf ^ 1) * G * CH_ELEMS, scn);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // the last chunk's epilogue (chunk c sits in accA when c is even)
  if constexpr (PAIR) {
    if (pendA) epilogue(accA, nchunks - 1);
    if (pendB) epilogue(accB, nchunks - 1);
  } else {
    const bool lastA = ((nchunks - 1) & 1) == 0;
    float b0[TT];
#pragma unroll
    for (int t = 0; t < TT; ++t) b0[t] = best[t];
    if (lastA) {
#pragma unroll
      for (int e = 0; e < 8 * TT; ++e) epi_step(accA, e);
    } else {
#pragma unroll
      for (int e = 0; e < 8 * TT; ++e) epi_step(accB, e);
    }
#pragma unroll
    for (int t = 0; t < TT; ++t) bch[t] = best[t] != b0[t] ? nchunks - 1 : bch[t];
  }
  const int last_base = (nchunks - 1) * 32 + 4 * h;

#pragma unroll
  for (int t = 0; t < TT; ++t) {
    // absolute indices, then merge the half-waves (disjoint centroid subsets of one row):
    // the k-th smallest of two sorted triples is min over i + j = k of max(a_i, b_j)
    int myi;
    if constexpr (PAIR) {
      myi = bidx[t] + last_base;
    } else {
      const uint32_t slot = __float_as_uint(best[t]) & 15u;
      myi = bch[t] * 32 + 4 * h + (int)((slot & 3u) + 8u * (slot >> 2));
    }
    const int mys = sidx[t] + last_base;
    const float ob = __shfl_xor(best[t], 32, 64), os = __shfl_xor(second[t], 32, 64);
    const int oi = __shfl_xor(myi, 32, 64);
    const float sec = fminf(fmaxf(best[t], ob), fminf(second[t], os));
    const bool take = ob < best[t] || (ob == best[t] && oi < myi);
    const int idx = take ? oi : myi;
    const float bv = fminf(best[t], ob);
    // a row whose distances never compared (all NaN / inf) keeps an out-of-range index:
    // clamp it for the loads below; the NaN margin flags the row for the exact re-solve
    const bool idx_ok = idx >= 0 && idx < Cpad;
    int idx2 = idx;
    float thr = INFINITY;
    if (PAIR) {
      const float ot = __shfl_xor(third[t], 32, 64);
      const int osi = __shfl_xor(mys, 32, 64);
      thr = fminf(fminf(third[t], ot), fminf(fmaxf(second[t], ob), fmaxf(best[t], os)));
      // the runner-up: the other list's head against the winner list's second
      idx2 = take ? ((best[t] < os || (best[t] == os && myi < osi)) ? myi : osi)
                  : ((ob < second[t] || (ob == second[t] && oi < mys)) ? oi : mys);
    }
    // exact fp32 squared distances from x = (xh + xl) / xs (branch-free: padded columns
    // hold x = 0 and read c = 0) -- to the chosen centre, and (PAIR) to the runner-up
    const float ixs = 1.f / xscale;
    const int idc = idx_ok ? idx : 0;
    const int idc2 = idx2 >= 0 && idx2 < Cpad ? idx2 : idc;
    float s = 0.f, s2 = 0.f;
    if constexpr (!NOD) {
    const float* cp = C32 + (int64_t)idc * ldc;
    const float* cq = C32 + (int64_t)idc2 * ldc;
    // every centre-row load in flight before the first use (one L2 round trip, not KS)
    float4 cu[KS], cwv[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int c0 = ks * 16 + 8 * h;
      cu[ks] = *reinterpret_cast<const float4*>(cp + (c0 < Dx ? c0 : 0));
      cwv[ks] = *reinterpret_cast<const float4*>(cp + (c0 + 4 < Dx ? c0 + 4 : 0));
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int c0 = ks * 16 + 8 * h;
      const bool v0 = c0 < Dx, v1 = c0 + 4 < Dx;
      float4 u = cu[ks];
      float4 w = cwv[ks];
      if (!v0) u = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!v1) w = make_float4(0.f, 0.f, 0.f, 0.f);
      const float cv[8] = {u.x, u.y, u.z, u.w, w.x, w.y, w.z, w.w};
      float cw[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (PAIR) {
        float4 u2 = *reinterpret_cast<const float4*>(cq + (v0 ? c0 : 0));
        float4 w2 = *reinterpret_cast<const float4*>(cq + (v1 ? c0 + 4 : 0));
        if (!v0) u2 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!v1) w2 = make_float4(0.f, 0.f, 0.f, 0.f);
        cw[0] = u2.x; cw[1] = u2.y; cw[2] = u2.z; cw[3] = u2.w;
        cw[4] = w2.x; cw[5] = w2.y; cw[6] = w2.z; cw[7] = w2.w;
      }
      const uint32_t* ph = reinterpret_cast<const uint32_t*>(&bh[t][ks]);
      const uint32_t* pl = reinterpret_cast<const uint32_t*>(&bl[t][ks]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t hw = ph[j >> 1], lw = pl[j >> 1];
        const float xh = f16_bits_to_f32((j & 1) ? (hw >> 16) : (hw & 0xffffu));
        const float xl = f16_bits_to_f32((j & 1) ? (lw >> 16) : (lw & 0xffffu));
        const float xv = (xh + xl) * ixs;
        const float df = xv - cv[j];
        s = fmaf(df, df, s);
        if (PAIR) {
          const float dg = xv - cw[j];
          s2 = fmaf(dg, dg, s2);
        }
      }
    }
    s += __shfl_xor(s, 32, 64);
    if (PAIR) s2 += __shfl_xor(s2, 32, 64);
    }
    const int64_t row_l = row_base + t * 32 + r;                  // position in this launch
    const bool ok = row_l < n && h == 0;
    const int64_t row = rowlist ? (int64_t)rowlist[ok ? row_l : 0] : row_l;   // the data row
    // in the scaled units of bv, sec; the plain screen's slot codes move each key by less
    // than 2^-19 of its magnitude (twice that allowed for)
    float bound = 2.f * (sscale * (eps_x * sqrtf(xn[t]) + eps0) + eps_e * sqrtf(xe[t]));
    if constexpr (!PAIR) bound += 0x1p-18f * (fabsf(bv) + fabsf(sec));
    bool fl = ok && (!(sec - bv > bound) || !idx_ok);      // near-tie (or NaN): exact re-solve
    int pick = idc;
    float pd = s;
    if (PAIR && fl && idx_ok && idc2 == idx2 && thr - bv > bound) {
      // every other centre is provably farther than both: the exact pair decides
      fl = false;
      const bool second_wins = s2 < s || (s2 == s && idx2 < idx);
      pick = second_wins ? idx2 : idc;
      pd = second_wins ? s2 : s;
    }
    if (ok) {
      assign[row] = pick;
      if (!NOD && mind) mind[row] = pd;
      if (bnd) {
        // Hamerly bounds for the next Lloyd iteration (unscaled distances, not squared):
        // ub >= ||x - c_pick||, lb <= ||x - c|| for every other centre.  Screened partial
        // distances (||c||^2 - 2 x.c) are within bound / (2 S) of the exact ones (the whole
        // bound is used), plus fp32 rounding of ||x||^2 + partial.  Near ties: (inf, 0) --
        // rechecked next time.
        float2 o = make_float2(INFINITY, 0.f);
        if (!fl && !PAIR) {
          const float inv = 1.f / sscale;
          const float pb = bv * inv, psec = sec * inv, mg = bound * inv;
          const float slack = 0x1p-20f * (xn[t] + fabsf(pb) + fabsf(psec));
          o.x = sqrtf(fmaxf(xn[t] + pb + mg + slack, 0.f)) * (1.f + 0x1p-20f);
          o.y = sqrtf(fmaxf(xn[t] + psec - mg - slack, 0.f)) * (1.f - 0x1p-20f);
        }
        bnd[row] = o;
      }
    }
    const uint64_t m = __ballot(fl);
    if (m) {
      const int leader = __ffsll((unsigned long long)m) - 1;
      int base = 0;
      if (lane == leader) base = atomicAdd(flag_cnt, (int)__popcll(m));
      base = __shfl(base, leader, 64);
      if (fl) flag_rows[base + __popcll(m & ((1ull << lane) - 1ull))] = (int32_t)row;
    }
  }
}

// ---------------------------------------------------------------------------------
constexpr int kUpdThreads = 512;
constexpr int kUpdWaves = kUpdThreads / kWave;

// Rows per chunk R (host-chosen, <= 65536 so sorted indices fit uint16): the largest of
// 16384..1024 whose LDS image fits.  Bigger chunks amortise the per-chunk slab
// read-modify-write (Kp x D floats) over more X bytes.
__host__ __device__ inline int upd_lds_bytes(int Kp, int R) {
  // start[Kp+1] int + per-(wave, cluster) uint16 counts + sorted[R] uint16
  return (int)(sizeof(int) * (Kp + 1) + sizeof(uint16_t) * (kUpdWaves * Kp + R));
}
inline int upd_rows(int Kp) {
  for (int R = 16384; R >= 8192; R >>= 1)              // 2 blocks per CU
    if (upd_lds_bytes(Kp, R) <= 80 * 1024) return R;
  for (int R = 16384; R >= 256; R >>= 1)               // 1 block per CU
    if (upd_lds_bytes(Kp, R) <= 160 * 1024) return R;
  return 0;
}

// One block: chunks of R rows; slab (block-private) = [Kp][D] sums + [Kp] counts.
// Counting sort by cluster that is STABLE without any sort pass: wave w owns rows
// [w R/8, (w+1) R/8) of the chunk; per-(wave, cluster) counts give each wave its base
// inside every bucket, and inside a wave the 64-row groups are scattered in row order
// with ballot ranking (peel one key per step: rank = popcount of same-key lanes below).
// Bucket order is therefore row order -> bitwise-deterministic sums for any k (the old
// in-bucket insertion sort was O(bucket^2) per thread, i.e. quadratic at small k).
// DV: floats per lane per row (scalar path, D <= 64 * DV); LPR > 0: vector path, LPR
// lanes x float4 per row (D <= 4 * LPR, D % 4 == 0, 16-B rows), 64 / LPR rows per load.
template <int DV, int LPR>
__global__ __launch_bounds__(kUpdThreads) void kmeans_update_kernel(
    const float* __restrict__ X, int64_t n, int64_t ldx, int D, const int32_t* __restrict__ assign,
    int Kp, int R, float* __restrict__ slab, float* __restrict__ cnt_slab) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  int* start = smem;                                    // [Kp+1] bucket starts
  // [waves][Kp] uint16 counts -> per-wave bases (seg <= 2048 rows per wave fits 16 bits).
  // Counted as 32-bit LDS atomics on the word shared by waves 2j / 2j+1 (halves never carry).
  uint16_t* cntw = reinterpret_cast<uint16_t*>(start + Kp + 1);
  uint32_t* cnt32 = reinterpret_cast<uint32_t*>(cntw);  // [waves/2][Kp] words
  uint16_t* sorted = cntw + kUpdWaves * Kp;             // [R]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int seg = R / kUpdWaves;                        // rows per wave segment (multiple of 64)
  uint16_t* mycw = cntw + (wid >> 1) * 2 * Kp;          // element (key) at mycw[2*key + (wid&1)]
  const int half = wid & 1;
  float* myslab = slab + (int64_t)blockIdx.x * Kp * D;
  float* mycnt = cnt_slab + (int64_t)blockIdx.x * Kp;
  const int64_t nch = (n + R - 1) / R;
  for (int64_t cidx = blockIdx.x; cidx < nch; cidx += gridDim.x) {
    const int64_t r0 = cidx * R;
    const int rows = (int)min((int64_t)R, n - r0);
    for (int i = threadIdx.x; i < kUpdWaves / 2 * Kp; i += kUpdThreads) cnt32[i] = 0u;
    __syncthreads();
    const int s0 = wid * seg, s1 = min(rows, s0 + seg);
    for (int i = s0 + lane; i < s1; i += kWave)
      atomicAdd(&cnt32[(wid >> 1) * Kp + assign[r0 + i]], 1u << (16 * half));
    __syncthreads();
    // per cluster: exclusive prefix over waves (in place), total -> start[]
    for (int c = threadIdx.x; c < Kp; c += kUpdThreads) {
      int run = 0;
#pragma unroll
      for (int j = 0; j < kUpdWaves / 2; ++j) {
        const uint32_t v = cnt32[j * Kp + c];
        const int lo = (int)(v & 0xffffu), hi = (int)(v >> 16);
        cnt32[j * Kp + c] = (uint32_t)run | ((uint32_t)(run + lo) << 16);
        run += lo + hi;
      }
      start[c] = run;
    }
    __syncthreads();
    if (wid == 0) {   // exclusive scan of bucket sizes by one wave
      int carry = 0;
      for (int b = 0; b < Kp; b += 64) {
        const int v = (b + lane < Kp) ? start[b + lane] : 0;
        int x = v;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const int y = __shfl_up(x, off, 64);
          if (lane >= off) x += y;
        }
        if (b + lane < Kp) start[b + lane] = carry + x - v;
        carry += __shfl(x, 63, 64);
      }
      if (lane == 0) start[Kp] = carry;
    }
    __syncthreads();
    // stable scatter: this wave's groups in row order; mycw[k] is the running base
    for (int g = s0; g < s1; g += kWave) {
      const int i = g + lane;
      const int key = i < s1 ? assign[r0 + i] : -1;
      if (Kp <= 32) {
        // few clusters: peel one key per step (<= 32 steps, usually a handful)
        uint64_t todo = __ballot(i < s1);
        while (todo) {
          const int leader = __ffsll((unsigned long long)todo) - 1;
          const int k = __shfl(key, leader, 64);
          const uint64_t m = __ballot(key == k);
          if (key == k) {
            const int rank = __popcll(m & ((1ull << lane) - 1ull));
            sorted[start[k] + mycw[2 * k + half] + rank] = (uint16_t)i;
          }
          if (lane == leader) mycw[2 * k + half] = (uint16_t)(mycw[2 * k + half] + __popcll(m));
          todo &= ~m;
        }
      } else {
        // many clusters (up to 64 distinct keys per group): bitonic-sort the 64
        // (key, lane) pairs in registers (21 compare-exchange steps), then every lane's
        // rank inside its key run comes from one ballot of the run heads -- the same
        // stable order as the peeling loop at a fraction of its ~64 iterations
        uint32_t v = ((uint32_t)(key < 0 ? 0xFFFF : key) << 6) | (uint32_t)lane;
#pragma unroll
        for (int kk = 2; kk <= 64; kk <<= 1) {
#pragma unroll
          for (int j = kk >> 1; j > 0; j >>= 1) {
            const uint32_t o = (uint32_t)__shfl_xor((int)v, j, 64);
            const bool keep_min = ((lane & kk) == 0) == ((lane & j) == 0);
            v = keep_min ? (v < o ? v : o) : (v > o ? v : o);
          }
        }
        const int k = (int)(v >> 6);
        const bool valid = k != 0xFFFF;
        const int prev = __shfl_up((int)v, 1, 64) >> 6;
        const int next = __shfl_down((int)v, 1, 64) >> 6;
        const uint64_t heads = __ballot(valid && (lane == 0 || prev != k));
        const uint64_t upto = ~0ull >> (63 - lane);                  // bits 0..lane
        const int run0 = 63 - __clzll((long long)(heads & upto));
        const int rank = lane - run0;
        if (valid) {
          sorted[start[k] + mycw[2 * k + half] + rank] = (uint16_t)(g + (int)(v & 63u));
          if (lane == 63 || next != k) mycw[2 * k + half] = (uint16_t)(mycw[2 * k + half] + rank + 1);
        }
      }
    }
    __syncthreads();
    // wave w owns clusters [c0, c1): its rows are the contiguous sorted range
    const int c0 = (int)((int64_t)Kp * wid / kUpdWaves), c1 = (int)((int64_t)Kp * (wid + 1) / kUpdWaves);
    if constexpr (LPR > 0) {
      // Streaming form: the wave's sorted range is cut at cluster boundaries into RPI
      // contiguous pieces, one per row slot (LPR lanes x float4 = one row); each slot
      // streams its rows with U loads in flight and flushes its register sum to the
      // block slab whenever the cluster changes.  No cluster spans two slots (cut points
      // are bucket starts), so every cluster is summed by one slot in row order
      // (deterministic) and loads stay in flight across cluster boundaries -- the old
      // per-cluster loop waited one HBM round trip per (small) cluster.
      constexpr int RPI = kWave / LPR;
      constexpr int U = 8;
      const int slot = lane / LPR, col = 4 * (lane % LPR);
      const bool cok = col < D;
      const int b0 = start[c0], b1 = start[c1];
      auto cut = [&](int sl) {                    // first cluster of piece sl
        if (sl <= 0) return c0;
        if (sl >= RPI) return c1;
        const int t = b0 + (int)((int64_t)(b1 - b0) * sl / RPI);
        int lo = c0, hi = c1;                     // smallest c in [c0, c1] with start[c] >= t
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (start[mid] >= t) hi = mid; else lo = mid + 1;
        }
        return lo;
      };
      int c = cut(slot);
      const int pe = start[cut(slot + 1)];
      const int pb = start[c];
      int cend = c < c1 ? start[c + 1] : pb;      // (empty piece at the last cluster: no rows)
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      auto flush = [&](int cc) {
        if (!cok) return;
        float4* dst = reinterpret_cast<float4*>(myslab + (int64_t)cc * D + col);
        float4 d4 = *dst;
        d4.x += acc.x; d4.y += acc.y; d4.z += acc.z; d4.w += acc.w;
        *dst = d4;
      };
      for (int t = pb; __ballot(t < pe) != 0ull; t += U) {
        float4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int pos = t + u;
          x[u] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (cok && pos < pe) x[u] = *reinterpret_cast<const float4*>(X + (r0 + sorted[pos]) * ldx + col);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int pos = t + u;
          if (pos < pe) {
            while (pos >= cend) {                 // leave cluster c (flush it if it had rows)
              if (cend > start[c]) flush(c);
              acc = make_float4(0.f, 0.f, 0.f, 0.f);
              ++c;
              cend = start[c + 1];
            }
            acc.x += x[u].x; acc.y += x[u].y; acc.z += x[u].z; acc.w += x[u].w;
          }
        }
      }
      if (pe > pb) flush(c);
      for (int cc = c0 + lane; cc < c1; cc += kWave) {
        const int sz = start[cc + 1] - start[cc];
        if (sz) mycnt[cc] += (float)sz;
      }
    } else {
    for (int c = c0; c < c1; ++c) {
      const int b0 = start[c], b1 = start[c + 1];
      if (b0 == b1) continue;
      float acc[DV];
#pragma unroll
      for (int v = 0; v < DV; ++v) acc[v] = 0.f;
      int i = b0;
      for (; i + 4 <= b1; i += 4) {       // 4 rows in flight
        float x[4][DV];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float* xp = X + (r0 + sorted[i + u]) * ldx;
#pragma unroll
          for (int v = 0; v < DV; ++v) {
            const int col = lane + 64 * v;
            x[u][v] = col < D ? xp[col] : 0.f;
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int v = 0; v < DV; ++v) acc[v] += x[u][v];
      }
      for (; i < b1; ++i) {
        const float* xp = X + (r0 + sorted[i]) * ldx;
#pragma unroll
        for (int v = 0; v < DV; ++v) {
          const int col = lane + 64 * v;
          acc[v] += col < D ? xp[col] : 0.f;
        }
      }
      float* dst = myslab + (int64_t)c * D;
#pragma unroll
      for (int v = 0; v < DV; ++v) {
        const int col = lane + 64 * v;
        if (col < D) dst[col] += acc[v];
      }
      if (lane == 0) mycnt[c] += (float)(b1 - b0);
    }
    }
    __syncthreads();
  }
}

// sums[k][d] = sum_g slab[g][k][d] (fixed order), counts likewise.
__global__ void kmeans_reduce_kernel(const float* __restrict__ slab, const float* __restrict__ cnt_slab,
                                     int G, int64_t KD, int Kp, double* __restrict__ sums,
                                     double* __restrict__ counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < KD) {
    double s = 0.0;
    for (int g = 0; g < G; ++g) s += (double)slab[(int64_t)g * KD + i];
    sums[i] = s;
  }
  if (i < Kp) {
    double s = 0.0;
    for (int g = 0; g < G; ++g) s += (double)cnt_slab[(int64_t)g * Kp + i];
    counts[i] = s;
  }
}

}  // namespace

// D must be a multiple of 16 (<= 256), X rows 16-B aligned (ldx % 4 == 0); Cpad % 32 == 0.
// Dx: true feature count (% 4 == 0); Chi/Clo are [Cpad][Dp] with Dp = roundup(Dx, 32).
// rowlist (optional): process rows rowlist[0..n) of X (the screen pass's near-ties).
O3S_API int o3s_kmeans_assign(const float* X, int64_t n, int64_t ldx, int Dx, const void* Chi,
                              const void* Clo, const float* cn, int Cpad, int32_t* assign, float* mind,
                              const int32_t* rowlist, hipStream_t st) {
  if (n <= 0) return 0;
  const int D = (Dx + 31) / 32 * 32;
  if (Dx % 4 != 0 || D > 256 || ldx % 4 != 0 || Cpad % 32 != 0) return -1;
  const int rows_per_block = kAssignWaves * 32;
  const int grid = (int)((n + rows_per_block - 1) / rows_per_block);
  const uint16_t* hi = (const uint16_t*)Chi;
  const uint16_t* lo = (const uint16_t*)Clo;
  // chunk buffers: 2 buffers x G chunks x (hi + lo) x 32 x D bf16 = 128 KB at every D
  const size_t stage_bytes = 2 * (D <= 128 ? 4 : 2) * 2 * 32 * (size_t)D * 2;
  const bool cnl = stage_bytes + sizeof(float) * (size_t)Cpad <= 160 * 1024;
#define O3S_KA(KS)                                                                                   \
  case KS:                                                                                           \
    if (cnl)                                                                                         \
      hipLaunchKernelGGL((kmeans_assign_kernel<KS, 1, true>), dim3(grid), dim3(kAssignThreads),      \
                         stage_bytes + sizeof(float) * (size_t)Cpad, st, X, n, ldx, hi, lo, cn, Cpad, \
                         assign, mind, Dx, rowlist);                                                 \
    else                                                                                             \
      hipLaunchKernelGGL((kmeans_assign_kernel<KS, 1, false>), dim3(grid), dim3(kAssignThreads),     \
                         stage_bytes, st, X, n, ldx, hi, lo, cn, Cpad, assign, mind, Dx, rowlist);   \
    break;
  switch (D / 16) {
    O3S_KA(2) O3S_KA(4) O3S_KA(6) O3S_KA(8) O3S_KA(10) O3S_KA(12) O3S_KA(14) O3S_KA(16)
    default: return -2;
  }
#undef O3S_KA
  O3S_CHECK_LAUNCH();
  return 0;
}

// Screen pass (see kmeans_screen_kernel).  Ch16: fp16 bits of -2 C ms [Cpad][D]; C32: fp32
// centres [K][ldc] (ldc % 4 == 0); bound S E = S (eps_x ||x|| + eps0) + eps_e ||dx xs||
// (eps_e = eps_e' ms: the error norm is kept in the scaled units); xscale = xs, sscale = xs ms; flag_cnt (zeroed by the caller) / flag_rows [n]: near-tie rows for
// o3s_kmeans_assign(rowlist).  tt: 32-row tiles per wave (1 or 2).
namespace {
// X (fp32 [n][ldx], Dx valid columns) -> the screen kernel's pre-split rows: per row D/8
// groups (group g = 2 ks + h: dims 8 g .. 8 g + 7) of 16 B scaled-fp16 hi + 16 B lo (the
// split_f16 of the kernel's prologue, zero past Dx), and ||x||^2 in fp32.  One lane per
// group; the row norm is a shuffle reduction over the row's lanes.
template <int D>
__global__ __launch_bounds__(256) void kmeans_presplit_kernel(const float* __restrict__ X, int64_t n, int64_t ldx,
                                                              int Dx, float xscale, uint4* __restrict__ XP,
                                                              float2* __restrict__ XN) {
  constexpr int G = D / 8;                     // groups per row (power of two up to 64 lanes)
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = tid / G;
  const int g = (int)(tid % G);
  float s = 0.f, e = 0.f;
  if (row < n) {
    uint32_t ph[4], pl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c0 = 8 * g + 2 * j;
      const float v0 = c0 < Dx ? X[row * ldx + c0] : 0.f;
      const float v1 = c0 + 1 < Dx ? X[row * ldx + c0 + 1] : 0.f;
      short h0, l0, h1, l1;
      const float d0 = split_f16e(v0, xscale, h0, l0);
      const float d1 = split_f16e(v1, xscale, h1, l1);
      ph[j] = (uint32_t)(uint16_t)h0 | ((uint32_t)(uint16_t)h1 << 16);
      pl[j] = (uint32_t)(uint16_t)l0 | ((uint32_t)(uint16_t)l1 << 16);
      s = fmaf(v0, v0, s);
      s = fmaf(v1, v1, s);
      e = fmaf(d0, d0, e);
      e = fmaf(d1, d1, e);
    }
    XP[(row * G + g) * 2] = make_uint4(ph[0], ph[1], ph[2], ph[3]);
    XP[(row * G + g) * 2 + 1] = make_uint4(pl[0], pl[1], pl[2], pl[3]);
  }
#pragma unroll
  for (int o = 1; o < G; o <<= 1) {
    s += __shfl_xor(s, o, 64);
    e += __shfl_xor(e, o, 64);
  }
  if (row < n && g == 0) XN[row] = make_float2(s, e);
}
}  // namespace

// Pre-split rows for the screen kernel (see kmeans_presplit_kernel): XP [n][D / 8][2] x 16 B,
// XN [n] fp32; D = Dx rounded up to 32 (<= 128).
O3S_API int o3s_kmeans_presplit(const float* X, int64_t n, int64_t ldx, int Dx, float xscale, void* XP, float* XN2,
                                hipStream_t st) {
  float2* XN = reinterpret_cast<float2*>(XN2);
  if (n <= 0) return 0;
  const int D = (Dx + 31) / 32 * 32;
  if (Dx % 4 != 0 || D > 128) return -1;
  const int64_t threads = n * (D / 8);
  const dim3 grid((unsigned)((threads + 255) / 256));
  switch (D) {
    case 32: hipLaunchKernelGGL((kmeans_presplit_kernel<32>), grid, dim3(256), 0, st, X, n, ldx, Dx, xscale, (uint4*)XP, XN); break;
    case 64: hipLaunchKernelGGL((kmeans_presplit_kernel<64>), grid, dim3(256), 0, st, X, n, ldx, Dx, xscale, (uint4*)XP, XN); break;
    case 96: hipLaunchKernelGGL((kmeans_presplit_kernel<96>), grid, dim3(256), 0, st, X, n, ldx, Dx, xscale, (uint4*)XP, XN); break;
    case 128: hipLaunchKernelGGL((kmeans_presplit_kernel<128>), grid, dim3(256), 0, st, X, n, ldx, Dx, xscale, (uint4*)XP, XN); break;
    default: return -2;
  }
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_API int o3s_kmeans_screen2(const float* X, int64_t n, int64_t ldx, int Dx, const void* Chi, const float* cn,
                               const float* C32, int ldc, int Cpad, float eps_x, float eps0, float eps_e,
                               float xscale, float sscale, int32_t* assign, float* mind, int32_t* flag_cnt,
                               int32_t* flag_rows, int tt, int pair, const void* XP, const float* XN2,
                               const int32_t* rowlist, float* bnd2, hipStream_t st) {
  float2* bnd = reinterpret_cast<float2*>(bnd2);
  const float2* XN = reinterpret_cast<const float2*>(XN2);
  if (n <= 0) return 0;
  const int D = (Dx + 31) / 32 * 32;
  if (Dx % 4 != 0 || D > 160 || ldx % 4 != 0 || ldc % 4 != 0 || Cpad % 32 != 0 || n > 0x7fffffffll) return -1;
  if (tt != 1 && tt != 2) return -1;
  const size_t cdyn = sizeof(float) * (size_t)Cpad;
  const uint16_t* hi = (const uint16_t*)Chi;
#define O3S_KS(KS, TT)                                                                                     \
  {                                                                                                        \
    if (pair) O3S_KSP(KS, 1, true) else O3S_KSP(KS, TT, false)   /* PAIR: one tile per wave (registers) */ \
  }
#define O3S_KSP(KS, TT, P)                                                                                 \
  {                                                                                                        \
    const int rows_per_block = kScrWaves * 32 * TT;                                                        \
    const int64_t grid = (n + rows_per_block - 1) / rows_per_block;                                        \
    const size_t dyn = ScrLds<KS>::BYTES + cdyn;                                                           \
    if (dyn > 160 * 1024) return -3;                                                                       \
    if (XP && !P && !mind)                                                                          \
      hipLaunchKernelGGL((kmeans_screen_kernel<KS, TT, P, true, true>), dim3((unsigned)grid), dim3(kScrThreads), dyn, \
                         st, X, n, ldx, hi, cn, C32, ldc, Cpad, eps_x, eps0, eps_e, xscale, sscale, assign, mind,     \
                         flag_cnt, flag_rows, Dx, (const uint4*)XP, XN, rowlist, bnd);                     \
    else if (XP && !P)                                                                                     \
      hipLaunchKernelGGL((kmeans_screen_kernel<KS, TT, P, true>), dim3((unsigned)grid), dim3(kScrThreads), dyn, st, \
                         X, n, ldx, hi, cn, C32, ldc, Cpad, eps_x, eps0, eps_e, xscale, sscale, assign, mind, flag_cnt, \
                         flag_rows, Dx, (const uint4*)XP, XN, rowlist, bnd);                               \
    else if (!P && !mind)                                                                                  \
      hipLaunchKernelGGL((kmeans_screen_kernel<KS, TT, P, false, true>), dim3((unsigned)grid), dim3(kScrThreads), dyn, \
                         st, X, n, ldx, hi, cn, C32, ldc, Cpad, eps_x, eps0, eps_e, xscale, sscale, assign, mind,     \
                         flag_cnt, flag_rows, Dx, nullptr, nullptr, rowlist, bnd);                         \
    else                                                                                                   \
      hipLaunchKernelGGL((kmeans_screen_kernel<KS, TT, P>), dim3((unsigned)grid), dim3(kScrThreads), dyn, st, X, n, \
                         ldx, hi, cn, C32, ldc, Cpad, eps_x, eps0, eps_e, xscale, sscale, assign, mind, flag_cnt,   \
                         flag_rows, Dx, nullptr, nullptr, rowlist, bnd);                                   \
  }
  switch (D / 16) {
    case 2: if (tt == 2) O3S_KS(2, 2) else O3S_KS(2, 1) break;
    case 4: if (tt == 2) O3S_KS(4, 2) else O3S_KS(4, 1) break;
    case 6: if (tt == 2) O3S_KS(6, 2) else O3S_KS(6, 1) break;
    case 8: if (tt == 2) O3S_KS(8, 2) else O3S_KS(8, 1) break;
    case 10: O3S_KS(10, 1) break;
    default: return -2;
  }
#undef O3S_KS
#undef O3S_KSP
  O3S_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------
// Hamerly bound update of a Lloyd iteration (models/kmeans.py): per row, the upper bound
// on the distance to its centre grows by that centre's shift and the lower bound on every
// other centre shrinks by the largest shift; a row whose bounds no longer certify its
// centre (ub >= lb, or NaN) must be screened again.  Two passes, no atomics, rows in
// ascending order: block b owns the contiguous rows [b R, (b + 1) R); pass 0 updates the
// bounds and counts the block's rows to recheck; pass 1 (only when the caller wants the
// list) writes them at the block's prefix offset, ranked by ballots in row order.
constexpr int kBndThreads = 256;

__device__ __forceinline__ bool bnd_recheck(float2 b) { return !(b.x < b.y); }

__global__ __launch_bounds__(kBndThreads) void kmeans_bounds_kernel(
    const int32_t* __restrict__ a, float2* __restrict__ bnd, int64_t n, int64_t per_block,
    const float* __restrict__ delta, float dmax, int pass, int32_t* __restrict__ cnt,
    const int64_t* __restrict__ offs, int32_t* __restrict__ rows) {
  __shared__ int wtot[kBndThreads / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * per_block;
  const int64_t r1 = r0 + per_block < n ? r0 + per_block : n;
  int64_t out = pass ? offs[blockIdx.x] : 0;
  int total = 0;
  for (int64_t base = r0; base < r1; base += kBndThreads) {
    const int64_t i = base + threadIdx.x;
    bool need = false;
    if (i < r1) {
      float2 bv = bnd[i];
      if (pass == 0) {
        bv.x += delta[a[i]];
        bv.y -= dmax;
        bnd[i] = bv;
      }
      need = bnd_recheck(bv);
    }
    const uint64_t m = __ballot(need);
    if (pass == 0) {
      total += __popcll(m);                                  // wave-uniform
      continue;
    }
    if (lane == 0) wtot[wid] = __popcll(m);
    __syncthreads();
    int before = 0, all = 0;
#pragma unroll
    for (int q = 0; q < kBndThreads / 64; ++q) {
      before += q < wid ? wtot[q] : 0;
      all += wtot[q];
    }
    if (need) rows[out + before + __popcll(m & ((1ull << lane) - 1ull))] = (int32_t)i;
    out += all;
    __syncthreads();                                       // wtot reused next chunk
  }
  if (pass == 0) {
    if (lane == 0) wtot[wid] = total;
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      for (int q = 0; q < kBndThreads / 64; ++q) t += wtot[q];
      cnt[blockIdx.x] = t;
    }
  }
}

// pass 0: a int32 [n] centres, bnd fp32 [n][2] (ub, lb) moved in place by delta (fp32 [K],
// rounded up) / dmax; cnt int32 [grid] = rows to recheck per block.  pass 1: offs int64
// [grid] (exclusive prefix of cnt) -> rows int32 (ascending).  Rows per block: ceil(n / grid).
O3S_API int o3s_kmeans_bounds(const int32_t* a, float* bnd, int64_t n, const float* delta, float dmax, int pass,
                              int32_t* cnt, const int64_t* offs, int32_t* rows, int grid, hipStream_t st) {
  if (n <= 0) return 0;
  if (n > 0x7fffffffll || grid <= 0 || (pass == 1 && (!offs || !rows))) return -1;
  const int64_t per_block = (n + grid - 1) / grid;
  hipLaunchKernelGGL(kmeans_bounds_kernel, dim3(grid), dim3(kBndThreads), 0, st, a, reinterpret_cast<float2*>(bnd),
                     n, per_block, delta, dmax, pass, cnt, offs, rows);
  O3S_CHECK_LAUNCH();
  return 0;
}

// The screen without row list / bounds (the original entry point).
O3S_API int o3s_kmeans_update_ws(int Kp, int D, int grid, int64_t* slab_floats, int64_t* cnt_floats,
                                 int* lds_bytes) {
  const int R = upd_rows(Kp);
  *slab_floats = (int64_t)grid * Kp * D;
  *cnt_floats = (int64_t)grid * Kp;
  *lds_bytes = R ? upd_lds_bytes(Kp, R) : -1;   // -1: Kp too large for the LDS sort
  return R ? 0 : -3;
}

// slab/cnt_slab must be zeroed by the caller (hipMemsetAsync) before each call.
O3S_API int o3s_kmeans_update(const float* X, int64_t n, int64_t ldx, int D, const int32_t* assign, int Kp,
                              float* slab, float* cnt_slab, int grid, double* sums, double* counts,
                              hipStream_t st) {
  if (D > 256 || n < 0) return -1;
  const int R = upd_rows(Kp);
  if (!R) return -3;
  const int lds = upd_lds_bytes(Kp, R);
  if (n > 0) {
#define O3S_KU(DV, LPR)                                                                               \
  hipLaunchKernelGGL((kmeans_update_kernel<DV, LPR>), dim3(grid), dim3(kUpdThreads), lds, st, X, n, ldx, D, \
                     assign, Kp, R, slab, cnt_slab);
    const bool vec = D % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)X & 15) == 0;
    if (vec) {
      if (D <= 32) { O3S_KU(1, 8) } else if (D <= 64) { O3S_KU(1, 16) } else if (D <= 128) { O3S_KU(2, 32) }
      else { O3S_KU(4, 64) }
    } else {
      if (D <= 64) { O3S_KU(1, 0) } else if (D <= 128) { O3S_KU(2, 0) } else if (D <= 192) { O3S_KU(3, 0) }
      else { O3S_KU(4, 0) }
    }
#undef O3S_KU
    O3S_CHECK_LAUNCH();
  }
  const int64_t KD = (int64_t)Kp * D;
  const int64_t work = KD > Kp ? KD : Kp;
  hipLaunchKernelGGL(kmeans_reduce_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, st, slab, cnt_slab,
                     grid, KD, Kp, sums, counts);
  O3S_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------
// k-means|| seeding, step 2 (Spark LocalKMeans.kMeansPlusPlus on the weighted candidates):
// greedy k-means++ -- per step, `trials` weighted draws from w * d2 (inverse CDF over a
// prefix sum), each draw's potential sum_i w_i min(d2_i, |p_i - c|^2), the best one kept.
// Distances by the |p|^2 + |c|^2 - 2 p.c form of the torch reference
// (models/kmeans._local_kmeanspp) over fp32-rounded coordinates, products and sums in fp64;
// draws from the same counter-hash uniforms U [k][trials + 1].
//
// Two launches per step, spread over the GPU: kpp_dist_kernel (one row per thread, every
// candidate row of the chip at once: the trials' distances cd [trials][m] and per-block
// partial potentials) and kpp_pick_kernel (one block: the potentials summed over the blocks
// in a fixed order, the pick, d2 = min(d2, cd[best]), the prefix sum of w * d2 in LDS and
// the next step's draws).  The host loop in o3s_kmeanspp enqueues all 2k launches.  (A
// single workgroup running all k steps spent 0.17 s of a 0.33 s k-means|| init at k = 1024,
// m = 4097 -- 94% of it in the fp64 distance sums one CU can issue:
// profiles/kmeans_init_phases_r5.json.)
namespace {
constexpr int kPPThreads = 512;             // kpp_pick_kernel
constexpr int kPDThreads = 256;             // kpp_dist_kernel
constexpr int kPPMaxT = 16;

__device__ double pp_block_sum(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  return t;
}

// first index i with cs[i] > u * tot (searchsorted right), clamped; tot <= 0: uniform
__device__ int pp_draw(const double* cs, int m, double tot, double u) {
  if (!(tot > 0.0)) {
    const long long r = (long long)(u * m);
    return (int)(r < m - 1 ? r : m - 1);
  }
  const double x = u * tot;
  int lo = 0, hi = m;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cs[mid] > x) hi = mid; else lo = mid + 1;
  }
  return lo < m - 1 ? lo : m - 1;
}

// mode 0: d2[i] = |p_i - p_cand[0]|^2 (the first centre); mode 1: cd[j][i] = distance of
// row i to trial candidate j and partial[block][j] = sum over the block's rows of
// w_i min(d2_i, cd[j][i]).  PT: fp32 [D][m]; pn: |p|^2 of the rounded rows (fp64).
__device__ void kpp_dist(const float* __restrict__ PT, const double* __restrict__ w, const double* __restrict__ pn,
                         int m, int D, int trials, const int* __restrict__ cand, int mode, double* __restrict__ d2,
                         double* __restrict__ cd, double* __restrict__ partial, int blk, double* sc, double* red) {
  // sc: [trials][D] candidate coordinates (LDS); red: [kPDThreads / 64]
  const int nt = mode == 0 ? 1 : trials;
  for (int e = threadIdx.x; e < nt * D; e += kPDThreads) {
    const int j = e / D, d = e - j * D;
    sc[e] = (double)PT[(int64_t)d * m + cand[j]];
  }
  __syncthreads();
  const int i = blk * kPDThreads + threadIdx.x;
  const bool ok = i < m;
  const int ic = ok ? i : m - 1;
  // 8 coordinates per round, loaded before use (one L2 round trip per 8 instead of per 1)
  constexpr int UD = 8;
  if (mode == 0) {
    double s = 0.0;
    for (int d0 = 0; d0 < D; d0 += UD) {
      float x[UD];
#pragma unroll
      for (int u = 0; u < UD; ++u) x[u] = d0 + u < D ? PT[(int64_t)(d0 + u) * m + ic] : 0.f;
#pragma unroll
      for (int u = 0; u < UD; ++u)
        if (d0 + u < D) {
          const double t = (double)x[u] - sc[d0 + u];
          s = fma(t, t, s);
        }
    }
    if (ok) d2[i] = s;
    return;
  }
  double dot[kPPMaxT];
#pragma unroll
  for (int j = 0; j < kPPMaxT; ++j) dot[j] = 0.0;
  for (int d0 = 0; d0 < D; d0 += UD) {
    float x[UD];
#pragma unroll
    for (int u = 0; u < UD; ++u) x[u] = d0 + u < D ? PT[(int64_t)(d0 + u) * m + ic] : 0.f;
#pragma unroll
    for (int u = 0; u < UD; ++u) {
      if (d0 + u < D) {
        const double xv = (double)x[u];
#pragma unroll
        for (int j = 0; j < kPPMaxT; ++j)
          if (j < nt) dot[j] = fma(xv, sc[j * D + d0 + u], dot[j]);
      }
    }
  }
  const double wi = ok ? w[i] : 0.0, di = ok ? d2[i] : 0.0, pi = pn[ic];
#pragma unroll
  for (int j = 0; j < kPPMaxT; ++j) {
    if (j < nt) {
      const double c = fmax(pi + pn[cand[j]] - 2.0 * dot[j], 0.0);
      if (ok) cd[(int64_t)j * m + i] = c;
      const double s = pp_block_sum(wi * fmin(di, c), red);
      if (threadIdx.x == 0) partial[(int64_t)blk * kPPMaxT + j] = s;
    }
  }
}

__global__ __launch_bounds__(kPDThreads) void kpp_dist_kernel(const float* __restrict__ PT,
                                                               const double* __restrict__ w,
                                                               const double* __restrict__ pn, int m, int D,
                                                               int trials, const int* __restrict__ cand, int mode,
                                                               double* __restrict__ d2, double* __restrict__ cd,
                                                               double* __restrict__ partial) {
  extern __shared__ double sc[];
  __shared__ double red[kPDThreads / 64];
  if (mode == 0 || gridDim.y == 1) {
    kpp_dist(PT, w, pn, m, D, trials, cand, mode, d2, cd, partial, blockIdx.x, sc, red);
    return;
  }
  // mode 1 on a (row block, trial) grid: one trial per block -- the same FMA sequence per
  // (row, trial) as the all-trials loop, spread over trials x more blocks (the one-block-
  // per-256-rows grid kept ~16 CUs busy for ~80 us per greedy step)
  const int j = blockIdx.y;
  const int cj = cand[j];
  for (int d = threadIdx.x; d < D; d += kPDThreads) sc[d] = (double)PT[(int64_t)d * m + cj];
  __syncthreads();
  const int blk = blockIdx.x;
  const int i = blk * kPDThreads + threadIdx.x;
  const bool ok = i < m;
  const int ic = ok ? i : m - 1;
  constexpr int UD = 8;
  double dot = 0.0;
  for (int d0 = 0; d0 < D; d0 += UD) {
    float x[UD];
#pragma unroll
    for (int u = 0; u < UD; ++u) x[u] = d0 + u < D ? PT[(int64_t)(d0 + u) * m + ic] : 0.f;
#pragma unroll
    for (int u = 0; u < UD; ++u)
      if (d0 + u < D) dot = fma((double)x[u], sc[d0 + u], dot);
  }
  const double wi = ok ? w[i] : 0.0, di = ok ? d2[i] : 0.0, pi = pn[ic];
  const double c = fmax(pi + pn[cj] - 2.0 * dot, 0.0);
  if (ok) cd[(int64_t)j * m + i] = c;
  const double sj = pp_block_sum(wi * fmin(di, c), red);
  if (threadIdx.x == 0) partial[(int64_t)blk * kPPMaxT + j] = sj;
}

// One block.  mode 0 (t = 1): prefix sum of w * d2, the step-1 draws.  mode 1 (step t):
// pick = argmin of the trials' potentials (block partials summed in order), picks[t],
// d2 = min(d2, cd[best]), then (t + 1 < k) the prefix sum and step t+1's draws.  mode 2
// (t = 0): prefix sum of w alone and the first draw.  LDS: cs [m] (m <= kPPLdsRows) else
// the global cs.
constexpr int kPPLdsRows = 16384;
template <int NTH>
__device__ void kpp_pick(const double* __restrict__ w, int m, int k, int trials, const double* __restrict__ U, int t,
                         int mode, int nblocks, const double* __restrict__ partial, const double* __restrict__ cd,
                         double* __restrict__ d2, double* __restrict__ csg, int* __restrict__ cand,
                         int* __restrict__ picks, double* lcs, double* part, int& s_best) {
  double* const cs = lcs != nullptr ? lcs : csg;
  const int tid = threadIdx.x;
  const int nt = trials + 1;
  if (mode == 1) {
    // trial j's potential = its block partials summed in block order: the partials are
    // loaded by all threads at once (part[] as staging), then summed per trial from LDS
    double pj = 0.0;
    for (int b0 = 0; b0 < nblocks; b0 += NTH / kPPMaxT) {
      const int bb = b0 + tid / kPPMaxT, jj = tid % kPPMaxT;
      __syncthreads();
      part[tid] = (bb < nblocks && jj < trials) ? partial[(int64_t)bb * kPPMaxT + jj] : 0.0;
      __syncthreads();
      if (tid < trials) {
        const int nb = min(NTH / kPPMaxT, nblocks - b0);
        for (int q = 0; q < nb; ++q) pj += part[q * kPPMaxT + tid];
      }
    }
    __syncthreads();
    if (tid < trials) part[tid] = pj;
    __syncthreads();
    if (tid == 0) {
      int best = 0;
      for (int j = 1; j < trials; ++j)
        if (part[j] < part[best]) best = j;
      s_best = best;
      picks[t] = cand[best];
    }
    __syncthreads();
    if (t + 1 >= k) return;                  // last step: d2 is not needed any more
  }
  const int best = mode == 1 ? s_best : 0;
  // p_i = w_i * d2_i (d2 updated with the pick first): coalesced pass into cs, then each
  // thread scans its contiguous chunk of cs
  for (int i = tid; i < m; i += NTH) {
    double pi = w[i];
    if (mode != 2) {
      double di = d2[i];
      if (mode == 1) {
        di = fmin(di, cd[(int64_t)best * m + i]);
        d2[i] = di;
      }
      pi *= di;
    }
    cs[i] = pi;
  }
  __syncthreads();
  const int per = (m + NTH - 1) / NTH;
  const int a = tid * per, e = min(m, a + per);
  double s = 0.0;
  for (int i = a; i < e; ++i) {
    s += cs[i];
    cs[i] = s;                               // local running sum, offset below
  }
  part[tid] = s;
  __syncthreads();
  for (int off = 1; off < NTH; off <<= 1) {   // Hillis-Steele, fixed order
    const double add = tid >= off ? part[tid - off] : 0.0;
    __syncthreads();
    part[tid] += add;
    __syncthreads();
  }
  const double base = tid ? part[tid - 1] : 0.0;
  for (int i = a; i < e; ++i) cs[i] += base;
  __syncthreads();
  const double tot = part[NTH - 1];
  if (mode == 2) {
    if (tid == 0) {
      const int first = pp_draw(cs, m, tot, U[0]);
      cand[0] = first;
      picks[0] = first;
    }
  } else {
    const int tn = mode == 0 ? 1 : t + 1;    // the step the draws are for
    if (tid < trials) cand[tid] = pp_draw(cs, m, tot, U[(int64_t)tn * nt + tid]);
  }
}

__global__ __launch_bounds__(kPPThreads) void kpp_pick_kernel(const double* __restrict__ w, int m, int k, int trials,
                                                               const double* __restrict__ U, int t, int mode,
                                                               int nblocks, const double* __restrict__ partial,
                                                               const double* __restrict__ cd, double* __restrict__ d2,
                                                               double* __restrict__ csg, int* __restrict__ cand,
                                                               int* __restrict__ picks) {
  extern __shared__ double lcs[];
  __shared__ double part[kPPThreads];
  __shared__ int s_best;
  kpp_pick<kPPThreads>(w, m, k, trials, U, t, mode, nblocks, partial, cd, d2, csg, cand, picks,
                       m <= kPPLdsRows ? lcs : nullptr, part, s_best);
}

}  // namespace

// PT = fp32(P)^T [D][m], w [m] weights, pn [m] = |fp32(p)|^2 (fp64 sums), U [k][trials + 1]
// uniforms; ws: d2 [m], cs [m], cd [trials][m] fp64, partial [ceil(m / 256)][16] fp64,
// cand [16] int32 scratch; picks [k] int32 out.  trials <= 16.  (One cooperative launch with
// grid barriers between the phases measured no faster than the 2k launches: 0.104 vs 0.096 s
// at k = 1024, m = 4097 -- each grid barrier writes back and invalidates the L2.)
O3S_API int o3s_kmeanspp(const float* PT, const double* w, const double* pn, int m, int D, int k, int trials,
                         const double* U, double* d2, double* cs, double* cd, double* partial, int* cand,
                         int* picks, hipStream_t st) {
  if (m <= 0 || k <= 0 || D <= 0 || trials < 1 || trials > kPPMaxT) return -1;
  const size_t dl = sizeof(double) * (size_t)trials * D;
  if (dl > 64 * 1024) return -2;
  const int nb = (m + kPDThreads - 1) / kPDThreads;
  const size_t pl = m <= kPPLdsRows ? sizeof(double) * (size_t)m : 0;
  hipLaunchKernelGGL(kpp_pick_kernel, dim3(1), dim3(kPPThreads), pl, st, w, m, k, trials, U, 0, 2, nb, partial, cd, d2,
                     cs, cand, picks);
  if (k > 1) {
    hipLaunchKernelGGL(kpp_dist_kernel, dim3(nb), dim3(kPDThreads), sizeof(double) * D, st, PT, w, pn, m, D, trials,
                       cand, 0, d2, cd, partial);
    hipLaunchKernelGGL(kpp_pick_kernel, dim3(1), dim3(kPPThreads), pl, st, w, m, k, trials, U, 1, 0, nb, partial, cd,
                       d2, cs, cand, picks);
  }
  for (int t = 1; t < k; ++t) {
    hipLaunchKernelGGL(kpp_dist_kernel, dim3(nb, trials), dim3(kPDThreads), sizeof(double) * D, st, PT, w, pn, m, D,
                       trials, cand, 1, d2, cd, partial);
    hipLaunchKernelGGL(kpp_pick_kernel, dim3(1), dim3(kPPThreads), pl, st, w, m, k, trials, U, t, 1, nb, partial, cd,
                       d2, cs, cand, picks);
  }
  O3S_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------
// Shifted moments of the rows in ONE pass (the Lloyd cost identity's centring): per block
// of consecutive rows, fp64 sums of (x - s) per column and of ||x - s||^2, with s a shift
// near the data (models/kmeans.py: a row of rank 0) so the later centring about the exact
// mean cancels nothing.  Thread t owns the float4 column group t % G (G = D / 4) of rows
// t / G, t / G + 256 / G, ...; the block's partial row [D + 1] is written in a fixed order.
namespace {
constexpr int kMomThreads = 256;
__global__ __launch_bounds__(kMomThreads) void kmeans_moments_kernel(const float* __restrict__ X, int64_t n,
                                                                     int64_t ldx, int D, const float* __restrict__ sh,
                                                                     int64_t rows_per_block, double* __restrict__ part) {
  __shared__ double red[kMomThreads][5];
  const int G = D / 4;
  const int per = kMomThreads / G;                       // rows per sweep of the block
  const int t = threadIdx.x;
  const int cg = t % G, r0 = t / G;
  const bool active = r0 < per;
  const int64_t b0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t b1 = b0 + rows_per_block < n ? b0 + rows_per_block : n;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0, q = 0.0;
  const float4 c = active ? *reinterpret_cast<const float4*>(sh + 4 * cg) : make_float4(0.f, 0.f, 0.f, 0.f);
  if (active) {
    for (int64_t r = b0 + r0; r < b1; r += per) {
      const float4 v = *reinterpret_cast<const float4*>(X + r * ldx + 4 * cg);
      const double d0 = (double)v.x - c.x, d1 = (double)v.y - c.y, d2 = (double)v.z - c.z, d3 = (double)v.w - c.w;
      s0 += d0; s1 += d1; s2 += d2; s3 += d3;
      q = fma(d0, d0, fma(d1, d1, fma(d2, d2, fma(d3, d3, q))));
    }
  }
  red[t][0] = s0; red[t][1] = s1; red[t][2] = s2; red[t][3] = s3; red[t][4] = q;
  __syncthreads();
  double* out = part + (int64_t)blockIdx.x * (D + 1);
  if (t < G) {                                           // column group t: its threads t, t + G, ...
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    for (int k = t; k < per * G; k += G) { a0 += red[k][0]; a1 += red[k][1]; a2 += red[k][2]; a3 += red[k][3]; }
    out[4 * t] = a0; out[4 * t + 1] = a1; out[4 * t + 2] = a2; out[4 * t + 3] = a3;
  }
  if (t == 0) {
    double a = 0.0;
    for (int k = 0; k < per * G; ++k) a += red[k][4];
    out[D] = a;
  }
}
}  // namespace

// part: fp64 [grid][D + 1] (column sums of x - sh, then the sum of ||x - sh||^2), rows split
// into grid contiguous ranges; D % 4 == 0, D <= 1024, 16-B aligned rows and shift.
O3S_API int o3s_kmeans_moments(const float* X, int64_t n, int64_t ldx, int D, const float* sh, int grid,
                               double* part, hipStream_t st) {
  if (D % 4 != 0 || D <= 0 || D > 4 * kMomThreads || ldx % 4 != 0 || grid <= 0) return -1;
  if (n <= 0) return 0;
  const int64_t rpb = (n + grid - 1) / grid;
  hipLaunchKernelGGL(kmeans_moments_kernel, dim3(grid), dim3(kMomThreads), 0, st, X, n, ldx, D, sh, rpb, part);
  O3S_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------
// Training cost of an assignment: sum over rows of ||x - c_a(x)||^2, directly from the rows
// (one streaming pass; the centre rows are L2-resident gathers).  Thread t owns float4
// column group t % G of rows t / G, t / G + 256 / G, ... of its block's contiguous range;
// a row's four squared differences are summed in fp32 (fma), everything above in fp64,
// the block partial in a fixed order.
namespace {
__global__ __launch_bounds__(kMomThreads) void kmeans_cost_kernel(const float* __restrict__ X, int64_t n, int64_t ldx,
                                                                  int D, const int32_t* __restrict__ a,
                                                                  const float* __restrict__ C, int ldc,
                                                                  int64_t rows_per_block, double* __restrict__ part) {
  __shared__ double red[kMomThreads];
  const int G = D / 4;
  const int per = kMomThreads / G;
  const int t = threadIdx.x;
  const int cg = t % G, r0 = t / G;
  const int64_t b0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t b1 = b0 + rows_per_block < n ? b0 + rows_per_block : n;
  double acc = 0.0;
  if (r0 < per) {
    for (int64_t r = b0 + r0; r < b1; r += per) {
      const float4 x = *reinterpret_cast<const float4*>(X + r * ldx + 4 * cg);
      const float4 c = *reinterpret_cast<const float4*>(C + (int64_t)a[r] * ldc + 4 * cg);
      const float d0 = x.x - c.x, d1 = x.y - c.y, d2 = x.z - c.z, d3 = x.w - c.w;
      acc += (double)fmaf(d0, d0, fmaf(d1, d1, fmaf(d2, d2, d3 * d3)));
    }
  }
  red[t] = acc;
  __syncthreads();
  if (t == 0) {
    double s = 0.0;
    for (int k = 0; k < kMomThreads; ++k) s += red[k];
    part[blockIdx.x] = s;
  }
}
}  // namespace

// part: fp64 [grid] partial costs (rows split into grid contiguous ranges); C: fp32 centre
// rows [.][ldc] indexed by a; D % 4 == 0, 16-B aligned rows.
O3S_API int o3s_kmeans_cost(const float* X, int64_t n, int64_t ldx, int D, const int32_t* a, const float* C, int ldc,
                            int grid, double* part, hipStream_t st) {
  if (D % 4 != 0 || D <= 0 || D > 4 * kMomThreads || ldx % 4 != 0 || ldc % 4 != 0 || grid <= 0) return -1;
  if (n <= 0) return 0;
  const int64_t rpb = (n + grid - 1) / grid;
  hipLaunchKernelGGL(kmeans_cost_kernel, dim3(grid), dim3(kMomThreads), 0, st, X, n, ldx, D, a, C, ldc, rpb, part);
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_PRELOAD(kmeans)
