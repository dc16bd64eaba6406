// Decision-tree histogram build (gfx950): DecisionTree / RandomForest / GBT.
//
// Replaces Spark's per-level DTStatsAggregator pass (binned features -> per (node,
// feature, bin) label statistics, reduced with reduceByKey; reached through the
// Classification/Regression widgets -> fit, orangecontrib/spark/base/spark_ml_estimator.py:22).
//
// Data layout: binned features uint8 [n][F] (row-major, one 64-B line per row at F=64),
// rows grouped by tree node through a permutation `order` (the engine re-partitions it
// after every level), so a work item = one contiguous run of rows of ONE node.
//
// LDS-privatised histograms with NO atomics and NO bank conflicts: lane (rs, f) of a
// wave owns feature f of row-slot rs, so each lane updates only its own columns of an LDS
// image laid out [rs][bin][stat][f] (f fastest: 64 lanes -> 64 banks), and every wave
// has its own image (plain read-modify-writes: LDS float atomics -- ds_add_f32 --
// measured 7x slower here, profiles/gbt_hist_lds_atomic_experiment.json).  At the end
// the block sums its waves' images in a fixed order and writes ONE fp32 slab row per
// work item; the engine sums slab rows per node in a fixed order (deterministic).
//
// Stat modes: REG (S = 3: w, w*y, w*y^2 -- variance impurity, GBT residual trees) and
// CLS (S = #classes: weighted class counts -- gini/entropy).
#include "common.h"

#include <stdlib.h>


using namespace o3s;

namespace {

// A wave's private image is 64*B*SL floats whatever FP is (SL = LDS stats: classes for
// CLS, 2 for REG -- the regression image holds w and w*y; the split gain needs only
// those, and the node's sum of w*y^2 is accumulated in registers by the lanes of
// feature 0).  At B = 32 that is 16 KB per wave, so 2-wave blocks fit 5 per CU.
// Each lane gathers U rows (order -> row -> bins/y) per batch and the next batch's
// gathers are issued before the current batch's LDS updates, so the dependent HBM
// latency overlaps the read-modify-writes.
constexpr int kHistWaves = 2;
constexpr int kHistThreads = kHistWaves * kWave;

// bins + row * F computed on the SALU (row and F are wave-uniform): left to the compiler,
// the multiply was fused with the per-lane feature offset into one v_mad_i64_i32 per row
// (a multi-pass VALU op) in the histogram's per-row loop.  The result is an SGPR base for
// the saddr form of the byte gather.
typedef const uint8_t __attribute__((address_space(1)))* gbytes;   // global (not flat) loads
__device__ __forceinline__ gbytes scalar_row(const uint8_t* base, int32_t row, int32_t F) {
  const uint64_t b = (uint64_t)base;
  uint32_t lo, hi;
  asm("s_mul_i32 %0, %2, %3\n\ts_mul_hi_i32 %1, %2, %3\n\ts_add_u32 %0, %0, %4\n\ts_addc_u32 %1, %1, %5"
      : "=&s"(lo), "=&s"(hi)
      : "s"(row), "s"(F), "s"((uint32_t)b), "s"((uint32_t)(b >> 32))
      : "scc");
  // (readfirstlane of the SGPR results: marks them uniform for the divergence analysis,
  // which treats inline-asm outputs as divergent -- else the base goes through VGPRs)
  lo = __builtin_amdgcn_readfirstlane(lo);
  hi = __builtin_amdgcn_readfirstlane(hi);
  return (gbytes)(((uint64_t)hi << 32) | lo);
}

// FP: features per row-slot (power of 2, <= 64); RS = 64 / FP row-slots per wave.
// HW: per-row weights present (a compile-time switch: a runtime null test per row
// became a branch around every weight load and split the counted vmcnt waits).
// YP: y / w are stored in POSITION order (y[p] belongs to row order[p]; the partition
// moves them with the rows), so they stream contiguously instead of costing one random
// cache-line gather each per row -- only the 64-B bins row is gathered.
// DMA (one row-slot per wave, F % 16 == 0): the chunk's 32 rows are fetched by two LDS-DMA
// instructions (global_load_lds_dwordx4: 4 lanes x 16 B per row, 16 rows each) into a
// per-wave double-buffered stage, and each lane reads its feature's byte from LDS.  The
// per-row 64-lane byte gathers it replaces kept the texture addressers ~55% busy
// (TA_BUSY_avr, profiles/kernel_experiments_r6.json); taking them off buys 3-5% on every
// layout -- the rest is the dependent LDS read-add-write chain per row.
template <int FP, bool CLS, bool HW, bool YP, int U, bool DMA = false>
__global__ __launch_bounds__(kHistThreads, 4) void tree_hist_kernel(
    const uint8_t* __restrict__ bins, int F, int fg0, int B, int S, const int32_t* __restrict__ order,
    const float* __restrict__ y, const float* __restrict__ w, const int64_t* __restrict__ item_lo,
    const int64_t* __restrict__ item_hi, float* __restrict__ slab, int64_t slab_stride) {
  constexpr int RS = kWave / FP;
  const int SL = CLS ? S : 2;                                     // stats kept in LDS
  // CLS: [wave][rs][B][S][FP] (+pad); REG: [wave][rs][B][FP][2] -- a cell's (w, w*y) pair
  // is one 8-B LDS word, updated by one ds_read_b64 / v_pk_add_f32 / ds_write_b64
  // (no static LDS: at F = 64, B = 32 a block's two 16-KB images are exactly a fifth of
  // the CU's 160 KB, so five blocks -- ten waves -- are resident; the REG w*y^2 partials
  // leave through the slab instead of an LDS scratch, see the block reduction)
  extern __shared__ __attribute__((aligned(16))) float hist[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform (SGPR)
  const int rs = lane / FP, f = lane % FP;
  const int region = B * SL * FP + (RS > 1 ? 16 : 0);             // +16: rs-regions on distinct banks
  const int per_wave = RS * region;
  float* my = hist + wid * per_wave + rs * region;
  for (int i = threadIdx.x; i < kHistWaves * per_wave; i += kHistThreads) hist[i] = 0.f;
  __syncthreads();
  const int fcol = fg0 + f;
  const bool fok = fcol < F;
  const int64_t lo = item_lo[blockIdx.x], hi = item_hi[blockIdx.x];
  float wy2 = 0.f;                                                // REG: sum of w*y^2 (lanes f == 0)
  // Positions are 32-bit offsets inside the item (items hold <= 2^31 rows); loads are
  // unconditional (clamped to the item; rows past it get weight 0), so the compiler
  // emits counted vmcnt waits instead of draining every load at a branch merge.
  const int32_t* __restrict__ ord = order + lo;
  const int32_t nl = (int32_t)(hi - lo);
  const float* __restrict__ yl = YP ? y + lo : y;
  const float* __restrict__ wl = (YP && HW) ? w + lo : w;
  if constexpr (RS == 1) {
    // One row per wave-instruction (lane = feature).  The per-row metadata comes in
    // 32-row chunks -- lane l loads order[] / y / w of position l of the chunk, ONE
    // vector load each per 32 rows -- and is broadcast per row with v_readlane, so a row
    // costs one 64-B gather, one LDS read + write and a few VALU (the first version
    // issued three uniform vector loads per row and ran at half this rate:
    // tools/bench_hist.py 62.5M rows 6.2 -> 2.8 ms).  Chunks of a wave: wid,
    // wid + kHistWaves, ...; two chunk buffers swap roles: while chunk c is accumulated,
    // chunk c+1's 32 gathers and chunk c+2's order[] entries are in flight.
    constexpr int32_t CH = 32;                     // < 63 loads in flight: vmcnt stays countable
    constexpr int32_t cstep = kHistWaves * CH;
    const int32_t j0w = wid * CH;
    const int fc = fok ? fcol : 0;
    auto ld_ord = [&](int32_t jb, int32_t& ov) {
      const int32_t j = jb + j0w + (lane & (CH - 1));
      ov = ord[j < nl ? j : nl - 1];
    };
    // DMA stage: per wave two buffers of CH rows x 64 B, after the histogram images
    uint8_t* const stg = reinterpret_cast<uint8_t*>(hist + kHistWaves * per_wave) + wid * (2 * CH * 64);
    const int piece = 16 * (lane & 3);
    const bool pok = fg0 + piece < F;                // 16-B pieces past the row: a valid dummy address
    auto ld_chunk = [&](int32_t jb, int32_t ov, int (&bo)[CH], float& yv, float& wv) {
      if constexpr (DMA) {
        const int buf = ((jb / cstep) & 1) * (CH * 64);
#pragma unroll
        for (int k = 0; k < CH / 16; ++k) {
          const int32_t row = __shfl(ov, 16 * k + (lane >> 2), 64);
          const uint8_t* src = pok ? bins + (int64_t)row * F + fg0 + piece : bins;
          __builtin_amdgcn_global_load_lds(src, stg + buf + k * 1024, 16, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);         // the DMAs before this chunk's y / w loads
      } else {
#pragma unroll
        for (int q = 0; q < CH; ++q) {
          const int32_t row = __builtin_amdgcn_readlane(ov, q);
          bo[q] = scalar_row(bins, row, F)[(uint32_t)fc];
        }
      }
      const int32_t j = jb + j0w + (lane & (CH - 1));
      const int32_t jc = j < nl ? j : nl - 1;
      yv = YP ? yl[jc] : y[ov];
      wv = HW ? (YP ? wl[jc] : w[ov]) : 1.f;   // rows past the item: zeroed in acc_chunk
    };
    // (Grouping rows so several LDS read-modify-writes share one wait -- duplicates
    // merged first -- measured slower: the extra VALU outweighs the LDS round trips.)
    auto acc_chunk = [&](int32_t jb, const int (&bo_r)[CH], float yv, float wv) {
      int bo[CH];
      if constexpr (DMA) {
        // this chunk's DMAs have landed once at most the VMEM ops issued after them are
        // outstanding: its y (+ w), the next chunk's order[] load, its two DMAs and its y
        // (+ w) -- 4 (+ 2) at the least whatever order the compiler gave y / w and the DMAs
        if constexpr (HW) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        const int buf = ((jb / cstep) & 1) * (CH * 64);
#pragma unroll
        for (int q = 0; q < CH; ++q) bo[q] = stg[buf + q * 64 + f];
      } else {
#pragma unroll
        for (int q = 0; q < CH; ++q) bo[q] = bo_r[q];
      }
      if constexpr (CLS) {
#pragma unroll
        for (int q = 0; q < CH; ++q) {
          const float yq = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(yv), q));
          const float wr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wv), q));
          const float wq = jb + j0w + q < nl ? wr : 0.f;                 // wave-uniform
          my[bo[q] * SL * FP + f + (int)yq * FP] += wq;
        }
      } else {
        // per-position work once per chunk, vectorised (lane q = position q): validity,
        // w and w*y, and the node's w*y^2 partial (lanes < CH); a row then costs two
        // broadcasts, one LDS address and one packed add
        const int32_t jl = jb + j0w + (lane & (CH - 1));
        const float wl0 = jl < nl ? wv : 0.f;
        const float wyl = wl0 * yv;
        if (lane < CH) wy2 = fmaf(wyl, yv, wy2);
        if (!HW && jb + j0w + CH <= nl) {
          // unit weights, a full chunk: w = 1 for every row -- one broadcast per row
#pragma unroll
          for (int q = 0; q < CH; ++q) {
            const float wyq = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wyl), q));
            float2_* cell = reinterpret_cast<float2_*>(my + (bo[q] * FP + f) * 2);
            *cell += float2_{1.f, wyq};
          }
        } else {
#pragma unroll
          for (int q = 0; q < CH; ++q) {
            const float wq = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wl0), q));
            const float wyq = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wyl), q));
            float2_* cell = reinterpret_cast<float2_*>(my + (bo[q] * FP + f) * 2);
            *cell += float2_{wq, wyq};
          }
        }
      }
    };
    if (j0w < nl) {
      // per step: order[] of chunk c+2, then the gathers of chunk c+1, then the LDS updates
      // of chunk c.  The order[] load goes FIRST: vmcnt retires in issue order, so the
      // readlanes of chunk c+1's rows (next step) wait only for loads issued before chunk
      // c+1's gathers, and two chunks of gathers stay in flight.  (Issued after the
      // gathers, the next step's readlanes drained them with vmcnt(0): one chunk in
      // flight, its latency exposed once per chunk.)  sched_barrier keeps the phases in
      // this order (the scheduler would pull loads next to their consumers).  The loop runs
      // whole chunk PAIRS with no exit between the halves: an exit there let the compiler
      // sink the first half's gathers past it (they are dead on that path), next to their
      // consumers.  A pair's second chunk past the item costs clamped, cached loads and a
      // zero-weight accumulate.
      int bA[CH], bB[CH];
      int32_t o1, o2;
      float yA, yB, wA, wB;
      const int32_t npair = ((nl - j0w + cstep - 1) / cstep + 1) / 2;
      ld_ord(0, o1);
      ld_ord(cstep, o2);
      __builtin_amdgcn_sched_barrier(0);   // o2 before chunk 0's gathers (see above)
      ld_chunk(0, o1, bA, yA, wA);
      for (int32_t pi = 0; pi < npair; ++pi) {
        const int32_t jb = pi * 2 * cstep;
        __builtin_amdgcn_sched_barrier(0);
        ld_ord(jb + 2 * cstep, o1);
        __builtin_amdgcn_sched_barrier(0);
        ld_chunk(jb + cstep, o2, bB, yB, wB);
        __builtin_amdgcn_sched_barrier(0);
        acc_chunk(jb, bA, yA, wA);
        __builtin_amdgcn_sched_barrier(0);
        ld_ord(jb + 3 * cstep, o2);
        __builtin_amdgcn_sched_barrier(0);
        ld_chunk(jb + 2 * cstep, o1, bA, yA, wA);
        __builtin_amdgcn_sched_barrier(0);
        acc_chunk(jb + cstep, bB, yB, wB);
      }
    }
  } else {
    // Several row-slots per wave (FP < 64): lanes gather their own rows.  Batch k of a
    // wave = U*RS consecutive positions k*step + wid*U*RS + u*RS + rs; the two batch
    // buffers swap roles (a register rotation would force the compiler to drain every
    // in-flight load): batch k+1's gathers and batch k+2's order[] reads fly while batch
    // k is accumulated.
    constexpr int32_t step = kHistWaves * U * RS;
    const int32_t jw = wid * (U * RS) + rs;
    auto ld_rows = [&](int32_t jb, int32_t (&r)[U]) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int32_t j = jb + jw + u * RS;
        r[u] = ord[j < nl ? j : nl - 1];
      }
    };
    auto ld_data = [&](int32_t jb, const int32_t (&r)[U], uint8_t (&bo)[U], float (&yo)[U], float (&wo)[U]) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t row = r[u];
        bo[u] = bins[row * F + (fok ? fcol : 0)];
        if (YP) {
          const int32_t j = jb + jw + u * RS;
          const int32_t jc = j < nl ? j : nl - 1;
          yo[u] = yl[jc];
          wo[u] = HW ? wl[jc] : 1.f;
        } else {
          yo[u] = y[row];
          wo[u] = HW ? w[row] : 1.f;
        }
      }
    };
    auto accumulate = [&](int32_t jb, const uint8_t (&bo)[U], const float (&yo)[U], const float (&wo)[U]) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = fok && (jb + jw + u * RS < nl);
        const float wv = ok ? wo[u] : 0.f;
        if (CLS) {
          my[bo[u] * SL * FP + f + (int)yo[u] * FP] += wv;
        } else {
          const float wy = wv * yo[u];
          float2_* cell = reinterpret_cast<float2_*>(my + (bo[u] * FP + f) * 2);
          *cell += float2_{wv, wy};
          wy2 = fmaf(wy, yo[u], wy2);
        }
      }
    };
    int32_t rA[U], rB[U];
    uint8_t bA[U], bB[U];   // bytes: an int copy made the compiler widen them at the loop head (a drain)
    float yA[U], yB[U], wA[U], wB[U];
    if (jw < nl) {
      // order[] of batch k+2 is issued BEFORE batch k+1's gathers, and the loop runs whole
      // batch pairs (see the RS == 1 path)
      const int32_t npair = ((nl + step - 1) / step + 1) / 2;
      ld_rows(0, rA);
      ld_rows(step, rB);
      __builtin_amdgcn_sched_barrier(0);
      ld_data(0, rA, bA, yA, wA);
      for (int32_t pi = 0; pi < npair; ++pi) {
        const int32_t j0 = pi * 2 * step;
        __builtin_amdgcn_sched_barrier(0);
        ld_rows(j0 + 2 * step, rA);
        __builtin_amdgcn_sched_barrier(0);
        ld_data(j0 + step, rB, bB, yB, wB);
        __builtin_amdgcn_sched_barrier(0);
        accumulate(j0, bA, yA, wA);
        __builtin_amdgcn_sched_barrier(0);
        ld_rows(j0 + 3 * step, rB);
        __builtin_amdgcn_sched_barrier(0);
        ld_data(j0 + 2 * step, rA, bA, yA, wA);
        __builtin_amdgcn_sched_barrier(0);
        accumulate(j0 + step, bB, yB, wB);
      }
    }
  }
  float* out = slab + (int64_t)blockIdx.x * slab_stride;
  // REG stat 2 (w*y^2) is a node total, stored in (feature 0, bin 0), zero elsewhere.
  // Wave q parks its partial (summed over its row-slots in a fixed order) in the slab cell
  // (feature 0, bin q) -- global memory, visible to the block after the barrier -- and the
  // thread that owns (feature 0, bin 0) adds them in wave order and clears the others.
  if constexpr (!CLS) {
    if constexpr (RS == 1) wy2 = group_sum<32>(wy2);               // chunk partials of lanes 0..CH-1
    else wy2 = group_sum<64>(f == 0 ? wy2 : 0.f);                  // lanes f == 0 of every row-slot
    if (fg0 == 0 && lane == 0) out[(int64_t)wid * S + 2] = wy2;
  }
  __syncthreads();
  // fixed-order block reduction -> slab[item][f][b][s] (features of this group only).
  // Feature fastest across lanes: the 64 lanes of a wave read one (bin, stat) row of the
  // image -- 64 consecutive floats, one per bank.  (Mapping (bin, stat) fastest put every
  // lane of a wave on the same bank: 64 floats apart -- the kernel's measured LDS bank
  // conflicts, profiles/pmc_kmeans_gbt.json.)  The slab row is then written with a stride
  // of B*S floats per lane; the block writes the whole row, so L2 merges the lines.
  const int cells = FP * B * S;
  for (int i = threadIdx.x; i < cells; i += kHistThreads) {
    const int ff = i % FP, rem = i / FP;
    const int bb = rem / S, ss = rem % S;
    if (fg0 + ff >= F) continue;
    float acc = 0.f;
    if (CLS || ss < 2) {
      for (int q = 0; q < kHistWaves; ++q)
        for (int r = 0; r < RS; ++r)
          acc += hist[q * per_wave + r * region + (CLS ? (bb * SL + ss) * FP + ff : (bb * FP + ff) * 2 + ss)];
    } else if (fg0 + ff == 0 && bb == 0) {
#pragma unroll
      for (int q = 0; q < kHistWaves; ++q) acc += out[(int64_t)q * S + 2];   // the waves' partials
#pragma unroll
      for (int q = 1; q < kHistWaves; ++q) out[(int64_t)q * S + 2] = 0.f;
    } else if (fg0 + ff == 0 && bb < kHistWaves) {
      continue;                                                    // cleared by the (bin 0) owner
    }
    out[((int64_t)(fg0 + ff) * B + bb) * S + ss] = acc;
  }
}

// ---------------------------------------------------------------------------------
// Level partition: every splitting segment of `order` is stably split into the rows
// going left (bins[row][feat] <= bin) followed by the rows going right.  Work items are
// the histogram items (contiguous runs inside one segment); pass 1 counts each item's
// left rows, the engine turns the counts into per-item destinations (tiny scans), pass 2
// writes each row to its destination.  Ranks inside an item come from wave ballots +
// a block scan, so the split is stable and deterministic.
constexpr int kPartThreads = 256;
constexpr int kPartWaves = kPartThreads / kWave;
constexpr int kPartU = 4;                          // rows per thread per round (count, scatter)

// bins element (row, feat) at row * rs + feat * cs: the partition reads a feature-major
// copy (rs = 1, cs = n), so within a segment (rows in ascending order after every stable
// split) neighbouring lanes hit neighbouring bytes of one feature column instead of one
// byte per 64-B row.
__device__ __forceinline__ bool goes_left(const uint8_t* __restrict__ bins, int64_t rs, int64_t cs, int32_t row,
                                          int feat, int bin) {
  return (int)bins[(int64_t)row * rs + (int64_t)feat * cs] <= bin;
}

__global__ __launch_bounds__(kPartThreads) void tree_part_count_kernel(
    const uint8_t* __restrict__ bins, int64_t rs, int64_t cs, const int32_t* __restrict__ order, const int64_t* __restrict__ it_lo,
    const int64_t* __restrict__ it_hi, const int32_t* __restrict__ it_feat, const int32_t* __restrict__ it_bin,
    int64_t* __restrict__ it_left, uint8_t* __restrict__ flags) {
  __shared__ int wsum[kPartWaves];
  const int64_t lo = it_lo[blockIdx.x], hi = it_hi[blockIdx.x];
  const int feat = it_feat[blockIdx.x], bin = it_bin[blockIdx.x];
  int cnt = 0;
  // kPartU rows per thread per round: their order[] loads, then their gathers, issue
  // together (one dependent load pair per row left the memory pipe mostly idle)
  for (int64_t p0 = lo + threadIdx.x; p0 < hi; p0 += kPartThreads * kPartU) {
    int32_t row[kPartU];
#pragma unroll
    for (int k = 0; k < kPartU; ++k) {
      const int64_t p = p0 + (int64_t)k * kPartThreads;
      row[k] = p < hi ? order[p] : 0;
    }
    bool l[kPartU];
#pragma unroll
    for (int k = 0; k < kPartU; ++k) l[k] = goes_left(bins, rs, cs, row[k], feat, bin);   // the random gathers
#pragma unroll
    for (int k = 0; k < kPartU; ++k) {
      const int64_t p = p0 + (int64_t)k * kPartThreads;
      if (p < hi) {
        flags[p] = l[k];                                        // pass 2 reads this sequentially
        cnt += l[k];
      }
    }
  }
  cnt = wave_sum_i(cnt);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) wsum[wid] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int i = 0; i < kPartWaves; ++i) t += wsum[i];
    it_left[blockIdx.x] = t;
  }
}

// Last split level of a tree (children at maxDepth are leaves): instead of partitioning
// the rows and histogramming the children, one pass over every splitting segment
// routes each row by its split (bins[row][feat] <= bin) and
//   * (boosting, acc != null) adds the child's leaf value to the row's prediction,
//   * accumulates the child's sum of w*y^2 (REG impurity; the children's w and w*y come
//     from the parent's histogram) as one fp32 partial per (item, side).
// Rows are read in position order (y / w are position-ordered payloads).
__global__ __launch_bounds__(kPartThreads) void tree_final_level_kernel(
    const uint8_t* __restrict__ bins, int64_t rs, int64_t cs, const int32_t* __restrict__ order,
    const int64_t* __restrict__ it_lo, const int64_t* __restrict__ it_hi, const int32_t* __restrict__ it_feat,
    const int32_t* __restrict__ it_bin, const double* __restrict__ it_vl, const double* __restrict__ it_vr,
    const float* __restrict__ y, const float* __restrict__ w, double* __restrict__ acc, float* __restrict__ part) {
  __shared__ float red[2][kPartWaves];
  const int64_t lo = it_lo[blockIdx.x], hi = it_hi[blockIdx.x];
  const int feat = it_feat[blockIdx.x], bin = it_bin[blockIdx.x];
  const double vl = acc ? it_vl[blockIdx.x] : 0.0, vr = acc ? it_vr[blockIdx.x] : 0.0;
  float sl = 0.f, sr = 0.f;
  for (int64_t p = lo + threadIdx.x; p < hi; p += kPartThreads) {
    const int32_t row = order[p];
    const bool l = goes_left(bins, rs, cs, row, feat, bin);
    if (acc) acc[row] += l ? vl : vr;
    if (part) {
      const float yy = y[p], ww = w ? w[p] : 1.f;
      const float v = ww * yy * yy;
      sl += l ? v : 0.f;
      sr += l ? 0.f : v;
    }
  }
  if (!part) return;
  sl = wave_sum(sl);
  sr = wave_sum(sr);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { red[0][wid] = sl; red[1][wid] = sr; }
  __syncthreads();
  if (threadIdx.x < 2) {
    float a = 0.f;
    for (int q = 0; q < kPartWaves; ++q) a += red[threadIdx.x][q];
    part[(int64_t)blockIdx.x * 2 + threadIdx.x] = a;
  }
}

__global__ __launch_bounds__(kPartThreads) void tree_part_scatter_kernel(
    const int32_t* __restrict__ order, int32_t* __restrict__ out,
    const int64_t* __restrict__ it_lo, const int64_t* __restrict__ it_hi, const int32_t* __restrict__ it_feat,
    const int32_t* __restrict__ it_bin, const int64_t* __restrict__ dst_left, const int64_t* __restrict__ dst_right,
    const uint8_t* __restrict__ flags, const float* __restrict__ py, float* __restrict__ py_out,
    const float* __restrict__ pw, float* __restrict__ pw_out) {
  // kPartU sub-rounds of kPartThreads positions per round: every load of the round first,
  // then one barrier for the wave counts of all sub-rounds (instead of one round trip and
  // two barriers per kPartThreads positions); destinations as before, sub-round by sub-round
  __shared__ int wl[kPartU][kPartWaves];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t lo = it_lo[blockIdx.x], hi = it_hi[blockIdx.x];
  int64_t nl = dst_left[blockIdx.x], nr = dst_right[blockIdx.x];
  const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  for (int64_t base = lo; base < hi; base += (int64_t)kPartThreads * kPartU) {
    int32_t row[kPartU];
    bool left[kPartU];
    float yv[kPartU], wv[kPartU];
#pragma unroll
    for (int k = 0; k < kPartU; ++k) {
      const int64_t p = base + (int64_t)k * kPartThreads + threadIdx.x;
      const bool ok = p < hi;
      const int64_t pc = ok ? p : lo;
      row[k] = order[pc];
      left[k] = ok && flags[pc];
      yv[k] = py ? py[pc] : 0.f;
      wv[k] = pw ? pw[pc] : 0.f;
    }
    uint64_t m[kPartU];
#pragma unroll
    for (int k = 0; k < kPartU; ++k) {
      m[k] = __ballot(left[k]);
      if (lane == 0) wl[k][wid] = __popcll(m[k]);
    }
    __syncthreads();
    int64_t accl = 0, accr = 0;                                  // lefts / rights of earlier sub-rounds
#pragma unroll
    for (int k = 0; k < kPartU; ++k) {
      int before = 0, total = 0;
#pragma unroll
      for (int i = 0; i < kPartWaves; ++i) {
        before += i < wid ? wl[k][i] : 0;
        total += wl[k][i];
      }
      const int rank_l = before + __popcll(m[k] & below);       // lefts before me in this sub-round
      const int64_t round_base = base + (int64_t)k * kPartThreads;
      const int64_t rem = hi - round_base;
      const int valid = rem <= 0 ? 0 : (rem < kPartThreads ? (int)rem : kPartThreads);
      if ((int)threadIdx.x < valid) {
        // rights before me = idx - lefts before; position-ordered payloads move with the row
        const int64_t d = left[k] ? nl + accl + rank_l : nr + accr + ((int)threadIdx.x - rank_l);
        out[d] = row[k];
        if (py) py_out[d] = yv[k];
        if (pw) pw_out[d] = wv[k];
      }
      accl += total;
      accr += valid - total;
    }
    nl += accl;
    nr += accr;
    __syncthreads();                                              // wl reused next round
  }
}

// Destinations of the level partition's scatter: per segment (one block each), the
// exclusive prefix of its items' left counts gives each item's first left slot and the
// prefix of the right counts (after the segment's nleft lefts) its first right slot.
// Replaces a dozen small device ops per level (cumsums, gathers, index_add).
__device__ __forceinline__ int64_t block_incl_scan_i64(int64_t v, int64_t* wtot, int64_t& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t t = __shfl_up(v, off, 64);
    if (lane >= off) v += t;
  }
  if (lane == 63) wtot[wid] = v;
  __syncthreads();
  int64_t before = 0;
  total = 0;
#pragma unroll
  for (int q = 0; q < kPartWaves; ++q) {
    before += q < wid ? wtot[q] : 0;
    total += wtot[q];
  }
  __syncthreads();                                               // wtot reused by the next call
  return v + before;
}

__global__ __launch_bounds__(kPartThreads) void tree_part_dest_kernel(
    const int64_t* __restrict__ it_lo, const int64_t* __restrict__ it_hi, const int64_t* __restrict__ it_left,
    const int64_t* __restrict__ seg_first, const int64_t* __restrict__ seg_lo, int64_t* __restrict__ dst_left,
    int64_t* __restrict__ dst_right, int64_t* __restrict__ nleft) {
  __shared__ int64_t wtot[kPartWaves];
  const int s = blockIdx.x;
  const int64_t a = seg_first[s], b = seg_first[s + 1], base = seg_lo[s];
  int64_t carry = 0, tot;
  for (int64_t c = a; c < b; c += kPartThreads) {
    const int64_t i = c + threadIdx.x;
    const int64_t v = i < b ? it_left[i] : 0;
    const int64_t inc = block_incl_scan_i64(v, wtot, tot);
    if (i < b) dst_left[i] = base + carry + inc - v;
    carry += tot;
  }
  const int64_t L = carry;
  if (threadIdx.x == 0) nleft[s] = L;
  carry = 0;
  for (int64_t c = a; c < b; c += kPartThreads) {
    const int64_t i = c + threadIdx.x;
    const int64_t v = i < b ? (it_hi[i] - it_lo[i]) - it_left[i] : 0;
    const int64_t inc = block_incl_scan_i64(v, wtot, tot);
    if (i < b) dst_right[i] = base + L + carry + inc - v;
    carry += tot;
  }
}

// ---------------------------------------------------------------------------------
// Feature-major copy of the binned matrix ([n][F] -> [F][n], uint8) for the partition.
// One block = 256 rows x <= 64 features staged through LDS: 4-byte coalesced row reads
// (F % 4 == 0), 4-byte coalesced column writes; rows are padded by 4 bytes so the byte
// scatter into the [feature][row] tile spreads over banks.
constexpr int kTrRows = 256;
__global__ __launch_bounds__(256) void u8_transpose_kernel(const uint8_t* __restrict__ in, int64_t n, int F,
                                                           uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[64][kTrRows + 4];
  const int64_t r0 = (int64_t)blockIdx.x * kTrRows;
  const int f0 = blockIdx.y * 64;
  const int fw = F - f0 < 64 ? F - f0 : 64;                 // % 4 == 0
  const int rows = n - r0 < kTrRows ? (int)(n - r0) : kTrRows;
  const int wq = fw / 4;                                    // 4-byte words per tile row
  for (int w = threadIdx.x; w < kTrRows * wq; w += 256) {
    const int r = w / wq, q = w % wq;
    if (r < rows) {
      const uint32_t v = *reinterpret_cast<const uint32_t*>(in + (r0 + r) * F + f0 + 4 * q);
      tile[4 * q + 0][r] = (uint8_t)v;
      tile[4 * q + 1][r] = (uint8_t)(v >> 8);
      tile[4 * q + 2][r] = (uint8_t)(v >> 16);
      tile[4 * q + 3][r] = (uint8_t)(v >> 24);
    }
  }
  __syncthreads();
  const bool full = rows == kTrRows && (n & 3) == 0;
  for (int w = threadIdx.x; w < fw * (kTrRows / 4); w += 256) {
    const int f = w / (kTrRows / 4), q = w % (kTrRows / 4);
    uint8_t* dst = out + (int64_t)(f0 + f) * n + r0 + 4 * q;
    if (full) {
      *reinterpret_cast<uint32_t*>(dst) = *reinterpret_cast<const uint32_t*>(&tile[f][4 * q]);
    } else {
      for (int j = 0; j < 4; ++j)
        if (4 * q + j < rows) dst[j] = tile[f][4 * q + j];
    }
  }
}

// ---------------------------------------------------------------------------------
// Quantile binning: bin = #thresholds < x (torch.bucketize(right=False) semantics) for
// every element of X [n][F] fp32.  All features' thresholds sit in LDS ([F][Tp+1] with
// +inf padding to a power of two Tp; the +1 row pad puts consecutive features of one
// wave on different banks); each element is a branchless log2(Tp)-step search.  One
// streaming pass: X read once, bins written once (row-major, coalesced bytes).
// BF16: X holds bf16 bit patterns (the engine's default GPU vector storage), widened
// exactly in registers -- no fp32 copy of the matrix.  out_t (optional): the same bins
// feature-major [F][n] in the same pass (the partition's per-row feature reads), instead
// of a separate transpose of the finished row-major matrix: a block's 64-row chunk is
// staged in LDS as [F][64] and written out as one 64-byte run per feature (written
// straight from registers, lane = feature, every byte landed in a different cache line:
// GBT fit 0.139 -> 0.255 s/tree, profiles/config_gbt_full_500Mx64_n1_r5.json).
constexpr int kBinRows = 64;
constexpr int kBinTS = kBinRows + 4;             // LDS row stride of the [F][64] bin tile
template <bool BF16>
__global__ __launch_bounds__(256) void bin_features_kernel(const void* __restrict__ Xv, int64_t n, int64_t ldx,
                                                           int F, const float* __restrict__ th, int Tp,
                                                           uint8_t* __restrict__ out, uint8_t* __restrict__ out_t,
                                                           int64_t ldt) {
  extern __shared__ float sth[];
  const int TS = Tp + 1;
  uint8_t* const tile = reinterpret_cast<uint8_t*>(sth + F * TS);
  for (int i = threadIdx.x; i < F * Tp; i += 256) sth[(i / Tp) * TS + i % Tp] = th[i];
  __syncthreads();
  const int64_t nchunks = (n + kBinRows - 1) / kBinRows;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t r0 = c * kBinRows;
    const int rows = n - r0 < kBinRows ? (int)(n - r0) : kBinRows;
    for (int li = threadIdx.x; li < rows * F; li += 256) {
      const int lr = li / F, f = li - lr * F;
      float x;
      if constexpr (BF16)
        x = bf16_to_f32(reinterpret_cast<const uint16_t*>(Xv)[(r0 + lr) * ldx + f]);
      else
        x = reinterpret_cast<const float*>(Xv)[(r0 + lr) * ldx + f];
      const float* a = sth + f * TS;
      int b = 0;
      for (int st = Tp >> 1; st > 0; st >>= 1) b += (a[b + st - 1] < x) ? st : 0;
      out[(r0 + lr) * F + f] = (uint8_t)b;
      if (out_t != nullptr) tile[f * kBinTS + lr] = (uint8_t)b;
    }
    if (out_t != nullptr) {
      __syncthreads();
      for (int e = threadIdx.x; e < F * kBinRows; e += 256) {
        const int f = e / kBinRows, lr = e - f * kBinRows;
        if (lr < rows) out_t[(int64_t)f * ldt + r0 + lr] = tile[f * kBinTS + lr];
      }
      __syncthreads();                             // the tile is rewritten by the next chunk
    }
  }
}

// Vector fast path (F % 8 == 0, 16-B aligned rows): a lane bins 8 consecutive features of
// one row -- one 16-B (bf16) or two 16-B (fp32) loads, eight independent branchless
// searches, one 8-B store -- instead of one 2-/4-B load and one byte store per element
// (the scalar kernel above ran the 500M x 64 binning at 75 ms, mostly memory-instruction
// issue).  ROWS-row chunks (256 when the LDS tile fits): a thread issues the loads of up to
// four of its items before the first search, so each block keeps several row loads in
// flight per barrier; the feature-major copy leaves the [F][ROWS] LDS tile as 4-row dwords
// (ldt % 4 == 0; one byte per lane otherwise).
template <bool BF16, int ROWS, int LVC = 0>
__global__ __launch_bounds__(256) void bin_features_vec_kernel(const void* __restrict__ Xv, int64_t n, int64_t ldx,
                                                               int F, const float* __restrict__ th, int Tp,
                                                               uint8_t* __restrict__ out, uint8_t* __restrict__ out_t,
                                                               int64_t ldt) {
  constexpr int TSR = ROWS + 4;                          // tile row stride (bytes, % 4 == 0)
  extern __shared__ float sth[];
  const int TS = Tp + 1;
  uint8_t* const tile = reinterpret_cast<uint8_t*>(sth + F * TS);
  const int G = F >> 3;                                  // 8-feature groups per row
  // LVC > 0 (Tp == 2^LVC): thresholds in search-tree order, per level, the G features of one
  // k-slice (features 8 g + k) interleaved: level L of feature 8 g + k at sth[k G (Tp - 1) +
  // G (2^L - 1) + g 2^L + j], j in [0, 2^L) holding threshold (2 j + 1) 2^(LVC - 1 - L) - 1.
  // A lane walks r = g 2^L + j, r' = 2 r + (t < x), from a per-(k, L) uniform base, and the
  // eight features' searches run interleaved level by level (eight independent LDS chains, no
  // loop) -- the runtime-depth search below spent ~6 VALU and a full LDS round trip per level
  // and feature.  A wave's level-L lookups fall in one block of G 2^L floats (distinct banks
  // up to level 3 at G = 8; the [F][Tp + 1] table put 75% of the LDS cycles in bank conflicts).
  if constexpr (LVC > 0) {
    for (int i = threadIdx.x; i < F * (Tp - 1); i += 256) {
      const int k = i / (G * (Tp - 1)), rem = i % (G * (Tp - 1));
      int L = 0;
      while (G * ((2 << L) - 1) <= rem) ++L;               // rem in level L's block
      const int off = rem - G * ((1 << L) - 1);
      const int g = off >> L, j = off & ((1 << L) - 1);
      sth[i] = th[(8 * g + k) * Tp + (2 * j + 1) * (1 << (LVC - 1 - L)) - 1];
    }
  } else {
    for (int i = threadIdx.x; i < F * Tp; i += 256) sth[(i / Tp) * TS + i % Tp] = th[i];
  }
  __syncthreads();
  const bool dw = (ldt & 3) == 0 && ((uintptr_t)out_t & 3) == 0;
  const int64_t nchunks = (n + ROWS - 1) / ROWS;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t r0 = c * ROWS;
    const int rows = n - r0 < ROWS ? (int)(n - r0) : ROWS;
    const int items = rows * G;
    for (int li0 = threadIdx.x; li0 < items; li0 += 4 * 256) {
      float x[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int li = li0 + u * 256;
        const int lr = li / G, g = li - lr * G;
        const int64_t row = r0 + (li < items ? lr : 0);
        const int gg = li < items ? g : 0;
        if constexpr (BF16) {
          const uint4 v = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(Xv) + row * ldx + 8 * gg);
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            x[u][2 * k] = __uint_as_float(w[k] << 16);
            x[u][2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
          }
        } else {
          const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(Xv) + row * ldx + 8 * gg);
          const float4 a = p[0], b = p[1];
          x[u][0] = a.x; x[u][1] = a.y; x[u][2] = a.z; x[u][3] = a.w;
          x[u][4] = b.x; x[u][5] = b.y; x[u][6] = b.z; x[u][7] = b.w;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int li = li0 + u * 256;
        if (li >= items) break;
        const int lr = li / G, g = li - lr * G;
        const int64_t row = r0 + lr;
        int bin[8];
        if constexpr (LVC > 0) {
          int g0 = g;
          asm volatile("" : "+v"(g0));                     // keep g = li - lr G out of the addresses
#pragma unroll
          for (int k = 0; k < 8; ++k) bin[k] = g0;
#pragma unroll
          for (int L = 0; L < LVC; ++L) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const float t = sth[G * (k * ((1 << LVC) - 1) + (1 << L) - 1) + bin[k]];
              bin[k] = 2 * bin[k] + (t < x[u][k] ? 1 : 0);
            }
          }
#pragma unroll
          for (int k = 0; k < 8; ++k) bin[k] &= (1 << LVC) - 1;
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float* a = sth + (8 * g + k) * TS;
            int bk = 0;
            for (int st = Tp >> 1; st > 0; st >>= 1) bk += (a[bk + st - 1] < x[u][k]) ? st : 0;
            bin[k] = bk;
          }
        }
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int bk = bin[k];
          if (k < 4) lo |= (uint32_t)bk << (8 * k);
          else hi |= (uint32_t)bk << (8 * (k - 4));
          if (out_t != nullptr) tile[(8 * g + k) * TSR + lr] = (uint8_t)bk;
        }
        *reinterpret_cast<uint2*>(out + row * F + 8 * g) = make_uint2(lo, hi);
      }
    }
    if (out_t != nullptr) {
      __syncthreads();
      if (dw) {
        constexpr int Q = ROWS / 4;
        for (int e = threadIdx.x; e < F * Q; e += 256) {
          const int f = e / Q, q = e - f * Q;
          const int lr = 4 * q;
          if (lr + 3 < rows) {
            *reinterpret_cast<uint32_t*>(out_t + (int64_t)f * ldt + r0 + lr) =
                *reinterpret_cast<const uint32_t*>(tile + f * TSR + lr);
          } else {
            for (int j = lr; j < rows; ++j) out_t[(int64_t)f * ldt + r0 + j] = tile[f * TSR + j];
          }
        }
      } else {
        for (int e = threadIdx.x; e < F * ROWS; e += 256) {
          const int f = e / ROWS, lr = e - f * ROWS;
          if (lr < rows) out_t[(int64_t)f * ldt + r0 + lr] = tile[f * TSR + lr];
        }
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------------
// Leaf apply (boosting): when a segment of `order` becomes a leaf, every row in it gets
// the leaf's (weighted) value added to its running prediction: acc[order[p]] += val.
// Items are contiguous runs inside one leaf segment, so each row is touched once per
// tree -- this replaces building a per-row leaf-id column and gathering from it.
__global__ __launch_bounds__(256) void tree_leaf_apply_kernel(const int32_t* __restrict__ order,
                                                              const int64_t* __restrict__ it_lo,
                                                              const int64_t* __restrict__ it_hi,
                                                              const double* __restrict__ it_val,
                                                              double* __restrict__ acc) {
  const int64_t lo = it_lo[blockIdx.x], hi = it_hi[blockIdx.x];
  const double v = it_val[blockIdx.x];
  for (int64_t p = lo + threadIdx.x; p < hi; p += 256) {
    const int32_t row = order[p];
    acc[row] += v;
  }
}

// ---------------------------------------------------------------------------------
// Deterministic fp64 range sums of slab rows: out[j][c] = sum_{r in [lo_j, lo_j+cnt_j)} in[r][c],
// rows added in ascending order (the engine calls it twice: fp32 item slabs -> fp64
// partials over fixed runs of <= 64 items, then partials -> one row per segment), so a
// node's histogram is bitwise reproducible and never rounds bin weights past 2^24.
// One thread per column (lanes read consecutive columns: coalesced), 4 rows in flight.
template <typename T>
__global__ __launch_bounds__(256) void slab_range_sum_kernel(const T* __restrict__ in, int64_t C,
                                                             const int64_t* __restrict__ lo,
                                                             const int64_t* __restrict__ cnt,
                                                             double* __restrict__ out) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const int64_t r0 = lo[blockIdx.y], n = cnt[blockIdx.y];
  const T* p = in + r0 * C + c;
  double acc = 0.0;
  int64_t r = 0;
  for (; r + 4 <= n; r += 4) {
    const double a = (double)p[(r + 0) * C], b = (double)p[(r + 1) * C];
    const double d = (double)p[(r + 2) * C], e = (double)p[(r + 3) * C];
    acc += a; acc += b; acc += d; acc += e;                // ascending order, no reassociation
  }
  for (; r < n; ++r) acc += (double)p[r * C];
  out[(int64_t)blockIdx.y * C + c] = acc;
}

// ---------------------------------------------------------------------------------
// Best split per node, fused (replaces ~40 small device ops per tree level).  One block
// per node: thread f scans feature f's bins once in ascending order, keeping the
// cumulative left stats (right = node total - left), and evaluates every threshold's
// gain with Spark's impurity definitions (variance from (w, w*y) sums; gini / entropy
// from class counts); the block then keeps the largest gain (ties -> lowest candidate
// index f*(B-1)+b, deterministic).  The node total comes from feature 0 (REG: stat 2,
// the sum of w*y^2, is stored in feature 0's bin 0 only).
// out (fp64, k nodes): [best idx | best gain | impurity | weight | wL(best) | wR(best) |
// values k x V] -- the exact bundle the engine copies to the host once per level.
constexpr int kSplitThreads = 256;
constexpr int kSplitMaxS = 64;

// SM: compile-time bound on S (register-resident stats for S <= 8)
template <int SM>
__device__ __forceinline__ double split_imp(const double* st, int S, int kind, double& wsum) {
  // kind 1 = gini, 2 = entropy (classification stats: class weights)
  double w = 0.0;
#pragma unroll
  for (int s = 0; s < SM; ++s)
    if (s < S) w += st[s];
  wsum = w;
  if (!(w > 0.0)) return 0.0;
  const double inv = 1.0 / (w > 1e-300 ? w : 1e-300);
  double acc = 0.0;
#pragma unroll
  for (int s = 0; s < SM; ++s) {
    if (s >= S) continue;
    const double p = st[s] * inv;
    if (kind == 1) acc += p * p;
    else if (p > 0.0) acc -= p * log2(p);
  }
  return kind == 1 ? 1.0 - acc : acc;
}

template <bool CLS, int SM>
__global__ __launch_bounds__(kSplitThreads) void tree_split_kernel(
    const double* __restrict__ H, int k, int F, int B, int S, int kind, const int32_t* __restrict__ nb,
    const uint8_t* __restrict__ fmask, double min_inst, double min_w, double min_wfrac,
    const double* __restrict__ mw_node, double* __restrict__ out) {
  __shared__ double tot[kSplitMaxS];
  __shared__ double rg[kSplitThreads], rwl[kSplitThreads], rwr[kSplitThreads];
  __shared__ int ri[kSplitThreads];
  const int node = blockIdx.x;
  const double* Hn = H + (int64_t)node * F * B * S;
  for (int s = threadIdx.x; s < S; s += kSplitThreads) {
    double a = 0.0;
    for (int b = 0; b < B; ++b) a += Hn[b * S + s];
    tot[s] = a;
  }
  __syncthreads();
  double imp_p, w_p;
  if (CLS) {
    imp_p = split_imp<kSplitMaxS>(tot, S, kind, w_p);
  } else {
    w_p = tot[0];
    const double wc = w_p > 1e-300 ? w_p : 1e-300;
    const double mean = tot[1] / wc;
    const double v = tot[2] / wc - mean * mean;
    imp_p = w_p > 0.0 ? (v > 0.0 ? v : 0.0) : 0.0;
  }
  const double W = w_p > 1e-300 ? w_p : 1e-300;
  // minimum child weight: per node (forests: each tree's own root fraction), else a
  // fraction of this node's weight (the root level), else one value
  const double mw = mw_node ? mw_node[node] : (min_wfrac > 0.0 ? min_wfrac * w_p : min_w);
  double bg = -INFINITY, bwl = 0.0, bwr = 0.0;
  int bi = 0x7fffffff;
  double left[SM], right[SM];
  for (int f = threadIdx.x; f < F; f += kSplitThreads) {
    const double* Hf = Hn + (int64_t)f * B * S;
    const bool fon = fmask == nullptr || fmask[(int64_t)node * F + f];
    const int nbf = nb[f];
#pragma unroll
    for (int s = 0; s < SM; ++s) left[s] = 0.0;
    for (int b = 0; b < B - 1; ++b) {
#pragma unroll
      for (int s = 0; s < SM; ++s)
        if (s < S) left[s] += Hf[b * S + s];
      double g, wL, wR;
      if (CLS) {
#pragma unroll
        for (int s = 0; s < SM; ++s) right[s] = s < S ? tot[s] - left[s] : 0.0;
        const double iL = split_imp<SM>(left, S, kind, wL);
        const double iR = split_imp<SM>(right, S, kind, wR);
        g = imp_p - (wL / W) * iL - (wR / W) * iR;
      } else {
        wL = left[0];
        wR = tot[0] - left[0];
        const double sL = left[1], sR = tot[1] - left[1], sP = tot[1];
        g = (sL * sL / (wL > 1e-300 ? wL : 1e-300) + sR * sR / (wR > 1e-300 ? wR : 1e-300) - sP * sP / W) / W;
      }
      bool ok = wL >= min_inst && wR >= min_inst && b < nbf && fon;
      if (mw > 0.0) ok = ok && wL >= mw && wR >= mw;
      const int idx = f * (B - 1) + b;
      if (ok && (g > bg || (g == bg && idx < bi))) { bg = g; bi = idx; bwl = wL; bwr = wR; }
    }
  }
  rg[threadIdx.x] = bg; ri[threadIdx.x] = bi; rwl[threadIdx.x] = bwl; rwr[threadIdx.x] = bwr;
  __syncthreads();
  for (int h = kSplitThreads / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) {
      const int o = threadIdx.x + h;
      if (rg[o] > rg[threadIdx.x] || (rg[o] == rg[threadIdx.x] && ri[o] < ri[threadIdx.x])) {
        rg[threadIdx.x] = rg[o]; ri[threadIdx.x] = ri[o]; rwl[threadIdx.x] = rwl[o]; rwr[threadIdx.x] = rwr[o];
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const int best = ri[0] == 0x7fffffff ? 0 : ri[0];
    out[node] = (double)best;
    out[k + node] = rg[0];
    out[2 * k + node] = imp_p;
    out[3 * k + node] = w_p;
    out[4 * k + node] = rwl[0];
    out[5 * k + node] = rwr[0];
  }
  const int V = CLS ? S : 1;
  for (int v = threadIdx.x; v < V; v += kSplitThreads)
    out[6 * k + (int64_t)node * V + v] = CLS ? tot[v] / W : tot[1] / W;
}

// ---------------------------------------------------------------------------------
// Boosting step epilogue, fused (Spark GradientBoostedTrees: after tree m the training
// (and validation) loss of F_m, and the pseudo-residuals of tree m+1): ONE pass over
// (y, F, w) instead of ~15 elementwise / reduction launches.  loss 0 = logistic
// (y in {-1, +1}: loss 2*log(1 + e^{-2yF}), computed stably; residual 4y / (1 + e^{2yF})),
// 1 = squared ((y-F)^2; 2(y-F)), 2 = absolute (|y-F|; sign(y-F)).  Per-block partial
// sums [sum loss*w, sum w, sum loss*wv, sum wv] (fp64; fixed grid and fixed-order block
// reduction, so reproducible); target (fp32, may be null) gets the residuals.
constexpr int kGbtThreads = 256;
__global__ __launch_bounds__(kGbtThreads) void gbt_grad_loss_kernel(
    const double* __restrict__ y, const double* __restrict__ F, const double* __restrict__ w,
    const double* __restrict__ wv, int64_t n, int loss, float* __restrict__ target, double* __restrict__ partial) {
  __shared__ double red[4][kGbtThreads / kWave];
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  const int64_t stride = (int64_t)gridDim.x * kGbtThreads;
  for (int64_t i = (int64_t)blockIdx.x * kGbtThreads + threadIdx.x; i < n; i += stride) {
    const double yi = y[i], fi = F[i];
    double l, g;
    if (loss == 0) {
      // z = -2yF; loss 2 log(1 + e^z) and residual 4y sigmoid(z) from ONE exp: e = e^{-|z|}
      const double z = -2.0 * yi * fi;
      const double e = exp(-fabs(z));
      l = 2.0 * (fmax(z, 0.0) + log1p(e));
      g = 4.0 * yi * (z >= 0.0 ? 1.0 / (1.0 + e) : e / (1.0 + e));
    } else if (loss == 1) {
      const double d = yi - fi;
      l = d * d;
      g = 2.0 * d;
    } else {
      const double d = yi - fi;
      l = fabs(d);
      g = (double)((d > 0.0) - (d < 0.0));
    }
    const double wi = w ? w[i] : 1.0;
    s0 += l * wi;
    s1 += wi;
    if (wv) {
      const double vi = wv[i];
      s2 += l * vi;
      s3 += vi;
    }
    if (target) target[i] = (float)g;
  }
  s0 = wave_sum_d(s0); s1 = wave_sum_d(s1); s2 = wave_sum_d(s2); s3 = wave_sum_d(s3);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { red[0][wid] = s0; red[1][wid] = s1; red[2][wid] = s2; red[3][wid] = s3; }
  __syncthreads();
  if (threadIdx.x < 4) {
    double a = 0.0;
    for (int q = 0; q < kGbtThreads / kWave; ++q) a += red[threadIdx.x][q];
    partial[(int64_t)blockIdx.x * 4 + threadIdx.x] = a;
  }
}

// Histogram subtraction for a whole level: node 2p + sr[p] is the scanned smaller child
// Hs[p], node 2p + 1 - sr[p] its sibling parent[p] - Hs[p], cleaned of the rounding
// residue fractional weights leave in bins the sibling does not populate (CLS: counts
// clamped at 0; REG: (w, w*y) zeroed where w <= 0, the node's w*y^2 -- stat 2 of
// feature 0 bin 0 -- clamped at 0).  One thread per (node pair, feature x bin) cell.
__global__ __launch_bounds__(256) void tree_sibling_kernel(const double* __restrict__ Hs,
                                                           const double* __restrict__ parent,
                                                           const uint8_t* __restrict__ sr, int64_t P, int FB, int S,
                                                           int cls, double* __restrict__ H) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= P * FB) return;
  const int64_t p = g / FB;
  const int fb = (int)(g % FB);
  const int64_t C = (int64_t)FB * S;
  const double* hs = Hs + p * C + (int64_t)fb * S;
  const double* pa = parent + p * C + (int64_t)fb * S;
  const int s_small = sr[p] ? 1 : 0;
  double* hsm = H + (2 * p + s_small) * C + (int64_t)fb * S;
  double* hsb = H + (2 * p + 1 - s_small) * C + (int64_t)fb * S;
  if (cls) {
    for (int s = 0; s < S; ++s) {
      const double a = hs[s];
      const double d = pa[s] - a;
      hsm[s] = a;
      hsb[s] = d > 0.0 ? d : 0.0;
    }
    return;
  }
  const double w = pa[0] - hs[0], wy = pa[1] - hs[1], y2 = pa[2] - hs[2];
  const bool empty = !(w > 0.0);
  hsm[0] = hs[0]; hsm[1] = hs[1]; hsm[2] = hs[2];
  hsb[0] = empty ? 0.0 : w;
  hsb[1] = empty ? 0.0 : wy;
  hsb[2] = fb == 0 ? (y2 > 0.0 ? y2 : 0.0) : y2;
}

// Per-tree row weights of a forest in one pass: out[t][i] = w[i] * draw(seed_t, rows[i])
// with draw = Poisson(lam) by CDF inversion over `table` (cdf_0 .. cdf_{kmax-1}, fp64,
// built by the caller exactly as ops/sampling.py does) or Bernoulli(rate) -- the same
// draws as sampling.poisson_counts / bernoulli_mask (stream 1 / stream 0).
__global__ __launch_bounds__(256) void forest_weights_kernel(const int64_t* __restrict__ rows, int64_t n,
                                                             const uint32_t* __restrict__ seeds,
                                                             const double* __restrict__ table, int kmax,
                                                             float rate, const float* __restrict__ w,
                                                             float* __restrict__ out) {
  const int t = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t r = rows[i];
  float v;
  if (table) {
    const double u = hash_uniform(seeds[t], 1u, r);
    int k = 0;
    for (int j = 0; j < kmax; ++j) k += table[j] < u;
    v = (float)k;
  } else {
    v = hash_uniform(seeds[t], 0u, r) < (double)rate ? 1.f : 0.f;
  }
  out[(int64_t)t * n + i] = w ? w[i] * v : v;
}

// ---------------------------------------------------------------------------------
// GBT tree epilogue, fused (replaces the last level's routing pass, every level's
// leaf_apply scatter and the boosting step's gbt_grad_loss pass): ONE sequential pass
// over the rows in ROW order.  Each row walks the finished tree on its row-major bins
// (a wave stages its 64 consecutive rows -- 64 x F bytes, coalesced -- in LDS and reads
// the split features from there), then
//   * Fm[i] += value(leaf)            (leaf values pre-scaled by the tree weight),
//   * the loss of the updated Fm       (partials [sum l*wd, sum wd, sum l*wv, sum wv]),
//   * target[i] = next tree's residual (fp32, may be null),
//   * (REG) sum of w*y^2 of the leaves at depth D -- the children the last split level
//     created, whose w and w*y came from their parent's histogram -- with y the residual
//     this tree was fit to, recomputed from (yy, Fm before the update) exactly as the
//     previous pass wrote it (first tree: y = yy).
// The old path gathered every row twice at random (feature-major byte + an fp64
// read-modify-write of acc[order[p]]); this one streams bins / yy / Fm once.
// Per-leaf sums: every wave owns an LDS array of the 2^D leaf sums and adds its rows with
// ONE LDS atomic add per chunk (ds_add_f32, no return); lanes that hit the same leaf in
// one instruction are serialised by the LDS in lane order, instructions in program order,
// so a wave's sums are a fixed sequence of fp32 adds (deterministic).  Each wave writes
// its array as one fp32 slab row; the rows are summed in fp64 in a fixed order.  (A
// register-owned variant -- the owner lane adds each broadcast row -- cost ~2300
// instructions per 64 rows: 5.2 ms per 100M rows, profiles/gbt_r6_kernels.json.)
constexpr int kLeafThreads = 256;
constexpr int kLeafWaves = kLeafThreads / kWave;

__device__ __forceinline__ void gbt_point(int loss, double yi, double fi, double& l, double& g) {
  if (loss == 0) {
    const double z = -2.0 * yi * fi;
    const double e = exp(-fabs(z));
    l = 2.0 * (fmax(z, 0.0) + log1p(e));
    g = 4.0 * yi * (z >= 0.0 ? 1.0 / (1.0 + e) : e / (1.0 + e));
  } else if (loss == 1) {
    const double d = yi - fi;
    l = d * d;
    g = 2.0 * d;
  } else {
    const double d = yi - fi;
    l = fabs(d);
    g = (double)((d > 0.0) - (d < 0.0));
  }
}

// Y2: per-leaf w*y^2 sums of the leaves at depth D (L = 2^D).
template <bool STAGE, bool Y2>
__global__ __launch_bounds__(kLeafThreads) void gbt_leaf_pass_kernel(
    const uint8_t* __restrict__ bins, int64_t n, int F, int Fs, const int32_t* __restrict__ node_fb, int nodes,
    const double* __restrict__ node_val, int D, const double* __restrict__ yy, double* __restrict__ Fm,
    const float* __restrict__ wt, const double* __restrict__ wd, const double* __restrict__ wv, int loss,
    int first, float* __restrict__ target, double* __restrict__ partial, float* __restrict__ y2slab, int L) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  int32_t* tree = reinterpret_cast<int32_t*>(lds);                         // [nodes]
  float* y2w = reinterpret_cast<float*>(lds + 4 * ((nodes + 3) & ~3));     // [waves][L]
  uint8_t* stage = reinterpret_cast<uint8_t*>(y2w + (Y2 ? kLeafWaves * L : 0));   // [waves][64][Fs]
  __shared__ double red[4][kLeafWaves];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < nodes; i += kLeafThreads) tree[i] = node_fb[i];
  if constexpr (Y2)
    for (int i = threadIdx.x; i < kLeafWaves * L; i += kLeafThreads) y2w[i] = 0.f;
  __syncthreads();
  uint8_t* my_stage = stage + wid * 64 * Fs;
  float* my_y2 = y2w + wid * L;
  const int leaf0 = 1 << D;                                                // first node id at depth D
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  const int64_t nchunks = (n + 63) / 64;
  const int64_t wstride = (int64_t)gridDim.x * kLeafWaves;
  for (int64_t c = (int64_t)blockIdx.x * kLeafWaves + wid; c < nchunks; c += wstride) {
    const int64_t r0 = c * 64;
    const int rows = n - r0 < 64 ? (int)(n - r0) : 64;
    const int64_t i = r0 + (lane < rows ? lane : rows - 1);
    const bool ok = lane < rows;
    const double yi = yy[i], fo = Fm[i];
    const float ww = wt ? wt[i] : 1.f;
    if constexpr (STAGE) {
      // the wave's rows are one contiguous run of rows * F bytes: 16-byte coalesced reads
      // (F % 16 == 0) into rows of Fs bytes (Fs / 4 odd: the lanes' rows on distinct banks)
      const int qpr = F >> 4, qtot = rows * qpr;
      const uint4* src = reinterpret_cast<const uint4*>(bins + r0 * F);
      for (int e = lane; e < qtot; e += 64) {
        const int rr = e / qpr, q = e - rr * qpr;
        const uint4 v = src[e];
        uint32_t* d = reinterpret_cast<uint32_t*>(my_stage + rr * Fs + 16 * q);
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    int node = 1;
    for (int d = 0; d < D; ++d) {
      const int32_t fb = node < nodes ? tree[node] : -1;
      if (fb < 0) break;                                                   // a leaf (lane-divergent)
      const int f = fb & 0xffff, sb = (fb >> 16) & 0x7fff;
      const int b = STAGE ? (int)my_stage[lane * Fs + f] : (int)bins[i * F + f];
      node = 2 * node + (b > sb ? 1 : 0);
    }
    const double fn = fo + node_val[node];
    double l, g;
    gbt_point(loss, yi, fn, l, g);
    if (ok) {
      Fm[i] = fn;
      if (target) target[i] = (float)g;
      const double wi = wd ? wd[i] : 1.0;
      s0 += l * wi;
      s1 += wi;
      if (wv) {
        const double vi = wv[i];
        s2 += l * vi;
        s3 += vi;
      }
    }
    if constexpr (Y2) {
      // the residual this tree was fit to (fp32, as the previous pass wrote it)
      float yo;
      if (first) {
        yo = (float)yi;
      } else {
        double lo_, go_;
        gbt_point(loss, yi, fo, lo_, go_);
        yo = (float)go_;
      }
      if (ok && node >= leaf0) atomicAdd(my_y2 + (node - leaf0), ww * yo * yo);
    }
    if constexpr (STAGE) __builtin_amdgcn_wave_barrier();                  // the stage is rewritten next chunk
  }
  s0 = wave_sum_d(s0); s1 = wave_sum_d(s1); s2 = wave_sum_d(s2); s3 = wave_sum_d(s3);
  if (lane == 0) { red[0][wid] = s0; red[1][wid] = s1; red[2][wid] = s2; red[3][wid] = s3; }
  __syncthreads();
  if (threadIdx.x < 4) {
    double a = 0.0;
    for (int q = 0; q < kLeafWaves; ++q) a += red[threadIdx.x][q];
    partial[(int64_t)blockIdx.x * 4 + threadIdx.x] = a;
  }
  if constexpr (Y2) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float* row = y2slab + ((int64_t)blockIdx.x * kLeafWaves + wid) * L;
    for (int k = lane; k < L; k += 64) row[k] = my_y2[k];
  }
}

}  // namespace

// Fused GBT tree epilogue (gbt_leaf_pass_kernel).  bins: [n][F] uint8; node_fb: int32
// [nodes] heap-ordered (root 1): feature | split bin << 16 for internal nodes, -1 for
// leaves / absent; node_val: fp64 [nodes] leaf value * tree weight; D: the tree's max
// depth (<= 10; leaves at depth D own y2slab columns node - 2^D, L = 2^D).  yy / Fm /
// wd / wv fp64 [n] (wd, wv nullable), wt fp32 [n] (nullable), target fp32 [n] (nullable).
// partial: fp64 [grid][4]; y2slab: fp32 [grid * 4][L] (one row per wave) or null.
O3S_API int o3s_gbt_leaf_pass(const uint8_t* bins, int64_t n, int F, const int32_t* node_fb, int nodes,
                              const double* node_val, int D, const double* yy, double* Fm, const float* wt,
                              const double* wd, const double* wv, int loss, int first, float* target,
                              double* partial, float* y2slab, int grid, hipStream_t st) {
  if (n <= 0) return 0;
  if (F <= 0 || F > 0xffff || nodes <= 1 || D < 0 || D > 10 || loss < 0 || loss > 2 || grid <= 0) return -1;
  const int L = 1 << D;
  const bool y2 = y2slab != nullptr;
  const bool stage = (F % 16) == 0 && F <= 256 && ((uintptr_t)bins & 15) == 0;
  const int Fs = stage ? ((F / 4) % 2 == 0 ? F + 4 : F) : 0;
  const size_t lds = 4 * (size_t)((nodes + 3) & ~3) + (y2 ? 4 * (size_t)kLeafWaves * L : 0) +
                     (size_t)kLeafWaves * 64 * Fs;
  if (lds > 64 * 1024) return -2;
#define O3S_LP(S, Y)                                                                                       \
  hipLaunchKernelGGL((gbt_leaf_pass_kernel<S, Y>), dim3(grid), dim3(kLeafThreads), lds, st, bins, n, F, Fs,   \
                     node_fb, nodes, node_val, D, yy, Fm, wt, wd, wv, loss, first, target, partial, y2slab, L)
  if (stage && y2) O3S_LP(true, true);
  else if (stage) O3S_LP(true, false);
  else if (y2) O3S_LP(false, true);
  else O3S_LP(false, false);
#undef O3S_LP
  O3S_CHECK_LAUNCH();
  return 0;
}

// acc[order[p]] += it_val[i] for p in [it_lo[i], it_hi[i]) (items of leaf segments).
O3S_API int o3s_tree_leaf_apply(const int32_t* order, const int64_t* it_lo, const int64_t* it_hi,
                                const double* it_val, int n_items, double* acc, hipStream_t st) {
  if (n_items <= 0) return 0;
  hipLaunchKernelGGL(tree_leaf_apply_kernel, dim3(n_items), dim3(256), 0, st, order, it_lo, it_hi, it_val, acc);
  O3S_CHECK_LAUNCH();
  return 0;
}

// out[j] = ordered fp64 sum of rows [lo[j], lo[j] + cnt[j]) of in ([*][C], fp32 if
// in_f64 == 0 else fp64); n_out <= 65535 ranges per launch.
O3S_API int o3s_slab_range_sum(const void* in, int in_f64, int64_t C, const int64_t* lo, const int64_t* cnt,
                               int n_out, double* out, hipStream_t st) {
  if (n_out <= 0 || C <= 0) return 0;
  if (n_out > 65535) return -1;
  const dim3 grid((unsigned)((C + 255) / 256), (unsigned)n_out);
  if (in_f64)
    hipLaunchKernelGGL(slab_range_sum_kernel<double>, grid, dim3(256), 0, st, (const double*)in, C, lo, cnt, out);
  else
    hipLaunchKernelGGL(slab_range_sum_kernel<float>, grid, dim3(256), 0, st, (const float*)in, C, lo, cnt, out);
  O3S_CHECK_LAUNCH();
  return 0;
}

// O3S_BIN_EYT=0: the runtime-depth search over the row-major [F][Tp + 1] table instead of
// the unrolled search-tree kernel (A/B; read per call)
static bool bin_eyt() {
  const char* e = getenv("O3S_BIN_EYT");
  return !(e && e[0] == '0');
}

template <bool BF16>
static void bin_vec256_launch(int LV, unsigned grid, size_t lds, hipStream_t st, const void* X, int64_t n,
                              int64_t ldx, int F, const float* th, int Tp, uint8_t* out, uint8_t* out_t,
                              int64_t ldt) {
#define O3S_BIN_LV(LVC)                                                                                   \
  hipLaunchKernelGGL((bin_features_vec_kernel<BF16, 256, LVC>), dim3(grid), dim3(256), lds, st, X, n, ldx, F, th, \
                     Tp, out, out_t, ldt)
  switch (bin_eyt() ? LV : 0) {
    case 4: O3S_BIN_LV(4); break;
    case 5: O3S_BIN_LV(5); break;
    case 6: O3S_BIN_LV(6); break;
    case 7: O3S_BIN_LV(7); break;
    case 8: O3S_BIN_LV(8); break;
    default: O3S_BIN_LV(0); break;
  }
#undef O3S_BIN_LV
}

// X: [n][F] fp32 (bf16 != 0: bf16) with row stride ldx; th: [F][Tp] fp32 sorted, +inf
// padded, Tp a power of two <= 256 with at least one pad per feature; out: [n][F] uint8;
// out_t (optional): feature f of row r at out_t[f * ldt + r] (ldt >= n: a block of rows of
// a larger feature-major matrix, out_t pointing at its first row).
O3S_API int o3s_bin_features2(const void* X, int bf16, int64_t n, int64_t ldx, int F, const float* th, int Tp,
                              uint8_t* out, uint8_t* out_t, int64_t ldt, hipStream_t st) {
  if (n <= 0) return 0;
  if (Tp < 1 || Tp > 256 || (Tp & (Tp - 1)) || F <= 0) return -1;
  const size_t lds = sizeof(float) * (size_t)F * (Tp + 1) + (size_t)F * kBinTS;
  if (lds > 160 * 1024) return -2;
  const int64_t nchunks = (n + kBinRows - 1) / kBinRows;
  const unsigned grid = (unsigned)(nchunks < 8192 ? nchunks : 8192);
  if (out_t != nullptr && ldt < n) return -3;
  const bool vec = F % 8 == 0 && ldx % 8 == 0 && ((uintptr_t)X & 15) == 0;
  // vector kernel: 256-row chunks when that tile fits beside the thresholds
  const size_t lds256 = sizeof(float) * (size_t)F * (Tp + 1) + (size_t)F * (256 + 4);
  const bool big = lds256 <= 64 * 1024;
  const int64_t nch256 = (n + 255) / 256;
  const unsigned grid256 = (unsigned)(nch256 < 4096 ? nch256 : 4096);
  int LV = 0;
  while ((1 << LV) < Tp) ++LV;
  if (vec && big && bf16)
    bin_vec256_launch<true>(LV, grid256, lds256, st, X, n, ldx, F, th, Tp, out, out_t, ldt);
  else if (vec && big)
    bin_vec256_launch<false>(LV, grid256, lds256, st, X, n, ldx, F, th, Tp, out, out_t, ldt);
  else if (vec && bf16)
    hipLaunchKernelGGL((bin_features_vec_kernel<true, kBinRows>), dim3(grid), dim3(256), lds, st, X, n, ldx, F, th,
                       Tp, out, out_t, ldt);
  else if (vec)
    hipLaunchKernelGGL((bin_features_vec_kernel<false, kBinRows>), dim3(grid), dim3(256), lds, st, X, n, ldx, F, th,
                       Tp, out, out_t, ldt);
  else if (bf16)
    hipLaunchKernelGGL(bin_features_kernel<true>, dim3(grid), dim3(256), lds, st, X, n, ldx, F, th, Tp, out, out_t,
                       ldt);
  else
    hipLaunchKernelGGL(bin_features_kernel<false>, dim3(grid), dim3(256), lds, st, X, n, ldx, F, th, Tp, out, out_t,
                       ldt);
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_API int o3s_bin_features(const float* X, int64_t n, int64_t ldx, int F, const float* th, int Tp, uint8_t* out,
                             hipStream_t st) {
  return o3s_bin_features2(X, 0, n, ldx, F, th, Tp, out, nullptr, n, st);
}

// in: [n][F] uint8 with F % 4 == 0; out: [F][n].
O3S_API int o3s_u8_transpose(const uint8_t* in, int64_t n, int F, uint8_t* out, hipStream_t st) {
  if (n <= 0) return 0;
  if (F % 4 != 0 || F <= 0) return -1;
  const dim3 grid((unsigned)((n + kTrRows - 1) / kTrRows), (unsigned)((F + 63) / 64));
  hipLaunchKernelGGL(u8_transpose_kernel, grid, dim3(256), 0, st, in, n, F, out);
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_API int o3s_tree_partition(const uint8_t* bins, int64_t rs, int64_t cs, const int32_t* order, int32_t* out,
                               const int64_t* it_lo, const int64_t* it_hi, const int32_t* it_feat,
                               const int32_t* it_bin, int64_t* it_left, const int64_t* dst_left,
                               const int64_t* dst_right, uint8_t* flags, int n_items, int pass, const float* py,
                               float* py_out, const float* pw, float* pw_out, hipStream_t st) {
  if ((py != nullptr) != (py_out != nullptr) || (pw != nullptr) != (pw_out != nullptr)) return -1;
  if (n_items <= 0) return 0;
  if (pass == 0)
    hipLaunchKernelGGL(tree_part_count_kernel, dim3(n_items), dim3(kPartThreads), 0, st, bins, rs, cs, order, it_lo,
                       it_hi, it_feat, it_bin, it_left, flags);
  else
    hipLaunchKernelGGL(tree_part_scatter_kernel, dim3(n_items), dim3(kPartThreads), 0, st, order, out,
                       it_lo, it_hi, it_feat, it_bin, dst_left, dst_right, flags, py, py_out, pw, pw_out);
  O3S_CHECK_LAUNCH();
  return 0;
}

// Items of segment s are [seg_first[s], seg_first[s+1]) (nseg + 1 entries); writes the
// scatter destinations of every item and nleft[s].
O3S_API int o3s_tree_part_dest(const int64_t* it_lo, const int64_t* it_hi, const int64_t* it_left,
                               const int64_t* seg_first, const int64_t* seg_lo, int nseg, int64_t* dst_left,
                               int64_t* dst_right, int64_t* nleft, hipStream_t st) {
  if (nseg <= 0) return 0;
  hipLaunchKernelGGL(tree_part_dest_kernel, dim3(nseg), dim3(kPartThreads), 0, st, it_lo, it_hi, it_left, seg_first,
                     seg_lo, dst_left, dst_right, nleft);
  O3S_CHECK_LAUNCH();
  return 0;
}

constexpr int kHistDmaBytes = kHistWaves * 2 * 32 * 64;   // two 32-row x 64-B stages per wave

// O3S_HIST_DMA=0: the per-row byte gathers instead of the LDS-DMA row stage (A/B timing)
static bool hist_dma() {
  static const bool v = [] {
    const char* e = getenv("O3S_HIST_DMA");
    return !(e && e[0] == '0');
  }();
  return v;
}

// Shared-memory bytes needed for (F-group width fp, B bins, S stats); 0 if it cannot fit.
O3S_API int o3s_tree_hist_lds(int fp, int B, int S, int cls) {
  const int RS = 64 / fp;
  const int SL = cls ? S : 2;
  const int64_t bytes = (int64_t)kHistWaves * RS * (B * SL * fp + (RS > 1 ? 16 : 0)) * 4;
  return bytes <= 160 * 1024 ? (int)bytes : 0;
}

// One launch per feature group of 64: items = contiguous position ranges of `order`.
// slab: [n_items][F*B*S] fp32 (every cell written).  cls: 0 = REG (S must be 3), 1 = CLS.
O3S_API int o3s_tree_hist(const uint8_t* bins, int64_t n, int F, int B, int S, int cls, const int32_t* order,
                          const float* y, const float* w, const int64_t* item_lo, const int64_t* item_hi,
                          int n_items, float* slab, int ypos, hipStream_t st) {
  if (n_items <= 0) return 0;
  if (!cls && S != 3) return -1;
  int fp = 1;
  while (fp < F && fp < 64) fp <<= 1;
  if (fp < 4) fp = 4;
  const int lds = o3s_tree_hist_lds(fp, B, S, cls);
  if (lds == 0) return -2;
  // the LDS-DMA row stage: 16-B aligned rows and room beside the images
  const bool dma = fp == 64 && F % 16 == 0 && ((uintptr_t)bins & 15) == 0 && lds + kHistDmaBytes <= 160 * 1024 &&
                   hist_dma();
  const int64_t stride = (int64_t)F * B * S;
  for (int fg0 = 0; fg0 < F; fg0 += fp) {
#define O3S_TH2(FPV, C, W, P)                                                                           \
  if (FPV == 64 && dma)                                                                                 \
    hipLaunchKernelGGL((tree_hist_kernel<FPV, C, W, P, 8, true>), dim3(n_items), dim3(kHistThreads),        \
                       lds + kHistDmaBytes, st, bins, F, fg0, B, S, order, y, w, item_lo, item_hi, slab, stride); \
  else                                                                                                  \
    hipLaunchKernelGGL((tree_hist_kernel<FPV, C, W, P, 8>), dim3(n_items), dim3(kHistThreads), lds, st, bins, \
                       F, fg0, B, S, order, y, w, item_lo, item_hi, slab, stride);
#define O3S_TH1(FPV, C, W)                                                                              \
  if (ypos) { O3S_TH2(FPV, C, W, true) } else { O3S_TH2(FPV, C, W, false) }
#define O3S_TH(FPV)                                                                                     \
  if (fp == FPV) {                                                                                      \
    if (cls && w) { O3S_TH1(FPV, true, true) }                                                          \
    else if (cls) { O3S_TH1(FPV, true, false) }                                                         \
    else if (w) { O3S_TH1(FPV, false, true) }                                                           \
    else { O3S_TH1(FPV, false, false) }                                                                 \
  }
    O3S_TH(4) O3S_TH(8) O3S_TH(16) O3S_TH(32) O3S_TH(64)
#undef O3S_TH
#undef O3S_TH1
#undef O3S_TH2
    O3S_CHECK_LAUNCH();
  }
  (void)n;
  return 0;
}

// H: [k][F][B][S] fp64 node histograms; nb[F]: valid thresholds per feature; fmask
// [k][F] (uint8, null = all features); kind 0 = variance (S == 3), 1 = gini, 2 = entropy.
// mw_node (fp64 [k], nullable): per-node minimum child weight; else min_wfrac > 0 (root
// level): that fraction of the node's weight; else min_w.  out: fp64 [6k + k*V] (see tree_split_kernel).
O3S_API int o3s_tree_split(const double* H, int k, int F, int B, int S, int kind, const int32_t* nb,
                           const uint8_t* fmask, double min_inst, double min_w, double min_wfrac,
                           const double* mw_node, double* out, hipStream_t st) {
  if (k <= 0) return 0;
  if (F <= 0 || B < 2 || S <= 0 || S > kSplitMaxS || kind < 0 || kind > 2) return -1;
  if (kind == 0 && S != 3) return -1;
  if (kind == 0)
    hipLaunchKernelGGL((tree_split_kernel<false, 3>), dim3(k), dim3(kSplitThreads), 0, st, H, k, F, B, S, kind, nb,
                       fmask, min_inst, min_w, min_wfrac, mw_node, out);
  else if (S <= 8)
    hipLaunchKernelGGL((tree_split_kernel<true, 8>), dim3(k), dim3(kSplitThreads), 0, st, H, k, F, B, S, kind, nb,
                       fmask, min_inst, min_w, min_wfrac, mw_node, out);
  else
    hipLaunchKernelGGL((tree_split_kernel<true, kSplitMaxS>), dim3(k), dim3(kSplitThreads), 0, st, H, k, F, B, S,
                       kind, nb, fmask, min_inst, min_w, min_wfrac, mw_node, out);
  O3S_CHECK_LAUNCH();
  return 0;
}

// y, F, w, wv: fp64 [n] (w / wv may be null: unit training weights / no validation);
// target: fp32 [n] or null; partial: fp64 [n_blocks][4].
O3S_API int o3s_gbt_grad_loss(const double* y, const double* F, const double* w, const double* wv, int64_t n,
                              int loss, float* target, double* partial, int n_blocks, hipStream_t st) {
  if (n <= 0) return 0;
  if (loss < 0 || loss > 2 || n_blocks <= 0) return -1;
  hipLaunchKernelGGL(gbt_grad_loss_kernel, dim3(n_blocks), dim3(kGbtThreads), 0, st, y, F, w, wv, n, loss, target,
                     partial);
  O3S_CHECK_LAUNCH();
  return 0;
}

// Hs, parent: fp64 [P][FB*S]; sr: uint8 [P]; H: fp64 [2P][FB*S]; cls: 0 = REG (S == 3).
O3S_API int o3s_tree_sibling(const double* Hs, const double* parent, const uint8_t* sr, int64_t P, int FB, int S,
                             int cls, double* H, hipStream_t st) {
  if (P <= 0) return 0;
  if (FB <= 0 || S <= 0 || (!cls && S != 3)) return -1;
  const int64_t n = P * FB;
  hipLaunchKernelGGL(tree_sibling_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, Hs, parent, sr, P, FB,
                     S, cls, H);
  O3S_CHECK_LAUNCH();
  return 0;
}

// rows: int64 [n] global row ids; seeds: uint32 [T]; table: fp64 [kmax] (Poisson) or null
// (Bernoulli with `rate`); w: fp32 [n] or null; out: fp32 [T][n].
O3S_API int o3s_forest_weights(const int64_t* rows, int64_t n, const uint32_t* seeds, int T, const double* table,
                               int kmax, float rate, const float* w, float* out, hipStream_t st) {
  if (n <= 0 || T <= 0) return 0;
  if (T > 65535 || (table && kmax <= 0)) return -1;
  hipLaunchKernelGGL(forest_weights_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)T), dim3(256), 0, st, rows, n,
                     seeds, table, kmax, rate, w, out);
  O3S_CHECK_LAUNCH();
  return 0;
}

// Items as in o3s_tree_partition (it_vl / it_vr: leaf values of the item's left / right
// child); acc (fp64 [n_rows]) and part (fp32 [n_items][2]) may each be null.
O3S_API int o3s_tree_final_level(const uint8_t* bins, int64_t rs, int64_t cs, const int32_t* order,
                                 const int64_t* it_lo, const int64_t* it_hi, const int32_t* it_feat,
                                 const int32_t* it_bin, const double* it_vl, const double* it_vr, const float* y,
                                 const float* w, double* acc, float* part, int n_items, hipStream_t st) {
  if (n_items <= 0) return 0;
  if (part && !y) return -1;
  hipLaunchKernelGGL(tree_final_level_kernel, dim3(n_items), dim3(kPartThreads), 0, st, bins, rs, cs, order, it_lo,
                     it_hi, it_feat, it_bin, it_vl, it_vr, y, w, acc, part);
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_PRELOAD(trees)
