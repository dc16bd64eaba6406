// Dense exact ALS solves, ONE WAVE PER ROW: the long rows of an exact ALS half-iteration
// (the item side of the ALS config: ~200 ratings per row at rank 128; every row with more
// ratings than the Woodbury limit, or lam_u = 0).  Spark solves each row's normal equations
// with a per-row Cholesky (reached through the Recommendation widget -> ALS.fit,
// orangecontrib/spark/widgets/ml/spark_ml_recommendation.py:15); this is that solve:
//
//   A_u = G + sum_c w_c y_c y_c^T + lam_u I,   b_u = sum_c b_c y_c,   x_u = A_u^{-1} b_u
//
// Structure (replaces the one-row-per-4-wave-block kernel, whose serial diagonal phase and
// two block barriers per panel parked 3 of 4 waves: MFMA busy 0.16):
// * a 256-thread block = 4 INDEPENDENT waves, one per SIMD (launch bounds (256, 1): the
//   whole 512-register file per wave); each wave walks its own rows (row gw + k * GW of the
//   length-sorted list), no block barrier after the prologue;
// * the factor rows of a row's ratings are gathered by LDS-DMA (global_load_lds_dwordx4,
//   per-lane source = a factor row, lane-linear image) into a per-wave ring of DEPTH steps
//   of 16 ratings, with w / b of the step DMA'd beside them; the ring is a continuous
//   STREAM across rows, so the next row's first steps are in flight while this row
//   factors.  The rating indices of a step are DMA'd into its slot DEPTH steps ahead (an
//   index cursor walks the stream in front of the producer), so no ordinary vector load
//   is ever consumed while a DMA is outstanding and no step waits on a scalar-cache miss;
//   the consumer waits with a counted s_waitcnt vmcnt (later steps stay in flight);
// * the system is held as the NL = NT (NT + 1) / 2 upper 32 x 32 tiles in MFMA accumulator
//   layout (lane l: column l & 31, rows (v & 3) + 8 (v >> 2) + 4 (l >> 5) in register v):
//   160 registers at rank 128;
//   Gram   per 16 ratings, sqrt(w_c) y_c split into bf16 hi + lo, and per tile three
//          v_mfma_f32_32x32x16_bf16 (hi.hi + lo.hi + hi.lo: ~2^-16 relative, the numerics
//          of the previous kernel); A and B fragments are the same registers (lane = dim,
//          8 k-slots = 8 ratings);
//   per 32-wide panel p (A = U^T U, U_pp = L_pp^T):
//     A  the diagonal tile is factored by this wave (lane i holds row i, column c's
//        multipliers by v_readlane inside 4-column blocks, the deferred rank-4 update of
//        the later columns two at a time on v_pk_fma_f32 from a transposed LDS block);
//        lanes 32-63 run the same recurrence on the identity, giving X_p = L_pp^-1, and
//        y_p = X_p r_p (solving along the pivots instead, one more v_readlane + FMA per
//        column on the serial chain, cost more than this pass over X_p);
//     B  U_pi = X_p S_pi as bf16x3 on v_mfma_f32_32x32x16_bf16 (6 instead of 16
//        v_mfma_f32_32x32x2_f32: a quarter of the matrix-pipe cycles), B operand = the
//        tile's own registers split hi / lo; r_i -= U_pi^T y_p (a sum over the tile's
//        registers + one lane swap);
//     C  S_ji -= U_pj^T U_pi, bf16x3 with BOTH operands straight from registers (register
//        v of tile (p, j) pairs with register v of tile (p, i): the same k index);
//   backward U x = y: per p the products U_pi x_i are summed across lanes through one LDS
//   transpose, x_p = X_p^T t with X_p parked in the diagonal tile's registers.
// * implicit G: its upper tiles live in LDS once per block, in accumulator order (one
//   ds_read_b128 per 4 registers).
#include "als_mfma.h"

using namespace o3s;
using namespace o3s::als;

namespace {

// DEEP (explicit: no G in LDS): the 40 KB G would take carry a fourth ring step at ranks
// 96 / 128 (implicit keeps G in LDS: reading it per row from global memory spilled)
template <int R, bool DEEP = false>
struct DW {
  static constexpr int NT = R / 32;
  static constexpr int NL = NT * (NT + 1) / 2;
  static constexpr int CH = 16;                         // ratings per step (one k-block of 16)
  static constexpr int LPR = R / 4;                     // lanes per factor row (16 B each)
  static constexpr int LPS = R == 96 ? 32 : LPR;        // lane span of a row in one DMA
  static constexpr int RS = R == 96 ? 128 : R;          // LDS row stride (floats)
  static constexpr int RPI = 64 / LPS;                  // rows per DMA instruction
  static constexpr int NI = CH / RPI;                   // row DMAs per step
  static constexpr int NIS = NI + 2;                    // + the w / b / index and metadata DMAs
  static constexpr int DEPTH = R >= 96 ? (DEEP ? 4 : 3) : (R == 64 ? 5 : 8);
  static constexpr int SLOT = CH * RS;                  // floats per ring slot
  static constexpr int TS = 32 * 33;                    // padded 32 x 32 scratch tile
  static constexpr int MAHEAD = DEPTH;                  // row metadata fetched this far ahead
  static constexpr int MR = 3 * DEPTH + 1;              // ... into a ring of MR rows
  static constexpr int WAVE = DEPTH * SLOT + DEPTH * 48 + MR * 8 + TS + R;   // floats per wave
  static constexpr int GL = NL * 1024;                  // implicit G, accumulator order
};

// TIM (diagnostic, o3s_als_dense_wave_timed): per-wave shader-clock totals of the row
// setup, the Gram loop (of which: inside advance(), i.e. producing + waiting for the DMA
// ring), the factorisation + forward solve (of which per panel: A the diagonal factor, the
// y_p / X_p hand-off, B the U_pi products, C the trailing update), and the backward solve +
// store, written to ((long long*)dbg)[wave][9]
template <int R, bool IMPL, bool DBG = false, bool TIM = false>
__global__ __launch_bounds__(256, 1) void als_dense_wave_kernel(
    const int32_t* __restrict__ meta, const int32_t* __restrict__ cols, const float* __restrict__ w,
    const float* __restrict__ b, const float* __restrict__ F, const float* __restrict__ G, int64_t nrows,
    float* __restrict__ X, float* __restrict__ dbg, const float* __restrict__ gd = nullptr) {
  using D = DW<R, !IMPL>;
  constexpr int NT = D::NT, NL = D::NL, CH = D::CH, DEPTH = D::DEPTH, RS = D::RS, LPS = D::LPS,
                RPI = D::RPI, NI = D::NI, SLOT = D::SLOT, MR = D::MR, MAHEAD = D::MAHEAD;
  // ONE __shared__ array (a second object beside the DMA ring can make hipcc wait vmcnt(0)
  // before ring reads)
  __shared__ __attribute__((aligned(16))) float lds[4 * D::WAVE + (IMPL ? D::GL : R)];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // G first: its per-lane reads are one base register + immediate offsets (< 64 KB)
  float* const sG = lds;                                  // [NL][4][64][4]
  float* const wl = lds + (IMPL ? D::GL : 0) + wid * D::WAVE;
  float* const ring = wl;                                 // [DEPTH][CH][RS]
  float* const swb = wl + DEPTH * SLOT;                   // [DEPTH][w 16 | b 16 | idx 16]
  float* const smeta = swb + DEPTH * 48;                  // [MR][8] row metadata ring
  float* const scr = smeta + MR * 8;                      // [32][33] scratch tile
  float* const sr = scr + D::TS;                          // [R] rhs -> y -> x

  if constexpr (IMPL) {
    // G's upper tiles in accumulator order: lane l's registers 4k..4k+3 of tile t at
    // sG[t][k][l][0..3] (no DMA is in flight yet: a plain __syncthreads is a bare barrier)
    const int h = lane >> 5, q = lane & 31;
    for (int t = wid; t < NL; t += 4) {
      int tj = 0, tt = t;
      while (tt >= NT - tj) { tt -= NT - tj; ++tj; }
      const int ti = tj + tt;
#pragma unroll
      for (int v = 0; v < 16; ++v)
        sG[t * 1024 + (v >> 2) * 256 + lane * 4 + (v & 3)] = G[(32 * tj + rowof(v, h)) * R + 32 * ti + q];
    }
    __syncthreads();
  } else {
    // diagonal G (the eigenbasis solve: G = diag(eig), rotated tables): R floats after the
    // waves' areas, staged once per block -- a per-row global read of gd would be waited
    // for with vmcnt(0), draining the DMA ring
    float* const sGd = lds + 4 * D::WAVE;
    for (int c = threadIdx.x; c < R; c += 256) sGd[c] = gd != nullptr ? gd[c] : 0.f;
    __syncthreads();
  }

  const int64_t GW = (int64_t)gridDim.x * 4;
  const int64_t gw = (int64_t)blockIdx.x * 4 + wid;
  // this wave's k-th row is row gw + k GW of the (length-sorted) list
  auto has_row = [&](int k) { return gw + (int64_t)k * GW < nrows; };

  // ---- row metadata {p0, n, u, lam_u} (host-built, list order) reaches LDS by DMA, MAHEAD
  // rows ahead of the index cursor (one row per step at most, the same rate the cursor can
  // move), into a ring of MR slots: every walk below reads it there, none through the
  // scalar cache (a strided / gathered s_load missed once per row per walk) ----
  auto meta_dma = [&](int k, int slot) {       // lanes 0..7: row k's 8 dwords -> slot
    int64_t idx = gw + (int64_t)k * GW;
    idx = idx < nrows ? idx : nrows - 1;
    int ln = lane;
    asm volatile("" : "+v"(ln));
    if (ln < 8)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const float*>(meta + idx * 8 + ln), smeta + slot * 8, 4, 0, 0);
  };
  struct RowMeta {
    int64_t p0, p1;
    int64_t u;
    float lam;
  };
  auto meta_read = [&](int slot) {
    const u32x4_t m = *reinterpret_cast<const u32x4_t*>(smeta + slot * 8);
    const float lm = smeta[slot * 8 + 4];
    RowMeta r;
    const uint32_t lo = __builtin_amdgcn_readfirstlane(m[0]), hi = __builtin_amdgcn_readfirstlane(m[1]);
    r.p0 = (int64_t)(((uint64_t)hi << 32) | lo);
    r.p1 = r.p0 + (int32_t)__builtin_amdgcn_readfirstlane(m[2]);
    r.u = (int32_t)__builtin_amdgcn_readfirstlane(m[3]);
    r.lam = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, lm)));
    return r;
  };
  auto next_mod = [](int s) { return s + 1 == MR ? 0 : s + 1; };

  // ---- producer: the stream of 16-rating steps over this wave's rows.  The rating indices
  // of a step come from its ring slot, DMA'd there DEPTH steps earlier by an index cursor
  // walking the same stream ahead (with the w / b DMA of the step that last used the slot):
  // reading them through the scalar cache instead stalled every step on a miss ----
  int xk = -1, xms = MR - 1;                   // index cursor: row, its metadata slot
  int64_t xj = 0, xe = 0;
  auto cursor_next = [&]() -> bool {           // the cursor's next step; false at stream end
    while (xj >= xe) {
      if (!has_row(xk + 1)) return false;
      ++xk;
      xms = next_mod(xms);
      const RowMeta m = meta_read(xms);
      xj = m.p0;
      xe = m.p1;
    }
    return true;
  };
  auto index_src = [&](int ln) {                // lanes 32..47: the cursor step's indices
    const int64_t jx = xj + (ln & 15) < xe - 1 ? xj + (ln & 15) : xe - 1;
    return reinterpret_cast<const float*>(cols + jx);
  };
  long long tacc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  long long tp = TIM ? (long long)clock64() : 0;
  auto stamp = [&](int ph) {
    if constexpr (TIM) {
      const long long now = (long long)clock64();
      tacc[ph] += now - tp;
      tp = now;
    }
  };
  int mk = 0, mslot = 0;                       // next row whose metadata is fetched, its slot
  int pk = -1, pms = MR - 1;                   // producer: row, its metadata slot
  int64_t pj = 0, pe = 0;
  int issued = 0, pslot = 0;
  auto produce = [&]() {
    while (pj >= pe) {
      if (!has_row(pk + 1)) return;
      ++pk;
      pms = next_mod(pms);
      const RowMeta m = meta_read(pms);
      pj = m.p0;
      pe = m.p1;
    }
    const int64_t last = pe - 1;
    float* const dst = ring + pslot * SLOT;
    float* const wb = swb + pslot * 48;
    // per-lane address terms recomputed per call (hoisted, they sat in spill slots whose
    // reloads drained the DMA ring with vmcnt(0))
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int rr = ln / LPS, lo = ln % LPS;
    const int32_t* const si = reinterpret_cast<const int32_t*>(wb + 32);
    int32_t ci[NI];
#pragma unroll
    for (int ins = 0; ins < NI; ++ins) ci[ins] = si[ins * RPI + rr];
#pragma unroll
    for (int ins = 0; ins < NI; ++ins) {
      const float* src = F + (int64_t)ci[ins] * R + 4 * lo;
      if constexpr (R == 96) {
        if (lo < 24) __builtin_amdgcn_global_load_lds(src, dst + ins * RPI * RS, 16, 0, 0);
      } else {
        __builtin_amdgcn_global_load_lds(src, dst + ins * RPI * RS, 16, 0, 0);
      }
    }
    // w / b of this step beside it, the indices of the step DEPTH ahead behind them
    const bool ahead = cursor_next();
    if (ln < 32 || (ahead && ln < 48)) {
      const int64_t jj = pj + (ln & 15) < last ? pj + (ln & 15) : last;
      const float* src = ln < 16 ? w + jj : ln < 32 ? b + jj : index_src(ln);
      __builtin_amdgcn_global_load_lds(src, wb, 4, 0, 0);
    }
    if (ahead) xj += CH;
    // one metadata row per step (every step issues the same NIS DMAs): the next one once
    // the cursor is within MAHEAD rows of it, else the last one again (same bytes)
    if (mk <= xk + MAHEAD) {
      meta_dma(mk, mslot);
      ++mk;
      mslot = next_mod(mslot);
    } else {
      meta_dma(mk - 1, mslot == 0 ? MR - 1 : mslot - 1);
    }
    pj += CH;
    ++issued;
    pslot = pslot + 1 == DEPTH ? 0 : pslot + 1;
  };

  {
    // the metadata of the first MAHEAD + DEPTH + 1 rows and the indices of the first DEPTH
    // steps, synchronously (the index cursor's first DEPTH steps may cross DEPTH rows)
    for (; mk <= MAHEAD + DEPTH; ++mk) meta_dma(mk, mk);
    mslot = mk;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int ln = lane;
    asm volatile("" : "+v"(ln));
    for (int k = 0; k < DEPTH && cursor_next(); ++k) {
      if (ln >= 32 && ln < 48) __builtin_amdgcn_global_load_lds(index_src(ln), swb + k * 48, 4, 0, 0);
      xj += CH;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  for (int i = 0; i < DEPTH - 1; ++i) produce();
  int consumed = 0, cslot = 0;

  int cms = MR - 1;
  for (int k = 0; has_row(k); ++k) {
    const int64_t idx = gw + (int64_t)k * GW;
    cms = next_mod(cms);
    const RowMeta rm = meta_read(cms);
    const int64_t u = rm.u, p0 = rm.p0, p1 = rm.p1;
    const float lu = rm.lam;
    // the lane's coordinates, laundered per PHASE: lane-dependent constants (identity
    // columns, diagonal masks, LDS addresses) are recomputed where they are used instead of
    // being hoisted across the Gram loop into registers that then spill inside it
    int q = lane & 31, h = lane >> 5;
    asm volatile("" : "+v"(q), "+v"(h));
    // the system starts as G + lam_u I (G from its LDS copy), the Gram accumulates on top
    f32x16_t acc[NL];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      // !IMPL: lam_u plus the diagonal G (zero when explicit) on the diagonal
      float dj = lu;
      if constexpr (!IMPL) dj += lds[4 * D::WAVE + 32 * j + q];
#pragma unroll
      for (int i = j; i < NT; ++i) {
        const int t = tix<NT>(j, i);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float4_ g = {0.f, 0.f, 0.f, 0.f};
          if constexpr (IMPL) g = *reinterpret_cast<const float4_*>(sG + t * 1024 + k * 256 + lane * 4);
          const float gv[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            acc[t][4 * k + e] = (i == j && rowof(4 * k + e, h) == q) ? (IMPL ? gv[e] + lu : dj) : gv[e];
        }
      }
    }
    float rh[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) rh[j] = 0.f;
    stamp(0);

    // ---- Gram, software-pipelined in place: after the MFMAs of tile row j of step s
    // (tiles (j, j..NT-1)), fragment block j is dead for step s and is rebuilt for step
    // s+1 (LDS reads, sqrt(w) scaling, hi / lo split, rhs FMAs) in the same basic block as
    // the remaining MFMAs of step s, so the scheduler can place that VALU work in the MFMA
    // gaps (one wave per SIMD hides ~5 single-issue instructions per
    // v_mfma_f32_32x32x16_bf16) without a second fragment set (the registers are full at
    // rank 128).  The ring slot of step s is read out one iteration earlier, so
    // produce() still keeps two steps in flight. ----
    auto advance = [&]() {
      stamp(1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot being refilled is read out
      produce();
      stamp(4);
      wait_steps<D::NIS>(issued - 1 - consumed);
      stamp(9);
    };
    float sw[8], bb[8];
    auto step_scale = [&](int64_t j0) {            // sqrt(w) and b of the step's 8 ratings per lane half
      const float* wb = swb + cslot * 48;
      const int nv = (int)(p1 - j0 < CH ? p1 - j0 : CH);
      const float4_ w0 = *reinterpret_cast<const float4_*>(wb + 8 * h);
      const float4_ w1 = *reinterpret_cast<const float4_*>(wb + 8 * h + 4);
      const float4_ b0 = *reinterpret_cast<const float4_*>(wb + 16 + 8 * h);
      const float4_ b1 = *reinterpret_cast<const float4_*>(wb + 16 + 8 * h + 4);
      const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const bool ok = 8 * h + k < nv;
        sw[k] = ok ? __builtin_amdgcn_sqrtf(fmaxf(wv[k], 0.f)) : 0.f;   // v_sqrt_f32 (1 ulp; sqrtf expands to ~12 VALU)
        bb[k] = ok ? bv[k] : 0.f;
      }
    };
    bf16x8_t hi[NT], lo[NT];
    auto load_block = [&](int j) {                 // fragment block j of the step in cslot
      const float* sl = ring + cslot * SLOT;
      float y[8], z[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) y[k] = sl[(8 * h + k) * RS + 32 * j + q];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        rh[j] = fmaf(bb[k], y[k], rh[j]);
        z[k] = sw[k] * y[k];
      }
      split8(z, hi[j], lo[j]);
    };
    auto mfma_row = [&](int j) {                   // tiles (j, j..NT-1) of the current step
#pragma unroll
      for (int i = j; i < NT; ++i) {
        f32x16_t& a = acc[tix<NT>(j, i)];
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(hi[j], hi[i], a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lo[j], hi[i], a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(hi[j], lo[i], a, 0, 0, 0);
      }
    };
    auto next_slot = [&]() {
      ++consumed;
      cslot = cslot + 1 == DEPTH ? 0 : cslot + 1;
    };
    if (p1 > p0) {
      advance();
      step_scale(p0);
#pragma unroll
      for (int j = 0; j < NT; ++j) load_block(j);
      next_slot();
      for (int64_t j0 = p0 + CH; j0 < p1; j0 += CH) {
        advance();
        step_scale(j0);                 // step s+1's scales ...
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          mfma_row(j);                  // ... step s's tile row j ...
          load_block(j);                // ... then block j rebuilt for step s+1
        }
        next_slot();
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) mfma_row(j);
    }

    stamp(1);
    // ---- rhs ----
    q = lane & 31;
    h = lane >> 5;
    asm volatile("" : "+v"(q), "+v"(h));
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const float t = rh[j] + __shfl_xor(rh[j], 32, 64);
      if (h == 0) sr[32 * j + q] = t;
    }
    lane_sync();

    if (DBG && idx < 64) {                // diagnostic dump: the assembled system (C layout)
#pragma unroll
      for (int t = 0; t < NL; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) dbg[((idx * 2) * NL + t) * 1024 + v * 64 + lane] = acc[t][v];
    }
    // ---- blocked Cholesky A = U^T U, forward solve U^T y = rhs riding along ----
#pragma unroll
    for (int p = 0; p < NT; ++p) {
      f32x16_t& dg = acc[tix<NT>(p, p)];
#pragma unroll
      for (int v = 0; v < 16; ++v) scr[rowof(v, h) * 33 + q] = dg[v];
      lane_sync();
      // A: lanes 0-31 row q of the tile -> row q of L; lanes 32-63 column q of the
      // identity -> column q of X_p = L_pp^-1 (the same right-looking FMA with the lane's
      // own multiplier).  4-column blocks: v_readlane inside, then one rank-4 update of
      // the later columns.
      f32x2_t v2[16];                      // v[k] = v2[k / 2][k % 2]: pairs for v_pk_fma_f32
#pragma unroll
      for (int k = 0; k < 32; ++k) v2[k >> 1][k & 1] = scr[q * 33 + k];   // every lane loads (a
#pragma unroll                                                          // per-lane conditional load
      for (int k = 0; k < 32; ++k)                                      // became 32 branches)
        v2[k >> 1][k & 1] = h ? (k == q ? 1.f : 0.f) : v2[k >> 1][k & 1];
      float* const sT = scr;                 // [4][64]: the block's 4 multipliers of every lane
#pragma unroll
      for (int c0 = 0; c0 < 32; c0 += 4) {
#pragma unroll
        for (int c = c0; c < c0 + 4; ++c) {
          // lane c's entries c..c0+3 of the Schur complement, read together: by symmetry
          // (bitwise: every lane runs the same FMAs on its row) a_j rs = L_jc, so the
          // multipliers need no second v_readlane after the pivot's rsqrt
          float a[4];
#pragma unroll
          for (int j = c; j < c0 + 4; ++j) a[j - c0] = rl(v2[j >> 1][j & 1], c);
          const float rs = __builtin_amdgcn_rsqf(__builtin_amdgcn_fmed3f(a[c - c0], 1e-30f, 3.0e38f));
          const float t = v2[c >> 1][c & 1] * rs;
          v2[c >> 1][c & 1] = t;
#pragma unroll
          for (int j = c + 1; j < c0 + 4; ++j) v2[j >> 1][j & 1] = fmaf(-t, a[j - c0] * rs, v2[j >> 1][j & 1]);
        }
        if (c0 + 4 < 32) {
          // rank-4 update of the later columns, two per v_pk_fma_f32: L[j..j+3][c] of rows
          // j = 4g.. read as one float4 from the transposed block
#pragma unroll
          for (int k = 0; k < 4; ++k) sT[k * 64 + lane] = v2[(c0 + k) >> 1][k & 1];
          lane_sync();
#pragma unroll
          for (int g = c0 / 4 + 1; g < 8; ++g) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const float4_ l = *reinterpret_cast<const float4_*>(sT + k * 64 + 4 * g);
              const float m = -v2[(c0 + k) >> 1][k & 1];
              const f32x2_t mm = {m, m};
              v2[2 * g] = __builtin_elementwise_fma(mm, f32x2_t{l.x, l.y}, v2[2 * g]);
              v2[2 * g + 1] = __builtin_elementwise_fma(mm, f32x2_t{l.z, l.w}, v2[2 * g + 1]);
            }
          }
          lane_sync();                                               // sT reads done
        }
      }
      float v[32];
#pragma unroll
      for (int k = 0; k < 32; ++k) v[k] = v2[k >> 1][k & 1];
      stamp(5);
      if (h == 1) {
#pragma unroll
        for (int k = 0; k < 32; ++k) scr[k * 33 + q] = v[k];        // X_p[k][q]
      }
      lane_sync();
      {
        // both lane halves run it (no exec split; the upper half's sums are dropped), four
        // partial sums so the FMA chain is 8 deep instead of 32
        float y4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 32; ++j) y4[j & 3] = fmaf(scr[q * 33 + j], sr[32 * p + j], y4[j & 3]);
        lane_sync();
        if (h == 0) sr[32 * p + q] = (y4[0] + y4[1]) + (y4[2] + y4[3]);   // y_p = X_p r_p
      }
      lane_sync();
      float xa[16], yv[16];
#pragma unroll
      for (int vv = 0; vv < 16; ++vv) {
        xa[vv] = scr[q * 33 + rowof(vv, h)];                        // X_p[q][r(v, h)]: A operand
        yv[vv] = sr[32 * p + rowof(vv, h)];
      }
#pragma unroll
      for (int vv = 0; vv < 16; ++vv) dg[vv] = scr[rowof(vv, h) * 33 + q];   // X_p, C layout
      // B: U_pi = X_p S_pi; r_i -= U_pi^T y_p.  bf16x3 on v_mfma_f32_32x32x16_bf16 (the
      // Gram's numerics): register v of a tile is k-slot v & 7 of k-block v >> 3 for BOTH
      // operands (lane half h holds k = rowof(v, h)), so the k pairing is consistent
      stamp(6);
      bf16x8_t xh[2], xl[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        float z8[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) z8[k] = xa[8 * m + k];
        split8(z8, xh[m], xl[m]);
      }
#pragma unroll
      for (int i = p + 1; i < NT; ++i) {
        f32x16_t& s = acc[tix<NT>(p, i)];
        f32x16_t z;
#pragma unroll
        for (int vv = 0; vv < 16; ++vv) z[vv] = 0.f;
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          bf16x8_t sh, sl;
          split_half(s, m, sh, sl);
          z = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh[m], sh, z, 0, 0, 0);
          z = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xl[m], sh, z, 0, 0, 0);
          z = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh[m], sl, z, 0, 0, 0);
        }
        s = z;
        float part = 0.f;
#pragma unroll
        for (int vv = 0; vv < 16; ++vv) part = fmaf(z[vv], yv[vv], part);
        part += __shfl_xor(part, 32, 64);
        if (h == 0) sr[32 * i + q] -= part;
      }
      lane_sync();
      stamp(7);
      // C: S_ji -= U_pj^T U_pi, operands straight from the panel tiles' registers (bf16x3,
      // -U_pj by flipping the bf16 sign bits)
      bf16x8_t uh[NT][2], ul[NT][2];
#pragma unroll
      for (int i = p + 1; i < NT; ++i)
#pragma unroll
        for (int m = 0; m < 2; ++m) split_half(acc[tix<NT>(p, i)], m, uh[i][m], ul[i][m]);
#pragma unroll
      for (int j = p + 1; j < NT; ++j) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const bf16x8_t nh = neg8(uh[j][m]), nl = neg8(ul[j][m]);
#pragma unroll
          for (int i = j; i < NT; ++i) {
            f32x16_t& s = acc[tix<NT>(j, i)];
            s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(nh, uh[i][m], s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(nl, uh[i][m], s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(nh, ul[i][m], s, 0, 0, 0);
          }
        }
      }
      stamp(8);
    }

    stamp(2);
    if (DBG && idx < 64) {                // diagnostic dump: U / X_p tiles and y
#pragma unroll
      for (int t = 0; t < NL; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) dbg[((idx * 2 + 1) * NL + t) * 1024 + v * 64 + lane] = acc[t][v];
      for (int c = lane; c < R; c += 64) dbg[128 * NL * 1024 + idx * R + c] = sr[c];
    }
    // ---- backward U x = y ----
#pragma unroll
    for (int p = NT - 1; p >= 0; --p) {
      if (p < NT - 1) {
        float prod[16];
#pragma unroll
        for (int vv = 0; vv < 16; ++vv) prod[vv] = 0.f;
#pragma unroll
        for (int i = p + 1; i < NT; ++i) {
          const float xi = sr[32 * i + q];
          const f32x16_t& ui = acc[tix<NT>(p, i)];
#pragma unroll
          for (int vv = 0; vv < 16; ++vv) prod[vv] = fmaf(ui[vv], xi, prod[vv]);
        }
        lane_sync();
#pragma unroll
        for (int vv = 0; vv < 16; ++vv) scr[rowof(vv, h) * 33 + q] = prod[vv];
        lane_sync();
        float s4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 32; ++k) s4[k & 3] += scr[q * 33 + k];
        if (h == 0) sr[32 * p + q] -= (s4[0] + s4[1]) + (s4[2] + s4[3]);
      }
      lane_sync();
      const f32x16_t& xp = acc[tix<NT>(p, p)];
      float t2[2] = {0.f, 0.f};
#pragma unroll
      for (int vv = 0; vv < 16; ++vv) t2[vv & 1] = fmaf(xp[vv], sr[32 * p + rowof(vv, h)], t2[vv & 1]);
      float t = t2[0] + t2[1];
      t += __shfl_xor(t, 32, 64);
      if (h == 0) sr[32 * p + q] = t;
      lane_sync();
    }
#pragma unroll
    for (int c = 0; c < R; c += 64)
      if (c + lane < R) X[u * R + c + lane] = sr[c + lane];
    stamp(3);
  }
  // every DMA this wave issued was waited for by the step that consumed it
  if constexpr (TIM) {
    if (lane == 0)
      for (int ph = 0; ph < 10; ++ph) reinterpret_cast<long long*>(dbg)[gw * 10 + ph] = tacc[ph];
  }
}

template <int R>
int launch(int implicit, const int32_t* meta, const int32_t* cols, const float* w, const float* b, const float* F,
           const float* G, int64_t nrows, float* X, int grid, float* dbg, hipStream_t st, const float* gd = nullptr) {
  if (dbg != nullptr) {
    if (implicit)
      hipLaunchKernelGGL((als_dense_wave_kernel<R, true, true>), dim3(grid), dim3(256), 0, st, meta, cols, w, b, F, G,
                         nrows, X, dbg, nullptr);
    else
      hipLaunchKernelGGL((als_dense_wave_kernel<R, false, true>), dim3(grid), dim3(256), 0, st, meta, cols, w, b, F,
                         G, nrows, X, dbg, gd);
  } else if (implicit) {
    hipLaunchKernelGGL((als_dense_wave_kernel<R, true>), dim3(grid), dim3(256), 0, st, meta, cols, w, b, F, G, nrows,
                       X, nullptr, nullptr);
  } else {
    hipLaunchKernelGGL((als_dense_wave_kernel<R, false>), dim3(grid), dim3(256), 0, st, meta, cols, w, b, F, G, nrows,
                       X, nullptr, gd);
  }
  O3S_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// Dense exact solves of ``nrows`` rows, one wave per row, ``grid`` blocks of 4 waves
// (persistent: 1 block per CU, wave gw takes list rows gw, gw + 4 grid, ...).  meta: int32
// [nrows][8] in list order (the caller lists rows longest first for balance):
// {p0 lo, p0 hi, n >= 1, u, lam_u bits, 0, 0, 0} -- row u's ratings are [p0, p0 + n) of
// cols / w / b; x_u written into X[u]; implicit: G = Y^T Y (fp32 R x R).  Diagnostic: a
// non-null dbg [(64 rows x 2 stages x NL tiles x 1024) + 64 x R] receives, for the first
// 64 listed rows, the accumulator tiles (raw C layout: [v][lane]) after the system is
// assembled and after the forward factorisation, plus y (grid forced to 1).
O3S_API int o3s_als_dense_wave_dbg(int implicit, int R, const int32_t* meta, const int32_t* cols, const float* w,
                                   const float* b, const float* F, const float* G, int64_t nrows, float* X, int grid,
                                   float* dbg, hipStream_t st) {
  if (nrows < 0 || (implicit && !G) || grid <= 0) return -1;
  if (nrows == 0) return 0;
  const int64_t need = (nrows + 3) / 4;
  if (grid > need) grid = (int)need;
  if (dbg != nullptr) grid = 1;
  switch (R) {
    case 32: return launch<32>(implicit, meta, cols, w, b, F, G, nrows, X, grid, dbg, st);
    case 64: return launch<64>(implicit, meta, cols, w, b, F, G, nrows, X, grid, dbg, st);
    case 96: return launch<96>(implicit, meta, cols, w, b, F, G, nrows, X, grid, dbg, st);
    case 128: return launch<128>(implicit, meta, cols, w, b, F, G, nrows, X, grid, dbg, st);
    default: return -2;
  }
}

// Diagnostic (tools/als_dense_phases.py): als_dense_wave_kernel<128, implicit> with the TIM
// phase clocks; tim: int64 [grid * 4][10] (row setup, Gram, factor + forward, backward +
// store, of the Gram loop produce(), of the factorisation A, hand-off, B, C, and of the
// Gram loop the DMA waits).
O3S_API int o3s_als_dense_wave_timed(const int32_t* meta, const int32_t* cols, const float* w, const float* b,
                                     const float* F, const float* G, int64_t nrows, float* X, int grid, long long* tim,
                                     hipStream_t st) {
  if (nrows <= 0 || !G || grid <= 0 || !tim) return -1;
  hipLaunchKernelGGL((als_dense_wave_kernel<128, true, false, true>), dim3(grid), dim3(256), 0, st, meta, cols, w, b,
                     F, G, nrows, X, reinterpret_cast<float*>(tim));
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_API int o3s_als_dense_wave(int implicit, int R, const int32_t* meta, const int32_t* cols, const float* w,
                               const float* b, const float* F, const float* G, int64_t nrows, float* X, int grid,
                               hipStream_t st) {
  return o3s_als_dense_wave_dbg(implicit, R, meta, cols, w, b, F, G, nrows, X, grid, nullptr, st);
}

// Diagonal-G solves (the eigenbasis half-iterations: F = the rotated table F Q, G =
// diag(gd)): the explicit build (no G image in LDS, so a 4-step gather ring at ranks 96 /
// 128) with gd[c] + lam_u on the diagonal.  gd: fp32 [R].  Timing parity with the full-G
// build (profiles/kernel_experiments_r6.json); it spares the R x R diag(eig) and the G
// image's LDS.
O3S_API int o3s_als_dense_wave_gd(int R, const int32_t* meta, const int32_t* cols, const float* w, const float* b,
                                  const float* F, const float* gd, int64_t nrows, float* X, int grid, hipStream_t st) {
  if (nrows < 0 || !gd || grid <= 0) return -1;
  if (nrows == 0) return 0;
  const int64_t need = (nrows + 3) / 4;
  if (grid > need) grid = (int)need;
  switch (R) {
    case 32: return launch<32>(0, meta, cols, w, b, F, nullptr, nrows, X, grid, nullptr, st, gd);
    case 64: return launch<64>(0, meta, cols, w, b, F, nullptr, nrows, X, grid, nullptr, st, gd);
    case 96: return launch<96>(0, meta, cols, w, b, F, nullptr, nrows, X, grid, nullptr, st, gd);
    case 128: return launch<128>(0, meta, cols, w, b, F, nullptr, nrows, X, grid, nullptr, st, gd);
    default: return -2;
  }
}

O3S_PRELOAD(als_dense)
