// Generalised-linear-model streaming kernels (gfx950).
//
// Replaces the per-partition gradient closure that Spark MLlib runs inside
// `treeAggregate` for LogisticRegression / LinearSVC / LinearRegression (reached in
// the reference through OWSparkEstimator.apply -> `fit`,
// orangecontrib/spark/base/spark_ml_estimator.py:19-25).
//
// Layout: X is a row-major bf16 matrix [n, ld] (ld % 8 == 0, zero padded).  A row
// is split over LPR lanes ("row group"); lane c of a group owns the 16-B chunks
// c, c+LPR, ... (CPL chunks).  A wave therefore streams 64/LPR consecutive rows per
// `global_load_dwordx4` -- for D = 256 that is two rows per wave-instruction, 1 KiB
// contiguous -- and the gradient  X^T r  is lane-local (each lane always touches
// the same 8*CPL columns), so only the per-row dot product needs a cross-lane sum.
//
// The op is a GEMV: HBM bound (512 B/row at D=256), so MFMA buys nothing here
// (SURVEY §7.5 item 2); the budget is bytes.  VALU work per row is ~6x below the
// HBM-bound cycle budget at 256 CUs, so the kernel runs at the streaming rate.
//
// Cross-block reduction: one fp32 slab row per block + `glm_finish` (fp64, fixed
// order) -> bitwise deterministic results, no float atomics (Guideline 12).
//
// SRC == 1 ("synthetic lineage"): instead of loading a chunk, the lane regenerates
// it from the counter hash used by `synth_glm_kernel`, so rows that did not fit in
// HBM are recomputed from lineage on every pass -- the MI355X equivalent of Spark's
// MEMORY_ONLY caching, where evicted partitions are recomputed.  Regenerated and
// materialised rows are bit-identical.
#include "common.h"

using namespace o3s;

namespace {

enum { LOSS_LOGISTIC = 0, LOSS_HINGE = 1, LOSS_SQUARED = 2 };

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;

// Synthetic features: word i = mix24(fk + i * 0x9E3779) of the row's feature key fk
// supplies the four features 4i..4i+3, one per byte b: x = (2b - 255) / 256, i.e. 256
// symmetric levels in (-1, 1) (mean 0, var ~1/3), every one EXACT in bf16 (<= 8
// significant bits).  Exactness lets the lineage pass skip the bf16 round trip: it
// decodes a byte with one v_cvt_f32_ubyteN and folds the affine map into the weights
// (see glm_grad_kernel), two hashes per 16-B chunk.
//
// mix24 is a bijective 32-bit mixer built from full-rate VALU ops only: two
// v_mad_u32_u24 steps h <- (h mod 2^24) * C + h (a bijection for even C: the low 24 bits
// are multiplied by the odd C + 1, the top byte is recovered from the carry) between
// xorshifts -- 5 issue cycles per word, vs 13 for murmur's fmix32 whose two
// v_mul_lo_u32 are quarter rate.  On byte-uniformity (chi^2), cross-column correlation
// and word-uniqueness tests it matches fmix32 (see ops/glm.py::_mix24, the torch twin).
__host__ __device__ __forceinline__ uint32_t umad24(uint32_t a, uint32_t c, uint32_t add) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul24(a, c) + add;
#else
  return (a & 0xFFFFFFu) * c + add;
#endif
}
__host__ __device__ __forceinline__ uint32_t mix24(uint32_t h) {
  h ^= h >> 16;
  h = umad24(h, 0xED5AD4u, h);
  h ^= h >> 15;
  return umad24(h, 0x2C1B3Cu, h);
}
// Feature key of global row `row` (labels use the murmur row_key of common.h).
__device__ __forceinline__ uint32_t feat_key(uint32_t seed, int64_t row) {
  const uint32_t lo = (uint32_t)(row & 0xffffffffll);
  const uint32_t hi = (uint32_t)((uint64_t)row >> 32);
  return mix24(mix24(lo + seed * 0x9E3779B1u) ^ umad24(hi, 0x7FEB35u, 0x165667u));
}
__device__ __forceinline__ uint32_t synth_word(uint32_t fk, int i) {
  return mix24(umad24((uint32_t)i, 0x9E3779u, fk));
}
__device__ __forceinline__ float synth_byte(uint32_t h, int q) {
  return (float)((h >> (8 * q)) & 0xffu);     // -> v_cvt_f32_ubyte{q}
}
constexpr float kSynthScale = 1.0f / 128.0f, kSynthShift = -255.0f / 256.0f;
// One 16-B chunk (8 features) of synthetic row `rk` at chunk index ch, as bf16.
__device__ __forceinline__ short8 synth_chunk(uint32_t fk, int ch) {
  short8 v;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const uint32_t h = synth_word(fk, 2 * ch + p);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      v[4 * p + q] = (short)f32_to_bf16(fmaf(synth_byte(h, q), kSynthScale, kSynthShift));
  }
  return v;
}
// Label draw for a synthetic row: y ~ Bernoulli(sigmoid(margin_true)).
__device__ __forceinline__ float synth_label(uint32_t rk, float margin_true) {
  const float u = (float)(fmix32(rk ^ 0xA511E9B3u) >> 8) * (1.0f / 16777216.0f);
  return u < sigmoidf(margin_true) ? 1.0f : 0.0f;
}

// ---------------------------------------------------------------------------
// "Transpose" reduction of U per-row partial sums over the LPR lanes of a row group.
// A butterfly would cost U*log2(LPR) cross-lane ops; recursive halving costs
// U/2 + U/4 + ... + (remaining butterfly) -- for LPR=32, U=8: 9 instead of 40 -- and
// leaves every lane with the COMPLETE sums of NF = U >> H consecutive rows
// (H = min(log2 U, log2 LPR)), so the per-row epilogue (sigmoid, loss) runs once per
// row instead of once per lane-row.
constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x / 2); }

template <int LPR, int U>
struct RowReduce {
  static constexpr int LL = ilog2(LPR), LU = ilog2(U);
  static constexpr int H = LL < LU ? LL : LU;   // halving steps
  static constexpr int NF = U >> H;             // rows finished per lane
  // first row index owned by group-lane c
  __device__ static __forceinline__ int base(int c) {
    int b = 0;
#pragma unroll
    for (int s = 0; s < H; ++s) b += ((c >> (LL - 1 - s)) & 1) * (U >> (s + 1));
    return b;
  }
  // group-lane holding row u (lower, butterflied bits zero)
  __host__ __device__ static constexpr int owner(int u) {
    int c = 0;
    for (int s = 0; s < H; ++s) c += (((u - u % NF) >> (LU - 1 - s)) & 1) << (LL - 1 - s);
    return c;
  }
  // true for exactly one lane per finished row
  __device__ static __forceinline__ bool representative(int c) {
    return (c & ((1 << (LL - H)) - 1)) == 0;
  }
  __device__ static __forceinline__ void run(float (&v)[U], int c) {
    int n = U;
#pragma unroll
    for (int s = 0; s < LL; ++s) {
      const int off = LPR >> (s + 1);
      if (s < H) {
        const bool up = (c & off) != 0;
        n >>= 1;
#pragma unroll
        for (int j = 0; j < U / 2; ++j) {
          if (j < n) {
            const float keep = up ? v[j + n] : v[j];
            const float send = up ? v[j] : v[j + n];
            v[j] = keep + __shfl_xor(send, off, kWave);
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < NF; ++j) v[j] += __shfl_xor(v[j], off, kWave);
      }
    }
  }
};

template <int LPR, int CPL, int UNROLL, int LOSS, int SRC>
__global__ __launch_bounds__(kBlock) void glm_grad_kernel(
    const uint16_t* __restrict__ X, int64_t ld, int64_t n, const float* __restrict__ y,
    const float* __restrict__ sw, const float* __restrict__ coef, const float* __restrict__ bptr,
    uint32_t seed, int64_t row0, const float* __restrict__ wtrue, float btrue,
    float* __restrict__ partial, int pstride) {
  constexpr int G = kWave / LPR;             // rows per wave-instruction
  constexpr int RT = G * UNROLL;             // rows per wave tile
  constexpr int DP = LPR * CPL * 8;          // padded feature count
  using RR = RowReduce<LPR, UNROLL>;
  constexpr int NF = RR::NF;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int g = lane / LPR, c = lane % LPR;
  const int nch = (int)(ld / 8);
  const int ubase = RR::base(c);
  const bool rep = RR::representative(c);
  // read from device memory so a device-side optimizer step never syncs the host
  const float intercept = *bptr;

  // SRC == 1 works on raw bytes b (x = b*kSynthScale + kSynthShift): the weights are
  // pre-scaled by kSynthScale and each lane's dot products start from the shift term
  // kSynthShift * sum(w over its columns); X^T r accumulates r*b/128 plus a per-lane
  // residual sum rs, corrected once at the end.
  float w[CPL][8], wt[CPL][8], acc[CPL][8];
  float wshift = 0.f, wtshift = 0.f, rs = 0.f;
#pragma unroll
  for (int k = 0; k < CPL; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = 8 * (c + k * LPR) + j;
      const float wv = col < ld ? coef[col] : 0.f;
      const float wtv = (SRC == 1 && col < ld) ? wtrue[col] : 0.f;
      w[k][j] = SRC == 1 ? wv * kSynthScale : wv;
      wt[k][j] = wtv * kSynthScale;
      wshift += wv;
      wtshift += wtv;
      acc[k][j] = 0.f;
    }
  wshift *= kSynthShift;
  wtshift *= kSynthShift;
  float acc_r = 0.f, acc_loss = 0.f, acc_w = 0.f;

  const int64_t ntiles = (n + RT - 1) / RT;
  const int64_t gw = (int64_t)blockIdx.x * kWavesPerBlock + wid;
  const int64_t nw = (int64_t)gridDim.x * kWavesPerBlock;
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t base = t * RT;
    // Loads are issued unconditionally from clamped addresses and masked in
    // registers afterwards: a per-load `ok ? load : 0` makes hipcc branch around
    // every load and serialise them (CDNA guide §5, "three .s-level traps" (c)).
    // SRC == 1: rows past n are harmless (their residual is masked to 0) and columns
    // past ld meet zero weights and are never written out, so no masking is needed.
    short8 xv[UNROLL][CPL];
    float xf[UNROLL][CPL][8];          // SRC == 1: decoded once, reused by dot and X^T r
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t row = base + u * G + g;
      const bool ok = row < n;
      const int64_t rowc = ok ? row : n - 1;
      const uint32_t rk = SRC == 1 ? feat_key(seed, row0 + row) : 0u;
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const int ch = c + k * LPR;
        if (SRC == 0) {
          const bool okc = ok && ch < nch;
          const int chc = ch < nch ? ch : nch - 1;
          short8 v = __builtin_nontemporal_load(reinterpret_cast<const short8*>(X + rowc * ld + 8 * chc));
          xv[u][k] = okc ? v : short8{0, 0, 0, 0, 0, 0, 0, 0};
        } else {
          const uint32_t h0 = synth_word(rk, 2 * ch), h1 = synth_word(rk, 2 * ch + 1);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            xf[u][k][j] = synth_byte(h0, j);
            xf[u][k][4 + j] = synth_byte(h1, j);
          }
        }
      }
    }
    // labels / weights of the rows this lane finishes
    float yy[NF], ww[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int64_t row = base + (ubase + j) * G + g;
      const bool ok = row < n;
      const int64_t rowc = ok ? row : n - 1;
      if (SRC == 0) {
        const float yv = y[rowc];
        const float wv = sw ? sw[rowc] : 1.f;
        yy[j] = ok ? yv : 0.f;
        ww[j] = ok ? wv : 0.f;
      } else {
        ww[j] = ok ? 1.f : 0.f;
      }
    }
    float dot[UNROLL], dtrue[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      float d = SRC == 1 ? wshift : 0.f, dt = wtshift;
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        float x[8];
        if (SRC == 0) {
          unpack8(xv[u][k], x);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = xf[u][k][j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          d = fmaf(x[j], w[k][j], d);
          if (SRC == 1) dt = fmaf(x[j], wt[k][j], dt);
        }
      }
      dot[u] = d;
      dtrue[u] = dt;
    }
    RR::run(dot, c);
    if (SRC == 1) {
      RR::run(dtrue, c);
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const int64_t row = base + (ubase + j) * G + g;
        yy[j] = synth_label(row_key(seed, row0 + row), dtrue[j] + btrue);
      }
    }
    float res[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const float m = dot[j] + intercept;
      float r, l;
      if (LOSS == LOSS_LOGISTIC) {
        const float e = __expf(-fabsf(m));
        const float inv = __builtin_amdgcn_rcpf(1.0f + e);
        const float p = m >= 0.f ? inv : e * inv;   // sigmoid(m)
        r = (p - yy[j]) * ww[j];
        l = ww[j] * (fmaxf(m, 0.f) + __logf(1.0f + e) - yy[j] * m);
      } else if (LOSS == LOSS_HINGE) {
        const float s = 2.f * yy[j] - 1.f;
        const float mg = 1.f - s * m;
        r = mg > 0.f ? -s * ww[j] : 0.f;
        l = mg > 0.f ? ww[j] * mg : 0.f;
      } else {
        const float e = m - yy[j];
        r = e * ww[j];
        l = 0.5f * ww[j] * e * e;
      }
      res[j] = r;
      if (rep) { acc_r += r; acc_loss += l; acc_w += ww[j]; }
    }
    // Re-unpack from the packed registers for X^T r instead of keeping 8*UNROLL*CPL
    // unpacked floats live across the reduction (halves the VGPR footprint).
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        if (SRC == 0) asm volatile("" : "+v"(xv[u][k]));
        else {
#pragma unroll
          for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(xf[u][k][j]));
        }
      }
    // broadcast each row's residual back to its LPR lanes, accumulate X^T r
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      float r = __shfl(res[u % NF], g * LPR + RR::owner(u), kWave);
      if (SRC == 1) { rs += r; r *= kSynthScale; }
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        float x[8];
        if (SRC == 0) {
          unpack8(xv[u][k], x);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = xf[u][k][j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[k][j] = fmaf(r, x[j], acc[k][j]);
      }
    }
  }

  if (SRC == 1) {
#pragma unroll
    for (int k = 0; k < CPL; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[k][j] = fmaf(rs, kSynthShift, acc[k][j]);
  }
  // Sum the G row groups of the wave (lanes c, c+LPR, ...), then the 4 waves via LDS.
#pragma unroll
  for (int k = 0; k < CPL; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = acc[k][j];
#pragma unroll
      for (int off = LPR; off < kWave; off <<= 1) v += __shfl_xor(v, off, kWave);
      acc[k][j] = v;
    }
  acc_r = wave_sum(acc_r);
  acc_loss = wave_sum(acc_loss);
  acc_w = wave_sum(acc_w);

  __shared__ float red[kWavesPerBlock][DP + 4];
  if (lane < LPR) {
#pragma unroll
    for (int k = 0; k < CPL; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[wid][8 * (c + k * LPR) + j] = acc[k][j];
  }
  if (lane == 0) {
    red[wid][DP] = acc_r;
    red[wid][DP + 1] = acc_loss;
    red[wid][DP + 2] = acc_w;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < DP + 3; i += kBlock) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < kWavesPerBlock; ++q) s += red[q][i];
    partial[(int64_t)blockIdx.x * pstride + i] = s;
  }
}

// ---------------------------------------------------------------------------
// Mixed pass: resident rows (HBM stream, memory bound) and lineage rows (regenerated
// in-kernel, VALU bound) in ONE launch.  Two back-to-back or two-stream launches leave
// one resource idle (the first grid fills every CU slot, so the second kernel only
// starts as the first drains: profiles/glm_overlap.json, 63.8 ms vs 41 + 25 ms alone).
// Here every wave walks one interleaved sequence of S = Tr + Tl row tiles in which
// lineage tiles are spread evenly (Bresenham: tile s is lineage iff
// floor((s+1) Tl / S) > floor(s Tl / S)), so at any moment each CU holds a mix of
// load-bound and ALU-bound waves and both roles finish together.  Both roles use the
// same lane->column mapping (the lineage one), so they share w / acc registers.
template <int LOSS>
__device__ __forceinline__ void loss_terms(float m, float yv, float wv, float& r, float& l) {
  if (LOSS == LOSS_LOGISTIC) {
    const float e = __expf(-fabsf(m));
    const float inv = __builtin_amdgcn_rcpf(1.0f + e);
    const float p = m >= 0.f ? inv : e * inv;
    r = (p - yv) * wv;
    l = wv * (fmaxf(m, 0.f) + __logf(1.0f + e) - yv * m);
  } else if (LOSS == LOSS_HINGE) {
    const float s = 2.f * yv - 1.f;
    const float mg = 1.f - s * m;
    r = mg > 0.f ? -s * wv : 0.f;
    l = mg > 0.f ? wv * mg : 0.f;
  } else {
    const float e = m - yv;
    r = e * wv;
    l = 0.5f * wv * e * e;
  }
}

// Cross-lane sums for the LPR = 8, two-rows-per-lane layout without LDS traffic: the
// quad butterflies use quad_perm DPP, the cross-quad halving row_half_mirror (lane i <->
// 7 - i: after the quad sums every lane of a quad holds the same value, so the mirror
// partner serves as lane i ^ 4).  Leaves lanes c < 4 with row 0's sum and lanes c >= 4
// with row 1's -- the RowReduce<8, 2> layout (base(c) = c >> 2) -- in v[0].  Replaces
// three ds_bpermute round trips (and their lgkmcnt waits) per tile by five DPP adds.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF,
                                                               false));
}
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141;
__device__ __forceinline__ void row_reduce_8x2(float (&v)[2], int c) {
  v[0] += dpp_f<kDppXor1>(v[0]);
  v[1] += dpp_f<kDppXor1>(v[1]);
  v[0] += dpp_f<kDppXor2>(v[0]);
  v[1] += dpp_f<kDppXor2>(v[1]);
  const bool up = (c & 4) != 0;
  const float keep = up ? v[1] : v[0], send = up ? v[0] : v[1];
  v[0] = keep + dpp_f<kDppHalfMirror>(send);
}

// One tile of RT rows.  SRC 0: rows of X (bf16 in HBM); SRC 1: rows regenerated from
// their lineage (raw bytes b, x = b*kSynthScale + kSynthShift, the affine map folded into
// the dot product and a per-lane residual sum rs).  Labels / weights of both roles come
// from the materialised label column (y, sw already offset to the role's first row).
// Mini-batch sampling (miniBatchFraction < 1, mllib GradientDescent's per-iteration
// `data.sample(false, fraction, seed + i)`): row r of iteration t is kept iff
// row_key(sample_key(seed, t), global r) >> 8 < fraction * 2^24.  The mask only zeroes a
// row's weight (its residual, loss and weight-sum terms), so it costs one hash per row,
// needs no compaction pass, and the kept set is independent of the sharding.
struct RowSampler {
  uint32_t key, thr;   // thr >= 2^24: every row kept (sampling off)
  int64_t grow0;       // global index of the role's row 0
  __device__ __forceinline__ bool on() const { return thr < (1u << 24); }
  __device__ __forceinline__ bool keep(int64_t row) const { return (row_key(key, grow0 + row) >> 8) < thr; }
};
__host__ __device__ __forceinline__ uint32_t sample_key(uint32_t seed, uint32_t iter) {
  return fmix32(seed ^ fmix32(iter * 0x9E3779B1u + 0x7F4A7C15u));
}

template <int LPR, int CPL, int UNROLL, int LOSS, int SRC, bool SMP>
__device__ __forceinline__ void mixed_tile(
    int64_t base, int64_t n, const uint16_t* __restrict__ X, int64_t ld, int nch,
    const float* __restrict__ y, const float* __restrict__ sw, uint32_t seed, int64_t row0,
    const float (&w)[CPL][8], float wshift, float intercept, int g, int c, const RowSampler smp,
    float (&acc)[CPL][8], float& rs, float& acc_r, float& acc_loss, float& acc_w) {
  constexpr int G = kWave / LPR;
  using RR = RowReduce<LPR, UNROLL>;
  constexpr int NF = RR::NF;
  const int ubase = RR::base(c);
  const bool rep = RR::representative(c);
  short8 xv[UNROLL][CPL];
  float xf[UNROLL][CPL][8];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t row = base + u * G + g;
    const bool ok = row < n;
    const int64_t rowc = ok ? row : n - 1;
    if (SRC == 0) {
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const int ch = c + k * LPR;
        const int chc = ch < nch ? ch : nch - 1;
        short8 v = __builtin_nontemporal_load(reinterpret_cast<const short8*>(X + rowc * ld + 8 * chc));
        xv[u][k] = (ok && ch < nch) ? v : short8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    } else {
      const uint32_t rk = feat_key(seed, row0 + row);
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const int ch = c + k * LPR;
        const uint32_t h0 = synth_word(rk, 2 * ch), h1 = synth_word(rk, 2 * ch + 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          xf[u][k][j] = synth_byte(h0, j);
          xf[u][k][4 + j] = synth_byte(h1, j);
        }
      }
    }
  }
  float yy[NF], ww[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int64_t row = base + (ubase + j) * G + g;
    const bool ok = row < n;
    const int64_t rowc = ok ? row : n - 1;
    const float yv = y[rowc];
    const float wv = sw ? sw[rowc] : 1.f;
    yy[j] = ok ? yv : 0.f;
    ww[j] = ok ? wv : 0.f;
    if constexpr (SMP) {
      if (!smp.keep(row)) ww[j] = 0.f;
    }
  }
  float dot[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    // two interleaved partial sums -> v_pk_fma_f32 (one issue per two features)
    float2_ d2 = {0.f, 0.f};
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      float x[8];
      if (SRC == 0) unpack8(xv[u][k], x);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = xf[u][k][j];
      }
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const float2_ xx = {x[j], x[j + 1]}, ww2 = {w[k][j], w[k][j + 1]};
        d2 = __builtin_elementwise_fma(xx, ww2, d2);
      }
    }
    const float d = d2.x + d2.y;
    dot[u] = SRC == 1 ? fmaf(d, kSynthScale, wshift) : d;
  }
  constexpr bool kDpp = LPR == 8 && UNROLL == 2;
  if constexpr (kDpp) row_reduce_8x2(dot, c);
  else RR::run(dot, c);
  float res[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    float r, l;
    loss_terms<LOSS>(dot[j] + intercept, yy[j], ww[j], r, l);
    res[j] = r;
    if (rep) { acc_r += r; acc_loss += l; acc_w += ww[j]; }
  }
#pragma unroll
  for (int u = 0; u < UNROLL; ++u)
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      if (SRC == 0) asm volatile("" : "+v"(xv[u][k]));
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(xf[u][k][j]));
      }
    }
  float other = 0.f;
  if constexpr (kDpp) other = dpp_f<kDppHalfMirror>(res[0]);   // the other row's residual
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    float r;
    if constexpr (kDpp) r = ((c & 4) != 0) == (u == 0) ? other : res[0];
    else r = __shfl(res[u % NF], g * LPR + RR::owner(u), kWave);
    if (SRC == 1) { rs += r; r *= kSynthScale; }
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      float x[8];
      if (SRC == 0) unpack8(xv[u][k], x);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = xf[u][k][j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[k][j] = fmaf(r, x[j], acc[k][j]);
    }
  }
}

// y / sw hold n_res + n_lin entries: the resident rows' labels, then the lineage rows'.
// MW: minimum waves per SIMD the register allocator must allow (2 = no constraint at
// D = 256, 174 VGPRs; 3 = 168 VGPRs with a 4-register spill outside the tile loop).
// Every wave walks the interleaved tile sequence (both roles per wave; fixed-role layouts
// -- some waves regenerating, the others streaming -- measured slower and were removed).
template <int LPR, int CPL, int UNROLL, int LOSS, int MW, bool SMP>
__global__ __launch_bounds__(kBlock, MW) void glm_grad_mixed_kernel(
    const uint16_t* __restrict__ X, int64_t ld, int64_t n_res, const float* __restrict__ y,
    const float* __restrict__ sw, const float* __restrict__ y_lin, const float* __restrict__ sw_lin,
    const float* __restrict__ coef, const float* __restrict__ bptr, uint32_t seed, int64_t row0, int64_t n_lin,
    float* __restrict__ partial, int pstride, int64_t res_row0, const int64_t* __restrict__ t_dev, uint32_t sseed,
    uint32_t sthr, int pacc) {
  constexpr int G = kWave / LPR;
  constexpr int RT = G * UNROLL;
  constexpr int DP = LPR * CPL * 8;
  using RR = RowReduce<LPR, UNROLL>;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int g = lane / LPR, c = lane % LPR;
  const int nch = (int)(ld / 8);
  const float intercept = *bptr;
  // iteration t of a device-side SGD loop = t_dev + 1 (the update kernel advances it)
  // (SMP = false: the sampler is compiled out -- no hash, no extra registers)
  const uint32_t skey = SMP ? sample_key(sseed, (uint32_t)((t_dev ? t_dev[0] : 0) + 1)) : 0u;
  const RowSampler smp_res{skey, sthr, res_row0}, smp_lin{skey, sthr, row0};

  float w[CPL][8], acc[CPL][8];
  float wshift = 0.f, rs = 0.f;
#pragma unroll
  for (int k = 0; k < CPL; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = 8 * (c + k * LPR) + j;
      w[k][j] = col < ld ? coef[col] : 0.f;
      wshift += w[k][j];
      acc[k][j] = 0.f;
    }
  wshift *= kSynthShift;
  float acc_r = 0.f, acc_loss = 0.f, acc_w = 0.f;

  const int64_t Tr = (n_res + RT - 1) / RT, Tl = (n_lin + RT - 1) / RT, S = Tr + Tl;
  const int64_t gw = (int64_t)blockIdx.x * kWavesPerBlock + wid;
  const int64_t nw = (int64_t)gridDim.x * kWavesPerBlock;
  if (gw < S) {
    // lineage tiles before unit s: L = floor(s Tl / S), rem = s Tl mod S (s Tl < 2^62)
    int64_t L = gw * Tl / S, rem = gw * Tl - L * S;
    const int64_t q0 = nw * Tl / S, r0 = nw * Tl - q0 * S;
    for (int64_t s = gw; s < S; s += nw) {
      if (rem + Tl >= S)
        mixed_tile<LPR, CPL, UNROLL, LOSS, 1, SMP>(L * RT, n_lin, X, ld, nch, y_lin, sw_lin, seed, row0, w,
                                              wshift, intercept, g, c, smp_lin, acc, rs, acc_r, acc_loss,
                                              acc_w);
      else
        mixed_tile<LPR, CPL, UNROLL, LOSS, 0, SMP>((s - L) * RT, n_res, X, ld, nch, y, sw, seed, row0, w,
                                              wshift, intercept, g, c, smp_res, acc, rs, acc_r, acc_loss,
                                              acc_w);
      rem += r0;
      L += q0;
      if (rem >= S) { rem -= S; ++L; }
    }
  }
#pragma unroll
  for (int k = 0; k < CPL; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = fmaf(rs, kSynthShift, acc[k][j]);
#pragma unroll
      for (int off = LPR; off < kWave; off <<= 1) v += __shfl_xor(v, off, kWave);
      acc[k][j] = v;
    }
  acc_r = wave_sum(acc_r);
  acc_loss = wave_sum(acc_loss);
  acc_w = wave_sum(acc_w);
  __shared__ float red[kWavesPerBlock][DP + 4];
  if (lane < LPR) {
#pragma unroll
    for (int k = 0; k < CPL; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[wid][8 * (c + k * LPR) + j] = acc[k][j];
  }
  if (lane == 0) {
    red[wid][DP] = acc_r;
    red[wid][DP + 1] = acc_loss;
    red[wid][DP + 2] = acc_w;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < DP + 3; i += kBlock) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < kWavesPerBlock; ++q) s += red[q][i];
    float* const pp = partial + (int64_t)blockIdx.x * pstride + i;
    *pp = pacc ? *pp + s : s;           // pacc: later slices of a split pass add in
  }
}

// ---------------------------------------------------------------------------
// Summarizer pass of a gradient-descent fit, fused with its first gradient: per column
// s1 = sum w x, s2 = sum w x^2 and syx = sum w y x, per row sum w, sum w y, sum w y^2,
// over the resident rows of X and n_lin lineage rows in ONE interleaved launch (same
// tile schedule as glm_grad_mixed_kernel).  At the initial iterate every coefficient is
// zero, so each row's margin is the intercept b0 and the step-1 gradient of every loss
// is a combination of s1 and syx (logistic: sigmoid(b0) s1 - syx) -- the fit's first
// step needs no pass of its own (models/glm.py: DeviceSGD.first_step_from_stats).
// UNW: a full tile (every row < n) of an unweighted fit -- w = 1 is folded away, which
// drops the w*x product from every element (the pass is VALU-bound on lineage tiles).
template <int LPR, int CPL, int SRC, bool UNW>
__device__ __forceinline__ void stats_tile(int64_t base, int64_t n, const uint16_t* __restrict__ X, int64_t ld,
                                           int nch, const float* __restrict__ y, const float* __restrict__ sw,
                                           uint32_t seed, int64_t row0, int g, int c, float2_ (&s1)[CPL][4],
                                           float2_ (&s2)[CPL][4], float2_ (&syx)[CPL][4], float (&rsum)[3]) {
  constexpr int G = kWave / LPR;
  constexpr int U = CPL >= 8 ? 1 : 8 / CPL;
  short8 xv[U][CPL];
  uint32_t fk[U];
  float yv[U], wv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t row = base + u * G + g;
    const bool ok = row < n;
    const int64_t rowc = ok ? row : n - 1;
    yv[u] = y[rowc];
    if (UNW) {
      wv[u] = 1.f;
    } else {
      const float w0 = sw ? sw[rowc] : 1.f;
      wv[u] = ok ? w0 : 0.f;
    }
    if (SRC == 0) {
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const int ch = c + k * LPR;
        const int chc = ch < nch ? ch : nch - 1;
        short8 v = __builtin_nontemporal_load(reinterpret_cast<const short8*>(X + rowc * ld + 8 * chc));
        xv[u][k] = ch < nch ? v : short8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    } else {
      fk[u] = feat_key(seed, row0 + rowc);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const float2_ w2 = {wv[u], wv[u]};
    const float wy = wv[u] * yv[u];
    const float2_ wy2 = {wy, wy};
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      float x[8];
      if (SRC == 0) {
        unpack8(xv[u][k], x);
      } else {
        // lineage rows: the feature bytes straight from the hash (x = b/128 - 255/256 is
        // exact), no bf16 round trip
        const int ch = c + k * LPR;
        const uint32_t h0 = synth_word(fk[u], 2 * ch), h1 = synth_word(fk[u], 2 * ch + 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          x[j] = fmaf(synth_byte(h0, j), kSynthScale, kSynthShift);
          x[4 + j] = fmaf(synth_byte(h1, j), kSynthScale, kSynthShift);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float2_ xx = {x[2 * j], x[2 * j + 1]};
        const float2_ wx = UNW ? xx : w2 * xx;
        s1[k][j] += wx;
        s2[k][j] = __builtin_elementwise_fma(wx, xx, s2[k][j]);
        syx[k][j] = __builtin_elementwise_fma(wy2, xx, syx[k][j]);
      }
    }
    if (c == 0) {
      rsum[0] += wv[u];
      rsum[1] += wy;
      rsum[2] = fmaf(wy, yv[u], rsum[2]);
    }
  }
}

template <int LPR, int CPL, int MW>
__global__ __launch_bounds__(kBlock, MW) void glm_stats_mixed_kernel(
    const uint16_t* __restrict__ X, int64_t ld, int64_t n_res, const float* __restrict__ y,
    const float* __restrict__ sw, uint32_t seed, int64_t row0, int64_t n_lin, float* __restrict__ partial,
    int pstride) {
  constexpr int G = kWave / LPR;
  constexpr int U = CPL >= 8 ? 1 : 8 / CPL;
  constexpr int RT = G * U;
  constexpr int DP = LPR * CPL * 8;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int g = lane / LPR, c = lane % LPR;
  const int nch = (int)(ld / 8);
  const float* y_lin = y + n_res;
  const float* sw_lin = sw ? sw + n_res : nullptr;
  float2_ s1[CPL][4], s2[CPL][4], syx[CPL][4];
#pragma unroll
  for (int k = 0; k < CPL; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) s1[k][j] = s2[k][j] = syx[k][j] = float2_{0.f, 0.f};
  float rsum[3] = {0.f, 0.f, 0.f};
  const int64_t Tr = (n_res + RT - 1) / RT, Tl = (n_lin + RT - 1) / RT, S = Tr + Tl;
  const int64_t gw = (int64_t)blockIdx.x * kWavesPerBlock + wid;
  const int64_t nw = (int64_t)gridDim.x * kWavesPerBlock;
  if (gw < S) {
    int64_t L = gw * Tl / S, rem = gw * Tl - L * S;
    const int64_t q0 = nw * Tl / S, r0 = nw * Tl - q0 * S;
    for (int64_t s = gw; s < S; s += nw) {
      if (rem + Tl >= S) {
        const int64_t base = L * RT;
        if (sw == nullptr && base + RT <= n_lin)
          stats_tile<LPR, CPL, 1, true>(base, n_lin, X, ld, nch, y_lin, sw_lin, seed, row0, g, c, s1, s2, syx, rsum);
        else
          stats_tile<LPR, CPL, 1, false>(base, n_lin, X, ld, nch, y_lin, sw_lin, seed, row0, g, c, s1, s2, syx, rsum);
      } else {
        const int64_t base = (s - L) * RT;
        if (sw == nullptr && base + RT <= n_res)
          stats_tile<LPR, CPL, 0, true>(base, n_res, X, ld, nch, y, sw, seed, row0, g, c, s1, s2, syx, rsum);
        else
          stats_tile<LPR, CPL, 0, false>(base, n_res, X, ld, nch, y, sw, seed, row0, g, c, s1, s2, syx, rsum);
      }
      rem += r0;
      L += q0;
      if (rem >= S) { rem -= S; ++L; }
    }
  }
  // fold the G row groups of the wave, then the waves through LDS in a fixed order
  __shared__ float red[kWavesPerBlock][3 * DP + 4];
#pragma unroll
  for (int k = 0; k < CPL; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float a = s1[k][j][h], b = s2[k][j][h], e = syx[k][j][h];
#pragma unroll
        for (int off = LPR; off < kWave; off <<= 1) {
          a += __shfl_xor(a, off, kWave);
          b += __shfl_xor(b, off, kWave);
          e += __shfl_xor(e, off, kWave);
        }
        const int col = 8 * (c + k * LPR) + 2 * j + h;
        if (lane < LPR) {
          red[wid][col] = a;
          red[wid][DP + col] = b;
          red[wid][2 * DP + col] = e;
        }
      }
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const float v = wave_sum(rsum[q]);
    if (lane == 0) red[wid][3 * DP + q] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * DP + 3; i += kBlock) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < kWavesPerBlock; ++q) s += red[q][i];
    partial[(int64_t)blockIdx.x * pstride + i] = s;
  }
}

// Materialise synthetic rows [row0, row0+n) into X (bf16) and labels y.
template <int LPR, int CPL>
__global__ __launch_bounds__(kBlock) void synth_glm_kernel(
    uint16_t* __restrict__ X, int64_t ld, int64_t n, float* __restrict__ y, uint32_t seed,
    int64_t row0, const float* __restrict__ wtrue, float btrue) {
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, c = lane % LPR;
  float wt[CPL][8];
#pragma unroll
  for (int k = 0; k < CPL; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = 8 * (c + k * LPR) + j;
      wt[k][j] = col < ld ? wtrue[col] : 0.f;
    }
  const int64_t gw = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) / kWave;
  const int64_t ntiles = (n + G - 1) / G;
  for (int64_t t = gw; t < ntiles; t += nw) {
    const int64_t row = t * G + g;
    const bool ok = row < n;
    const uint32_t rk = row_key(seed, row0 + row), fk = feat_key(seed, row0 + row);
    float dt = 0.f;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const int ch = c + k * LPR;
      if (8 * ch < ld) {
        short8 v = synth_chunk(fk, ch);
        float x[8];
        unpack8(v, x);
#pragma unroll
        for (int j = 0; j < 8; ++j) dt = fmaf(x[j], wt[k][j], dt);
        if (ok) *reinterpret_cast<short8*>(X + row * ld + 8 * ch) = v;
      }
    }
    dt = group_sum<LPR>(dt);
    if (ok && c == 0) y[row] = synth_label(rk, dt + btrue);
  }
}

// margins[i] = x_i . coef + intercept (model.transform / predict path).
template <int LPR, int CPL>
__global__ __launch_bounds__(kBlock) void glm_margin_kernel(
    const uint16_t* __restrict__ X, int64_t ld, int64_t n, const float* __restrict__ coef,
    float intercept, float* __restrict__ out) {
  constexpr int G = kWave / LPR;
  constexpr int UNROLL = CPL >= 8 ? 1 : 8 / CPL;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, c = lane % LPR;
  const int nch = (int)(ld / 8);
  float w[CPL][8];
#pragma unroll
  for (int k = 0; k < CPL; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = 8 * (c + k * LPR) + j;
      w[k][j] = col < ld ? coef[col] : 0.f;
    }
  const int64_t gw = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) / kWave;
  const int64_t RT = (int64_t)G * UNROLL;
  const int64_t ntiles = (n + RT - 1) / RT;
  for (int64_t t = gw; t < ntiles; t += nw) {
    short8 xv[UNROLL][CPL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t row = t * RT + u * G + g;
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const int ch = c + k * LPR;
        xv[u][k] = (row < n && ch < nch)
                       ? *reinterpret_cast<const short8*>(X + row * ld + 8 * ch)
                       : short8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t row = t * RT + u * G + g;
      float d = 0.f;
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        float x[8];
        unpack8(xv[u][k], x);
#pragma unroll
        for (int j = 0; j < 8; ++j) d = fmaf(x[j], w[k][j], d);
      }
      d = group_sum<LPR>(d);
      if (row < n && c == 0) out[row] = d + intercept;
    }
  }
}

// Weighted column moments (Spark's MultivariateOnlineSummarizer subset used by the
// GLM solvers for standardization): per column sum(w*x), sum(w*x^2), plus sum(w).
// Same lane layout as the gradient pass; one slab row per block, fp64 finish.
template <int LPR, int CPL, int SRC>
__global__ __launch_bounds__(kBlock) void glm_colstats_kernel(
    const uint16_t* __restrict__ X, int64_t ld, int64_t n, const float* __restrict__ sw,
    uint32_t seed, int64_t row0, float* __restrict__ partial, int pstride) {
  constexpr int G = kWave / LPR;
  constexpr int UNROLL = CPL >= 4 ? 1 : 4 / CPL;
  constexpr int DP = LPR * CPL * 8;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int g = lane / LPR, c = lane % LPR;
  const int nch = (int)(ld / 8);
  float s1[CPL][8], s2[CPL][8];
#pragma unroll
  for (int k = 0; k < CPL; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) s1[k][j] = s2[k][j] = 0.f;
  float sw_acc = 0.f;
  const int64_t RT = (int64_t)G * UNROLL;
  const int64_t ntiles = (n + RT - 1) / RT;
  const int64_t gw = (int64_t)blockIdx.x * kWavesPerBlock + wid;
  const int64_t nw = (int64_t)gridDim.x * kWavesPerBlock;
  for (int64_t t = gw; t < ntiles; t += nw) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t row = t * RT + u * G + g;
      const bool ok = row < n;
      const int64_t rowc = ok ? row : n - 1;
      const float wv = sw ? sw[rowc] : 1.f;
      const float w = ok ? wv : 0.f;
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const int ch = c + k * LPR;
        const int chc = ch < nch ? ch : nch - 1;
        short8 v = SRC == 0 ? __builtin_nontemporal_load(reinterpret_cast<const short8*>(X + rowc * ld + 8 * chc))
                            : synth_chunk(feat_key(seed, row0 + rowc), chc);
        const float wk = ch < nch ? w : 0.f;
        float x[8];
        unpack8(v, x);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float wx = wk * x[j];
          s1[k][j] += wx;
          s2[k][j] = fmaf(wx, x[j], s2[k][j]);
        }
      }
      if (c == 0) sw_acc += w;
    }
  }
#pragma unroll
  for (int k = 0; k < CPL; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = s1[k][j], b = s2[k][j];
#pragma unroll
      for (int off = LPR; off < kWave; off <<= 1) {
        a += __shfl_xor(a, off, kWave);
        b += __shfl_xor(b, off, kWave);
      }
      s1[k][j] = a;
      s2[k][j] = b;
    }
  sw_acc = wave_sum(sw_acc);
  // waves add into one LDS row in turn (fixed order -> deterministic)
  __shared__ float red[2 * DP + 2];
  for (int q = 0; q < kWavesPerBlock; ++q) {
    if (wid == q) {
      if (lane < LPR) {
#pragma unroll
        for (int k = 0; k < CPL; ++k)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int i1 = 8 * (c + k * LPR) + j;
            red[i1] = (q == 0 ? 0.f : red[i1]) + s1[k][j];
            red[DP + i1] = (q == 0 ? 0.f : red[DP + i1]) + s2[k][j];
          }
      }
      if (lane == 0) red[2 * DP] = (q == 0 ? 0.f : red[2 * DP]) + sw_acc;
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < 2 * DP + 1; i += kBlock) partial[(int64_t)blockIdx.x * pstride + i] = red[i];
}

// out[i] = sum_b partial[b][i] in fp64, fixed order (deterministic).  Block = 32
// columns x 32 strided partial-row groups; each thread sums nblocks/32 rows, then the
// 32 group sums of a column are combined in LDS in a fixed order.
__global__ __launch_bounds__(1024) void glm_finish_kernel(const float* __restrict__ partial, int nblocks,
                                                          int pstride, int ncols, double* __restrict__ out,
                                                          int accumulate) {
  __shared__ double red[32][33];
  const int cx = threadIdx.x & 31, gy = threadIdx.x >> 5;
  const int i = blockIdx.x * 32 + cx;
  double s = 0.0;
  if (i < ncols)
    for (int b = gy; b < nblocks; b += 32) s += (double)partial[(int64_t)b * pstride + i];
  red[gy][cx] = s;
  __syncthreads();
  if (gy == 0 && i < ncols) {
    double t = 0.0;
#pragma unroll 8
    for (int q = 0; q < 32; ++q) t += red[q][cx];
    out[i] = accumulate ? out[i] + t : t;
  }
}

// One device-side gradient-descent step on the all-reduced pass result `out`
// (DeviceSGD): standardised coefficients bt <- bt - eta*(g/W + l2*bt), intercept
// b <- b - eta * sum(r)/W, then refresh the fp32 kernel operand coef_eff (dpad
// coefficients + intercept) and record the loss -- no host round trip per step.
__global__ __launch_bounds__(256) void glm_sgd_update_kernel(
    const double* __restrict__ out, int dpad, double* __restrict__ bt, double* __restrict__ b,
    const double* __restrict__ inv_std, const double* __restrict__ l2v, double l2, double eta,
    int fit_intercept, float* __restrict__ coef_eff, double* __restrict__ loss_slot) {
  const double W = out[dpad + 2];
  const double invW = W > 0.0 ? 1.0 / W : 0.0;
  for (int i = threadIdx.x; i < dpad; i += blockDim.x) {
    const double inv = inv_std[i];
    const double reg = l2v ? l2v[i] : l2;
    const double v = bt[i] - eta * (out[i] * inv * invW + reg * bt[i]);
    bt[i] = v;
    coef_eff[i] = (float)(v * inv);
  }
  if (threadIdx.x == 0) {
    double bv = b[0];
    if (fit_intercept) bv -= eta * out[dpad] * invW;
    b[0] = bv;
    coef_eff[dpad] = (float)bv;
    if (loss_slot) loss_slot[0] = out[dpad + 1] * invW;
  }
}

// Graph-capturable variant: the step counter lives on the device (t <- t + 1, eta =
// step_size / sqrt(t), loss recorded at loss_hist[t - 1] while t <= cap), so a captured
// step has no per-step host arguments and can be replayed from a HIP graph.  An L1 term
// (elastic net / mllib L1Updater) is applied as the proximal soft-threshold
// bt <- sign(bt) max(|bt| - eta * l1, 0) after the gradient step.
__global__ __launch_bounds__(256) void glm_sgd_update_dev_kernel(
    const double* __restrict__ out, int dpad, double* __restrict__ bt, double* __restrict__ b,
    const double* __restrict__ inv_std, const double* __restrict__ l2v, double l2, const double* __restrict__ l1v,
    double l1, double step_size, int fit_intercept, float* __restrict__ coef_eff, double* __restrict__ loss_hist,
    int64_t cap, int64_t* __restrict__ t_dev) {
  const int64_t t = t_dev[0] + 1;
  const double eta = step_size / sqrt((double)t);
  const double W = out[dpad + 2];
  const double invW = W > 0.0 ? 1.0 / W : 0.0;
  const bool prox = l1v != nullptr || l1 > 0.0;
  for (int i = threadIdx.x; i < dpad; i += blockDim.x) {
    const double inv = inv_std[i];
    const double reg = l2v ? l2v[i] : l2;
    double v = bt[i] - eta * (out[i] * inv * invW + reg * bt[i]);
    if (prox) {
      const double sh = eta * (l1v ? l1v[i] : l1);
      v = v > sh ? v - sh : (v < -sh ? v + sh : 0.0);
    }
    bt[i] = v;
    coef_eff[i] = (float)(v * inv);
  }
  __syncthreads();                       // every lane has read t_dev before it moves
  if (threadIdx.x == 0) {
    double bv = b[0];
    if (fit_intercept) bv -= eta * out[dpad] * invW;
    b[0] = bv;
    coef_eff[dpad] = (float)bv;
    if (t <= cap) loss_hist[t - 1] = out[dpad + 1] * invW;
    t_dev[0] = t;
  }
}

int pick_lpr(int nch) {
  int l = 4;
  while (l < nch && l < 64) l <<= 1;
  return l;
}
int pick_cpl(int nch) {
  if (nch <= 64) return 1;
  const int need = (nch + 63) / 64;
  int c = 2;
  while (c < need) c <<= 1;
  return c;  // 2,4,8,16 (caller checks <= 16)
}

template <int LPR, int CPL, int LOSS, int SRC>
void launch_grad(int grid, hipStream_t st, const uint16_t* X, int64_t ld, int64_t n,
                 const float* y, const float* sw, const float* coef, const float* b, uint32_t seed,
                 int64_t row0, const float* wt, float bt, float* partial, int pstride) {
  // rows in flight per lane: 8 loads for the streaming pass; the lineage pass keeps
  // fewer chunks live (its hash work, not memory latency, is the limiter)
  constexpr int UNROLL = SRC == 1 ? (CPL >= 8 ? 1 : 8 / CPL) : (CPL == 1 ? 8 : (CPL == 2 ? 2 : 1));
  hipLaunchKernelGGL((glm_grad_kernel<LPR, CPL, UNROLL, LOSS, SRC>), dim3(grid), dim3(kBlock), 0,
                     st, X, ld, n, y, sw, coef, b, seed, row0, wt, bt, partial, pstride);
}

template <int LOSS, int SRC>
int dispatch_grad(int lpr, int cpl, int grid, hipStream_t st, const uint16_t* X, int64_t ld,
                  int64_t n, const float* y, const float* sw, const float* coef, const float* b,
                  uint32_t seed, int64_t row0, const float* wt, float bt, float* partial,
                  int pstride) {
#define O3S_G(L, C)                                                                         \
  if (lpr == L && cpl == C) {                                                               \
    launch_grad<L, C, LOSS, SRC>(grid, st, X, ld, n, y, sw, coef, b, seed, row0, wt, bt,   \
                                 partial, pstride);                                         \
    return 0;                                                                               \
  }
  if constexpr (SRC == 0) {
    O3S_G(4, 1) O3S_G(8, 1) O3S_G(16, 1) O3S_G(32, 1) O3S_G(64, 1)
    O3S_G(64, 2) O3S_G(64, 4) O3S_G(64, 8) O3S_G(64, 16)
  } else {
    O3S_G(4, 1) O3S_G(8, 1) O3S_G(4, 4) O3S_G(8, 4) O3S_G(16, 4) O3S_G(32, 4)
    O3S_G(64, 4) O3S_G(64, 8) O3S_G(64, 16)
  }
#undef O3S_G
  return -1;
}

}  // namespace

// Number of fp32 slots per partial-slab row and the padded width for `ld`.
O3S_API int o3s_glm_layout(int64_t ld, int* dpad, int* pstride) {
  const int nch = (int)(ld / 8);
  const int lpr = pick_lpr(nch), cpl = pick_cpl(nch);
  if (ld % 8 != 0 || cpl > 16) return -1;
  *dpad = lpr * cpl * 8;
  *pstride = *dpad + 4;
  return 0;
}

// Gradient/loss pass.  out (fp64, dpad+3): [grad (dpad) | sum r | loss | weight sum],
// overwritten (accumulate == 0) or added to.  coef holds dpad+1 floats: the padded
// coefficients followed by the intercept.  partial must hold grid * pstride floats.
// src: 0 = X in memory, 1 = synthetic lineage.
O3S_API int o3s_glm_grad(int loss, int src, const void* X, int64_t ld, int64_t n, const float* y,
                         const float* sw, const float* coef, uint32_t seed,
                         int64_t row0, const float* wtrue, float btrue, float* partial,
                         int grid, double* out, int accumulate, hipStream_t st) {
  const int nch = (int)(ld / 8);
  const int lpr = pick_lpr(nch), cpl = pick_cpl(nch);
  if (ld % 8 != 0 || cpl > 16 || grid <= 0) return -1;
  const int dpad = lpr * cpl * 8, pstride = dpad + 4;
  const uint16_t* Xh = (const uint16_t*)X;
  int rc = -1;
  // The lineage pass is VALU bound and its per-row work (row key, cross-lane dot
  // reduction, label draw, residual broadcast) is replicated on every lane of a row,
  // so it uses 4x fewer lanes per row with 4x more columns each (same padded width).
  int lpr_s = lpr, cpl_s = cpl;
  if (cpl == 1 && lpr >= 16) { lpr_s = lpr / 4; cpl_s = 4; }
  else if (cpl == 2) { lpr_s = 32; cpl_s = 4; }
  if (n > 0) {
    if (src == 0) {
      if (loss == LOSS_LOGISTIC)
        rc = dispatch_grad<LOSS_LOGISTIC, 0>(lpr, cpl, grid, st, Xh, ld, n, y, sw, coef, coef + dpad, seed, row0, wtrue, btrue, partial, pstride);
      else if (loss == LOSS_HINGE)
        rc = dispatch_grad<LOSS_HINGE, 0>(lpr, cpl, grid, st, Xh, ld, n, y, sw, coef, coef + dpad, seed, row0, wtrue, btrue, partial, pstride);
      else
        rc = dispatch_grad<LOSS_SQUARED, 0>(lpr, cpl, grid, st, Xh, ld, n, y, sw, coef, coef + dpad, seed, row0, wtrue, btrue, partial, pstride);
    } else {
      if (loss == LOSS_LOGISTIC)
        rc = dispatch_grad<LOSS_LOGISTIC, 1>(lpr_s, cpl_s, grid, st, Xh, ld, n, y, sw, coef, coef + dpad, seed, row0, wtrue, btrue, partial, pstride);
      else if (loss == LOSS_HINGE)
        rc = dispatch_grad<LOSS_HINGE, 1>(lpr_s, cpl_s, grid, st, Xh, ld, n, y, sw, coef, coef + dpad, seed, row0, wtrue, btrue, partial, pstride);
      else
        rc = dispatch_grad<LOSS_SQUARED, 1>(lpr_s, cpl_s, grid, st, Xh, ld, n, y, sw, coef, coef + dpad, seed, row0, wtrue, btrue, partial, pstride);
    }
    if (rc != 0) return rc;
  } else {
    if (accumulate) return 0;
    hipMemsetAsync(partial, 0, sizeof(float) * pstride * (size_t)grid, st);
  }
  O3S_CHECK_LAUNCH();
  const int ncols = dpad + 3;
  hipLaunchKernelGGL(glm_finish_kernel, dim3((ncols + 31) / 32), dim3(1024), 0, st, partial, grid,
                     pstride, ncols, out, accumulate);
  O3S_CHECK_LAUNCH();
  return 0;
}

template <int L, int C, int MW, bool SMP = false>
static void launch_mixed(int loss, int grid, hipStream_t st, const uint16_t* X, int64_t ld, int64_t n_res,
                         const float* y, const float* sw, const float* y_lin, const float* sw_lin, const float* coef,
                         const float* b, uint32_t seed, int64_t row0, int64_t n_lin, float* partial, int pstride,
                         int64_t res_row0, const int64_t* t_dev, uint32_t sseed, uint32_t sthr, int pacc) {
  constexpr int U = C >= 8 ? 1 : 8 / C;
  if (loss == LOSS_LOGISTIC)
    hipLaunchKernelGGL((glm_grad_mixed_kernel<L, C, U, LOSS_LOGISTIC, MW, SMP>), dim3(grid), dim3(kBlock), 0,
                       st, X, ld, n_res, y, sw, y_lin, sw_lin, coef, b, seed, row0, n_lin, partial, pstride,
                       res_row0, t_dev, sseed, sthr, pacc);
  else if (loss == LOSS_HINGE)
    hipLaunchKernelGGL((glm_grad_mixed_kernel<L, C, U, LOSS_HINGE, MW, SMP>), dim3(grid), dim3(kBlock), 0,
                       st, X, ld, n_res, y, sw, y_lin, sw_lin, coef, b, seed, row0, n_lin, partial, pstride,
                       res_row0, t_dev, sseed, sthr, pacc);
  else
    hipLaunchKernelGGL((glm_grad_mixed_kernel<L, C, U, LOSS_SQUARED, MW, SMP>), dim3(grid), dim3(kBlock), 0,
                       st, X, ld, n_res, y, sw, y_lin, sw_lin, coef, b, seed, row0, n_lin, partial, pstride,
                       res_row0, t_dev, sseed, sthr, pacc);
}

// Mixed resident + lineage pass in one launch (see glm_grad_mixed_kernel): n_res rows
// of X plus n_lin synthetic rows starting at global row row0; y / sw cover all
// n_res + n_lin rows.  Same out / coef / partial
// contract as o3s_glm_grad (out is overwritten).  waves: 3 asks the register allocator
// for 3 waves/SIMD (see glm_grad_mixed_kernel), anything else 2.  Mini-batch sampling: res_row0 is the global
// index of resident row 0, t_dev (may be null = iteration 1) the device step counter,
// sthr = fraction * 2^24 (>= 2^24: no sampling), sseed the sampling seed.
O3S_API int o3s_glm_grad_mixed(int loss, const void* X, int64_t ld, int64_t n_res, const float* y,
                               const float* sw, const float* coef, uint32_t seed, int64_t row0,
                               int64_t n_lin, float* partial, int grid, double* out, int waves,
                               int64_t res_row0, const int64_t* t_dev, uint32_t sseed,
                               uint32_t sthr, int splits, hipStream_t st) {
  const int nch = (int)(ld / 8);
  const int lpr = pick_lpr(nch), cpl = pick_cpl(nch);
  if (ld % 8 != 0 || cpl > 16 || grid <= 0 || n_res < 0 || n_lin < 0) return -1;
  const int dpad = lpr * cpl * 8, pstride = dpad + 4;
  int lpr_s = lpr, cpl_s = cpl;
  if (cpl == 1 && lpr >= 16) { lpr_s = lpr / 4; cpl_s = 4; }
  else if (cpl == 2) { lpr_s = 32; cpl_s = 4; }
  const uint16_t* Xh = (const uint16_t*)X;
  const float* b = coef + dpad;
  const bool smp = sthr < (1u << 24);
#define O3S_MX(L, C)                                                                                  \
  if (!done && lpr_s == L && cpl_s == C) {                                                            \
    done = true;                                                                                      \
    if (waves == 3 && smp)                                                                            \
      launch_mixed<L, C, 3, true>(loss, grid, st, XS, ld, NR, YR, SWR, YL, SWL, coef, b, seed, RL0, NL, PS,     \
                                  pstride, RR0, t_dev, sseed, sthr, k > 0);                                     \
    else if (waves == 3)                                                                              \
      launch_mixed<L, C, 3>(loss, grid, st, XS, ld, NR, YR, SWR, YL, SWL, coef, b, seed, RL0, NL, PS, pstride,  \
                            RR0, t_dev, sseed, sthr, k > 0);                                                    \
    else if (smp)                                                                                     \
      launch_mixed<L, C, 2, true>(loss, grid, st, XS, ld, NR, YR, SWR, YL, SWL, coef, b, seed, RL0, NL, PS,     \
                                  pstride, RR0, t_dev, sseed, sthr, k > 0);                                     \
    else                                                                                              \
      launch_mixed<L, C, 2>(loss, grid, st, XS, ld, NR, YR, SWR, YL, SWL, coef, b, seed, RL0, NL, PS, pstride,  \
                            RR0, t_dev, sseed, sthr, k > 0);                                                    \
  }
  // splits > 1: the pass runs as that many launches over consecutive 1/splits slices of
  // the resident and of the lineage rows; later slices add their block sums into the
  // first slice's slabs (slice order fixed: as deterministic as one launch).  A
  // grid-stride tile walk drifts over a long launch -- waves that started together end up
  // gigabytes apart, so the resident stream touches a wider address window; restarting
  // the walk every 1/splits of a 255 GB table measured 44.2 -> 43.7 ms even with a finish
  // per slice (tools/bench_glm_split_ab.py).
  const int K = splits < 1 ? 1 : splits;
  for (int k = 0; k < K; ++k) {
    const int64_t r_lo = n_res * k / K, r_hi = n_res * (k + 1) / K;
    const int64_t l_lo = n_lin * k / K, l_hi = n_lin * (k + 1) / K;
    const uint16_t* XS = Xh + r_lo * ld;
    const int64_t NR = r_hi - r_lo, NL = l_hi - l_lo, RL0 = row0 + l_lo, RR0 = res_row0 + r_lo;
    const float* YR = y + r_lo;
    const float* SWR = sw ? sw + r_lo : nullptr;
    const float* YL = y + n_res + l_lo;
    const float* SWL = sw ? sw + n_res + l_lo : nullptr;
    float* PS = partial;                 // slices after the first add into the same slabs
    bool done = false;
    O3S_MX(4, 1) O3S_MX(8, 1) O3S_MX(4, 4) O3S_MX(8, 4) O3S_MX(16, 4) O3S_MX(32, 4)
    O3S_MX(64, 4) O3S_MX(64, 8) O3S_MX(64, 16)
    if (!done) return -1;
    O3S_CHECK_LAUNCH();
  }
#undef O3S_MX
  const int ncols = dpad + 3;
  hipLaunchKernelGGL(glm_finish_kernel, dim3((ncols + 31) / 32), dim3(1024), 0, st, partial, grid,
                     pstride, ncols, out, 0);
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_API int o3s_synth_glm(void* X, int64_t ld, int64_t n, float* y, uint32_t seed, int64_t row0,
                          const float* wtrue, float btrue, int grid, hipStream_t st) {
  const int nch = (int)(ld / 8);
  const int lpr = pick_lpr(nch), cpl = pick_cpl(nch);
  if (ld % 8 != 0 || cpl > 16) return -1;
  if (n <= 0) return 0;
  uint16_t* Xh = (uint16_t*)X;
#define O3S_S(L, C)                                                                           \
  if (lpr == L && cpl == C) {                                                                 \
    hipLaunchKernelGGL((synth_glm_kernel<L, C>), dim3(grid), dim3(kBlock), 0, st, Xh, ld, n, y, \
                       seed, row0, wtrue, btrue);                                             \
    O3S_CHECK_LAUNCH();                                                                       \
    return 0;                                                                                 \
  }
  O3S_S(4, 1) O3S_S(8, 1) O3S_S(16, 1) O3S_S(32, 1) O3S_S(64, 1)
  O3S_S(64, 2) O3S_S(64, 4) O3S_S(64, 8) O3S_S(64, 16)
#undef O3S_S
  return -1;
}

O3S_API int o3s_glm_margin(const void* X, int64_t ld, int64_t n, const float* coef,
                           float intercept, float* out, int grid, hipStream_t st) {
  const int nch = (int)(ld / 8);
  const int lpr = pick_lpr(nch), cpl = pick_cpl(nch);
  if (ld % 8 != 0 || cpl > 16) return -1;
  if (n <= 0) return 0;
  const uint16_t* Xh = (const uint16_t*)X;
#define O3S_M(L, C)                                                                            \
  if (lpr == L && cpl == C) {                                                                  \
    hipLaunchKernelGGL((glm_margin_kernel<L, C>), dim3(grid), dim3(kBlock), 0, st, Xh, ld, n,   \
                       coef, intercept, out);                                                  \
    O3S_CHECK_LAUNCH();                                                                        \
    return 0;                                                                                  \
  }
  O3S_M(4, 1) O3S_M(8, 1) O3S_M(16, 1) O3S_M(32, 1) O3S_M(64, 1)
  O3S_M(64, 2) O3S_M(64, 4) O3S_M(64, 8) O3S_M(64, 16)
#undef O3S_M
  return -1;
}

// Column moments: out (fp64, 2*dpad+1) = [sum w x | sum w x^2 | sum w].  partial must hold
// grid * (2*dpad+2) floats.
O3S_API int o3s_glm_colstats(int src, const void* X, int64_t ld, int64_t n, const float* sw,
                             uint32_t seed, int64_t row0, float* partial, int grid, double* out,
                             hipStream_t st) {
  const int nch = (int)(ld / 8);
  const int lpr = pick_lpr(nch), cpl = pick_cpl(nch);
  if (ld % 8 != 0 || cpl > 16 || grid <= 0) return -1;
  const int dpad = lpr * cpl * 8, pstride = 2 * dpad + 2;
  const uint16_t* Xh = (const uint16_t*)X;
  if (n > 0) {
    bool done = false;
#define O3S_C(L, C)                                                                            \
  if (!done && lpr == L && cpl == C) {                                                         \
    if (src == 0)                                                                              \
      hipLaunchKernelGGL((glm_colstats_kernel<L, C, 0>), dim3(grid), dim3(kBlock), 0, st, Xh,   \
                         ld, n, sw, seed, row0, partial, pstride);                             \
    else                                                                                       \
      hipLaunchKernelGGL((glm_colstats_kernel<L, C, 1>), dim3(grid), dim3(kBlock), 0, st, Xh,   \
                         ld, n, sw, seed, row0, partial, pstride);                             \
    done = true;                                                                               \
  }
    O3S_C(4, 1) O3S_C(8, 1) O3S_C(16, 1) O3S_C(32, 1) O3S_C(64, 1)
    O3S_C(64, 2) O3S_C(64, 4) O3S_C(64, 8) O3S_C(64, 16)
#undef O3S_C
    if (!done) return -1;
  } else {
    hipMemsetAsync(partial, 0, sizeof(float) * pstride * (size_t)grid, st);
  }
  O3S_CHECK_LAUNCH();
  const int ncols = 2 * dpad + 1;
  hipLaunchKernelGGL(glm_finish_kernel, dim3((ncols + 31) / 32), dim3(1024), 0, st, partial, grid,
                     pstride, ncols, out, 0);
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_API int o3s_glm_sgd_update(const double* out, int dpad, double* bt, double* b, const double* inv_std,
                               const double* l2v, double l2, double eta, int fit_intercept, float* coef_eff,
                               double* loss_slot, hipStream_t st) {
  hipLaunchKernelGGL(glm_sgd_update_kernel, dim3(1), dim3(256), 0, st, out, dpad, bt, b, inv_std, l2v, l2,
                     eta, fit_intercept, coef_eff, loss_slot);
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_API int o3s_glm_sgd_update_dev(const double* out, int dpad, double* bt, double* b, const double* inv_std,
                                   const double* l2v, double l2, const double* l1v, double l1, double step_size,
                                   int fit_intercept, float* coef_eff, double* loss_hist, int64_t cap,
                                   int64_t* t_dev, hipStream_t st) {
  hipLaunchKernelGGL(glm_sgd_update_dev_kernel, dim3(1), dim3(256), 0, st, out, dpad, bt, b, inv_std, l2v, l2,
                     l1v, l1, step_size, fit_intercept, coef_eff, loss_hist, cap, t_dev);
  O3S_CHECK_LAUNCH();
  return 0;
}

// Fused summarizer + first-gradient pass (glm_stats_mixed_kernel): out (fp64, 3*dpad+3) =
// [s1 | s2 | syx | sum w | sum w y | sum w y^2]; partial holds grid * (3*dpad+4) floats.
// Returns -2 when the row layout has no stats instantiation (ld > 2048): the caller then
// uses o3s_glm_colstats plus a regular first pass.
O3S_API int o3s_glm_stats_mixed(const void* X, int64_t ld, int64_t n_res, const float* y, const float* sw,
                                uint32_t seed, int64_t row0, int64_t n_lin, float* partial, int grid, double* out,
                                int waves, hipStream_t st) {
  const int nch = (int)(ld / 8);
  const int lpr = pick_lpr(nch), cpl = pick_cpl(nch);
  if (ld % 8 != 0 || cpl > 16 || grid <= 0 || n_res < 0 || n_lin < 0) return -1;
  const int dpad = lpr * cpl * 8, pstride = 3 * dpad + 4;
  int lpr_s = lpr, cpl_s = cpl;
  if (cpl == 1 && lpr >= 16) { lpr_s = lpr / 4; cpl_s = 4; }
  else if (cpl == 2) { lpr_s = 32; cpl_s = 4; }
  const uint16_t* Xh = (const uint16_t*)X;
  bool done = false;
#define O3S_ST(L, C)                                                                                        \
  if (!done && lpr_s == L && cpl_s == C) {                                                                  \
    done = true;                                                                                            \
    if (waves == 3)                                                                                         \
      hipLaunchKernelGGL((glm_stats_mixed_kernel<L, C, 3>), dim3(grid), dim3(kBlock), 0, st, Xh, ld, n_res, y, \
                         sw, seed, row0, n_lin, partial, pstride);                                          \
    else                                                                                                    \
      hipLaunchKernelGGL((glm_stats_mixed_kernel<L, C, 2>), dim3(grid), dim3(kBlock), 0, st, Xh, ld, n_res, y, \
                         sw, seed, row0, n_lin, partial, pstride);                                          \
  }
  O3S_ST(4, 1) O3S_ST(8, 1) O3S_ST(4, 4) O3S_ST(8, 4) O3S_ST(16, 4) O3S_ST(32, 4) O3S_ST(64, 4)
#undef O3S_ST
  if (!done) return -2;
  O3S_CHECK_LAUNCH();
  const int ncols = 3 * dpad + 3;
  hipLaunchKernelGGL(glm_finish_kernel, dim3((ncols + 31) / 32), dim3(1024), 0, st, partial, grid, pstride, ncols,
                     out, 0);
  O3S_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------
// Multinomial (softmax) logistic regression, one fused pass over bf16 rows:
//   margins M = X W^T + b (MFMA), row log-sum-exp, residual R = w (softmax(M) - onehot(y)),
//   gradient G = R^T X (MFMA), sum(R) per class and the weighted cross-entropy.
// Reference: Spark's MultinomialLogisticRegression aggregator reached from the
// Classification widget (orangecontrib/spark/widgets/ml/spark_ml_classification.py:15,
// SURVEY §2.8 "Multinomial: X.W with C classes uses MFMA").
//
// Layout (v_mfma_f32_32x32x16_bf16; lane (r = lane&31, h = lane>>5)):
//   forward  A = W split (32 classes x 16 dims, class r, dims 8h..+8), B = X (row r, the
//            same 8 dims -- exactly the 16-B global load of the row) -> acc[v] = margin of
//            row r, class 8(v>>2) + 4h + (v&3);
//   backward A = R split (class r, rows 8h..+8 of a 16-row step), B = X^T (rows 8h..+8,
//            dim r of a 32-dim block, read transposed from this wave's LDS copy of the
//            tile) -> G[nb][v] = dG of class 8(v>>2) + 4h + (v&3), dim 32 nb + r.
// X is exact in bf16; W is split into three bf16 terms (hi + mid + lo: margins and loss
// at fp32 level), the residuals R (|R| <= w) into two (hi + lo: ~2^-17 relative per term
// of the gradient sums).  The MFMA
// work is a few % of the HBM time of a tile: the kernel streams X once per pass (the
// next tile's rows are loaded while this tile computes).  One wave per SIMD (the
// 128-register gradient accumulators); per-wave slab rows, summed in fp64 by
// glm_finish_kernel in a fixed order (no float atomics).
namespace {

typedef float sm_f32x16 __attribute__((ext_vector_type(16)));
typedef short sm_bf16x8 __attribute__((ext_vector_type(8)));
constexpr int kSmWaves = 4;
constexpr int kSmThreads = kSmWaves * kWave;

template <int NB>
struct SmLds {
  static constexpr int D = 32 * NB;
  static constexpr int WLD = D + 8;     // +16 B per row: conflict-free 16-B fragment reads
  static constexpr int XLD = D + 8;
  static constexpr int RLD = 40;        // 80-B rows: the 16-B R fragment reads hit distinct banks
  static constexpr int W_ELEMS = 3 * 32 * WLD;
  static constexpr int WAVE_ELEMS = 32 * XLD + 2 * 32 * RLD;
  static constexpr int ELEMS = W_ELEMS + kSmWaves * WAVE_ELEMS;
};

template <int NB>
__global__ __launch_bounds__(kSmThreads, 1) void glm_softmax_kernel(
    const uint16_t* __restrict__ X, int64_t n, int64_t ldx, const int32_t* __restrict__ y,
    const float* __restrict__ sw, const uint16_t* __restrict__ Wsp, const float* __restrict__ bias, int K,
    float* __restrict__ partial, int pstride) {
  using L = SmLds<NB>;
  constexpr int D = L::D, KS = 2 * NB, WLD = L::WLD, XLD = L::XLD, RLD = L::RLD;
  __shared__ __attribute__((aligned(16))) uint16_t smem[L::ELEMS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  uint16_t* Ws = smem;
  uint16_t* Xs = smem + L::W_ELEMS + wid * L::WAVE_ELEMS;
  uint16_t* Rs = Xs + 32 * XLD;

  // W splits [3][32][D] -> LDS (padded rows)
  for (int p = threadIdx.x; p < 3 * 32 * (D / 8); p += kSmThreads) {
    const int row = p / (D / 8), k8 = p % (D / 8);
    *reinterpret_cast<sm_bf16x8*>(Ws + row * WLD + k8 * 8) =
        *reinterpret_cast<const sm_bf16x8*>(Wsp + (int64_t)row * D + k8 * 8);
  }
  float bl[16];
  int cls[16];
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    cls[v] = 8 * (v >> 2) + 4 * h + (v & 3);
    bl[v] = cls[v] < K ? bias[cls[v]] : -INFINITY;
  }
  __syncthreads();

  sm_f32x16 G[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int v = 0; v < 16; ++v) G[b][v] = 0.f;
  float gb[16];
#pragma unroll
  for (int v = 0; v < 16; ++v) gb[v] = 0.f;
  float lossacc = 0.f;

  const int64_t ntiles = (n + 31) / 32;
  const int64_t step = (int64_t)gridDim.x * kSmWaves;
  int64_t tile = (int64_t)blockIdx.x * kSmWaves + wid;
  sm_bf16x8 xb[KS], xn[KS];
  auto load = [&](int64_t t, sm_bf16x8 (&dst)[KS]) {
    int64_t row = t * 32 + r;
    row = row < n ? row : n - 1;
    const uint16_t* src = X + row * ldx;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int col = ks * 16 + 8 * h;
      if (col < ldx) {
        dst[ks] = *reinterpret_cast<const sm_bf16x8*>(src + col);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) dst[ks][j] = 0;
      }
    }
  };
  if (tile < ntiles) load(tile, xb);
  for (; tile < ntiles; tile += step) {
    if (tile + step < ntiles) load(tile + step, xn);
    const int64_t row = tile * 32 + r;
    const bool valid = row < n;
    const int yl = valid ? y[row] : -1;
    const float wr = valid ? (sw ? sw[row] : 1.f) : 0.f;
    // ---- forward: margins of row r, 16 classes per lane
    sm_f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = bl[v];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const sm_bf16x8 a = *reinterpret_cast<const sm_bf16x8*>(Ws + (s * 32 + r) * WLD + ks * 16 + 8 * h);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, xb[ks], acc, 0, 0, 0);
      }
      *reinterpret_cast<sm_bf16x8*>(Xs + r * XLD + ks * 16 + 8 * h) = xb[ks];   // for the X^T reads
    }
    // ---- row softmax (the two half-waves hold disjoint class subsets of row r)
    float mx = -INFINITY;
#pragma unroll
    for (int v = 0; v < 16; ++v) mx = fmaxf(mx, acc[v]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float se = 0.f;
#pragma unroll
    for (int v = 0; v < 16; ++v) se += __expf(acc[v] - mx);
    se += __shfl_xor(se, 32, 64);
    const float lse = mx + __logf(se);
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const bool hit = cls[v] == yl;
      const float p = __expf(acc[v] - lse);
      const float rv = wr * (p - (hit ? 1.f : 0.f));
      gb[v] += rv;
      if (hit) lossacc += wr * (lse - acc[v]);
      const uint16_t a0 = f32_to_bf16(rv);
      Rs[(0 * 32 + cls[v]) * RLD + r] = a0;
      Rs[(1 * 32 + cls[v]) * RLD + r] = f32_to_bf16(rv - bf16_to_f32(a0));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // ---- backward: G[class][dim] += sum over the tile's rows of R[row][class] X[row][dim]
    sm_bf16x8 ar[2][2];
#pragma unroll
    for (int rs = 0; rs < 2; ++rs)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        ar[rs][s] = *reinterpret_cast<const sm_bf16x8*>(Rs + (s * 32 + r) * RLD + rs * 16 + 8 * h);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
      for (int rs = 0; rs < 2; ++rs) {
        sm_bf16x8 bx;
#pragma unroll
        for (int q = 0; q < 8; ++q) bx[q] = (short)Xs[(rs * 16 + 8 * h + q) * XLD + b * 32 + r];
#pragma unroll
        for (int s = 0; s < 2; ++s) G[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[rs][s], bx, G[b], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    // tile's LDS reads done before it is overwritten
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) xb[ks] = xn[ks];
  }
  // ---- this wave's slab row: [G class-major 32 x D | sum R (32) | loss]
  float* out = partial + ((int64_t)blockIdx.x * kSmWaves + wid) * pstride;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int v = 0; v < 16; ++v) out[cls[v] * D + b * 32 + r] = G[b][v];
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    float s = gb[v];
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);   // over the 32 rows (same h)
    if (r == 0) out[32 * D + cls[v]] = s;
  }
  const float lt = wave_sum(lossacc);
  if (lane == 0) out[32 * D + 32] = lt;
}

}  // namespace

// One multinomial pass: out (fp64, [32 * D | 32 | 1]) = (gradient class-major over
// D = 32 * ceil(d / 32) dims, per-class residual sums, weighted cross-entropy) over the n
// rows of X (bf16, row stride ldx, ldx % 8 == 0).  y: int32 labels in [0, K); sw: fp32
// weights or null; Wsp: bf16 [3][32][D] (hi, mid, lo splits of the class-major
// coefficients, zero-padded); bias: fp32 [32].  partial: fp32 [grid * 4][32 D + 33].
O3S_API int o3s_glm_softmax(const void* X, int64_t n, int64_t ldx, int d, const int32_t* y, const float* sw,
                            const void* Wsp, const float* bias, int K, float* partial, int grid, double* out,
                            hipStream_t st) {
  const int nb = (d + 31) / 32;
  if (ldx % 8 != 0 || nb < 1 || nb > 8 || K < 1 || K > 32 || grid <= 0) return -1;
  const int D = 32 * nb, pstride = 32 * D + 33;
  const uint16_t* Xh = (const uint16_t*)X;
  const uint16_t* Wh = (const uint16_t*)Wsp;
  if (n > 0) {
    switch (nb) {
#define O3S_SM(NBV) \
  case NBV: hipLaunchKernelGGL((glm_softmax_kernel<NBV>), dim3(grid), dim3(kSmThreads), 0, st, Xh, n, ldx, y, sw, \
                               Wh, bias, K, partial, pstride); break;
      O3S_SM(1) O3S_SM(2) O3S_SM(3) O3S_SM(4) O3S_SM(5) O3S_SM(6) O3S_SM(7) O3S_SM(8)
#undef O3S_SM
      default: return -1;
    }
  } else {
    hipMemsetAsync(partial, 0, sizeof(float) * pstride * (size_t)grid * kSmWaves, st);
  }
  O3S_CHECK_LAUNCH();
  hipLaunchKernelGGL(glm_finish_kernel, dim3((pstride + 31) / 32), dim3(1024), 0, st, partial, grid * kSmWaves,
                     pstride, pstride, out, 0);
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_PRELOAD(glm)
