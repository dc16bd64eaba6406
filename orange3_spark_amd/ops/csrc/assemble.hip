// VectorAssembler in one pass (gfx950): k numeric / vector columns of any dtype, with
// null masks, gathered straight into the padded row-major feature matrix the GLM / tree /
// k-means kernels consume (bf16 [n, ld], ld % 8 == 0, zero padded; or fp32).
//
// Reference: the Dataset Builder widget's commit, VectorAssembler(inputCols=features,
// outputCol='features').transform(df) (orangecontrib/spark/widgets/ml/spark_ml_dataset.py:
// 575-576) -- the first compute step of the tutorial chain.  The torch composition it
// replaces (per-column fp64 casts, a concat, an isnan pass, a padded bf16 copy) moved
// ~5 passes and 8 B/element of scratch; here every input byte is read once and every
// output byte written once.
//
// Mapping: a 256-thread block owns 64 consecutive rows; lane r of each wave is row
// row0 + r, and the block's 4 waves take the row's 16-B output chunks round robin.  All
// 64 lanes of a wave work on the same output chunk, so the per-column source lookup
// (column map in LDS) and the dtype switch are wave-uniform, and the reads of a columnar
// source are 64 consecutive elements (coalesced).  The 64 rows x ld block of output is
// written by the block within a short window, so L2 merges the 16-B row segments into
// full lines before write-back.
//
// handleInvalid: a row is invalid if any of its values is null (mask) or NaN; the kernel
// writes a per-row flag and adds the block's count to *nbad (one integer atomic per
// block).  Invalid values are stored as NaN ("keep" semantics); the caller raises
// ("error") or compacts ("skip") using the count.
#include <hip/hip_fp16.h>

#include <type_traits>

#include "common.h"

using namespace o3s;

namespace {

enum { DT_F64 = 0, DT_F32 = 1, DT_BF16 = 2, DT_F16 = 3, DT_I64 = 4, DT_I32 = 5, DT_I16 = 6, DT_I8 = 7, DT_U8 = 8,
       DT_BOOL = 9 };

struct AsmSrc {
  const void* ptr;          // column data: [n] (width 1) or row-major [n, stride] (vector)
  const uint8_t* valid;     // optional per-row validity (1 = valid), null = all valid
  int64_t stride;           // elements between consecutive rows (1 for a scalar column)
  int32_t width;            // values contributed per row
  int32_t dtype;
};

constexpr int kRows = 64;
constexpr int kThreads = 256;
constexpr int kMaxSrc = 512;

__device__ __forceinline__ float load_as_float(const AsmSrc& s, int64_t row, int e) {
  const int64_t i = row * s.stride + e;
  switch (s.dtype) {
    case DT_F64: return (float)reinterpret_cast<const double*>(s.ptr)[i];
    case DT_F32: return reinterpret_cast<const float*>(s.ptr)[i];
    case DT_BF16: return bf16_to_f32(reinterpret_cast<const uint16_t*>(s.ptr)[i]);
    case DT_F16: return __half2float(reinterpret_cast<const __half*>(s.ptr)[i]);
    case DT_I64: return (float)reinterpret_cast<const int64_t*>(s.ptr)[i];
    case DT_I32: return (float)reinterpret_cast<const int32_t*>(s.ptr)[i];
    case DT_I16: return (float)reinterpret_cast<const int16_t*>(s.ptr)[i];
    case DT_I8: return (float)reinterpret_cast<const int8_t*>(s.ptr)[i];
    default: return (float)reinterpret_cast<const uint8_t*>(s.ptr)[i];     // u8 / bool
  }
}

// colmap[j] = (source index, element within source) for output column j < D; j >= D: pad.
template <int OUT>   // 0: bf16 out, 1: fp32 out
__global__ __launch_bounds__(kThreads) void assemble_kernel(const AsmSrc* __restrict__ srcs, int nsrc,
                                                            const int2* __restrict__ colmap, int D, int ld,
                                                            int64_t n, void* __restrict__ out,
                                                            uint8_t* __restrict__ bad, int* __restrict__ nbad) {
  __shared__ AsmSrc s_src[kMaxSrc];
  __shared__ uint8_t s_bad[kRows];
  for (int i = threadIdx.x; i < nsrc; i += kThreads) s_src[i] = srcs[i];
  if (threadIdx.x < kRows) s_bad[threadIdx.x] = 0;
  __syncthreads();
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int nch = ld / 8;
  const int64_t nblk = (n + kRows - 1) / kRows;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t row = blk * kRows + lane;
    const bool ok = row < n;
    const int64_t rowc = ok ? row : n - 1;
    bool rbad = false;
    for (int ch = wid; ch < nch; ch += kThreads / kWave) {
      float v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int j = 8 * ch + q;
        float x = 0.f;
        if (j < D) {                                  // wave-uniform
          const int2 m = colmap[j];
          const AsmSrc& s = s_src[m.x];
          x = load_as_float(s, rowc, m.y);
          const bool valid = s.valid == nullptr || s.valid[rowc] != 0;
          if (!valid) x = __builtin_nanf("");
          rbad |= !(x == x);
        }
        v[q] = x;
      }
      if (ok) {
        if (OUT == 0) {
          short8 o;
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] = (short)f32_to_bf16(v[q]);
          *reinterpret_cast<short8*>(reinterpret_cast<uint16_t*>(out) + row * ld + 8 * ch) = o;
        } else {
          float* po = reinterpret_cast<float*>(out) + row * ld + 8 * ch;
          *reinterpret_cast<float4_*>(po) = float4_{v[0], v[1], v[2], v[3]};
          *reinterpret_cast<float4_*>(po + 4) = float4_{v[4], v[5], v[6], v[7]};
        }
      }
    }
    if (ok && rbad) s_bad[lane] = 1;                  // benign race: every writer stores 1
    __syncthreads();
    if (wid == 0) {
      const int b = (ok && s_bad[lane]) ? 1 : 0;
      if (ok && bad) bad[row] = (uint8_t)b;
      const int cnt = wave_sum_i(b);
      if (lane == 0 && cnt) atomicAdd(nbad, cnt);
      s_bad[lane] = 0;
    }
    __syncthreads();
  }
}

// Fast path: every source a plain [n] column of one dtype T (the common wide table of
// float / double columns).  A block owns 256 rows (4 per lane) and walks the output in
// windows of kCW = 64 columns (LDS tile 33 KB for bf16 out):
//   load:  wave w takes columns w, w + 4, ...; lane l reads rows l, l + 64, ... of 8 columns
//          per batch (32 independent loads in flight, each wave load a 256-B contiguous run
//          of one column), converts and writes them transposed into an LDS tile whose row
//          stride is an odd number of dwords, so the 64 lanes -- 64 rows -- land on 64
//          different banks;
//   store: the tile goes out row-major, 16 B per lane, each row's window one contiguous
//          256-B (bf16) / 512-B (fp32) run.
// Every input byte is read once as part of a long sequential run and every output line is
// written whole -- the generic kernel above reads 64 elements of 8 different sources per
// wave step and writes 16-B pieces of 64 rows 512 B apart.
typedef unsigned int uint4_ __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ float to_f(T v) { return (float)v; }

// 256-row blocks measured 4.8-4.9 TB/s against 4.2 for 128-row blocks at 100M x 256 fp32
// -> bf16; 32- / 128-column windows, 16-column batches and 8-B row-pair loads were no
// faster (profiles/assemble_kernel_100Mx256.json) and were removed.
template <typename T, int OUT>
__global__ __launch_bounds__(kThreads) void assemble_cols_kernel(const AsmSrc* __restrict__ srcs, int D, int ld,
                                                                 int64_t n, void* __restrict__ out,
                                                                 uint8_t* __restrict__ bad, int* __restrict__ nbad) {
  constexpr int kCW = 64, kCBatch = 8, RPL = 4;
  constexpr int kCRows = 64 * RPL;
  constexpr int PAD = OUT == 0 ? 2 : 1;
  constexpr int LS = kCW + PAD;                       // tile row stride (elements): 65 / 129 dwords
  using OT = typename std::conditional<OUT == 0, uint16_t, float>::type;
  __shared__ OT tile[kCRows * LS];
  __shared__ uint8_t s_bad[kCRows];
  for (int i = threadIdx.x; i < kCRows; i += kThreads) s_bad[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & (kWave - 1);
  // wave index made provably uniform: the source descriptors are then read with scalar
  // loads (constant cache) instead of an LDS table, which keeps LDS for the tile alone
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t nblk = (n + kCRows - 1) / kCRows;
  // XCD-aware walk: workgroups are dealt to the 8 XCDs round robin, so block b of a grid of
  // G (G % 8 == 0) takes row block it G + (b % 8) G/8 + b/8 in sweep it -- every XCD streams
  // one contiguous G/8-block range of each column per sweep instead of every 8th block
  const int64_t G = gridDim.x;
  const int64_t xoff = (G % 8 == 0) ? (int64_t)(blockIdx.x % 8) * (G / 8) + blockIdx.x / 8 : blockIdx.x;
  for (int64_t blk = xoff; blk < nblk; blk += G) {
    const int64_t row0 = blk * kCRows;
    auto rib = [&](int i) { return lane + 64 * i; };   // row in block
    int64_t rr[RPL];
    bool rbad[RPL];
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
      rr[i] = row0 + rib(i) < n ? row0 + rib(i) : n - 1;
      rbad[i] = false;
    }
    for (int c0 = 0; c0 < ld; c0 += kCW) {
      const int cw = ld - c0 < kCW ? ld - c0 : kCW;
      for (int jb = wid; jb < cw; jb += 4 * kCBatch) {
        T v[kCBatch][RPL];
#pragma unroll
        for (int q = 0; q < kCBatch; ++q) {
          const int j = c0 + jb + 4 * q;                // wave-uniform
          if (jb + 4 * q < cw && j < D) {
            const T* p = reinterpret_cast<const T*>(srcs[j].ptr);
#pragma unroll
            for (int i = 0; i < RPL; ++i) v[q][i] = p[rr[i]];
          }
        }
#pragma unroll
        for (int q = 0; q < kCBatch; ++q) {
          const int jl = jb + 4 * q, j = c0 + jl;
          if (jl >= cw) break;
          const uint8_t* vm = j < D ? srcs[j].valid : nullptr;
#pragma unroll
          for (int i = 0; i < RPL; ++i) {
            float a = 0.f;
            if (j < D) {
              a = to_f(v[q][i]);
              if (vm != nullptr && !vm[rr[i]]) a = __builtin_nanf("");
              rbad[i] |= !(a == a);
            }
            if constexpr (OUT == 0) tile[rib(i) * LS + jl] = f32_to_bf16(a);
            else tile[rib(i) * LS + jl] = a;
          }
        }
      }
      __syncthreads();
      const int cpr = cw / 8;                          // 16-B (bf16) / 32-B (fp32) chunks per row
      for (int e = threadIdx.x; e < kCRows * cpr; e += kThreads) {
        const int r = e / cpr, k = e - r * cpr;
        const int64_t row = row0 + r;
        if (row < n) {
          if constexpr (OUT == 0) {
            const uint32_t* t = reinterpret_cast<const uint32_t*>(&tile[r * LS + 8 * k]);
            uint4_ o;
            o.x = t[0]; o.y = t[1]; o.z = t[2]; o.w = t[3];
            *reinterpret_cast<uint4_*>(reinterpret_cast<uint16_t*>(out) + row * ld + c0 + 8 * k) = o;
          } else {
            const float* t = &tile[r * LS + 8 * k];
            float* po = reinterpret_cast<float*>(out) + row * ld + c0 + 8 * k;
            *reinterpret_cast<float4_*>(po) = float4_{t[0], t[1], t[2], t[3]};
            *reinterpret_cast<float4_*>(po + 4) = float4_{t[4], t[5], t[6], t[7]};
          }
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < RPL; ++i)
      if (rbad[i] && row0 + rib(i) < n) s_bad[rib(i)] = 1;   // benign race: every writer stores 1
    __syncthreads();
    for (int r = threadIdx.x; r < kCRows; r += kThreads) {
      // whole waves take part (kCRows is a multiple of 64): the wave sum below is uniform
      const bool ok = row0 + r < n;
      const int b = (ok && s_bad[r]) ? 1 : 0;
      if (ok && bad) bad[row0 + r] = (uint8_t)b;
      const int cnt = wave_sum_i(b);
      if (lane == 0 && cnt) atomicAdd(nbad, cnt);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kCRows; i += kThreads) s_bad[i] = 0;
    __syncthreads();
  }
}

}  // namespace

// srcs: device array of nsrc AsmSrc; colmap: device int2[D]; out: [n, ld] (bf16 when
// out_f32 == 0, else fp32), ld % 8 == 0, ld >= D; bad: optional uint8[n]; nbad: int (zeroed
// by the caller).
O3S_API int o3s_assemble(const void* srcs, int nsrc, const void* colmap, int D, int ld, int64_t n, void* out,
                         int out_f32, void* bad, void* nbad, int grid, hipStream_t st) {
  if (nsrc <= 0 || nsrc > kMaxSrc || ld % 8 != 0 || ld < D || n < 0 || grid <= 0) return -1;
  if (n == 0) return 0;
  if (out_f32)
    hipLaunchKernelGGL(assemble_kernel<1>, dim3(grid), dim3(kThreads), 0, st, (const AsmSrc*)srcs, nsrc,
                       (const int2*)colmap, D, ld, n, out, (uint8_t*)bad, (int*)nbad);
  else
    hipLaunchKernelGGL(assemble_kernel<0>, dim3(grid), dim3(kThreads), 0, st, (const AsmSrc*)srcs, nsrc,
                       (const int2*)colmap, D, ld, n, out, (uint8_t*)bad, (int*)nbad);
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_API int o3s_assemble_src_size() { return (int)sizeof(AsmSrc); }

// Fast path (see assemble_cols_kernel): srcs[j] is output column j for j < D, every source a
// contiguous [n] column of dtype src_dtype (DT_F32 or DT_F64), ld % 8 == 0, D <= 512.
O3S_API int o3s_assemble_cols(const void* srcs, int src_dtype, int D, int ld, int64_t n, void* out, int out_f32,
                              void* bad, void* nbad, int grid, hipStream_t st) {
  if (D <= 0 || D > kMaxSrc || ld % 8 != 0 || ld < D || n < 0 || grid <= 0) return -1;
  if (src_dtype != DT_F32 && src_dtype != DT_F64) return -2;
  if (n == 0) return 0;
#define O3S_ASM_COLS(T, O)                                                                               \
  hipLaunchKernelGGL((assemble_cols_kernel<T, O>), dim3(grid), dim3(kThreads), 0, st, (const AsmSrc*)srcs, \
                     D, ld, n, out, (uint8_t*)bad, (int*)nbad)
  if (src_dtype == DT_F32) {
    if (out_f32) { O3S_ASM_COLS(float, 1); } else { O3S_ASM_COLS(float, 0); }
  } else {
    if (out_f32) { O3S_ASM_COLS(double, 1); } else { O3S_ASM_COLS(double, 0); }
  }
#undef O3S_ASM_COLS
  O3S_CHECK_LAUNCH();
  return 0;
}

O3S_PRELOAD(assemble)
