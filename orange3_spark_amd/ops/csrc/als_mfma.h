// Register-level helpers of the dense exact-ALS kernel (als_dense.hip), kept apart so a
// variant kernel can share them (the round-6 wave-pair A/B did): MFMA fragment types, the
// 32 x 32 accumulator layout, bf16 hi / lo splits (bf16x3 products), counted DMA waits.
#pragma once
#include "common.h"

namespace o3s {
namespace als {

typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float rl(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}
__device__ __forceinline__ constexpr int rowof(int v, int h) { return (v & 3) + 8 * (v >> 2) + 4 * h; }

// Cross-lane hand-off through LDS inside ONE wave: the hardware runs a wave's LDS
// instructions in order, but the compiler reasons per lane and may move a load past
// another lane's store (e.g. forward a lane's own conditional store and sink the load into
// the other branch).  This compiler barrier pins every LDS access on its side.
__device__ __forceinline__ void lane_sync() { asm volatile("" ::: "memory"); }
template <int NT>
__device__ __forceinline__ constexpr int tix(int j, int i) { return j * NT - j * (j - 1) / 2 + (i - j); }

// s_waitcnt vmcnt(n * NIS) for a wave-uniform n in [0, 7]: the DMAs of the n later steps
// stay in flight (loads retire in order, so this is exactly "this step has landed")
// (the counter holds 63: a larger count is clamped, i.e. waits for more; the kernels never
// keep more than DEPTH - 1 steps = at most 63 DMAs in flight)
__device__ __forceinline__ constexpr int vm_cap(int n) { return n < 63 ? n : 63; }
template <int NIS>
__device__ __forceinline__ void wait_steps(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vm_cap(1 * NIS)) : "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vm_cap(2 * NIS)) : "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vm_cap(3 * NIS)) : "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vm_cap(4 * NIS)) : "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vm_cap(5 * NIS)) : "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vm_cap(6 * NIS)) : "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vm_cap(7 * NIS)) : "memory"); break;
  }
}

// z = s * y for 8 ratings -> bf16 hi (RNE) and lo = bf16(z - hi), packed as MFMA fragments
__device__ __forceinline__ void split8(const float (&z)[8], bf16x8_t& hi, bf16x8_t& lo) {
  u32x4_t H, L;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f32x2_t a = {z[2 * k], z[2 * k + 1]};
    const unsigned hu = __builtin_bit_cast(unsigned, __builtin_convertvector(a, bf16x2_t));
    const f32x2_t hf = {__builtin_bit_cast(float, hu << 16), __builtin_bit_cast(float, hu & 0xffff0000u)};
    const unsigned lu = __builtin_bit_cast(unsigned, __builtin_convertvector(a - hf, bf16x2_t));
    H[k] = hu;
    L[k] = lu;
  }
  hi = __builtin_bit_cast(bf16x8_t, H);
  lo = __builtin_bit_cast(bf16x8_t, L);
}

// registers 8 m .. 8 m + 7 of an accumulator tile -> bf16 hi / lo MFMA fragments
__device__ __forceinline__ void split_half(const f32x16_t& t, int m, bf16x8_t& hi, bf16x8_t& lo) {
  float z[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) z[k] = t[8 * m + k];
  split8(z, hi, lo);
}
__device__ __forceinline__ bf16x8_t neg8(bf16x8_t v) {
  return __builtin_bit_cast(bf16x8_t, __builtin_bit_cast(u32x4_t, v) ^ 0x80008000u);
}

}  // namespace als
}  // namespace o3s
