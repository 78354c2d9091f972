// Shared helpers for the CDNA4 (gfx950) kernels of vodascheduler_amd.
//
// Conventions
//  * wave64 everywhere: lane = threadIdx.x & 63, reductions over 64 lanes.
//  * bf16 is carried as raw uint16_t in memory and converted with the clang __bf16
//    type (hipcc lowers the f32->bf16 conversion to v_cvt_pk_bf16_f32 on gfx950).
//  * Memory-bound kernels always move 8-16 B per lane (guide §6 Guideline 13).
//  * Every launch goes onto the caller's stream (torch.cuda.current_stream()), so the
//    kernels are hipGraph-capturable: no allocation / sync inside launch functions.
#pragma once

#include <hip/hip_runtime.h>
#include <cmath>

#include "host_common.h"
#include <cstdint>
#include <stdexcept>
#include <string>

namespace voda {


inline int dtype_size(int dt) { return dt == kF32 ? 4 : 2; }

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(uint32_t(v) << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = static_cast<__bf16>(f);  // RNE, v_cvt_pk_bf16_f32 on gfx950
  return __builtin_bit_cast(uint16_t, b);
}

__device__ __forceinline__ float h2f(uint16_t v) { return static_cast<float>(__builtin_bit_cast(_Float16, v)); }
__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, static_cast<_Float16>(f)); }

// Load/store 4 consecutive elements of type T as float4 (16 B for f32, 8 B for 16-bit).
template <typename T> struct Vec4;
template <> struct Vec4<float> {
  static __device__ __forceinline__ float4 load(const float* p, int64_t i4) {
    return reinterpret_cast<const float4*>(p)[i4];
  }
  static __device__ __forceinline__ void store(float* p, int64_t i4, float4 v) {
    reinterpret_cast<float4*>(p)[i4] = v;
  }
  static __device__ __forceinline__ float load1(const float* p, int64_t i) { return p[i]; }
  static __device__ __forceinline__ void store1(float* p, int64_t i, float v) { p[i] = v; }
};
struct BF16 { uint16_t x; };
struct F16 { uint16_t x; };
template <> struct Vec4<BF16> {
  static __device__ __forceinline__ float4 load(const BF16* p, int64_t i4) {
    uint2 u = reinterpret_cast<const uint2*>(p)[i4];
    return make_float4(bf2f(u.x & 0xffff), bf2f(u.x >> 16), bf2f(u.y & 0xffff), bf2f(u.y >> 16));
  }
  static __device__ __forceinline__ void store(BF16* p, int64_t i4, float4 v) {
    uint2 u;
    u.x = uint32_t(f2bf(v.x)) | (uint32_t(f2bf(v.y)) << 16);
    u.y = uint32_t(f2bf(v.z)) | (uint32_t(f2bf(v.w)) << 16);
    reinterpret_cast<uint2*>(p)[i4] = u;
  }
  static __device__ __forceinline__ float load1(const BF16* p, int64_t i) { return bf2f(p[i].x); }
  static __device__ __forceinline__ void store1(BF16* p, int64_t i, float v) { p[i].x = f2bf(v); }
};
template <> struct Vec4<F16> {
  static __device__ __forceinline__ float4 load(const F16* p, int64_t i4) {
    uint2 u = reinterpret_cast<const uint2*>(p)[i4];
    return make_float4(h2f(u.x & 0xffff), h2f(u.x >> 16), h2f(u.y & 0xffff), h2f(u.y >> 16));
  }
  static __device__ __forceinline__ void store(F16* p, int64_t i4, float4 v) {
    uint2 u;
    u.x = uint32_t(f2h(v.x)) | (uint32_t(f2h(v.y)) << 16);
    u.y = uint32_t(f2h(v.z)) | (uint32_t(f2h(v.w)) << 16);
    reinterpret_cast<uint2*>(p)[i4] = u;
  }
  static __device__ __forceinline__ float load1(const F16* p, int64_t i) { return h2f(p[i].x); }
  static __device__ __forceinline__ void store1(F16* p, int64_t i, float v) { p[i].x = f2h(v); }
};

// 64-lane butterfly reductions (lowered to DPP / ds_swizzle by hipcc).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Grid size for grid-stride memory-bound kernels: enough blocks to fill 256 CUs with
// several resident blocks each, capped (guide §6 Guideline 11).
// Grid of a streaming (elementwise) kernel: one work item per thread.  The kernels keep their
// grid-stride loops, so a cap stays correct, but on MI355X the uncapped grid streams faster (a
// 110 M-parameter AdamW step 709 -> 555 us vs 2048 grid-striding blocks, profiles/r5/optim_grid_cap.jsonl).
inline unsigned stream_grid(int64_t work_items, int block = 256, int64_t cap = int64_t(1) << 30) {
  int64_t g = (work_items + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<unsigned>(g);
}


// tanh-approximated GELU (activation.hip, the fused-epilogue GEMMs of splitgemm.hip):
//   g(h)  = 0.5 h (1 + tanh(u)),  u = k (h + c h^3);  g'(h) = 0.5 (1 + t) + 0.5 h (1 - t^2) k (1 + 3 c h^2)
constexpr float kGeluK = 0.7978845608028654f;
constexpr float kGeluC = 0.044715f;

// The kernels are VALU-bound, not HBM-bound, with the textbook formula (an IEEE divide is
// ~10 instructions): written as a logistic, 0.5 (1 + tanh(u)) = 1 / (1 + e^{-2u}), with
// v_exp_f32 (exp2) and v_rcp_f32 (1 ulp) it is 7 VALU ops forward, ~13 backward.
//   s = 1 / (1 + 2^{h (A + B h^2)}),  A = -2 k log2(e),  B = A c;   g = h s
//   g' = s + 2 k h s (1 - s) (1 + 3 c h^2),  s (1 - s) = e s^2
constexpr float kGeluA = -2.f * kGeluK * 1.4426950408889634f;
constexpr float kGeluB = kGeluA * kGeluC;

// exponent clamped at 64 so that e stays finite (s = 2^-64 then; e s = 1 - s exactly enough)
__device__ __forceinline__ float gelu_exp(float h, float h2) {
  return __builtin_amdgcn_exp2f(fminf(h * __builtin_fmaf(kGeluB, h2, kGeluA), 64.f));
}

__device__ __forceinline__ float gelu_tanh_f(float h) { return h * __builtin_amdgcn_rcpf(1.f + gelu_exp(h, h * h)); }

__device__ __forceinline__ float gelu_tanh_grad(float h) {
  const float h2 = h * h;
  const float e = gelu_exp(h, h2);
  const float s = __builtin_amdgcn_rcpf(1.f + e);
  // s (1 - s) = e s^2: no cancellation as s -> 1
  return __builtin_fmaf(2.f * kGeluK * h * e * s * s, __builtin_fmaf(3.f * kGeluC, h2, 1.f), s);
}


inline void check_launch() { VODA_HIP_CHECK(hipGetLastError()); }

}  // namespace voda
