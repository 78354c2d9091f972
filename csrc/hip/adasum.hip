// Adasum gradient combination (CDNA4 / gfx950).
//
// Horovod's optional `op=hvd.Adasum` reduction (reference
// examples/py/pytorch/pytorch_mnist_elastic.py:32,102,108-109,188) combines
// two gradients a, b PER TENSOR as
//     adasum(a, b) = (1 - a.b / (2|a|^2)) a + (1 - a.b / (2|b|^2)) b
// and an N-rank reduction applies it along a binary tree.  Here a bucket is a contiguous
// slice of the flat gradient buffer holding many parameters ("segments"), so the kernels
// are segmented:
//   1. adasum_partials: every workgroup reduces (a.b, a.a, b.b) over one <= kChunk slice of
//      one segment (16 B loads, wave64 butterflies, LDS across the 4 waves) and writes
//      the three fp32 partials to its own workspace slot -- no atomics, so the result is
//      bit-identical on every rank (all ranks run the same tree on the same gathered data
//      and must stay replicas).
//   2. adasum_combine: every workgroup re-reduces its segment's partials in a fixed order
//      (cheap: a few hundred floats at most), derives the two coefficients and writes
//      out = ca*a + cb*b for its slice.  `out` may alias `a`.
// The block table (segment id, slice start/end per workgroup; first block and block count
// per segment) is built once per bucket on the host and lives on the device.
#include "common.h"
#include "ops.h"

namespace voda {

constexpr int kAdasumThreads = 256;

struct AdasumMeta {
  const int64_t* blk_seg;    // [nblk]
  const int64_t* blk_lo;     // [nblk]
  const int64_t* blk_hi;     // [nblk]
  const int64_t* seg_first;  // [nseg]
  const int64_t* seg_nblk;   // [nseg]
};

__device__ __forceinline__ AdasumMeta adasum_meta(const int64_t* meta, int64_t nblk, int64_t nseg) {
  AdasumMeta m;
  m.blk_seg = meta;
  m.blk_lo = meta + nblk;
  m.blk_hi = meta + 2 * nblk;
  m.seg_first = meta + 3 * nblk;
  m.seg_nblk = meta + 3 * nblk + nseg;
  return m;
}

// Block-wide sum of three values; result valid in thread 0.
__device__ __forceinline__ float3 block_sum3(float x, float y, float z) {
  __shared__ float red[3][kAdasumThreads / 64];
  x = wave_sum(x);
  y = wave_sum(y);
  z = wave_sum(z);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wid] = x;
    red[1][wid] = y;
    red[2][wid] = z;
  }
  __syncthreads();
  float3 r = make_float3(0.f, 0.f, 0.f);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 0; w < kAdasumThreads / 64; ++w) {
      r.x += red[0][w];
      r.y += red[1][w];
      r.z += red[2][w];
    }
  }
  return r;
}

template <typename T>
__global__ __launch_bounds__(kAdasumThreads) void adasum_partials_kernel(const T* __restrict__ a,
                                                                         const T* __restrict__ b,
                                                                         const int64_t* __restrict__ meta,
                                                                         int64_t nblk, int64_t nseg,
                                                                         float* __restrict__ partials) {
  const AdasumMeta m = adasum_meta(meta, nblk, nseg);
  const int64_t lo = m.blk_lo[blockIdx.x], hi = m.blk_hi[blockIdx.x];
  float dot = 0.f, aa = 0.f, bb = 0.f;
  // 4-wide path over the 4-aligned interior, scalar head/tail (wave-uniform bounds)
  const int64_t lo4 = (lo + 3) >> 2, hi4 = hi >> 2;
  if (lo4 < hi4) {
    for (int64_t i = lo4 + threadIdx.x; i < hi4; i += kAdasumThreads) {
      const float4 x = Vec4<T>::load(a, i), y = Vec4<T>::load(b, i);
      dot += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
      aa += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
      bb += y.x * y.x + y.y * y.y + y.z * y.z + y.w * y.w;
    }
    for (int64_t i = lo + threadIdx.x; i < (lo4 << 2); i += kAdasumThreads) {
      const float x = Vec4<T>::load1(a, i), y = Vec4<T>::load1(b, i);
      dot += x * y; aa += x * x; bb += y * y;
    }
    for (int64_t i = (hi4 << 2) + threadIdx.x; i < hi; i += kAdasumThreads) {
      const float x = Vec4<T>::load1(a, i), y = Vec4<T>::load1(b, i);
      dot += x * y; aa += x * x; bb += y * y;
    }
  } else {
    for (int64_t i = lo + threadIdx.x; i < hi; i += kAdasumThreads) {
      const float x = Vec4<T>::load1(a, i), y = Vec4<T>::load1(b, i);
      dot += x * y; aa += x * x; bb += y * y;
    }
  }
  const float3 r = block_sum3(dot, aa, bb);
  if (threadIdx.x == 0) {
    partials[3 * blockIdx.x + 0] = r.x;
    partials[3 * blockIdx.x + 1] = r.y;
    partials[3 * blockIdx.x + 2] = r.z;
  }
}

template <typename T>
__global__ __launch_bounds__(kAdasumThreads) void adasum_combine_kernel(const T* a, const T* __restrict__ b, T* out,
                                                                        const int64_t* __restrict__ meta,
                                                                        int64_t nblk, int64_t nseg,
                                                                        const float* __restrict__ partials) {
  const AdasumMeta m = adasum_meta(meta, nblk, nseg);
  const int64_t seg = m.blk_seg[blockIdx.x];
  const int64_t first = m.seg_first[seg], cnt = m.seg_nblk[seg];
  float dot = 0.f, aa = 0.f, bb = 0.f;
  for (int64_t k = threadIdx.x; k < cnt; k += kAdasumThreads) {
    dot += partials[3 * (first + k) + 0];
    aa += partials[3 * (first + k) + 1];
    bb += partials[3 * (first + k) + 2];
  }
  const float3 r = block_sum3(dot, aa, bb);
  __shared__ float coef[2];
  if (threadIdx.x == 0) {
    // Horovod's guards: a (near-)zero operand keeps coefficient 1 (adasum(a, 0) == a)
    coef[0] = r.y >= 1e-30f ? 1.f - 0.5f * r.x / r.y : 1.f;
    coef[1] = r.z >= 1e-30f ? 1.f - 0.5f * r.x / r.z : 1.f;
  }
  __syncthreads();
  const float ca = coef[0], cb = coef[1];
  const int64_t lo = m.blk_lo[blockIdx.x], hi = m.blk_hi[blockIdx.x];
  const int64_t lo4 = (lo + 3) >> 2, hi4 = hi >> 2;
  if (lo4 < hi4) {
    for (int64_t i = lo4 + threadIdx.x; i < hi4; i += kAdasumThreads) {
      const float4 x = Vec4<T>::load(a, i), y = Vec4<T>::load(b, i);
      Vec4<T>::store(out, i, make_float4(ca * x.x + cb * y.x, ca * x.y + cb * y.y, ca * x.z + cb * y.z,
                                         ca * x.w + cb * y.w));
    }
    for (int64_t i = lo + threadIdx.x; i < (lo4 << 2); i += kAdasumThreads)
      Vec4<T>::store1(out, i, ca * Vec4<T>::load1(a, i) + cb * Vec4<T>::load1(b, i));
    for (int64_t i = (hi4 << 2) + threadIdx.x; i < hi; i += kAdasumThreads)
      Vec4<T>::store1(out, i, ca * Vec4<T>::load1(a, i) + cb * Vec4<T>::load1(b, i));
  } else {
    for (int64_t i = lo + threadIdx.x; i < hi; i += kAdasumThreads)
      Vec4<T>::store1(out, i, ca * Vec4<T>::load1(a, i) + cb * Vec4<T>::load1(b, i));
  }
}

#define ADASUM_DISPATCH(DTV, ALIAS, ...)                              \
  [&] {                                                               \
    if (DTV == kF32) { using ALIAS = float; __VA_ARGS__(); }          \
    else if (DTV == kBF16) { using ALIAS = BF16; __VA_ARGS__(); }     \
    else { using ALIAS = F16; __VA_ARGS__(); }                        \
  }()

void adasum_combine(uintptr_t a, uintptr_t b, uintptr_t out, int dt, uintptr_t meta, int64_t nblk, int64_t nseg,
                    uintptr_t partials, uintptr_t stream) {
  VODA_CHECK(nblk >= 0 && nseg >= 0, "negative table size");
  if (nblk == 0) return;
  VODA_CHECK(nblk <= int64_t(1) << 31, "too many blocks");
  ADASUM_DISPATCH(dt, T, [&] {
    hipLaunchKernelGGL((adasum_partials_kernel<T>), dim3(unsigned(nblk)), dim3(kAdasumThreads), 0,
                       as_stream(stream), reinterpret_cast<const T*>(a), reinterpret_cast<const T*>(b),
                       reinterpret_cast<const int64_t*>(meta), nblk, nseg, reinterpret_cast<float*>(partials));
    check_launch();
    hipLaunchKernelGGL((adasum_combine_kernel<T>), dim3(unsigned(nblk)), dim3(kAdasumThreads), 0,
                       as_stream(stream), reinterpret_cast<const T*>(a), reinterpret_cast<const T*>(b),
                       reinterpret_cast<T*>(out), reinterpret_cast<const int64_t*>(meta), nblk, nseg,
                       reinterpret_cast<const float*>(partials));
    check_launch();
  });
}

}  // namespace voda
