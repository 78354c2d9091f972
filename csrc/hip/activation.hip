// tanh-approximated GELU forward / backward (the BERT / Keras-Transformer FFN activation).
//
// The FFN pre-activation h = x W1^T + b1 ([tokens, 4*d], 50 MB bf16 per BERT-base layer at
// batch 64 x 128) is the largest activation of the transformer step; PyTorch's elementwise
// GELU kernels ran at ~60 % of HBM bandwidth (0.62 ms per step, profiles/).  Here every lane
// moves 16 B per access (8 bf16), the math is fp32 with one v_exp_f32 + one v_rcp_f32 per element, and the
// backward writes dh into a separate buffer the caller allocates (dy may still be read by others).
//
//   g(h)  = 0.5 h (1 + tanh(u)),             u = k (h + c h^3), k = sqrt(2/pi), c = 0.044715
//   g'(h) = 0.5 (1 + t) + 0.5 h (1 - t^2) k (1 + 3 c h^2)
#include "common.h"
#include "ops.h"

namespace voda {

namespace {

constexpr int kBlock = 256;
// 8 elements per lane as ONE 16 B access for 16-bit types (two for fp32)
template <typename T> struct Pack8;
template <typename T> struct Pack8Half {  // bf16 / fp16: uint4 = 8 x 16 bit
  static __device__ __forceinline__ void load(const T* p, int64_t i, float (&v)[8]) {
    const uint4 u = reinterpret_cast<const uint4*>(p)[i];
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = Vec4<T>::load1(reinterpret_cast<const T*>(&w[k]), 0);
      v[2 * k + 1] = Vec4<T>::load1(reinterpret_cast<const T*>(&w[k]), 1);
    }
  }
  static __device__ __forceinline__ void store(T* p, int64_t i, const float (&v)[8]) {
    alignas(16) T q[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) Vec4<T>::store1(q, k, v[k]);
    reinterpret_cast<uint4*>(p)[i] = *reinterpret_cast<const uint4*>(q);
  }
};
template <> struct Pack8<BF16> : Pack8Half<BF16> {};
template <> struct Pack8<F16> : Pack8Half<F16> {};
template <> struct Pack8<float> {
  static __device__ __forceinline__ void load(const float* p, int64_t i, float (&v)[8]) {
    const float4 a = reinterpret_cast<const float4*>(p)[2 * i], b = reinterpret_cast<const float4*>(p)[2 * i + 1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, int64_t i, const float (&v)[8]) {
    reinterpret_cast<float4*>(p)[2 * i] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[2 * i + 1] = make_float4(v[4], v[5], v[6], v[7]);
  }
};

// kItems 8-element groups per lane, all loads issued before any math (bytes in flight);
// the grid covers the tensor in one pass (no grid-stride tail imbalance)
constexpr int kItems = 2;

template <typename T>
__global__ __launch_bounds__(kBlock) void gelu_fwd_kernel(const T* __restrict__ h, T* __restrict__ y, int64_t n8,
                                                          int64_t n) {
  const int64_t base = int64_t(blockIdx.x) * (kBlock * kItems) + threadIdx.x;
  float v[kItems][8];
#pragma unroll
  for (int k = 0; k < kItems; ++k)
    if (base + k * kBlock < n8) Pack8<T>::load(h, base + k * kBlock, v[k]);
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    if (base + k * kBlock >= n8) continue;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[k][e] = gelu_tanh_f(v[k][e]);
    Pack8<T>::store(y, base + k * kBlock, v[k]);
  }
  if (blockIdx.x == gridDim.x - 1)  // < 8 tail elements
    for (int64_t j = n8 * 8 + threadIdx.x; j < n; j += kBlock) Vec4<T>::store1(y, j, gelu_tanh_f(Vec4<T>::load1(h, j)));
}

template <typename T>
__global__ __launch_bounds__(kBlock) void gelu_bwd_kernel(const T* __restrict__ h, const T* dy, T* dh, int64_t n8,
                                                          int64_t n) {
  // dy and dh may alias (in-place backward): no __restrict__ on them
  const int64_t base = int64_t(blockIdx.x) * (kBlock * kItems) + threadIdx.x;
  float v[kItems][8], g[kItems][8];
#pragma unroll
  for (int k = 0; k < kItems; ++k)
    if (base + k * kBlock < n8) {
      Pack8<T>::load(h, base + k * kBlock, v[k]);
      Pack8<T>::load(dy, base + k * kBlock, g[k]);
    }
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    if (base + k * kBlock >= n8) continue;
#pragma unroll
    for (int e = 0; e < 8; ++e) g[k][e] *= gelu_tanh_grad(v[k][e]);
    Pack8<T>::store(dh, base + k * kBlock, g[k]);
  }
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t j = n8 * 8 + threadIdx.x; j < n; j += kBlock)
      Vec4<T>::store1(dh, j, Vec4<T>::load1(dy, j) * gelu_tanh_grad(Vec4<T>::load1(h, j)));
}

template <typename F>
void dispatch(int dt, F&& f) {
  if (dt == kBF16) f(BF16{});
  else if (dt == kF16) f(F16{});
  else if (dt == kF32) f(float{});
  else VODA_CHECK(false, "gelu: unsupported dtype");
}

unsigned gelu_grid(int64_t n8) {
  const int64_t g = (n8 + kBlock * kItems - 1) / (kBlock * kItems);
  VODA_CHECK(g < (int64_t(1) << 31), "gelu: tensor too large");
  return unsigned(g < 1 ? 1 : g);
}

}  // namespace

void gelu_tanh_fwd(uintptr_t h, uintptr_t y, int64_t n, int dt, uintptr_t stream) {
  if (n == 0) return;
  const int64_t n8 = n / 8;
  dispatch(dt, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(gelu_fwd_kernel<T>, dim3(gelu_grid(n8)), dim3(kBlock), 0, as_stream(stream),
                       reinterpret_cast<const T*>(h), reinterpret_cast<T*>(y), n8, n);
  });
  check_launch();
}

void gelu_tanh_bwd(uintptr_t h, uintptr_t dy, uintptr_t dh, int64_t n, int dt, uintptr_t stream) {
  if (n == 0) return;
  const int64_t n8 = n / 8;
  dispatch(dt, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(gelu_bwd_kernel<T>, dim3(gelu_grid(n8)), dim3(kBlock), 0, as_stream(stream),
                       reinterpret_cast<const T*>(h), reinterpret_cast<const T*>(dy), reinterpret_cast<T*>(dh),
                       n8, n);
  });
  check_launch();
}

}  // namespace voda
