// Fused optimizer steps over flat fp32 master buffers (CDNA4 / gfx950).
//
// The reference workloads run SGD+momentum (ResNet50/VGG16, torch MNIST), Adam (Keras
// MNIST) and RMSprop (InceptionV3, Transformer) through TF/PyTorch per-parameter ops
// (reference examples/py/tensorflow2/tensorflow2_keras_cifar_elastic.py:156-164,
// examples/py/pytorch/pytorch_mnist_elastic.py:112-113).  Here every
// parameter of a job lives in ONE flat fp32 buffer, so a step is ONE HBM-streaming
// launch: param/grad/state are read once and written once with 16-B (f32) or 8-B
// (bf16/f16) accesses per lane, one float4 group per thread (opt_grid; the loops still
// grid-stride, so any grid is correct).
// Optionally the kernel also emits a low-precision copy of the updated weights
// (bf16/f16 model weights + fp32 master), fusing the cast that would otherwise be a
// second pass.  Semantics match torch.optim.{SGD,Adam,AdamW,RMSprop}.
#include "common.h"

#include <cstdlib>
#include "ops.h"

namespace voda {

struct NoLP {};

template <typename LP>
__device__ __forceinline__ void store_lp(LP* q, int64_t i4, float4 v) { Vec4<LP>::store(q, i4, v); }
template <>
__device__ __forceinline__ void store_lp<NoLP>(NoLP*, int64_t, float4) {}
template <typename LP>
__device__ __forceinline__ void store_lp1(LP* q, int64_t i, float v) { Vec4<LP>::store1(q, i, v); }
template <>
__device__ __forceinline__ void store_lp1<NoLP>(NoLP*, int64_t, float) {}

#define F4_APPLY(OUT, EXPR_X, EXPR_Y, EXPR_Z, EXPR_W) \
  OUT.x = (EXPR_X); OUT.y = (EXPR_Y); OUT.z = (EXPR_Z); OUT.w = (EXPR_W);

// ---------------------------------------------------------------------------------
// SGD (+momentum, dampening, nesterov, L2 weight decay), torch.optim.SGD semantics.
// ---------------------------------------------------------------------------------
struct SgdArgs {
  float lr, momentum, dampening, wd, grad_scale;
  int nesterov, first_step;
};

__device__ __forceinline__ float sgd1(float& p, float g, float& b, const SgdArgs& a) {
  g = g * a.grad_scale + a.wd * p;
  if (a.momentum != 0.f) {
    b = a.first_step ? g : a.momentum * b + (1.f - a.dampening) * g;
    g = a.nesterov ? g + a.momentum * b : b;
  }
  p -= a.lr * g;
  return p;
}

template <typename GT, typename LP>
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, const GT* __restrict__ g,
                                                  float* __restrict__ buf, LP* __restrict__ q,
                                                  int64_t n, SgdArgs a) {
  const int64_t n4 = n >> 2;
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  const bool mom = a.momentum != 0.f;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = Vec4<float>::load(p, i);
    float4 gv = Vec4<GT>::load(g, i);
    float4 bv = mom ? Vec4<float>::load(buf, i) : make_float4(0.f, 0.f, 0.f, 0.f);
    sgd1(pv.x, gv.x, bv.x, a);
    sgd1(pv.y, gv.y, bv.y, a);
    sgd1(pv.z, gv.z, bv.z, a);
    sgd1(pv.w, gv.w, bv.w, a);
    Vec4<float>::store(p, i, pv);
    if (mom) Vec4<float>::store(buf, i, bv);
    store_lp<LP>(q, i, pv);
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += blockDim.x) {
      float pv = p[i], bv = mom ? buf[i] : 0.f;
      sgd1(pv, Vec4<GT>::load1(g, i), bv, a);
      p[i] = pv;
      if (mom) buf[i] = bv;
      store_lp1<LP>(q, i, pv);
    }
  }
}

// ---------------------------------------------------------------------------------
// Adam / AdamW, torch.optim.Adam(W) semantics (no amsgrad).
// ---------------------------------------------------------------------------------
struct AdamArgs {
  float lr, beta1, beta2, eps, wd, grad_scale;
  float step_size;     // lr / bias_correction1
  float inv_sqrt_bc2;  // 1 / sqrt(bias_correction2)
  int adamw;
};

__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, const AdamArgs& a) {
  g *= a.grad_scale;
  if (a.adamw) p *= (1.f - a.lr * a.wd);
  else g += a.wd * p;
  m = a.beta1 * m + (1.f - a.beta1) * g;
  v = a.beta2 * v + (1.f - a.beta2) * g * g;
  const float denom = sqrtf(v) * a.inv_sqrt_bc2 + a.eps;
  p -= a.step_size * (m / denom);
}

// One float4 group of every array per thread.  Two groups in flight
// were measured equal within noise (110 M-parameter AdamW step, benchmarks/bench_adam.py:
// 708 / 690 us with a bf16 copy, 669 / 686 us without; profiles/r4/bench_adam_variants.log) and
// were removed in round 5; non-temporal state stores did not help either.
template <typename GT, typename LP>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const GT* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   LP* __restrict__ q, int64_t n, AdamArgs a,
                                                   const int64_t* __restrict__ dstep) {
  if (dstep != nullptr) {
    // step counter read on the device: the launch stays valid inside a captured hipGraph
    // that is replayed every step (the counter is advanced by a captured add before us)
    const float t = float(*dstep);
    a.step_size = a.lr / (1.f - powf(a.beta1, t));
    a.inv_sqrt_bc2 = rsqrtf(1.f - powf(a.beta2, t));
  }
  const int64_t n4 = n >> 2;
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i < n4; i += stride) {
    float4 pv = Vec4<float>::load(p, i);
    float4 gv = Vec4<GT>::load(g, i);
    float4 mv = Vec4<float>::load(m, i);
    float4 vv = Vec4<float>::load(v, i);
    adam1(pv.x, gv.x, mv.x, vv.x, a);
    adam1(pv.y, gv.y, mv.y, vv.y, a);
    adam1(pv.z, gv.z, mv.z, vv.z, a);
    adam1(pv.w, gv.w, mv.w, vv.w, a);
    Vec4<float>::store(p, i, pv);
    Vec4<float>::store(m, i, mv);
    Vec4<float>::store(v, i, vv);
    store_lp<LP>(q, i, pv);
  }
  if (blockIdx.x == 0) {
    for (int64_t j = (n4 << 2) + threadIdx.x; j < n; j += blockDim.x) {
      float pv = p[j], mv = m[j], vv = v[j];
      adam1(pv, Vec4<GT>::load1(g, j), mv, vv, a);
      p[j] = pv; m[j] = mv; v[j] = vv;
      store_lp1<LP>(q, j, pv);
    }
  }
}

// ---------------------------------------------------------------------------------
// RMSprop (+momentum, centered), torch.optim.RMSprop semantics.
// ---------------------------------------------------------------------------------
struct RmsArgs {
  float lr, alpha, eps, wd, momentum, grad_scale;
  int centered;
};

__device__ __forceinline__ void rms1(float& p, float g, float& sq, float& b, float& ga, const RmsArgs& a) {
  g = g * a.grad_scale + a.wd * p;
  sq = a.alpha * sq + (1.f - a.alpha) * g * g;
  float avg;
  if (a.centered) {
    ga = a.alpha * ga + (1.f - a.alpha) * g;
    avg = sqrtf(sq - ga * ga) + a.eps;
  } else {
    avg = sqrtf(sq) + a.eps;
  }
  if (a.momentum > 0.f) {
    b = a.momentum * b + g / avg;
    p -= a.lr * b;
  } else {
    p -= a.lr * g / avg;
  }
}

template <typename GT, typename LP>
__global__ __launch_bounds__(256) void rmsprop_kernel(float* __restrict__ p, const GT* __restrict__ g,
                                                      float* __restrict__ sq, float* __restrict__ buf,
                                                      float* __restrict__ gavg, LP* __restrict__ q,
                                                      int64_t n, RmsArgs a) {
  const int64_t n4 = n >> 2;
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  const bool mom = a.momentum > 0.f;
  const bool cen = a.centered != 0;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = Vec4<float>::load(p, i);
    float4 gv = Vec4<GT>::load(g, i);
    float4 sv = Vec4<float>::load(sq, i);
    float4 bv = mom ? Vec4<float>::load(buf, i) : z;
    float4 av = cen ? Vec4<float>::load(gavg, i) : z;
    rms1(pv.x, gv.x, sv.x, bv.x, av.x, a);
    rms1(pv.y, gv.y, sv.y, bv.y, av.y, a);
    rms1(pv.z, gv.z, sv.z, bv.z, av.z, a);
    rms1(pv.w, gv.w, sv.w, bv.w, av.w, a);
    Vec4<float>::store(p, i, pv);
    Vec4<float>::store(sq, i, sv);
    if (mom) Vec4<float>::store(buf, i, bv);
    if (cen) Vec4<float>::store(gavg, i, av);
    store_lp<LP>(q, i, pv);
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += blockDim.x) {
      float pv = p[i], sv = sq[i], bv = mom ? buf[i] : 0.f, av = cen ? gavg[i] : 0.f;
      rms1(pv, Vec4<GT>::load1(g, i), sv, bv, av, a);
      p[i] = pv; sq[i] = sv;
      if (mom) buf[i] = bv;
      if (cen) gavg[i] = av;
      store_lp1<LP>(q, i, pv);
    }
  }
}

// ---------------------------------------------------------------------------------
// Host launchers: dtype dispatch.
// ---------------------------------------------------------------------------------
#define DISPATCH_GT_LP(GDT, LDT, ...)                                                   \
  [&] {                                                                                 \
    if (GDT == kF32) {                                                                  \
      using GT = float;                                                                 \
      if (LDT < 0) { using LP = NoLP; __VA_ARGS__(); }                                   \
      else if (LDT == kBF16) { using LP = BF16; __VA_ARGS__(); }                         \
      else { using LP = F16; __VA_ARGS__(); }                                            \
    } else if (GDT == kBF16) {                                                          \
      using GT = BF16;                                                                  \
      if (LDT < 0) { using LP = NoLP; __VA_ARGS__(); }                                   \
      else if (LDT == kBF16) { using LP = BF16; __VA_ARGS__(); }                         \
      else { using LP = F16; __VA_ARGS__(); }                                            \
    } else {                                                                            \
      using GT = F16;                                                                   \
      if (LDT < 0) { using LP = NoLP; __VA_ARGS__(); }                                   \
      else if (LDT == kBF16) { using LP = BF16; __VA_ARGS__(); }                         \
      else { using LP = F16; __VA_ARGS__(); }                                            \
    }                                                                                   \
  }()

// One float4 group per thread: the 110 M-parameter AdamW step takes 555 us (5.55 TB/s, above a
// plain device copy's 5.32) against 678-734 us with the grid capped at 1024-8192 blocks
// (benchmarks/bench_adam.py, profiles/r5/optim_grid_cap.jsonl).
unsigned opt_grid(int64_t n) { return stream_grid((n + 3) / 4); }

void sgd_step(uintptr_t p, uintptr_t g, int g_dtype, uintptr_t mom_buf, uintptr_t p_lp, int lp_dtype,
              int64_t n, float lr, float momentum, float dampening, float wd, bool nesterov,
              bool first_step, float grad_scale, uintptr_t stream) {
  VODA_CHECK(n >= 0, "negative size");
  VODA_CHECK(momentum == 0.f || mom_buf != 0, "momentum buffer required");
  if (n == 0) return;
  SgdArgs a{lr, momentum, dampening, wd, grad_scale, nesterov ? 1 : 0, first_step ? 1 : 0};
  unsigned grid = opt_grid(n);
  DISPATCH_GT_LP(g_dtype, lp_dtype, [&] {
    hipLaunchKernelGGL((sgd_kernel<GT, LP>), dim3(grid), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<float*>(p), reinterpret_cast<const GT*>(g),
                       reinterpret_cast<float*>(mom_buf), reinterpret_cast<LP*>(p_lp), n, a);
  });
  check_launch();
}

void adam_step(uintptr_t p, uintptr_t g, int g_dtype, uintptr_t m, uintptr_t v, uintptr_t p_lp,
               int lp_dtype, int64_t n, float lr, float beta1, float beta2, float eps, float wd,
               bool adamw, int64_t step, float grad_scale, uintptr_t step_ptr, uintptr_t stream) {
  VODA_CHECK(step >= 1 || step_ptr != 0, "adam step counter must start at 1");
  if (n == 0) return;
  const double st = double(std::max<int64_t>(step, 1));
  const double bc1 = 1.0 - std::pow(double(beta1), st);
  const double bc2 = 1.0 - std::pow(double(beta2), st);
  AdamArgs a{lr, beta1, beta2, eps, wd, grad_scale, float(lr / bc1), float(1.0 / std::sqrt(bc2)),
             adamw ? 1 : 0};
  unsigned grid = opt_grid(n);
  DISPATCH_GT_LP(g_dtype, lp_dtype, [&] {
    hipLaunchKernelGGL((adam_kernel<GT, LP>), dim3(grid), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<float*>(p), reinterpret_cast<const GT*>(g),
                       reinterpret_cast<float*>(m), reinterpret_cast<float*>(v),
                       reinterpret_cast<LP*>(p_lp), n, a, reinterpret_cast<const int64_t*>(step_ptr));
  });
  check_launch();
}

void rmsprop_step(uintptr_t p, uintptr_t g, int g_dtype, uintptr_t sq, uintptr_t mom_buf, uintptr_t gavg,
                  uintptr_t p_lp, int lp_dtype, int64_t n, float lr, float alpha, float eps, float wd,
                  float momentum, bool centered, float grad_scale, uintptr_t stream) {
  VODA_CHECK(momentum <= 0.f || mom_buf != 0, "momentum buffer required");
  VODA_CHECK(!centered || gavg != 0, "grad-average buffer required for centered RMSprop");
  if (n == 0) return;
  RmsArgs a{lr, alpha, eps, wd, momentum, grad_scale, centered ? 1 : 0};
  unsigned grid = opt_grid(n);
  DISPATCH_GT_LP(g_dtype, lp_dtype, [&] {
    hipLaunchKernelGGL((rmsprop_kernel<GT, LP>), dim3(grid), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<float*>(p), reinterpret_cast<const GT*>(g),
                       reinterpret_cast<float*>(sq), reinterpret_cast<float*>(mom_buf),
                       reinterpret_cast<float*>(gavg), reinterpret_cast<LP*>(p_lp), n, a);
  });
  check_launch();
}

}  // namespace voda
