// Gradient-bucket pack / scale / cast kernels (CDNA4 / gfx950).
//
// Horovod's fusion buffer ("collects per-gradient allreduce requests,
// packs them into a fusion buffer, runs one collective and unpacks, averaging by 1/N")
// and its fp16 compression (reference examples/py/pytorch/pytorch_mnist_elastic.py:116,
// tensorflow2_keras_cifar_elastic.py:145) become two launch shapes here:
//   * cast_scale: one flat bucket -> comm buffer (fp32 -> bf16/fp16 with the 1/N average
//     folded in) and back; the grads already live as views of the flat bucket, so no
//     gather is needed on the hot path.
//   * multi_tensor_copy: an arbitrary tensor list <-> one flat buffer in ONE launch
//     (the table travels in the kernel arguments), used for state broadcast on elastic
//     resize and for models whose params cannot be re-pointed into flat storage.
#include "common.h"
#include "ops.h"

namespace voda {

template <typename ST, typename DT>
__global__ __launch_bounds__(256) void cast_scale_kernel(const ST* __restrict__ src, DT* __restrict__ dst,
                                                         int64_t n, float scale) {
  const int64_t n4 = n >> 2;
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = Vec4<ST>::load(src, i);
    v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
    Vec4<DT>::store(dst, i, v);
  }
  if (blockIdx.x == 0)
    for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += blockDim.x)
      Vec4<DT>::store1(dst, i, Vec4<ST>::load1(src, i) * scale);
}

#define DISPATCH_DT(DTV, ALIAS, ...)                   \
  [&] {                                                \
    if (DTV == kF32) { using ALIAS = float; __VA_ARGS__(); }  \
    else if (DTV == kBF16) { using ALIAS = BF16; __VA_ARGS__(); } \
    else { using ALIAS = F16; __VA_ARGS__(); }          \
  }()

void cast_scale(uintptr_t src, int src_dt, uintptr_t dst, int dst_dt, int64_t n, float scale,
                uintptr_t stream) {
  VODA_CHECK(n >= 0, "negative size");
  if (n == 0) return;
  unsigned grid = stream_grid((n + 3) / 4);
  DISPATCH_DT(src_dt, ST, [&] {
    DISPATCH_DT(dst_dt, DT, [&] {
      hipLaunchKernelGGL((cast_scale_kernel<ST, DT>), dim3(grid), dim3(256), 0, as_stream(stream),
                         reinterpret_cast<const ST*>(src), reinterpret_cast<DT*>(dst), n, scale);
    });
  });
  check_launch();
}

// ---------------------------------------------------------------------------------
// multi-tensor copy: blockIdx.y selects the tensor, blockIdx.x grid-strides over it.
// ---------------------------------------------------------------------------------
constexpr int kMaxTensorsPerLaunch = 64;
struct TensorTable {
  const void* src[kMaxTensorsPerLaunch];
  void* dst[kMaxTensorsPerLaunch];
  int64_t n[kMaxTensorsPerLaunch];
};

template <typename ST, typename DT>
__global__ __launch_bounds__(256) void multi_copy_kernel(TensorTable t, float scale) {
  const ST* __restrict__ src = reinterpret_cast<const ST*>(t.src[blockIdx.y]);
  DT* __restrict__ dst = reinterpret_cast<DT*>(t.dst[blockIdx.y]);
  const int64_t n = t.n[blockIdx.y];
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  const int64_t tid = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  // vector path only when both sides are aligned for a 4-element access (wave-uniform)
  const uintptr_t amask = (uintptr_t(src) % (4 * sizeof(ST))) | (uintptr_t(dst) % (4 * sizeof(DT)));
  int64_t done = 0;
  if (amask == 0) {
    const int64_t n4 = n >> 2;
    for (int64_t i = tid; i < n4; i += stride) {
      float4 v = Vec4<ST>::load(src, i);
      v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
      Vec4<DT>::store(dst, i, v);
    }
    done = n4 << 2;
  }
  for (int64_t i = done + tid; i < n; i += stride) Vec4<DT>::store1(dst, i, Vec4<ST>::load1(src, i) * scale);
}

void multi_tensor_copy(const std::vector<uintptr_t>& srcs, const std::vector<uintptr_t>& dsts,
                       const std::vector<int64_t>& ns, int src_dt, int dst_dt, float scale,
                       uintptr_t stream) {
  VODA_CHECK(srcs.size() == dsts.size() && srcs.size() == ns.size(), "table size mismatch");
  for (size_t base = 0; base < srcs.size(); base += kMaxTensorsPerLaunch) {
    const size_t cnt = std::min<size_t>(kMaxTensorsPerLaunch, srcs.size() - base);
    TensorTable t{};
    int64_t maxn = 0;
    for (size_t k = 0; k < cnt; ++k) {
      t.src[k] = reinterpret_cast<const void*>(srcs[base + k]);
      t.dst[k] = reinterpret_cast<void*>(dsts[base + k]);
      t.n[k] = ns[base + k];
      VODA_CHECK(ns[base + k] >= 0, "negative size");
      maxn = std::max(maxn, ns[base + k]);
    }
    if (maxn == 0) continue;
    int64_t gx = (maxn / 4 + 255) / 256;
    gx = std::max<int64_t>(1, std::min<int64_t>(gx, 512));
    DISPATCH_DT(src_dt, ST, [&] {
      DISPATCH_DT(dst_dt, DT, [&] {
        hipLaunchKernelGGL((multi_copy_kernel<ST, DT>), dim3(unsigned(gx), unsigned(cnt)), dim3(256), 0,
                           as_stream(stream), t, scale);
      });
    });
    check_launch();
  }
}

}  // namespace voda
