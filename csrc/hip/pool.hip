// Max pooling for channels_last (NHWC) activations: forward records the argmax as a 1-byte
// window offset, backward GATHERS (no atomics, no zero-fill pass): every input pixel sums
// the gradients of the <= ceil(k/s)^2 windows whose argmax it was.
//
// PyTorch's NHWC max_pool2d backward scatters into a zero-filled buffer and measured 0.62 ms
// per ResNet-50 (bs 256) step on MI355X (profiles/) for a 411 MB gradient; the gather form
// reads dy + the argmax bytes of the covering windows and writes each dx element once.
// A thread owns 8 consecutive channels of one pixel (16-byte bf16 loads/stores).
#include "common.h"
#include "ops.h"

namespace voda {

namespace {

struct PoolGeom {
  int N, H, W, C, Ho, Wo, k, s, p;
};

template <typename T> struct V8;
template <> struct V8<BF16> {
  using Raw = uint4;  // loaded now, converted later: many loads in flight per thread
  static __device__ __forceinline__ Raw load_raw(const BF16* p) { return *reinterpret_cast<const uint4*>(p); }
  static __device__ __forceinline__ void cvt(const Raw& u, float (&v)[8]) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) { v[2 * k] = bf2f(w[k] & 0xffff); v[2 * k + 1] = bf2f(w[k] >> 16); }
  }
  static __device__ __forceinline__ void load(const BF16* p, float (&v)[8]) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) { v[2 * k] = bf2f(w[k] & 0xffff); v[2 * k + 1] = bf2f(w[k] >> 16); }
  }
  static __device__ __forceinline__ void store(BF16* p, const float (&v)[8]) {
    uint4 u;
    u.x = uint32_t(f2bf(v[0])) | (uint32_t(f2bf(v[1])) << 16);
    u.y = uint32_t(f2bf(v[2])) | (uint32_t(f2bf(v[3])) << 16);
    u.z = uint32_t(f2bf(v[4])) | (uint32_t(f2bf(v[5])) << 16);
    u.w = uint32_t(f2bf(v[6])) | (uint32_t(f2bf(v[7])) << 16);
    *reinterpret_cast<uint4*>(p) = u;
  }
};
template <> struct V8<float> {
  struct Raw {
    float4 a, b;
  };
  static __device__ __forceinline__ Raw load_raw(const float* p) {
    return {*reinterpret_cast<const float4*>(p), *reinterpret_cast<const float4*>(p + 4)};
  }
  static __device__ __forceinline__ void cvt(const Raw& r, float (&v)[8]) {
    v[0] = r.a.x; v[1] = r.a.y; v[2] = r.a.z; v[3] = r.a.w; v[4] = r.b.x; v[5] = r.b.y; v[6] = r.b.z; v[7] = r.b.w;
  }
  static __device__ __forceinline__ void load(const float* p, float (&v)[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[8]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};

// One workgroup row per output (forward) / input (backward) pixel row: blockIdx.x = n * rows +
// row (scalar decode), threads over (column, channel group) of that row in 32-bit math.  The
// first version decoded a flat 64-bit index per element (three 64-bit div/mod sequences per
// thread) and ran VALU-bound at 2.5-3.5 TB/s (profiles/r2_rocprof_resnet50_final.md).
template <typename T>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ idx, PoolGeom g) {
  const int CG = g.C / 8;
  const int j = int(blockIdx.y) * 256 + int(threadIdx.x);
  if (j >= g.Wo * CG) return;
  const int n = int(blockIdx.x) / g.Ho, ho = int(blockIdx.x) % g.Ho;
  const int wo = j / CG, cg = j - wo * CG;
  float best[8];
  uint32_t arg[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) { best[c] = -__builtin_huge_valf(); arg[c] = 0; }
  const T* xn = x + int64_t(n) * g.H * g.W * g.C + cg * 8;
  for (int kh = 0; kh < g.k; ++kh) {
    const int h = ho * g.s - g.p + kh;
    if (h < 0 || h >= g.H) continue;
    for (int kw = 0; kw < g.k; ++kw) {
      const int w = wo * g.s - g.p + kw;
      if (w < 0 || w >= g.W) continue;
      float v[8];
      V8<T>::load(xn + (int64_t(h) * g.W + w) * g.C, v);
      const uint32_t o = uint32_t(kh * g.k + kw);
#pragma unroll
      for (int c = 0; c < 8; ++c)
        if (v[c] > best[c] || (v[c] != v[c] && best[c] == best[c])) { best[c] = v[c]; arg[c] = o; }
    }
  }
  const int64_t i = (int64_t(blockIdx.x) * g.Wo + wo) * CG + cg;
  V8<T>::store(y + i * 8, best);
  uint2 a;
  a.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
  a.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
  *reinterpret_cast<uint2*>(idx + i * 8) = a;
}

template <typename T>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                          T* __restrict__ dx, PoolGeom g) {
  const int CG = g.C / 8;
  const int j = int(blockIdx.y) * 256 + int(threadIdx.x);
  if (j >= g.W * CG) return;
  const int n = int(blockIdx.x) / g.H, h = int(blockIdx.x) % g.H;
  const int w = j / CG, cg = j - w * CG;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // windows (ho, wo) with ho*s - p <= h <= ho*s - p + k - 1
  const int ho0 = max(0, (h + g.p - g.k + g.s) / g.s), ho1 = min(g.Ho - 1, (h + g.p) / g.s);
  const int wo0 = max(0, (w + g.p - g.k + g.s) / g.s), wo1 = min(g.Wo - 1, (w + g.p) / g.s);
  const int64_t nbase = int64_t(n) * g.Ho * g.Wo * g.C + cg * 8;
  for (int ho = ho0; ho <= ho1; ++ho) {
    const int kh = h - (ho * g.s - g.p);
    if (kh < 0 || kh >= g.k) continue;
    for (int wo = wo0; wo <= wo1; ++wo) {
      const int kw = w - (wo * g.s - g.p);
      if (kw < 0 || kw >= g.k) continue;
      const int64_t o = nbase + (int64_t(ho) * g.Wo + wo) * g.C;
      const uint2 a = *reinterpret_cast<const uint2*>(idx + o);
      const uint32_t want = uint32_t(kh * g.k + kw);
      float d[8];
      V8<T>::load(dy + o, d);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const uint32_t ac = ((c < 4 ? a.x : a.y) >> (8 * (c & 3))) & 0xff;
        if (ac == want) acc[c] += d[c];
      }
    }
  }
  V8<T>::store(dx + ((int64_t(blockIdx.x) * g.W + w) * CG + cg) * 8, acc);
}

// Compile-time windows (ResNet's 3x3 / stride 2): every window load of a thread is issued
// before the first compare (clamped addresses, out-of-image taps masked afterwards).  The
// runtime-window kernels above branch between loads, so each thread waits on one load at
// a time: 3.3 TB/s forward, 2.4 TB/s backward on the 411 MB stem tensor (rocprofv3,
// profiles/raw/r2_stem_split_kernel_stats.csv).
template <typename T, int K, int S>
__global__ __launch_bounds__(256) void maxpool_fwd_fixed_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                                uint8_t* __restrict__ idx, PoolGeom g) {
  const int CG = g.C / 8;
  const int j = int(blockIdx.y) * 256 + int(threadIdx.x);
  if (j >= g.Wo * CG) return;
  const int n = int(blockIdx.x) / g.Ho, ho = int(blockIdx.x) % g.Ho;
  const int wo = j / CG, cg = j - wo * CG;
  const T* xn = x + int64_t(n) * g.H * g.W * g.C + cg * 8;
  const int h0 = ho * S - g.p, w0 = wo * S - g.p;
  typename V8<T>::Raw raw[K * K];
#pragma unroll
  for (int kh = 0; kh < K; ++kh) {
    const int hc = min(max(h0 + kh, 0), g.H - 1);
#pragma unroll
    for (int kw = 0; kw < K; ++kw) {
      const int wc = min(max(w0 + kw, 0), g.W - 1);
      raw[kh * K + kw] = V8<T>::load_raw(xn + (int64_t(hc) * g.W + wc) * g.C);
    }
  }
  float best[8];
  uint32_t arg[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) { best[c] = -__builtin_huge_valf(); arg[c] = 0; }
#pragma unroll
  for (int kh = 0; kh < K; ++kh) {
#pragma unroll
    for (int kw = 0; kw < K; ++kw) {
      const bool ok = unsigned(h0 + kh) < unsigned(g.H) && unsigned(w0 + kw) < unsigned(g.W);
      float v[8];
      V8<T>::cvt(raw[kh * K + kw], v);
#pragma unroll
      for (int c = 0; c < 8; ++c)
        if (ok && (v[c] > best[c] || (v[c] != v[c] && best[c] == best[c]))) { best[c] = v[c]; arg[c] = kh * K + kw; }
    }
  }
  const int64_t i = (int64_t(blockIdx.x) * g.Wo + wo) * CG + cg;
  V8<T>::store(y + i * 8, best);
  uint2 a;
  a.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
  a.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
  *reinterpret_cast<uint2*>(idx + i * 8) = a;
}

template <typename T, int K, int S>
__global__ __launch_bounds__(256) void maxpool_bwd_fixed_kernel(const T* __restrict__ dy,
                                                                const uint8_t* __restrict__ idx,
                                                                T* __restrict__ dx, PoolGeom g) {
  constexpr int NW = (K + S - 1) / S;  // windows per dimension covering a pixel
  const int CG = g.C / 8;
  const int j = int(blockIdx.y) * 256 + int(threadIdx.x);
  if (j >= g.W * CG) return;
  const int n = int(blockIdx.x) / g.H, h = int(blockIdx.x) % g.H;
  const int w = j / CG, cg = j - w * CG;
  const int ho0 = max(0, (h + g.p - K + S) / S), wo0 = max(0, (w + g.p - K + S) / S);
  const int64_t nbase = int64_t(n) * g.Ho * g.Wo * g.C + cg * 8;
  uint2 a[NW * NW];
  typename V8<T>::Raw raw[NW * NW];
#pragma unroll
  for (int dh = 0; dh < NW; ++dh) {
    const int hoc = min(ho0 + dh, g.Ho - 1);
#pragma unroll
    for (int dw = 0; dw < NW; ++dw) {
      const int64_t o = nbase + (int64_t(hoc) * g.Wo + min(wo0 + dw, g.Wo - 1)) * g.C;
      a[dh * NW + dw] = *reinterpret_cast<const uint2*>(idx + o);
      raw[dh * NW + dw] = V8<T>::load_raw(dy + o);
    }
  }
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int dh = 0; dh < NW; ++dh) {
    const int ho = ho0 + dh, kh = h - (ho * S - g.p);
#pragma unroll
    for (int dw = 0; dw < NW; ++dw) {
      const int wo = wo0 + dw, kw = w - (wo * S - g.p);
      const bool ok = ho < g.Ho && wo < g.Wo && unsigned(kh) < unsigned(K) && unsigned(kw) < unsigned(K);
      const uint32_t want = ok ? uint32_t(kh * K + kw) : 0x100u;  // 0x100 matches no byte
      float d[8];
      V8<T>::cvt(raw[dh * NW + dw], d);
      const uint2 u = a[dh * NW + dw];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const uint32_t ac = ((c < 4 ? u.x : u.y) >> (8 * (c & 3))) & 0xff;
        if (ac == want) acc[c] += d[c];
      }
    }
  }
  V8<T>::store(dx + ((int64_t(blockIdx.x) * g.W + w) * CG + cg) * 8, acc);
}

}  // namespace

void maxpool2d_fwd(uintptr_t x, uintptr_t y, uintptr_t idx, int N, int H, int W, int C, int Ho, int Wo, int k, int s,
                   int p, int dt, uintptr_t stream) {
  VODA_CHECK(C % 8 == 0 && k * k <= 255, "maxpool: C % 8 == 0 and k*k < 256 required");
  VODA_CHECK(int64_t(Wo) * (C / 8) < (int64_t(1) << 24) && int64_t(N) * Ho < (int64_t(1) << 31), "maxpool: shape too large");
  const PoolGeom g{N, H, W, C, Ho, Wo, k, s, p};
  const dim3 grid(unsigned(int64_t(N) * Ho), unsigned((Wo * (C / 8) + 255) / 256));
  const bool k3s2 = k == 3 && s == 2;
  if (dt == kBF16 && k3s2)
    hipLaunchKernelGGL((maxpool_fwd_fixed_kernel<BF16, 3, 2>), dim3(grid), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const BF16*>(x), reinterpret_cast<BF16*>(y), reinterpret_cast<uint8_t*>(idx), g);
  else if (dt == kF32 && k3s2)
    hipLaunchKernelGGL((maxpool_fwd_fixed_kernel<float, 3, 2>), dim3(grid), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const float*>(x), reinterpret_cast<float*>(y), reinterpret_cast<uint8_t*>(idx), g);
  else if (dt == kBF16)
    hipLaunchKernelGGL((maxpool_fwd_kernel<BF16>), dim3(grid), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const BF16*>(x), reinterpret_cast<BF16*>(y), reinterpret_cast<uint8_t*>(idx), g);
  else if (dt == kF32)
    hipLaunchKernelGGL((maxpool_fwd_kernel<float>), dim3(grid), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const float*>(x), reinterpret_cast<float*>(y), reinterpret_cast<uint8_t*>(idx), g);
  else
    throw std::invalid_argument("maxpool: dtype must be bf16 or fp32");
  check_launch();
}

void maxpool2d_bwd(uintptr_t dy, uintptr_t idx, uintptr_t dx, int N, int H, int W, int C, int Ho, int Wo, int k, int s,
                   int p, int dt, uintptr_t stream) {
  VODA_CHECK(C % 8 == 0, "maxpool: C % 8 == 0 required");
  VODA_CHECK(int64_t(W) * (C / 8) < (int64_t(1) << 24) && int64_t(N) * H < (int64_t(1) << 31), "maxpool: shape too large");
  const PoolGeom g{N, H, W, C, Ho, Wo, k, s, p};
  const dim3 grid(unsigned(int64_t(N) * H), unsigned((W * (C / 8) + 255) / 256));
  const bool k3s2 = k == 3 && s == 2;
  if (dt == kBF16 && k3s2)
    hipLaunchKernelGGL((maxpool_bwd_fixed_kernel<BF16, 3, 2>), dim3(grid), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const BF16*>(dy), reinterpret_cast<const uint8_t*>(idx), reinterpret_cast<BF16*>(dx), g);
  else if (dt == kF32 && k3s2)
    hipLaunchKernelGGL((maxpool_bwd_fixed_kernel<float, 3, 2>), dim3(grid), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const float*>(dy), reinterpret_cast<const uint8_t*>(idx), reinterpret_cast<float*>(dx), g);
  else if (dt == kBF16)
    hipLaunchKernelGGL((maxpool_bwd_kernel<BF16>), dim3(grid), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const BF16*>(dy), reinterpret_cast<const uint8_t*>(idx), reinterpret_cast<BF16*>(dx), g);
  else if (dt == kF32)
    hipLaunchKernelGGL((maxpool_bwd_kernel<float>), dim3(grid), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const float*>(dy), reinterpret_cast<const uint8_t*>(idx), reinterpret_cast<float*>(dx), g);
  else
    throw std::invalid_argument("maxpool: dtype must be bf16 or fp32");
  check_launch();
}

// ---- global average pool backward (ResNet head): dx[n][hw][c] = g[n][c] * scale written
// straight into the channels_last layout.  Autograd's expand-then-contiguous ran as two
// strided copy kernels, 23 + 83 us per ResNet-50 bs-256 step for a 51 MB write (0.6 TB/s);
// here a thread writes 8 channels (16 B) of one pixel.
namespace {
template <typename TG, typename TO>
__global__ __launch_bounds__(256) void gap_bwd_kernel(const TG* __restrict__ g, TO* __restrict__ dx, int HW, int C,
                                                      float scale) {
  const int CG = C / 8;
  const int j = int(blockIdx.y) * 256 + int(threadIdx.x);
  if (j >= HW * CG) return;
  const int n = blockIdx.x;
  const int px = j / CG, cg = j - px * CG;
  float v[8];
  V8<TG>::load(g + int64_t(n) * C + cg * 8, v);
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] *= scale;
  V8<TO>::store(dx + (int64_t(n) * HW + px) * C + cg * 8, v);
}
}  // namespace

void global_avgpool_bwd(uintptr_t g, uintptr_t dx, int N, int HW, int C, float scale, int g_dt, int dt,
                        uintptr_t stream) {
  VODA_CHECK(C % 8 == 0, "global_avgpool_bwd: C must be a multiple of 8");
  VODA_CHECK(g % 16 == 0 && dx % 16 == 0, "global_avgpool_bwd: misaligned operands");
  if (int64_t(N) * HW == 0) return;
  const dim3 grid(unsigned(N), unsigned((int64_t(HW) * (C / 8) + 255) / 256));
  hipStream_t s = as_stream(stream);
  auto go = [&](auto gt, auto ot) {
    using TG = decltype(gt);
    using TO = decltype(ot);
    hipLaunchKernelGGL((gap_bwd_kernel<TG, TO>), grid, dim3(256), 0, s, reinterpret_cast<const TG*>(g),
                       reinterpret_cast<TO*>(dx), HW, C, scale);
  };
  if (g_dt == kF32 && dt == kBF16) go(float{}, BF16{});
  else if (g_dt == kBF16 && dt == kBF16) go(BF16{}, BF16{});
  else if (g_dt == kF32 && dt == kF32) go(float{}, float{});
  else throw std::invalid_argument("global_avgpool_bwd: unsupported dtypes");
  check_launch();
}

// ---- stride-s pixel subsampling of a channels_last tensor (the input of ResNet's stride-2
// 1x1 downsample convolutions) and its adjoint, dx[:, :, ::s, ::s] += g.  PyTorch runs both
// as generic strided elementwise kernels (69 + 38 + 21 us forward, 61 + 33 + 19 us backward
// per ResNet-50 bs-256 step, 2.7-3.4 TB/s); a thread here moves 8 channels of one pixel (16 B
// bf16, 32 B fp32: the fp32 strided add took 65 us per call as a PyTorch kernel).
namespace {
template <typename T, bool ADD>
__global__ __launch_bounds__(256) void subsample_kernel(const T* __restrict__ src, T* __restrict__ dst, int H, int W,
                                                        int C, int Ho, int Wo, int s) {
  const int CG = C / 8;
  const int j = int(blockIdx.y) * 256 + int(threadIdx.x);
  if (j >= Wo * CG) return;
  const int nho = blockIdx.x;
  const int n = nho / Ho, ho = nho - (nho / Ho) * Ho;
  const int wo = j / CG, cg = j - wo * CG;
  const int64_t full = ((int64_t(n) * H + int64_t(ho) * s) * W + int64_t(wo) * s) * C + cg * 8;
  const int64_t sub = (int64_t(nho) * Wo + wo) * C + cg * 8;
  if constexpr (!ADD) {
    float a[8];  // gather
    V8<T>::load(src + full, a);
    V8<T>::store(dst + sub, a);
  } else {
    float a[8], b[8];
    V8<T>::load(src + sub, a);   // g (subsampled)
    V8<T>::load(dst + full, b);  // dx (full resolution), updated in place
#pragma unroll
    for (int k = 0; k < 8; ++k) b[k] += a[k];
    V8<T>::store(dst + full, b);
  }
}
}  // namespace

void subsample2d(uintptr_t src, uintptr_t dst, int N, int H, int W, int C, int s, bool add, int dt,
                 uintptr_t stream) {
  VODA_CHECK(C % 8 == 0 && s >= 1, "subsample2d: C must be a multiple of 8");
  VODA_CHECK(src % 16 == 0 && dst % 16 == 0, "subsample2d: misaligned operands");
  const int Ho = (H + s - 1) / s, Wo = (W + s - 1) / s;
  if (int64_t(N) * Ho * Wo == 0) return;
  const dim3 grid(unsigned(N * Ho), unsigned((int64_t(Wo) * (C / 8) + 255) / 256));
  hipStream_t st = as_stream(stream);
  VODA_CHECK(dt == kBF16 || dt == kF32, "subsample2d: bf16 / fp32 activations only");
  auto go = [&](auto tag) {
    using T = decltype(tag);
    const T* a = reinterpret_cast<const T*>(src);
    T* b = reinterpret_cast<T*>(dst);
    if (add) hipLaunchKernelGGL((subsample_kernel<T, true>), grid, dim3(256), 0, st, a, b, H, W, C, Ho, Wo, s);
    else hipLaunchKernelGGL((subsample_kernel<T, false>), grid, dim3(256), 0, st, a, b, H, W, C, Ho, Wo, s);
  };
  if (dt == kF32) go(float{});
  else go(BF16{});
  check_launch();
}

}  // namespace voda
