// Fused softmax cross-entropy over the rows of a logits matrix (CDNA4, gfx950).
//
//   lse[r]     = log sum_{c < V} exp(x[r][c])
//   loss[r]    = lse[r] - x[r][label[r]]                 (0 for label == ignore)
//   correct[r] = argmax_{c < V} x[r][c] == label[r]      (first maximum, as torch.argmax)
//   dx[r][c]   = scale * (exp(x[r][c] - lse[r]) - [c == label[r]])   c < V, else 0
//
// The stock path (logits.float() -> log_softmax -> nll_loss -> argmax, and the same chain
// backwards) reads and writes the vocab-sized logits about eight times in fp32; here the
// forward reads the bf16 logits once and the backward reads them once and writes dx once
// (profiles/: BERT-base MLM head 1280 x 30522, NMT head 10240 x 15000).  Columns V .. ld-1
// are padding of a vocab rounded up for 16-byte rows: excluded from the softmax, zero in dx.
//
// One 256-thread workgroup per row; each lane streams 16-byte vectors and keeps an online
// (max, sum-exp) pair plus its argmax, merged across the wave by butterfly shuffles and
// across the 4 waves through LDS.  NaN / inf logits propagate into lse and the loss (the
// trainer's replay guard relies on a non-finite loss).  The mean over non-ignored rows and
// the backward scale stay on the device (no host sync: hipGraph-capturable).
#include "common.h"
#include "ops.h"

namespace voda {

namespace {

constexpr int kXentThreads = 256;
constexpr float kLog2e = 1.4426950408889634f;

template <typename T> struct XVec;
template <> struct XVec<BF16> {
  static constexpr int N = 8;
  static __device__ __forceinline__ void load(const BF16* p, float* v) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = bf2f(w[i] & 0xffff);
      v[2 * i + 1] = bf2f(w[i] >> 16);
    }
  }
  static __device__ __forceinline__ void store(BF16* p, const float* v) {
    uint4 u;
    u.x = uint32_t(f2bf(v[0])) | (uint32_t(f2bf(v[1])) << 16);
    u.y = uint32_t(f2bf(v[2])) | (uint32_t(f2bf(v[3])) << 16);
    u.z = uint32_t(f2bf(v[4])) | (uint32_t(f2bf(v[5])) << 16);
    u.w = uint32_t(f2bf(v[6])) | (uint32_t(f2bf(v[7])) << 16);
    *reinterpret_cast<uint4*>(p) = u;
  }
};
template <> struct XVec<float> {
  static constexpr int N = 4;
  static __device__ __forceinline__ void load(const float* p, float* v) {
    const float4 u = *reinterpret_cast<const float4*>(p);
    v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w;
  }
  static __device__ __forceinline__ void store(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};

template <typename T> __device__ __forceinline__ float xload1(const T* p);
template <> __device__ __forceinline__ float xload1<BF16>(const BF16* p) { return bf2f(p->x); }
template <> __device__ __forceinline__ float xload1<float>(const float* p) { return *p; }

// running state of one lane / wave / workgroup
struct XState {
  float m;    // max so far (-inf when empty)
  float s;    // sum exp(x - m)
  float am;   // argmax value
  int ai;     // argmax column (INT_MAX when empty)
};

__device__ __forceinline__ void xmerge(XState& a, const XState& b) {
  const float m = fmaxf(a.m, b.m);
  // exp2 of (-inf) - (-inf) would be NaN for two empty states: guard the empty side
  const float sa = a.m == -INFINITY ? 0.f : a.s * exp2f((a.m - m) * kLog2e);
  const float sb = b.m == -INFINITY ? 0.f : b.s * exp2f((b.m - m) * kLog2e);
  a.s = sa + sb;
  a.m = m;
  if (b.am > a.am || (b.am == a.am && b.ai < a.ai)) {
    a.am = b.am;
    a.ai = b.ai;
  }
}

__device__ __forceinline__ XState xshfl(const XState& v, int o) {
  XState r;
  r.m = __shfl_xor(v.m, o, 64);
  r.s = __shfl_xor(v.s, o, 64);
  r.am = __shfl_xor(v.am, o, 64);
  r.ai = __shfl_xor(v.ai, o, 64);
  return r;
}

template <typename T>
__global__ __launch_bounds__(kXentThreads) void xent_fwd_kernel(const T* __restrict__ x, int64_t ld, int V,
                                                              const int64_t* __restrict__ labels, int64_t ignore,
                                                              float* __restrict__ lse, float* __restrict__ loss,
                                                              float* __restrict__ correct) {
  constexpr int VN = XVec<T>::N;
  const int64_t r = blockIdx.x;
  const T* row = x + r * ld;
  XState st{-INFINITY, 0.f, -INFINITY, 0x7fffffff};
  bool nan_seen = false;
  const int vfull = V / VN * VN;
  // online (max, sum-exp, argmax) update with one loaded vector of columns c .. c+VN-1
  auto absorb = [&](const float (&v)[VN], int c) {
    float vm = v[0];
    int vi = 0;
#pragma unroll
    for (int j = 1; j < VN; ++j)
      if (v[j] > vm) { vm = v[j]; vi = j; }
    const float m = fmaxf(st.m, vm);
    float s = st.m == -INFINITY ? 0.f : st.s * exp2f((st.m - m) * kLog2e);
#pragma unroll
    for (int j = 0; j < VN; ++j) {
      s += v[j] == -INFINITY ? 0.f : exp2f((v[j] - m) * kLog2e);  // all -inf so far: m is -inf too
      nan_seen |= v[j] != v[j];
    }
    st.s = s;
    st.m = m;
    if (vm > st.am) { st.am = vm; st.ai = c + vi; }  // columns grow within a lane: strict >
  };
  // XU vectors per lane loaded before the first is absorbed: XU loads in flight instead of
  // one dependent HBM round trip per vector (the online update chains the iterations)
  constexpr int XU = 4;
  constexpr int kStride = kXentThreads * VN;
  int c = threadIdx.x * VN;
  for (; c + (XU - 1) * kStride < vfull; c += XU * kStride) {
    float v[XU][VN];
#pragma unroll
    for (int u = 0; u < XU; ++u) XVec<T>::load(row + c + u * kStride, v[u]);
#pragma unroll
    for (int u = 0; u < XU; ++u) absorb(v[u], c + u * kStride);
  }
  for (; c < vfull; c += kStride) {
    float v[VN];
    XVec<T>::load(row + c, v);
    absorb(v, c);
  }
  for (int c = vfull + threadIdx.x; c < V; c += kXentThreads) {  // tail (V not a multiple of VN)
    const float v = xload1(row + c);
    XState t{v, 1.f, v, c};
    nan_seen |= v != v;
    xmerge(st, t);
  }
  if (nan_seen) st.s = NAN;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) xmerge(st, xshfl(st, o));
  __shared__ XState part[kXentThreads / 64];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) part[wave] = st;
  __syncthreads();
  if (threadIdx.x == 0) {
    XState a = part[0];
#pragma unroll
    for (int w = 1; w < kXentThreads / 64; ++w) xmerge(a, part[w]);
    const float l = a.m + logf(a.s);
    lse[r] = l;
    const int64_t y = labels[r];
    const bool valid = y != ignore && y >= 0 && y < V;
    loss[r] = valid ? l - xload1(row + y) : 0.f;
    correct[r] = valid && int64_t(a.ai) == y ? 1.f : 0.f;
  }
}

// scale: device scalar (d loss / n_valid), so the step needs no host value
template <typename T>
__global__ __launch_bounds__(kXentThreads) void xent_bwd_kernel(const T* __restrict__ x, T* __restrict__ dx, int64_t ld,
                                                              int V, const int64_t* __restrict__ labels,
                                                              int64_t ignore, const float* __restrict__ lse,
                                                              const float* __restrict__ scale_p) {
  constexpr int VN = XVec<T>::N;
  const int64_t r = blockIdx.x;
  const T* row = x + r * ld;
  T* drow = dx + r * ld;
  const int64_t y = labels[r];
  const bool valid = y != ignore && y >= 0 && y < V;
  const float scale = valid ? *scale_p : 0.f;
  const float l = lse[r];
  const int ldi = int(ld);
  const int vfull = ldi / VN * VN;  // ld is a multiple of VN (checked on the host)
  auto emit = [&](float (&v)[VN], int c) {
#pragma unroll
    for (int j = 0; j < VN; ++j) {
      const int col = c + j;
      const float p = exp2f((v[j] - l) * kLog2e);
      v[j] = col < V ? scale * (p - (int64_t(col) == y ? 1.f : 0.f)) : 0.f;
    }
    XVec<T>::store(drow + c, v);
  };
  constexpr int XU = 4;  // loads in flight per lane, as in the forward
  constexpr int kStride = kXentThreads * VN;
  int c = threadIdx.x * VN;
  for (; c + (XU - 1) * kStride < vfull; c += XU * kStride) {
    float v[XU][VN];
#pragma unroll
    for (int u = 0; u < XU; ++u) XVec<T>::load(row + c + u * kStride, v[u]);
#pragma unroll
    for (int u = 0; u < XU; ++u) emit(v[u], c + u * kStride);
  }
  for (; c < vfull; c += kStride) {
    float v[VN];
    XVec<T>::load(row + c, v);
    emit(v, c);
  }
}

}  // namespace

void xent_fwd(uintptr_t x, int64_t rows, int64_t ld, int V, int dt, uintptr_t labels, int64_t ignore, uintptr_t lse,
              uintptr_t loss, uintptr_t correct, uintptr_t stream) {
  VODA_CHECK(rows > 0 && V > 0 && ld >= V, "xent: bad shape");
  VODA_CHECK(rows <= 0x7fffffff, "xent: too many rows");
  VODA_CHECK(x % 16 == 0 && ld % (dt == kF32 ? 4 : 8) == 0, "xent: rows must be 16-byte aligned");
  if (dt == kBF16) {
    hipLaunchKernelGGL((xent_fwd_kernel<BF16>), dim3(unsigned(rows)), dim3(kXentThreads), 0, as_stream(stream),
                       reinterpret_cast<const BF16*>(x), ld, V, reinterpret_cast<const int64_t*>(labels), ignore,
                       reinterpret_cast<float*>(lse), reinterpret_cast<float*>(loss),
                       reinterpret_cast<float*>(correct));
  } else {
    VODA_CHECK(dt == kF32, "xent: logits must be bf16 or fp32");
    hipLaunchKernelGGL((xent_fwd_kernel<float>), dim3(unsigned(rows)), dim3(kXentThreads), 0, as_stream(stream),
                       reinterpret_cast<const float*>(x), ld, V, reinterpret_cast<const int64_t*>(labels), ignore,
                       reinterpret_cast<float*>(lse), reinterpret_cast<float*>(loss),
                       reinterpret_cast<float*>(correct));
  }
  check_launch();
}

void xent_bwd(uintptr_t x, uintptr_t dx, int64_t rows, int64_t ld, int V, int dt, uintptr_t labels, int64_t ignore,
              uintptr_t lse, uintptr_t scale, uintptr_t stream) {
  VODA_CHECK(rows > 0 && V > 0 && ld >= V, "xent: bad shape");
  VODA_CHECK(rows <= 0x7fffffff && ld <= 0x7fffffff, "xent: too large");
  VODA_CHECK(x % 16 == 0 && dx % 16 == 0 && ld % (dt == kF32 ? 4 : 8) == 0, "xent: rows must be 16-byte aligned");
  if (dt == kBF16) {
    hipLaunchKernelGGL((xent_bwd_kernel<BF16>), dim3(unsigned(rows)), dim3(kXentThreads), 0, as_stream(stream),
                       reinterpret_cast<const BF16*>(x), reinterpret_cast<BF16*>(dx), ld, V,
                       reinterpret_cast<const int64_t*>(labels), ignore, reinterpret_cast<const float*>(lse),
                       reinterpret_cast<const float*>(scale));
  } else {
    VODA_CHECK(dt == kF32, "xent: logits must be bf16 or fp32");
    hipLaunchKernelGGL((xent_bwd_kernel<float>), dim3(unsigned(rows)), dim3(kXentThreads), 0, as_stream(stream),
                       reinterpret_cast<const float*>(x), reinterpret_cast<float*>(dx), ld, V,
                       reinterpret_cast<const int64_t*>(labels), ignore, reinterpret_cast<const float*>(lse),
                       reinterpret_cast<const float*>(scale));
  }
  check_launch();
}

}  // namespace voda
