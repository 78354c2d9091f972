// Fused BatchNorm(+residual add)(+ReLU) for channels_last (NHWC) activations on CDNA4.
//
// The ResNet-50 / InceptionV3 / VGG jobs of the trace spend ~half of their step in
// BatchNorm, ReLU and the residual add when those run as separate library kernels
// (MIOpen BN fwd/bwd + elementwise ReLU / add / ReLU-backward: profiles/).  Here the
// activation is viewed as a row-major [M = N*H*W][C] matrix and each op touches it the
// minimum number of times:
//
//   forward  (train): stats pass   read x                 -> per-block partial sums
//                     finalize     per channel: mean, invstd, running stats, a=g*invstd, b=beta-mean*a
//                     apply pass   read x (+ residual r), write y = relu(a*x + b (+ r))
//   backward        : reduce pass  read dy, ReLU bit-mask, x -> partial sums of g and g*x
//                     finalize     dgamma, dbeta, per-channel (a, c2, c0)
//                     apply pass   read dy, bit-mask, x; write dx = a*g + c2*x + c0 (+ dr = g)
//   with g = dy * (y > 0) when the forward applied ReLU.  The forward apply pass writes the
//   ReLU mask as ONE BIT per element ([M][C/8] bytes, bit k of byte (r, g) = channel 8g+k),
//   so each backward pass reads 1/16 of the bytes it would read from the saved bf16 output
//   (-25 % backward HBM traffic), and
//   dx = a*(g - mean(g) - xhat*mean(g*xhat)) folded into per-channel constants.
//
// Layout / mapping: a thread owns ONE group of 8 consecutive channels (16 B of bf16) for
// the whole kernel, so per-channel constants live in registers; a block of 256 threads
// covers floor(256 / (C/8)) rows per iteration (one contiguous 4 KB span of memory: fully
// coalesced dwordx4 loads), and blocks own contiguous row chunks.  C > 2048 uses grid.y
// channel slices.  Partial sums are fp32 per block; the finalize kernels reduce them with
// 32 row-groups per channel group and double accumulation.
#include "common.h"

#include <cstdlib>
#include "ops.h"

namespace voda {

namespace {

constexpr int kBlock = 256;
constexpr int kVec = 8;            // channels per thread
constexpr int kMaxTpr = kBlock;    // channel groups per block slice (<= 2048 channels)

template <typename T> struct Vec8;
template <> struct Vec8<BF16> {
  using Raw = uint4;  // 8 elements as loaded: 4 VGPRs held in flight instead of 8 floats
  static __device__ __forceinline__ Raw load_raw(const BF16* p, int64_t i) {
    return *reinterpret_cast<const uint4*>(p + i);
  }
  static __device__ __forceinline__ void cvt(const Raw& u, float (&v)[8]) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) { v[2 * k] = bf2f(w[k] & 0xffff); v[2 * k + 1] = bf2f(w[k] >> 16); }
  }
  static __device__ __forceinline__ void load(const BF16* p, int64_t i, float (&v)[8]) {
    uint4 u = *reinterpret_cast<const uint4*>(p + i);
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) { v[2 * k] = bf2f(w[k] & 0xffff); v[2 * k + 1] = bf2f(w[k] >> 16); }
  }
  static __device__ __forceinline__ void store(BF16* p, int64_t i, const float (&v)[8]) {
    uint4 u;
    u.x = uint32_t(f2bf(v[0])) | (uint32_t(f2bf(v[1])) << 16);
    u.y = uint32_t(f2bf(v[2])) | (uint32_t(f2bf(v[3])) << 16);
    u.z = uint32_t(f2bf(v[4])) | (uint32_t(f2bf(v[5])) << 16);
    u.w = uint32_t(f2bf(v[6])) | (uint32_t(f2bf(v[7])) << 16);
    *reinterpret_cast<uint4*>(p + i) = u;
  }
};
template <> struct Vec8<F16> {
  using Raw = uint4;
  static __device__ __forceinline__ Raw load_raw(const F16* p, int64_t i) {
    return *reinterpret_cast<const uint4*>(p + i);
  }
  static __device__ __forceinline__ void cvt(const Raw& u, float (&v)[8]) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) { v[2 * k] = h2f(w[k] & 0xffff); v[2 * k + 1] = h2f(w[k] >> 16); }
  }
  static __device__ __forceinline__ void load(const F16* p, int64_t i, float (&v)[8]) {
    uint4 u = *reinterpret_cast<const uint4*>(p + i);
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) { v[2 * k] = h2f(w[k] & 0xffff); v[2 * k + 1] = h2f(w[k] >> 16); }
  }
  static __device__ __forceinline__ void store(F16* p, int64_t i, const float (&v)[8]) {
    uint4 u;
    u.x = uint32_t(f2h(v[0])) | (uint32_t(f2h(v[1])) << 16);
    u.y = uint32_t(f2h(v[2])) | (uint32_t(f2h(v[3])) << 16);
    u.z = uint32_t(f2h(v[4])) | (uint32_t(f2h(v[5])) << 16);
    u.w = uint32_t(f2h(v[6])) | (uint32_t(f2h(v[7])) << 16);
    *reinterpret_cast<uint4*>(p + i) = u;
  }
};
template <> struct Vec8<float> {
  struct Raw {
    float4 a, b;
  };
  static __device__ __forceinline__ Raw load_raw(const float* p, int64_t i) {
    return {*reinterpret_cast<const float4*>(p + i), *reinterpret_cast<const float4*>(p + i + 4)};
  }
  static __device__ __forceinline__ void cvt(const Raw& r, float (&v)[8]) {
    v[0] = r.a.x; v[1] = r.a.y; v[2] = r.a.z; v[3] = r.a.w; v[4] = r.b.x; v[5] = r.b.y; v[6] = r.b.z; v[7] = r.b.w;
  }
  static __device__ __forceinline__ void load(const float* p, int64_t i, float (&v)[8]) {
    float4 a = *reinterpret_cast<const float4*>(p + i);
    float4 b = *reinterpret_cast<const float4*>(p + i + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, int64_t i, const float (&v)[8]) {
    *reinterpret_cast<float4*>(p + i) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + i + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};

// Thread -> (channel group, row offset) mapping shared by every pass.
struct Map {
  int tpr;        // channel groups handled by this block slice
  int rpi;        // rows per iteration
  int cg;         // this thread's channel group (global), valid if active
  int rsub;       // this thread's row offset inside an iteration
  bool active;
};

__device__ __forceinline__ Map make_map(int C) {
  Map m;
  const int groups = C / kVec;
  const int slice0 = blockIdx.y * kMaxTpr;
  m.tpr = min(groups - slice0, kMaxTpr);
  m.rpi = kBlock / m.tpr;
  const int t = threadIdx.x;
  m.active = t < m.rpi * m.tpr;
  m.cg = slice0 + (m.active ? t % m.tpr : 0);
  m.rsub = m.active ? t / m.tpr : 0;
  return m;
}

// Rows [r0, r1) owned by block ``bid`` (contiguous chunk of iterations).
__device__ __forceinline__ void block_rows(int64_t M, int rpi, int64_t bid, int64_t& r0, int64_t& r1) {
  const int64_t iters = (M + rpi - 1) / rpi;
  const int64_t per = (iters + gridDim.x - 1) / gridDim.x;
  r0 = bid * per * rpi;
  r1 = min<int64_t>(M, r0 + per * rpi);
}

// Reduction passes walk rows in one of two orders (reduce_walk below):
//   sweep = 0: each block walks its own contiguous chunk;
//   sweep = 1: the whole grid sweeps the tensor front to back (iteration i of every block
//              covers one contiguous span), so the data read LAST sits at the END of the
//              tensor -- the apply pass that follows walks its blocks back to front and
//              meets those rows first, while they can still be in the 256 MB MALL.
//   sweep = 2: the reduction sweeps back to front (Walk below), the apply pass front to back.
// Apply passes: chunk of block blockIdx.x, or of the mirrored block in sweep mode 1.
__device__ __forceinline__ void apply_rows(int64_t M, int rpi, int sweep, int64_t& r0, int64_t& r1) {
  block_rows(M, rpi, sweep == 1 ? int64_t(gridDim.x) - 1 - blockIdx.x : int64_t(blockIdx.x), r0, r1);
}

// Block-level reduction of two 8-channel accumulators over the row offsets that share a
// channel group; thread (rsub == 0) ends up with the block's sums.  Writes the partials.
__device__ __forceinline__ void reduce_and_store(const Map& m, float (&s1)[8], float (&s2)[8], float* part1,
                                                 float* part2, int C) {
  __shared__ float red[2][kBlock][kVec + 1];
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < kVec; ++k) { red[0][t][k] = s1[k]; red[1][t][k] = s2[k]; }
  __syncthreads();
  if (m.active && m.rsub == 0) {
    const int tl = t;  // = channel group index within the slice
    for (int r = 1; r < m.rpi; ++r) {
      const int o = tl + r * m.tpr;
#pragma unroll
      for (int k = 0; k < kVec; ++k) { s1[k] += red[0][o][k]; s2[k] += red[1][o][k]; }
    }
    const int64_t base = int64_t(blockIdx.x) * C + int64_t(m.cg) * kVec;
#pragma unroll
    for (int k = 0; k < kVec; ++k) { part1[base + k] = s1[k]; part2[base + k] = s2[k]; }
  }
}

// Three-accumulator form (dual-BN backward reduce): part1/2/3 get sum g, sum g*x, sum g*x2.
__device__ __forceinline__ void reduce_and_store3(const Map& m, float (&s1)[8], float (&s2)[8], float (&s3)[8],
                                                  float* part1, float* part2, float* part3, int C) {
  __shared__ float red3[3][kBlock][kVec + 1];
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < kVec; ++k) { red3[0][t][k] = s1[k]; red3[1][t][k] = s2[k]; red3[2][t][k] = s3[k]; }
  __syncthreads();
  if (m.active && m.rsub == 0) {
    for (int r = 1; r < m.rpi; ++r) {
      const int o = t + r * m.tpr;
#pragma unroll
      for (int k = 0; k < kVec; ++k) { s1[k] += red3[0][o][k]; s2[k] += red3[1][o][k]; s3[k] += red3[2][o][k]; }
    }
    const int64_t base = int64_t(blockIdx.x) * C + int64_t(m.cg) * kVec;
#pragma unroll
    for (int k = 0; k < kVec; ++k) { part1[base + k] = s1[k]; part2[base + k] = s2[k]; part3[base + k] = s3[k]; }
  }
}

// ---------------------------------------------------------------- forward: statistics
// Buffer-descriptor loads of the reduction passes.  The row walk is split into a
// block-uniform part (the base row of an iteration -> descriptor base, and the row step ->
// scalar soffset) and a per-lane part that never changes (this lane's byte offset inside a
// row span -> one 32-bit voffset).  No 64-bit per-row address math is left in VGPRs (stats
// U=8: 124 -> 88 VGPRs, backward reduce U=4: 132 -> 70).  num_records clamps the descriptor
// at the end of this block's rows: the tail rows load as zeros (they add nothing to either
// sum), so there is no remainder loop.  Measured effect on the ResNet-50 step: -0.05 ms;
// the passes are not occupancy-bound (1024 vs 2048 blocks, 4 vs 8 rows in flight: same or
// slower), they run at ~4.2-4.4 TB/s aggregate over ResNet-50's many small tensors.
// The descriptor inputs are wave-uniform by construction (kernargs, blockIdx, loop counter);
// readfirstlane makes that provable, so the loads are not wrapped in waterfall loops.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const void* base, int64_t bytes) {
  const int64_t b = bytes < 0 ? 0 : (bytes > 0x7fffffff ? 0x7fffffff : bytes);
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(p));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(p >> 32));
  const int n = __builtin_amdgcn_readfirstlane(int(b));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uint64_t(hi) << 32) | lo), 0, n, 0x00020000);
}

template <typename T> struct BufRow;
template <> struct BufRow<BF16> {
  using Raw = uint4;
  static __device__ __forceinline__ Raw load(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct BufRow<F16> : BufRow<BF16> {};
template <> struct BufRow<float> {
  using Raw = Vec8<float>::Raw;
  static __device__ __forceinline__ Raw load(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    const auto a = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
    const auto b = __builtin_amdgcn_raw_buffer_load_b128(r, voff + 16, soff, 0);
    return {make_float4(__uint_as_float(a[0]), __uint_as_float(a[1]), __uint_as_float(a[2]), __uint_as_float(a[3])),
            make_float4(__uint_as_float(b[0]), __uint_as_float(b[1]), __uint_as_float(b[2]), __uint_as_float(b[3]))};
  }
};

// Uniform walk of a reduction pass: iterations at base rows first, first + step, ... < end,
// taken U at a time.  ``groups`` = number of U-iteration groups; group i starts at row
// first + order(i) * U * step, with order(i) = n - 1 - i when ``rev`` (sweep = 2: the grid
// sweeps the tensor BACK to front, so it first meets the rows the producing GEMM / conv wrote
// last -- still in the 256 MB MALL -- and the front-to-back apply pass that follows meets the
// rows the reduction read last).
struct Walk {
  int64_t first, step, end, groups;
  bool rev;
  __device__ __forceinline__ int64_t base(int64_t i, int U) const {
    return first + (rev ? groups - 1 - i : i) * U * step;
  }
};
__device__ __forceinline__ Walk reduce_walk(const Map& m, int64_t M, int sweep, int U) {
  Walk w;
  if (sweep) {
    w.first = int64_t(blockIdx.x) * m.rpi;
    w.step = int64_t(gridDim.x) * m.rpi;
    w.end = M;
  } else {
    block_rows(M, m.rpi, blockIdx.x, w.first, w.end);
    w.step = m.rpi;
  }
  const int64_t stride = int64_t(U) * w.step;
  w.groups = w.end > w.first ? (w.end - w.first + stride - 1) / stride : 0;
  w.rev = sweep == 2;
  return w;
}

template <typename T, int U>
__global__ __launch_bounds__(kBlock) void bn_stats_kernel(const T* __restrict__ x, float* __restrict__ part,
                                                          int64_t M, int C, int sweep) {
  const Map m = make_map(C);
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (m.active) {
    const Walk w = reduce_walk(m, M, sweep, U);
    const int64_t end = w.end;
    const int64_t row_bytes = int64_t(C) * sizeof(T);
    const int voff = int(m.rsub * row_bytes + int64_t(m.cg) * kVec * sizeof(T));
    const int sstep = int(w.step * row_bytes);  // <= 2048 blocks x 4 KB
    for (int64_t i = 0; i < w.groups; ++i) {
      const int64_t b = w.base(i, U);
      const auto rs = rows_rsrc(x + b * C, (end - b) * row_bytes);
      typename BufRow<T>::Raw raw[U];
#pragma unroll
      for (int u = 0; u < U; ++u) raw[u] = BufRow<T>::load(rs, voff, u * sstep);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float v[8];
        Vec8<T>::cvt(raw[u], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) { s1[k] += v[k]; s2[k] = fmaf(v[k], v[k], s2[k]); }
      }
    }
  }
  reduce_and_store(m, s1, s2, part, part + int64_t(gridDim.x) * C, C);
}

// ---------------------------------------------------------------- backward: reductions
__device__ __forceinline__ void apply_mask(float (&g)[8], uint8_t mb) {
#pragma unroll
  for (int k = 0; k < 8; ++k) g[k] = ((mb >> k) & 1) ? g[k] : 0.f;
}

template <typename T, bool RELU, int U>
__global__ __launch_bounds__(kBlock) void bn_bwd_reduce_kernel(const T* __restrict__ dy,
                                                               const uint8_t* __restrict__ mask,
                                                               const T* __restrict__ x, float* __restrict__ part,
                                                               int64_t M, int C, int sweep) {
  const Map m = make_map(C);
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (m.active) {
    const Walk w = reduce_walk(m, M, sweep, U);
    const int64_t end = w.end;
    const int CB = C / kVec;
    const int64_t row_bytes = int64_t(C) * sizeof(T);
    const int voff = int(m.rsub * row_bytes + int64_t(m.cg) * kVec * sizeof(T));
    const int moff = m.rsub * CB + m.cg;
    const int sstep = int(w.step * row_bytes), mstep = int(w.step * CB);
    // U rows of dy and x (2U x 16 B per lane) + their mask bytes in flight per thread
    for (int64_t i = 0; i < w.groups; ++i) {
      const int64_t b = w.base(i, U);
      const auto rg = rows_rsrc(dy + b * C, (end - b) * row_bytes);
      const auto rx = rows_rsrc(x + b * C, (end - b) * row_bytes);
      const auto rm = rows_rsrc(mask + (RELU ? b * CB : 0), RELU ? (end - b) * CB : 0);
      typename BufRow<T>::Raw gr[U], xr[U];
      uint32_t mb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        gr[u] = BufRow<T>::load(rg, voff, u * sstep);
        xr[u] = BufRow<T>::load(rx, voff, u * sstep);
        if constexpr (RELU) mb[u] = __builtin_amdgcn_raw_buffer_load_b8(rm, moff, u * mstep, 0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float g[8], xv[8];
        Vec8<T>::cvt(gr[u], g);
        Vec8<T>::cvt(xr[u], xv);
        if constexpr (RELU) apply_mask(g, uint8_t(mb[u]));
#pragma unroll
        for (int k = 0; k < 8; ++k) { s1[k] += g[k]; s2[k] = fmaf(g[k], xv[k], s2[k]); }
      }
    }
  }
  reduce_and_store(m, s1, s2, part, part + int64_t(gridDim.x) * C, C);
}

// ---------------------------------------------------------------- finalize kernels
// Block = 8 channels x 64 row groups; double accumulation of the per-block partials, then a
// tree reduction over the row groups in LDS (the finalize is pure L2 latency: up to 2048
// partial rows per channel).
constexpr int kFinCh = 8, kFinRg = 64;

__device__ __forceinline__ void fin_reduce(const float* __restrict__ p1, const float* __restrict__ p2, int nb, int C,
                                           int c, double& S1, double& S2) {
  __shared__ double red[2][kFinRg][kFinCh + 1];
  const int cl = threadIdx.x % kFinCh, rg = threadIdx.x / kFinCh;
  // 4 independent loads per array in flight per thread
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, b0 = 0.f, b1 = 0.f, b2 = 0.f, b3 = 0.f;
  if (c < C) {
    int r = rg;
    for (; r + 3 * kFinRg < nb; r += 4 * kFinRg) {
      a0 += p1[int64_t(r) * C + c];
      a1 += p1[int64_t(r + kFinRg) * C + c];
      a2 += p1[int64_t(r + 2 * kFinRg) * C + c];
      a3 += p1[int64_t(r + 3 * kFinRg) * C + c];
      b0 += p2[int64_t(r) * C + c];
      b1 += p2[int64_t(r + kFinRg) * C + c];
      b2 += p2[int64_t(r + 2 * kFinRg) * C + c];
      b3 += p2[int64_t(r + 3 * kFinRg) * C + c];
    }
    for (; r < nb; r += kFinRg) {
      a0 += p1[int64_t(r) * C + c];
      b0 += p2[int64_t(r) * C + c];
    }
  }
  red[0][rg][cl] = (double(a0) + double(a1)) + (double(a2) + double(a3));
  red[1][rg][cl] = (double(b0) + double(b1)) + (double(b2) + double(b3));
  __syncthreads();
#pragma unroll
  for (int h = kFinRg / 2; h > 0; h >>= 1) {
    if (rg < h) {
      red[0][rg][cl] += red[0][rg + h][cl];
      red[1][rg][cl] += red[1][rg + h][cl];
    }
    __syncthreads();
  }
  S1 = red[0][0][cl];
  S2 = red[1][0][cl];
}

__global__ __launch_bounds__(kFinCh* kFinRg) void bn_fwd_finalize_kernel(
    const float* __restrict__ part, int nb, int64_t M, int C, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ running_mean, float* __restrict__ running_var,
    float* __restrict__ save_mean, float* __restrict__ save_invstd, float* __restrict__ ab, float eps,
    float momentum) {
  const int c = blockIdx.x * kFinCh + threadIdx.x % kFinCh;
  double S1, S2;
  fin_reduce(part, part + int64_t(nb) * C, nb, C, c, S1, S2);
  if (threadIdx.x / kFinCh == 0 && c < C) {
    const double mean = S1 / double(M);
    double var = S2 / double(M) - mean * mean;
    if (var < 0.0) var = 0.0;
    const float invstd = float(1.0 / sqrt(var + double(eps)));
    save_mean[c] = float(mean);
    save_invstd[c] = invstd;
    if (running_mean != nullptr) {
      const double unbiased = M > 1 ? var * double(M) / double(M - 1) : var;
      running_mean[c] = float((1.0 - momentum) * running_mean[c] + momentum * mean);
      running_var[c] = float((1.0 - momentum) * running_var[c] + momentum * unbiased);
    }
    const float g = gamma != nullptr ? gamma[c] : 1.f;
    const float b = beta != nullptr ? beta[c] : 0.f;
    const float a = g * invstd;
    ab[c] = a;
    ab[C + c] = b - float(mean) * a;
  }
}

// ``p1`` / ``p2``: the [nb][C] partials of sum g and sum g*x (a dual-BN backward shares p1
// between its two BatchNorms, see bn_bwd_reduce2_kernel)
__global__ __launch_bounds__(kFinCh* kFinRg) void bn_bwd_finalize_kernel(
    const float* __restrict__ p1, const float* __restrict__ p2, int nb, int64_t M, int C,
    const float* __restrict__ gamma, const float* __restrict__ save_mean, const float* __restrict__ save_invstd,
    float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ k3, int accumulate) {
  const int c = blockIdx.x * kFinCh + threadIdx.x % kFinCh;
  double S1, S2;  // sum g, sum g*x
  fin_reduce(p1, p2, nb, C, c, S1, S2);
  if (threadIdx.x / kFinCh == 0 && c < C) {
    const double mean = save_mean[c], invstd = save_invstd[c];
    const double db = S1;
    const double dg = invstd * (S2 - mean * S1);
    // accumulate: add straight into the optimizer's flat fp32 gradient buffer
    if (dgamma != nullptr) dgamma[c] = accumulate ? dgamma[c] + float(dg) : float(dg);
    if (dbeta != nullptr) dbeta[c] = accumulate ? dbeta[c] + float(db) : float(db);
    const double g = gamma != nullptr ? gamma[c] : 1.0;
    const double a = g * invstd;
    const double c2 = -a * invstd * dg / double(M);
    const double c0 = -a * db / double(M) - c2 * mean;
    k3[c] = float(a);
    k3[C + c] = float(c2);
    k3[2 * C + c] = float(c0);
  }
}

// ---------------------------------------------------------------- elementwise passes
__device__ __forceinline__ uint8_t pos_bits(const float (&v)[8]) {
  uint32_t b = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) b |= (v[k] > 0.f ? 1u : 0u) << k;
  return uint8_t(b);
}

// Apply passes: U rows of every input in flight per thread (all loads issued before the
// first store; BnTune::apply_u selects U).  U = 4 vs the former fwd 2 / bwd 1:
// ResNet-50 step kernel time 23.32 -> 23.21 ms, the residual passes ~2 % faster each
// (profiles/r3/raw/bn_apply_u/); the passes stay near 4.5 TB/s, bandwidth- not latency-bound.
template <typename T, bool RES, bool RELU, int U = 2>
__global__ __launch_bounds__(kBlock) void bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                          const float* __restrict__ ab, T* __restrict__ y,
                                                          uint8_t* __restrict__ mask, int64_t M, int C,
                                                          int sweep) {
  const Map m = make_map(C);
  if (!m.active) return;
  int64_t r0, r1;
  apply_rows(M, m.rpi, sweep, r0, r1);
  const int64_t col = int64_t(m.cg) * kVec;
  float a[8], b[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { a[k] = ab[col + k]; b[k] = ab[C + col + k]; }
  const int64_t step = m.rpi;
  const int CB = C / kVec;
  int64_t r = r0 + m.rsub;
  for (; r + (U - 1) * step < r1; r += U * step) {
    typename Vec8<T>::Raw xr[U], qr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xr[u] = Vec8<T>::load_raw(x, (r + u * step) * C + col);
      if constexpr (RES) qr[u] = Vec8<T>::load_raw(res, (r + u * step) * C + col);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float v[8], q[8];
      Vec8<T>::cvt(xr[u], v);
      if constexpr (RES) Vec8<T>::cvt(qr[u], q);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        v[k] = fmaf(v[k], a[k], b[k]);
        if constexpr (RES) v[k] += q[k];
        if constexpr (RELU) v[k] = fmaxf(v[k], 0.f);
      }
      Vec8<T>::store(y, (r + u * step) * C + col, v);
      if constexpr (RELU) {
        if (mask != nullptr) mask[(r + u * step) * CB + m.cg] = pos_bits(v);
      }
    }
  }
  for (; r < r1; r += step) {
    float v[8], q[8];
    Vec8<T>::load(x, r * C + col, v);
    if constexpr (RES) Vec8<T>::load(res, r * C + col, q);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v[k] = fmaf(v[k], a[k], b[k]);
      if constexpr (RES) v[k] += q[k];
      if constexpr (RELU) v[k] = fmaxf(v[k], 0.f);
    }
    Vec8<T>::store(y, r * C + col, v);
    if constexpr (RELU) {
      if (mask != nullptr) mask[r * CB + m.cg] = pos_bits(v);
    }
  }
}

template <typename T, bool RELU, bool DRES, int U = 1>
__global__ __launch_bounds__(kBlock) void bn_bwd_apply_kernel(const T* __restrict__ dy,
                                                              const uint8_t* __restrict__ mask,
                                                              const T* __restrict__ x, const float* __restrict__ k3,
                                                              T* __restrict__ dx, T* __restrict__ dres, int64_t M,
                                                              int C, int sweep) {
  const Map m = make_map(C);
  if (!m.active) return;
  int64_t r0, r1;
  apply_rows(M, m.rpi, sweep, r0, r1);
  const int64_t col = int64_t(m.cg) * kVec;
  float a[8], c2[8], c0[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { a[k] = k3[col + k]; c2[k] = k3[C + col + k]; c0[k] = k3[2 * C + col + k]; }
  const int64_t step = m.rpi;
  const int CB = C / kVec;
  int64_t r = r0 + m.rsub;
  if constexpr (U > 1) {
    for (; r + (U - 1) * step < r1; r += U * step) {
      typename Vec8<T>::Raw gr[U], xr[U];
      uint8_t mb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        gr[u] = Vec8<T>::load_raw(dy, (r + u * step) * C + col);
        xr[u] = Vec8<T>::load_raw(x, (r + u * step) * C + col);
        if constexpr (RELU) mb[u] = mask[(r + u * step) * CB + m.cg];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float g[8], xv[8], o[8];
        Vec8<T>::cvt(gr[u], g);
        Vec8<T>::cvt(xr[u], xv);
        if constexpr (RELU) apply_mask(g, mb[u]);
        if constexpr (DRES) Vec8<T>::store(dres, (r + u * step) * C + col, g);
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = fmaf(a[k], g[k], fmaf(c2[k], xv[k], c0[k]));
        Vec8<T>::store(dx, (r + u * step) * C + col, o);
      }
    }
  }
  for (; r < r1; r += step) {
    float g[8], xv[8];
    Vec8<T>::load(dy, r * C + col, g);
    Vec8<T>::load(x, r * C + col, xv);
    if constexpr (RELU) apply_mask(g, mask[r * CB + m.cg]);
    if constexpr (DRES) Vec8<T>::store(dres, r * C + col, g);
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = fmaf(a[k], g[k], fmaf(c2[k], xv[k], c0[k]));
    Vec8<T>::store(dx, r * C + col, o);
  }
}

// ---------------------------------------------------------------- dual BN (downsample blocks)
// A ResNet downsample block ends in relu(bn3(y3) + bn_ds(y_ds)).  As two fused BNs that is
// an apply pass writing bn_ds(y_ds) (read 1, write 1) that the bn3 pass reads back as its
// residual, and backward a bn3 pass writing the residual gradient g that bn_ds reduces and
// applies again: 11 tensor passes.  Both BNs see the same g = dy * (out > 0), so one reduce
// pass (dy, mask, y3, y_ds -> sum g, sum g*y3, sum g*y_ds) and one apply pass
// (-> dy3, dy_ds) cover both, and the forward reads y_ds directly: 3 + 3 + 5 = 11 -> 8 passes
// of the block's largest tensor (stats of y3 / y_ds come from their GEMM epilogues).
template <typename T, bool RELU, int U = 4>
__global__ __launch_bounds__(kBlock) void bn_apply2_kernel(const T* __restrict__ x, const T* __restrict__ x2,
                                                           const float* __restrict__ ab, const float* __restrict__ ab2,
                                                           T* __restrict__ y, uint8_t* __restrict__ mask, int64_t M,
                                                           int C, int sweep) {
  const Map m = make_map(C);
  if (!m.active) return;
  int64_t r0, r1;
  apply_rows(M, m.rpi, sweep, r0, r1);
  const int64_t col = int64_t(m.cg) * kVec;
  float a[8], b[8], a2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = ab[col + k];
    a2[k] = ab2[col + k];
    b[k] = ab[C + col + k] + ab2[C + col + k];  // both shifts folded into one
  }
  const int64_t step = m.rpi;
  const int CB = C / kVec;
  int64_t r = r0 + m.rsub;
  auto body = [&](const typename Vec8<T>::Raw& xr, const typename Vec8<T>::Raw& qr, int64_t row) {
    float v[8], q[8];
    Vec8<T>::cvt(xr, v);
    Vec8<T>::cvt(qr, q);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v[k] = fmaf(v[k], a[k], fmaf(q[k], a2[k], b[k]));
      if constexpr (RELU) v[k] = fmaxf(v[k], 0.f);
    }
    Vec8<T>::store(y, row * C + col, v);
    if constexpr (RELU) mask[row * CB + m.cg] = pos_bits(v);
  };
  for (; r + (U - 1) * step < r1; r += U * step) {
    typename Vec8<T>::Raw xr[U], qr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xr[u] = Vec8<T>::load_raw(x, (r + u * step) * C + col);
      qr[u] = Vec8<T>::load_raw(x2, (r + u * step) * C + col);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) body(xr[u], qr[u], r + u * step);
  }
  for (; r < r1; r += step) body(Vec8<T>::load_raw(x, r * C + col), Vec8<T>::load_raw(x2, r * C + col), r);
}

template <typename T, bool RELU, int U>
__global__ __launch_bounds__(kBlock) void bn_bwd_reduce2_kernel(const T* __restrict__ dy,
                                                                const uint8_t* __restrict__ mask,
                                                                const T* __restrict__ x, const T* __restrict__ x2,
                                                                float* __restrict__ part, int64_t M, int C, int sweep) {
  const Map m = make_map(C);
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s3[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (m.active) {
    const Walk w = reduce_walk(m, M, sweep, U);
    const int64_t end = w.end;
    const int CB = C / kVec;
    const int64_t row_bytes = int64_t(C) * sizeof(T);
    const int voff = int(m.rsub * row_bytes + int64_t(m.cg) * kVec * sizeof(T));
    const int moff = m.rsub * CB + m.cg;
    const int sstep = int(w.step * row_bytes), mstep = int(w.step * CB);
    for (int64_t i = 0; i < w.groups; ++i) {
      const int64_t b = w.base(i, U);
      const auto rg = rows_rsrc(dy + b * C, (end - b) * row_bytes);
      const auto rx = rows_rsrc(x + b * C, (end - b) * row_bytes);
      const auto rq = rows_rsrc(x2 + b * C, (end - b) * row_bytes);
      const auto rm = rows_rsrc(mask + (RELU ? b * CB : 0), RELU ? (end - b) * CB : 0);
      typename BufRow<T>::Raw gr[U], xr[U], qr[U];
      uint32_t mb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        gr[u] = BufRow<T>::load(rg, voff, u * sstep);
        xr[u] = BufRow<T>::load(rx, voff, u * sstep);
        qr[u] = BufRow<T>::load(rq, voff, u * sstep);
        if constexpr (RELU) mb[u] = __builtin_amdgcn_raw_buffer_load_b8(rm, moff, u * mstep, 0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float g[8], xv[8], qv[8];
        Vec8<T>::cvt(gr[u], g);
        Vec8<T>::cvt(xr[u], xv);
        Vec8<T>::cvt(qr[u], qv);
        if constexpr (RELU) apply_mask(g, uint8_t(mb[u]));
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          s1[k] += g[k];
          s2[k] = fmaf(g[k], xv[k], s2[k]);
          s3[k] = fmaf(g[k], qv[k], s3[k]);
        }
      }
    }
  }
  const int64_t nbC = int64_t(gridDim.x) * C;
  reduce_and_store3(m, s1, s2, s3, part, part + nbC, part + 2 * nbC, C);
}

template <typename T, bool RELU, int U = 4>
__global__ __launch_bounds__(kBlock) void bn_bwd_apply2_kernel(const T* __restrict__ dy,
                                                               const uint8_t* __restrict__ mask,
                                                               const T* __restrict__ x, const T* __restrict__ x2,
                                                               const float* __restrict__ k3,
                                                               const float* __restrict__ k3b, T* __restrict__ dx,
                                                               T* __restrict__ dx2, int64_t M, int C, int sweep) {
  const Map m = make_map(C);
  if (!m.active) return;
  int64_t r0, r1;
  apply_rows(M, m.rpi, sweep, r0, r1);
  const int64_t col = int64_t(m.cg) * kVec;
  float a[8], c2[8], c0[8], e[8], e2[8], e0[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = k3[col + k]; c2[k] = k3[C + col + k]; c0[k] = k3[2 * C + col + k];
    e[k] = k3b[col + k]; e2[k] = k3b[C + col + k]; e0[k] = k3b[2 * C + col + k];
  }
  const int64_t step = m.rpi;
  const int CB = C / kVec;
  int64_t r = r0 + m.rsub;
  auto body = [&](const typename Vec8<T>::Raw& gr, const typename Vec8<T>::Raw& xr, const typename Vec8<T>::Raw& qr,
                  uint8_t mb, int64_t row) {
    float g[8], xv[8], qv[8], o[8], o2[8];
    Vec8<T>::cvt(gr, g);
    Vec8<T>::cvt(xr, xv);
    Vec8<T>::cvt(qr, qv);
    if constexpr (RELU) apply_mask(g, mb);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o[k] = fmaf(a[k], g[k], fmaf(c2[k], xv[k], c0[k]));
      o2[k] = fmaf(e[k], g[k], fmaf(e2[k], qv[k], e0[k]));
    }
    Vec8<T>::store(dx, row * C + col, o);
    Vec8<T>::store(dx2, row * C + col, o2);
  };
  for (; r + (U - 1) * step < r1; r += U * step) {
    typename Vec8<T>::Raw gr[U], xr[U], qr[U];
    uint8_t mb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      gr[u] = Vec8<T>::load_raw(dy, (r + u * step) * C + col);
      xr[u] = Vec8<T>::load_raw(x, (r + u * step) * C + col);
      qr[u] = Vec8<T>::load_raw(x2, (r + u * step) * C + col);
      mb[u] = RELU ? mask[(r + u * step) * CB + m.cg] : uint8_t(0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) body(gr[u], xr[u], qr[u], mb[u], r + u * step);
  }
  for (; r < r1; r += step)
    body(Vec8<T>::load_raw(dy, r * C + col), Vec8<T>::load_raw(x, r * C + col), Vec8<T>::load_raw(x2, r * C + col),
         RELU ? mask[r * CB + m.cg] : uint8_t(0), r);
}

// ---------------------------------------------------------------- stem: BN + ReLU + max pool
// ResNet stem: relu(bn(conv7x7(x))) -> maxpool 3x3/2.  Unfused, the 112x112 activation (411 MB
// at bs 256) is written by the BN apply pass, read by the pool, and in backward the pool
// writes its 411 MB gradient that both BN passes read again.  Fused:
//   forward : stats pass over x (as above), then ONE pass that computes relu(a*x+b) in
//             registers for each pooling window and writes only the pooled output and a
//             1-byte argmax per element (0xFF when the window max is 0: relu clamped every
//             element, so no gradient flows -- relu'(<=0) = 0, as in the unfused backward);
//   backward: the BN reduce and apply passes gather g = (pool backward of dy) on the fly
//             from dy_pool + argmax bytes (cached: 1/4 of the input's pixels) and never
//             materialise it.
struct PoolG {
  int N, H, W, C, Ho, Wo, k, s, p;
};

// Window shape K x K, stride S at compile time (the stem's 3x3/2): all window loads of a
// thread are issued before the first use (clamped addresses, out-of-image taps masked).
template <typename T, int K, int S>
__global__ __launch_bounds__(kBlock) void bn_pool_fwd_kernel(const T* __restrict__ x, const float* __restrict__ ab,
                                                             T* __restrict__ y, uint8_t* __restrict__ idx, PoolG g) {
  const int CG = g.C / kVec;
  const int j = int(blockIdx.y) * kBlock + int(threadIdx.x);
  if (j >= g.Wo * CG) return;
  const int n = int(blockIdx.x) / g.Ho, ho = int(blockIdx.x) % g.Ho;
  const int wo = j / CG, cg = j - wo * CG;
  const T* xn = x + int64_t(n) * g.H * g.W * g.C + cg * kVec;
  const int h0 = ho * S - g.p, w0 = wo * S - g.p;
  typename Vec8<T>::Raw raw[K * K];
#pragma unroll
  for (int kh = 0; kh < K; ++kh) {
    const int hc = min(max(h0 + kh, 0), g.H - 1);
#pragma unroll
    for (int kw = 0; kw < K; ++kw)
      raw[kh * K + kw] = Vec8<T>::load_raw(xn, (int64_t(hc) * g.W + min(max(w0 + kw, 0), g.W - 1)) * g.C);
  }
  float a[8], b[8], best[8];
  uint32_t arg[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    a[c] = ab[cg * kVec + c];
    b[c] = ab[g.C + cg * kVec + c];
    best[c] = 0.f;  // relu output >= 0: a window whose max stays 0 passes no gradient
    arg[c] = 0xFF;
  }
#pragma unroll
  for (int kh = 0; kh < K; ++kh) {
#pragma unroll
    for (int kw = 0; kw < K; ++kw) {
      const bool ok = unsigned(h0 + kh) < unsigned(g.H) && unsigned(w0 + kw) < unsigned(g.W);
      float v[8];
      Vec8<T>::cvt(raw[kh * K + kw], v);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        // bf16 rounding is monotonic, so max-then-round == round-then-max (the unfused values)
        const float r = fmaf(v[c], a[c], b[c]);
        if (ok && r > best[c]) { best[c] = r; arg[c] = uint32_t(kh * K + kw); }
      }
    }
  }
  const int64_t i = (int64_t(blockIdx.x) * g.Wo + wo) * CG + cg;
  Vec8<T>::store(y, i * kVec, best);
  uint2 u;
  u.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
  u.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
  *reinterpret_cast<uint2*>(idx + i * kVec) = u;
}

// g[8] at input pixel (n, h, w), channel group cg: the sum of dy_pool over the windows whose
// argmax byte names this pixel (0xFF never does); all (K+S-1)/S squared windows loaded first.
template <typename T, int K, int S>
__device__ __forceinline__ void pool_grad_gather(const T* __restrict__ dyp, const uint8_t* __restrict__ idx,
                                                 const PoolG& g, int n, int h, int w, int cg, float (&acc)[8]) {
  constexpr int NW = (K + S - 1) / S;
  const int ho0 = max(0, (h + g.p - K + S) / S), wo0 = max(0, (w + g.p - K + S) / S);
  const int64_t nbase = int64_t(n) * g.Ho * g.Wo * g.C + cg * kVec;
  uint2 a[NW * NW];
  typename Vec8<T>::Raw raw[NW * NW];
#pragma unroll
  for (int dh = 0; dh < NW; ++dh) {
    const int hoc = min(ho0 + dh, g.Ho - 1);
#pragma unroll
    for (int dw = 0; dw < NW; ++dw) {
      const int64_t o = nbase + (int64_t(hoc) * g.Wo + min(wo0 + dw, g.Wo - 1)) * g.C;
      a[dh * NW + dw] = *reinterpret_cast<const uint2*>(idx + o);
      raw[dh * NW + dw] = Vec8<T>::load_raw(dyp, o);
    }
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = 0.f;
#pragma unroll
  for (int dh = 0; dh < NW; ++dh) {
    const int ho = ho0 + dh, kh = h - (ho * S - g.p);
#pragma unroll
    for (int dw = 0; dw < NW; ++dw) {
      const int wo = wo0 + dw, kw = w - (wo * S - g.p);
      const bool ok = ho < g.Ho && wo < g.Wo && unsigned(kh) < unsigned(K) && unsigned(kw) < unsigned(K);
      const uint32_t want = ok ? uint32_t(kh * K + kw) : 0x100u;  // 0x100 matches no byte
      float d[8];
      Vec8<T>::cvt(raw[dh * NW + dw], d);
      const uint2 u = a[dh * NW + dw];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const uint32_t ac = ((c < 4 ? u.x : u.y) >> (8 * (c & 3))) & 0xff;
        if (ac == want) acc[c] += d[c];
      }
    }
  }
}

// Reduce pass: block b owns image rows [b*per, (b+1)*per) of the N*H rows; thread (cg =
// t % tpr, column offset t / tpr) walks the row's columns with step rpi.
template <typename T, int K, int S>
__global__ __launch_bounds__(kBlock) void bn_pool_bwd_reduce_kernel(const T* __restrict__ dyp,
                                                                    const uint8_t* __restrict__ idx,
                                                                    const T* __restrict__ x, float* __restrict__ part,
                                                                    PoolG g) {
  const Map m = make_map(g.C);
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (m.active) {
    const int rows = g.N * g.H;
    const int per = (rows + int(gridDim.x) - 1) / int(gridDim.x);
    const int r0 = int(blockIdx.x) * per, r1 = min(rows, r0 + per);
    for (int r = r0; r < r1; ++r) {
      const int n = r / g.H, h = r - n * g.H;
      const T* xr = x + int64_t(r) * g.W * g.C + int64_t(m.cg) * kVec;
      for (int w = m.rsub; w < g.W; w += m.rpi) {
        const auto xraw = Vec8<T>::load_raw(xr, int64_t(w) * g.C);
        float gr[8], xv[8];
        pool_grad_gather<T, K, S>(dyp, idx, g, n, h, w, m.cg, gr);
        Vec8<T>::cvt(xraw, xv);
#pragma unroll
        for (int k = 0; k < 8; ++k) { s1[k] += gr[k]; s2[k] = fmaf(gr[k], xv[k], s2[k]); }
      }
    }
  }
  reduce_and_store(m, s1, s2, part, part + int64_t(gridDim.x) * g.C, g.C);
}

template <typename T, int K, int S>
__global__ __launch_bounds__(kBlock) void bn_pool_bwd_apply_kernel(const T* __restrict__ dyp,
                                                                   const uint8_t* __restrict__ idx,
                                                                   const T* __restrict__ x,
                                                                   const float* __restrict__ k3, T* __restrict__ dx,
                                                                   PoolG g) {
  const int CG = g.C / kVec;
  const int j = int(blockIdx.y) * kBlock + int(threadIdx.x);
  if (j >= g.W * CG) return;
  const int n = int(blockIdx.x) / g.H, h = int(blockIdx.x) % g.H;
  const int w = j / CG, cg = j - w * CG;
  const int64_t off = (int64_t(blockIdx.x) * g.W + w) * g.C + cg * kVec;
  const auto xraw = Vec8<T>::load_raw(x, off);
  float gr[8], xv[8], o[8];
  pool_grad_gather<T, K, S>(dyp, idx, g, n, h, w, cg, gr);
  Vec8<T>::cvt(xraw, xv);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = cg * kVec + k;
    o[k] = fmaf(k3[c], gr[k], fmaf(k3[g.C + c], xv[k], k3[2 * g.C + c]));
  }
  Vec8<T>::store(dx, off, o);
}

// 3x3 / stride-2 / pad-1 windows (the ResNet stem) with one thread per 2 x 2 block of input
// pixels (rows 2m, 2m+1, columns 2k, 2k+1) and channel group: the 4 windows (m + a, k + b),
// a, b in {0, 1}, that can select any of the 4 pixels are loaded once and shared, instead of
// every pixel loading its (up to) 4 windows on its own -- the dy / argmax gather was 8 of
// the 9 loads per pixel of the generic passes above (stem backward reduce + apply: 190 + 293
// us per ResNet-50 bs-256 step, ~1.8x their byte floor).  Pixel (dh, dw) is tap
// (kh, kw) = (dh - 2a + 1, dw - 2b + 1) of window (a, b) when both are in [0, 3).
template <typename T>
__device__ __forceinline__ void pool22_grads(const T* __restrict__ dyp, const uint8_t* __restrict__ idx,
                                             const PoolG& g, int n, int m, int k, int cg, float (&gr)[4][8]) {
  uint2 a[4];
  typename Vec8<T>::Raw raw[4];
  const int64_t nbase = int64_t(n) * g.Ho * g.Wo * g.C + cg * kVec;
#pragma unroll
  for (int wi = 0; wi < 4; ++wi) {
    const int ho = min(m + (wi >> 1), g.Ho - 1), wo = min(k + (wi & 1), g.Wo - 1);
    const int64_t o = nbase + (int64_t(ho) * g.Wo + wo) * g.C;
    a[wi] = *reinterpret_cast<const uint2*>(idx + o);
    raw[wi] = Vec8<T>::load_raw(dyp, o);
  }
#pragma unroll
  for (int px = 0; px < 4; ++px)
#pragma unroll
    for (int c = 0; c < 8; ++c) gr[px][c] = 0.f;
#pragma unroll
  for (int wi = 0; wi < 4; ++wi) {
    const int wa = wi >> 1, wb = wi & 1;
    const bool win_ok = m + wa < g.Ho && k + wb < g.Wo;
    float d[8];
    Vec8<T>::cvt(raw[wi], d);
#pragma unroll
    for (int px = 0; px < 4; ++px) {
      const int kh = (px >> 1) - 2 * wa + 1, kw = (px & 1) - 2 * wb + 1;
      if (kh < 0 || kh > 2 || kw < 0 || kw > 2) continue;  // compile-time after unrolling
      const uint32_t want = win_ok ? uint32_t(kh * 3 + kw) : 0x100u;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const uint32_t ac = ((c < 4 ? a[wi].x : a[wi].y) >> (8 * (c & 3))) & 0xff;
        if (ac == want) gr[px][c] += d[c];
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void bn_pool_bwd_reduce22_kernel(const T* __restrict__ dyp,
                                                                      const uint8_t* __restrict__ idx,
                                                                      const T* __restrict__ x,
                                                                      float* __restrict__ part, PoolG g) {
  const Map mp = make_map(g.C);
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (mp.active) {
    const int Hm = (g.H + 1) / 2, Wk = (g.W + 1) / 2;
    const int rows = g.N * Hm;
    const int per = (rows + int(gridDim.x) - 1) / int(gridDim.x);
    const int r0 = int(blockIdx.x) * per, r1 = min(rows, r0 + per);
    for (int r = r0; r < r1; ++r) {
      const int n = r / Hm, m = r - n * Hm;
      for (int k = mp.rsub; k < Wk; k += mp.rpi) {
        typename Vec8<T>::Raw xr[4];
#pragma unroll
        for (int px = 0; px < 4; ++px) {
          const int h = min(2 * m + (px >> 1), g.H - 1), w = min(2 * k + (px & 1), g.W - 1);
          xr[px] = Vec8<T>::load_raw(x, ((int64_t(n) * g.H + h) * g.W + w) * g.C + int64_t(mp.cg) * kVec);
        }
        float gr[4][8];
        pool22_grads<T>(dyp, idx, g, n, m, k, mp.cg, gr);
#pragma unroll
        for (int px = 0; px < 4; ++px) {
          // a clamped duplicate pixel past the image edge has no window selecting it: gr = 0
          float xv[8];
          Vec8<T>::cvt(xr[px], xv);
#pragma unroll
          for (int c = 0; c < 8; ++c) { s1[c] += gr[px][c]; s2[c] = fmaf(gr[px][c], xv[c], s2[c]); }
        }
      }
    }
  }
  reduce_and_store(mp, s1, s2, part, part + int64_t(gridDim.x) * g.C, g.C);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void bn_pool_bwd_apply22_kernel(const T* __restrict__ dyp,
                                                                     const uint8_t* __restrict__ idx,
                                                                     const T* __restrict__ x,
                                                                     const float* __restrict__ k3, T* __restrict__ dx,
                                                                     PoolG g) {
  const int CG = g.C / kVec;
  const int Hm = (g.H + 1) / 2, Wk = (g.W + 1) / 2;
  const int j = int(blockIdx.y) * kBlock + int(threadIdx.x);
  if (j >= Wk * CG) return;
  const int n = int(blockIdx.x) / Hm, m = int(blockIdx.x) - (int(blockIdx.x) / Hm) * Hm;
  const int k = j / CG, cg = j - k * CG;
  typename Vec8<T>::Raw xr[4];
  int64_t off[4];
#pragma unroll
  for (int px = 0; px < 4; ++px) {
    const int h = min(2 * m + (px >> 1), g.H - 1), w = min(2 * k + (px & 1), g.W - 1);
    off[px] = ((int64_t(n) * g.H + h) * g.W + w) * g.C + cg * kVec;
    xr[px] = Vec8<T>::load_raw(x, off[px]);
  }
  float gr[4][8];
  pool22_grads<T>(dyp, idx, g, n, m, k, cg, gr);
  float a[8], c2[8], c0[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    a[c] = k3[cg * kVec + c];
    c2[c] = k3[g.C + cg * kVec + c];
    c0[c] = k3[2 * g.C + cg * kVec + c];
  }
#pragma unroll
  for (int px = 0; px < 4; ++px) {
    if (2 * m + (px >> 1) >= g.H || 2 * k + (px & 1) >= g.W) continue;
    float xv[8], o[8];
    Vec8<T>::cvt(xr[px], xv);
#pragma unroll
    for (int c = 0; c < 8; ++c) o[c] = fmaf(a[c], gr[px][c], fmaf(c2[c], xv[c], c0[c]));
    Vec8<T>::store(dx, off[px], o);
  }
}

// ---------------------------------------------------------------- launch helpers
struct Grid {
  dim3 grid;
  int nb;
};

Grid bn_grid(int64_t M, int C, int64_t cap_blocks, int iters_per_block) {
  const int groups = C / kVec;
  const int slices = (groups + kMaxTpr - 1) / kMaxTpr;
  const int tpr = std::min(groups, kMaxTpr);
  const int rpi = kBlock / tpr;
  const int64_t iters = (M + rpi - 1) / rpi;
  int64_t nb = (iters + iters_per_block - 1) / iters_per_block;
  nb = std::max<int64_t>(1, std::min<int64_t>(nb, cap_blocks));
  return {dim3(unsigned(nb), unsigned(slices)), int(nb)};
}

// Tuning of the reduction / apply passes (fixed at the measured defaults since round 5;
// bn_set_tuning reaches the other settings, and tests/test_batchnorm_gpu.py checks that every
// reduction walk gives the default's results):
//   deep    rows in flight 4 / 8 / 16 (stats) and 2 / 4 / 8 (backward reduce): level 1
//   blocks  reduction grid cap: 256 = one 4-wave block per CU (512 for fp32 tensors)
//   sweep   grid-sweep reduction + mirrored apply order: 1 (2 = sweep back to front + apply
//           front to back, see Walk)
// Measured on MI355X (profiles/raw/r2_bn_grid_trace.md, ResNet-50 bs-256 step A/B in
// profiles/raw/r2_ab_bn_grid.jsonl): the reduction passes of the large tensors ran at 3.8-4.2
// TB/s with 1024 long-lived blocks each walking its own chunk; one block per CU sweeping
// the tensor together brings the per-step stats + reduce + finalize time 4.64 -> 4.02 ms,
// and the step 26.95 -> 26.23 ms.  Unroll level 2 and grids of 384-2048 blocks are slower.
// fp32 tensors: with 32-byte rows per thread one block per CU leaves the fp32 backward reduce at
// ~3.8 TB/s; two blocks per CU take the fp32 ResNet-50 step's reduce passes 4.86 -> 3.52 ms
// (~5.2 TB/s), 1024 blocks 3.57 ms (profiles/r4/bn_reduce_grid_fp32.md)
struct BnTune {
  int deep;  // rows in flight: 0 -> 4 (stats) / 2 (backward reduce), 1 -> 8 / 4, 2 -> 16 / 8
  int blocks;
  int sweep;
  int blocks_f32 = 512;   // reduction grid cap for fp32 tensors
  int apply_cap = 8192;   // apply-pass grid cap
  int apply_iters = 4;    // row iterations per apply block
  int apply_u = 4;        // rows in flight in the apply passes: 4, 2, or 0 -> fwd 2 / bwd 1
};
BnTune& bn_tune() {
  static BnTune t{1, 256, 1};  // the measured defaults; bn_set_tuning changes them (tests)
  return t;
}

Grid apply_grid(int64_t M, int C) { return bn_grid(M, C, bn_tune().apply_cap, bn_tune().apply_iters); }

// partial-sum blocks: bounded so that the partial arrays stay <= 2M floats each.  dt < 0: the
// largest grid of any dtype (workspace sizing)
Grid reduce_grid(int64_t M, int C, int dt) {
  const BnTune& t = bn_tune();
  const int blocks = dt == kF32 ? t.blocks_f32 : (dt < 0 ? std::max(t.blocks, t.blocks_f32) : t.blocks);
  const int64_t cap = std::max<int64_t>(1, std::min<int64_t>(blocks, (int64_t(1) << 21) / C));
  return bn_grid(M, C, cap, 8);
}

int bn_unroll_level() { return bn_tune().deep; }

template <typename F>
void dispatch_dt(int dt, F&& f) {
  if (dt == kBF16) f(BF16{});
  else if (dt == kF16) f(F16{});
  else if (dt == kF32) f(float{});
  else throw std::invalid_argument("batchnorm: unsupported dtype");
}

}  // namespace

void bn_set_tuning(int deep, int blocks, int sweep) {
  BnTune& t = bn_tune();
  if (deep >= 0) t.deep = std::min(2, deep);
  if (blocks > 0) t.blocks = std::max(64, std::min(8192, blocks));
  if (sweep >= 0) t.sweep = std::min(2, sweep);
}

std::vector<int> bn_get_tuning() {
  const BnTune& t = bn_tune();
  return {t.deep, t.blocks, t.sweep};
}

int64_t bn_workspace_floats(int64_t M, int C) {
  const Grid g = reduce_grid(M, C, -1);
  return int64_t(2) * g.nb * C + 3 * int64_t(C);
}

void bn_fwd_train(uintptr_t x, uintptr_t residual, uintptr_t gamma, uintptr_t beta, uintptr_t running_mean,
                  uintptr_t running_var, uintptr_t save_mean, uintptr_t save_invstd, uintptr_t y, uintptr_t mask,
                  uintptr_t workspace, int64_t M, int C, float eps, float momentum, bool relu, int dt,
                  uintptr_t stream, int pre_nb) {
  VODA_CHECK(C % kVec == 0, "batchnorm: C must be a multiple of 8");
  VODA_CHECK(M > 0, "batchnorm: empty input");
  hipStream_t s = as_stream(stream);
  float* ws = reinterpret_cast<float*>(workspace);
  // pre_nb > 0: the producing GEMM already wrote pre_nb partial rows (gemm_bnstats.hip)
  const Grid rg = reduce_grid(M, C, dt);
  const int nb = pre_nb > 0 ? pre_nb : rg.nb;
  float* ab = ws + int64_t(2) * nb * C;
  const Grid ag = apply_grid(M, C);
  const int sw = bn_tune().sweep;
  dispatch_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    const T* xp = reinterpret_cast<const T*>(x);
    const int lv = bn_unroll_level();
    if (pre_nb > 0) {
    } else if (lv >= 2)
      hipLaunchKernelGGL((bn_stats_kernel<T, 16>), rg.grid, dim3(kBlock), 0, s, xp, ws, M, C, sw);
    else if (lv == 1)
      hipLaunchKernelGGL((bn_stats_kernel<T, 8>), rg.grid, dim3(kBlock), 0, s, xp, ws, M, C, sw);
    else
      hipLaunchKernelGGL((bn_stats_kernel<T, 4>), rg.grid, dim3(kBlock), 0, s, xp, ws, M, C, sw);
    hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinCh * kFinRg), 0, s, ws,
                       nb, M, C, reinterpret_cast<const float*>(gamma), reinterpret_cast<const float*>(beta),
                       reinterpret_cast<float*>(running_mean), reinterpret_cast<float*>(running_var),
                       reinterpret_cast<float*>(save_mean), reinterpret_cast<float*>(save_invstd), ab, eps, momentum);
    const T* rp = reinterpret_cast<const T*>(residual);
    T* yp = reinterpret_cast<T*>(y);
    uint8_t* mp = reinterpret_cast<uint8_t*>(mask);
    auto app = [&](auto res_c, auto relu_c) {
      constexpr bool RS = decltype(res_c)::value, RL = decltype(relu_c)::value;
      if (bn_tune().apply_u == 4)
        hipLaunchKernelGGL((bn_apply_kernel<T, RS, RL, 4>), ag.grid, dim3(kBlock), 0, s, xp, rp, ab, yp, mp, M, C, sw);
      else
        hipLaunchKernelGGL((bn_apply_kernel<T, RS, RL, 2>), ag.grid, dim3(kBlock), 0, s, xp, rp, ab, yp, mp, M, C, sw);
    };
    if (residual) {
      if (relu) app(std::true_type{}, std::true_type{});
      else app(std::true_type{}, std::false_type{});
    } else {
      if (relu) app(std::false_type{}, std::true_type{});
      else app(std::false_type{}, std::false_type{});
    }
  });
  check_launch();
}

void bn_apply(uintptr_t x, uintptr_t residual, uintptr_t ab, uintptr_t y, int64_t M, int C, bool relu, int dt,
              uintptr_t stream) {
  VODA_CHECK(C % kVec == 0, "batchnorm: C must be a multiple of 8");
  hipStream_t s = as_stream(stream);
  const Grid ag = apply_grid(M, C);
  const float* abp = reinterpret_cast<const float*>(ab);
  dispatch_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    const T* xp = reinterpret_cast<const T*>(x);
    const T* rp = reinterpret_cast<const T*>(residual);
    T* yp = reinterpret_cast<T*>(y);
    uint8_t* np = nullptr;
    if (residual) {
      if (relu) hipLaunchKernelGGL((bn_apply_kernel<T, true, true>), ag.grid, dim3(kBlock), 0, s, xp, rp, abp, yp, np, M, C, 0);
      else hipLaunchKernelGGL((bn_apply_kernel<T, true, false>), ag.grid, dim3(kBlock), 0, s, xp, rp, abp, yp, np, M, C, 0);
    } else {
      if (relu) hipLaunchKernelGGL((bn_apply_kernel<T, false, true>), ag.grid, dim3(kBlock), 0, s, xp, rp, abp, yp, np, M, C, 0);
      else hipLaunchKernelGGL((bn_apply_kernel<T, false, false>), ag.grid, dim3(kBlock), 0, s, xp, rp, abp, yp, np, M, C, 0);
    }
  });
  check_launch();
}

void bn_bwd(uintptr_t dy, uintptr_t mask, uintptr_t x, uintptr_t save_mean, uintptr_t save_invstd, uintptr_t gamma,
            uintptr_t dx, uintptr_t dres, uintptr_t dgamma, uintptr_t dbeta, uintptr_t workspace, int64_t M, int C,
            bool relu, bool accumulate, int dt, uintptr_t stream, uintptr_t pre_part, int pre_nb) {
  VODA_CHECK(C % kVec == 0, "batchnorm: C must be a multiple of 8");
  VODA_CHECK(!relu || mask != 0, "batchnorm backward: ReLU needs the forward's bit-mask");
  VODA_CHECK(pre_nb <= 0 || pre_part != 0, "batchnorm backward: precomputed sums need their partials");
  hipStream_t s = as_stream(stream);
  float* ws = reinterpret_cast<float*>(workspace);
  const Grid rg = reduce_grid(M, C, dt);
  // pre_nb > 0: the producer of dy already reduced sum g / sum g*x (conv1x1_f32.hip
  // gemm_f32_dgrad_bn): [2][pre_nb][C] partials at pre_part, no reduce pass
  const bool pre = pre_nb > 0;
  const int nb = pre ? pre_nb : rg.nb;
  const float* p1 = pre ? reinterpret_cast<const float*>(pre_part) : ws;
  float* k3 = pre ? ws : ws + int64_t(2) * rg.nb * C;
  const Grid ag = apply_grid(M, C);
  const int sw = bn_tune().sweep;
  dispatch_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    const T* dyp = reinterpret_cast<const T*>(dy);
    const uint8_t* yp = reinterpret_cast<const uint8_t*>(mask);
    const T* xp = reinterpret_cast<const T*>(x);
    const int lv = bn_unroll_level();
    auto red = [&](auto relu_c, auto u_c) {
      constexpr bool RL = decltype(relu_c)::value;
      constexpr int UU = decltype(u_c)::value;
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, RL, UU>), rg.grid, dim3(kBlock), 0, s, dyp, yp, xp, ws, M, C, sw);
    };
    using RT = std::true_type;
    using RF = std::false_type;
    if (pre) {
    } else if (relu) {
      if (lv >= 2) red(RT{}, std::integral_constant<int, 8>{});
      else if (lv == 1) red(RT{}, std::integral_constant<int, 4>{});
      else red(RT{}, std::integral_constant<int, 2>{});
    } else {
      if (lv >= 2) red(RF{}, std::integral_constant<int, 8>{});
      else if (lv == 1) red(RF{}, std::integral_constant<int, 4>{});
      else red(RF{}, std::integral_constant<int, 2>{});
    }
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinCh * kFinRg), 0, s, p1,
                       p1 + int64_t(nb) * C, nb, M, C, reinterpret_cast<const float*>(gamma), reinterpret_cast<const float*>(save_mean),
                       reinterpret_cast<const float*>(save_invstd), reinterpret_cast<float*>(dgamma),
                       reinterpret_cast<float*>(dbeta), k3, int(accumulate));
    T* dxp = reinterpret_cast<T*>(dx);
    T* drp = reinterpret_cast<T*>(dres);
    auto app = [&](auto relu_c, auto dres_c) {
      constexpr bool RL = decltype(relu_c)::value, DR = decltype(dres_c)::value;
      const int u = bn_tune().apply_u;
      if (u == 4)
        hipLaunchKernelGGL((bn_bwd_apply_kernel<T, RL, DR, 4>), ag.grid, dim3(kBlock), 0, s, dyp, yp, xp, k3, dxp, drp, M, C, sw);
      else if (u == 2)
        hipLaunchKernelGGL((bn_bwd_apply_kernel<T, RL, DR, 2>), ag.grid, dim3(kBlock), 0, s, dyp, yp, xp, k3, dxp, drp, M, C, sw);
      else
        hipLaunchKernelGGL((bn_bwd_apply_kernel<T, RL, DR, 1>), ag.grid, dim3(kBlock), 0, s, dyp, yp, xp, k3, dxp, drp, M, C, sw);
    };
    if (relu) {
      if (dres) app(std::true_type{}, std::true_type{});
      else app(std::true_type{}, std::false_type{});
    } else {
      if (dres) app(std::false_type{}, std::true_type{});
      else app(std::false_type{}, std::false_type{});
    }
  });
  check_launch();
}

// ---- dual BN: relu(bn(x) + bn2(x2)) (ResNet downsample blocks) ----
int64_t bn2_workspace_floats(int64_t M, int C) {
  const Grid g = reduce_grid(M, C, -1);
  return int64_t(3) * g.nb * C + 6 * int64_t(C);
}

void bn2_fwd_train(uintptr_t x, uintptr_t x2, uintptr_t gamma, uintptr_t beta, uintptr_t running_mean,
                   uintptr_t running_var, uintptr_t save_mean, uintptr_t save_invstd, uintptr_t gamma2, uintptr_t beta2,
                   uintptr_t running_mean2, uintptr_t running_var2, uintptr_t save_mean2, uintptr_t save_invstd2,
                   uintptr_t y, uintptr_t mask, uintptr_t workspace, uintptr_t workspace2, int64_t M, int C, float eps,
                   float momentum, bool relu, int dt, uintptr_t stream, int pre_nb, int pre_nb2) {
  VODA_CHECK(C % kVec == 0, "batchnorm: C must be a multiple of 8");
  VODA_CHECK(M > 0, "batchnorm: empty input");
  VODA_CHECK(!relu || mask != 0, "batchnorm: ReLU needs a mask buffer");
  hipStream_t s = as_stream(stream);
  const Grid rg = reduce_grid(M, C, dt);
  const Grid ag = apply_grid(M, C);
  const int sw = bn_tune().sweep;
  float* abs_[2];
  dispatch_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    const uintptr_t xs[2] = {x, x2}, ws_[2] = {workspace, workspace2}, g_[2] = {gamma, gamma2}, b_[2] = {beta, beta2};
    const uintptr_t rm_[2] = {running_mean, running_mean2}, rv_[2] = {running_var, running_var2};
    const uintptr_t sm_[2] = {save_mean, save_mean2}, si_[2] = {save_invstd, save_invstd2};
    const int pre[2] = {pre_nb, pre_nb2};
    for (int i = 0; i < 2; ++i) {
      float* ws = reinterpret_cast<float*>(ws_[i]);
      const int nb = pre[i] > 0 ? pre[i] : rg.nb;
      abs_[i] = ws + int64_t(2) * nb * C;
      if (pre[i] <= 0)
        hipLaunchKernelGGL((bn_stats_kernel<T, 8>), rg.grid, dim3(kBlock), 0, s, reinterpret_cast<const T*>(xs[i]),
                           ws, M, C, sw);
      hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinCh * kFinRg), 0, s, ws,
                         nb, M, C, reinterpret_cast<const float*>(g_[i]), reinterpret_cast<const float*>(b_[i]),
                         reinterpret_cast<float*>(rm_[i]), reinterpret_cast<float*>(rv_[i]),
                         reinterpret_cast<float*>(sm_[i]), reinterpret_cast<float*>(si_[i]), abs_[i], eps, momentum);
    }
    const T* xp = reinterpret_cast<const T*>(x);
    const T* qp = reinterpret_cast<const T*>(x2);
    T* yp = reinterpret_cast<T*>(y);
    uint8_t* mp = reinterpret_cast<uint8_t*>(mask);
    if (relu)
      hipLaunchKernelGGL((bn_apply2_kernel<T, true>), ag.grid, dim3(kBlock), 0, s, xp, qp, abs_[0], abs_[1], yp, mp, M, C,
                         sw);
    else
      hipLaunchKernelGGL((bn_apply2_kernel<T, false>), ag.grid, dim3(kBlock), 0, s, xp, qp, abs_[0], abs_[1], yp, mp, M,
                         C, sw);
  });
  check_launch();
}

void bn2_bwd(uintptr_t dy, uintptr_t mask, uintptr_t x, uintptr_t x2, uintptr_t save_mean, uintptr_t save_invstd,
             uintptr_t gamma, uintptr_t save_mean2, uintptr_t save_invstd2, uintptr_t gamma2, uintptr_t dx,
             uintptr_t dx2, uintptr_t dgamma, uintptr_t dbeta, uintptr_t dgamma2, uintptr_t dbeta2,
             uintptr_t workspace, int64_t M, int C, bool relu, bool accumulate, int dt, uintptr_t stream,
             uintptr_t pre_part, int pre_nb) {
  VODA_CHECK(C % kVec == 0, "batchnorm: C must be a multiple of 8");
  VODA_CHECK(!relu || mask != 0, "batchnorm backward: ReLU needs the forward's bit-mask");
  VODA_CHECK(pre_nb <= 0 || pre_part != 0, "batchnorm backward: precomputed sums need their partials");
  hipStream_t s = as_stream(stream);
  float* ws = reinterpret_cast<float*>(workspace);
  const Grid rg = reduce_grid(M, C, dt);
  // pre_nb > 0: [3][pre_nb][C] partials (sum g, sum g*x, sum g*x2) from the producer of dy
  const bool pre = pre_nb > 0;
  const int nb = pre ? pre_nb : rg.nb;
  const int64_t nbC = int64_t(nb) * C;
  const float* part = pre ? reinterpret_cast<const float*>(pre_part) : ws;
  float* k3 = pre ? ws : ws + 3 * nbC;
  float* k3b = k3 + 3 * int64_t(C);
  const Grid ag = apply_grid(M, C);
  const int sw = bn_tune().sweep;
  dispatch_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    const T* dyp = reinterpret_cast<const T*>(dy);
    const uint8_t* mp = reinterpret_cast<const uint8_t*>(mask);
    const T* xp = reinterpret_cast<const T*>(x);
    const T* qp = reinterpret_cast<const T*>(x2);
    if (pre) {
    } else if (relu)
      hipLaunchKernelGGL((bn_bwd_reduce2_kernel<T, true, 4>), rg.grid, dim3(kBlock), 0, s, dyp, mp, xp, qp, ws, M, C, sw);
    else
      hipLaunchKernelGGL((bn_bwd_reduce2_kernel<T, false, 4>), rg.grid, dim3(kBlock), 0, s, dyp, mp, xp, qp, ws, M, C,
                         sw);
    const dim3 fg((C + kFinCh - 1) / kFinCh), fb(kFinCh * kFinRg);
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, fg, fb, 0, s, part, part + nbC, nb, M, C,
                       reinterpret_cast<const float*>(gamma), reinterpret_cast<const float*>(save_mean),
                       reinterpret_cast<const float*>(save_invstd), reinterpret_cast<float*>(dgamma),
                       reinterpret_cast<float*>(dbeta), k3, int(accumulate));
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, fg, fb, 0, s, part, part + 2 * nbC, nb, M, C,
                       reinterpret_cast<const float*>(gamma2), reinterpret_cast<const float*>(save_mean2),
                       reinterpret_cast<const float*>(save_invstd2), reinterpret_cast<float*>(dgamma2),
                       reinterpret_cast<float*>(dbeta2), k3b, int(accumulate));
    T* dxp = reinterpret_cast<T*>(dx);
    T* dqp = reinterpret_cast<T*>(dx2);
    if (relu)
      hipLaunchKernelGGL((bn_bwd_apply2_kernel<T, true>), ag.grid, dim3(kBlock), 0, s, dyp, mp, xp, qp, k3, k3b, dxp, dqp,
                         M, C, sw);
    else
      hipLaunchKernelGGL((bn_bwd_apply2_kernel<T, false>), ag.grid, dim3(kBlock), 0, s, dyp, mp, xp, qp, k3, k3b, dxp,
                         dqp, M, C, sw);
  });
  check_launch();
}

// ---- stem BN + ReLU + max pool ----
namespace {
constexpr int kPoolRedBlocks = 2048;  // 8 four-wave blocks per CU: the gather loop is latency-bound
int pool_red_blocks(int N, int H) { return std::max(1, std::min(kPoolRedBlocks, N * H)); }
// 2x2-pixel-block backward passes (round 3: reduce 190 -> 130 us, apply 293 -> 177 us); the
// generic one-pixel-per-thread passes stay for geometries they do not cover
bool pool22_enabled() { return true; }
void check_pool(int N, int H, int W, int C, int Ho, int Wo, int k, int s, int p) {
  VODA_CHECK(C % kVec == 0 && C <= kVec * kMaxTpr, "bn_pool: C must be a multiple of 8 and <= 2048");
  VODA_CHECK(k == 3 && s == 2 && p >= 0 && 2 * p <= k, "bn_pool: only the 3x3 / stride-2 window is compiled");
  VODA_CHECK(Ho == (H + 2 * p - k) / s + 1 && Wo == (W + 2 * p - k) / s + 1, "bn_pool: output size mismatch");
  VODA_CHECK(int64_t(N) * H < (int64_t(1) << 31) && int64_t(W) * (C / kVec) < (int64_t(1) << 24),
             "bn_pool: shape too large");
}
}  // namespace

int64_t bn_pool_workspace_floats(int N, int H, int C) {
  return int64_t(2) * pool_red_blocks(N, H) * C + 3 * int64_t(C);
}

void bn_pool_fwd_train(uintptr_t x, uintptr_t gamma, uintptr_t beta, uintptr_t running_mean, uintptr_t running_var,
                       uintptr_t save_mean, uintptr_t save_invstd, uintptr_t y, uintptr_t idx, uintptr_t workspace,
                       int N, int H, int W, int C, int Ho, int Wo, int k, int s, int p, float eps, float momentum,
                       int dt, uintptr_t stream, int pre_nb) {
  check_pool(N, H, W, C, Ho, Wo, k, s, p);
  hipStream_t st = as_stream(stream);
  const int64_t M = int64_t(N) * H * W;
  float* ws = reinterpret_cast<float*>(workspace);
  // the statistics pass on a grid of at most pool_red_blocks partial rows (fits the workspace),
  // or the pre_nb rows the producing convolution already wrote (stem.hip)
  const Grid rg = bn_grid(M, C, pool_red_blocks(N, H), 8);
  const int nb = pre_nb > 0 ? pre_nb : rg.nb;
  float* ab = ws + int64_t(2) * nb * C;
  const PoolG g{N, H, W, C, Ho, Wo, k, s, p};
  const dim3 pgrid(unsigned(int64_t(N) * Ho), unsigned((Wo * (C / kVec) + kBlock - 1) / kBlock));
  dispatch_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    const T* xp = reinterpret_cast<const T*>(x);
    if (pre_nb <= 0) hipLaunchKernelGGL((bn_stats_kernel<T, 8>), rg.grid, dim3(kBlock), 0, st, xp, ws, M, C, 1);
    hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinCh * kFinRg), 0, st, ws,
                       nb, M, C, reinterpret_cast<const float*>(gamma), reinterpret_cast<const float*>(beta),
                       reinterpret_cast<float*>(running_mean), reinterpret_cast<float*>(running_var),
                       reinterpret_cast<float*>(save_mean), reinterpret_cast<float*>(save_invstd), ab, eps, momentum);
    hipLaunchKernelGGL((bn_pool_fwd_kernel<T, 3, 2>), pgrid, dim3(kBlock), 0, st, xp, ab, reinterpret_cast<T*>(y),
                       reinterpret_cast<uint8_t*>(idx), g);
  });
  check_launch();
}

void bn_pool_bwd(uintptr_t dy, uintptr_t idx, uintptr_t x, uintptr_t save_mean, uintptr_t save_invstd,
                 uintptr_t gamma, uintptr_t dx, uintptr_t dgamma, uintptr_t dbeta, uintptr_t workspace, int N, int H,
                 int W, int C, int Ho, int Wo, int k, int s, int p, bool accumulate, int dt, uintptr_t stream) {
  check_pool(N, H, W, C, Ho, Wo, k, s, p);
  hipStream_t st = as_stream(stream);
  const int64_t M = int64_t(N) * H * W;
  float* ws = reinterpret_cast<float*>(workspace);
  const int nb = pool_red_blocks(N, H);
  float* k3 = ws + int64_t(2) * nb * C;
  const PoolG g{N, H, W, C, Ho, Wo, k, s, p};
  const dim3 agrid(unsigned(int64_t(N) * H), unsigned((W * (C / kVec) + kBlock - 1) / kBlock));
  // pad 1 (the stem): 2 x 2 input pixels per thread share their 4 windows (see pool22_grads)
  const bool p22 = p == 1 && pool22_enabled();
  const dim3 agrid22(unsigned(int64_t(N) * ((H + 1) / 2)), unsigned(((W + 1) / 2 * (C / kVec) + kBlock - 1) / kBlock));
  dispatch_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    const T* dyp = reinterpret_cast<const T*>(dy);
    const uint8_t* ip = reinterpret_cast<const uint8_t*>(idx);
    const T* xp = reinterpret_cast<const T*>(x);
    if (p22)
      hipLaunchKernelGGL((bn_pool_bwd_reduce22_kernel<T>), dim3(nb), dim3(kBlock), 0, st, dyp, ip, xp, ws, g);
    else
      hipLaunchKernelGGL((bn_pool_bwd_reduce_kernel<T, 3, 2>), dim3(nb), dim3(kBlock), 0, st, dyp, ip, xp, ws, g);
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinCh * kFinRg), 0, st, ws,
                       ws + int64_t(nb) * C, nb, M, C, reinterpret_cast<const float*>(gamma), reinterpret_cast<const float*>(save_mean),
                       reinterpret_cast<const float*>(save_invstd), reinterpret_cast<float*>(dgamma),
                       reinterpret_cast<float*>(dbeta), k3, int(accumulate));
    if (p22)
      hipLaunchKernelGGL((bn_pool_bwd_apply22_kernel<T>), agrid22, dim3(kBlock), 0, st, dyp, ip, xp, k3,
                         reinterpret_cast<T*>(dx), g);
    else
      hipLaunchKernelGGL((bn_pool_bwd_apply_kernel<T, 3, 2>), agrid, dim3(kBlock), 0, st, dyp, ip, xp, k3,
                         reinterpret_cast<T*>(dx), g);
  });
  check_launch();
}

}  // namespace voda
