// Column sums for Linear-layer backward: db += sum_rows(dY) for dY [M][N] (bf16/fp16/fp32),
// accumulated straight into the parameter's gradient buffer (fp32 or 16-bit).
//
// The stock path (``dy.sum(0)`` + the autograd accumulate-add) costs a ~20 us reduction plus
// a ~6 us add kernel per Linear per step on BERT-base (8192 x 768 / 3072 dY, profiles/):
// the reduction is latency-bound far from the 12-50 MB it has to read.  Here a thread owns
// 8 consecutive columns (one 16-byte load per row), a block covers floor(256 / (N/8)) rows
// per iteration, every block writes one fp32 partial row, and a finalize kernel (8 columns x
// 32 row groups per block) sums the partials in fp32 and adds them into the gradient.
#include "common.h"
#include "ops.h"

namespace voda {

namespace {

constexpr int kBlock = 256;

template <typename T> __device__ __forceinline__ void load8(const T* p, float (&v)[8]);
template <> __device__ __forceinline__ void load8<BF16>(const BF16* p, float (&v)[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) { v[2 * k] = bf2f(w[k] & 0xffff); v[2 * k + 1] = bf2f(w[k] >> 16); }
}
template <> __device__ __forceinline__ void load8<F16>(const F16* p, float (&v)[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) { v[2 * k] = h2f(w[k] & 0xffff); v[2 * k + 1] = h2f(w[k] >> 16); }
}
template <> __device__ __forceinline__ void load8<float>(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void colsum_partial_kernel(const T* __restrict__ x, float* __restrict__ part,
                                                               int64_t M, int N) {
  const int groups = N / 8;
  const int slice0 = blockIdx.y * kBlock;
  const int tpr = min(groups - slice0, kBlock);
  const int rpi = kBlock / tpr;
  const int t = threadIdx.x;
  const bool active = t < rpi * tpr;
  const int cg = slice0 + (active ? t % tpr : 0);
  const int rsub = active ? t / tpr : 0;
  const int64_t iters = (M + rpi - 1) / rpi;
  const int64_t per = (iters + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = int64_t(blockIdx.x) * per * rpi;
  const int64_t r1 = min<int64_t>(M, r0 + per * rpi);
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (active) {
    const int64_t col = int64_t(cg) * 8;
    int64_t r = r0 + rsub;
    for (; r + 3 * rpi < r1; r += 4 * rpi) {
      float a[8], b[8], c[8], d[8];
      load8<T>(x + r * N + col, a);
      load8<T>(x + (r + rpi) * N + col, b);
      load8<T>(x + (r + 2 * rpi) * N + col, c);
      load8<T>(x + (r + 3 * rpi) * N + col, d);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += (a[k] + b[k]) + (c[k] + d[k]);
    }
    for (; r < r1; r += rpi) {
      float a[8];
      load8<T>(x + r * N + col, a);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += a[k];
    }
  }
  __shared__ float red[kBlock][9];
#pragma unroll
  for (int k = 0; k < 8; ++k) red[t][k] = s[k];
  __syncthreads();
  if (active && rsub == 0) {
    for (int rr = 1; rr < rpi; ++rr)
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += red[t + rr * tpr][k];
    float* out = part + int64_t(blockIdx.x) * N + int64_t(cg) * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = s[k];
  }
}

template <typename OT>
__global__ __launch_bounds__(256) void colsum_finalize_kernel(const float* __restrict__ part, int nb, int N,
                                                             OT* __restrict__ out, int accumulate) {
  __shared__ float red[32][9];
  const int cl = threadIdx.x % 8, rg = threadIdx.x / 8;
  const int c = blockIdx.x * 8 + cl;
  float a = 0.f;
  if (c < N)
    for (int r = rg; r < nb; r += 32) a += part[int64_t(r) * N + c];
  red[rg][cl] = a;
  __syncthreads();
  if (rg == 0 && c < N) {
    float tot = 0.f;
    for (int k = 0; k < 32; ++k) tot += red[k][cl];
    if (accumulate) tot += Vec4<OT>::load1(out, c);
    Vec4<OT>::store1(out, c, tot);
  }
}

int colsum_blocks(int64_t M, int N) {
  const int groups = N / 8;
  const int tpr = std::min(groups, kBlock);
  const int rpi = kBlock / tpr;
  const int64_t iters = (M + rpi - 1) / rpi;
  const int64_t cap = std::max<int64_t>(1, std::min<int64_t>(512, (1 << 20) / N));
  return int(std::max<int64_t>(1, std::min<int64_t>((iters + 7) / 8, cap)));
}

}  // namespace

int64_t colsum_workspace_floats(int64_t M, int N) { return int64_t(colsum_blocks(M, N)) * N; }

void colsum_accumulate(uintptr_t x, int64_t M, int N, int dt, uintptr_t out, int out_dt, bool accumulate,
                       uintptr_t workspace, uintptr_t stream) {
  VODA_CHECK(N % 8 == 0, "colsum: N must be a multiple of 8");
  VODA_CHECK(M > 0, "colsum: empty input");
  hipStream_t s = as_stream(stream);
  const int nb = colsum_blocks(M, N);
  const dim3 grid(unsigned(nb), unsigned((N / 8 + kBlock - 1) / kBlock));
  float* ws = reinterpret_cast<float*>(workspace);
  if (dt == kBF16)
    hipLaunchKernelGGL((colsum_partial_kernel<BF16>), grid, dim3(kBlock), 0, s, reinterpret_cast<const BF16*>(x), ws, M, N);
  else if (dt == kF16)
    hipLaunchKernelGGL((colsum_partial_kernel<F16>), grid, dim3(kBlock), 0, s, reinterpret_cast<const F16*>(x), ws, M, N);
  else
    hipLaunchKernelGGL((colsum_partial_kernel<float>), grid, dim3(kBlock), 0, s, reinterpret_cast<const float*>(x), ws, M, N);
  const dim3 fg(unsigned((N + 7) / 8));
  if (out_dt == kF32)
    hipLaunchKernelGGL((colsum_finalize_kernel<float>), fg, dim3(256), 0, s, ws, nb, N, reinterpret_cast<float*>(out), int(accumulate));
  else if (out_dt == kBF16)
    hipLaunchKernelGGL((colsum_finalize_kernel<BF16>), fg, dim3(256), 0, s, ws, nb, N, reinterpret_cast<BF16*>(out), int(accumulate));
  else
    hipLaunchKernelGGL((colsum_finalize_kernel<F16>), fg, dim3(256), 0, s, ws, nb, N, reinterpret_cast<F16*>(out), int(accumulate));
  check_launch();
}

}  // namespace voda
