// LayerNorm forward / backward for CDNA4 (gfx950).
//
// Workload: the Transformer NMT job's encoder/decoder LayerNorms (reference
// examples/py/tensorflow2/neural_machine_translation_with_transformer.py:203-204,257-259:
// 10,240 rows x 256 cols) and BERT-base (rows x 768).  HBM-bound, so:
//   * one wave64 per row, the row held in registers (N <= 64 lanes x 4 x MAXITER),
//     8-B (bf16) / 16-B (f32) loads per lane, mean and variance by two register passes
//     (no Welford, no re-read), butterfly reductions across the 64 lanes;
//   * backward computes dx in the same register-resident pass and accumulates the
//     per-column dgamma/dbeta partials in registers across the rows a block visits,
//     then combines the 4 waves through LDS and writes ONE partial row per block;
//     a second small kernel sums those partials per column.
#include "common.h"

#include <cstdlib>
#include "ops.h"

namespace voda {

// 4 elements of T as raw bits (loaded now, converted later: lets several loads be in flight)
template <typename T> struct Raw4 {
  using type = uint2;
  static __device__ __forceinline__ type load(const T* p, int64_t i4) { return reinterpret_cast<const uint2*>(p)[i4]; }
  static __device__ __forceinline__ float4 cvt(type u) {
    const T* q = reinterpret_cast<const T*>(&u);
    return Vec4<T>::load(q, 0);
  }
};
template <> struct Raw4<float> {
  using type = float4;
  static __device__ __forceinline__ type load(const float* p, int64_t i4) { return reinterpret_cast<const float4*>(p)[i4]; }
  static __device__ __forceinline__ float4 cvt(type u) { return u; }
};

template <typename WT>
__device__ __forceinline__ float4 load_w4(const void* w, int64_t c4) {
  return Vec4<WT>::load(reinterpret_cast<const WT*>(w), c4);
}

// MAXITER: upper bound on 256-column chunks per row (row held as MAXITER float4 per lane)
// RES: y = LN(x + res) with the rounded sum written to ``sum`` (the residual-stream value the
// next sublayer reads and the backward normalises): the transformer block's residual add
// fused into the normalisation pass (one read of each input, no separate add kernel).
template <typename T, typename WT, int MAXITER, bool RES = false>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, const void* __restrict__ gamma,
                                                     const void* __restrict__ beta, T* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int64_t M, int N, float eps, const T* __restrict__ res,
                                                     T* __restrict__ sum) {
  const int lane = threadIdx.x & 63;
  const int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int N4 = N >> 2;
  const T* xr = x + row * N;
  float4 v[MAXITER];
  float s = 0.f;
#pragma unroll
  for (int it = 0; it < MAXITER; ++it)  // unconditional (clamped) loads, zeroed after
    v[it] = Vec4<T>::load(xr, min(it * 64 + lane, N4 - 1));
  // gamma / beta issued with the row, not after the two reductions (a dependent L2 round trip
  // at the end of every row otherwise)
  float4 gw[MAXITER], bw[MAXITER];
#pragma unroll
  for (int it = 0; it < MAXITER; ++it) {
    const int c4 = min(it * 64 + lane, N4 - 1);
    gw[it] = gamma ? load_w4<WT>(gamma, c4) : make_float4(1.f, 1.f, 1.f, 1.f);
    bw[it] = beta ? load_w4<WT>(beta, c4) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if constexpr (RES) {
    const T* rr = res + row * N;
    T* sr = sum + row * N;
    float4 r[MAXITER];
#pragma unroll
    for (int it = 0; it < MAXITER; ++it) r[it] = Vec4<T>::load(rr, min(it * 64 + lane, N4 - 1));
#pragma unroll
    for (int it = 0; it < MAXITER; ++it) {
      float4 t = make_float4(v[it].x + r[it].x, v[it].y + r[it].y, v[it].z + r[it].z, v[it].w + r[it].w);
      alignas(16) T q[4];
      Vec4<T>::store(q, 0, t);  // round to T: statistics of exactly the stored sum
      v[it] = Vec4<T>::load(q, 0);
      if (it * 64 + lane < N4) Vec4<T>::store(sr, it * 64 + lane, v[it]);
    }
  }
#pragma unroll
  for (int it = 0; it < MAXITER; ++it) {
    if (it * 64 + lane >= N4) v[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    s += (v[it].x + v[it].y) + (v[it].z + v[it].w);
  }
  const float inv_n = 1.f / float(N);
  const float mu = wave_sum(s) * inv_n;
  float ss = 0.f;
#pragma unroll
  for (int it = 0; it < MAXITER; ++it) {
    const int c4 = it * 64 + lane;
    if (c4 < N4) {
      const float a = v[it].x - mu, b = v[it].y - mu, c = v[it].z - mu, d = v[it].w - mu;
      ss += (a * a + b * b) + (c * c + d * d);
    }
  }
  const float rs = rsqrtf(wave_sum(ss) * inv_n + eps);
  T* yr = y + row * N;
#pragma unroll
  for (int it = 0; it < MAXITER; ++it) {
    const int c4 = it * 64 + lane;
    if (c4 < N4) {
      const float4 g = gw[it], b = bw[it];
      float4 o;
      o.x = (v[it].x - mu) * rs * g.x + b.x;
      o.y = (v[it].y - mu) * rs * g.y + b.y;
      o.z = (v[it].z - mu) * rs * g.z + b.z;
      o.w = (v[it].w - mu) * rs * g.w + b.w;
      Vec4<T>::store(yr, c4, o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mu;
    rstd_out[row] = rs;
  }
}

// W waves per block (4 or 8): each block writes ONE partial row of dgamma / dbeta, so the grid
// is capped (kLnBwdBlockCap) and more rows in flight per CU have to come from more waves per block
template <typename T, typename WT, int MAXITER, int W = 4>
__global__ __launch_bounds__(64 * W) void ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const void* __restrict__ gamma, T* __restrict__ dx,
                                                     float* __restrict__ part_g, float* __restrict__ part_b,
                                                     int64_t M, int N, float* __restrict__ part_x) {
  // part_x (optional): per-block column sums of dx -- the bias gradient of the Linear whose
  // output is this LayerNorm's input (a post-LN sublayer's last projection), folded in here
  // instead of a separate column-sum pass over dx (ops/dense.BiasHandoff)
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [W][N]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int N4 = N >> 2;
  const float inv_n = 1.f / float(N);
  float4 g[MAXITER], ag[MAXITER], ab[MAXITER], ax[MAXITER];
#pragma unroll
  for (int it = 0; it < MAXITER; ++it) {
    const int c4 = it * 64 + lane;
    g[it] = (gamma && c4 < N4) ? load_w4<WT>(gamma, c4) : make_float4(1.f, 1.f, 1.f, 1.f);
    ag[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    ab[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    ax[it] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // A wave owns rows wave + W*blockIdx.x + k * W*gridDim.x.  The grid is capped (one fp32
  // partial row per block for dgamma/dbeta), so a wave walks several rows; R of them are
  // loaded together before any is reduced, which keeps R row-loads in flight per wave
  // instead of one dependent HBM round trip per row (BERT-base 8192 x 768: 25 -> ~8 us).
  // (8 rows at N <= 768 measured slower in the BERT-base step: 10.36-10.41 vs 10.30-10.33 ms)
  constexpr int R = MAXITER <= 3 ? 4 : (MAXITER <= 4 ? 2 : 1);
  const int64_t rstride = int64_t(gridDim.x) * W;
  for (int64_t row0 = int64_t(blockIdx.x) * W + wave; row0 < M; row0 += rstride * R) {
    // every load is unconditional (clamped row / column) and kept as raw bits until all R
    // rows are in flight; out-of-range lanes are zeroed after the conversion.  A branch or a
    // conversion right behind each load makes hipcc wait for it before issuing the next one.
    typename Raw4<T>::type xr[R][MAXITER], dr[R][MAXITER];
    float mur[R], rsr[R];  // the rows' statistics ride with the row loads (a load issued in the
                           // compute loop below would put one more dependent round trip per row)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int64_t row = min(row0 + j * rstride, M - 1);
#pragma unroll
      for (int it = 0; it < MAXITER; ++it) {
        const int c4 = min(it * 64 + lane, N4 - 1);
        xr[j][it] = Raw4<T>::load(x + row * N, c4);
        dr[j][it] = Raw4<T>::load(dy + row * N, c4);
      }
      mur[j] = mean[row];
      rsr[j] = rstd[row];
    }
    float4 xv[R][MAXITER], dv[R][MAXITER];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const bool rok = row0 + j * rstride < M;
#pragma unroll
      for (int it = 0; it < MAXITER; ++it) {
        const bool ok = rok && (it * 64 + lane < N4);
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        xv[j][it] = ok ? Raw4<T>::cvt(xr[j][it]) : z;
        dv[j][it] = ok ? Raw4<T>::cvt(dr[j][it]) : z;
      }
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int64_t row = row0 + j * rstride;
      if (row >= M) break;  // wave-uniform
      const float mu = mur[j], rs = rsr[j];
      float4 xh[MAXITER], dg[MAXITER];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int it = 0; it < MAXITER; ++it) {
        const int c4 = it * 64 + lane;
        if (c4 < N4) {
          const float4 xw = xv[j][it], dw = dv[j][it];
          xh[it] = make_float4((xw.x - mu) * rs, (xw.y - mu) * rs, (xw.z - mu) * rs, (xw.w - mu) * rs);
          dg[it] = make_float4(dw.x * g[it].x, dw.y * g[it].y, dw.z * g[it].z, dw.w * g[it].w);
          ag[it].x += dw.x * xh[it].x; ag[it].y += dw.y * xh[it].y;
          ag[it].z += dw.z * xh[it].z; ag[it].w += dw.w * xh[it].w;
          ab[it].x += dw.x; ab[it].y += dw.y; ab[it].z += dw.z; ab[it].w += dw.w;
          s1 += (dg[it].x * xh[it].x + dg[it].y * xh[it].y) + (dg[it].z * xh[it].z + dg[it].w * xh[it].w);
          s2 += (dg[it].x + dg[it].y) + (dg[it].z + dg[it].w);
        } else {
          xh[it] = make_float4(0.f, 0.f, 0.f, 0.f);
          dg[it] = xh[it];
        }
      }
      const float c1 = wave_sum(s1) * inv_n;
      const float c2 = wave_sum(s2) * inv_n;
#pragma unroll
      for (int it = 0; it < MAXITER; ++it) {
        const int c4 = it * 64 + lane;
        if (c4 < N4) {
          float4 o;
          o.x = (dg[it].x - xh[it].x * c1 - c2) * rs;
          o.y = (dg[it].y - xh[it].y * c1 - c2) * rs;
          o.z = (dg[it].z - xh[it].z * c1 - c2) * rs;
          o.w = (dg[it].w - xh[it].w * c1 - c2) * rs;
          Vec4<T>::store(dx + row * N, c4, o);
          ax[it].x += o.x; ax[it].y += o.y; ax[it].z += o.z; ax[it].w += o.w;
        }
      }
    }
  }
  if (part_g == nullptr) return;  // gamma/beta gradients not requested
  // combine the W waves' column partials through LDS, gamma, beta [, dx]: one partial row per
  // block (col_sum_kernel adds them up)
  // (one call per array with the array named statically: selecting ag / ab / ax by a loop index
  // made hipcc keep all three in scratch for the whole kernel, 160 B per lane, and the row loop
  // read-modify-wrote them there)
  auto combine = [&](const float4 (&acc)[MAXITER], float* __restrict__ part) {
#pragma unroll
    for (int it = 0; it < MAXITER; ++it) {
      const int c4 = it * 64 + lane;
      if (c4 < N4) reinterpret_cast<float4*>(lds + wave * N)[c4] = acc[it];
    }
    __syncthreads();
    float* out = part + int64_t(blockIdx.x) * N;
    for (int c = threadIdx.x; c < N; c += 64 * W) {
      float t = (lds[c] + lds[N + c]) + (lds[2 * N + c] + lds[3 * N + c]);
      if constexpr (W == 8) t += (lds[4 * N + c] + lds[5 * N + c]) + (lds[6 * N + c] + lds[7 * N + c]);
      out[c] = t;
    }
    __syncthreads();
  };
  combine(ag, part_g);
  combine(ab, part_b);
  if (part_x != nullptr) combine(ax, part_x);
}

// Column sums of a [rows][N] fp32 partial matrix: out[c] = sum_r part[r][c] (cast to WT).
// 32 columns x 8 row-groups per block; every thread keeps 4 independent loads in flight
// (rows <= 256, so <= 32 loads per thread) -- the first version (64 columns x 4 groups,
// 1024 rows) was latency-bound at 64 us per call on BERT (rocprof, profiles/).
// blockIdx.y selects (part, out), (part_b, out_b) or (part_c, out_c): dgamma, dbeta [and the
// input Linear's dbias] in one launch; accumulate: out += sum (the optimizer's flat gradient
// buffer, no autograd add afterwards).
template <typename WT>
__global__ __launch_bounds__(256) void col_sum_kernel(const float* __restrict__ part_a, WT* __restrict__ out_a,
                                                      const float* __restrict__ part_b, WT* __restrict__ out_b,
                                                      int rows, int N, int accumulate,
                                                      const float* __restrict__ part_c = nullptr,
                                                      WT* __restrict__ out_c = nullptr) {
  __shared__ float red[8][33];
  const float* __restrict__ part = blockIdx.y == 0 ? part_a : (blockIdx.y == 1 ? part_b : part_c);
  WT* __restrict__ out = blockIdx.y == 0 ? out_a : (blockIdx.y == 1 ? out_b : out_c);
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + tx;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < N) {
    int r = ty;
    for (; r + 24 < rows; r += 32) {
      s0 += part[int64_t(r) * N + c];
      s1 += part[int64_t(r + 8) * N + c];
      s2 += part[int64_t(r + 16) * N + c];
      s3 += part[int64_t(r + 24) * N + c];
    }
    for (; r < rows; r += 8) s0 += part[int64_t(r) * N + c];
  }
  red[ty][tx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ty == 0 && c < N) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][tx];
    if (accumulate) t += Vec4<WT>::load1(out, c);
    Vec4<WT>::store1(out, c, t);
  }
}

#define LN_DISPATCH_ITER(N, ...)                                     \
  [&] {                                                              \
    const int _it = (N + 255) / 256;                                 \
    if (_it <= 1) { constexpr int MI = 1; __VA_ARGS__(); }           \
    else if (_it <= 2) { constexpr int MI = 2; __VA_ARGS__(); }      \
    else if (_it <= 3) { constexpr int MI = 3; __VA_ARGS__(); }      \
    else if (_it <= 4) { constexpr int MI = 4; __VA_ARGS__(); }      \
    else if (_it <= 8) { constexpr int MI = 8; __VA_ARGS__(); }      \
    else { constexpr int MI = 16; __VA_ARGS__(); }                   \
  }()

#define LN_DISPATCH_T(DT, WDT, ...)                                                     \
  [&] {                                                                                 \
    if (DT == kF32) { using T = float; using WT = float; __VA_ARGS__(); }               \
    else if (DT == kBF16) {                                                             \
      using T = BF16;                                                                   \
      if (WDT == kF32) { using WT = float; __VA_ARGS__(); } else { using WT = BF16; __VA_ARGS__(); } \
    } else {                                                                            \
      using T = F16;                                                                    \
      if (WDT == kF32) { using WT = float; __VA_ARGS__(); } else { using WT = F16; __VA_ARGS__(); } \
    }                                                                                   \
  }()

void layernorm_fwd(uintptr_t x, uintptr_t gamma, uintptr_t beta, uintptr_t y, uintptr_t mean, uintptr_t rstd,
                   int64_t M, int N, float eps, int dt, int wdt, uintptr_t residual, uintptr_t sum, uintptr_t stream) {
  VODA_CHECK((residual == 0) == (sum == 0), "layernorm: residual and sum go together");
  VODA_CHECK(N > 0 && N % 4 == 0 && N <= kLayerNormMaxN, "layernorm: N must be a multiple of 4 and <= 4096");
  VODA_CHECK(dt != kF32 || wdt == kF32, "layernorm: fp32 input needs fp32 weights");
  if (M == 0) return;
  const unsigned grid = unsigned((M + 3) / 4);
  LN_DISPATCH_T(dt, wdt, [&] {
    LN_DISPATCH_ITER(N, [&] {
      if (residual)
        hipLaunchKernelGGL((ln_fwd_kernel<T, WT, MI, true>), dim3(grid), dim3(256), 0, as_stream(stream),
                           reinterpret_cast<const T*>(x), reinterpret_cast<const void*>(gamma),
                           reinterpret_cast<const void*>(beta), reinterpret_cast<T*>(y),
                           reinterpret_cast<float*>(mean), reinterpret_cast<float*>(rstd), M, N, eps,
                           reinterpret_cast<const T*>(residual), reinterpret_cast<T*>(sum));
      else
        hipLaunchKernelGGL((ln_fwd_kernel<T, WT, MI, false>), dim3(grid), dim3(256), 0, as_stream(stream),
                           reinterpret_cast<const T*>(x), reinterpret_cast<const void*>(gamma),
                           reinterpret_cast<const void*>(beta), reinterpret_cast<T*>(y),
                           reinterpret_cast<float*>(mean), reinterpret_cast<float*>(rstd), M, N, eps,
                           static_cast<const T*>(nullptr), static_cast<T*>(nullptr));
    });
  });
  check_launch();
}

// Backward grid cap = rows of fp32 dgamma/dbeta partials: 256 blocks of 4 waves is ONE wave per
// SIMD, each walking M / 1024 rows with R rows of loads in flight.  768 / 1024 blocks took the row
// pass 17.0 -> 15.0 us but the dgamma/dbeta column sum over 3x / 4x the partial rows 5.1 -> 9.9 /
// 12.4 us (profiles/r3/raw/ab_ln_bwd_grid_kernels.txt), so 256 it is.  (An atomic-add dgamma/dbeta
// variant showed no gain within noise, profiles/raw/r2_ab_ln_atomic.jsonl, and was not bitwise
// reproducible; removed in round 5.)
constexpr int kLnBwdBlockCap = 256;
int ln_bwd_block_cap() { return kLnBwdBlockCap; }
// Waves per backward block for N <= 1024 (larger rows keep 4: LDS of W x N floats): 8 gives two
// waves per SIMD at the same 256 partial rows.  Settable for the A/B (benchmarks/bench_layernorm.py).
int g_ln_bwd_waves = 8;
void layernorm_set_bwd_waves(int w) {
  VODA_CHECK(w == 4 || w == 8, "layernorm: 4 or 8 waves per backward block");
  g_ln_bwd_waves = w;
}

int layernorm_bwd_partial_rows(int64_t M) {
  int64_t g = (M + 3) / 4;
  return int(std::max<int64_t>(1, std::min<int64_t>(g, ln_bwd_block_cap())));
}

void layernorm_bwd(uintptr_t dy, uintptr_t x, uintptr_t mean, uintptr_t rstd, uintptr_t gamma, uintptr_t dx,
                   uintptr_t dgamma, uintptr_t dbeta, uintptr_t workspace, int64_t M, int N, int dt, int wdt,
                   bool accumulate, uintptr_t stream, uintptr_t dbias_in) {
  VODA_CHECK(N > 0 && N % 4 == 0 && N <= kLayerNormMaxN, "layernorm: N must be a multiple of 4 and <= 4096");
  if (M == 0) return;
  const int grid = layernorm_bwd_partial_rows(M);
  float* pg = nullptr;
  float* pb = nullptr;
  float* px = nullptr;  // dbias_in: the input Linear's bias gradient, workspace holds 3 partial sets
  if (dgamma != 0) {
    VODA_CHECK(dbeta != 0, "layernorm_bwd: dbeta required");
    VODA_CHECK(workspace != 0, "layernorm_bwd: workspace required");
    pg = reinterpret_cast<float*>(workspace);
    pb = pg + int64_t(grid) * N;
    if (dbias_in != 0) px = pb + int64_t(grid) * N;
  } else {
    VODA_CHECK(dbias_in == 0, "layernorm_bwd: the input bias sum rides with dgamma / dbeta");
  }
  const int W = (g_ln_bwd_waves == 8 && N <= 1024) ? 8 : 4;
  const size_t lds = size_t(W) * N * sizeof(float);
  LN_DISPATCH_T(dt, wdt, [&] {
    LN_DISPATCH_ITER(N, [&] {
      if constexpr (MI <= 4) {
        if (W == 8) {
          hipLaunchKernelGGL((ln_bwd_kernel<T, WT, MI, 8>), dim3(grid), dim3(512), pg ? lds : 0,
                             as_stream(stream), reinterpret_cast<const T*>(dy), reinterpret_cast<const T*>(x),
                             reinterpret_cast<const float*>(mean), reinterpret_cast<const float*>(rstd),
                             reinterpret_cast<const void*>(gamma), reinterpret_cast<T*>(dx), pg, pb, M, N, px);
          return;
        }
      }
      hipLaunchKernelGGL((ln_bwd_kernel<T, WT, MI, 4>), dim3(grid), dim3(256), pg ? lds : 0,
                         as_stream(stream), reinterpret_cast<const T*>(dy), reinterpret_cast<const T*>(x),
                         reinterpret_cast<const float*>(mean), reinterpret_cast<const float*>(rstd),
                         reinterpret_cast<const void*>(gamma), reinterpret_cast<T*>(dx), pg, pb, M, N, px);
    });
    if (pg) {
      const unsigned cg = unsigned((N + 31) / 32);
      hipLaunchKernelGGL((col_sum_kernel<WT>), dim3(cg, px ? 3 : 2), dim3(256), 0, as_stream(stream), pg,
                         reinterpret_cast<WT*>(dgamma), pb, reinterpret_cast<WT*>(dbeta), grid, N,
                         accumulate ? 1 : 0, px, reinterpret_cast<WT*>(dbias_in));
    }
  });
  check_launch();
}

}  // namespace voda
