// 1x1 convolution forward as a GEMM with the batch-norm statistics of its output in the
// epilogue:  Y[M][N] = X[M][K] . W[N][K]^T  (bf16 in / out, fp32 accumulation), plus per
// workgroup partial sums of Y and Y^2 per output channel for the BN finalize kernel
// (batchnorm.hip, unchanged).
//
// Target: ResNet-50's stage-1/2 1x1 convolutions that are memory-bound -- the expansions
// (conv3 / downsample: K = 64 or 128 channels in, N = 4K out) and the stage-1 reductions
// (conv1: K = 256 in, N = 64 out) -- at M = 0.8 M / 0.2 M pixels (bs 256).  The BN statistics
// pass that follows re-reads their outputs (411 / 205 MB for the expansions) at ~4.5 TB/s
// (~90 / ~45 us per layer, profiles/r3/).  Here the statistics come from the accumulators.
//
// Design (v_mfma_f32_32x32x16_bf16, 4 waves, persistent, two workgroups per CU):
//  * a workgroup owns one column tile (NT x 32 output channels) and walks every G-th 128-row
//    tile; its W tile stays in LDS (row pitch 2K + 16 B: the 16-lane groups of ds_read_b128
//    land on distinct banks);
//  * wave w computes rows 32 w .. 32 w + 31 of the row tile against all NT column tiles; the
//    X operand is read straight from global memory into registers (16 B = one MFMA fragment
//    per lane per k-step), double-buffered across row tiles so the next tile's loads are in
//    flight during this tile's MFMAs and stores;
//  * D rows are pixels: a lane holds one output channel of 16 pixels, so the statistics are
//    in-lane sums carried across the whole walk; the output goes out through a per-wave
//    [32 px][64 ch] LDS staging tile as 16-byte stores of whole 128-byte row segments.
#include "common.h"
#include "ops.h"

namespace voda {

namespace {

typedef __bf16 gb_bf16x8 __attribute__((ext_vector_type(8)));
typedef float gb_f32x16 __attribute__((ext_vector_type(16)));

constexpr int kGThreads = 256;
constexpr int kGRows = 128;              // rows per row tile (32 per wave)
constexpr int kGStgStride = 144;         // staging row pitch (128 B + 16 pad)
constexpr int kGStgB = 32 * kGStgStride;  // per wave

struct GArgs {
  const uint16_t* x;  // [M][K]
  const uint16_t* w;  // [N][K]
  uint16_t* y;        // [M][N]
  float* part;        // [2][G][N]
  int64_t M;
  int N, G;
  int accumulate;     // Y += X W^T (the statistics then describe X W^T alone)
};

__device__ __forceinline__ gb_bf16x8 gb_ld16(const uint16_t* p) {
  return __builtin_bit_cast(gb_bf16x8, *reinterpret_cast<const uint4*>(p));
}

template <int NT, int KS>
__global__ __launch_bounds__(kGThreads, 2) void gemm_bnstats_kernel(GArgs p) {
  constexpr int K = 16 * KS;
  constexpr int PW = 2 * K + 16;  // LDS bytes per W row
  constexpr int NC = 32 * NT;     // columns per workgroup
  __shared__ __attribute__((aligned(16))) unsigned char wl[NC * PW];
  __shared__ __attribute__((aligned(16))) unsigned char stg[4 * kGStgB];
  __shared__ float red[4][2][NC];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int lc = lane & 31, lh = lane >> 5;
  const int nt = blockIdx.x / p.G, g = blockIdx.x - (blockIdx.x / p.G) * p.G;
  const int n0 = nt * NC;

  // ---- W tile [NC][K] into LDS
  for (int i = tid; i < NC * (K / 8); i += kGThreads) {
    const int r = i / (K / 8), c = i - r * (K / 8);
    *reinterpret_cast<uint4*>(wl + r * PW + c * 16) =
        *reinterpret_cast<const uint4*>(p.w + int64_t(n0 + r) * K + c * 8);
  }
  __syncthreads();

  gb_f32x16 acc[NT];
  float s1[NT], s2[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) { s1[t] = 0.f; s2[t] = 0.f; }

  const int64_t ntiles = (p.M + kGRows - 1) / kGRows;
  unsigned char* my_stg = stg + wave * kGStgB;
  gb_bf16x8 cur[KS], nxt[KS];
  auto load_a = [&](int64_t mt, gb_bf16x8 (&dst)[KS]) {
    int64_t row = mt * kGRows + 32 * wave + lc;
    row = row < p.M ? row : p.M - 1;  // rows past M: any valid row, masked in the epilogue
    const uint16_t* src = p.x + row * K + 8 * lh;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) dst[ks] = gb_ld16(src + 16 * ks);
  };
  int64_t mt = g;
  if (mt < ntiles) load_a(mt, cur);
  for (; mt < ntiles; mt += p.G) {
    const bool more = mt + p.G < ntiles;
    if (more) load_a(mt + p.G, nxt);
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = gb_f32x16{};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const gb_bf16x8 b = *reinterpret_cast<const gb_bf16x8*>(wl + (32 * t + lc) * PW + (16 * ks + 8 * lh) * 2);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[ks], b, acc[t], 0, 0, 0);
      }
    }
    // ---- epilogue: statistics (rows < M), bf16 through the staging tile, 16-byte stores.
    // The statistics are of the bf16-ROUNDED outputs -- the tensor BN then normalises (a BN
    // statistics pass over the stored Y would see exactly these values), not of the fp32
    // accumulators.  (Accumulating form: they describe the rounded X W^T alone.)
    const int64_t rbase = mt * kGRows + 32 * wave;
    const bool full = rbase + 32 <= p.M;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (full) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float v = bf2f(f2bf(acc[t][r]));
          s1[t] += v; s2[t] = fmaf(v, v, s2[t]);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float keep = rbase + (r & 3) + 8 * (r >> 2) + 4 * lh < p.M ? 1.f : 0.f;
          const float v = bf2f(f2bf(acc[t][r])) * keep;
          s1[t] += v; s2[t] = fmaf(v, v, s2[t]);
        }
      }
    }
#pragma unroll
    for (int pp = 0; pp < NT / 2; ++pp) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int px = (r & 3) + 8 * (r >> 2) + 4 * lh;
        *reinterpret_cast<uint16_t*>(my_stg + px * kGStgStride + lc * 2) = f2bf(acc[2 * pp][r]);
        *reinterpret_cast<uint16_t*>(my_stg + px * kGStgStride + (32 + lc) * 2) = f2bf(acc[2 * pp + 1][r]);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = i * 64 + lane;
        const int px = q >> 3, part = q & 7;
        uint4 v = *reinterpret_cast<const uint4*>(my_stg + px * kGStgStride + part * 16);
        if (rbase + px < p.M) {
          uint4* dst = reinterpret_cast<uint4*>(p.y + (rbase + px) * p.N + n0 + 64 * pp + part * 8);
          if (p.accumulate) {  // 8 bf16 sums in fp32, one rounding of each
            const uint4 o = *dst;
            const uint32_t a[4] = {v.x, v.y, v.z, v.w}, b[4] = {o.x, o.y, o.z, o.w};
            uint32_t r[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float lo = bf2f(uint16_t(a[q] & 0xffff)) + bf2f(uint16_t(b[q] & 0xffff));
              const float hi = bf2f(uint16_t(a[q] >> 16)) + bf2f(uint16_t(b[q] >> 16));
              r[q] = uint32_t(f2bf(lo)) | (uint32_t(f2bf(hi)) << 16);
            }
            v = make_uint4(r[0], r[1], r[2], r[3]);
          }
          *dst = v;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (more) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) cur[ks] = nxt[ks];
    }
  }

  // ---- partials: lanes lc (+ half lh) hold channel 32 t + lc of this wave's rows
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    s1[t] += __shfl_xor(s1[t], 32);
    s2[t] += __shfl_xor(s2[t], 32);
    if (lh == 0) {
      red[wave][0][32 * t + lc] = s1[t];
      red[wave][1][32 * t + lc] = s2[t];
    }
  }
  __syncthreads();
  for (int c = tid; c < NC; c += kGThreads) {
    const float a1 = (red[0][0][c] + red[1][0][c]) + (red[2][0][c] + red[3][0][c]);
    const float a2 = (red[0][1][c] + red[1][1][c]) + (red[2][1][c] + red[3][1][c]);
    p.part[int64_t(g) * p.N + n0 + c] = a1;
    p.part[int64_t(p.G) * p.N + int64_t(g) * p.N + n0 + c] = a2;
  }
}

int gb_cus() {
  static int g = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
      hipDeviceProp_t pr;
      if (hipGetDeviceProperties(&pr, dev) == hipSuccess && pr.multiProcessorCount > 0) cus = pr.multiProcessorCount;
    }
    return cus;
  }();
  return g;
}

// columns per workgroup for a (K, N): NT x 32, NT = 8 at K = 64, 4 at K = 128, 2 at K = 256
// (the W tile stays <= 64 KB of LDS and the double-buffered X fragments <= 128 VGPRs)
int gb_nt(int K) { return K == 64 ? 8 : (K == 128 ? 4 : 2); }

}  // namespace

bool gemm_bnstats_supported(int64_t M, int N, int K) {
  // K = 256: at most two column tiles (every column tile re-reads the whole X operand)
  return M > 0 && (K == 64 || K == 128 || (K == 256 && N <= 128)) && N % (32 * gb_nt(K)) == 0;
}

int gemm_bnstats_groups(int64_t M, int N, int K) {
  if (!gemm_bnstats_supported(M, N, K)) return 0;
  const int ncol = N / (32 * gb_nt(K));
  const int64_t ntiles = (M + kGRows - 1) / kGRows;
  return int(std::max<int64_t>(1, std::min<int64_t>(ntiles, (2 * gb_cus() + ncol - 1) / ncol)));
}

void gemm_bnstats(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t part, int64_t M, int N, int K, int G,
                  uintptr_t stream, bool accumulate) {
  VODA_CHECK(gemm_bnstats_supported(M, N, K), "gemm_bnstats: K must be 64, 128 or 256 and N a multiple of the tile");
  VODA_CHECK(G == gemm_bnstats_groups(M, N, K), "gemm_bnstats: group count mismatch");
  VODA_CHECK(x % 16 == 0 && w % 16 == 0 && y % 16 == 0 && part % 4 == 0, "gemm_bnstats: misaligned operands");
  const int ncol = N / (32 * gb_nt(K));
  GArgs a{reinterpret_cast<const uint16_t*>(x), reinterpret_cast<const uint16_t*>(w), reinterpret_cast<uint16_t*>(y),
          reinterpret_cast<float*>(part), M, N, G, accumulate ? 1 : 0};
  hipStream_t s = as_stream(stream);
  if (K == 64)
    hipLaunchKernelGGL((gemm_bnstats_kernel<8, 4>), dim3(ncol * G), dim3(kGThreads), 0, s, a);
  else if (K == 128)
    hipLaunchKernelGGL((gemm_bnstats_kernel<4, 8>), dim3(ncol * G), dim3(kGThreads), 0, s, a);
  else
    hipLaunchKernelGGL((gemm_bnstats_kernel<2, 16>), dim3(ncol * G), dim3(kGThreads), 0, s, a);
  check_launch();
}

}  // namespace voda
