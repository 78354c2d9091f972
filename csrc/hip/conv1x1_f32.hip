// fp32 1x1-convolution GEMMs on the f32-input MFMA of gfx950 (v_mfma_f32_32x32x2_f32: exact
// fp32, one rounding per product, 157 TF = the fp32 VALU rate; no xf32 on CDNA4).  The
// reference trains in fp32 (tensorflow2_keras_cifar_elastic.py:147-166), so ResNet-50's
// fp32 step is the headline's; these kernels own the 1x1 convolutions of its bottlenecks:
//
//   forward       Y[M][N] (+)= X[M][K] . W[N][K]^T  with the BN statistics of Y's columns in
//                 the epilogue (per-workgroup partial sums for batchnorm.hip's finalize) --
//                 the statistics pass over Y disappears;
//
// Operand layout of v_mfma_f32_32x32x2_f32: lane l holds A[i = l&31][k = l>>5] and
// B[k = l>>5][j = l&31] (one f32 each); C/D: col = l&31, row = (reg&3) + 8(reg>>2) + 4(l>>5).
//
// Forward (gemm_f32_stats_kernel), the fp32 twin of gemm_bnstats.hip: a workgroup keeps the
// W column tile [NC][K] in LDS (row pitch K + 4 floats: the 16-lane groups of ds_read_b128
// cover all 64 banks once) and walks every G-th 128-row tile; each wave owns 32 rows.  The
// reduction index is PERMUTED inside every 8-wide k chunk: lane half h takes k = 8q + 4h + s
// for MFMA s = 0..3, so each lane feeds four MFMAs from ONE 16-byte load of X (straight from
// global memory, double-buffered across row tiles) and one 16-byte LDS read of W -- the sum is
// over the same k set, in a different (equally exact-per-product) order.
//
// The split-K fp32 weight-gradient kernel and its streaming form for narrow outputs were removed
// in round 5: MIOpen's igemm_wrw ran every ResNet-50 1x1 weight gradient faster (split-K 13.6 vs
// 9.7 ms summed over the layers, streaming 400 vs 252 us on 56x56 64 -> 256;
// profiles/r4/resnet50_fp32_1x1_own_vs_miopen.jsonl, resnet50_fp32_1x1_wgrad_stream.jsonl).
#include "common.h"
#include "ops.h"

#include <algorithm>
#include <type_traits>
#include <cstdlib>

namespace voda {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------------------------------
// forward GEMM + BN statistics
// ------------------------------------------------------------------------------------------
constexpr int kFThreads = 256;
constexpr int kFRows = 128;  // rows per row tile (32 per wave)

struct FArgs {
  const float* x;  // [M][K]
  const float* w;  // [N][K], or [K][N] when w_kn (an input gradient's dY . W[Cout][Cin])
  float* y;        // [M][N]
  float* part;     // [2][G][N] (null: no statistics)
  int64_t M;
  int N, G;
  int accumulate;  // Y += X W^T (statistics then describe X W^T alone)
  int w_kn;
};

template <int NT, int K, bool DBUF>
__global__ __launch_bounds__(kFThreads, 2) void gemm_f32_stats_kernel(FArgs p) {
  constexpr int PK = K + 4;     // LDS floats per W row
  constexpr int NC = 32 * NT;   // columns per workgroup
  constexpr int KQ = K / 8;     // 8-wide k chunks
  __shared__ __attribute__((aligned(16))) float wl[NC * PK];
  __shared__ float red[4][2][NC];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int lc = lane & 31, lh = lane >> 5;
  const int nt = blockIdx.x / p.G, g = blockIdx.x - nt * p.G;
  const int n0 = nt * NC;

  if (p.w_kn) {
    // W^T stored [K][N]: 16-byte loads along n, transposed into the [n][k] LDS rows (the
    // input gradient runs without a transposed copy of the weight per call)
    for (int i = tid; i < K * (NC / 4); i += kFThreads) {
      const int k = i / (NC / 4), c = i - k * (NC / 4);
      const float4 v = *reinterpret_cast<const float4*>(p.w + int64_t(k) * p.N + n0 + 4 * c);
      wl[(4 * c + 0) * PK + k] = v.x;
      wl[(4 * c + 1) * PK + k] = v.y;
      wl[(4 * c + 2) * PK + k] = v.z;
      wl[(4 * c + 3) * PK + k] = v.w;
    }
  } else {
    for (int i = tid; i < NC * (K / 4); i += kFThreads) {
      const int r = i / (K / 4), c = i - r * (K / 4);
      *reinterpret_cast<float4*>(wl + r * PK + 4 * c) = *reinterpret_cast<const float4*>(p.w + int64_t(n0 + r) * K + 4 * c);
    }
  }
  __syncthreads();

  f32x16 acc[NT];
  float s1[NT], s2[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) { s1[t] = 0.f; s2[t] = 0.f; }

  const int64_t ntiles = (p.M + kFRows - 1) / kFRows;
  float4 cur[KQ], nxt[DBUF ? KQ : 1];
  auto src_of = [&](int64_t mt) {
    int64_t row = mt * kFRows + 32 * wave + lc;
    row = row < p.M ? row : p.M - 1;  // rows past M: any valid row, masked in the epilogue
    return p.x + row * K + 4 * lh;
  };
  auto load_a = [&](int64_t mt, float4 (&dst)[KQ]) {
    const float* src = src_of(mt);
#pragma unroll
    for (int q = 0; q < KQ; ++q) dst[q] = *reinterpret_cast<const float4*>(src + 8 * q);
  };
  int64_t mt = g;
  if (mt < ntiles) load_a(mt, cur);
  for (; mt < ntiles; mt += p.G) {
    const bool more = mt + p.G < ntiles;
    if constexpr (DBUF) {
      if (more) {
        const float* src = src_of(mt + p.G);
#pragma unroll
        for (int q = 0; q < KQ; ++q) nxt[q] = *reinterpret_cast<const float4*>(src + 8 * q);
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const float4 a = cur[q];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float4 b = *reinterpret_cast<const float4*>(wl + (32 * t + lc) * PK + 8 * q + 4 * lh);
        acc[t] = mfma32(a.x, b.x, acc[t]);
        acc[t] = mfma32(a.y, b.y, acc[t]);
        acc[t] = mfma32(a.z, b.z, acc[t]);
        acc[t] = mfma32(a.w, b.w, acc[t]);
      }
      // keep the scheduler from hoisting every chunk's W reads ahead of the MFMAs (register
      // pressure -> scratch spills at K >= 128)
      if ((q & 1) == 1) __builtin_amdgcn_sched_barrier(0);
      if constexpr (!DBUF) {
        // single buffer, pipelined by halves: once the first half of the k chunks has fed its
        // MFMAs, those registers take the NEXT row tile's first half, so the loads are in
        // flight during the second half's MFMAs (and the epilogue)
        if (q == KQ / 2 - 1 && more) {
          const float* src = src_of(mt + p.G);
#pragma unroll
          for (int qq = 0; qq < KQ / 2; ++qq) cur[qq] = *reinterpret_cast<const float4*>(src + 8 * qq);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    if constexpr (!DBUF) {
      if (more) {  // the second half: in flight during the epilogue
        const float* src = src_of(mt + p.G);
#pragma unroll
        for (int qq = KQ / 2; qq < KQ; ++qq) cur[qq] = *reinterpret_cast<const float4*>(src + 8 * qq);
      }
    }
    // ---- epilogue: statistics (rows < M) and the fp32 output (128-byte half-wave rows)
    const int64_t rbase = mt * kFRows + 32 * wave;
    const bool full = rbase + 32 <= p.M;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float* ycol = p.y + n0 + 32 * t + lc;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = rbase + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const bool keep = full || row < p.M;
        const float v = acc[t][r];
        if (keep) {
          float* dst = ycol + row * p.N;
          *dst = p.accumulate ? *dst + v : v;
          s1[t] += v;
          s2[t] = fmaf(v, v, s2[t]);
        }
      }
    }
    if constexpr (DBUF) {
      if (more) {
#pragma unroll
        for (int q = 0; q < KQ; ++q) cur[q] = nxt[q];
      }
    }
  }

  if (p.part == nullptr) return;
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
  for (int c = tid; c < NC; c += kFThreads) {
    const float a1 = (red[0][0][c] + red[1][0][c]) + (red[2][0][c] + red[3][0][c]);
    const float a2 = (red[0][1][c] + red[1][1][c]) + (red[2][1][c] + red[3][1][c]);
    p.part[int64_t(g) * p.N + n0 + c] = a1;
    p.part[int64_t(p.G) * p.N + int64_t(g) * p.N + n0 + c] = a2;
  }
}

// ------------------------------------------------------------------------------------------
// input gradient of an identity bottleneck's first 1x1 convolution with the BN handoffs fused
// ------------------------------------------------------------------------------------------
// In a ResNet identity block b the block input x_b feeds conv1_b and the shortcut, and x_b is
// the output of the previous block's relu(bn3(y3) + shortcut).  Its gradient is
//
//   dx_b = dY1 . W1  +  dout_b * [out_b > 0]               (conv1_b input grad + shortcut grad)
//
// and it is immediately consumed by bn3_{b-1}'s backward, whose first pass only reduces
// sum(g) and sum(g * y3_{b-1}) with g = dx_b * [out_{b-1} > 0].  Unfused that is: bn3_b's
// backward writing the masked shortcut gradient (1 tensor), hipBLASLt reading it back as the
// beta = 1 operand (1), and bn3_{b-1}'s reduce pass reading dx_b and y3_{b-1} again (2).  Here
// the epilogue reads dout_b and its 1-bit ReLU mask directly (the shortcut gradient is never
// written) and accumulates bn3_{b-1}'s two sums -- three for a downsample block's dual BN, whose
// shortcut input y_ds gets its own sum(g * y_ds) -- with y3_{b-1} read once: 4 -> 1 tensor passes
// per block.  The sums leave as per-workgroup partials [NS][G][N] for batchnorm.hip's finalize.
// The C-side operands of a 32-column tile are loaded as one batch before any of its results is
// written (a load -> add -> store chain per element serialises on possible aliasing).
struct DArgs {
  const float* x;          // dY1 [M][K]
  const float* w;          // W1 [K = Cout][N = Cin]
  float* y;                // dx_b [M][N]
  const float* cg;         // dout_b [M][N]
  const uint32_t* cmask;   // bn3_b's ReLU bits [M][N/32] words (bit j of word (r, c/32) = column c), or null
  const uint32_t* smask;   // bn3_{b-1}'s ReLU bits (NS > 0)
  const float* s1;         // y3_{b-1} [M][N] (NS > 0)
  const float* s2;         // y_ds_{b-1} [M][N] (NS == 3)
  float* part;             // [NS][G][N]
  int64_t M;
  int N, G;
};

// The epilogue keeps its C-side operands in flight: the loads of 32-column tile t + 1 are
// issued before tile t is finished, and tile 0's before the row tile's MFMAs.  The mask words
// of the wave's 32 rows are one load per lane, spread to the lanes' rows by ds_bpermute.  To
// leave registers for that, a wave holds fewer columns than the statistics GEMM (NT 4 / 2 / 1 at
// K = 64 / 128 / 256); the column groups of one row group are XCD neighbours, so the repeated
// dY row loads hit the same L2.
template <int NT, int NS>
struct EpiBuf {
  float cv[16];
  float v1[NS > 0 ? 16 : 1];
  float v2[NS == 3 ? 16 : 1];
  uint32_t cm, sm;
};

template <int NT, int K, int NS>
__global__ __launch_bounds__(kFThreads, 2) void gemm_f32_dgrad_bn_kernel(DArgs p) {
  static_assert(NS == 0 || NS == 2 || NS == 3, "0, 2 or 3 sums");
  constexpr int PK = K + 4;
  constexpr int NC = 32 * NT;
  constexpr int KQ = K / 8;
  __shared__ __attribute__((aligned(16))) float wl[NC * PK];
  __shared__ float red[4][NS > 0 ? NS : 1][NC];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int lc = lane & 31, lh = lane >> 5;
  // XCD-aware: hardware places block b on XCD b % 8; logical blocks L = (b % 8) * (grid / 8) + b / 8
  // are contiguous per XCD, and L = g * ncol + nt keeps the column groups of row group g together
  const int ncol = p.N / NC;
  int lb = blockIdx.x;
  if (gridDim.x % 8 == 0) lb = (lb % 8) * int(gridDim.x / 8) + lb / 8;
  const int g = lb / ncol, nt = lb - g * ncol;
  const int n0 = nt * NC;
  const int NW = p.N / 32;  // mask words per row

  for (int i = tid; i < K * (NC / 4); i += kFThreads) {  // W [K][N] -> [n][k] LDS rows
    const int k = i / (NC / 4), c = i - k * (NC / 4);
    const float4 v = *reinterpret_cast<const float4*>(p.w + int64_t(k) * p.N + n0 + 4 * c);
    wl[(4 * c + 0) * PK + k] = v.x;
    wl[(4 * c + 1) * PK + k] = v.y;
    wl[(4 * c + 2) * PK + k] = v.z;
    wl[(4 * c + 3) * PK + k] = v.w;
  }
  __syncthreads();

  f32x16 acc[NT];
  float sa[NT], sb[NT], sc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) { sa[t] = 0.f; sb[t] = 0.f; sc[t] = 0.f; }

  const int64_t ntiles = (p.M + kFRows - 1) / kFRows;
  float4 cur[KQ];
  auto src_of = [&](int64_t mt) {
    int64_t row = mt * kFRows + 32 * wave + lc;
    row = row < p.M ? row : p.M - 1;
    return p.x + row * K + 4 * lh;
  };
  // Buffer resources over the wave's 32 rows starting at rbase: element (r, lane) sits at the
  // per-lane byte offset lane_off plus the wave-uniform row offset of r (a scalar soffset), so
  // the 16 rows cost no 64-bit address registers; rows past M fall outside num_records (loads
  // return 0, stores are dropped).
  auto rsrc = [](const void* base, int64_t bytes) {
    const int64_t b = bytes < 0 ? 0 : (bytes > 0x7fffffff ? 0x7fffffff : bytes);
    const uint64_t a = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(a));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uint64_t(hi) << 32) | lo), 0,
                                             __builtin_amdgcn_readfirstlane(int(b)), 0x00020000);
  };
  auto roff = [&](int r) { return ((r & 3) + 8 * (r >> 2)) * p.N * 4; };  // wave-uniform
  // C-side operands of 32-column tile t of the wave's rows [rbase, rbase + 32)
  auto epi_load = [&](EpiBuf<NT, NS>& b, int64_t rbase, int t) {
    const int64_t left = (p.M - rbase) * p.N * 4;
    const int voff = (4 * lh * p.N + n0 + 32 * t + lc) * 4;
    const auto rc = rsrc(p.cg + rbase * p.N, left);
#pragma unroll
    for (int r = 0; r < 16; ++r) b.cv[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rc, voff, roff(r), 0));
    if constexpr (NS > 0) {
      const auto r1 = rsrc(p.s1 + rbase * p.N, left);
#pragma unroll
      for (int r = 0; r < 16; ++r) b.v1[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r1, voff, roff(r), 0));
    }
    if constexpr (NS == 3) {
      const auto r2 = rsrc(p.s2 + rbase * p.N, left);
#pragma unroll
      for (int r = 0; r < 16; ++r) b.v2[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r2, voff, roff(r), 0));
    }
    // mask words: lane lc loads row rbase + lc's word of this column tile
    const int64_t mleft = (p.M - rbase) * NW * 4;
    const int moff = (lc * NW + ((n0 + 32 * t) >> 5)) * 4;
    b.cm = p.cmask != nullptr ? __builtin_amdgcn_raw_buffer_load_b32(rsrc(p.cmask + rbase * NW, mleft), moff, 0, 0)
                              : 0xffffffffu;
    if constexpr (NS > 0) b.sm = __builtin_amdgcn_raw_buffer_load_b32(rsrc(p.smask + rbase * NW, mleft), moff, 0, 0);
  };
  EpiBuf<NT, NS> eb[2];
  int64_t mt = g;
  if (mt < ntiles) {
    const float* src = src_of(mt);
#pragma unroll
    for (int q = 0; q < KQ; ++q) cur[q] = *reinterpret_cast<const float4*>(src + 8 * q);
  }
  for (; mt < ntiles; mt += p.G) {
    const bool more = mt + p.G < ntiles;
    const int64_t rbase = mt * kFRows + 32 * wave;
    epi_load(eb[0], rbase, 0);  // in flight during the MFMAs
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const float4 a = cur[q];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float4 b = *reinterpret_cast<const float4*>(wl + (32 * t + lc) * PK + 8 * q + 4 * lh);
        acc[t] = mfma32(a.x, b.x, acc[t]);
        acc[t] = mfma32(a.y, b.y, acc[t]);
        acc[t] = mfma32(a.z, b.z, acc[t]);
        acc[t] = mfma32(a.w, b.w, acc[t]);
      }
      if ((q & 1) == 1) __builtin_amdgcn_sched_barrier(0);
      // single X buffer pipelined by halves (see gemm_f32_stats_kernel)
      if (q == KQ / 2 - 1 && more) {
        const float* src = src_of(mt + p.G);
#pragma unroll
        for (int qq = 0; qq < KQ / 2; ++qq) cur[qq] = *reinterpret_cast<const float4*>(src + 8 * qq);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (more) {
      const float* src = src_of(mt + p.G);
#pragma unroll
      for (int qq = KQ / 2; qq < KQ; ++qq) cur[qq] = *reinterpret_cast<const float4*>(src + 8 * qq);
    }
    const auto ry = rsrc(p.y + rbase * p.N, (p.M - rbase) * p.N * 4);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (t + 1 < NT) epi_load(eb[(t + 1) & 1], rbase, t + 1);
      __builtin_amdgcn_sched_barrier(0);
      const EpiBuf<NT, NS>& b = eb[t & 1];
      const int voff = (4 * lh * p.N + n0 + 32 * t + lc) * 4;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int wr = (r & 3) + 8 * (r >> 2) + 4 * lh;  // row within the wave's 32
        const uint32_t cmw = uint32_t(__shfl(int(b.cm), wr));
        const float v = acc[t][r] + (((cmw >> lc) & 1u) ? b.cv[r] : 0.f);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ry, voff, roff(r), 0);
        if constexpr (NS > 0) {
          // rows past M: their smask word loaded as 0 (outside the buffer), so they add nothing
          const uint32_t smw = uint32_t(__shfl(int(b.sm), wr));
          const float gg = ((smw >> lc) & 1u) ? v : 0.f;
          sa[t] += gg;
          sb[t] = fmaf(gg, b.v1[r], sb[t]);
          if constexpr (NS == 3) sc[t] = fmaf(gg, b.v2[r], sc[t]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  if constexpr (NS > 0) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      sa[t] += __shfl_xor(sa[t], 32);
      sb[t] += __shfl_xor(sb[t], 32);
      if constexpr (NS == 3) sc[t] += __shfl_xor(sc[t], 32);
      if (lh == 0) {
        red[wave][0][32 * t + lc] = sa[t];
        red[wave][1][32 * t + lc] = sb[t];
        if constexpr (NS == 3) red[wave][2][32 * t + lc] = sc[t];
      }
    }
    __syncthreads();
    for (int c = tid; c < NC; c += kFThreads) {
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        const float a = (red[0][j][c] + red[1][j][c]) + (red[2][j][c] + red[3][j][c]);
        p.part[(int64_t(j) * p.G + g) * p.N + n0 + c] = a;
      }
    }
  }
}

int f32_cus() {
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

// columns per workgroup: the W tile stays <= ~68 KB of LDS (two workgroups per CU)
int gf_nt(int K) { return K == 64 ? 8 : (K == 128 ? 4 : 2); }

}  // namespace

// columns per wave of the fused input gradient (gemm_f32_dgrad_bn_kernel): what fits 256 VGPRs
// with two tiles of epilogue operands in flight (-Rpass-analysis=kernel-resource-usage: no spills)
int gd_nt(int K, int nsums) { return K == 64 ? 2 : (K == 128 && nsums < 3 ? 2 : 1); }

bool gemm_f32_dgrad_bn_supported(int64_t M, int N, int K) {
  return M > 0 && (K == 64 || K == 128 || K == 256) && N % 64 == 0;
}

// row groups: ~2 workgroups per CU over all column groups, total a multiple of 8 (XCD mapping)
int gemm_f32_dgrad_bn_groups(int64_t M, int N, int K, int nsums) {
  if (!gemm_f32_dgrad_bn_supported(M, N, K)) return 0;
  const int ncol = N / (32 * gd_nt(K, nsums));
  const int64_t ntiles = (M + kFRows - 1) / kFRows;
  int64_t G = std::max<int64_t>(1, std::min<int64_t>(ntiles, (2 * f32_cus() + ncol - 1) / ncol));
  while ((G * ncol) % 8 != 0 && G < ntiles) ++G;
  return int(G);
}

bool gemm_f32_stats_supported(int64_t M, int N, int K) {
  return M > 0 && (K == 64 || K == 128 || K == 256) && N % (32 * gf_nt(K)) == 0;
}

int gemm_f32_stats_groups(int64_t M, int N, int K) {
  if (!gemm_f32_stats_supported(M, N, K)) return 0;
  const int ncol = N / (32 * gf_nt(K));
  const int64_t ntiles = (M + kFRows - 1) / kFRows;
  return int(std::max<int64_t>(1, std::min<int64_t>(ntiles, (2 * f32_cus() + ncol - 1) / ncol)));
}

void gemm_f32_stats(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t part, int64_t M, int N, int K, int G,
                    uintptr_t stream, bool accumulate, bool w_kn) {
  VODA_CHECK(gemm_f32_stats_supported(M, N, K), "gemm_f32_stats: K must be 64, 128 or 256 and N a multiple of the tile");
  VODA_CHECK(G == gemm_f32_stats_groups(M, N, K), "gemm_f32_stats: group count mismatch");
  VODA_CHECK(x % 16 == 0 && w % 16 == 0 && y % 4 == 0 && part % 4 == 0, "gemm_f32_stats: misaligned operands");
  const int nt = gf_nt(K);
  const int ncol = N / (32 * nt);
  FArgs a{reinterpret_cast<const float*>(x), reinterpret_cast<const float*>(w), reinterpret_cast<float*>(y),
          reinterpret_cast<float*>(part), M, N, G, accumulate ? 1 : 0, w_kn ? 1 : 0};
  hipStream_t s = as_stream(stream);
  if (K == 64)
    hipLaunchKernelGGL((gemm_f32_stats_kernel<8, 64, true>), dim3(ncol * G), dim3(kFThreads), 0, s, a);
  else if (K == 128)
    hipLaunchKernelGGL((gemm_f32_stats_kernel<4, 128, false>), dim3(ncol * G), dim3(kFThreads), 0, s, a);
  else
    hipLaunchKernelGGL((gemm_f32_stats_kernel<2, 256, false>), dim3(ncol * G), dim3(kFThreads), 0, s, a);
  check_launch();
}

void gemm_f32_dgrad_bn(uintptr_t dy, uintptr_t w, uintptr_t y, uintptr_t cg, uintptr_t cmask, uintptr_t smask,
                       uintptr_t s1, uintptr_t s2, uintptr_t part, int64_t M, int N, int K, int G, int nsums,
                       uintptr_t stream) {
  VODA_CHECK(gemm_f32_dgrad_bn_supported(M, N, K), "gemm_f32_dgrad_bn: K must be 64, 128 or 256 and N a multiple of 64");
  VODA_CHECK(G == gemm_f32_dgrad_bn_groups(M, N, K, nsums), "gemm_f32_dgrad_bn: group count mismatch");
  VODA_CHECK(nsums == 0 || nsums == 2 || nsums == 3, "gemm_f32_dgrad_bn: 0, 2 or 3 sums");
  VODA_CHECK(nsums == 0 || (smask != 0 && s1 != 0 && part != 0 && (nsums == 2 || s2 != 0)),
             "gemm_f32_dgrad_bn: the BN sums need the ReLU bits, the BN input(s) and a partials buffer");
  VODA_CHECK(dy % 16 == 0 && w % 16 == 0 && y % 4 == 0 && cg % 4 == 0 && cmask % 4 == 0 && smask % 4 == 0,
             "gemm_f32_dgrad_bn: misaligned operands");
  const int ncol = N / (32 * gd_nt(K, nsums));
  DArgs a{reinterpret_cast<const float*>(dy), reinterpret_cast<const float*>(w), reinterpret_cast<float*>(y),
          reinterpret_cast<const float*>(cg), reinterpret_cast<const uint32_t*>(cmask),
          reinterpret_cast<const uint32_t*>(smask), reinterpret_cast<const float*>(s1),
          reinterpret_cast<const float*>(s2), reinterpret_cast<float*>(part), M, N, G};
  hipStream_t s = as_stream(stream);
  const dim3 grid(ncol * G), block(kFThreads);
  auto go = [&](auto ns_c) {
    constexpr int NS = decltype(ns_c)::value;
    if (K == 64) hipLaunchKernelGGL((gemm_f32_dgrad_bn_kernel<2, 64, NS>), grid, block, 0, s, a);
    else if (K == 128) {
      if constexpr (NS < 3) hipLaunchKernelGGL((gemm_f32_dgrad_bn_kernel<2, 128, NS>), grid, block, 0, s, a);
      else hipLaunchKernelGGL((gemm_f32_dgrad_bn_kernel<1, 128, NS>), grid, block, 0, s, a);
    }
    else hipLaunchKernelGGL((gemm_f32_dgrad_bn_kernel<1, 256, NS>), grid, block, 0, s, a);
  };
  if (nsums == 0) go(std::integral_constant<int, 0>{});
  else if (nsums == 2) go(std::integral_constant<int, 2>{});
  else go(std::integral_constant<int, 3>{});
  check_launch();
}

}  // namespace voda
