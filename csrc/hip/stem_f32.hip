// ResNet stem at the reference's precision (fp32): 7x7 / stride-2 / pad-3 convolution of a
// 1..3-channel fp32 image into 64 channels on the f32-input MFMA (v_mfma_f32_32x32x2_f32,
// exact fp32), with the batch-norm statistics of its output computed in the epilogue.
//
// What it replaces (profiles/r5/rocprof_resnet50_fp32_tile_gemm_off.md, one fp32 ResNet-50
// bs256 step): MIOpen's output zero-fill (127 us), igemm_fwd (749 us, ~81 TF on the 60 GFLOP of
// the layer) and the BN statistics pass that re-reads the 822 MB output (197 us).
//
// Design (same skeleton as the bf16 stem of stem.hip; the fp32 operands change the data layout):
//  * the reduction of one filter row kh is k = kw * 3 + c (21 real terms, padded to 24 = three
//    8-wide chunks with zero filter weights), not the bf16 kernel's 8 pixels x 4 channels = 32:
//    168 instead of 224 MFMAs per output row and wave;
//  * input rows live in a 16-slot LDS ring as flat fp32 [264 px][3 ch] (zero outside the image);
//    output pixel wo's window of filter row kh starts at flat index 6 wo, so the permuted-k
//    fragment of lane half h (k = 8 q + 4 h + s for MFMA s) is the float4 at 6 wo + 8 q + 4 h:
//    two ds_read_b64 (24-byte pixel pitch: 8-byte aligned) feed four MFMAs;
//  * a workgroup (4 waves = 2 channel tiles x 2 pixel halves) produces one output row
//    (Wo <= 128) at a time; the filter fragments of the wave's channel tile (7 kh x 3 chunks
//    x float4 = 84 VGPRs) stay in registers for the whole persistent row chunk;
//  * consecutive output rows share 5 of their 7 input rows: the steady state loads the 2 new
//    rows into registers two output rows ahead, while the current row's MFMAs run;
//  * D rows = pixels, columns = channels: a lane holds one channel of 16 pixels, so the
//    per-channel sums / sums of squares are in-lane adds carried across the chunk, and each
//    output store is 32 lanes x 4 B = one 128-byte channels_last segment; stores go through a
//    per-row buffer resource whose bound drops the pixels past Wo.
#include "common.h"

#include <algorithm>
#include <type_traits>
#include "ops.h"

namespace voda {

namespace {

typedef float sf_f32x16 __attribute__((ext_vector_type(16)));
typedef float sf_f32x4 __attribute__((ext_vector_type(4)));  // native vector: HIP's float4 struct
                                                             // arrays are copied through scratch

constexpr int kFK = 7, kFS = 2, kFP = 3;           // filter, stride, padding
constexpr int kFCo = 64;                           // output channels (two 32-wide MFMA tiles)
constexpr int kFC = 3;                             // input channels held per pixel in LDS
constexpr int kFWaves = 4;
constexpr int kFThreads = 64 * kFWaves;
constexpr int kFMaxWo = 128;                       // 2 pixel halves x 2 tiles x 32
constexpr int kFRowPx = 2 * kFMaxWo + 8;           // 264 LDS pixels per input row (wi = -3 ..)
constexpr int kFRowF = kFRowPx * kFC;              // 792 floats
constexpr int kFRowB = kFRowF * 4;                 // 3168 B
constexpr int kFSlots = 16;                        // LDS ring of input rows
constexpr int kFKq = 3;                            // 8-wide k chunks per filter row (24 >= 21)
constexpr int kFPf = (2 * kFRowF + kFThreads - 1) / kFThreads;  // prefetch floats per thread (7)

struct StemF32Args {
  const float* x;                     // image, element strides below
  int64_t sN, sC, sH, sW;
  int cin;
  const float* w;                     // [64][cin][7][7], element strides below
  int64_t sw0, sw1, sw2, sw3;
  float* y;                           // [N][Ho][Wo][64] (channels_last)
  float* part;                        // [2][gridDim.x][64]
  int N, H, W, Ho, Wo;
};

__device__ __forceinline__ sf_f32x16 sf_mfma(float a, float b, sf_f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t sf_rsrc(const void* base, int64_t bytes) {
  const int64_t b = bytes < 0 ? 0 : (bytes > 0x7fffffff ? 0x7fffffff : bytes);
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uint64_t(hi) << 32) | lo), 0,
                                           __builtin_amdgcn_readfirstlane(int(b)), 0x00020000);
}

// byte offset of element j of the flat LDS row of input row hi (pixel wi = j / 3 - 3, channel
// j % 3) in the image, or an offset past the buffer's bound (the load returns 0) outside the
// image and for channels >= cin: branch-free, 32-bit
template <typename Args>
__device__ __forceinline__ uint32_t sf_off(const Args& a, int64_t n, int hi, int j) {
  const int px = j / kFC, c = j - px * kFC;
  const int wi = px - kFP;
  const bool ok = unsigned(hi) < unsigned(a.H) && unsigned(wi) < unsigned(a.W) && c < a.cin;
  const uint32_t o = uint32_t((n * a.sN + c * a.sC + int64_t(hi) * a.sH + int64_t(wi) * a.sW) * 4);
  return ok ? o : 0xfffffff0u;
}

__device__ __forceinline__ float sf_load(__amdgpu_buffer_rsrc_t rx, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, int(off), 0, 0));
}

// the 7 input rows of output row ho into the ring, loads issued in batches of B before their
// LDS writes
template <int B, int RF = kFRowF, typename Args>
__device__ __forceinline__ void sf_fill_window(float* ring, const Args& a, __amdgpu_buffer_rsrc_t rx, int64_t n, int ho,
                                               int tid) {
  constexpr int kTotal = kFK * RF;                              // 5544 (forward rows)
  constexpr int kIters = (kTotal + kFThreads - 1) / kFThreads;  // 22
#pragma unroll
  for (int b = 0; b < kIters; b += B) {
    float v[B];
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const int i = min(tid + (b + u) * kFThreads, kTotal - 1);
      const int r = i / RF, j = i - r * RF;
      v[u] = sf_load(rx, sf_off(a, n, kFS * ho - kFP + r, j));
    }
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const int i = tid + (b + u) * kFThreads;
      if (b + u < kIters && i < kTotal) {
        const int r = i / RF, j = i - r * RF;
        ring[((kFS * ho - kFP + r) & (kFSlots - 1)) * RF + j] = v[u];
      }
    }
  }
}

__global__ __launch_bounds__(kFThreads, 2) void stem_f32_fwd_kernel(StemF32Args a) {
  __shared__ __attribute__((aligned(16))) float ring[kFSlots * kFRowF];  // 50.7 KB
  __shared__ float red[kFWaves][2][32];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int lc = lane & 31, lh = lane >> 5;
  const int ct = wave & 1, ph = wave >> 1;  // channel tile, pixel half

  // ---- filter fragments: the workgroup packs W as [64 co][7 kh][24 k] (k = kw * 3 + c, zero
  // for k >= 21 or c >= cin) into the ring's LDS, then lane (co = 32 ct + lc, half lh) reads
  // float4 [co][kh][8 q + 4 lh] for q = 0..2
  {
    constexpr int kWElems = kFCo * kFK * kFKq * 8;  // 10752
    constexpr int kPer = kWElems / kFThreads;       // 42
#pragma unroll
    for (int b = 0; b < kPer; b += 14) {
      float v[14];
#pragma unroll
      for (int i = 0; i < 14; ++i) {
        const int e = tid + (b + i) * kFThreads;
        const int co = e / (kFK * 24), r = e - co * (kFK * 24);
        const int kh = r / 24, k = r - kh * 24;
        const int kw = k / kFC, c = k - kw * kFC;
        v[i] = (k < kFK * kFC && c < a.cin) ? a.w[co * a.sw0 + c * a.sw1 + kh * a.sw2 + kw * a.sw3] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 14; ++i) ring[tid + (b + i) * kFThreads] = v[i];
    }
  }
  __syncthreads();
  float4 wf[kFK][kFKq];
#pragma unroll
  for (int kh = 0; kh < kFK; ++kh)
#pragma unroll
    for (int q = 0; q < kFKq; ++q) {
      float4 f = *reinterpret_cast<const float4*>(&ring[((32 * ct + lc) * kFK + kh) * 24 + 8 * q + 4 * lh]);
      // opaque to the optimizer: keeps the fragment resident instead of re-deriving it
      asm volatile("" : "+v"(f.x), "+v"(f.y), "+v"(f.z), "+v"(f.w));
      wf[kh][q] = f;
    }
  __syncthreads();  // the ring's LDS is reused below

  // the image through one buffer resource (32-bit offsets; out-of-image elements read 0)
  const auto rx = sf_rsrc(a.x, (int64_t(a.N - 1) * a.sN + int64_t(a.cin - 1) * a.sC + int64_t(a.H - 1) * a.sH +
                                int64_t(a.W - 1) * a.sW + 1) * 4);
  // this thread's share of a 2-row refill: flat slot i = tid + 256 k of 2 x 792 is input row
  // i / 792 (of the two), element i % 792

  float s1 = 0.f, s2 = 0.f;  // channel 32 ct + lc
  const int64_t rows = int64_t(a.N) * a.Ho;
  const int64_t per = (rows + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = int64_t(blockIdx.x) * per;
  const int64_t r1 = r0 + per < rows ? r0 + per : rows;
  const int px0 = 64 * ph;  // this wave's first output pixel (tiles px0, px0 + 32)
  // A operand of pixel tile t: flat index 6 (px0 + 32 t + lc) + 8 q + 4 lh of the row's slot
  const int abase = 6 * (px0 + lc) + 4 * lh;
  // output stores: lane (channel 32 ct + lc) of pixel px0 + 4 lh + row (r & 3) + 8 (r >> 2)
  const int vy = ((px0 + 4 * lh) * kFCo + 32 * ct + lc) * 4;

  int64_t n = r0 / a.Ho;
  int ho = int(r0 - n * a.Ho);
  float pf[2][kFPf];
  bool vv[2] = {false, false};
  bool in_lds = false;
  auto load_rows = [&](float (&dst)[kFPf], int hbase) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < kFPf; ++k) {
      const int i = min(tid + k * kFThreads, 2 * kFRowF - 1);
      const int r = i / kFRowF;
      dst[k] = sf_load(rx, sf_off(a, n, hbase + r, i - r * kFRowF));
    }
  };
  auto step = [&](int64_t row, auto bc) __attribute__((always_inline)) {
    constexpr int B = decltype(bc)::value, O = 1 - B;
    if (!in_lds) sf_fill_window<4>(ring, a, rx, n, ho, tid);  // first row of a chunk / image
    __syncthreads();
    const bool nxt1 = row + 1 < r1 && ho + 1 < a.Ho;
    const bool nxt2 = nxt1 && row + 2 < r1 && ho + 2 < a.Ho;
    if (nxt1 && !vv[B]) {
      load_rows(pf[B], kFS * ho + 4);
      vv[B] = true;
    }
    vv[O] = nxt2;
    if (nxt2) load_rows(pf[O], kFS * ho + 6);
    // ---- 7 filter rows x 3 chunks x 4 k-steps, 2 pixel tiles of 32
    sf_f32x16 acc0 = {}, acc1 = {};
#pragma unroll
    for (int kh = 0; kh < kFK; ++kh) {
      const float* src = &ring[((kFS * ho - kFP + kh) & (kFSlots - 1)) * kFRowF + abase];
#pragma unroll
      for (int q = 0; q < kFKq; ++q) {
        const float2 a0l = *reinterpret_cast<const float2*>(src + 8 * q);
        const float2 a0h = *reinterpret_cast<const float2*>(src + 8 * q + 2);
        const float2 a1l = *reinterpret_cast<const float2*>(src + 6 * 32 + 8 * q);
        const float2 a1h = *reinterpret_cast<const float2*>(src + 6 * 32 + 8 * q + 2);
        const float4 f = wf[kh][q];
        acc0 = sf_mfma(a0l.x, f.x, acc0);
        acc1 = sf_mfma(a1l.x, f.x, acc1);
        acc0 = sf_mfma(a0l.y, f.y, acc0);
        acc1 = sf_mfma(a1l.y, f.y, acc1);
        acc0 = sf_mfma(a0h.x, f.z, acc0);
        acc1 = sf_mfma(a1h.x, f.z, acc1);
        acc0 = sf_mfma(a0h.y, f.w, acc0);
        acc1 = sf_mfma(a1h.y, f.w, acc1);
      }
    }
    // ---- row + 1's 2 new input rows into their ring slots (outside this row's window)
    if (vv[B]) {
#pragma unroll
      for (int k = 0; k < kFPf; ++k) {
        const int i = tid + k * kFThreads;
        if (i < 2 * kFRowF) {
          const int r = i / kFRowF;
          ring[((kFS * ho + 4 + r) & (kFSlots - 1)) * kFRowF + i - r * kFRowF] = pf[B][k];
        }
      }
    }
    in_lds = vv[B];
    vv[B] = false;
    // ---- epilogue: statistics of the valid pixels, stores (pixels >= Wo dropped by the bound)
    auto stats = [&](const sf_f32x16& acc, int tbase) {
      if (tbase + 32 <= a.Wo) {  // full tile (wave-uniform): no masking
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          s1 += acc[r];
          s2 = fmaf(acc[r], acc[r], s2);
        }
      } else if (tbase < a.Wo) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float keep = tbase + (r & 3) + 8 * (r >> 2) + 4 * lh < a.Wo ? 1.f : 0.f;
          const float v = acc[r] * keep;
          s1 += v;
          s2 = fmaf(v, v, s2);
        }
      }
    };
    stats(acc0, px0);
    stats(acc1, px0 + 32);
    const auto ry = sf_rsrc(a.y + row * a.Wo * kFCo, int64_t(a.Wo) * kFCo * 4);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int so = ((r & 3) + 8 * (r >> 2)) * kFCo * 4;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc0[r]), ry, vy, so, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc1[r]), ry, vy, so + 32 * kFCo * 4, 0);
    }
    __syncthreads();  // every wave is done reading this row's window
    if (++ho == a.Ho) {
      ho = 0;
      ++n;
    }
  };
  for (int64_t row = r0; row < r1; row += 2) {
    step(row, std::integral_constant<int, 0>{});
    if (row + 1 < r1) step(row + 1, std::integral_constant<int, 1>{});
  }

  // ---- one partial row per workgroup: waves t and t + 2 hold channel tile t
  s1 += __shfl_xor(s1, 32);
  s2 += __shfl_xor(s2, 32);
  if (lh == 0) {
    red[wave][0][lc] = s1;
    red[wave][1][lc] = s2;
  }
  __syncthreads();
  if (tid < kFCo) {
    const int c = tid, t = c >> 5, l = c & 31;
    a.part[int64_t(blockIdx.x) * kFCo + c] = red[t][0][l] + red[t + 2][0][l];
    a.part[int64_t(gridDim.x) * kFCo + int64_t(blockIdx.x) * kFCo + c] = red[t][1][l] + red[t + 2][1][l];
  }
}

// ---------------------------------------------------------------- weight gradient
// dW[co][c][kh][kw] = sum over output pixels p of dY[p][co] * X[2 ho - 3 + kh][2 wo - 3 + kw][c]:
// a GEMM whose reduction runs over the 3.2 M output pixels (bs 256) into a 64 x 147 result.
// MIOpen's igemm_wrw for it: 948 us per fp32 ResNet-50 bs256 step (~64 TF) plus a zero-fill
// (profiles/r5/rocprof_resnet50_fp32_tile_gemm_off.md).  Here D^T[k][co] with k = kh * 21 +
// kw * 3 + c on the MFMA rows (147 -> 5 tiles of 32) and the 64 channels on the columns
// (2 tiles), so the padding is 9 % (the pixel-major formulation would pad 147 -> 7 x 32):
//  * per output row (same persistent row chunks and 16-slot input ring as the forward, rows of
//    232 pixels: Wo <= 112), the dY row is staged as-is ([px][64] fp32) and the 7 input rows
//    as flat [px][3] rows; a k-step reduces 2 pixels (the lane halves);
//  * the A operand of lane (k, half h) at pixel pair p is ring[slot(kh)][k % 21 + 6 (p + h)]: one
//    ds_read_b32 at a per-lane base plus a compile-time offset; B is dY[p + h][co], one
//    ds_read_b32 (lanes read 32 consecutive channels);
//  * waves = 2 channel tiles x 2 pixel halves (alternate pixel pairs), all 5 k tiles each (80
//    accumulators): every SIMD does the same work (a 3 + 2 split of the k tiles ran 707 us);
//    one fp32 partial [147][64] per wave pair, summed by the slice / final kernels below.
constexpr int kWMaxWo = 112;
constexpr int kWRowPx = 2 * kWMaxWo + 8;                        // 232
constexpr int kWRowF = kWRowPx * kFC;                           // 696 floats
constexpr int kWK = kFK * kFK * kFC;                            // 147
constexpr int kWPf = (2 * kWRowF + kFThreads - 1) / kFThreads;  // 6 ring floats per thread
constexpr int kWDy4 = kWMaxWo * kFCo / 4 / kFThreads;           // 7 dY float4 per thread

struct StemF32WArgs {
  const float* x;
  int64_t sN, sC, sH, sW;
  int cin;
  const float* dy;  // [N][Ho][Wo][64] fp32 (channels_last)
  float* part;      // [gridDim.x][147][64]
  int N, H, W, Ho, Wo;
};

// wave (ct, ph): channel tile ct, all 5 k tiles, the pixel pairs p = 4 j + 2 ph of every row
constexpr int NT = 5;
__device__ __forceinline__ void sf_wgrad_rows(const StemF32WArgs& a, float* ring, float* dyl) {
  constexpr int t0 = 0;
  const int ph = threadIdx.x >> 7;
  const int tid = threadIdx.x;
  const int lane = tid & 63, lc = lane & 31, lh = lane >> 5;
  const int ct = (tid >> 6) & 1;
  const auto rx = sf_rsrc(a.x, (int64_t(a.N - 1) * a.sN + int64_t(a.cin - 1) * a.sC + int64_t(a.H - 1) * a.sH +
                                int64_t(a.W - 1) * a.sW + 1) * 4);
  const int64_t rows = int64_t(a.N) * a.Ho;
  const int64_t per = (rows + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = int64_t(blockIdx.x) * per;
  const int64_t r1 = r0 + per < rows ? r0 + per : rows;
  const int ndy4 = a.Wo * kFCo / 4;  // float4 of one dY row
  // k rows of this lane in tile t0 + i (clamped: rows past 146 are computed, never stored)
  int kh_[NT], kr_[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    const int kk = min(32 * (t0 + i) + lc, kWK - 1);
    kh_[i] = kk / (kFK * kFC);
    kr_[i] = kk - kh_[i] * (kFK * kFC) + 6 * lh;
  }
  const int boff = lh * kFCo + 32 * ct + lc;

  sf_f32x16 acc[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) acc[i] = sf_f32x16{};

  int64_t n = r0 / a.Ho;
  int ho = int(r0 - n * a.Ho);
  float pf[2][kWPf];
  sf_f32x4 pd[2][kWDy4];
  bool vv[2] = {false, false};
  bool in_lds = false;
  auto load_rows = [&](float (&dst)[kWPf], sf_f32x4 (&dd)[kWDy4], int hbase, int64_t drow)
      __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < kWPf; ++k) {
      const int i = min(tid + k * kFThreads, 2 * kWRowF - 1);
      const int r = i / kWRowF;
      dst[k] = sf_load(rx, sf_off(a, n, hbase + r, i - r * kWRowF));
    }
    const sf_f32x4* src = reinterpret_cast<const sf_f32x4*>(a.dy + drow * a.Wo * kFCo);
#pragma unroll
    for (int k = 0; k < kWDy4; ++k) dd[k] = src[min(tid + k * kFThreads, ndy4 - 1)];
  };
  auto step = [&](int64_t row, auto bc) __attribute__((always_inline)) {
    constexpr int B = decltype(bc)::value, O = 1 - B;
    if (!in_lds) {  // first row of a chunk / image: the 7 ring rows and the dY row
      sf_fill_window<4, kWRowF>(ring, a, rx, n, ho, tid);
      const float4* src = reinterpret_cast<const float4*>(a.dy + row * a.Wo * kFCo);
      for (int i = tid; i < ndy4; i += kFThreads) reinterpret_cast<float4*>(dyl)[i] = src[i];
    }
    __syncthreads();
    const bool nxt1 = row + 1 < r1 && ho + 1 < a.Ho;
    const bool nxt2 = nxt1 && row + 2 < r1 && ho + 2 < a.Ho;
    if (nxt1 && !vv[B]) {
      load_rows(pf[B], pd[B], kFS * ho + 4, row + 1);
      vv[B] = true;
    }
    vv[O] = nxt2;
    if (nxt2) load_rows(pf[O], pd[O], kFS * ho + 6, row + 2);
    int ao[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) ao[i] = ((kFS * ho - kFP + kh_[i]) & (kFSlots - 1)) * kWRowF + kr_[i];
    // ---- k-steps over pixel pairs (p, p + 1); dY rows past Wo are zero
    for (int p = 2 * ph; p < a.Wo; p += 16) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int pp = p + 4 * u;
        const float b = dyl[boff + pp * kFCo];
#pragma unroll
        for (int i = 0; i < NT; ++i) acc[i] = sf_mfma(ring[ao[i] + 6 * pp], b, acc[i]);
      }
    }
    __syncthreads();  // every wave is done with this row's window and dY row
    if (vv[B]) {
#pragma unroll
      for (int k = 0; k < kWPf; ++k) {
        const int i = tid + k * kFThreads;
        if (i < 2 * kWRowF) {
          const int r = i / kWRowF;
          ring[((kFS * ho + 4 + r) & (kFSlots - 1)) * kWRowF + i - r * kWRowF] = pf[B][k];
        }
      }
#pragma unroll
      for (int k = 0; k < kWDy4; ++k) {
        const int i = tid + k * kFThreads;
        if (i < ndy4) reinterpret_cast<sf_f32x4*>(dyl)[i] = pd[B][k];
      }
    }
    in_lds = vv[B];
    vv[B] = false;
    if (++ho == a.Ho) {
      ho = 0;
      ++n;
    }
  };
  for (int64_t row = r0; row < r1; row += 2) {
    step(row, std::integral_constant<int, 0>{});
    if (row + 1 < r1) step(row + 1, std::integral_constant<int, 1>{});
  }
  // ---- partial [147][64] of pixel half ph: lane holds column co = 32 ct + lc of rows
  // k = 32 i + crow
  float* out = a.part + (2 * int64_t(blockIdx.x) + ph) * kWK * kFCo + 32 * ct + lc;
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = 32 * (t0 + i) + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (k < kWK) out[k * kFCo] = acc[i][r];
    }
}

__global__ __launch_bounds__(kFThreads, 2) void stem_f32_wgrad_kernel(StemF32WArgs a) {
  __shared__ __attribute__((aligned(16))) float ring[kFSlots * kWRowF];  // 44.5 KB
  __shared__ __attribute__((aligned(16))) float dyl[kWMaxWo * kFCo];  // 28.7 KB
  // pixel rows Wo .. 111 of the dY tile stay zero (the last 16-pixel block of a row reads past Wo;
  // with p = 2 ph + 16 j < Wo <= 112, no pair starts past pixel 110)
  for (int i = threadIdx.x; i < (kWMaxWo - a.Wo) * kFCo; i += kFThreads) dyl[a.Wo * kFCo + i] = 0.f;
  sf_wgrad_rows(a, ring, dyl);
}

// partials [nb][147][64] -> [nsl][147][64] (each slice sums <= ceil(nb / nsl) rows)
__global__ __launch_bounds__(256) void stem_f32_wgrad_slice_kernel(const float4* __restrict__ part, int nb,
                                                                   float4* __restrict__ tmp) {
  constexpr int e4n = kWK * kFCo / 4;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= e4n) return;
  const int sl = blockIdx.y, nsl = gridDim.y;
  const int per = (nb + nsl - 1) / nsl;
  const int b0 = sl * per, b1 = min(nb, b0 + per);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int b = b0; b < b1; ++b) {
    const float4 v = part[int64_t(b) * e4n + e];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  tmp[int64_t(sl) * e4n + e] = s;
}

// [nsl][147][64] -> dW[co][c][kh][kw] (element strides) (+)=, one thread per (k, co)
__global__ __launch_bounds__(256) void stem_f32_wgrad_final_kernel(const float* __restrict__ tmp, int nsl, int cin,
                                                                   float* __restrict__ dw, int64_t s0, int64_t s1,
                                                                   int64_t s2, int64_t s3, int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // k * 64 + co
  if (i >= kWK * kFCo) return;
  const int k = i / kFCo, co = i - k * kFCo;
  const int kh = k / (kFK * kFC), r = k - kh * (kFK * kFC);
  const int kw = r / kFC, c = r - kw * kFC;
  if (c >= cin) return;
  float v = 0.f;
  for (int sl = 0; sl < nsl; ++sl) v += tmp[int64_t(sl) * kWK * kFCo + i];
  float* o = dw + co * s0 + c * s1 + kh * s2 + kw * s3;
  *o = v + (accumulate ? *o : 0.f);
}

}  // namespace

constexpr int kWMaxSlicesF32 = 64;

int64_t stem_wgrad_f32_workspace_floats(int N, int Ho) {
  return int64_t(2 * stem_partial_rows(N, Ho) + kWMaxSlicesF32) * kWK * kFCo;
}

bool stem_wgrad_f32_supported(int Wo) { return Wo >= 1 && Wo <= kWMaxWo; }

void stem_conv_wgrad_f32(uintptr_t x, int64_t sN, int64_t sC, int64_t sH, int64_t sW, int Cin, uintptr_t dy,
                         uintptr_t dw, int64_t s0, int64_t s1, int64_t s2, int64_t s3, uintptr_t ws, int N, int H,
                         int W, int Ho, int Wo, bool accumulate, uintptr_t stream) {
  VODA_CHECK(Cin >= 1 && Cin <= kFC, "stem_wgrad_f32: 1..3 input channels");
  VODA_CHECK(Ho == (H + 2 * kFP - kFK) / kFS + 1 && Wo == (W + 2 * kFP - kFK) / kFS + 1,
             "stem_wgrad_f32: output size mismatch (7x7, stride 2, pad 3)");
  VODA_CHECK(stem_wgrad_f32_supported(Wo), "stem_wgrad_f32: output width must be <= 112");
  VODA_CHECK(x % 4 == 0 && dy % 16 == 0 && dw % 4 == 0 && ws % 16 == 0, "stem_wgrad_f32: misaligned operands");
  VODA_CHECK(sN >= 0 && sC >= 0 && sH >= 0 && sW >= 0 &&
                 (int64_t(N - 1) * sN + int64_t(Cin - 1) * sC + int64_t(H - 1) * sH + int64_t(W - 1) * sW + 1) * 4 <
                     (int64_t(1) << 31),
             "stem_wgrad_f32: image must span < 2 GB (32-bit buffer offsets)");
  hipStream_t s = as_stream(stream);
  const int nb = stem_partial_rows(N, Ho);
  float* part = reinterpret_cast<float*>(ws);
  float* tmp = part + int64_t(2 * nb) * kWK * kFCo;  // partials: [nb][2 pixel halves][147][64]
  const int nsl = std::min(kWMaxSlicesF32, 2 * nb);
  StemF32WArgs a{reinterpret_cast<const float*>(x), sN, sC, sH, sW, Cin, reinterpret_cast<const float*>(dy), part,
                 N, H, W, Ho, Wo};
  hipLaunchKernelGGL(stem_f32_wgrad_kernel, dim3(nb), dim3(kFThreads), 0, s, a);
  hipLaunchKernelGGL(stem_f32_wgrad_slice_kernel, dim3((kWK * kFCo / 4 + 255) / 256, nsl), dim3(256), 0, s,
                     reinterpret_cast<const float4*>(part), 2 * nb, reinterpret_cast<float4*>(tmp));
  hipLaunchKernelGGL(stem_f32_wgrad_final_kernel, dim3((kWK * kFCo + 255) / 256), dim3(256), 0, s, tmp, nsl, Cin,
                     reinterpret_cast<float*>(dw), s0, s1, s2, s3, int(accumulate));
  check_launch();
}

void stem_conv_fwd_f32(uintptr_t x, int64_t sN, int64_t sC, int64_t sH, int64_t sW, int Cin, uintptr_t w,
                       int64_t sw0, int64_t sw1, int64_t sw2, int64_t sw3, uintptr_t y, uintptr_t part, int nb, int N,
                       int H, int W, int Ho, int Wo, uintptr_t stream) {
  VODA_CHECK(Cin >= 1 && Cin <= kFC, "stem_conv_f32: 1..3 input channels");
  VODA_CHECK(Ho == (H + 2 * kFP - kFK) / kFS + 1 && Wo == (W + 2 * kFP - kFK) / kFS + 1,
             "stem_conv_f32: output size mismatch (7x7, stride 2, pad 3)");
  VODA_CHECK(Wo >= 1 && Wo <= kFMaxWo, "stem_conv_f32: output width must be <= 128");
  VODA_CHECK(nb == stem_partial_rows(N, Ho), "stem_conv_f32: partial-row count mismatch");
  VODA_CHECK(x % 4 == 0 && w % 4 == 0 && y % 16 == 0 && part % 4 == 0, "stem_conv_f32: misaligned operands");
  VODA_CHECK(sN >= 0 && sC >= 0 && sH >= 0 && sW >= 0 &&
                 (int64_t(N - 1) * sN + int64_t(Cin - 1) * sC + int64_t(H - 1) * sH + int64_t(W - 1) * sW + 1) * 4 <
                     (int64_t(1) << 31),
             "stem_conv_f32: image must span < 2 GB (32-bit buffer offsets)");
  VODA_CHECK(int64_t(Wo) * kFCo * 4 < (int64_t(1) << 31), "stem_conv_f32: output row too large");
  StemF32Args a{reinterpret_cast<const float*>(x), sN, sC, sH, sW, Cin, reinterpret_cast<const float*>(w), sw0, sw1,
                sw2, sw3, reinterpret_cast<float*>(y), reinterpret_cast<float*>(part), N, H, W, Ho, Wo};
  hipLaunchKernelGGL(stem_f32_fwd_kernel, dim3(nb), dim3(kFThreads), 0, as_stream(stream), a);
  check_launch();
}

}  // namespace voda
