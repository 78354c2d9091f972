// ResNet stem: 7x7 / stride-2 / pad-3 convolution of a 3-channel image into 64 channels,
// with the batch-norm statistics of its output computed in the epilogue.
//
// What it replaces (profiles/r3/rocprof_resnet50_bf16_stem.md, ResNet-50 bs256 bf16):
// an fp32 -> bf16 cast of the image (58 us), MIOpen's output zero-fill (90 us), MIOpen's
// igemm_fwd (371 us, ~165 TFLOP/s) and the separate BN statistics pass that re-reads the
// 411 MB output (111 us).
//
// Design (one implicit GEMM, MFMA v_mfma_f32_32x32x16_bf16):
//  * the image is first packed to NHWC with 4 channels (the 4th is zero): one pixel = 8 B,
//    so the 8 input pixels under one filter row (kw = 0..6 plus a zero-weight 8th) are one
//    64-byte span, i.e. K = 7 rows x 8 px x 4 ch = 224 = 14 MFMA k-steps;
//  * a workgroup (4 waves) produces one output row (Wo <= 128 pixels, 32 per wave) of all
//    64 channels from the 7 input rows under it, held in a 16-row LDS ring (264 px x 8 B per
//    row, zero outside the image); the pixel-side MFMA operand is one ds_read_b128 per k-step;
//  * the grid is persistent (two workgroups per CU) and each workgroup walks a contiguous
//    chunk of output rows: consecutive rows share 5 of their 7 input rows, so the steady
//    state loads only the 2 new rows, into registers, while the current row's MFMAs run
//    (a first version that re-staged all 7 rows synchronously per output row ran 291 us);
//  * the filter-side operand (2 channel tiles x 14 k-steps x 8 bf16 = 112 VGPRs per lane)
//    is gathered once per workgroup and stays in registers;
//  * D rows = pixels, columns = channels: a lane holds one channel of 16 pixels, so the
//    per-channel sum and sum of squares are in-lane adds over the tile, carried in 4
//    registers across the whole chunk; one partial row per workgroup goes to the BN
//    finalize kernel (batchnorm.hip), which is unchanged;
//  * the output tile is transposed through LDS (row stride 144 B) and written as 16-byte
//    stores of whole 128-byte pixel rows (channels_last).
#include "common.h"

#include <cstdlib>
#include <type_traits>
#include "ops.h"

namespace voda {

namespace {

typedef __bf16 st_bf16x8 __attribute__((ext_vector_type(8)));
typedef float st_f32x16 __attribute__((ext_vector_type(16)));

constexpr int kSK = 7, kSS = 2, kSP = 3;  // filter, stride, padding
constexpr int kSCo = 64;                  // output channels (two 32-wide MFMA tiles)
constexpr int kSWaves = 4;
constexpr int kSThreads = 64 * kSWaves;
constexpr int kSTile = 32;                      // output pixels per wave
constexpr int kSMaxWo = kSWaves * kSTile;       // 128
constexpr int kSRowPx = 2 * kSMaxWo + 8;        // 264 LDS pixels per input row
constexpr int kSRowB = kSRowPx * 8;             // 2112 B
constexpr int kSOutStride = 144;                // B per staged output pixel (128 + 16 pad)
constexpr int kSKSteps = kSK * 2;               // 14
constexpr int kSSlots = 16;                     // LDS ring of input rows (>= 7 in use + 2 refilled)
constexpr int kSPf = (2 * kSRowPx + kSThreads - 1) / kSThreads;  // prefetch slots per thread (3)

struct StemArgs {
  const uint2* x4;       // [N][H][W] pixels of 4 bf16
  const uint16_t* w;     // bf16 filter, element strides below
  int64_t sw0, sw1, sw2, sw3;  // co, ci, kh, kw
  int cin;
  uint16_t* y;           // [N][Ho][Wo][64] bf16
  float* part;           // [2][gridDim.x][64]
  int N, H, W, Ho, Wo;
};

__device__ __forceinline__ st_f32x16 st_mfma(st_bf16x8 a, st_bf16x8 b, st_f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// one 8-byte input pixel of the packed image, zero outside it; branch-free (clamped load +
// select) so that a row's loads issue back to back without exec-mask branches and waits
__device__ __forceinline__ uint2 st_pixel(const uint2* x4, int H, int W, int64_t n, int hi, int wi) {
  const bool ok = unsigned(hi) < unsigned(H) && unsigned(wi) < unsigned(W);
  const int hc = min(max(hi, 0), H - 1), wc = min(max(wi, 0), W - 1);
  const uint2 v = x4[(n * H + hc) * W + wc];
  const uint32_t m = ok ? 0xffffffffu : 0u;
  return make_uint2(v.x & m, v.y & m);
}

// the 7 input rows of output row ho into the ring, loads issued in batches of B before their
// LDS writes (a load-then-write loop waited out one global latency per element: 8 per thread)
template <int B>
__device__ __forceinline__ void st_fill_window(unsigned char* ring, const uint2* x4, int H, int W, int64_t n, int ho,
                                               int tid) {
  constexpr int kTotal = kSK * kSRowPx;                    // 1848
  constexpr int kIters = (kTotal + kSThreads - 1) / kSThreads;  // 8
#pragma unroll
  for (int b = 0; b < kIters; b += B) {
    uint2 v[B];
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const int i = min(tid + (b + u) * kSThreads, kTotal - 1);
      const int r = i / kSRowPx, j = i - r * kSRowPx;
      v[u] = st_pixel(x4, H, W, n, kSS * ho - kSP + r, j - kSP);
    }
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const int i = tid + (b + u) * kSThreads;
      if (i < kTotal) {
        const int r = i / kSRowPx, j = i - r * kSRowPx;
        *reinterpret_cast<uint2*>(ring + ((kSS * ho - kSP + r) & (kSSlots - 1)) * kSRowB + j * 8) = v[u];
      }
    }
  }
}

__global__ __launch_bounds__(kSThreads, 2) void stem_conv7x7_fwd_kernel(StemArgs a) {
  // input rows live in a ring of kSSlots LDS rows, slot = hi & (kSSlots - 1): consecutive
  // output rows share 5 of their 7 input rows, so the steady state loads 2 new rows per
  // output row -- prefetched into registers while the MFMAs of earlier rows run
  __shared__ __attribute__((aligned(16))) unsigned char lds_in[kSSlots * kSRowB];
  __shared__ __attribute__((aligned(16))) unsigned char lds_out[kSMaxWo * kSOutStride];
  __shared__ float red[kSWaves][2][32];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int lc = lane & 31, lh = lane >> 5;
  // wave = (channel tile ct) x (64-pixel half ph): 14 filter fragments per lane (56 VGPRs)
  // instead of 28 -- the 2-tile variant sat at the 256-register limit with spills
  const int ct = wave & 1, ph = wave >> 1;

  // filter fragments: B[k][co] for co = 32 ct + lc, k-chunk = 8 lh .. 8 lh + 7 of k-step ks
  // (kh = ks / 2, pixels kw = 4 (ks & 1) + 2 lh + q, q = 0, 1, channels 0..3).  The workgroup
  // first packs the filter as [64][224] bf16 (zeros at kw = 7 and past Cin) into the ring's
  // LDS (coalesced 2-byte loads, 14 in flight per thread), then every lane reads its
  // fragments as 16-byte LDS reads.  (Per-lane gathers -- 224 dependent 2-byte global loads per
  // lane -- were a large part of a ~50 us fixed cost per launch.)
  {
    uint16_t* wp = reinterpret_cast<uint16_t*>(lds_in);
    constexpr int kWElems = kSCo * kSKSteps * 16;  // 14336
    constexpr int kPer = kWElems / kSThreads;       // 56
#pragma unroll
    for (int b = 0; b < kPer; b += 14) {
      uint16_t v[14];
#pragma unroll
      for (int i = 0; i < 14; ++i) {
        const int e = tid + (b + i) * kSThreads;
        const int co = e / (kSKSteps * 16), k = e - co * (kSKSteps * 16);
        const int kh = k >> 5, kw = (k >> 2) & 7, c = k & 3;
        v[i] = (kw < kSK && c < a.cin) ? a.w[co * a.sw0 + c * a.sw1 + kh * a.sw2 + kw * a.sw3] : uint16_t(0);
      }
#pragma unroll
      for (int i = 0; i < 14; ++i) wp[tid + (b + i) * kSThreads] = v[i];
    }
  }
  __syncthreads();
  st_bf16x8 wf[kSKSteps];
#pragma unroll
  for (int ks = 0; ks < kSKSteps; ++ks) {
    uint4 pk = *reinterpret_cast<const uint4*>(lds_in + ((32 * ct + lc) * kSKSteps * 16 + ks * 16 + 8 * lh) * 2);
    // opaque to the optimizer: keeps the fragment resident instead of re-deriving it inside
    // the row loop (register-pressure rematerialisation)
    asm volatile("" : "+v"(pk.x), "+v"(pk.y), "+v"(pk.z), "+v"(pk.w));
    wf[ks] = __builtin_bit_cast(st_bf16x8, pk);
  }
  __syncthreads();  // the ring's LDS is reused below

  // this thread's share of a 2-row refill: slots tid, tid + 256, tid + 512 of 2 x kSRowPx
  int pr[kSPf], pj[kSPf];
#pragma unroll
  for (int k = 0; k < kSPf; ++k) {
    const int i = tid + k * kSThreads;
    pr[k] = i < 2 * kSRowPx ? i / kSRowPx : -1;
    pj[k] = i < 2 * kSRowPx ? i - (i / kSRowPx) * kSRowPx : 0;
  }

  float s1 = 0.f, s2 = 0.f;  // channel 32 ct + lc, pixel rows of half lh
  const int64_t rows = int64_t(a.N) * a.Ho;
  const int64_t per = (rows + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = int64_t(blockIdx.x) * per;
  const int64_t r1 = r0 + per < rows ? r0 + per : rows;
  const int px0 = 64 * ph;             // this wave's first output pixel
  const int wo0 = px0 + lc;            // MFMA A rows of pixel tile 0 (tile 1: + 32)

  int64_t n = r0 / a.Ho;
  int ho = int(r0 - n * a.Ho);
  // two rows of prefetch in flight: the 2 new input rows of row + 1 (written into the ring
  // after this row's MFMAs) and of row + 2 (issued now) -- a global load's latency
  // (~1-2 us) is longer than one row's MFMA work (~0.4 us)
  // Two register buffers alternate roles row by row (the loop body is instantiated twice);
  // a buffer copy-rotation at the end of each row made every row wait for the loads it had just
  // issued (vmcnt is in order), i.e. a one-row prefetch distance again.
  uint2 pf[2][kSPf];
  bool vv[2] = {false, false};  // buffer b holds the next row's 2 new input rows
  bool in_lds = false;          // this row's window is complete in the ring
  auto load_rows = [&](uint2 (&dst)[kSPf], int hbase) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < kSPf; ++k) dst[k] = st_pixel(a.x4, a.H, a.W, n, hbase + max(pr[k], 0), pj[k] - kSP);
  };
  // buffer [B]: row + 1's new rows (valid if vv[B]); [1 - B]: receives row + 2's new rows
  auto step = [&](int64_t row, auto bc) __attribute__((always_inline)) {
    constexpr int B = decltype(bc)::value, O = 1 - B;
    // ---- this row's input window: hi = 2 ho - 3 .. 2 ho + 3
    if (!in_lds) st_fill_window<4>(lds_in, a.x4, a.H, a.W, n, ho, tid);  // first row of a chunk / image
    __syncthreads();
    // ---- prefetch (same image only): rows 2 ho + 4, 2 ho + 5 for row + 1 unless already in
    // flight, rows 2 ho + 6, 2 ho + 7 for row + 2
    const bool nxt1 = row + 1 < r1 && ho + 1 < a.Ho;
    const bool nxt2 = nxt1 && row + 2 < r1 && ho + 2 < a.Ho;
    if (nxt1 && !vv[B]) {
      load_rows(pf[B], kSS * ho + 4);
      vv[B] = true;
    }
    vv[O] = nxt2;
    if (nxt2) load_rows(pf[O], kSS * ho + 6);
    // ---- 14 k-steps (kh-outer, 2 per kh), 2 pixel tiles of 32
    st_f32x16 acc0 = {}, acc1 = {};
#pragma unroll
    for (int kh = 0; kh < kSK; ++kh) {
      const int slot = (kSS * ho - kSP + kh) & (kSSlots - 1);
      const int off = slot * kSRowB + (2 * wo0 + 2 * lh) * 8;
      const st_bf16x8 p00 = *reinterpret_cast<const st_bf16x8*>(lds_in + off);
      const st_bf16x8 p10 = *reinterpret_cast<const st_bf16x8*>(lds_in + off + 2 * 32 * 8);
      const st_bf16x8 p01 = *reinterpret_cast<const st_bf16x8*>(lds_in + off + 4 * 8);
      const st_bf16x8 p11 = *reinterpret_cast<const st_bf16x8*>(lds_in + off + 2 * 32 * 8 + 4 * 8);
      acc0 = st_mfma(p00, wf[2 * kh], acc0);
      acc1 = st_mfma(p10, wf[2 * kh], acc1);
      acc0 = st_mfma(p01, wf[2 * kh + 1], acc0);
      acc1 = st_mfma(p11, wf[2 * kh + 1], acc1);
    }
    // ---- row + 1's 2 new input rows into their ring slots (outside this row's window),
    // before this row's output stores are issued
    if (vv[B]) {
#pragma unroll
      for (int k = 0; k < kSPf; ++k)
        if (pr[k] >= 0) {
          const int hi = kSS * ho + 4 + pr[k];
          *reinterpret_cast<uint2*>(lds_in + (hi & (kSSlots - 1)) * kSRowB + pj[k] * 8) = pf[B][k];
        }
    }
    in_lds = vv[B];
    vv[B] = false;
    // ---- epilogue: statistics of the valid pixels, bf16 tile into the staging rows
    {
      auto stats = [&](const st_f32x16& acc, int tbase) {
        if (tbase + 32 <= a.Wo) {  // full tile (wave-uniform): no masking
#pragma unroll
          for (int r = 0; r < 16; ++r) { s1 += acc[r]; s2 = fmaf(acc[r], acc[r], s2); }
        } else if (tbase < a.Wo) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float keep = tbase + (r & 3) + 8 * (r >> 2) + 4 * lh < a.Wo ? 1.f : 0.f;
            const float v = acc[r] * keep;
            s1 += v; s2 = fmaf(v, v, s2);
          }
        }
      };
      stats(acc0, px0);
      stats(acc1, px0 + 32);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int px = px0 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        *reinterpret_cast<uint16_t*>(lds_out + px * kSOutStride + (32 * ct + lc) * 2) = f2bf(acc0[r]);
        *reinterpret_cast<uint16_t*>(lds_out + (px + 32) * kSOutStride + (32 * ct + lc) * 2) = f2bf(acc1[r]);
      }
    }
    __syncthreads();  // staging complete; every wave is done reading this row's window
    // ---- whole 128-byte pixel rows out: wave w stores pixels 32 w .. 32 w + 31
    uint16_t* ybase = a.y + (row * a.Wo + wave * kSTile) * kSCo;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = i * 64 + lane;
      const int px = q >> 3, part = q & 7;
      if (wave * kSTile + px < a.Wo) {
        const uint4 v = *reinterpret_cast<const uint4*>(lds_out + (wave * kSTile + px) * kSOutStride + part * 16);
        *reinterpret_cast<uint4*>(ybase + px * kSCo + part * 8) = v;
      }
    }
    if (++ho == a.Ho) { ho = 0; ++n; }
  };
  for (int64_t row = r0; row < r1; row += 2) {
    step(row, std::integral_constant<int, 0>{});
    if (row + 1 < r1) step(row + 1, std::integral_constant<int, 1>{});
  }

  // ---- one partial row per workgroup: lane lc (+ half lh) of wave (ct, ph) holds channel
  // 32 ct + lc
  s1 += __shfl_xor(s1, 32);
  s2 += __shfl_xor(s2, 32);
  if (lh == 0) {
    red[wave][0][lc] = s1;
    red[wave][1][lc] = s2;
  }
  __syncthreads();
  if (tid < kSCo) {
    const int c = tid, t = c >> 5, l = c & 31;  // waves t and t + 2 hold channel tile t
    const float a1 = red[t][0][l] + red[t + 2][0][l], a2 = red[t][1][l] + red[t + 2][1][l];
    a.part[int64_t(blockIdx.x) * kSCo + c] = a1;
    a.part[int64_t(gridDim.x) * kSCo + int64_t(blockIdx.x) * kSCo + c] = a2;
  }
}

// ---------------------------------------------------------------- weight gradient
// dW[co][kh][kw][c] = sum over output pixels p of dY[p][co] * X4[2 ho - 3 + kh][2 wo - 3 + kw][c]:
// a GEMM whose reduction runs over the 3.2 M output pixels (bs 256) into a 64 x 224 result.
// MIOpen's igemm_wrw for it: 237 us on the NHWC-4 image + workspace clear / cast / fold
// kernels.  Here, per output row (same persistent row chunks and 16-row input ring as the
// forward):
//  * the dY row (Wo x 64 bf16) is staged as [128 px][192 B] rows -- 192 B makes the
//    transposed reads conflict-free (row q of the 4-row block lands 48 dwords further, so the
//    8 (row, 16-column block) pairs a half-wave reads fill the 64 banks once);
//  * both MFMA operands need 8 consecutive PIXELS per lane: ds_read_b64_tr_b16 (4 rows x 16
//    columns per 16-lane group, any 8-byte-aligned address per lane) reads them as columns --
//    for the image operand the "rows" are the im2col rows of consecutive output pixels, which
//    start 2 input pixels (16 B) apart in the ring: overlapping rows, no im2col buffer;
//  * D = 2 channel tiles x 7 filter rows of 32 x 32; wave w owns channel tile w & 1 and filter
//    rows 0-3 (w < 2) or 4-6, accumulated over the whole row chunk; one fp32 partial
//    [64][224] per workgroup, summed by stem_wgrad_reduce_kernel.
constexpr int kWRowB = 192;
constexpr int kWTileB = kSMaxWo * kWRowB;  // 24576 B
constexpr int kWK = kSK * 32;              // 224 packed filter columns
constexpr int kWDyPf = (kSMaxWo * 8 + kSThreads - 1) / kSThreads;  // 16-B dY chunks per thread (4)

struct StemWArgs {
  const uint2* x4;
  const uint16_t* dy;  // [N][Ho][Wo][64] bf16
  float* part;         // [gridDim.x][64][224]
  int N, H, W, Ho, Wo;
};

typedef __bf16 st_bf16x4_v __attribute__((__vector_size__(4 * sizeof(__bf16))));
typedef __attribute__((address_space(3))) st_bf16x4_v st_lds_bf16x4;

typedef uint32_t st_u32x4 __attribute__((ext_vector_type(4)));
// named native vectors: HIP's uint4 struct is copied with memcpy, which kept an array of them
// in scratch
struct St4 {
  st_u32x4 v0, v1, v2, v3;
};

__device__ __forceinline__ uint2 st_tr_read(const unsigned char* p) {
  const st_bf16x4_v v = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((st_lds_bf16x4*)(p));
  return __builtin_bit_cast(uint2, v);
}

__device__ __forceinline__ st_bf16x8 st_frag(const unsigned char* lo, const unsigned char* hi) {
  const uint2 a = st_tr_read(lo), b = st_tr_read(hi);
  return __builtin_bit_cast(st_bf16x8, make_uint4(a.x, a.y, b.x, b.y));
}

__global__ __launch_bounds__(kSThreads, 2) void stem_conv7x7_wgrad_kernel(StemWArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char ring[kSSlots * kSRowB];
  __shared__ __attribute__((aligned(16))) unsigned char dyt[kWTileB];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int lh = lane >> 5, lg = (lane >> 4) & 1, lq = (lane & 15) >> 2, lp = lane & 3;
  const int ct = wave & 1;             // channel tile
  const int kh0 = wave < 2 ? 0 : 4;    // filter rows kh0 .. kh0 + nkh - 1
  const int nkh = wave < 2 ? 4 : 3;

  // pixel rows Wo .. 127 of the dY tile stay zero: they add nothing
  for (int i = tid; i < (kSMaxWo - a.Wo) * (kWRowB / 16); i += kSThreads)
    *reinterpret_cast<uint4*>(dyt + a.Wo * kWRowB + i * 16) = make_uint4(0u, 0u, 0u, 0u);

  int pr[kSPf], pj[kSPf];
#pragma unroll
  for (int k = 0; k < kSPf; ++k) {
    const int i = tid + k * kSThreads;
    pr[k] = i < 2 * kSRowPx ? i / kSRowPx : -1;
    pj[k] = i < 2 * kSRowPx ? i - (i / kSRowPx) * kSRowPx : 0;
  }

  st_f32x16 acc0 = {}, acc1 = {}, acc2 = {}, acc3 = {};
  const int64_t rows = int64_t(a.N) * a.Ho;
  const int64_t per = (rows + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = int64_t(blockIdx.x) * per;
  const int64_t r1 = r0 + per < rows ? r0 + per : rows;
  const int nchunk = a.Wo * 8;  // 16-B chunks of one dY row

  // per-lane byte offsets of the transposed reads (k-step 0, first 4-row block)
  const int a_off = (8 * lh + lq) * kWRowB + (32 * ct + 16 * lg + 4 * lp) * 2;
  const int b_off = (2 * (8 * lh + lq) + 4 * lg + lp) * 8;

  int64_t n = r0 / a.Ho;
  int ho = int(r0 - n * a.Ho);
  uint2 pf[kSPf];
  // two rows of prefetch in flight (see the forward kernel): row + 1's ring rows and dY row in
  // the "a" registers (written after this row's MFMAs), row + 2's in the "b" registers.
  // Named uint4s: an indexed uint4[4] was promoted to LDS.
  static_assert(kWDyPf == 4, "dY prefetch slots");
  uint2 pfa[kSPf], pfb[kSPf];
  uint4 da0, da1, da2, da3, db0, db1, db2, db3;
  bool pa = false, in_lds = false;
  auto load_rows = [&](uint2 (&dst)[kSPf], int hbase) {
#pragma unroll
    for (int k = 0; k < kSPf; ++k) dst[k] = st_pixel(a.x4, a.H, a.W, n, hbase + max(pr[k], 0), pj[k] - kSP);
  };
  auto load_dy = [&](int64_t r, uint4& d0, uint4& d1, uint4& d2, uint4& d3) {
    const uint4* nd = reinterpret_cast<const uint4*>(a.dy + r * a.Wo * kSCo);
    d0 = nd[min(tid, nchunk - 1)];
    d1 = nd[min(tid + kSThreads, nchunk - 1)];
    d2 = nd[min(tid + 2 * kSThreads, nchunk - 1)];
    d3 = nd[min(tid + 3 * kSThreads, nchunk - 1)];
  };
  for (int64_t row = r0; row < r1; ++row) {
    if (!in_lds) {  // first row of the chunk or of an image: the 7 ring rows and the dY row
      for (int i = tid; i < kSK * kSRowPx; i += kSThreads) {
        const int r = i / kSRowPx, j = i - r * kSRowPx;
        const int hi = kSS * ho - kSP + r;
        *reinterpret_cast<uint2*>(ring + (hi & (kSSlots - 1)) * kSRowB + j * 8) = st_pixel(a.x4, a.H, a.W, n, hi, j - kSP);
      }
      for (int i = tid; i < nchunk; i += kSThreads)
        *reinterpret_cast<uint4*>(dyt + (i >> 3) * kWRowB + (i & 7) * 16) =
            reinterpret_cast<const uint4*>(a.dy + row * a.Wo * kSCo)[i];
    }
    __syncthreads();
    // ---- prefetch (same image only)
    const bool nxt1 = row + 1 < r1 && ho + 1 < a.Ho;
    const bool nxt2 = nxt1 && row + 2 < r1 && ho + 2 < a.Ho;
    if (nxt1 && !pa) {
      load_rows(pfa, kSS * ho + 4);
      load_dy(row + 1, da0, da1, da2, da3);
      pa = true;
    }
    if (nxt2) {
      load_rows(pfb, kSS * ho + 6);
      load_dy(row + 2, db0, db1, db2, db3);
    }
    // ---- 8 k-steps of 16 output pixels; 4 filter-row tiles per wave (waves 2, 3: rows 4-6
    // and a discarded 4th, which keeps the accumulators in named registers -- an indexed
    // accumulator array was promoted to LDS)
    const int so0 = ((kSS * ho - kSP + kh0) & (kSSlots - 1)) * kSRowB;
    const int so1 = ((kSS * ho - kSP + kh0 + 1) & (kSSlots - 1)) * kSRowB;
    const int so2 = ((kSS * ho - kSP + kh0 + 2) & (kSSlots - 1)) * kSRowB;
    const int so3 = ((kSS * ho - kSP + kh0 + 3) & (kSSlots - 1)) * kSRowB;
#pragma unroll 2
    for (int ks = 0; ks < kSMaxWo / 16; ++ks) {
      const unsigned char* ap = dyt + a_off + ks * 16 * kWRowB;
      const st_bf16x8 af = st_frag(ap, ap + 4 * kWRowB);
      const unsigned char* bp = ring + b_off + ks * 16 * 16;
      acc0 = st_mfma(af, st_frag(bp + so0, bp + so0 + 64), acc0);
      acc1 = st_mfma(af, st_frag(bp + so1, bp + so1 + 64), acc1);
      acc2 = st_mfma(af, st_frag(bp + so2, bp + so2 + 64), acc2);
      acc3 = st_mfma(af, st_frag(bp + so3, bp + so3 + 64), acc3);
    }
    __syncthreads();  // every wave is done with this row's dY tile and window
    if (pa) {
#pragma unroll
      for (int k = 0; k < kSPf; ++k)
        if (pr[k] >= 0) {
          const int hi = kSS * ho + 4 + pr[k];
          *reinterpret_cast<uint2*>(ring + (hi & (kSSlots - 1)) * kSRowB + pj[k] * 8) = pfa[k];
        }
      auto put_dy = [&](int i, const uint4& v) {
        if (i < nchunk) *reinterpret_cast<uint4*>(dyt + (i >> 3) * kWRowB + (i & 7) * 16) = v;
      };
      put_dy(tid, da0);
      put_dy(tid + kSThreads, da1);
      put_dy(tid + 2 * kSThreads, da2);
      put_dy(tid + 3 * kSThreads, da3);
    }
    in_lds = pa;
#pragma unroll
    for (int k = 0; k < kSPf; ++k) pfa[k] = pfb[k];
    da0 = db0; da1 = db1; da2 = db2; da3 = db3;
    pa = nxt2;
    if (++ho == a.Ho) { ho = 0; ++n; }
  }

  // ---- partial [64][224]: lane holds column k = kh * 32 + (lane & 31), rows co
  float* out = a.part + int64_t(blockIdx.x) * kSCo * kWK + (lane & 31);
  auto put = [&](const st_f32x16& acc, int kh) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = 32 * ct + (r & 3) + 8 * (r >> 2) + 4 * lh;
      out[co * kWK + kh * 32] = acc[r];
    }
  };
  put(acc0, kh0);
  put(acc1, kh0 + 1);
  put(acc2, kh0 + 2);
  if (nkh == 4) put(acc3, kh0 + 3);
}

// partials [nb][64][224] -> [nsl][64][224] (float4, each slice sums <= 8 partial rows)
__global__ __launch_bounds__(256) void stem_wgrad_slice_kernel(const float4* __restrict__ part, int nb,
                                                               float4* __restrict__ tmp) {
  constexpr int e4n = kSCo * kWK / 4;
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

// [nsl][64][224] -> dW[co][c][kh][kw] (element strides), fp32 or bf16, (+)=; one thread per
// (co, kh, kw): its 4 packed channels are one float4 of every slice
template <typename OutT>
__global__ __launch_bounds__(256) void stem_wgrad_final_kernel(const float4* __restrict__ tmp, int nsl, int cin,
                                                               OutT* __restrict__ dw, int64_t s0, int64_t s1,
                                                               int64_t s2, int64_t s3, int accumulate) {
  constexpr int e4n = kSCo * kWK / 4;
  const int i = blockIdx.x * 256 + threadIdx.x;  // (co, kh, kw)
  if (i >= kSCo * kSK * kSK) return;
  const int kw = i % kSK, kh = (i / kSK) % kSK, co = i / (kSK * kSK);
  const int e4 = (co * kWK + kh * 32 + kw * 4) / 4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
  int sl = 0;
  for (; sl + 1 < nsl; sl += 2) {
    const float4 u = tmp[int64_t(sl) * e4n + e4], v = tmp[int64_t(sl + 1) * e4n + e4];
    a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
    b.x += v.x; b.y += v.y; b.z += v.z; b.w += v.w;
  }
  if (sl < nsl) {
    const float4 u = tmp[int64_t(sl) * e4n + e4];
    a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
  }
  const float val[4] = {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (c >= cin) break;
    OutT* o = dw + co * s0 + c * s1 + kh * s2 + kw * s3;
    if constexpr (sizeof(OutT) == 4) {
      *reinterpret_cast<float*>(o) = val[c] + (accumulate ? *reinterpret_cast<float*>(o) : 0.f);
    } else {
      uint16_t* q = reinterpret_cast<uint16_t*>(o);
      *q = f2bf(val[c] + (accumulate ? bf2f(*q) : 0.f));
    }
  }
}

// image [N][C<=4][H][W] (any strides, fp32 / bf16 / fp16) -> NHWC4 bf16, channel 3.. zero;
// grid (N * H, W / 256): no 64-bit index division per pixel
template <typename T>
__global__ __launch_bounds__(256) void stem_pack_kernel(const T* __restrict__ x, uint2* __restrict__ x4, int C, int H,
                                                        int W, int64_t sN, int64_t sC, int64_t sH, int64_t sW) {
  const int w = blockIdx.y * 256 + threadIdx.x;
  if (w >= W) return;
  const int nh = blockIdx.x;
  const int n = nh / H, h = nh - (nh / H) * H;
  const T* p = x + n * sN + h * sH + w * sW;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (c < C) v[c] = Vec4<T>::load1(p, c * sC);
  x4[int64_t(nh) * W + w] = make_uint2(uint32_t(f2bf(v[0])) | (uint32_t(f2bf(v[1])) << 16),
                                       uint32_t(f2bf(v[2])) | (uint32_t(f2bf(v[3])) << 16));
}

// fp32 NCHW rows (W % 4 == 0): 4 pixels per thread, one 16-byte load per channel plane and
// two 16-byte stores (the one-pixel version ran at ~3.9 TB/s on 4- and 8-byte accesses)
__global__ __launch_bounds__(256) void stem_pack4_f32_kernel(const float* __restrict__ x, uint4* __restrict__ x4,
                                                             int C, int H, int W, int64_t sN, int64_t sC,
                                                             int64_t sH) {
  const int w4 = blockIdx.y * 256 + threadIdx.x;
  if (4 * w4 >= W) return;
  const int nh = blockIdx.x;
  const int n = nh / H, h = nh - (nh / H) * H;
  const float* p = x + n * sN + h * sH + 4 * w4;
  float4 v[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] = c < C ? *reinterpret_cast<const float4*>(p + c * sC) : make_float4(0, 0, 0, 0);
  auto px = [&](float a0, float a1, float a2, float a3) {
    return make_uint2(uint32_t(f2bf(a0)) | (uint32_t(f2bf(a1)) << 16), uint32_t(f2bf(a2)) | (uint32_t(f2bf(a3)) << 16));
  };
  const uint2 q0 = px(v[0].x, v[1].x, v[2].x, v[3].x), q1 = px(v[0].y, v[1].y, v[2].y, v[3].y);
  const uint2 q2 = px(v[0].z, v[1].z, v[2].z, v[3].z), q3 = px(v[0].w, v[1].w, v[2].w, v[3].w);
  uint4* o = x4 + (int64_t(nh) * W + 4 * w4) / 2;
  o[0] = make_uint4(q0.x, q0.y, q1.x, q1.y);
  o[1] = make_uint4(q2.x, q2.y, q3.x, q3.y);
}

// fp32 channels_last 3-channel rows (sC = 1, sW = 3, W % 4 == 0): 4 pixels = 48 B = three
// 16-byte loads per thread, two 16-byte stores
__global__ __launch_bounds__(256) void stem_pack4_nhwc3_f32_kernel(const float* __restrict__ x,
                                                                   uint4* __restrict__ x4, int H, int W, int64_t sN,
                                                                   int64_t sH) {
  const int w4 = blockIdx.y * 256 + threadIdx.x;
  if (4 * w4 >= W) return;
  const int nh = blockIdx.x;
  const int n = nh / H, h = nh - (nh / H) * H;
  const float4* p = reinterpret_cast<const float4*>(x + n * sN + h * sH + 12 * w4);
  const float4 a = p[0], b = p[1], c = p[2];  // px0 rgb px1 rgb px2 rgb px3 rgb
  auto px = [](float r, float g, float bl) {
    return make_uint2(uint32_t(f2bf(r)) | (uint32_t(f2bf(g)) << 16), uint32_t(f2bf(bl)));
  };
  const uint2 q0 = px(a.x, a.y, a.z), q1 = px(a.w, b.x, b.y), q2 = px(b.z, b.w, c.x), q3 = px(c.y, c.z, c.w);
  uint4* o = x4 + (int64_t(nh) * W + 4 * w4) / 2;
  o[0] = make_uint4(q0.x, q0.y, q1.x, q1.y);
  o[1] = make_uint4(q2.x, q2.y, q3.x, q3.y);
}

int stem_grid_blocks() {
  static int g = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
      hipDeviceProp_t p;
      if (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0) cus = p.multiProcessorCount;
    }
    return 2 * cus;
  }();
  return g;
}

}  // namespace

constexpr int kWMaxSlices = 64;

int64_t stem_wgrad_workspace_floats(int N, int Ho) {
  return int64_t(stem_partial_rows(N, Ho) + kWMaxSlices) * kSCo * kWK;
}

void stem_conv_wgrad(uintptr_t x4, uintptr_t dy, uintptr_t dw, int64_t s0, int64_t s1, int64_t s2, int64_t s3,
                     int Cin, uintptr_t ws, int N, int H, int W, int Ho, int Wo, bool accumulate, int out_dt,
                     uintptr_t stream) {
  VODA_CHECK(Cin >= 1 && Cin <= 4, "stem_wgrad: Cin <= 4 only");
  VODA_CHECK(Ho == (H + 2 * kSP - kSK) / kSS + 1 && Wo == (W + 2 * kSP - kSK) / kSS + 1,
             "stem_wgrad: output size mismatch (7x7, stride 2, pad 3)");
  VODA_CHECK(Wo >= 1 && Wo <= kSMaxWo, "stem_wgrad: output width must be <= 128");
  VODA_CHECK(out_dt == kF32 || out_dt == kBF16, "stem_wgrad: dW must be fp32 or bf16");
  VODA_CHECK(x4 % 8 == 0 && dy % 16 == 0 && ws % 16 == 0, "stem_wgrad: misaligned operands");
  hipStream_t s = as_stream(stream);
  const int nb = stem_partial_rows(N, Ho);
  float* part = reinterpret_cast<float*>(ws);
  float* tmp = part + int64_t(nb) * kSCo * kWK;
  const int nsl = std::min(kWMaxSlices, nb);
  StemWArgs a{reinterpret_cast<const uint2*>(x4), reinterpret_cast<const uint16_t*>(dy), part, N, H, W, Ho, Wo};
  hipLaunchKernelGGL(stem_conv7x7_wgrad_kernel, dim3(nb), dim3(kSThreads), 0, s, a);
  hipLaunchKernelGGL(stem_wgrad_slice_kernel, dim3((kSCo * kWK / 4 + 255) / 256, nsl), dim3(256), 0, s,
                     reinterpret_cast<const float4*>(part), nb, reinterpret_cast<float4*>(tmp));
  const int total = kSCo * kSK * kSK;
  const float4* t4 = reinterpret_cast<const float4*>(tmp);
  if (out_dt == kF32)
    hipLaunchKernelGGL((stem_wgrad_final_kernel<float>), dim3((total + 255) / 256), dim3(256), 0, s, t4, nsl, Cin,
                       reinterpret_cast<float*>(dw), s0, s1, s2, s3, int(accumulate));
  else
    hipLaunchKernelGGL((stem_wgrad_final_kernel<uint16_t>), dim3((total + 255) / 256), dim3(256), 0, s, t4, nsl, Cin,
                       reinterpret_cast<uint16_t*>(dw), s0, s1, s2, s3, int(accumulate));
  check_launch();
}

int stem_partial_rows(int N, int Ho) {
  const int64_t rows = int64_t(N) * Ho;
  return int(std::max<int64_t>(1, std::min<int64_t>(stem_grid_blocks(), rows)));
}

void stem_pack(uintptr_t x, uintptr_t x4, int N, int C, int H, int W, int64_t sN, int64_t sC, int64_t sH, int64_t sW,
               int dt, uintptr_t stream) {
  VODA_CHECK(C >= 1 && C <= 4, "stem_pack: 1..4 input channels");
  VODA_CHECK(int64_t(N) * H < (int64_t(1) << 31), "stem_pack: too many image rows");
  if (int64_t(N) * H * W == 0) return;
  hipStream_t s = as_stream(stream);
  const dim3 grid(unsigned(N * H), unsigned((W + 255) / 256));
  uint2* o = reinterpret_cast<uint2*>(x4);
  const bool vec4 = dt == kF32 && sW == 1 && W % 4 == 0 && x % 16 == 0 && x4 % 16 == 0 && sN % 4 == 0 &&
                    sC % 4 == 0 && sH % 4 == 0;
  const bool nhwc3 = dt == kF32 && C == 3 && sC == 1 && sW == 3 && W % 4 == 0 && x % 16 == 0 && x4 % 16 == 0 &&
                     sN % 4 == 0 && sH % 4 == 0;
  if (nhwc3)
    hipLaunchKernelGGL(stem_pack4_nhwc3_f32_kernel, dim3(unsigned(N * H), unsigned((W / 4 + 255) / 256)), dim3(256), 0,
                       s, reinterpret_cast<const float*>(x), reinterpret_cast<uint4*>(x4), H, W, sN, sH);
  else if (vec4)
    hipLaunchKernelGGL(stem_pack4_f32_kernel, dim3(unsigned(N * H), unsigned((W / 4 + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const float*>(x), reinterpret_cast<uint4*>(x4), C, H, W, sN, sC, sH);
  else if (dt == kF32)
    hipLaunchKernelGGL((stem_pack_kernel<float>), grid, dim3(256), 0, s, reinterpret_cast<const float*>(x), o, C, H, W,
                       sN, sC, sH, sW);
  else if (dt == kBF16)
    hipLaunchKernelGGL((stem_pack_kernel<BF16>), grid, dim3(256), 0, s, reinterpret_cast<const BF16*>(x), o, C, H, W,
                       sN, sC, sH, sW);
  else if (dt == kF16)
    hipLaunchKernelGGL((stem_pack_kernel<F16>), grid, dim3(256), 0, s, reinterpret_cast<const F16*>(x), o, C, H, W, sN,
                       sC, sH, sW);
  else
    throw std::invalid_argument("stem_pack: unsupported dtype");
  check_launch();
}

void stem_conv_fwd(uintptr_t x4, uintptr_t w, int64_t sw0, int64_t sw1, int64_t sw2, int64_t sw3, int Cin, int Cout,
                   uintptr_t y, uintptr_t part, int nb, int N, int H, int W, int Ho, int Wo, uintptr_t stream) {
  VODA_CHECK(Cin >= 1 && Cin <= 4 && Cout == kSCo, "stem_conv: Cin <= 4 and Cout == 64 only");
  VODA_CHECK(Ho == (H + 2 * kSP - kSK) / kSS + 1 && Wo == (W + 2 * kSP - kSK) / kSS + 1,
             "stem_conv: output size mismatch (7x7, stride 2, pad 3)");
  VODA_CHECK(Wo >= 1 && Wo <= kSMaxWo, "stem_conv: output width must be <= 128");
  VODA_CHECK(nb == stem_partial_rows(N, Ho), "stem_conv: partial-row count mismatch");
  VODA_CHECK(x4 % 8 == 0 && y % 16 == 0 && part % 4 == 0, "stem_conv: misaligned operands");
  StemArgs a{reinterpret_cast<const uint2*>(x4), reinterpret_cast<const uint16_t*>(w), sw0, sw1, sw2, sw3, Cin,
             reinterpret_cast<uint16_t*>(y), reinterpret_cast<float*>(part), N, H, W, Ho, Wo};
  hipLaunchKernelGGL(stem_conv7x7_fwd_kernel, dim3(nb), dim3(kSThreads), 0, as_stream(stream), a);
  check_launch();
}

}  // namespace voda
