// Weight gradient of a 3x3 / stride-1 / pad-1 convolution with 64 input and 64 output
// channels (ResNet-50 layer1, ResNet-18/34 layer1), channels_last bf16 activations:
//
//   dW[co][kh][kw][ci] (+)= sum over pixels (n, h, w) of dY[n][h][w][co] * X[n][h+kh-1][w+kw-1][ci]
//
// MIOpen runs it as an atomic split-K igemm_wrw (~150 us at bs 256, 56 x 56) plus a workspace
// clear, a cast and the fold into the flat fp32 gradient (~15 us); the repo's 128 x 128-tile
// implicit-GEMM kernel (wgrad.hip) fills a quarter of its tile at 64 channels (360 us).
// Here the problem is what it is: a 64 x 576 result reduced over 0.8 M pixels.
//  * persistent workgroups (1 per CU, one wave per SIMD: the 144 accumulators and the 2-deep
//    prefetch need more than the 256 registers of two waves) walk contiguous chunks of rows; per row the dY
//    row is staged as [64 px][192 B] and the input rows h-1, h, h+1 sit in a 4-slot LDS ring
//    of [66 px][192 B] rows (zero outside the image); the 192-byte pixel pitch makes the
//    transposed reads below conflict-free;
//  * both MFMA operands need 8 consecutive PIXELS per lane: ds_read_b64_tr_b16 reads them as
//    columns (per-lane addresses: the im2col rows of tap (kh, kw) are the ring pixels shifted
//    by kw, no im2col buffer);
//  * D = 2 channel tiles x 18 (tap, 32-channel block) tiles of 32 x 32; wave w owns channel
//    tile w & 1 and 9 of the 18 column tiles (144 accumulator registers), accumulated over the
//    whole row chunk;
//  * the next rows' loads run two rows ahead in registers (a global load's ~1-2 us latency is
//    longer than a row's MFMA work), written into the LDS after each row's MFMAs;
//  * one fp32 partial [64][576] per workgroup; two small passes sum them and add the result
//    into the optimizer's flat gradient with the weight's strides.
#include "common.h"

#include "ops.h"

#include <cstdlib>

namespace voda {

namespace {

typedef __bf16 c64_bf16x8 __attribute__((ext_vector_type(8)));
typedef float c64_f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 c64_bf16x4_v __attribute__((__vector_size__(4 * sizeof(__bf16))));
typedef __attribute__((address_space(3))) c64_bf16x4_v c64_lds_bf16x4;

constexpr int kC = 64;                     // channels in and out
constexpr int kThreads = 256;
constexpr int kMaxW = 64;                  // output pixels per row (4 k-steps of 16)
constexpr int kPxB = 192;                  // LDS bytes per pixel (128 + 64 pad)
constexpr int kRingPx = kMaxW + 2;         // 66 pixels per input row (pad 1 each side)
constexpr int kSlotB = kRingPx * kPxB;     // 12672 B
constexpr int kSlots = 4;                  // rows h-1, h, h+1 + the next row
constexpr int kDyB = kMaxW * kPxB;         // 12288 B
constexpr int kK = 9 * kC;                 // 576 result columns (tap-major, channels_last)
constexpr int kRowChunks = kRingPx * 8;    // 16-B chunks of one ring row (528)
constexpr int kXPf = (kRowChunks + kThreads - 1) / kThreads;  // 3
constexpr int kDyPf = (kMaxW * 8 + kThreads - 1) / kThreads;  // 2

struct C64Args {
  const uint16_t* x;   // [N][H][W][64]
  const uint16_t* dy;  // [N][H][W][64]
  float* part;         // [gridDim.x][64][576]
  int N, H, W;
};

__device__ __forceinline__ uint2 c64_tr(const unsigned char* p) {
  const c64_bf16x4_v v = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((c64_lds_bf16x4*)(p));
  return __builtin_bit_cast(uint2, v);
}

__device__ __forceinline__ c64_bf16x8 c64_frag(const unsigned char* lo, const unsigned char* hi) {
  const uint2 a = c64_tr(lo), b = c64_tr(hi);
  return __builtin_bit_cast(c64_bf16x8, make_uint4(a.x, a.y, b.x, b.y));
}

// 16-byte chunk c (0..527) of ring row hi of image n: pixel j = c / 8 is input column j - 1
__device__ __forceinline__ uint4 c64_xchunk(const C64Args& a, int64_t n, int hi, int c) {
  const int j = c >> 3, part = c & 7;
  const int wi = j - 1;
  const bool ok = unsigned(hi) < unsigned(a.H) && unsigned(wi) < unsigned(a.W);
  const int hc = min(max(hi, 0), a.H - 1), wc = min(max(wi, 0), a.W - 1);
  const uint4 v = reinterpret_cast<const uint4*>(a.x + ((n * a.H + hc) * a.W + wc) * kC)[part];
  const uint32_t m = ok ? 0xffffffffu : 0u;
  return make_uint4(v.x & m, v.y & m, v.z & m, v.w & m);
}

__global__ __launch_bounds__(kThreads, 1) void conv3x3_c64_wgrad_kernel(C64Args a) {
  __shared__ __attribute__((aligned(16))) unsigned char ring[kSlots * kSlotB];
  __shared__ __attribute__((aligned(16))) unsigned char dyt[kDyB];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int lh = lane >> 5, lg = (lane >> 4) & 1, lq = (lane & 15) >> 2, lp = lane & 3;
  const int ct = wave & 1;            // output-channel tile
  const int kt0 = (wave >> 1) * 9;    // first of this wave's 9 (tap, channel-block) tiles

  for (int i = tid; i < (kMaxW - a.W) * (kPxB / 16); i += kThreads)
    *reinterpret_cast<uint4*>(dyt + a.W * kPxB + i * 16) = make_uint4(0u, 0u, 0u, 0u);

  c64_f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = c64_f32x16{};

  const int64_t rows = int64_t(a.N) * a.H;
  const int64_t per = (rows + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = int64_t(blockIdx.x) * per;
  const int64_t r1 = r0 + per < rows ? r0 + per : rows;
  const int dchunks = a.W * 8;

  // per-lane byte offsets of the transposed reads at k-step 0
  const int a_off = (8 * lh + lq) * kPxB + (32 * ct + 16 * lg + 4 * lp) * 2;
  const int b_off = (8 * lh + lq) * kPxB + (16 * lg + 4 * lp) * 2;

  int64_t n = r0 / a.H;
  int h = int(r0 - n * a.H);
  uint4 xa0, xa1, xa2, xb0, xb1, xb2, da0, da1, db0, db1;
  static_assert(kXPf == 3 && kDyPf == 2, "prefetch slots");
  auto load_x = [&](int hi, uint4& v0, uint4& v1, uint4& v2) {
    v0 = c64_xchunk(a, n, hi, tid);
    v1 = c64_xchunk(a, n, hi, tid + kThreads);
    v2 = c64_xchunk(a, n, hi, min(tid + 2 * kThreads, kRowChunks - 1));
  };
  auto load_dy = [&](int64_t r, uint4& v0, uint4& v1) {
    const uint4* d = reinterpret_cast<const uint4*>(a.dy + r * a.W * kC);
    v0 = d[min(tid, dchunks - 1)];
    v1 = d[min(tid + kThreads, dchunks - 1)];
  };
  auto put_x = [&](int hi, int c, const uint4& v) {
    if (c < kRowChunks)
      *reinterpret_cast<uint4*>(ring + (hi & (kSlots - 1)) * kSlotB + (c >> 3) * kPxB + (c & 7) * 16) = v;
  };
  auto put_dy = [&](int c, const uint4& v) {
    if (c < dchunks) *reinterpret_cast<uint4*>(dyt + (c >> 3) * kPxB + (c & 7) * 16) = v;
  };
  bool pa = false, in_lds = false;
  for (int64_t row = r0; row < r1; ++row) {
    if (!in_lds) {  // first row of the chunk or of an image: input rows h-1 .. h+1, dY row
      for (int r = 0; r < 3; ++r)
        for (int c = tid; c < kRowChunks; c += kThreads) put_x(h - 1 + r, c, c64_xchunk(a, n, h - 1 + r, c));
      for (int c = tid; c < dchunks; c += kThreads)
        put_dy(c, reinterpret_cast<const uint4*>(a.dy + row * a.W * kC)[c]);
    }
    __syncthreads();
    const bool nxt1 = row + 1 < r1 && h + 1 < a.H;
    const bool nxt2 = nxt1 && row + 2 < r1 && h + 2 < a.H;
    if (nxt1 && !pa) {
      load_x(h + 2, xa0, xa1, xa2);
      load_dy(row + 1, da0, da1);
      pa = true;
    }
    if (nxt2) {
      load_x(h + 3, xb0, xb1, xb2);
      load_dy(row + 2, db0, db1);
    }
    int so[3];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) so[kh] = ((h - 1 + kh) & (kSlots - 1)) * kSlotB;
#pragma unroll
    for (int ks = 0; ks < kMaxW / 16; ++ks) {
      const unsigned char* ap = dyt + a_off + ks * 16 * kPxB;
      const c64_bf16x8 af = c64_frag(ap, ap + 4 * kPxB);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int kt = kt0 + t;  // tap = kt / 2, channel block = kt & 1 (kt0 is 0 or 9)
        const int tap = kt >> 1, cb = kt & 1;
        const int kh = tap / 3, kw = tap - 3 * (tap / 3);
        const unsigned char* bp = ring + so[kh] + b_off + (ks * 16 + kw) * kPxB + cb * 64;
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, c64_frag(bp, bp + 4 * kPxB), acc[t], 0, 0, 0);
      }
    }
    __syncthreads();  // every wave is done with this row's dY tile and window
    if (pa) {
      put_x(h + 2, tid, xa0);
      put_x(h + 2, tid + kThreads, xa1);
      put_x(h + 2, tid + 2 * kThreads, xa2);
      put_dy(tid, da0);
      put_dy(tid + kThreads, da1);
    }
    in_lds = pa;
    xa0 = xb0; xa1 = xb1; xa2 = xb2; da0 = db0; da1 = db1;
    pa = nxt2;
    if (++h == a.H) { h = 0; ++n; }
  }

  float* out = a.part + int64_t(blockIdx.x) * kC * kK + (lane & 31);
#pragma unroll
  for (int t = 0; t < 9; ++t) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = 32 * ct + (r & 3) + 8 * (r >> 2) + 4 * lh;
      out[co * kK + (kt0 + t) * 32] = acc[t][r];
    }
  }
}

// ------------------------------------------------------------------------------------------
// fp32 twin (the reference-precision run) on v_mfma_f32_32x32x2_f32: a k-step is TWO pixels,
// and the f32 MFMA's operand layout (lane l: A[i = l&31][k = l>>5], B[k = l>>5][j = l&31]) is
// the pixel-major [px][channel] LDS image read straight -- 32 consecutive channels of one
// pixel per lane half, no transposed reads.  Same work split (wave w: output-channel tile
// w & 1, 9 of the 18 (tap, 32-channel block) tiles, 144 accumulators) and 4-slot ring of input
// rows.  The rows arrive by LDS-DMA (global_load_lds_dwordx4: an NHWC row is W x 256 contiguous
// bytes, the LDS image is unpadded [px][64 floats]): the next row's new input row and dY row
// are issued at the start of a row into buffers nobody reads during it (ring slot h + 2 and
// the other dY buffer) and waited for only before the row's closing barrier -- register
// prefetch did not survive compilation (the loads were sunk to their use after the MFMA loop,
// or the pad select hoisted above it: one exposed memory latency per chunk, half the time).
constexpr int kFPitch = 64;                     // floats per LDS pixel (DMA writes linearly)

struct C64ArgsF {
  const float* x;   // [N][H][W][64]
  const float* dy;  // [N][H][W][64]
  float* part;      // [gridDim.x][64][576]
  int N, H, W;
};

typedef float c64_f32x16f __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void c64_lds_void;

// LDS[m0 + 16 * lane] = global[gptr] (inline asm: hipcc must not see an LDS write in flight,
// or it would guard every LDS read of the row with a wait on it)
__device__ __forceinline__ void c64_dma16(const void* gptr, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gptr), "s"(lds_addr) : "memory", "m0");
}

// one row of `pieces` 16-byte pieces from global `src` to LDS `dst`, 1 KB per wave-instruction,
// instructions dealt round-robin to the 4 waves; lanes past the row stay idle (exec-masked)
__device__ __forceinline__ void c64_dma_row(const float* src, float* dst, int pieces, int wave, int lane) {
  for (int i = wave; i * 64 < pieces; i += 4) {
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(uint32_t(size_t((c64_lds_void*)(dst + 256 * i))));
    const int piece = i * 64 + lane;
    if (piece < pieces) c64_dma16(src + 4 * piece, m0);
  }
}

__device__ __forceinline__ void c64_wait_dma() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// One row's MFMAs of a wave.  Tiles are (tap, cb) with the 32-channel blocks of a tap
// INTERLEAVED: block cb holds input channels 2j + cb (j = lane & 31), so ONE ds_read_b64 of
// channels (2j, 2j + 1) feeds both blocks' MFMAs -- 5 B reads + 1 A read per pixel pair
// instead of 9 + 1.  Wave group g (= wave >> 1) owns tiles 0..7 = both blocks of taps
// 5g .. 5g + 3 (pointer pairs q = 0..3) and tile 8 = (tap 4, cb g) (pair q = 4, component g):
// the same code for both groups, so no per-group copies of the 144 accumulators.  Two register
// sets ping-pong over pixel pairs: the next pair's operands are read while the current pair's
// 9 MFMAs issue.
__device__ __forceinline__ float c64f_b(const float2 (&b)[5], int t, bool g) {
  return t < 8 ? ((t & 1) ? b[t >> 1].y : b[t >> 1].x) : (g ? b[4].y : b[4].x);
}

__device__ __forceinline__ void c64f_row_mfma(c64_f32x16f (&acc)[9], const float* ap, const float* const (&bq)[5],
                                              int steps, bool g) {
  float a0 = ap[0], a1;
  float2 b0[5], b1[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) b0[q] = *reinterpret_cast<const float2*>(bq[q]);
  int s = 0;
  for (; s + 1 < steps; s += 2) {
    const int o1 = 2 * (s + 1) * kFPitch;
    const int o2 = 2 * (s + 2 < steps ? s + 2 : steps - 1) * kFPitch;
    __builtin_amdgcn_sched_barrier(0);
    a1 = ap[o1];
#pragma unroll
    for (int q = 0; q < 5; ++q) b1[q] = *reinterpret_cast<const float2*>(bq[q] + o1);
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, c64f_b(b0, t, g), acc[t], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    a0 = ap[o2];
#pragma unroll
    for (int q = 0; q < 5; ++q) b0[q] = *reinterpret_cast<const float2*>(bq[q] + o2);
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, c64f_b(b1, t, g), acc[t], 0, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  if (s < steps) {
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, c64f_b(b0, t, g), acc[t], 0, 0, 0);
  }
}

// WMAX: widest image row the LDS image holds.  WMAX = 56 (ResNet layer1) fits two workgroups
// per CU (73.7 KB: a 4-slot ring of 58-pixel rows + ONE dY row buffer; 69 VGPRs + 144 AGPRs
// leave room for two waves per SIMD), so one workgroup's row boundary -- closing barrier, dY
// DMA, wait -- overlaps the other's MFMAs.  WMAX = 64: one workgroup per CU, dY double-
// buffered and fetched during the previous row.
template <int WMAX>
__global__ __launch_bounds__(kThreads, WMAX <= 56 ? 2 : 1) void conv3x3_c64_wgrad_f32_kernel(C64ArgsF a) {
  constexpr bool DBUF = WMAX > 56;
  constexpr int SLOT = (WMAX + 2) * kFPitch;  // floats per ring row (pad pixel each side)
  __shared__ __attribute__((aligned(1024))) float ring[kSlots * SLOT];
  __shared__ __attribute__((aligned(1024))) float dyt[DBUF ? 2 : 1][WMAX * kFPitch];

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int lh = lane >> 5, lr = lane & 31;
  const int ct = wave & 1;
  const int grp = wave >> 1;  // tile group (see c64f_row_mfma)

  // everything zero once: pad pixels, pixels >= W and the dY pixels >= W stay zero (the DMA
  // writes input pixels 1..W of a ring row and dY pixels 0..W-1 only)
  for (int i = tid; i < kSlots * SLOT / 4; i += kThreads) reinterpret_cast<float4*>(ring)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int i = tid; i < (DBUF ? 2 : 1) * WMAX * kFPitch / 4; i += kThreads)
    reinterpret_cast<float4*>(&dyt[0][0])[i] = make_float4(0.f, 0.f, 0.f, 0.f);

  c64_f32x16f acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = c64_f32x16f{};

  const int64_t rows = int64_t(a.N) * a.H;
  const int64_t per = (rows + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = int64_t(blockIdx.x) * per;
  const int64_t r1 = r0 + per < rows ? r0 + per : rows;
  const int pieces = a.W * 16;
  const int steps = (a.W + 1) / 2;

  int64_t n = r0 / a.H;
  int h = int(r0 - n * a.H);
  // input row hi of image n into its ring slot (pixels 1..W); rows outside the image: zeros
  auto stage_x = [&](int hi) {
    float* slot = ring + (hi & (kSlots - 1)) * SLOT;
    if (unsigned(hi) < unsigned(a.H)) {
      c64_dma_row(a.x + (n * a.H + hi) * int64_t(a.W) * kC, slot + kFPitch, pieces, wave, lane);
    } else {
      for (int i = tid; i < pieces; i += kThreads)
        reinterpret_cast<float4*>(slot + kFPitch)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  int buf = 0;
  bool in_lds = false;
  __syncthreads();
  for (int64_t row = r0; row < r1; ++row) {
    if (!in_lds) {  // first row of the chunk or of an image: input rows h-1 .. h+1 and the dY row
      stage_x(h - 1);
      stage_x(h);
      stage_x(h + 1);
      c64_dma_row(a.dy + row * a.W * kC, dyt[buf], pieces, wave, lane);
      c64_wait_dma();
      __syncthreads();
    }
    const bool nxt = row + 1 < r1 && h + 1 < a.H;
    if (nxt) {  // the next row's new input row (h + 2) [and dY row], landing during this row
      stage_x(h + 2);
      if constexpr (DBUF) c64_dma_row(a.dy + (row + 1) * a.W * kC, dyt[buf ^ 1], pieces, wave, lane);
    }
    const float* ap = dyt[buf] + lh * kFPitch + 32 * ct + lr;
    const float* bq[5];  // taps 5g .. 5g + 3 and tap 4, channels (2j, 2j + 1)
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const int tap = q < 4 ? 5 * grp + q : 4;
      const int kh = tap / 3, kw = tap - 3 * (tap / 3);
      bq[q] = ring + ((h - 1 + kh) & (kSlots - 1)) * SLOT + (lh + kw) * kFPitch + 2 * lr;
    }
    c64f_row_mfma(acc, ap, bq, steps, grp != 0);
    if constexpr (DBUF) {
      c64_wait_dma();   // this wave's pieces of the next row have landed
      __syncthreads();  // ... and everyone's; this row's reads are done
    } else {
      __syncthreads();  // this row's dY reads done: the single buffer takes the next row
      if (nxt) c64_dma_row(a.dy + (row + 1) * a.W * kC, dyt[0], pieces, wave, lane);
      c64_wait_dma();
      __syncthreads();
    }
    in_lds = nxt;
    if (DBUF && nxt) buf ^= 1;
    if (++h == a.H) { h = 0; ++n; }
  }

  float* out = a.part + int64_t(blockIdx.x) * kC * kK + 2 * lr;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int tap = t < 8 ? 5 * grp + (t >> 1) : 4, cb = t < 8 ? (t & 1) : grp;
    const int col = tap * kC + cb;  // tap * 64 + cb (+ 2j): interleaved channel blocks
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = 32 * ct + (r & 3) + 8 * (r >> 2) + 4 * lh;
      out[co * kK + col] = acc[t][r];
    }
  }
}

// partial sums in two passes: [nb][E] -> [nsl][E] (float4, each slice sums <= 8 partial rows)
// -> dW.  (The first version summed nb / 32 scalar rows per thread and then 32 more: two
// latency-bound ~10 us passes per call.)
__global__ __launch_bounds__(256) void c64_slice_kernel(const float4* __restrict__ part, int nb, int e4,
                                                        float4* __restrict__ tmp) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= e4) return;
  const int sl = blockIdx.y, nsl = gridDim.y;
  const int per = (nb + nsl - 1) / nsl;
  const int b0 = sl * per, b1 = min(nb, b0 + per);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int b = b0; b < b1; ++b) {
    const float4 v = part[int64_t(b) * e4 + e];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  tmp[int64_t(sl) * e4 + e] = s;
}

// [nsl][64][576] -> dW[co][ci][kh][kw] with element strides, fp32 or bf16, (+)=; 4 consecutive
// ci per thread (one float4 of every slice)
template <typename OutT>
__global__ __launch_bounds__(256) void c64_final_kernel(const float4* __restrict__ tmp, int nsl, OutT* __restrict__ dw,
                                                        int64_t s0, int64_t s1, int64_t s2, int64_t s3,
                                                        int accumulate) {
  const int e4 = blockIdx.x * 256 + threadIdx.x;  // (co * 576 + (kh * 3 + kw) * 64 + ci) / 4
  if (e4 >= kC * kK / 4) return;
  const int e = 4 * e4;
  const int co = e / kK, k = e - co * kK;
  const int tap = k >> 6, ci = k & 63;
  const int kh = tap / 3, kw = tap - 3 * kh;
  float4 s0v = make_float4(0.f, 0.f, 0.f, 0.f), s1v = s0v;
  int sl = 0;
  for (; sl + 1 < nsl; sl += 2) {
    const float4 a = tmp[int64_t(sl) * (kC * kK / 4) + e4], b = tmp[int64_t(sl + 1) * (kC * kK / 4) + e4];
    s0v.x += a.x; s0v.y += a.y; s0v.z += a.z; s0v.w += a.w;
    s1v.x += b.x; s1v.y += b.y; s1v.z += b.z; s1v.w += b.w;
  }
  if (sl < nsl) {
    const float4 a = tmp[int64_t(sl) * (kC * kK / 4) + e4];
    s0v.x += a.x; s0v.y += a.y; s0v.z += a.z; s0v.w += a.w;
  }
  const float v[4] = {s0v.x + s1v.x, s0v.y + s1v.y, s0v.z + s1v.z, s0v.w + s1v.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    OutT* o = dw + co * s0 + (ci + q) * s1 + kh * s2 + kw * s3;
    if constexpr (sizeof(OutT) == 4) {
      *reinterpret_cast<float*>(o) = v[q] + (accumulate ? *reinterpret_cast<float*>(o) : 0.f);
    } else {
      uint16_t* p = reinterpret_cast<uint16_t*>(o);
      *p = f2bf(v[q] + (accumulate ? bf2f(*p) : 0.f));
    }
  }
}

int c64_grid() {
  static int g = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
      hipDeviceProp_t p;
      if (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0) cus = p.multiProcessorCount;
    }
    return cus;  // one 4-wave workgroup per CU: 144 accumulators + 2-deep prefetch > 256 VGPRs
  }();
  return g;
}

int c64_blocks(int N, int H, int per_cu = 1) {
  return int(std::max<int64_t>(1, std::min<int64_t>(int64_t(per_cu) * c64_grid(), int64_t(N) * H)));
}

}  // namespace

constexpr int kMaxSlices = 64;

int64_t conv3x3_c64_wgrad_workspace_floats(int N, int H) {
  return int64_t(c64_blocks(N, H, 2) + kMaxSlices) * kC * kK;  // the fp32 W <= 56 kernel: 2 per CU
}

void conv3x3_c64_wgrad(uintptr_t x, uintptr_t dy, uintptr_t dw, int64_t s0, int64_t s1, int64_t s2, int64_t s3,
                       uintptr_t ws, int N, int H, int W, bool accumulate, int out_dt, uintptr_t stream, int in_dt) {
  VODA_CHECK(W >= 1 && W <= kMaxW && H >= 1, "conv3x3_c64_wgrad: image width must be 1..64");
  VODA_CHECK(out_dt == kF32 || out_dt == kBF16, "conv3x3_c64_wgrad: dW must be fp32 or bf16");
  VODA_CHECK(x % 16 == 0 && dy % 16 == 0 && ws % 16 == 0, "conv3x3_c64_wgrad: misaligned operands");
  hipStream_t s = as_stream(stream);
  const bool f32_two = in_dt == kF32 && W <= 56;
  const int nb = c64_blocks(N, H, f32_two ? 2 : 1);
  float* part = reinterpret_cast<float*>(ws);
  float* tmp = part + int64_t(nb) * kC * kK;
  const int nsl = std::min(kMaxSlices, nb);
  VODA_CHECK(in_dt == kBF16 || in_dt == kF32, "conv3x3_c64_wgrad: activations must be bf16 or fp32");
  if (in_dt == kF32) {
    C64ArgsF a{reinterpret_cast<const float*>(x), reinterpret_cast<const float*>(dy), part, N, H, W};
    if (f32_two) hipLaunchKernelGGL((conv3x3_c64_wgrad_f32_kernel<56>), dim3(nb), dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL((conv3x3_c64_wgrad_f32_kernel<kMaxW>), dim3(nb), dim3(kThreads), 0, s, a);
  } else {
    C64Args a{reinterpret_cast<const uint16_t*>(x), reinterpret_cast<const uint16_t*>(dy), part, N, H, W};
    hipLaunchKernelGGL(conv3x3_c64_wgrad_kernel, dim3(nb), dim3(kThreads), 0, s, a);
  }
  const int e4 = kC * kK / 4;
  hipLaunchKernelGGL(c64_slice_kernel, dim3((e4 + 255) / 256, nsl), dim3(256), 0, s,
                     reinterpret_cast<const float4*>(part), nb, e4, reinterpret_cast<float4*>(tmp));
  if (out_dt == kF32)
    hipLaunchKernelGGL((c64_final_kernel<float>), dim3((e4 + 255) / 256), dim3(256), 0, s,
                       reinterpret_cast<const float4*>(tmp), nsl, reinterpret_cast<float*>(dw), s0, s1, s2, s3,
                       int(accumulate));
  else
    hipLaunchKernelGGL((c64_final_kernel<uint16_t>), dim3((e4 + 255) / 256), dim3(256), 0, s,
                       reinterpret_cast<const float4*>(tmp), nsl, reinterpret_cast<uint16_t*>(dw), s0, s1, s2, s3,
                       int(accumulate));
  check_launch();
}

// ---- flipped, channel-transposed filter for the input gradient as a forward convolution
// (ops/conv3x3.dgrad_as_forward): wt[ci][co][kh][kw] = w[co][ci][K-1-kh][K-1-kw], written
// channels_last ([ci][kh][kw][co] in memory) and in the activations' dtype -- one launch instead
// of a flip, a layout copy and (under autocast) a cast.  The filter is at most a few MB (L2).
namespace {
// one 32 (co) x 32 (ci) tile of one filter tap per block, transposed through LDS: the reads run
// along ci (contiguous in a channels_last filter), the writes along co (contiguous in the output)
template <typename IT, typename OT>
__global__ __launch_bounds__(256) void filter_flip_t_kernel(const IT* __restrict__ w, int64_t s0, int64_t s1,
                                                            int64_t s2, int64_t s3, OT* __restrict__ out, int Cout,
                                                            int Cin, int K) {
  __shared__ float tile[32][33];
  const int co0 = blockIdx.x * 32, ci0 = blockIdx.y * 32;
  const int kh = int(blockIdx.z) / K, kw = int(blockIdx.z) - (int(blockIdx.z) / K) * K;  // source tap
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int co = co0 + ty + 8 * j, ci = ci0 + tx;
    tile[ty + 8 * j][tx] = (co < Cout && ci < Cin) ? Vec4<IT>::load1(w, co * s0 + ci * s1 + kh * s2 + kw * s3) : 0.f;
  }
  __syncthreads();
  // destination tap (K-1-kh, K-1-kw); out memory order [ci][kh'][kw'][co]
  const int64_t tap = int64_t(K - 1 - kh) * K + (K - 1 - kw);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int ci = ci0 + ty + 8 * j, co = co0 + tx;
    if (ci < Cin && co < Cout) Vec4<OT>::store1(out, (int64_t(ci) * K * K + tap) * Cout + co, tile[tx][ty + 8 * j]);
  }
}
}  // namespace

void filter_flip_t(uintptr_t w, int in_dt, int64_t s0, int64_t s1, int64_t s2, int64_t s3, uintptr_t out,
                   int out_dt, int Cout, int Cin, int K, uintptr_t stream) {
  VODA_CHECK(Cout > 0 && Cin > 0 && K > 0, "filter_flip_t: empty filter");
  VODA_CHECK((in_dt == kF32 || in_dt == kBF16) && (out_dt == kF32 || out_dt == kBF16),
             "filter_flip_t: fp32 or bf16");
  const dim3 grid(unsigned((Cout + 31) / 32), unsigned((Cin + 31) / 32), unsigned(K * K));
  hipStream_t s = as_stream(stream);
  auto go = [&](auto it, auto ot) {
    using IT = decltype(it);
    using OT = decltype(ot);
    hipLaunchKernelGGL((filter_flip_t_kernel<IT, OT>), grid, dim3(256), 0, s, reinterpret_cast<const IT*>(w), s0, s1,
                       s2, s3, reinterpret_cast<OT*>(out), Cout, Cin, K);
  };
  if (in_dt == kF32) {
    if (out_dt == kF32) go(float{}, float{});
    else go(float{}, BF16{});
  } else {
    if (out_dt == kF32) go(BF16{}, float{});
    else go(BF16{}, BF16{});
  }
  check_launch();
}

}  // namespace voda
