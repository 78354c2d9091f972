// Weight-gradient GEMM of Linear layers on CDNA4 MFMA (gfx950), bias gradient fused.
//
//   dW[N][K] (+)= dY[M][N]^T . X[M][K]        db[N] (+)= sum_m dY[m][N]
//
// hipBLASLt runs these "reduction = tokens" GEMMs at 190-490 TFLOP/s on BERT-base (M = 8192
// tokens, N, K in {768, 2304, 3072}; profiles/): a 768 x 768 weight is only 36 output tiles
// of 128 x 128 on 256 CUs.  Design:
//  * split-K over the token dimension so the grid covers the chip; each split writes an fp32
//    partial slab and a reduce kernel sums the slabs and accumulates into the optimizer's
//    flat bf16 gradient (beta = 1).  With one split the GEMM epilogue accumulates directly.
//  * both operands are row-major with the REDUCTION dimension as rows, so a 64-token x
//    128-column tile is staged into LDS as-is (16-byte global loads, XOR-swizzled 256-byte
//    rows) and the MFMA fragments -- 8 consecutive tokens of one column per lane -- come out
//    of the gfx950 transposing LDS read ds_read_b64_tr_b16 (guide T10, layout (b)); no
//    transpose pass anywhere.
//  * v_mfma_f32_32x32x16_bf16; 4 waves as 2 x 2, each wave a 64 x 64 sub-tile (2 x 2 MFMA
//    tiles, 64 fp32 accumulators per lane).  LDS double-buffered with register staging: the
//    loads of stage s+1 are issued before the MFMAs of stage s and written after them.
//  * XCD-aware block remap (guide T1): consecutive logical blocks land on the same XCD / L2.
//    Logical order split-major (kWgradSplitMajor): an XCD's ~grid/8 blocks are
//    neighbouring tiles of ONE split -- a (rows x cols) patch of the output whose workgroups
//    stream the same token range, so each dY / X stage fetched into the XCD's L2 feeds a whole
//    row / column of the patch.  The older order (0) put the splits of one tile on one XCD:
//    they read disjoint token ranges and share nothing.
//  * the bias gradient rides along: in workgroups of output-column block 0 the waves of
//    column half 0 also multiply their dY fragments by a ones operand (one extra MFMA per
//    dY fragment), which is sum_m dY[m][n] in fp32 with no second pass over dY.
#include "common.h"

#include <cstdlib>
#include "ops.h"

namespace voda {

namespace {

typedef __bf16 wg_bf16x8 __attribute__((ext_vector_type(8)));
typedef float wg_f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 wg_bf16x4_v __attribute__((__vector_size__(4 * sizeof(__bf16))));
typedef __attribute__((address_space(3))) wg_bf16x4_v wg_lds_bf16x4;

constexpr int kWgBN = 128;                          // output rows (n) per workgroup
constexpr int kWgBK = 128;                          // output cols (k) per workgroup
constexpr int kWgBM = 64;                           // tokens per LDS stage
constexpr int kWgThreads = 256;
constexpr int kWgRowBytes = 256;                    // 128 bf16 per LDS row
constexpr int kWgTileBytes = kWgBM * kWgRowBytes;   // 16 KB per operand tile

struct WgradArgs {
  const uint16_t* dy; int64_t ldy;   // [M][N]
  const uint16_t* x; int64_t ldx;    // [M][K]
  uint16_t* dw; int64_t ldw;         // [N][K]        (splits == 1)
  uint16_t* db;                      // [N] or null   (splits == 1)
  // out_f32: dW / db are fp32 (the optimizer's fp32 flat gradient of a bf16 model: one
  // rounding of the fp32 MFMA accumulators, none of the bf16 accumulate-and-round); the
  // pointers above are then reinterpreted as float*
  int out_f32;
  float* ws;                         // [S][N][K] + [S][N] partial slabs (splits > 1)
  const uint16_t* zero;              // >= 16 zero bytes: source of rows past the split (LDS-DMA path)
  int M, N, K, S, m_split, tiles_k, remap, accumulate, bias;
  int split_major;  // logical block order: 0 = splits of one tile adjacent, 1 = tiles of one split adjacent
  int zcol;         // LDS-DMA kernels: chunks past N / K read the zero buffer (1) or a clamped duplicate (0)
  int tiles_total;  // output tiles per tap (split_major decode)
  // epilogue addressing: dW column (and workspace column) offset and workspace row stride
  int col0, ws_ld;
  // implicit-GEMM convolution weight gradient (CONV kernels only): X rows are the input
  // pixels under kernel tap (kh, kw) of output pixel m = (img, ho, wo); taps = KH * KW
  // launches' worth of tiles share one grid, tap-major
  int taps, KW, H, W, Ho, Wo, cstride, pad, tiles_nk;
  int adv_n, adv_ho, adv_wo;  // BM output pixels expressed as (images, rows, columns)
};

// byte offset of 16-byte chunk ``ch`` (0..15) of LDS row ``r``: XOR swizzle that keeps both
// the 16-B row writes and the 32x32x16 transposed reads conflict-free (guide T10 (b))
__device__ __forceinline__ int wg_swz(int r, int ch) {
  return r * kWgRowBytes + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3)));
}

__device__ __forceinline__ uint2 wg_tr_read(const uint8_t* base, int off) {
  wg_bf16x4_v v = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((wg_lds_bf16x4*)(base + off));
  return __builtin_bit_cast(uint2, v);
}

// v if keep else 0, as lane-wise ANDs (a struct select here becomes a scratch round trip)
__device__ __forceinline__ uint4 wg_keep(uint4 v, bool keep) {
  const uint32_t m = keep ? 0xffffffffu : 0u;
  return make_uint4(v.x & m, v.y & m, v.z & m, v.w & m);
}

// MFMA operand -- 8 consecutive tokens (rows r..r+3 and r+4..r+7) of the column this lane
// receives -- from precomputed lane offsets (the swizzle term of a row depends only on
// row & 15 modulo the k-step, so a k-step's rows sit at a constant +4096 B: immediates).
__device__ __forceinline__ wg_bf16x8 wg_frag_at(const uint8_t* tile, int off_lo, int off_hi) {
  const uint2 lo = wg_tr_read(tile, off_lo);
  const uint2 hi = wg_tr_read(tile, off_hi);
  return __builtin_bit_cast(wg_bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
}

__device__ __forceinline__ wg_f32x16 wg_mfma(wg_bf16x8 a, wg_bf16x8 b, wg_f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// dW / db element (+)= v in the output precision (bf16 or fp32)
__device__ __forceinline__ void wg_store_out(uint16_t* base, int64_t idx, float v, int accumulate, int out_f32) {
  if (out_f32) {
    float* o = reinterpret_cast<float*>(base) + idx;
    *o = v + (accumulate ? *o : 0.f);
  } else {
    uint16_t* o = base + idx;
    *o = f2bf(v + (accumulate ? bf2f(*o) : 0.f));
  }
}

// C/D lane map of v_mfma_f32_32x32x16_bf16: col = lane & 31, row = (reg&3) + 8*(reg>>2) + 4*h.
// splits == 1: accumulate into dW / db directly; else write this split's fp32 slab.
__device__ __forceinline__ void wgrad_epilogue(const WgradArgs& p, int split, int n0, int k0, int wn, int wk,
                                               int lane, const wg_f32x16& c00, const wg_f32x16& c01,
                                               const wg_f32x16& c10, const wg_f32x16& c11, const wg_f32x16& cb0,
                                               const wg_f32x16& cb1, bool do_bias) {
  const int h = lane >> 5;
  const int col_l = lane & 31;
  auto store_tile = [&](const wg_f32x16& acc, int rbase, int cbase) {
    const int col = cbase + col_l;
    if (col >= p.K) return;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int row = rbase + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (row < p.N) {
        if (p.S == 1) {
          wg_store_out(p.dw, int64_t(row) * p.ldw + p.col0 + col, acc[reg], p.accumulate, p.out_f32);
        } else {
          p.ws[(int64_t(split) * p.N + row) * p.ws_ld + p.col0 + col] = acc[reg];
        }
      }
    }
  };
  const int rb0 = n0 + wn * 64, cb0i = k0 + wk * 64;
  store_tile(c00, rb0, cb0i);
  store_tile(c01, rb0, cb0i + 32);
  store_tile(c10, rb0 + 32, cb0i);
  store_tile(c11, rb0 + 32, cb0i + 32);
  if (do_bias && col_l == 0) {  // every column of cb holds the row sums; lanes 0 and 32 write
    float* wsb = p.ws + int64_t(p.S) * p.N * p.ws_ld + int64_t(split) * p.N;
    auto store_bias = [&](const wg_f32x16& acc, int rbase) {
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int row = rbase + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        if (row < p.N) {
          if (p.S == 1) {
            wg_store_out(p.db, row, acc[reg], p.accumulate, p.out_f32);
          } else {
            wsb[row] = acc[reg];
          }
        }
      }
    };
    store_bias(cb0, rb0);
    store_bias(cb1, rb0 + 32);
  }
}

__global__ __launch_bounds__(kWgThreads, 2) void wgrad_kernel(WgradArgs p) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[4 * kWgTileBytes];  // [buffer][dY | X]

  int bid = blockIdx.x;
  if (p.remap) bid = (bid & 7) * int(gridDim.x >> 3) + (bid >> 3);
  const int split = p.split_major ? bid / p.tiles_total : bid % p.S;
  const int tile = p.split_major ? bid - split * p.tiles_total : bid / p.S;
  const int n0 = (tile / p.tiles_k) * kWgBN;
  const int k0 = (tile % p.tiles_k) * kWgBK;
  const int mb = split * p.m_split;
  const int me = min(p.M, mb + p.m_split);
  const int nst = me > mb ? (me - mb + kWgBM - 1) / kWgBM : 0;

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const bool do_bias = __builtin_amdgcn_readfirstlane(p.bias && k0 == 0 && wk == 0);  // wave-uniform

  // ---- global -> register staging, two stages deep.  Thread t moves the 16-byte chunk
  // (t & 15) of tile rows (t >> 4) + 16 i, i = 0..3.  Row pointers advance by 64 rows per
  // stage (no per-load index arithmetic); rows past the split / matrix read a valid dummy
  // address and are zeroed at the LDS write, after the MFMAs (masking right after the load
  // would make hipcc wait for every load before the MFMAs).  Stage s+2 is loaded while stage s
  // is computed and stage s+1 (loaded one stage earlier) is written to LDS.
  struct Stg {
    uint4 a[4], b[4];
    uint32_t keep;  // bit i: chunk i of dY in range, bit 4+i: chunk i of X in range
  };
  Stg sx, sy;
  const int ch_t = t & 15, r_t = t >> 4;
  const bool col_a = n0 + ch_t * 8 < p.N, col_b = k0 + ch_t * 8 < p.K;
  const int64_t sa16 = int64_t(16) * p.ldy, sb16 = int64_t(16) * p.ldx;
  const uint16_t* cur_a = p.dy + int64_t(mb + r_t) * p.ldy + min(n0 + ch_t * 8, p.N - 8);
  const uint16_t* cur_b = p.x + int64_t(mb + r_t) * p.ldx + min(k0 + ch_t * 8, p.K - 8);
  int m_cur = mb + r_t;
  auto gload = [&](Stg& d) {
    d.keep = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool okm = m_cur + 16 * i < me;
      const uint16_t* ga = okm ? cur_a + i * sa16 : p.dy;
      const uint16_t* gb = okm ? cur_b + i * sb16 : p.x;
      d.a[i] = *reinterpret_cast<const uint4*>(ga);
      d.b[i] = *reinterpret_cast<const uint4*>(gb);
      d.keep |= (uint32_t(okm && col_a) << i) | (uint32_t(okm && col_b) << (4 + i));
    }
    cur_a += 4 * sa16;
    cur_b += 4 * sb16;
    m_cur += kWgBM;
  };
  // LDS image offset of those chunks: the swizzle term of row r_t + 16 i does not depend on i
  const int woff = wg_swz(r_t, ch_t);
  auto swrite = [&](const Stg& d, int buf) {
    uint8_t* A = smem + buf * 2 * kWgTileBytes;
    uint8_t* B = A + kWgTileBytes;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *reinterpret_cast<uint4*>(A + woff + 4096 * i) = wg_keep(d.a[i], (d.keep >> i) & 1);
      *reinterpret_cast<uint4*>(B + woff + 4096 * i) = wg_keep(d.b[i], (d.keep >> (4 + i)) & 1);
    }
  };

  wg_f32x16 c00, c01, c10, c11, cb0, cb1;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    c00[i] = 0.f; c01[i] = 0.f; c10[i] = 0.f; c11[i] = 0.f; cb0[i] = 0.f; cb1[i] = 0.f;
  }
  wg_bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = static_cast<__bf16>(1.0f);

  // lane offsets of the transposed reads (guide T10: lane 4q+p of a 16-lane group reads row q
  // of the block, columns 4p..4p+3; lane i of the group gets column i); k-step kk adds 4096*kk
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3, h = lane >> 5;
  const int bo = 8 * (pp & 1);
  const int chA = ((wn * 64 + 16 * (g & 1)) >> 3) + (pp >> 1);  // sub-tile 1: +4 chunks (32 columns)
  const int chB = ((wk * 64 + 16 * (g & 1)) >> 3) + (pp >> 1);
  const int r0 = 8 * h + q;
  const int oa0l = wg_swz(r0, chA) + bo, oa0h = wg_swz(r0 + 4, chA) + bo;
  const int oa1l = wg_swz(r0, chA + 4) + bo, oa1h = wg_swz(r0 + 4, chA + 4) + bo;
  const int ob0l = wg_swz(r0, chB) + bo, ob0h = wg_swz(r0 + 4, chB) + bo;
  const int ob1l = wg_swz(r0, chB + 4) + bo, ob1h = wg_swz(r0 + 4, chB + 4) + bo;

  auto compute = [&](int buf) {
    const uint8_t* A = smem + buf * 2 * kWgTileBytes;
    const uint8_t* B = A + kWgTileBytes;
    // fragments of k-step kk+1 are read while the MFMAs of k-step kk run
    wg_bf16x8 a0 = wg_frag_at(A, oa0l, oa0h), a1 = wg_frag_at(A, oa1l, oa1h);
    wg_bf16x8 b0 = wg_frag_at(B, ob0l, ob0h), b1 = wg_frag_at(B, ob1l, ob1h);
#pragma unroll
    for (int kk = 0; kk < kWgBM / 16; ++kk) {
      wg_bf16x8 na0 = a0, na1 = a1, nb0 = b0, nb1 = b1;
      if (kk + 1 < kWgBM / 16) {
        const uint8_t* An = A + 4096 * (kk + 1);
        const uint8_t* Bn = B + 4096 * (kk + 1);
        na0 = wg_frag_at(An, oa0l, oa0h); na1 = wg_frag_at(An, oa1l, oa1h);
        nb0 = wg_frag_at(Bn, ob0l, ob0h); nb1 = wg_frag_at(Bn, ob1l, ob1h);
      }
      c00 = wg_mfma(a0, b0, c00);
      c01 = wg_mfma(a0, b1, c01);
      c10 = wg_mfma(a1, b0, c10);
      c11 = wg_mfma(a1, b1, c11);
      if (do_bias) {
        cb0 = wg_mfma(a0, ones, cb0);
        cb1 = wg_mfma(a1, ones, cb1);
      }
      a0 = na0; a1 = na1; b0 = nb0; b1 = nb1;
    }
  };
  // one stage: load st+2 into ``ld``, compute st, write st+1 (held in ``wr``) to LDS
  auto iter = [&](int st, const Stg& wr, Stg& ld) {
    if (st + 2 < nst) gload(ld);
    compute(st & 1);
    if (st + 1 < nst) swrite(wr, (st + 1) & 1);
    __syncthreads();
  };

  if (nst > 0) {
    gload(sx);
    swrite(sx, 0);
    if (nst > 1) gload(sy);
  }
  __syncthreads();
  for (int st = 0; st < nst; st += 2) {  // unrolled by two: register sets stay compile-time
    iter(st, sy, sx);
    if (st + 1 < nst) iter(st + 1, sx, sy);
  }
  wgrad_epilogue(p, split, n0, k0, wn, wk, lane, c00, c01, c10, c11, cb0, cb1, do_bias);
}


// ---------------------------------------------------------------------------------------
// v2: the same tile, fed by an LDS ring of kWgStages stages filled with global_load_lds
// (16-byte LDS-DMA, no staging registers).  At ~1 workgroup per CU (grid ~ 256-432) the
// register-staged kernel above waits one full HBM latency per 64-token stage; here
// kWgStages - 1 stages stay in flight while the MFMAs run (guide §5 'Async global->LDS
// copy', 'Pipelining across barriers': one __shared__ array, counted vmcnt, raw
// s_barrier).  The LDS image is the same XOR-swizzled one: LDS-DMA writes lane-linearly,
// so the swizzle moves to the per-lane GLOBAL address (guide §5.4 rule 21): lane l of a
// wave-instruction fills row r = 4j + l/16, slot s = l%16, and loads chunk s ^ f(r).
// Rows past the split read a zero buffer; columns past N / K read clamped (finite) data
// that only reaches output rows / columns that are never stored.
// ---------------------------------------------------------------------------------------

// One 16-byte LDS-DMA per lane: LDS[m0 + 16 * lane] = global[gptr].  Issued as inline asm so
// that hipcc does not see an LDS write in flight: it would otherwise guard the next
// ds_read_b64_tr_b16 with s_waitcnt vmcnt(0) and drain the whole ring every stage.  The
// ring's completion is tracked by hand (wg_wait_vm) and published by the barrier.
__device__ __forceinline__ void wg_dma16(const void* gptr, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gptr), "s"(lds_addr) : "memory", "m0");
}

template <int N>
__device__ __forceinline__ void wg_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// kWgStages = 4: 128 KB ring, 1 workgroup/CU, 3 stages in flight; 2: 64 KB, 2 workgroups/CU
template <int PER>
__device__ __forceinline__ void wg_wait_ahead(int ahead) {  // vmcnt(ahead * PER), ahead <= 4
  switch (ahead) {
    case 4: wg_wait_vm<4 * PER>(); break;
    case 3: wg_wait_vm<3 * PER>(); break;
    case 2: wg_wait_vm<2 * PER>(); break;
    case 1: wg_wait_vm<PER>(); break;
    default: wg_wait_vm<0>(); break;
  }
}

// kWgStages ring stages of BM tokens each: <4, 64> 128 KB, 1 workgroup/CU; <2, 64> 64 KB,
// 2 workgroups/CU; <3, 64>; <4, 32> 64 KB with 3 stages in flight at 2 workgroups/CU.
template <int kWgStages, int BM, bool CONV = false>
__global__ __launch_bounds__(kWgThreads, 1) void wgrad_glds_kernel(WgradArgs p) {
  constexpr int TB = BM * kWgRowBytes;   // bytes per operand tile
  constexpr int SB = 2 * TB;             // bytes per stage (dY tile + X tile)
  constexpr int IPW = BM / 16;           // 1 KB LDS-DMA wave-instructions per wave per operand tile
  constexpr int PER = 2 * IPW;           // LDS-DMA instructions per lane per stage
  static_assert(BM % 16 == 0 && BM <= 64, "stage depth");
  __shared__ __attribute__((aligned(16))) uint8_t smem[kWgStages * SB];
  typedef __attribute__((address_space(3))) void lds_void;

  int bid = blockIdx.x;
  if (p.remap) bid = (bid & 7) * int(gridDim.x >> 3) + (bid >> 3);
  int tap = 0;
  if constexpr (CONV) {
    const int per_tap = p.S * p.tiles_nk;
    tap = bid / per_tap;
    bid -= tap * per_tap;
    p.col0 = tap * p.K;
  }
  const int split = p.split_major ? bid / p.tiles_total : bid % p.S;
  const int tile = p.split_major ? bid - split * p.tiles_total : bid / p.S;
  const int n0 = (tile / p.tiles_k) * kWgBN;
  const int k0 = (tile % p.tiles_k) * kWgBK;
  const int mb = split * p.m_split;
  const int me = min(p.M, mb + p.m_split);
  const int nst = me > mb ? (me - mb + BM - 1) / BM : 0;

  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wn = wave >> 1, wk = wave & 1;
  const bool do_bias = __builtin_amdgcn_readfirstlane(p.bias && k0 == 0 && wk == 0);

  // this lane's part of each of the wave's IPW wave-instructions per operand tile:
  // instruction i covers tile rows 4j .. 4j+3 with j = IPW*wave + i
  const int lr = lane >> 4, slot = lane & 15;
  // CONV: output pixel (img, ho, wo) of each of this lane's IPW rows, advanced by BM pixels
  // per issued stage (issue() is called for stages 0, 1, 2, ... in order)
  int pn[IPW], pho[IPW], pwo[IPW];
  int dh = 0, dw = 0;
  if constexpr (CONV) {
    dh = tap / p.KW - p.pad;
    dw = tap % p.KW - p.pad;
    const int hw = p.Ho * p.Wo;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int m = mb + 4 * (IPW * wave + i) + lr;
      pn[i] = m / hw;
      const int rem = m - pn[i] * hw;
      pho[i] = rem / p.Wo;
      pwo[i] = rem - pho[i] * p.Wo;
    }
  }
  // this lane's source rows of stage 0 (row 4j + lr of the tile, swizzled chunk), advanced by
  // BM rows per stage with one scalar multiply: no per-load 64-bit index arithmetic
  // Chunks past N / K (a 64-channel operand in a 128-column tile) read the zero buffer rather
  // than a clamped duplicate of the last chunk: their outputs are never stored, and one
  // shared 16-byte line costs the fill path nothing where 8 distinct duplicate reads per row
  // did (p.zcol = 0 restores the clamped reads for A/B runs).
  const uint16_t* row_a[IPW];
  const uint16_t* row_b[IPW];
  uint32_t colok_a = 0, colok_b = 0;
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int r = 4 * (IPW * wave + i) + lr;
    const int ch = slot ^ (((r & 3) << 2) | ((r >> 2) & 3));
    row_a[i] = p.dy + int64_t(mb + r) * p.ldy + min(n0 + ch * 8, p.N - 8);
    row_b[i] = CONV ? p.x : p.x + int64_t(mb + r) * p.ldx + min(k0 + ch * 8, p.K - 8);
    colok_a |= uint32_t(!p.zcol || n0 + ch * 8 < p.N) << i;
    colok_b |= uint32_t(!p.zcol || k0 + ch * 8 < p.K) << i;
  }
  auto issue = [&](int st) {
    uint8_t* A = smem + (st % kWgStages) * SB;
    uint8_t* B = A + TB;
    const int m_base = mb + st * BM;
    const int64_t adv_a = int64_t(st * BM) * p.ldy, adv_b = int64_t(st * BM) * p.ldx;
    const bool full = m_base + BM <= me;  // wave-uniform: no row of this stage is past the split
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int j = IPW * wave + i;
      const int r = 4 * j + lr;
      const int ch = slot ^ (((r & 3) << 2) | ((r >> 2) & 3));
      const int m = m_base + r;
      const bool okm = full || m < me;
      const uint16_t* ga = (okm && ((colok_a >> i) & 1)) ? row_a[i] + adv_a : p.zero;
      const uint16_t* gb;
      if constexpr (CONV) {
        const int hi = pho[i] * p.cstride + dh, wi = pwo[i] * p.cstride + dw;
        const bool ok = okm && ((colok_b >> i) & 1) && hi >= 0 && hi < p.H && wi >= 0 && wi < p.W;
        gb = ok ? p.x + (int64_t(pn[i] * p.H + hi) * p.W + wi) * p.ldx + min(k0 + ch * 8, p.K - 8) : p.zero;
        // advance this row by BM output pixels (single carries: the steps are < Wo and < Ho)
        pwo[i] += p.adv_wo;
        pho[i] += p.adv_ho;
        pn[i] += p.adv_n;
        if (pwo[i] >= p.Wo) { pwo[i] -= p.Wo; pho[i] += 1; }
        if (pho[i] >= p.Ho) { pho[i] -= p.Ho; pn[i] += 1; }
      } else {
        gb = (okm && ((colok_b >> i) & 1)) ? row_b[i] + adv_b : p.zero;
      }
      wg_dma16(ga, __builtin_amdgcn_readfirstlane(uint32_t(size_t((lds_void*)(A + 1024 * j)))));
      wg_dma16(gb, __builtin_amdgcn_readfirstlane(uint32_t(size_t((lds_void*)(B + 1024 * j)))));
    }
  };

  wg_f32x16 c00, c01, c10, c11, cb0, cb1;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    c00[i] = 0.f; c01[i] = 0.f; c10[i] = 0.f; c11[i] = 0.f; cb0[i] = 0.f; cb1[i] = 0.f;
  }
  wg_bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = static_cast<__bf16>(1.0f);
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3, h = lane >> 5;
  const int bo = 8 * (pp & 1);
  const int chA = ((wn * 64 + 16 * (g & 1)) >> 3) + (pp >> 1);
  const int chB = ((wk * 64 + 16 * (g & 1)) >> 3) + (pp >> 1);
  const int r0 = 8 * h + q;
  const int oa0l = wg_swz(r0, chA) + bo, oa0h = wg_swz(r0 + 4, chA) + bo;
  const int oa1l = wg_swz(r0, chA + 4) + bo, oa1h = wg_swz(r0 + 4, chA + 4) + bo;
  const int ob0l = wg_swz(r0, chB) + bo, ob0h = wg_swz(r0 + 4, chB) + bo;
  const int ob1l = wg_swz(r0, chB + 4) + bo, ob1h = wg_swz(r0 + 4, chB + 4) + bo;

  constexpr int D = kWgStages - 1;  // stages in flight ahead of the one being computed
#pragma unroll
  for (int s0 = 0; s0 < D; ++s0)
    if (s0 < nst) issue(s0);
  for (int st = 0; st < nst; ++st) {
    // stage st has landed once at most min(D - 1, nst - 1 - st) later stages are outstanding
    // (PER LDS-DMA instructions per stage per lane)
    wg_wait_ahead<PER>(min(D - 1, nst - 1 - st));
    __builtin_amdgcn_s_barrier();  // every wave's DMA of stage st landed; stage st-1 fully read
    if (st + D < nst) issue(st + D);  // refills the buffer of stage st-1
    const uint8_t* A = smem + (st % kWgStages) * SB;
    const uint8_t* B = A + TB;
    wg_bf16x8 a0 = wg_frag_at(A, oa0l, oa0h), a1 = wg_frag_at(A, oa1l, oa1h);
    wg_bf16x8 b0 = wg_frag_at(B, ob0l, ob0h), b1 = wg_frag_at(B, ob1l, ob1h);
#pragma unroll
    for (int kk = 0; kk < BM / 16; ++kk) {
      wg_bf16x8 na0 = a0, na1 = a1, nb0 = b0, nb1 = b1;
      if (kk + 1 < BM / 16) {
        const uint8_t* An = A + 4096 * (kk + 1);
        const uint8_t* Bn = B + 4096 * (kk + 1);
        na0 = wg_frag_at(An, oa0l, oa0h); na1 = wg_frag_at(An, oa1l, oa1h);
        nb0 = wg_frag_at(Bn, ob0l, ob0h); nb1 = wg_frag_at(Bn, ob1l, ob1h);
      }
      c00 = wg_mfma(a0, b0, c00);
      c01 = wg_mfma(a0, b1, c01);
      c10 = wg_mfma(a1, b0, c10);
      c11 = wg_mfma(a1, b1, c11);
      if (do_bias) {
        cb0 = wg_mfma(a0, ones, cb0);
        cb1 = wg_mfma(a1, ones, cb1);
      }
      a0 = na0; a1 = na1; b0 = nb0; b1 = nb1;
    }
    // all fragment reads of this stage are consumed by the MFMAs above before the next
    // barrier, after which another wave may refill this buffer
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  wgrad_epilogue(p, split, n0, k0, wn, wk, lane, c00, c01, c10, c11, cb0, cb1, do_bias);
}

// ---------------------------------------------------------------------------------------------
// Wide tile: 256 x 256 outputs per workgroup, 8 waves as 2 (n) x 4 (k), each a 128 x 64 sub-tile
// (4 x 2 MFMA tiles, 128 fp32 accumulators per lane).  Twice the MFMA work per operand byte of
// the 128 x 128 tile (128 vs 64 FLOP per byte staged), which is what the LDS-DMA fill rate
// per CU limits (MI355X_MICROARCH.md, ldsdma-fill): 6 fragment reads feed 8 MFMAs per k-step.
// An operand stage is two 128-column halves, each the 256-byte-row swizzled image above, so
// the fragment addressing is unchanged.  The bias gradient is a v_dot2c_f32_bf16 against ones
// on the dY fragments the n-waves already hold (4 dot2 per fragment, no extra MFMA or
// accumulator tile).
constexpr int kWwTile = 256;
constexpr int kWwThreads = 512;

// Epilogue of the 256 x 256 kernels (C lane map as in wgrad_epilogue): wave (wn, wk) holds
// rows n0 + 128 wn + 32 f, columns k0 + 128 (wk >> 1) + 64 (wk & 1) + 32 e; bs[f] = the bias
// partial sums of its dY fragments (waves with wk == 0 of output-column block 0).
__device__ __forceinline__ void wide_epilogue(const WgradArgs& p, int split, int n0, int k0, int wn, int wk, int lane,
                                              const wg_f32x16 (&c)[4][2], const float (&bs)[4], bool do_bias) {
  const int h = lane >> 5;
  const int col_l = lane & 31;
#pragma unroll
  for (int f = 0; f < 4; ++f) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int col = k0 + (wk >> 1) * 128 + (wk & 1) * 64 + 32 * e + col_l;
      if (col < p.K) {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int row = n0 + wn * 128 + 32 * f + (reg & 3) + 8 * (reg >> 2) + 4 * h;
          if (row < p.N) {
            if (p.S == 1) {
              wg_store_out(p.dw, int64_t(row) * p.ldw + col, c[f][e][reg], p.accumulate, p.out_f32);
            } else {
              p.ws[(int64_t(split) * p.N + row) * p.ws_ld + col] = c[f][e][reg];
            }
          }
        }
      }
    }
  }
  if (do_bias) {
    // lane l (< 32) and l + 32 hold tokens 8h..8h+7 of every k-step for row 32f + l
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const float tot = bs[f] + __shfl_xor(bs[f], 32);
      const int row = n0 + wn * 128 + 32 * f + col_l;
      if (h == 0 && row < p.N) {
        if (p.S == 1) {
          wg_store_out(p.db, row, tot, p.accumulate, p.out_f32);
        } else {
          p.ws[int64_t(p.S) * p.N * p.ws_ld + int64_t(split) * p.N + row] = tot;
        }
      }
    }
  }
}

// Epilogue of the transposed 256 x 256 accumulators (wgrad_wide2_kernel computes C^T = X^T dY:
// lane = output row n = n0 + 128 wn + 32 f + (lane & 31), registers 4g..4g+3 = four
// consecutive columns k = k0 + 128 (wk >> 1) + 64 (wk & 1) + 32 e + 8 g + 4 h + 0..3), so each
// store moves 16 bytes (fp32) or 8 bytes (bf16): a quarter of the store instructions of the
// one-dword-per-register layout, whose issue rate bounded the epilogue.
__device__ __forceinline__ void wide_epilogue_t(const WgradArgs& p, int split, int n0, int k0, int wn, int wk,
                                                int lane, const wg_f32x16 (&c)[4][2], const float (&bs)[4],
                                                bool do_bias) {
  const int h = lane >> 5;
  const int col_l = lane & 31;
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const int row = n0 + wn * 128 + 32 * f + col_l;
    if (row >= p.N) continue;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = k0 + (wk >> 1) * 128 + (wk & 1) * 64 + 32 * e + 8 * g + 4 * h;
        if (col >= p.K) continue;
        float4 v = make_float4(c[f][e][4 * g], c[f][e][4 * g + 1], c[f][e][4 * g + 2], c[f][e][4 * g + 3]);
        if (p.S > 1) {
          *reinterpret_cast<float4*>(p.ws + (int64_t(split) * p.N + row) * p.ws_ld + col) = v;
        } else if (p.out_f32) {
          float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(p.dw) + int64_t(row) * p.ldw + col);
          if (p.accumulate) {
            const float4 u = *o;
            v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
          }
          *o = v;
        } else {
          uint2* o = reinterpret_cast<uint2*>(p.dw + int64_t(row) * p.ldw + col);
          if (p.accumulate) {
            const uint2 u = *o;
            v.x += bf2f(u.x & 0xffff); v.y += bf2f(u.x >> 16); v.z += bf2f(u.y & 0xffff); v.w += bf2f(u.y >> 16);
          }
          *o = make_uint2(uint32_t(f2bf(v.x)) | (uint32_t(f2bf(v.y)) << 16),
                          uint32_t(f2bf(v.z)) | (uint32_t(f2bf(v.w)) << 16));
        }
      }
    }
  }
  if (do_bias) {
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const float tot = bs[f] + __shfl_xor(bs[f], 32);
      const int row = n0 + wn * 128 + 32 * f + col_l;
      if (h == 0 && row < p.N) {
        if (p.S == 1) {
          wg_store_out(p.db, row, tot, p.accumulate, p.out_f32);
        } else {
          p.ws[int64_t(p.S) * p.N * p.ws_ld + int64_t(split) * p.N + row] = tot;
        }
      }
    }
  }
}

template <int kStages, int BM>
__global__ __launch_bounds__(kWwThreads, 1) void wgrad_wide_kernel(WgradArgs p) {
  constexpr int TH = BM * kWgRowBytes;   // bytes per operand half (BM rows x 128 columns)
  constexpr int TB = 2 * TH;             // bytes per operand tile
  constexpr int SB = 2 * TB;             // bytes per stage
  constexpr int IPW = BM / 16;           // LDS-DMA wave-instructions per wave per operand tile
  constexpr int PER = 2 * IPW;           // per lane per stage
  constexpr int QR = BM / 4;             // wave-instructions per operand half
  static_assert(BM % 16 == 0 && BM <= 64, "stage depth");
  __shared__ __attribute__((aligned(16))) uint8_t smem[kStages * SB];
  typedef __attribute__((address_space(3))) void lds_void;

  int bid = blockIdx.x;
  if (p.remap) bid = (bid & 7) * int(gridDim.x >> 3) + (bid >> 3);
  const int split = p.split_major ? bid / p.tiles_total : bid % p.S;
  const int tile = p.split_major ? bid - split * p.tiles_total : bid / p.S;
  const int n0 = (tile / p.tiles_k) * kWwTile;
  const int k0 = (tile % p.tiles_k) * kWwTile;
  const int mb = split * p.m_split;
  const int me = min(p.M, mb + p.m_split);
  const int nst = me > mb ? (me - mb + BM - 1) / BM : 0;

  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wn = wave >> 2, wk = wave & 3;
  const bool do_bias = __builtin_amdgcn_readfirstlane(p.bias && k0 == 0 && wk == 0);

  const int lr = lane >> 4, slot = lane & 15;
  auto issue = [&](int st) {
    uint8_t* A = smem + (st % kStages) * SB;
    uint8_t* B = A + TB;
    const int m_base = mb + st * BM;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int j = IPW * wave + i;          // 0 .. 2*QR-1
      const int half = j / QR, rq = j % QR;  // rows 4rq .. 4rq+3 of column half ``half``
      const int r = 4 * rq + lr;
      const int ch = slot ^ (((r & 3) << 2) | ((r >> 2) & 3));
      const int m = m_base + r;
      const bool okm = m < me;
      const int cn = min(n0 + half * 128 + ch * 8, p.N - 8);
      const int ck = min(k0 + half * 128 + ch * 8, p.K - 8);
      const uint16_t* ga = okm ? p.dy + int64_t(m) * p.ldy + cn : p.zero;
      const uint16_t* gb = okm ? p.x + int64_t(m) * p.ldx + ck : p.zero;
      const int lo = half * TH + 1024 * rq;
      wg_dma16(ga, __builtin_amdgcn_readfirstlane(uint32_t(size_t((lds_void*)(A + lo)))));
      wg_dma16(gb, __builtin_amdgcn_readfirstlane(uint32_t(size_t((lds_void*)(B + lo)))));
    }
  };

  wg_f32x16 c[4][2];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int i = 0; i < 16; ++i) c[f][e][i] = 0.f;
  float bs[4] = {0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3, h = lane >> 5;
  const int bo = 8 * (pp & 1);
  const int r0 = 8 * h + q;
  const int cbase = 2 * (g & 1) + (pp >> 1);
  int oa[4][2], ob[2][2];
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    oa[f][0] = wn * TH + wg_swz(r0, cbase + 4 * f) + bo;
    oa[f][1] = wn * TH + wg_swz(r0 + 4, cbase + 4 * f) + bo;
  }
  const int kc = 8 * (wk & 1);  // 64-column quarter within the k half, in 8-column chunks
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    ob[e][0] = (wk >> 1) * TH + wg_swz(r0, kc + cbase + 4 * e) + bo;
    ob[e][1] = (wk >> 1) * TH + wg_swz(r0 + 4, kc + cbase + 4 * e) + bo;
  }
  typedef __bf16 wg_bf16x2 __attribute__((ext_vector_type(2)));
  const wg_bf16x2 one2 = {static_cast<__bf16>(1.0f), static_cast<__bf16>(1.0f)};

  // Pipelined across stages: the wait + barrier for stage st+1 and its first fragment reads
  // sit in front of the MFMAs of stage st's last k-step, so the reads' LDS latency hides
  // behind those MFMAs instead of stalling every wave after every barrier.  The refill issued
  // at that barrier overwrites stage st-1's buffer (consumed by MFMAs before the barrier), so
  // D = kStages - 2 stages are in flight beyond the one being waited for.
  static_assert(kStages >= 3, "cross-stage pipelining needs >= 3 ring stages");
  constexpr int D = kStages - 2;
  constexpr int KS = BM / 16;
  auto load_frags = [&](int st, int kk, wg_bf16x8 (&fa)[4], wg_bf16x8 (&fb)[2]) {
    const uint8_t* A = smem + (st % kStages) * SB + 4096 * kk;
    const uint8_t* B = A + TB;
#pragma unroll
    for (int f = 0; f < 4; ++f) fa[f] = wg_frag_at(A, oa[f][0], oa[f][1]);
#pragma unroll
    for (int e = 0; e < 2; ++e) fb[e] = wg_frag_at(B, ob[e][0], ob[e][1]);
  };
#pragma unroll
  for (int s0 = 0; s0 <= D; ++s0)
    if (s0 < nst) issue(s0);
  wg_bf16x8 a[4], b[2];
  if (nst > 0) {
    wg_wait_ahead<PER>(min(D, nst - 1));
    __builtin_amdgcn_s_barrier();
    load_frags(0, 0, a, b);
  }
  for (int st = 0; st < nst; ++st) {
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      wg_bf16x8 na[4], nb[2];
      if (kk + 1 < KS) {
        load_frags(st, kk + 1, na, nb);
      } else if (st + 1 < nst) {
        wg_wait_ahead<PER>(min(D - 1, nst - 2 - st));
        __builtin_amdgcn_s_barrier();  // stage st+1 landed everywhere; stage st-1 fully read
        if (st + 1 + D < nst) issue(st + 1 + D);
        load_frags(st + 1, 0, na, nb);
      }
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int e = 0; e < 2; ++e) c[f][e] = wg_mfma(a[f], b[e], c[f][e]);
      if (do_bias) {
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const uint4 u = __builtin_bit_cast(uint4, a[f]);
          bs[f] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(wg_bf16x2, u.x), one2, bs[f], false);
          bs[f] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(wg_bf16x2, u.y), one2, bs[f], false);
          bs[f] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(wg_bf16x2, u.z), one2, bs[f], false);
          bs[f] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(wg_bf16x2, u.w), one2, bs[f], false);
        }
      }
#pragma unroll
      for (int f = 0; f < 4; ++f) a[f] = na[f];
#pragma unroll
      for (int e = 0; e < 2; ++e) b[e] = nb[e];
    }
  }

  wide_epilogue(p, split, n0, k0, wn, wk, lane, c, bs, do_bias);
}

// 256 x 256 tile (8 waves as above) on 64-token stages: two LDS stages of 64 KB (128 KB),
// one in flight while the other is computed, one barrier per stage.  At 64 tokens a stage is
// 32 MFMAs per wave (2048 matrix cycles per SIMD at two waves per SIMD) behind each barrier
// -- twice the 32-token ring's -- and the loads are addressed from per-lane row pointers
// advanced by one scalar product per stage.  Waves 4-7 (the second-dispatched half, the
// loser of every issue arbitration) run at priority 1 (MI355X_MICROARCH.md, two waves per
// SIMD, item 4).
//
// Template: STAGES LDS stages of BM tokens (<2, 64>: 128 KB, one stage in flight; <3, 48>:
// 144 KB, two in flight); FILL_ONLY = a probe with the MFMAs and the epilogue removed (output
// undefined; benchmarks/bench_wgrad.py --variants 10,11 times the operand fill alone).
template <int STAGES, int BM, bool FILL_ONLY>
__global__ __launch_bounds__(kWwThreads, 1) void wgrad_wide2_kernel(WgradArgs p) {
  constexpr int TH = BM * kWgRowBytes;   // BM rows x 128 columns
  constexpr int TB = 2 * TH;             // per operand tile
  constexpr int SB = 2 * TB;             // per stage
  constexpr int IPW = BM / 16;           // 1 KB LDS-DMA wave-instructions per wave per operand tile
  constexpr int PER = 2 * IPW;           // LDS-DMA instructions per lane per stage
  constexpr int QR = BM / 4;             // wave-instructions per operand half
  constexpr int KS = BM / 16;            // k-steps per stage
  constexpr int D = STAGES - 1;          // stages in flight beyond the one being computed
  static_assert(BM % 16 == 0 && STAGES * SB <= 160 * 1024, "LDS ring");
  __shared__ __attribute__((aligned(16))) uint8_t smem[STAGES * SB];
  typedef __attribute__((address_space(3))) void lds_void;

  int bid = blockIdx.x;
  if (p.remap) bid = (bid & 7) * int(gridDim.x >> 3) + (bid >> 3);
  const int split = p.split_major ? bid / p.tiles_total : bid % p.S;
  const int tile = p.split_major ? bid - split * p.tiles_total : bid / p.S;
  const int n0 = (tile / p.tiles_k) * kWwTile;
  const int k0 = (tile % p.tiles_k) * kWwTile;
  const int mb = split * p.m_split;
  const int me = min(p.M, mb + p.m_split);
  const int nst = me > mb ? (me - mb + BM - 1) / BM : 0;
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wn = wave >> 2, wk = wave & 3;
  const bool do_bias = __builtin_amdgcn_readfirstlane(p.bias && k0 == 0 && wk == 0);
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);

  // LDS-DMA source rows of stage 0: instruction i of this wave fills rows 4 rq .. 4 rq + 3 of
  // column half ``half``; lane (lr, slot) row 4 rq + lr, swizzled 16-byte chunk
  const int lr = lane >> 4, slot = lane & 15;
  const uint16_t* row_a[IPW];
  const uint16_t* row_b[IPW];
  int row_r[IPW], lds_off[IPW];
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int j = IPW * wave + i;          // 0 .. 2*QR-1
    const int half = j / QR, rq = j % QR;
    const int r = 4 * rq + lr;
    const int ch = slot ^ (((r & 3) << 2) | ((r >> 2) & 3));
    row_r[i] = r;
    lds_off[i] = half * TH + 1024 * rq;
    row_a[i] = p.dy + int64_t(mb + r) * p.ldy + min(n0 + half * 128 + ch * 8, p.N - 8);
    row_b[i] = p.x + int64_t(mb + r) * p.ldx + min(k0 + half * 128 + ch * 8, p.K - 8);
  }
  auto issue = [&](int st) {
    uint8_t* A = smem + (st % STAGES) * SB;
    uint8_t* B = A + TB;
    const int m_base = mb + st * BM;
    const int64_t adv_a = int64_t(st * BM) * p.ldy, adv_b = int64_t(st * BM) * p.ldx;
    const bool full = m_base + BM <= me;  // wave-uniform
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const bool okm = full || m_base + row_r[i] < me;
      const uint16_t* ga = okm ? row_a[i] + adv_a : p.zero;
      const uint16_t* gb = okm ? row_b[i] + adv_b : p.zero;
      wg_dma16(ga, __builtin_amdgcn_readfirstlane(uint32_t(size_t((lds_void*)(A + lds_off[i])))));
      wg_dma16(gb, __builtin_amdgcn_readfirstlane(uint32_t(size_t((lds_void*)(B + lds_off[i])))));
    }
  };

  wg_f32x16 c[4][2];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int i = 0; i < 16; ++i) c[f][e][i] = 0.f;
  float bs[4] = {0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3, h = lane >> 5;
  const int bo = 8 * (pp & 1);
  const int r0 = 8 * h + q;
  const int cbase = 2 * (g & 1) + (pp >> 1);
  int oa[4][2], ob[2][2];
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    oa[f][0] = wn * TH + wg_swz(r0, cbase + 4 * f) + bo;
    oa[f][1] = wn * TH + wg_swz(r0 + 4, cbase + 4 * f) + bo;
  }
  const int kc = 8 * (wk & 1);
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    ob[e][0] = (wk >> 1) * TH + wg_swz(r0, kc + cbase + 4 * e) + bo;
    ob[e][1] = (wk >> 1) * TH + wg_swz(r0 + 4, kc + cbase + 4 * e) + bo;
  }
  typedef __bf16 wg_bf16x2 __attribute__((ext_vector_type(2)));
  const wg_bf16x2 one2 = {static_cast<__bf16>(1.0f), static_cast<__bf16>(1.0f)};
  auto load_frags = [&](const uint8_t* A, int kk, wg_bf16x8 (&fa)[4], wg_bf16x8 (&fb)[2]) {
    const uint8_t* Ak = A + 4096 * kk;
    const uint8_t* Bk = A + TB + 4096 * kk;
#pragma unroll
    for (int f = 0; f < 4; ++f) fa[f] = wg_frag_at(Ak, oa[f][0], oa[f][1]);
#pragma unroll
    for (int e = 0; e < 2; ++e) fb[e] = wg_frag_at(Bk, ob[e][0], ob[e][1]);
  };

#pragma unroll
  for (int s0 = 0; s0 < D; ++s0)
    if (s0 < nst) issue(s0);
  for (int st = 0; st < nst; ++st) {
    // this wave's DMAs of stage st landed (at most min(D - 1, nst - 1 - st) later stages
    // outstanding, PER instructions each)
    wg_wait_ahead<PER>(min(D - 1, nst - 1 - st));
    __builtin_amdgcn_s_barrier();   // everyone's landed; everyone finished reading stage st-1
    if (st + D < nst) issue(st + D);  // refills stage st-1's buffer while stage st is computed
    if constexpr (FILL_ONLY) continue;
    const uint8_t* A = smem + (st % STAGES) * SB;
    wg_bf16x8 a[4], b[2];
    load_frags(A, 0, a, b);
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      wg_bf16x8 na[4], nb[2];
      if (kk + 1 < KS) load_frags(A, kk + 1, na, nb);
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int e = 0; e < 2; ++e) c[f][e] = wg_mfma(b[e], a[f], c[f][e]);  // C^T tile: lane = n
      if (do_bias) {
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const uint4 u = __builtin_bit_cast(uint4, a[f]);
          bs[f] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(wg_bf16x2, u.x), one2, bs[f], false);
          bs[f] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(wg_bf16x2, u.y), one2, bs[f], false);
          bs[f] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(wg_bf16x2, u.z), one2, bs[f], false);
          bs[f] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(wg_bf16x2, u.w), one2, bs[f], false);
        }
      }
      if (kk + 1 < KS) {
#pragma unroll
        for (int f = 0; f < 4; ++f) a[f] = na[f];
#pragma unroll
        for (int e = 0; e < 2; ++e) b[e] = nb[e];
      }
    }
    // this stage's fragment reads are consumed before the next barrier releases its buffer
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (wave >= 4) __builtin_amdgcn_s_setprio(0);
  if constexpr (FILL_ONLY) return;
  wide_epilogue_t(p, split, n0, k0, wn, wk, lane, c, bs, do_bias);
}

// dW[n][k] (+)= sum_s ws[s][n][k]; db[n] (+)= sum_s wsb[s][n].  4 columns per thread (K % 8 == 0).
// OutT = uint16_t (bf16 gradient) or float (fp32 gradient).
__device__ __forceinline__ void wg_acc4(uint16_t* o, float4 s, int accumulate) {
  uint2* o2 = reinterpret_cast<uint2*>(o);
  if (accumulate) {
    const uint2 u = *o2;
    s.x += bf2f(u.x & 0xffff); s.y += bf2f(u.x >> 16); s.z += bf2f(u.y & 0xffff); s.w += bf2f(u.y >> 16);
  }
  uint2 r;
  r.x = uint32_t(f2bf(s.x)) | (uint32_t(f2bf(s.y)) << 16);
  r.y = uint32_t(f2bf(s.z)) | (uint32_t(f2bf(s.w)) << 16);
  *o2 = r;
}
__device__ __forceinline__ void wg_acc4(float* o, float4 s, int accumulate) {
  float4* o4 = reinterpret_cast<float4*>(o);
  if (accumulate) {
    const float4 u = *o4;
    s.x += u.x; s.y += u.y; s.z += u.z; s.w += u.w;
  }
  *o4 = s;
}
__device__ __forceinline__ float wg_ld(const uint16_t* o) { return bf2f(*o); }
__device__ __forceinline__ float wg_ld(const float* o) { return *o; }
__device__ __forceinline__ void wg_st(uint16_t* o, float v) { *o = f2bf(v); }
__device__ __forceinline__ void wg_st(float* o, float v) { *o = v; }

template <typename OutT>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ ws, int S, int N, int K,
                                                           OutT* __restrict__ dw, int64_t ldw,
                                                           OutT* __restrict__ db, int accumulate) {
  const int64_t NK = int64_t(N) * K;
  const int64_t n4 = NK >> 2;
  const int64_t total = n4 + (db != nullptr ? N : 0);
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += stride) {
    if (i < n4) {
      float4 s = reinterpret_cast<const float4*>(ws)[i];
      for (int sp = 1; sp < S; ++sp) {
        const float4 v = reinterpret_cast<const float4*>(ws + int64_t(sp) * NK)[i];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
      const int64_t e = i << 2;
      const int64_t row = e / K, col = e - row * K;
      wg_acc4(dw + row * ldw + col, s, accumulate);
    } else {
      const int64_t n = i - n4;
      const float* wsb = ws + int64_t(S) * NK;
      float s = 0.f;
      for (int sp = 0; sp < S; ++sp) s += wsb[int64_t(sp) * N + n];
      if (accumulate) s += wg_ld(db + n);
      wg_st(db + n, s);
    }
  }
}

template <typename OutT>
void wg_launch_reduce(const WgradArgs& a, int S, int N, int K, int64_t ldw, bool bias, hipStream_t s) {
  const int64_t work = (int64_t(N) * K) / 4 + (bias ? N : 0);
  hipLaunchKernelGGL((wgrad_reduce_kernel<OutT>), dim3(stream_grid(work)), dim3(256), 0, s, a.ws, S, N, K,
                     reinterpret_cast<OutT*>(a.dw), ldw, bias ? reinterpret_cast<OutT*>(a.db) : nullptr,
                     a.accumulate);
}

struct WgradPlan {
  int S, m_split, tiles_k, grid;
};

// Logical block order split-major (tiles of one split adjacent: ResNet-50 26.03 vs 26.26 ms,
// profiles/raw/r2_ab_wgrad_order.jsonl) and zero-buffer reads for chunks past N / K (23.47 vs
// 23.55 ms kernel time, profiles/r3/raw/ab_wgrad_zero_columns.txt) -- fixed since round 5 (the
// kernels keep the field so the other settings stay reachable from a test harness)
constexpr int kWgradSplitMajor = 1;
constexpr int kWgradZeroColumns = 1;

WgradPlan wgrad_plan(int M, int N, int K, int splits, int tile = kWgBN) {
  WgradPlan pl;
  const int tiles_n = (N + tile - 1) / tile;
  pl.tiles_k = (K + tile - 1) / tile;
  int S = std::max(1, splits);
  const int per = (M + S - 1) / S;
  pl.m_split = std::max(kWgBM, (per + kWgBM - 1) / kWgBM * kWgBM);
  pl.S = (M + pl.m_split - 1) / pl.m_split;  // no empty splits
  pl.grid = tiles_n * pl.tiles_k * pl.S;
  return pl;
}

}  // namespace

int64_t wgrad_workspace_floats(int M, int N, int K, int splits) {
  const WgradPlan pl = wgrad_plan(M, N, K, splits);
  return pl.S > 1 ? int64_t(pl.S) * (int64_t(N) * K + N) : 0;
}

void wgrad_gemm(uintptr_t dy, int64_t ldy, uintptr_t x, int64_t ldx, uintptr_t dw, int64_t ldw, uintptr_t db, int M,
                int N, int K, int splits, uintptr_t ws, bool accumulate, uintptr_t zero, int variant,
                int out_dt, uintptr_t stream) {
  VODA_CHECK(out_dt == kBF16 || out_dt == kF32, "wgrad: dW must be bf16 or fp32");
  VODA_CHECK(M > 0 && N >= 8 && K >= 8, "wgrad: empty problem");
  VODA_CHECK(N % 8 == 0 && K % 8 == 0, "wgrad: N and K must be multiples of 8");
  VODA_CHECK(ldy >= N && ldx >= K && ldw >= K, "wgrad: leading dimension too small");
  VODA_CHECK(ldy % 8 == 0 && ldx % 8 == 0 && ldw % 8 == 0, "wgrad: rows must be 16-byte aligned");
  VODA_CHECK(dy % 16 == 0 && x % 16 == 0 && dw % 16 == 0, "wgrad: operands must be 16-byte aligned");
  const bool wide = variant >= 6;
  const WgradPlan pl = wgrad_plan(M, N, K, splits, wide ? kWwTile : kWgBN);
  VODA_CHECK(pl.S == 1 || ws != 0, "wgrad: split-K needs a workspace");
  VODA_CHECK(variant == 0 || (zero != 0 && zero % 16 == 0), "wgrad: the LDS-DMA variant needs a zero buffer");
  WgradArgs a;
  a.dy = reinterpret_cast<const uint16_t*>(dy); a.ldy = ldy;
  a.x = reinterpret_cast<const uint16_t*>(x); a.ldx = ldx;
  a.dw = reinterpret_cast<uint16_t*>(dw); a.ldw = ldw;
  a.db = reinterpret_cast<uint16_t*>(db);
  a.ws = reinterpret_cast<float*>(ws);
  a.zero = reinterpret_cast<const uint16_t*>(zero);
  a.M = M; a.N = N; a.K = K; a.S = pl.S; a.m_split = pl.m_split; a.tiles_k = pl.tiles_k;
  a.col0 = 0; a.ws_ld = K;
  a.taps = 1; a.KW = 1; a.H = a.W = a.Ho = a.Wo = 1; a.cstride = 1; a.pad = 0; a.tiles_nk = 0;
  a.adv_n = a.adv_ho = a.adv_wo = 0;
  a.remap = (pl.grid % 8 == 0) ? 1 : 0;
  a.split_major = kWgradSplitMajor;
  a.zcol = kWgradZeroColumns;
  a.tiles_total = pl.grid / pl.S;
  a.accumulate = accumulate ? 1 : 0;
  a.bias = db != 0 ? 1 : 0;
  a.out_f32 = out_dt == kF32 ? 1 : 0;
  VODA_CHECK(!a.out_f32 || (ldw % 4 == 0 && dw % 16 == 0), "wgrad: fp32 dW rows must be 16-byte aligned");
  hipStream_t s = as_stream(stream);
  VODA_CHECK(variant >= 0 && variant <= 12, "wgrad: variant must be 0..12");
  if (variant == 0)
    hipLaunchKernelGGL(wgrad_kernel, dim3(unsigned(pl.grid)), dim3(kWgThreads), 0, s, a);
  else if (variant == 1)
    hipLaunchKernelGGL((wgrad_glds_kernel<4, 64>), dim3(unsigned(pl.grid)), dim3(kWgThreads), 0, s, a);
  else if (variant == 2)
    hipLaunchKernelGGL((wgrad_glds_kernel<2, 64>), dim3(unsigned(pl.grid)), dim3(kWgThreads), 0, s, a);
  else if (variant == 3)
    hipLaunchKernelGGL((wgrad_glds_kernel<3, 64>), dim3(unsigned(pl.grid)), dim3(kWgThreads), 0, s, a);
  else if (variant == 4)
    hipLaunchKernelGGL((wgrad_glds_kernel<4, 32>), dim3(unsigned(pl.grid)), dim3(kWgThreads), 0, s, a);
  else if (variant == 5)
    hipLaunchKernelGGL((wgrad_glds_kernel<5, 32>), dim3(unsigned(pl.grid)), dim3(kWgThreads), 0, s, a);
  else if (variant == 6)
    hipLaunchKernelGGL((wgrad_wide_kernel<4, 32>), dim3(unsigned(pl.grid)), dim3(kWwThreads), 0, s, a);
  else if (variant == 7)
    hipLaunchKernelGGL((wgrad_wide_kernel<5, 32>), dim3(unsigned(pl.grid)), dim3(kWwThreads), 0, s, a);
  else if (variant == 8)
    hipLaunchKernelGGL((wgrad_wide_kernel<3, 32>), dim3(unsigned(pl.grid)), dim3(kWwThreads), 0, s, a);
  else if (variant == 9)
    hipLaunchKernelGGL((wgrad_wide2_kernel<2, 64, false>), dim3(unsigned(pl.grid)), dim3(kWwThreads), 0, s, a);
  else if (variant == 10)
    hipLaunchKernelGGL((wgrad_wide2_kernel<3, 48, false>), dim3(unsigned(pl.grid)), dim3(kWwThreads), 0, s, a);
  else if (variant == 11)  // probe: operand fill of variant 9 alone (dW undefined)
    hipLaunchKernelGGL((wgrad_wide2_kernel<2, 64, true>), dim3(unsigned(pl.grid)), dim3(kWwThreads), 0, s, a);
  else  // 12, probe: operand fill of variant 10 alone
    hipLaunchKernelGGL((wgrad_wide2_kernel<3, 48, true>), dim3(unsigned(pl.grid)), dim3(kWwThreads), 0, s, a);
  check_launch();
  if (pl.S > 1) {
    if (a.out_f32)
      wg_launch_reduce<float>(a, pl.S, N, K, ldw, db != 0, s);
    else
      wg_launch_reduce<uint16_t>(a, pl.S, N, K, ldw, db != 0, s);
    check_launch();
  }
}

int64_t wgrad_conv_workspace_floats(int M, int Cout, int Cin, int taps, int splits) {
  const WgradPlan pl = wgrad_plan(M, Cout, Cin, splits);
  return pl.S > 1 ? int64_t(pl.S) * (int64_t(Cout) * Cin * taps + Cout) : 0;
}

// Convolution weight gradient dW[co][kh][kw][ci] (+)= sum_{img,ho,wo} dY[img,ho,wo][co] *
// X[img, ho*s+kh-pad, wo*s+kw-pad][ci] on NHWC activations and a channels_last weight
// ([Cout][KH][KW][Cin] in memory): one implicit GEMM per tap, all taps in one launch, X rows
// gathered by the LDS-DMA loader (zero rows outside the image).
void wgrad_conv(uintptr_t dy, uintptr_t x, uintptr_t dw, int Nimg, int H, int W, int Cin, int Ho, int Wo, int Cout,
                int KH, int KW, int stride, int pad, int splits, uintptr_t ws, bool accumulate, uintptr_t zero,
                int out_dt, uintptr_t stream) {
  VODA_CHECK(out_dt == kBF16 || out_dt == kF32, "wgrad_conv: dW must be bf16 or fp32");
  VODA_CHECK(Nimg > 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0 && KH > 0 && KW > 0 && stride > 0 && pad >= 0,
             "wgrad_conv: bad geometry");
  VODA_CHECK(Cin % 8 == 0 && Cout % 8 == 0 && Cin >= 8 && Cout >= 8, "wgrad_conv: channels must be multiples of 8");
  VODA_CHECK((Ho - 1) * stride - pad + KH - 1 < H + pad && (Wo - 1) * stride - pad + KW - 1 < W + pad,
             "wgrad_conv: output size inconsistent with the input");
  VODA_CHECK(dy % 16 == 0 && x % 16 == 0 && dw % 16 == 0 && zero != 0 && zero % 16 == 0,
             "wgrad_conv: operands must be 16-byte aligned");
  const int64_t M64 = int64_t(Nimg) * Ho * Wo;
  VODA_CHECK(M64 < (int64_t(1) << 31) && int64_t(Nimg) * H * W < (int64_t(1) << 31), "wgrad_conv: too many pixels");
  const int M = int(M64), taps = KH * KW;
  const WgradPlan pl = wgrad_plan(M, Cout, Cin, splits);
  VODA_CHECK(pl.S == 1 || ws != 0, "wgrad_conv: split-K needs a workspace");
  WgradArgs a;
  a.dy = reinterpret_cast<const uint16_t*>(dy); a.ldy = Cout;
  a.x = reinterpret_cast<const uint16_t*>(x); a.ldx = Cin;
  a.dw = reinterpret_cast<uint16_t*>(dw); a.ldw = int64_t(taps) * Cin;
  a.db = nullptr;
  a.ws = reinterpret_cast<float*>(ws);
  a.zero = reinterpret_cast<const uint16_t*>(zero);
  a.M = M; a.N = Cout; a.K = Cin; a.S = pl.S; a.m_split = pl.m_split; a.tiles_k = pl.tiles_k;
  a.col0 = 0; a.ws_ld = taps * Cin;
  a.taps = taps; a.KW = KW; a.H = H; a.W = W; a.Ho = Ho; a.Wo = Wo; a.cstride = stride; a.pad = pad;
  a.tiles_nk = pl.grid / pl.S;
  constexpr int BM = 64;  // tokens per stage of the kernel launched below
  a.adv_n = BM / (Ho * Wo);
  a.adv_ho = (BM % (Ho * Wo)) / Wo;
  a.adv_wo = (BM % (Ho * Wo)) % Wo;
  a.accumulate = accumulate ? 1 : 0;
  a.bias = 0;
  a.out_f32 = out_dt == kF32 ? 1 : 0;
  const int64_t grid = int64_t(pl.grid) * taps;
  a.remap = (grid % 8 == 0) ? 1 : 0;
  a.split_major = kWgradSplitMajor;
  a.zcol = kWgradZeroColumns;
  a.tiles_total = pl.grid / pl.S;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL((wgrad_glds_kernel<2, BM, true>), dim3(unsigned(grid)), dim3(kWgThreads), 0, s, a);
  check_launch();
  if (pl.S > 1) {
    const int Kt = taps * Cin;
    if (a.out_f32)
      wg_launch_reduce<float>(a, pl.S, Cout, Kt, a.ldw, false, s);
    else
      wg_launch_reduce<uint16_t>(a, pl.S, Cout, Kt, a.ldw, false, s);
    check_launch();
  }
}

}  // namespace voda
