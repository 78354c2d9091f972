// Fused multi-head attention (forward + backward) on CDNA4 MFMA for the short-sequence
// encoder/decoder workloads of the trace (BERT-base: T=128, head dim 64; reference
// Transformer: vendored Keras MultiHeadAttention, layers_tf25.py:421-463).
//
//   O = softmax(scale * Q K^T + mask) V      mask: key padding (-1e9, the reference's additive
//                                            mask), causal (-1e9), keys >= Tk (-inf)
//
// One workgroup = W waves (1, 2 or 4, from the row count: a T = 20 sequence of the reference
// NMT Transformer gets ONE wave, not a 128-row block that is 84 % padding) = 32 W rows of
// one (batch, head).  The other operand streams through LDS in tiles of 32 rows
// (flash-attention style, online softmax in the forward), so the sequence length is bounded
// only by ``kMaxT`` (BERT at seq 512) and the head dim by registers: D = 32 / 64 / 128 / 256
// (the reference Transformer's key_dim = 256).  All products are v_mfma_f32_32x32x16_bf16 tiles
// (lane l, r = l & 31, h = l >> 5: A[r][8h+j], B[8h+j][r]; C/D col = r,
// row = (reg&3) + 8*(reg>>2) + 4h), arranged so that no accumulator has to cross lanes:
//
//   forward (query on the lane):  S^T = K Q^T  -> online softmax is lane-local (+1 xor-32
//                                 shuffle) -> O^T += V^T P^T with P^T's registers used
//                                 directly as the B operand (guide §3 "accumulator tile as
//                                 the next MFMA's operand"; V^T staged transposed in LDS so
//                                 its permuted-k fragment is two 8-byte LDS reads).
//   dQ pass (query on the lane):  S^T, dP^T = V dO^T, dS^T = P^T (dP^T - delta),
//                                 dQ^T += K^T dS^T;  delta = rowsum(dO o O) is computed here
//                                 and written for the dK/dV pass.
//   dK/dV pass (key on the lane): S = Q K^T, dP = dO V^T, dV += P^T dO, dK += dS^T Q with
//                                 P / dS registers as A operands (Q^T, dO^T staged in LDS).
//
// Nothing is materialised in HBM except O, the log-sum-exp per row and delta per row; the
// q/k/v/o/dq/dk/dv tensors are addressed through (batch, head, row) strides, so packed
// [B, T, 3, H, D] projections are read and their gradients written in place.  For D = 256
// the dK/dV pass runs twice (dV, then dK) so each pass keeps only one 256-wide accumulator
// set (8 x 16 fp32 registers per lane) next to the two operand fragment sets.
#include "common.h"

#include <cstdlib>
#include "ops.h"

namespace voda {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kTile = 32;              // rows of the streamed operand per LDS stage
constexpr int kMaxT = 4096;            // max sequence length (host check)
constexpr float kMaskNeg = -1e9f;      // reference additive mask value
constexpr float kNegInf = -__builtin_huge_valf();

struct AttnArgs {
  const uint16_t* q; int64_t q_sb, q_sh, q_st;
  const uint16_t* k; int64_t k_sb, k_sh, k_st;
  const uint16_t* v; int64_t v_sb, v_sh, v_st;
  const uint16_t* o; int64_t o_sb, o_sh, o_st;     // forward output / backward input
  const uint16_t* dout; int64_t do_sb, do_sh, do_st;
  uint16_t* out; int64_t out_sb, out_sh, out_st;    // O (fwd) or dQ (bwd)
  uint16_t* dk; int64_t dk_sb, dk_sh, dk_st;
  uint16_t* dv; int64_t dv_sb, dv_sh, dv_st;
  float* lse;      // [B*H][Tq]
  float* delta;    // [B*H][Tq]
  const uint8_t* mask; int64_t mask_sb;             // [B][Tk], nonzero = attend (may be null)
  int B, H, Tq, Tk;
  float scale;
  int causal;
};

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// row of a C/D register inside a 32x32 tile
__device__ __forceinline__ int crow(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

__device__ __forceinline__ bf16x8 ld16(const uint16_t* p) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(p));
}
__device__ __forceinline__ bf16x8 zero_bf8() { return __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0)); }

// Fragment (k-step s) of accumulator registers x[8s .. 8s+7] as a bf16 MFMA operand.
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& x, int s) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = static_cast<__bf16>(x[8 * s + j]);
  return f;
}

// Transposed LDS images store row d's 32 keys rotated by 8 * ((d >> 3) & 3) (mod 32): the
// staging writes (8 lanes of a wave-instruction on rows 8 apart) then spread over 16 banks
// instead of one -- 16-way -> 4-way write conflicts -- and the fragment reads of lanes r and
// r + 16 (rows 16 apart) no longer share banks.  Groups of 4 keys stay contiguous.
__device__ __forceinline__ int trans_rot(int d) { return 8 * ((d >> 3) & 3); }

// Operand paired with an accumulator fragment: element j of lane half h must come from
// k-row 16s + 8(j>>2) + 4h + (j&3).  ``rowT`` points at transposed LDS row d (k contiguous,
// rotated by ``rot`` = trans_rot(d)).
__device__ __forceinline__ bf16x8 perm_frag(const uint16_t* rowT, int s, int h, int rot) {
  const uint2 lo = *reinterpret_cast<const uint2*>(rowT + ((16 * s + 4 * h + rot) & 31));
  const uint2 hi = *reinterpret_cast<const uint2*>(rowT + ((16 * s + 8 + 4 * h + rot) & 31));
  return __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
}

// Stage rows [t0, t0 + kTile) of a (b, h) slice (row stride st, D contiguous) into LDS
// row-major [kTile][D + PAD] and optionally transposed [D][kTile + PADT]; rows >= T are zero.
template <int D, bool ROWS, bool TRANS>
__device__ __forceinline__ void stage_tile(const uint16_t* __restrict__ g, int64_t st, int t0, int T, uint16_t* rows,
                                           int rstride, uint16_t* trans, int tstride) {
  constexpr int VPR = D / 8;  // 16-byte vectors per row
  for (int i = threadIdx.x; i < kTile * VPR; i += blockDim.x) {
    const int r = i / VPR, c = (i % VPR) * 8;
    uint4 u = make_uint4(0, 0, 0, 0);
    if (t0 + r < T) u = *reinterpret_cast<const uint4*>(g + int64_t(t0 + r) * st + c);
    if constexpr (ROWS) *reinterpret_cast<uint4*>(rows + r * rstride + c) = u;
    if constexpr (TRANS) {
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int d0 = c + 2 * k, d1 = d0 + 1;
        trans[d0 * tstride + ((r + trans_rot(d0)) & 31)] = uint16_t(w[k] & 0xffff);
        trans[d1 * tstride + ((r + trans_rot(d1)) & 31)] = uint16_t(w[k] >> 16);
      }
    }
  }
}

// Register-staged prefetch of one kTile-row tile (threads NT): the global loads of tile t + 1
// are issued right after tile t reached LDS, so they are in flight while tile t is computed,
// and land in LDS behind the next barrier.  PER = 16-byte vectors per thread per tile; used
// when PER <= 4 (head dim 64 at any workgroup size, 128 with >= 2 waves), else the kernels
// stage synchronously (stage_tile).  Out-of-range rows are clamped for the load and zeroed
// after it (no branch between the loads).
template <int D, int NT>
struct TileRegs {
  static constexpr int VPR = D / 8;
  static constexpr int NV = kTile * VPR;
  static constexpr int PER = (NV + NT - 1) / NT;
  uint4 v[PER];
  __device__ __forceinline__ void load(const uint16_t* __restrict__ g, int64_t st, int t0, int T) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = min(int(threadIdx.x) + j * NT, NV - 1);
      const int r = i / VPR, c = (i % VPR) * 8;
      v[j] = *reinterpret_cast<const uint4*>(g + int64_t(min(t0 + r, T - 1)) * st + c);
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = int(threadIdx.x) + j * NT;
      if (t0 + i / VPR >= T) v[j] = make_uint4(0, 0, 0, 0);
    }
  }
  template <bool ROWS, bool TRANS>
  __device__ __forceinline__ void store(uint16_t* rows, int rstride, uint16_t* trans, int tstride) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = int(threadIdx.x) + j * NT;
      if (NV % NT != 0 && i >= NV) break;
      const int r = i / VPR, c = (i % VPR) * 8;
      const uint4 u = v[j];
      if constexpr (ROWS) *reinterpret_cast<uint4*>(rows + r * rstride + c) = u;
      if constexpr (TRANS) {
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int d0 = c + 2 * k, d1 = d0 + 1;
          trans[d0 * tstride + ((r + trans_rot(d0)) & 31)] = uint16_t(w[k] & 0xffff);
          trans[d1 * tstride + ((r + trans_rot(d1)) & 31)] = uint16_t(w[k] >> 16);
        }
      }
    }
  }
};

// Mask codes of one 32-key tile, staged into LDS next to the K/V tile: 0 attend, 1 key
// padding (the reference's additive -1e9), 2 past Tk (-inf).  A lane needs 16 of the 32 keys
// (crow(i, h): four runs of 4 consecutive keys), i.e. four 4-byte LDS reads per tile instead
// of sixteen global byte loads on the softmax's critical path.
// ms[kTile] (a flag byte after the codes) = 1 when any key of the tile is masked, so an
// unmasked tile -- every tile of an unpadded batch -- skips the per-element mask work with one
// wave-uniform branch.  Wave 0 stages the codes (kTile <= 64 threads).
// The mask bytes are loaded one tile ahead, with the K/V tile (a load issued after the
// barrier and consumed before the next one put a full memory latency on every tile).
constexpr int kMaskBytes = kTile + 4;
struct MaskPF {
  uint32_t raw;  // mask byte of key kt + threadIdx.x (threads < kTile)
  __device__ __forceinline__ void load(const AttnArgs& a, const uint8_t* mrow, int kt) {
    raw = 1;
    if (mrow != nullptr && threadIdx.x < kTile) raw = mrow[min(kt + int(threadIdx.x), a.Tk - 1)];
  }
  __device__ __forceinline__ void store(const AttnArgs& a, int kt, uint8_t* ms) const {
    const int t = threadIdx.x;
    if (t < 64) {
      uint32_t code = 0;
      if (t < kTile) {
        code = kt + t >= a.Tk ? 2u : (raw == 0 ? 1u : 0u);
        ms[t] = uint8_t(code);
      }
      const uint64_t any = __ballot(code != 0);
      if (t == 0) ms[kTile] = any != 0 ? 1 : 0;
    }
  }
};
__device__ __forceinline__ bool tile_masked(const uint8_t* ms) {
  return __builtin_amdgcn_readfirstlane(uint32_t(ms[kTile])) != 0;
}
__device__ __forceinline__ void load_mask_words(const uint8_t* ms, int h, uint32_t (&mw)[4]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) mw[g] = *reinterpret_cast<const uint32_t*>(ms + 8 * g + 4 * h);
}
// additive mask of accumulator register i (key kt + crow(i, h)): -inf past Tk, -1e9 for key
// padding, else 0 -- two selects, no branch (a branchy form here compiled to ~50 exec-mask
// sequences per tile and made the softmax instruction-bound)
__device__ __forceinline__ float mask_code_add(const uint32_t (&mw)[4], int i) {
  const uint32_t code = (mw[i >> 2] >> (8 * (i & 3))) & 0xffu;
  const float pad = code != 0 ? kMaskNeg : 0.f;
  return code > 1 ? kNegInf : pad;
}
// (causal) a future key gets the reference's -1e9 unless it is already past Tk
__device__ __forceinline__ float causal_add(float add, int key, int query) {
  return (key > query && add == 0.f) ? kMaskNeg : add;
}

// Write a [32 x 32] tile held as (lane = row-of-output r, regs = 16 columns) -- i.e. an
// X^T accumulator whose lane is the output row -- into out[row][col0 + crow(reg)].
__device__ __forceinline__ void store_lane_rows(uint16_t* __restrict__ out, int64_t st, int row, int nrows, int col0,
                                                const f32x16& x, float mul, int h) {
  if (row >= nrows) return;
  uint16_t* p = out + int64_t(row) * st + col0;
#pragma unroll
  for (int g = 0; g < 4; ++g) {  // regs 4g..4g+3 = 4 consecutive columns 8g + 4h + 0..3
    const int c = 8 * g + 4 * h;
    uint2 u;
    u.x = uint32_t(f2bf(x[4 * g] * mul)) | (uint32_t(f2bf(x[4 * g + 1] * mul)) << 16);
    u.y = uint32_t(f2bf(x[4 * g + 2] * mul)) | (uint32_t(f2bf(x[4 * g + 3] * mul)) << 16);
    *reinterpret_cast<uint2*>(p + c) = u;
  }
}

// ======================================================================== forward
template <int D, int W>
__global__ __launch_bounds__(64 * W) void attn_fwd_kernel(AttnArgs a) {
  constexpr int KS = D / 16;           // k-steps over the head dim
  constexpr int DT = D / 32;           // 32-wide output tiles over the head dim
  constexpr int RS = D + 8;            // LDS row stride (elements)
  constexpr int TS = kTile + 8;        // transposed row stride
  // DIRECT (head dim >= 128 without the register prefetch, e.g. the NMT's D = 256 at T = 20):
  // the row-operand fragments come straight from global / L2 instead of an LDS image, which
  // cuts the workgroup's LDS from ~37 KB to ~20 KB (one-wave workgroups: LDS sets occupancy)
  constexpr bool DIRECT = TileRegs<D, 64 * W>::PER > 4 && D >= 128;
  __shared__ __attribute__((aligned(16))) uint16_t Ks[DIRECT ? 8 : kTile * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Vt[D * TS];
  __shared__ __attribute__((aligned(16))) uint8_t Ms[kMaskBytes];

  const int bh = blockIdx.y, b = bh / a.H, hh = bh % a.H;
  const uint16_t* kb = a.k + b * a.k_sb + hh * a.k_sh;
  const uint16_t* vb = a.v + b * a.v_sb + hh * a.v_sh;

  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, w = threadIdx.x >> 6;
  const int q = blockIdx.x * (32 * W) + w * 32 + r;  // this lane's query
  const int q_lo = __builtin_amdgcn_readfirstlane(blockIdx.x * (32 * W) + w * 32);  // the wave's first query
  const uint16_t* qrow = a.q + b * a.q_sb + hh * a.q_sh + int64_t(q) * a.q_st;
  bf16x8 qf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) qf[s] = q < a.Tq ? ld16(qrow + 16 * s + 8 * h) : zero_bf8();
  const uint8_t* mrow = a.mask != nullptr ? a.mask + b * a.mask_sb : nullptr;

  f32x16 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = zero16();
  float m = -1e30f, l = 0.f;
  using Regs = TileRegs<D, 64 * W>;
  constexpr bool PF = Regs::PER <= 4;
  Regs kr, vr;
  MaskPF mp;
  mp.load(a, mrow, 0);
  if constexpr (PF) {
    kr.load(kb, a.k_st, 0, a.Tk);
    vr.load(vb, a.v_st, 0, a.Tk);
  }
  for (int kt = 0; kt < a.Tk; kt += kTile) {
    __syncthreads();  // every wave is done with the previous tile
    if constexpr (PF) {
      kr.template store<true, false>(Ks, RS, nullptr, 0);
      vr.template store<false, true>(nullptr, 0, Vt, TS);
    } else {
      if constexpr (!DIRECT) stage_tile<D, true, false>(kb, a.k_st, kt, a.Tk, Ks, RS, nullptr, 0);
      stage_tile<D, false, true>(vb, a.v_st, kt, a.Tk, nullptr, 0, Vt, TS);
    }
    mp.store(a, kt, Ms);
    __syncthreads();
    if (kt + kTile < a.Tk) {  // next tile's loads overlap this tile's compute
      mp.load(a, mrow, kt + kTile);
      if constexpr (PF) {
        kr.load(kb, a.k_st, kt + kTile, a.Tk);
        vr.load(vb, a.v_st, kt + kTile, a.Tk);
      }
    }
    f32x16 s_acc = zero16();
    if constexpr (DIRECT) {
      const bool kv = kt + r < a.Tk;
      const uint16_t* krow = kb + int64_t(kt + r) * a.k_st + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) s_acc = mfma(kv ? ld16(krow + 16 * s) : zero_bf8(), qf[s], s_acc);
    } else {
#pragma unroll
      for (int s = 0; s < KS; ++s) s_acc = mfma(ld16(Ks + r * RS + 16 * s + 8 * h), qf[s], s_acc);
    }
    // wave-uniform: per-element mask work only on tiles with a masked key or a future key
    if (tile_masked(Ms) || (a.causal && kt + kTile - 1 > q_lo)) {
      uint32_t mw[4];
      load_mask_words(Ms, h, mw);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float add = mask_code_add(mw, i);
        if (a.causal) add = causal_add(add, kt + crow(i, h), q);
        s_acc[i] = s_acc[i] * a.scale + add;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) s_acc[i] *= a.scale;
    }
    float tmax = -1e30f;
#pragma unroll
    for (int i = 0; i < 16; ++i) tmax = fmaxf(tmax, s_acc[i]);
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mn = fmaxf(m, tmax);
    const float alpha = __expf(m - mn);
    float psum = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = __expf(s_acc[i] - mn);
      s_acc[i] = p;
      psum += p;
    }
    psum += __shfl_xor(psum, 32, 64);
    l = l * alpha + psum;
    m = mn;
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) o[t][i] *= alpha;
    const bf16x8 p0 = acc_frag(s_acc, 0), p1 = acc_frag(s_acc, 1);
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const uint16_t* vrow = Vt + (32 * t + r) * TS;
      o[t] = mfma(perm_frag(vrow, 0, h, trans_rot(r)), p0, o[t]);
      o[t] = mfma(perm_frag(vrow, 1, h, trans_rot(r)), p1, o[t]);
    }
  }
  const float inv = 1.f / l;
  uint16_t* obase = a.out + b * a.out_sb + hh * a.out_sh;
#pragma unroll
  for (int t = 0; t < DT; ++t) store_lane_rows(obase, a.out_st, q, a.Tq, 32 * t, o[t], inv, h);
  if (h == 0 && q < a.Tq) a.lse[int64_t(bh) * a.Tq + q] = m + __logf(l);
}

// ======================================================================== backward: dQ (+ delta)
// D <= 64 with 4 waves (BERT-base): registers capped for 3 waves per SIMD (147 VGPRs, no
// spill), so all 768 workgroups of a layer are resident at once (25.3 -> 23.9 us per layer).
template <int D, int W>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu((D <= 64 && W == 4) ? 3 : 1)))
void attn_bwd_dq_kernel(AttnArgs a) {
  constexpr int KS = D / 16, DT = D / 32, RS = D + 8, TS = kTile + 8;
  constexpr bool DIRECT = TileRegs<D, 64 * W>::PER > 4 && D >= 128;  // as in the forward
  __shared__ __attribute__((aligned(16))) uint16_t Ks[DIRECT ? 8 : kTile * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[DIRECT ? 8 : kTile * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Kt[D * TS];
  __shared__ __attribute__((aligned(16))) uint8_t Ms[kMaskBytes];

  const int bh = blockIdx.y, b = bh / a.H, hh = bh % a.H;
  const uint16_t* kb = a.k + b * a.k_sb + hh * a.k_sh;
  const uint16_t* vb = a.v + b * a.v_sb + hh * a.v_sh;

  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, w = threadIdx.x >> 6;
  const int q = blockIdx.x * (32 * W) + w * 32 + r;
  const int q_lo = __builtin_amdgcn_readfirstlane(blockIdx.x * (32 * W) + w * 32);
  const bool qv = q < a.Tq;
  const uint16_t* qrow = a.q + b * a.q_sb + hh * a.q_sh + int64_t(q) * a.q_st;
  const uint16_t* dorow = a.dout + b * a.do_sb + hh * a.do_sh + int64_t(q) * a.do_st;
  const uint16_t* orow = a.o + b * a.o_sb + hh * a.o_sh + int64_t(q) * a.o_st;
  bf16x8 qf[KS], dof[KS];
  float dpart = 0.f;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    qf[s] = qv ? ld16(qrow + 16 * s + 8 * h) : zero_bf8();
    dof[s] = qv ? ld16(dorow + 16 * s + 8 * h) : zero_bf8();
    const bf16x8 of = qv ? ld16(orow + 16 * s + 8 * h) : zero_bf8();
#pragma unroll
    for (int j = 0; j < 8; ++j) dpart += float(dof[s][j]) * float(of[j]);
  }
  const float delta = dpart + __shfl_xor(dpart, 32, 64);
  // rows past Tq: lse = +inf makes every P of the row 0 without a per-element select
  const float lse = qv ? a.lse[int64_t(bh) * a.Tq + q] : __builtin_huge_valf();
  if (h == 0 && qv) a.delta[int64_t(bh) * a.Tq + q] = delta;
  const uint8_t* mrow = a.mask != nullptr ? a.mask + b * a.mask_sb : nullptr;

  f32x16 dq[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) dq[t] = zero16();
  using Regs = TileRegs<D, 64 * W>;
  constexpr bool PF = Regs::PER <= 4;
  Regs kr, vr;
  MaskPF mp;
  mp.load(a, mrow, 0);
  if constexpr (PF) {
    kr.load(kb, a.k_st, 0, a.Tk);
    vr.load(vb, a.v_st, 0, a.Tk);
  }
  for (int kt = 0; kt < a.Tk; kt += kTile) {
    __syncthreads();
    if constexpr (PF) {
      kr.template store<true, true>(Ks, RS, Kt, TS);
      vr.template store<true, false>(Vs, RS, nullptr, 0);
    } else if constexpr (DIRECT) {
      stage_tile<D, false, true>(kb, a.k_st, kt, a.Tk, nullptr, 0, Kt, TS);  // K^T only
    } else {
      stage_tile<D, true, true>(kb, a.k_st, kt, a.Tk, Ks, RS, Kt, TS);
      stage_tile<D, true, false>(vb, a.v_st, kt, a.Tk, Vs, RS, nullptr, 0);
    }
    mp.store(a, kt, Ms);
    __syncthreads();
    if (kt + kTile < a.Tk) {
      mp.load(a, mrow, kt + kTile);
      if constexpr (PF) {
        kr.load(kb, a.k_st, kt + kTile, a.Tk);
        vr.load(vb, a.v_st, kt + kTile, a.Tk);
      }
    }
    f32x16 s_acc = zero16(), dp = zero16();
    if constexpr (DIRECT) {
      const bool kv = kt + r < a.Tk;
      const uint16_t* krow = kb + int64_t(kt + r) * a.k_st + 8 * h;
      const uint16_t* vrow = vb + int64_t(kt + r) * a.v_st + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        s_acc = mfma(kv ? ld16(krow + 16 * s) : zero_bf8(), qf[s], s_acc);
        dp = mfma(kv ? ld16(vrow + 16 * s) : zero_bf8(), dof[s], dp);
      }
    } else {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        s_acc = mfma(ld16(Ks + r * RS + 16 * s + 8 * h), qf[s], s_acc);
        dp = mfma(ld16(Vs + r * RS + 16 * s + 8 * h), dof[s], dp);
      }
    }
    if (tile_masked(Ms) || (a.causal && kt + kTile - 1 > q_lo)) {  // wave-uniform, as in the forward
      uint32_t mw[4];
      load_mask_words(Ms, h, mw);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float add = mask_code_add(mw, i);
        if (a.causal) add = causal_add(add, kt + crow(i, h), q);
        s_acc[i] = s_acc[i] * a.scale + add;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) s_acc[i] *= a.scale;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) s_acc[i] = __expf(s_acc[i] - lse) * (dp[i] - delta);  // dS^T
    const bf16x8 d0 = acc_frag(s_acc, 0), d1 = acc_frag(s_acc, 1);
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const uint16_t* krow = Kt + (32 * t + r) * TS;
      dq[t] = mfma(perm_frag(krow, 0, h, trans_rot(r)), d0, dq[t]);
      dq[t] = mfma(perm_frag(krow, 1, h, trans_rot(r)), d1, dq[t]);
    }
  }
  uint16_t* base = a.out + b * a.out_sb + hh * a.out_sh;
#pragma unroll
  for (int t = 0; t < DT; ++t) store_lane_rows(base, a.out_st, q, a.Tq, 32 * t, dq[t], a.scale, h);
}

// ======================================================================== backward: dK, dV
// MODE 0: dK and dV; 1: dV only; 2: dK only (D = 256 runs 1 then 2: one accumulator set each)
// (Capping this kernel at 3 waves per SIMD like the dQ pass spills the K / V fragments into
// the loop: 29.1 -> 33.4 us per BERT-base layer, so it keeps 2.)
template <int D, int W, int MODE>
__global__ __launch_bounds__(64 * W) void attn_bwd_dkv_kernel(AttnArgs a) {
  constexpr int KS = D / 16, DT = D / 32, RS = D + 8, TS = kTile + 8;
  constexpr bool DO_DV = MODE != 2, DO_DK = MODE != 1;
  constexpr bool DIRECT = TileRegs<D, 64 * W>::PER > 4 && D >= 128;  // as in the forward
  __shared__ __attribute__((aligned(16))) uint16_t Qs[DIRECT ? 8 : kTile * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Qt[DO_DK ? D * TS : 8];
  __shared__ __attribute__((aligned(16))) uint16_t Ds[(DO_DK && !DIRECT) ? kTile * RS : 8];
  __shared__ __attribute__((aligned(16))) uint16_t Dt[DO_DV ? D * TS : 8];
  __shared__ float lse_s[kTile], del_s[kTile];

  const int bh = blockIdx.y, b = bh / a.H, hh = bh % a.H;
  const uint16_t* qb = a.q + b * a.q_sb + hh * a.q_sh;
  const uint16_t* db = a.dout + b * a.do_sb + hh * a.do_sh;

  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, w = threadIdx.x >> 6;
  const int key = blockIdx.x * (32 * W) + w * 32 + r;
  const bool kv = key < a.Tk;
  const uint16_t* krow = a.k + b * a.k_sb + hh * a.k_sh + int64_t(key) * a.k_st;
  const uint16_t* vrow = a.v + b * a.v_sb + hh * a.v_sh + int64_t(key) * a.v_st;
  bf16x8 kf[KS], vf[DO_DK ? KS : 1];
#pragma unroll
  for (int s = 0; s < KS; ++s) kf[s] = kv ? ld16(krow + 16 * s + 8 * h) : zero_bf8();
  if constexpr (DO_DK) {
#pragma unroll
    for (int s = 0; s < KS; ++s) vf[s] = kv ? ld16(vrow + 16 * s + 8 * h) : zero_bf8();
  }
  const uint8_t* mrow = a.mask != nullptr ? a.mask + b * a.mask_sb : nullptr;
  // the key is the lane's: its additive mask is one constant (-inf past Tk, -1e9 padding)
  const float kadd = !kv ? kNegInf : ((mrow != nullptr && mrow[key] == 0) ? kMaskNeg : 0.f);
  const int key_hi = __builtin_amdgcn_readfirstlane(blockIdx.x * (32 * W) + w * 32 + 31);  // wave's last key

  f32x16 dk[DO_DK ? DT : 1], dv[DO_DV ? DT : 1];
  if constexpr (DO_DK) {
#pragma unroll
    for (int t = 0; t < DT; ++t) dk[t] = zero16();
  }
  if constexpr (DO_DV) {
#pragma unroll
    for (int t = 0; t < DT; ++t) dv[t] = zero16();
  }
  using Regs = TileRegs<D, 64 * W>;
  constexpr bool PF = Regs::PER <= 4;
  Regs qr, dr;
  float lse_r = 0.f, del_r = 0.f;  // row threadIdx.x of the prefetched tile (threads < kTile)
  auto load_rows = [&](int qt) {
    qr.load(qb, a.q_st, qt, a.Tq);
    dr.load(db, a.do_st, qt, a.Tq);
    const int i = min(int(threadIdx.x), kTile - 1);
    const bool ok = qt + i < a.Tq;
    const int64_t o = int64_t(bh) * a.Tq + min(qt + i, a.Tq - 1);
    lse_r = a.lse[o];
    del_r = a.delta[o];
    if (!ok) { lse_r = __builtin_huge_valf(); del_r = 0.f; }  // pad rows: P = 0
  };
  if constexpr (PF) load_rows(0);
  for (int qt = 0; qt < a.Tq; qt += kTile) {
    __syncthreads();
    if constexpr (PF) {
      qr.template store<true, DO_DK>(Qs, RS, Qt, TS);
      if constexpr (DO_DK) dr.template store<true, DO_DV>(Ds, RS, Dt, TS);
      else dr.template store<false, true>(nullptr, 0, Dt, TS);
      if (threadIdx.x < kTile) {
        lse_s[threadIdx.x] = lse_r;
        del_s[threadIdx.x] = del_r;
      }
    } else if constexpr (DIRECT) {  // transposed images only: row fragments come from global
      if constexpr (DO_DK) stage_tile<D, false, true>(qb, a.q_st, qt, a.Tq, nullptr, 0, Qt, TS);
      if constexpr (DO_DV) stage_tile<D, false, true>(db, a.do_st, qt, a.Tq, nullptr, 0, Dt, TS);
      for (int i = threadIdx.x; i < kTile; i += blockDim.x) {
        const bool ok = qt + i < a.Tq;
        lse_s[i] = ok ? a.lse[int64_t(bh) * a.Tq + qt + i] : __builtin_huge_valf();  // pad rows: P = 0
        del_s[i] = ok ? a.delta[int64_t(bh) * a.Tq + qt + i] : 0.f;
      }
    } else {
      stage_tile<D, true, DO_DK>(qb, a.q_st, qt, a.Tq, Qs, RS, Qt, TS);
      if constexpr (DO_DK) stage_tile<D, true, DO_DV>(db, a.do_st, qt, a.Tq, Ds, RS, Dt, TS);
      else stage_tile<D, false, true>(db, a.do_st, qt, a.Tq, nullptr, 0, Dt, TS);
      for (int i = threadIdx.x; i < kTile; i += blockDim.x) {
        const bool ok = qt + i < a.Tq;
        lse_s[i] = ok ? a.lse[int64_t(bh) * a.Tq + qt + i] : __builtin_huge_valf();  // pad rows: P = 0
        del_s[i] = ok ? a.delta[int64_t(bh) * a.Tq + qt + i] : 0.f;
      }
    }
    __syncthreads();
    if constexpr (PF) {
      if (qt + kTile < a.Tq) load_rows(qt + kTile);  // in flight during this tile's compute
    }
    f32x16 s_acc = zero16(), dp = zero16();
    if constexpr (DIRECT) {
      const bool qv = qt + r < a.Tq;
      const uint16_t* qrow = qb + int64_t(qt + r) * a.q_st + 8 * h;
      const uint16_t* drow = db + int64_t(qt + r) * a.do_st + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        s_acc = mfma(qv ? ld16(qrow + 16 * s) : zero_bf8(), kf[s], s_acc);
        if constexpr (DO_DK) dp = mfma(qv ? ld16(drow + 16 * s) : zero_bf8(), vf[s], dp);
      }
    } else {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        s_acc = mfma(ld16(Qs + r * RS + 16 * s + 8 * h), kf[s], s_acc);             // S[query][key]
        if constexpr (DO_DK) dp = mfma(ld16(Ds + r * RS + 16 * s + 8 * h), vf[s], dp);  // dP[query][key]
      }
    }
    // causal: only tiles with a query before the wave's last key need the per-element test
    if (a.causal && qt < key_hi) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ql = crow(i, h);
        const float add = causal_add(kadd, key, qt + ql);
        s_acc[i] = __expf(s_acc[i] * a.scale + add - lse_s[ql]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) s_acc[i] = __expf(s_acc[i] * a.scale + kadd - lse_s[crow(i, h)]);
    }
    if constexpr (DO_DK) {
#pragma unroll
      for (int i = 0; i < 16; ++i) dp[i] = s_acc[i] * (dp[i] - del_s[crow(i, h)]);  // dS
    }
    // dV^T += dO^T P and dK^T += Q^T dS: the transposed products put the key on the lane
    // (P / dS registers as the B operand, as P^T in the forward), so the epilogue stores rows
    if constexpr (DO_DV) {
      const bf16x8 p0 = acc_frag(s_acc, 0), p1 = acc_frag(s_acc, 1);
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        const uint16_t* drow = Dt + (32 * t + r) * TS;  // dO^T row (d = 32t + r)
        dv[t] = mfma(perm_frag(drow, 0, h, trans_rot(r)), p0, dv[t]);
        dv[t] = mfma(perm_frag(drow, 1, h, trans_rot(r)), p1, dv[t]);
      }
    }
    if constexpr (DO_DK) {
      const bf16x8 g0 = acc_frag(dp, 0), g1 = acc_frag(dp, 1);
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        const uint16_t* qrow = Qt + (32 * t + r) * TS;  // Q^T row
        dk[t] = mfma(perm_frag(qrow, 0, h, trans_rot(r)), g0, dk[t]);
        dk[t] = mfma(perm_frag(qrow, 1, h, trans_rot(r)), g1, dk[t]);
      }
    }
  }
  // dv[t] / dk[t]: lane = key, regs = d (32t + crow): 8-byte row stores
  uint16_t* dkb = a.dk + b * a.dk_sb + hh * a.dk_sh;
  uint16_t* dvb = a.dv + b * a.dv_sb + hh * a.dv_sh;
#pragma unroll
  for (int t = 0; t < DT; ++t) {
    if constexpr (DO_DK) store_lane_rows(dkb, a.dk_st, key, a.Tk, 32 * t, dk[t], a.scale, h);
    if constexpr (DO_DV) store_lane_rows(dvb, a.dv_st, key, a.Tk, 32 * t, dv[t], 1.f, h);
  }
}

// ======================================================================== fused backward, T <= 128
// One workgroup per (batch, head) computes dQ, dK and dV from a single read of Q, K, V, O and
// dO (the two-pass form reads K / V in the dQ pass and Q / dO in the dK/dV pass, each tile
// staged behind its own barrier pair): 4 waves, wave w owns keys 32w..32w+31 in the dK/dV
// phase and queries 32w..32w+31 in the dQ phase.  Every operand lives in LDS as a plain row
// image [128 rows][64] (128-byte rows); the transposed operands of the dV / dK / dQ products
// come out of the same images through ds_read_b64_tr_b16, so nothing is staged transposed.
//   prologue : Q, dO rows -> images A, B; delta = rowsum(dO o O); lse; mask codes
//   dK / dV  : per 32-query tile  S = Q K^T, dP = dO V^T (key on the lane), P, dS,
//              dV^T += dO^T P, dK^T += Q^T dS
//   dQ       : K, V rows (held in registers since the prologue) -> images A, B, then per
//              32-key tile S^T = K Q^T, dP^T = V dO^T (query on the lane), dQ^T += K^T dS^T
// LDS 33 KB: up to 4 workgroups per CU by LDS, registers permitting.
constexpr int kFusedT = 128;                       // max Tq, Tk
constexpr int kFusedImg = kFusedT * 64 * 2;        // one row image, bytes

// byte offset of element (row, col) of a row image: 16-byte chunk col / 8 XOR-swizzled by the
// row so that the row-fragment reads (lane r: row r, one chunk), the transposed reads (4 rows
// x 4 chunks per 32 lanes) and the 16-byte staging writes are all conflict-free
__device__ __forceinline__ int fimg_off(int row, int col) {
  const int x = (row >> 1) & 7;
  const int sw = ((x & 1) << 2) | (x & 2) | ((x >> 2) & 1);
  return row * 128 + 16 * ((col >> 3) ^ sw) + 2 * (col & 7);
}
// 8 consecutive elements (row, 8c .. 8c + 7)
__device__ __forceinline__ bf16x8 fimg_row(const uint8_t* img, int row, int c8) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(img + fimg_off(row, 8 * c8)));
}
typedef __bf16 fimg_bf16x4 __attribute__((__vector_size__(4 * sizeof(__bf16))));
typedef __attribute__((address_space(3))) fimg_bf16x4 fimg_lds_bf16x4;
__device__ __forceinline__ uint2 fimg_tr(const uint8_t* img, int off) {
  const fimg_bf16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((fimg_lds_bf16x4*)(img + off));
  return __builtin_bit_cast(uint2, v);
}
// Operand whose k index runs over the ROWS of an image, in acc_frag's permuted order (k-step
// s): lane (r, h) gets column c0 + r, rows R0 + 16s + 4h + 0..3 and R0 + 16s + 8 + 4h + 0..3.
// ds_read_b64_tr_b16: lane 4qq + p of a 16-lane group names row qq of a 4-row block, columns
// 4p..4p+3 of the group's 16; lane i of the group receives column i.
__device__ __forceinline__ bf16x8 fimg_trfrag(const uint8_t* img, int R0, int c0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15, qq = i >> 2, p = i & 3;
  const int col = c0 + 16 * (g & 1) + 4 * p;
  const int row = R0 + 16 * s + 4 * (g >> 1) + qq;
  const uint2 lo = fimg_tr(img, fimg_off(row, col));
  const uint2 hi = fimg_tr(img, fimg_off(row + 8, col));
  return __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
}

// Registers capped for 3 waves per SIMD (168; the K / V fragments spill 72 B): all 768
// BERT-base workgroups resident at once, 39.2 -> 37.0 us per layer.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void attn_bwd_fused_kernel(AttnArgs a) {
  constexpr int D = 64, KS = 4, DT = 2;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * kFusedImg + 2 * kFusedT * 4 + kFusedT + 16];
  uint8_t* imgA = smem;                 // Q rows, then K rows
  uint8_t* imgB = smem + kFusedImg;     // dO rows, then V rows
  float* lse_s = reinterpret_cast<float*>(smem + 2 * kFusedImg);
  float* del_s = lse_s + kFusedT;
  uint8_t* Ms = reinterpret_cast<uint8_t*>(del_s + kFusedT);  // codes of keys 0..127 + 4 tile flags

  const int bh = blockIdx.x, b = bh / a.H, hh = bh % a.H;
  const int t = threadIdx.x, lane = t & 63, r = lane & 31, h = lane >> 5, w = t >> 6;
  const int own = 32 * w + r;  // this lane's key (dK/dV phase) and query (dQ phase)
  const int Tq = a.Tq, Tk = a.Tk;

  // ---- prologue: every global load issued before any is used
  const bool kvv = own < Tk, qv = own < Tq;
  const uint16_t* krow = a.k + b * a.k_sb + hh * a.k_sh + int64_t(min(own, Tk - 1)) * a.k_st;
  const uint16_t* vrow = a.v + b * a.v_sb + hh * a.v_sh + int64_t(min(own, Tk - 1)) * a.v_st;
  const uint16_t* qrow = a.q + b * a.q_sb + hh * a.q_sh + int64_t(min(own, Tq - 1)) * a.q_st;
  const uint16_t* dorow = a.dout + b * a.do_sb + hh * a.do_sh + int64_t(min(own, Tq - 1)) * a.do_st;
  const uint16_t* orow = a.o + b * a.o_sb + hh * a.o_sh + int64_t(min(own, Tq - 1)) * a.o_st;
  bf16x8 kf[KS], vf[KS], qf[KS], dof[KS], of[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    kf[s] = ld16(krow + 16 * s + 8 * h);
    vf[s] = ld16(vrow + 16 * s + 8 * h);
    qf[s] = ld16(qrow + 16 * s + 8 * h);
    dof[s] = ld16(dorow + 16 * s + 8 * h);
    of[s] = ld16(orow + 16 * s + 8 * h);
  }
  const float lse_own = a.lse[int64_t(bh) * Tq + min(own, Tq - 1)];
  const uint8_t* mrow = a.mask != nullptr ? a.mask + b * a.mask_sb : nullptr;
  const uint32_t mraw = (mrow != nullptr && t < kFusedT) ? mrow[min(t, Tk - 1)] : 1u;
#pragma unroll
  for (int s = 0; s < KS; ++s) {  // rows past T are zero
    if (!kvv) { kf[s] = zero_bf8(); vf[s] = zero_bf8(); }
    if (!qv) { qf[s] = zero_bf8(); dof[s] = zero_bf8(); of[s] = zero_bf8(); }
  }
  float dpart = 0.f;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    *reinterpret_cast<uint4*>(imgA + fimg_off(own, 16 * s + 8 * h)) = __builtin_bit_cast(uint4, qf[s]);
    *reinterpret_cast<uint4*>(imgB + fimg_off(own, 16 * s + 8 * h)) = __builtin_bit_cast(uint4, dof[s]);
#pragma unroll
    for (int j = 0; j < 8; ++j) dpart += float(dof[s][j]) * float(of[s][j]);
  }
  const float delta_own = dpart + __shfl_xor(dpart, 32, 64);
  if (h == 0) {
    lse_s[own] = qv ? lse_own : __builtin_huge_valf();  // rows past Tq: P = 0
    del_s[own] = qv ? delta_own : 0.f;
  }
  // mask code of key t (threads 0..127 = waves 0, 1) and one flag per 32-key tile
  const uint32_t code = t < kFusedT ? (t >= Tk ? 2u : (mraw == 0 ? 1u : 0u)) : 0u;
  if (t < kFusedT) Ms[t] = uint8_t(code);
  const uint64_t any = __ballot(code != 0);
  if (w < 2 && lane == 0) {
    Ms[kFusedT + 2 * w] = uint32_t(any) != 0 ? 1 : 0;
    Ms[kFusedT + 2 * w + 1] = uint32_t(any >> 32) != 0 ? 1 : 0;
  }
  __syncthreads();

  // ---- dK / dV: key = own on the lane
  const uint32_t kcode = Ms[own];
  const float kadd = kcode == 2 ? kNegInf : (kcode == 1 ? kMaskNeg : 0.f);
  const int key_hi = __builtin_amdgcn_readfirstlane(32 * w + 31);
  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int tt = 0; tt < DT; ++tt) { dk[tt] = zero16(); dv[tt] = zero16(); }
  const int nqt = (Tq + 31) / 32;
  for (int qt = 0; qt < nqt; ++qt) {
    const int R0 = 32 * qt;
    f32x16 sacc = zero16(), dp = zero16();
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      sacc = mfma(fimg_row(imgA, R0 + r, 2 * s + h), kf[s], sacc);   // S[query][key]
      dp = mfma(fimg_row(imgB, R0 + r, 2 * s + h), vf[s], dp);       // dP[query][key]
    }
    if (a.causal && R0 < key_hi) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ql = R0 + crow(i, h);
        sacc[i] = __expf(sacc[i] * a.scale + causal_add(kadd, own, ql) - lse_s[ql]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[i] = __expf(sacc[i] * a.scale + kadd - lse_s[R0 + crow(i, h)]);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) dp[i] = sacc[i] * (dp[i] - del_s[R0 + crow(i, h)]);  // dS
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 pf = acc_frag(sacc, s), gf = acc_frag(dp, s);
#pragma unroll
      for (int tt = 0; tt < DT; ++tt) {
        dv[tt] = mfma(fimg_trfrag(imgB, R0, 32 * tt, s, lane), pf, dv[tt]);  // dV^T[d][key] += dO^T P
        dk[tt] = mfma(fimg_trfrag(imgA, R0, 32 * tt, s, lane), gf, dk[tt]);  // dK^T[d][key] += Q^T dS
      }
    }
  }
  uint16_t* dkb = a.dk + b * a.dk_sb + hh * a.dk_sh;
  uint16_t* dvb = a.dv + b * a.dv_sb + hh * a.dv_sh;
#pragma unroll
  for (int tt = 0; tt < DT; ++tt) {
    store_lane_rows(dkb, a.dk_st, own, Tk, 32 * tt, dk[tt], a.scale, h);
    store_lane_rows(dvb, a.dv_st, own, Tk, 32 * tt, dv[tt], 1.f, h);
  }

  // ---- K, V rows replace Q, dO in the images; this lane's query fragments are read back
  // first (re-read rather than held through the dK/dV phase: 32 fewer live registers there)
  bf16x8 qf2[KS], dof2[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    qf2[s] = fimg_row(imgA, own, 2 * s + h);
    dof2[s] = fimg_row(imgB, own, 2 * s + h);
  }
  __syncthreads();  // every wave is done reading images A / B
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    *reinterpret_cast<uint4*>(imgA + fimg_off(own, 16 * s + 8 * h)) = __builtin_bit_cast(uint4, kf[s]);
    *reinterpret_cast<uint4*>(imgB + fimg_off(own, 16 * s + 8 * h)) = __builtin_bit_cast(uint4, vf[s]);
  }
  __syncthreads();

  // ---- dQ: query = own on the lane
  const float lse_q = qv ? lse_own : __builtin_huge_valf();
  const float del_q = qv ? delta_own : 0.f;
  const int q_lo = __builtin_amdgcn_readfirstlane(32 * w);
  f32x16 dq[DT];
#pragma unroll
  for (int tt = 0; tt < DT; ++tt) dq[tt] = zero16();
  const int nkt = (Tk + 31) / 32;
  for (int kt = 0; kt < nkt; ++kt) {
    const int R0 = 32 * kt;
    f32x16 st = zero16(), dpt = zero16();
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      st = mfma(fimg_row(imgA, R0 + r, 2 * s + h), qf2[s], st);     // S^T[key][query]
      dpt = mfma(fimg_row(imgB, R0 + r, 2 * s + h), dof2[s], dpt);  // dP^T[key][query]
    }
    const bool tile_mask = __builtin_amdgcn_readfirstlane(uint32_t(Ms[kFusedT + kt])) != 0;
    if (tile_mask || (a.causal && R0 + 31 > q_lo)) {
      uint32_t mw[4];
      load_mask_words(Ms + R0, h, mw);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float add = mask_code_add(mw, i);
        if (a.causal) add = causal_add(add, R0 + crow(i, h), own);
        st[i] = st[i] * a.scale + add;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) st[i] *= a.scale;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) st[i] = __expf(st[i] - lse_q) * (dpt[i] - del_q);  // dS^T
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 gf = acc_frag(st, s);
#pragma unroll
      for (int tt = 0; tt < DT; ++tt) dq[tt] = mfma(fimg_trfrag(imgA, R0, 32 * tt, s, lane), gf, dq[tt]);  // K^T dS^T
    }
  }
  uint16_t* dqb = a.out + b * a.out_sb + hh * a.out_sh;
#pragma unroll
  for (int tt = 0; tt < DT; ++tt) store_lane_rows(dqb, a.out_st, own, Tq, 32 * tt, dq[tt], a.scale, h);
  if (h == 0 && qv) a.delta[int64_t(bh) * Tq + own] = delta_own;
}

// ======================================================================== resident forward, T <= 128
// Same geometry as the fused backward: one workgroup per (batch, head), wave w owns queries
// 32w..32w+31, K and V rows staged ONCE into two row images (each lane writes the row it
// loaded), one barrier, then all key tiles from LDS.  Every score of a query row is in the
// lane's registers (4 tiles x 16), so the softmax is exact in two passes -- no running max,
// no rescaling of the output accumulators -- and V^T comes out of the V row image through
// ds_read_b64_tr_b16 (no transposed staging writes).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void attn_fwd_res_kernel(AttnArgs a) {
  constexpr int KS = 4, DT = 2, NKT = kFusedT / 32;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * kFusedImg + kFusedT + 16];
  uint8_t* imgK = smem;
  uint8_t* imgV = smem + kFusedImg;
  uint8_t* Ms = smem + 2 * kFusedImg;  // codes of keys 0..127 + 4 tile flags

  const int bh = blockIdx.x, b = bh / a.H, hh = bh % a.H;
  const int t = threadIdx.x, lane = t & 63, r = lane & 31, h = lane >> 5, w = t >> 6;
  const int own = 32 * w + r;  // this lane's query; also the K / V row it stages
  const int Tq = a.Tq, Tk = a.Tk;
  const bool kvv = own < Tk, qv = own < Tq;
  const uint16_t* krow = a.k + b * a.k_sb + hh * a.k_sh + int64_t(min(own, Tk - 1)) * a.k_st;
  const uint16_t* vrow = a.v + b * a.v_sb + hh * a.v_sh + int64_t(min(own, Tk - 1)) * a.v_st;
  const uint16_t* qrow = a.q + b * a.q_sb + hh * a.q_sh + int64_t(min(own, Tq - 1)) * a.q_st;
  bf16x8 kf[KS], vf[KS], qf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    kf[s] = ld16(krow + 16 * s + 8 * h);
    vf[s] = ld16(vrow + 16 * s + 8 * h);
    qf[s] = ld16(qrow + 16 * s + 8 * h);
  }
  const uint8_t* mrow = a.mask != nullptr ? a.mask + b * a.mask_sb : nullptr;
  const uint32_t mraw = (mrow != nullptr && t < kFusedT) ? mrow[min(t, Tk - 1)] : 1u;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const uint4 kz = kvv ? __builtin_bit_cast(uint4, kf[s]) : make_uint4(0, 0, 0, 0);
    const uint4 vz = kvv ? __builtin_bit_cast(uint4, vf[s]) : make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(imgK + fimg_off(own, 16 * s + 8 * h)) = kz;
    *reinterpret_cast<uint4*>(imgV + fimg_off(own, 16 * s + 8 * h)) = vz;
    if (!qv) qf[s] = zero_bf8();
  }
  const uint32_t code = t < kFusedT ? (t >= Tk ? 2u : (mraw == 0 ? 1u : 0u)) : 0u;
  if (t < kFusedT) Ms[t] = uint8_t(code);
  const uint64_t any = __ballot(code != 0);
  if (w < 2 && lane == 0) {
    Ms[kFusedT + 2 * w] = uint32_t(any) != 0 ? 1 : 0;
    Ms[kFusedT + 2 * w + 1] = uint32_t(any >> 32) != 0 ? 1 : 0;
  }
  __syncthreads();

  // ---- scores S^T[key][query] of every key tile (lane = query), masked and scaled
  const int nkt = (Tk + 31) / 32;
  const int q_lo = __builtin_amdgcn_readfirstlane(32 * w);
  f32x16 sc[NKT];
  float m = -1e30f;
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    sc[kt] = zero16();
    if (kt < nkt) {
      const int R0 = 32 * kt;
#pragma unroll
      for (int s = 0; s < KS; ++s) sc[kt] = mfma(fimg_row(imgK, R0 + r, 2 * s + h), qf[s], sc[kt]);
      const bool tile_mask = __builtin_amdgcn_readfirstlane(uint32_t(Ms[kFusedT + kt])) != 0;
      if (tile_mask || (a.causal && R0 + 31 > q_lo)) {
        uint32_t mw[4];
        load_mask_words(Ms + R0, h, mw);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float add = mask_code_add(mw, i);
          if (a.causal) add = causal_add(add, R0 + crow(i, h), own);
          sc[kt][i] = sc[kt][i] * a.scale + add;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) sc[kt][i] *= a.scale;
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) m = fmaxf(m, sc[kt][i]);
    }
  }
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  // ---- P = exp(S - max), row sums, O^T[d][query] += V^T P^T
  float l = 0.f;
  f32x16 o[DT];
#pragma unroll
  for (int tt = 0; tt < DT; ++tt) o[tt] = zero16();
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    if (kt < nkt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = __expf(sc[kt][i] - m);
        sc[kt][i] = p;
        l += p;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = acc_frag(sc[kt], s);
#pragma unroll
        for (int tt = 0; tt < DT; ++tt) o[tt] = mfma(fimg_trfrag(imgV, 32 * kt, 32 * tt, s, lane), pf, o[tt]);
      }
    }
  }
  l += __shfl_xor(l, 32, 64);
  const float inv = 1.f / l;
  uint16_t* obase = a.out + b * a.out_sb + hh * a.out_sh;
#pragma unroll
  for (int tt = 0; tt < DT; ++tt) store_lane_rows(obase, a.out_st, own, Tq, 32 * tt, o[tt], inv, h);
  if (h == 0 && qv) a.lse[int64_t(bh) * Tq + own] = m + __logf(l);
}

// T <= 128: the fused single-pass backward (round 3: 53.0 -> 37.0 us per BERT-base layer); the
// two-pass backward stays for longer sequences
bool attn_fused_bwd_enabled() { return true; }

template <typename F>
void dispatch_d(int D, F&& f) {
  if (D == 32) f(std::integral_constant<int, 32>{});
  else if (D == 64) f(std::integral_constant<int, 64>{});
  else if (D == 128) f(std::integral_constant<int, 128>{});
  else if (D == 256) f(std::integral_constant<int, 256>{});
  else throw std::invalid_argument("attention: unsupported head dim");
}

// waves per workgroup from the number of rows the workgroup's lanes own
template <typename F>
void dispatch_w(int rows, F&& f) {
  // at most 4 waves: smaller workgroups (more per (batch, head)) measured slower
  // (profiles/raw/r2_ab_attn_maxw.jsonl)
  if (rows <= 32) f(std::integral_constant<int, 1>{});
  else if (rows <= 64) f(std::integral_constant<int, 2>{});
  else f(std::integral_constant<int, 4>{});
}

AttnArgs make_args(const std::vector<int64_t>& t, int B, int H, int Tq, int Tk, float scale, bool causal) {
  // t = 8 groups of (ptr, sb, sh, st): q, k, v, o, dout, out, dk, dv; then lse, delta, mask, mask_sb
  AttnArgs a;
  auto P = [&](int g) { return reinterpret_cast<uint16_t*>(uintptr_t(t[4 * g])); };
  a.q = P(0); a.q_sb = t[1]; a.q_sh = t[2]; a.q_st = t[3];
  a.k = P(1); a.k_sb = t[5]; a.k_sh = t[6]; a.k_st = t[7];
  a.v = P(2); a.v_sb = t[9]; a.v_sh = t[10]; a.v_st = t[11];
  a.o = P(3); a.o_sb = t[13]; a.o_sh = t[14]; a.o_st = t[15];
  a.dout = P(4); a.do_sb = t[17]; a.do_sh = t[18]; a.do_st = t[19];
  a.out = P(5); a.out_sb = t[21]; a.out_sh = t[22]; a.out_st = t[23];
  a.dk = P(6); a.dk_sb = t[25]; a.dk_sh = t[26]; a.dk_st = t[27];
  a.dv = P(7); a.dv_sb = t[29]; a.dv_sh = t[30]; a.dv_st = t[31];
  a.lse = reinterpret_cast<float*>(uintptr_t(t[32]));
  a.delta = reinterpret_cast<float*>(uintptr_t(t[33]));
  a.mask = reinterpret_cast<const uint8_t*>(uintptr_t(t[34]));
  a.mask_sb = t[35];
  a.B = B; a.H = H; a.Tq = Tq; a.Tk = Tk; a.scale = scale; a.causal = causal ? 1 : 0;
  return a;
}

}  // namespace

bool attention_supported(int D, int Tq, int Tk, int dt) {
  // kF32: attention_f32.hip (same shapes, fp32 MFMA)
  return (dt == kBF16 || dt == kF32) && (D == 32 || D == 64 || D == 128 || D == 256) && Tq >= 1 && Tk >= 1 && Tq <= kMaxT &&
         Tk <= kMaxT;
}

void attention_fwd(const std::vector<int64_t>& t, int B, int H, int Tq, int Tk, int D, float scale, bool causal,
                   uintptr_t stream) {
  VODA_CHECK(t.size() == 36, "attention_fwd: bad argument vector");
  VODA_CHECK(attention_supported(D, Tq, Tk, kBF16), "attention_fwd: unsupported shape");
  VODA_CHECK(int64_t(B) * H <= 65535, "attention_fwd: B*H exceeds the grid's y dimension");
  const AttnArgs a = make_args(t, B, H, Tq, Tk, scale, causal);
  if (D == 64 && Tq <= kFusedT && Tk <= kFusedT) {  // K / V-resident forward (round 3: 17.0 -> 14.9 us)
    hipLaunchKernelGGL(attn_fwd_res_kernel, dim3(unsigned(B * H)), dim3(256), 0, as_stream(stream), a);
    check_launch();
    return;
  }
  dispatch_d(D, [&](auto dc) {
    dispatch_w(Tq, [&](auto wc) {
      constexpr int DD = decltype(dc)::value, WW = decltype(wc)::value;
      const dim3 grid((Tq + 32 * WW - 1) / (32 * WW), unsigned(B * H));
      hipLaunchKernelGGL((attn_fwd_kernel<DD, WW>), grid, dim3(64 * WW), 0, as_stream(stream), a);
    });
  });
  check_launch();
}

void attention_bwd(const std::vector<int64_t>& t, int B, int H, int Tq, int Tk, int D, float scale, bool causal,
                   uintptr_t stream) {
  VODA_CHECK(t.size() == 36, "attention_bwd: bad argument vector");
  VODA_CHECK(attention_supported(D, Tq, Tk, kBF16), "attention_bwd: unsupported shape");
  VODA_CHECK(int64_t(B) * H <= 65535, "attention_bwd: B*H exceeds the grid's y dimension");
  const AttnArgs a = make_args(t, B, H, Tq, Tk, scale, causal);
  hipStream_t s = as_stream(stream);
  if (D == 64 && Tq <= kFusedT && Tk <= kFusedT && attn_fused_bwd_enabled()) {
    hipLaunchKernelGGL(attn_bwd_fused_kernel, dim3(unsigned(B * H)), dim3(256), 0, s, a);
    check_launch();
    return;
  }
  dispatch_d(D, [&](auto dc) {
    constexpr int DD = decltype(dc)::value;
    dispatch_w(Tq, [&](auto wc) {
      constexpr int WW = decltype(wc)::value;
      hipLaunchKernelGGL((attn_bwd_dq_kernel<DD, WW>), dim3((Tq + 32 * WW - 1) / (32 * WW), unsigned(B * H)),
                         dim3(64 * WW), 0, s, a);
    });
    dispatch_w(Tk, [&](auto wc) {
      constexpr int WW = decltype(wc)::value;
      const dim3 grid((Tk + 32 * WW - 1) / (32 * WW), unsigned(B * H));
      if constexpr (DD == 256) {
        hipLaunchKernelGGL((attn_bwd_dkv_kernel<DD, WW, 1>), grid, dim3(64 * WW), 0, s, a);
        hipLaunchKernelGGL((attn_bwd_dkv_kernel<DD, WW, 2>), grid, dim3(64 * WW), 0, s, a);
      } else {
        hipLaunchKernelGGL((attn_bwd_dkv_kernel<DD, WW, 0>), grid, dim3(64 * WW), 0, s, a);
      }
    });
  });
  check_launch();
}

}  // namespace voda
