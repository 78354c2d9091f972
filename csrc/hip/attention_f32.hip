// Fused multi-head attention at the reference's precision (fp32 in, fp32 out) on CDNA4's
// fp32-input MFMA, v_mfma_f32_32x32x2_f32: exact f32 products with one rounding per FMA
// (no xf32 on gfx950), 64 cycles per instruction per SIMD = 1/16 of the bf16 rate.
// Same contract as attention.hip (the bf16 kernels): O = softmax(scale Q K^T + mask) V with
// key padding (-1e9 additive, the reference's mask: layers_tf25.py:421-463,
// advanced_activations_tf25.py:300-318), causal (-1e9) and keys >= Tk (-inf); the log-sum-exp
// per row is kept for the backward, which runs a dQ pass (query on the lane) and a dK/dV
// pass (key on the lane).  Tensors are addressed through (batch, head, row) strides, so the
// packed [B, T, 3, H, D] projection is read and its gradient written in place.
//
// Fragment maps of 32x32x2 f32 (lane l, r = l & 31, h = l >> 5): A[row r][k = h],
// B[k = h][col r], one f32 VGPR each; C/D col = r, row = (reg&3) + 8 (reg>>2) + 4h.
//   * head-dim reductions: k-step s covers d = 4 (s>>1) + 2h + (s&1), so every lane reads
//     its operands as float2 (row-major LDS tiles with a 2-float row pad: the 32 rows of a
//     ds_read_b64 lane group land on 32 distinct bank pairs);
//   * key / query reductions take the accumulator REGISTERS of the previous product as the
//     B operand in place: k-step s pairs key (or query) crow(s, h) -- the one lane half h
//     holds in register s -- with the matching A element read from LDS, so P, dS never move
//     between lanes.
// Register-resident row operands (Q / dO on the query lane, K / V on the key lane) are
// kept in VGPRs when the head dim allows it and otherwise re-read from global (L1/L2) per
// tile, so D = 256 (the reference Transformer's key_dim) does not spill.
#include "common.h"

#include <cstdlib>
#include "ops.h"

namespace voda {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kT = 32;                 // rows of the streamed operand per LDS tile
constexpr int kFbT = 128, kFbP = 132;  // fused backward: rows, dS / Kt pitch
constexpr int kMaxT32 = 4096;
constexpr float kMaskNeg = -1e9f;
constexpr float kNegInf = -__builtin_huge_valf();

struct AttnArgsF {
  const float* q; int64_t q_sb, q_sh, q_st;
  const float* k; int64_t k_sb, k_sh, k_st;
  const float* v; int64_t v_sb, v_sh, v_st;
  const float* o; int64_t o_sb, o_sh, o_st;
  const float* dout; int64_t do_sb, do_sh, do_st;
  float* out; int64_t out_sb, out_sh, out_st;     // O (fwd) or dQ (bwd)
  float* dk; int64_t dk_sb, dk_sh, dk_st;
  float* dv; int64_t dv_sb, dv_sh, dv_st;
  float* lse;
  float* delta;
  const uint8_t* mask; int64_t mask_sb;
  int B, H, Tq, Tk;
  float scale;
  int causal;
};

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

__device__ __forceinline__ int crow(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// Stage rows [t0, t0 + kT) of a (batch, head) slice into LDS [kT][RS] (rows >= T zero).
template <int D, int RS>
__device__ __forceinline__ void stage(const float* __restrict__ g, int64_t st, int t0, int T, float* lds) {
  constexpr int VPR = D / 4;  // float4 per row
  for (int i = threadIdx.x; i < kT * VPR; i += blockDim.x) {
    const int r = i / VPR, c = (i % VPR) * 4;
    float4 u = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t0 + r < T) u = *reinterpret_cast<const float4*>(g + int64_t(t0 + r) * st + c);
    float2* p = reinterpret_cast<float2*>(lds + r * RS + c);  // RS is even: 8-byte aligned
    p[0] = make_float2(u.x, u.y);
    p[1] = make_float2(u.z, u.w);
  }
}

// Register prefetch of one [kT][D] tile: the next tile's global loads are issued before the
// current tile's MFMAs and written to LDS after them (the synchronous stage() above exposes
// the global-load latency once per tile: 4 times per workgroup at T = 128).  Used when the
// tile is at most 4 float4 per thread (D <= 64 with 4 waves).
template <int D, int NT>
struct TileRegs {
  static constexpr int VPR = D / 4;
  static constexpr int N = (kT * VPR + NT - 1) / NT;
  static constexpr bool kOn = N <= 4;
  float4 v[kOn ? N : 1];
  __device__ __forceinline__ void load(const float* __restrict__ g, int64_t st, int t0, int T) {
    if constexpr (kOn) {
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const int i = threadIdx.x + j * NT;
        const int r = i / VPR, c = (i % VPR) * 4;
        v[j] = (i < kT * VPR && t0 + r < T) ? *reinterpret_cast<const float4*>(g + int64_t(t0 + r) * st + c)
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
  template <int RS>
  __device__ __forceinline__ void store(float* lds) const {
    if constexpr (kOn) {
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const int i = threadIdx.x + j * NT;
        if (i < kT * VPR) {
          const int r = i / VPR, c = (i % VPR) * 4;
          float2* p = reinterpret_cast<float2*>(lds + r * RS + c);
          p[0] = make_float2(v[j].x, v[j].y);
          p[1] = make_float2(v[j].z, v[j].w);
        }
      }
    }
  }
};

// mask codes of one tile: 0 attend, 1 key padding (-1e9), 2 past Tk (-inf)
__device__ __forceinline__ void stage_mask(const AttnArgsF& a, const uint8_t* mrow, int kt, uint8_t* ms) {
  const int t = threadIdx.x;
  if (t < kT) {
    const int key = kt + t;
    ms[t] = key >= a.Tk ? 2 : ((mrow != nullptr && mrow[key] == 0) ? 1 : 0);
  }
}

__device__ __forceinline__ float mask_add_code(const AttnArgsF& a, uint32_t code, int key, int query) {
  if (code == 2) return kNegInf;
  if (code == 1) return kMaskNeg;
  if (a.causal && key > query) return kMaskNeg;
  return 0.f;
}

__device__ __forceinline__ float mask_add(const AttnArgsF& a, const uint8_t* ms, int kl, int key, int query) {
  const uint8_t code = ms[kl];
  if (code == 2) return kNegInf;
  if (code == 1) return kMaskNeg;
  if (a.causal && key > query) return kMaskNeg;
  return 0.f;
}

// A row operand of the head-dim reduction, as float2 pairs (steps 2t, 2t + 1).
template <int D, bool REG>
struct RowFrag {
  float2 f[REG ? D / 4 : 1];
  const float* row;
  bool valid;
  __device__ __forceinline__ void init(const float* p, bool ok, int h) {
    row = p + 2 * h;
    valid = ok;
    if constexpr (REG) {
#pragma unroll
      for (int t = 0; t < D / 4; ++t) f[t] = ok ? *reinterpret_cast<const float2*>(row + 4 * t) : make_float2(0.f, 0.f);
    }
  }
  __device__ __forceinline__ float2 get(int t) const {
    if constexpr (REG) return f[t];
    return valid ? *reinterpret_cast<const float2*>(row + 4 * t) : make_float2(0.f, 0.f);
  }
};

// acc += A_lds(row r) . frag over the head dim: ``lds_row`` = row r of a row-major LDS tile
// [kT][RS], already offset by the lane half's 2h (k-step s reads d = 4 (s>>1) + 2h + (s&1))
template <int D, int RS, bool REG, bool SB = true>
__device__ __forceinline__ void dot_hd(f32x16& acc, const float* lds_row, const RowFrag<D, REG>& fr) {
  // LDS operand of step t + 1 read while the two MFMAs of step t issue (the scheduler would
  // otherwise put a wait on each read right before its MFMAs)
  float2 x = *reinterpret_cast<const float2*>(lds_row);
#pragma unroll
  for (int t = 0; t < D / 4; ++t) {
    float2 xn = x;
    if (t + 1 < D / 4) xn = *reinterpret_cast<const float2*>(lds_row + 4 * (t + 1));
    const float2 y = fr.get(t);
    if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
    acc = mfma(x.x, y.x, acc);
    acc = mfma(x.y, y.y, acc);
    if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
    x = xn;
  }
}

// A-operand column of a key / query reduction: the 16 LDS elements [crow(i, h)][col] this lane
// feeds to MFMA step i, all read before the first of the 16 MFMAs
__device__ __forceinline__ void col16(const float* lds, int RS, int col, int h, float (&v)[16]) {
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = lds[crow(i, h) * RS + col];
}

// 32 per-row values of a tile (lse, delta) at rows crow(i, h): four float4 LDS reads
__device__ __forceinline__ void rows16(const float* arr, int h, float (&v)[16]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float4 q = *reinterpret_cast<const float4*>(arr + 8 * j + 4 * h);
    v[4 * j] = q.x; v[4 * j + 1] = q.y; v[4 * j + 2] = q.z; v[4 * j + 3] = q.w;
  }
}

// mask codes of the tile's keys crow(i, h) (i = 0..15): the 32 code bytes are read once as
// two broadcast 16-byte LDS loads instead of 16 dependent byte loads
struct TileCodes {
  uint32_t w[4];  // word j: codes of keys 8j + 4h .. 8j + 4h + 3
  __device__ __forceinline__ void load(const uint8_t* ms, int h) {
    const uint4 a = *reinterpret_cast<const uint4*>(ms), b = *reinterpret_cast<const uint4*>(ms + 16);
    w[0] = h ? a.y : a.x;
    w[1] = h ? a.w : a.z;
    w[2] = h ? b.y : b.x;
    w[3] = h ? b.w : b.z;
  }
  __device__ __forceinline__ uint32_t code(int i) const { return (w[i >> 2] >> (8 * (i & 3))) & 0xff; }
};

// store a transposed accumulator (lane = output row, regs = 16 columns) as float4s
__device__ __forceinline__ void store_row(float* __restrict__ out, int64_t st, int row, int nrows, int col0,
                                          const f32x16& x, float mul, int h) {
  if (row >= nrows) return;
  float* p = out + int64_t(row) * st + col0;
#pragma unroll
  for (int g = 0; g < 4; ++g)
    *reinterpret_cast<float4*>(p + 8 * g + 4 * h) =
        make_float4(x[4 * g] * mul, x[4 * g + 1] * mul, x[4 * g + 2] * mul, x[4 * g + 3] * mul);
}

// ======================================================================== forward
template <int D, int W>
__global__ __launch_bounds__(64 * W) void attn_f32_fwd(AttnArgsF a) {
  constexpr int RS = D + 2, DT = D / 32;
  constexpr bool REG = D <= 128;
  __shared__ __attribute__((aligned(16))) float Ks[kT * RS];
  __shared__ __attribute__((aligned(16))) float Vs[kT * RS];
  __shared__ __attribute__((aligned(16))) uint8_t Ms[kT];
  const int bh = blockIdx.y, b = bh / a.H, hh = bh % a.H;
  const float* kb = a.k + b * a.k_sb + hh * a.k_sh;
  const float* vb = a.v + b * a.v_sb + hh * a.v_sh;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, w = threadIdx.x >> 6;
  const int q = blockIdx.x * (32 * W) + w * 32 + r;
  RowFrag<D, REG> qf;
  qf.init(a.q + b * a.q_sb + hh * a.q_sh + int64_t(min(q, a.Tq - 1)) * a.q_st, q < a.Tq, h);
  const uint8_t* mrow = a.mask != nullptr ? a.mask + b * a.mask_sb : nullptr;
  f32x16 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = zero16();
  float m = -1e30f, l = 0.f;
  // no register prefetch of the next K / V tile here: measured slower on BERT-base (fwd 48.0 ->
  // 51.2 us, dQ 75.9 -> 81.6 us per layer: the extra VGPRs cost a wave per SIMD; the variant was
  // removed in round 5); the dK/dV pass keeps it (109.3 -> 94.5 us)
  for (int kt = 0; kt < a.Tk; kt += kT) {
    __syncthreads();
    stage<D, RS>(kb, a.k_st, kt, a.Tk, Ks);
    stage<D, RS>(vb, a.v_st, kt, a.Tk, Vs);
    stage_mask(a, mrow, kt, Ms);
    __syncthreads();
    f32x16 s = zero16();
    dot_hd<D, RS, REG>(s, Ks + r * RS + 2 * h, qf);  // S^T[key r][query]: lane = query
    TileCodes tc;
    tc.load(Ms, h);
    float tmax = -1e30f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kl = crow(i, h);
      const float v = s[i] * a.scale + mask_add_code(a, tc.code(i), kt + kl, q);
      s[i] = v;
      tmax = fmaxf(tmax, v);
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mn = fmaxf(m, tmax);
    const float alpha = __expf(m - mn);
    float psum = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = __expf(s[i] - mn);
      s[i] = p;
      psum += p;
    }
    psum += __shfl_xor(psum, 32, 64);
    l = l * alpha + psum;
    m = mn;
#pragma unroll
    for (int t = 0; t < DT; ++t) {
#pragma unroll
      for (int i = 0; i < 16; ++i) o[t][i] *= alpha;
      // O^T[d][query] += V^T[d][key] P^T[key][query]: step i pairs key crow(i, h) (register i)
      float vc[16];
      col16(Vs, RS, 32 * t + r, h, vc);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 16; ++i) o[t] = mfma(vc[i], s[i], o[t]);
    }
  }
  const float inv = 1.f / l;
  float* ob = a.out + b * a.out_sb + hh * a.out_sh;
#pragma unroll
  for (int t = 0; t < DT; ++t) store_row(ob, a.out_st, q, a.Tq, 32 * t, o[t], inv, h);
  if (h == 0 && q < a.Tq) a.lse[int64_t(bh) * a.Tq + q] = m + __logf(l);
}

// ======================================================================== backward: dQ (+ delta)
template <int D, int W>
__global__ __launch_bounds__(64 * W) void attn_f32_bwd_dq(AttnArgsF a) {
  constexpr int RS = D + 2, DT = D / 32;
  constexpr bool REG = D <= 64;
  __shared__ __attribute__((aligned(16))) float Ks[kT * RS];
  __shared__ __attribute__((aligned(16))) float Vs[kT * RS];
  __shared__ __attribute__((aligned(16))) uint8_t Ms[kT];
  const int bh = blockIdx.y, b = bh / a.H, hh = bh % a.H;
  const float* kb = a.k + b * a.k_sb + hh * a.k_sh;
  const float* vb = a.v + b * a.v_sb + hh * a.v_sh;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, w = threadIdx.x >> 6;
  const int q = blockIdx.x * (32 * W) + w * 32 + r;
  const bool qv = q < a.Tq;
  const int qc = min(q, a.Tq - 1);
  RowFrag<D, REG> qf, df;
  qf.init(a.q + b * a.q_sb + hh * a.q_sh + int64_t(qc) * a.q_st, qv, h);
  df.init(a.dout + b * a.do_sb + hh * a.do_sh + int64_t(qc) * a.do_st, qv, h);
  // delta = rowsum(dO o O): this lane's half of the head dim + the other half's lane
  const float* orow = a.o + b * a.o_sb + hh * a.o_sh + int64_t(qc) * a.o_st + 2 * h;
  float dpart = 0.f;
  if (qv) {
    // fully unrolled: a runtime index into the register-resident dO fragment would move it
    // to scratch memory (it did: 88-152 bytes per lane of spills in every dQ pass)
#pragma unroll
    for (int t = 0; t < D / 4; ++t) {
      const float2 ov = *reinterpret_cast<const float2*>(orow + 4 * t);
      const float2 dv = df.get(t);
      dpart += dv.x * ov.x + dv.y * ov.y;
    }
  }
  const float delta = dpart + __shfl_xor(dpart, 32, 64);
  const float lse = qv ? a.lse[int64_t(bh) * a.Tq + q] : 0.f;
  if (h == 0 && qv) a.delta[int64_t(bh) * a.Tq + q] = delta;
  const uint8_t* mrow = a.mask != nullptr ? a.mask + b * a.mask_sb : nullptr;
  f32x16 dq[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) dq[t] = zero16();
  // no register prefetch of the next K / V tile here (see attn_f32_fwd)
  for (int kt = 0; kt < a.Tk; kt += kT) {
    __syncthreads();
    stage<D, RS>(kb, a.k_st, kt, a.Tk, Ks);
    stage<D, RS>(vb, a.v_st, kt, a.Tk, Vs);
    stage_mask(a, mrow, kt, Ms);
    __syncthreads();
    f32x16 s = zero16(), dp = zero16();
    dot_hd<D, RS, REG>(s, Ks + r * RS + 2 * h, qf);   // S^T
    dot_hd<D, RS, REG>(dp, Vs + r * RS + 2 * h, df);  // dP^T = V dO^T
    TileCodes tc;
    tc.load(Ms, h);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kl = crow(i, h);
      const float p = qv ? __expf(s[i] * a.scale + mask_add_code(a, tc.code(i), kt + kl, q) - lse) : 0.f;
      s[i] = p * (dp[i] - delta);  // dS^T
    }
    // dQ^T[d][query] += K^T[d][key] dS^T[key][query]
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      float kc[16];
      col16(Ks, RS, 32 * t + r, h, kc);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 16; ++i) dq[t] = mfma(kc[i], s[i], dq[t]);
    }
  }
  float* base = a.out + b * a.out_sb + hh * a.out_sh;
#pragma unroll
  for (int t = 0; t < DT; ++t) store_row(base, a.out_st, q, a.Tq, 32 * t, dq[t], a.scale, h);
}

// ======================================================================== backward: dK, dV
// MODE 0: both; 1: dV only; 2: dK only (large head dims: one accumulator set per pass)
// two waves per SIMD at D <= 64: unbounded, the pass took 226 VGPRs + 64 AGPRs (one wave per
// SIMD, three rounds of the 768 BERT workgroups); bounded, 256 registers and no spills -- except
// <64, 2> (68 bytes of scratch), which keeps one wave per SIMD
template <int D, int W, int MODE>
__global__ __launch_bounds__(64 * W, (D < 64 || (D == 64 && W != 2)) ? 2 : 1) void attn_f32_bwd_dkv(AttnArgsF a) {
  constexpr int RS = D + 2, DT = D / 32;
  constexpr bool REG = D <= 64;
  constexpr bool DO_DV = MODE != 2, DO_DK = MODE != 1;
  __shared__ __attribute__((aligned(16))) float Qs[kT * RS];
  __shared__ __attribute__((aligned(16))) float Ds[kT * RS];
  __shared__ __attribute__((aligned(16))) float lse_s[kT];
  __shared__ __attribute__((aligned(16))) float del_s[kT];
  const int bh = blockIdx.y, b = bh / a.H, hh = bh % a.H;
  const float* qb = a.q + b * a.q_sb + hh * a.q_sh;
  const float* db = a.dout + b * a.do_sb + hh * a.do_sh;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, w = threadIdx.x >> 6;
  const int key = blockIdx.x * (32 * W) + w * 32 + r;
  const bool kv = key < a.Tk;
  const int kc = min(key, a.Tk - 1);
  RowFrag<D, REG> kf, vf;
  kf.init(a.k + b * a.k_sb + hh * a.k_sh + int64_t(kc) * a.k_st, kv, h);
  if constexpr (DO_DK) vf.init(a.v + b * a.v_sb + hh * a.v_sh + int64_t(kc) * a.v_st, kv, h);
  const uint8_t* mrow = a.mask != nullptr ? a.mask + b * a.mask_sb : nullptr;
  const bool kmasked = kv && mrow != nullptr && mrow[key] == 0;
  f32x16 dk[DO_DK ? DT : 1], dv[DO_DV ? DT : 1];
#pragma unroll
  for (int t = 0; t < (DO_DK ? DT : 1); ++t) dk[t] = zero16();
#pragma unroll
  for (int t = 0; t < (DO_DV ? DT : 1); ++t) dv[t] = zero16();
  TileRegs<D, 64 * W> qr, dr;
  constexpr bool PF = TileRegs<D, 64 * W>::kOn;
  if constexpr (PF) {
    qr.load(qb, a.q_st, 0, a.Tq);
    dr.load(db, a.do_st, 0, a.Tq);
  }
  for (int qt = 0; qt < a.Tq; qt += kT) {
    __syncthreads();
    if constexpr (PF) {
      qr.template store<RS>(Qs);
      dr.template store<RS>(Ds);
    } else {
      stage<D, RS>(qb, a.q_st, qt, a.Tq, Qs);
      stage<D, RS>(db, a.do_st, qt, a.Tq, Ds);
    }
    for (int i = threadIdx.x; i < kT; i += blockDim.x) {
      const bool ok = qt + i < a.Tq;
      lse_s[i] = ok ? a.lse[int64_t(bh) * a.Tq + qt + i] : __builtin_huge_valf();  // pad rows: P = 0
      del_s[i] = ok ? a.delta[int64_t(bh) * a.Tq + qt + i] : 0.f;
    }
    __syncthreads();
    if constexpr (PF) {
      if (qt + kT < a.Tq) {
        qr.load(qb, a.q_st, qt + kT, a.Tq);
        dr.load(db, a.do_st, qt + kT, a.Tq);
      }
    }
    f32x16 s = zero16(), dp = zero16();
    dot_hd<D, RS, REG>(s, Qs + r * RS + 2 * h, kf);               // S[query r][key]: lane = key
    if constexpr (DO_DK) dot_hd<D, RS, REG>(dp, Ds + r * RS + 2 * h, vf);  // dP = dO V^T
    float ls[16], ds[16];
    rows16(lse_s, h, ls);
    if constexpr (DO_DK) rows16(del_s, h, ds);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ql = crow(i, h);
      float add = 0.f;
      if (!kv) add = kNegInf;
      else if (kmasked || (a.causal && key > qt + ql)) add = kMaskNeg;
      const float p = __expf(s[i] * a.scale + add - ls[i]);
      s[i] = p;
      if constexpr (DO_DK) dp[i] = p * (dp[i] - ds[i]);  // dS
    }
    // dV^T[d][key] += dO^T[d][q] P[q][key];  dK^T[d][key] += Q^T[d][q] dS[q][key]
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      float dc[16], qc[16];
      if constexpr (DO_DV) col16(Ds, RS, 32 * t + r, h, dc);
      if constexpr (DO_DK) col16(Qs, RS, 32 * t + r, h, qc);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if constexpr (DO_DV) dv[t] = mfma(dc[i], s[i], dv[t]);
        if constexpr (DO_DK) dk[t] = mfma(qc[i], dp[i], dk[t]);
      }
    }
  }
  // lane = key, registers = head-dim columns 32t + crow(reg, h)
  float* dkb = a.dk + b * a.dk_sb + hh * a.dk_sh;
  float* dvb = a.dv + b * a.dv_sb + hh * a.dv_sh;
#pragma unroll
  for (int t = 0; t < DT; ++t) {
    if constexpr (DO_DK) store_row(dkb, a.dk_st, key, a.Tk, 32 * t, dk[t], a.scale, h);
    if constexpr (DO_DV) store_row(dvb, a.dv_st, key, a.Tk, 32 * t, dv[t], 1.f, h);
  }
}

// ======================================================================== fused backward, T <= 128
// BERT-base's shape (self-attention, Tq = Tk <= 128, D = 64): one workgroup per (batch, head)
// computes dK, dV AND dQ, instead of the dQ pass and the dK/dV pass above, which both recompute
// S = Q K^T and dP = dO V^T (7 T x T x D products per (batch, head); here 5):
//   phase 0  Q and dO rows of the whole head in LDS, delta = rowsum(dO o O), lse;
//   phase 1  lane = key (wave w: keys 32 w ..): per 32-query tile S, dP from the LDS rows,
//            P and dS in registers, dV += dO^T P, dK += Q^T dS (as attn_f32_bwd_dkv), and dS
//            stored into an LDS image [query][key] (pitch 132: conflict-free row writes by
//            consecutive keys, 16-byte aligned reads);
//   phase 2  lane = query (wave w: queries 32 w ..): K staged transposed (Kt [d][key], pitch
//            132, in the Q rows' LDS) and dQ^T[d][q] = K^T[d][k] dS^T[k][q] with the permuted
//            key order of conv1x1_f32.hip (key 8 j + 4 h + s for MFMA s): one 16-byte read of
//            each operand feeds four MFMAs.
// LDS: Q 33.8 KB + dO 33.8 KB + dS 67.6 KB + lse / delta = 136 KB (one workgroup per CU).
// BERT-base fp32 (B 64, H 12): 157.3 -> ~127 us per layer for the backward
// (profiles/r5/rocprof_bert_fp32_fused_attn_bwd.md, profiles/r5/attn_fused_bwd_modes.json).
// The four query tiles of phase 1 are unrolled with no scheduling barriers, so the compiler
// overlaps one tile's softmax VALU work with the previous tile's MFMAs (one wave per SIMD: the
// barriered loop of the two-pass kernels measured ~10 us per layer slower here).
// Eight waves, two per SIMD (four waves, one per SIMD, ran 212 vs 205 us per forward + backward
// call, profiles/r5/attn_fused_bwd_modes.json): phase 1 splits each key tile's four query tiles
// between two waves (dK / dV partials summed through the dO rows' LDS), phase 2 gives each wave
// one (query tile, d tile) pair.
template <int D>
__global__ __launch_bounds__(512, 1) void attn_f32_bwd_fused_t128(AttnArgsF a) {
  constexpr bool SB = false;
  constexpr int NQ = 2;  // query tiles per wave in phase 1
  constexpr int RS = D + 2, DT = D / 32;
  static_assert(D == 64, "fused backward: head dim 64");
  static_assert(kFbT * RS >= D * kFbP, "Kt must fit in the Q rows' LDS");
  __shared__ __attribute__((aligned(16))) float Qs[kFbT * RS];
  __shared__ __attribute__((aligned(16))) float Ds[kFbT * RS];
  __shared__ __attribute__((aligned(16))) float dSs[kFbT * kFbP];
  __shared__ __attribute__((aligned(16))) float lse_s[kFbT];
  __shared__ __attribute__((aligned(16))) float del_s[kFbT];
  const int T = a.Tq;  // == Tk
  const int bh = blockIdx.y, b = bh / a.H, hh = bh % a.H;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, w = threadIdx.x >> 6;
  const float* qb = a.q + b * a.q_sb + hh * a.q_sh;
  const float* db = a.dout + b * a.do_sb + hh * a.do_sh;
  const float* kb = a.k + b * a.k_sb + hh * a.k_sh;

  // ---- phase 0: Q, dO rows (rows >= T zero), lse (+inf past T: P = 0), delta
#pragma unroll
  for (int t0 = 0; t0 < kFbT; t0 += kT) {
    stage<D, RS>(qb, a.q_st, t0, T, Qs + t0 * RS);
    stage<D, RS>(db, a.do_st, t0, T, Ds + t0 * RS);
  }
  for (int i = threadIdx.x; i < kFbT; i += blockDim.x)
    lse_s[i] = i < T ? a.lse[int64_t(bh) * T + i] : __builtin_huge_valf();
  __syncthreads();
  if (w < 4) {
    const int q = 32 * w + r;
    float dpart = 0.f;
    if (q < T) {
      const float* orow = a.o + b * a.o_sb + hh * a.o_sh + int64_t(q) * a.o_st + 2 * h;
#pragma unroll
      for (int t = 0; t < D / 4; ++t) {
        const float2 ov = *reinterpret_cast<const float2*>(orow + 4 * t);
        const float2 dv = *reinterpret_cast<const float2*>(Ds + q * RS + 2 * h + 4 * t);
        dpart += dv.x * ov.x + dv.y * ov.y;
      }
    }
    const float delta = dpart + __shfl_xor(dpart, 32, 64);
    if (h == 0) del_s[q] = delta;  // rows >= T: 0
  }
  __syncthreads();

  // ---- phase 1: lane = key
  {
    const int kt = w & 3, qh = w >> 2;
    const int key = 32 * kt + r;
    const bool kv = key < T;
    const int kc = min(key, T - 1);
    RowFrag<D, true> kf, vf;
    kf.init(kb + int64_t(kc) * a.k_st, kv, h);
    vf.init(a.v + b * a.v_sb + hh * a.v_sh + int64_t(kc) * a.v_st, kv, h);
    const uint8_t* mrow = a.mask != nullptr ? a.mask + b * a.mask_sb : nullptr;
    const bool kmasked = kv && mrow != nullptr && mrow[key] == 0;
    f32x16 dk[DT], dv[DT];
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      dk[t] = zero16();
      dv[t] = zero16();
    }
#pragma unroll
    for (int it = 0; it < NQ; ++it) {
      const int qt = (qh * NQ + it) * kT;
      if (qt >= T) break;
      const float* qt_rows = Qs + qt * RS;
      const float* dt_rows = Ds + qt * RS;
      f32x16 s = zero16(), dp = zero16();
      dot_hd<D, RS, true, SB>(s, qt_rows + r * RS + 2 * h, kf);   // S[query r][key]: lane = key
      dot_hd<D, RS, true, SB>(dp, dt_rows + r * RS + 2 * h, vf);  // dP = dO V^T
      float ls[16], ds[16];
      rows16(lse_s + qt, h, ls);
      rows16(del_s + qt, h, ds);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ql = crow(i, h);
        float add = 0.f;
        if (!kv) add = kNegInf;
        else if (kmasked || (a.causal && key > qt + ql)) add = kMaskNeg;
        const float p = __expf(s[i] * a.scale + add - ls[i]);
        s[i] = p;
        dp[i] = p * (dp[i] - ds[i]);  // dS
        dSs[(qt + ql) * kFbP + key] = dp[i];
      }
      // dV^T[d][key] += dO^T[d][q] P[q][key];  dK^T[d][key] += Q^T[d][q] dS[q][key]
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        float dc[16], qc[16];
        col16(dt_rows, RS, 32 * t + r, h, dc);
        col16(qt_rows, RS, 32 * t + r, h, qc);
        if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          dv[t] = mfma(dc[i], s[i], dv[t]);
          dk[t] = mfma(qc[i], dp[i], dk[t]);
        }
      }
    }
    float* dkb = a.dk + b * a.dk_sb + hh * a.dk_sh;
    float* dvb = a.dv + b * a.dv_sb + hh * a.dv_sh;
    {
      // waves 4..7 hand their partial sums to waves 0..3 of the same key tile through the dO
      // rows' LDS (4 key tiles x 2 d tiles x 16 registers x 64 lanes = 8192 floats <= 8448)
      static_assert(4 * DT * 16 * 64 <= kFbT * RS, "partials must fit in the dO rows");
      float* red = Ds + (kt * DT * 16) * 64 + lane;
      __syncthreads();  // every wave is done reading the dO rows
      if (qh == 1) {
#pragma unroll
        for (int t = 0; t < DT; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i) red[(t * 16 + i) * 64] = dk[t][i];
      }
      __syncthreads();
      if (qh == 0) {
#pragma unroll
        for (int t = 0; t < DT; ++t) {
#pragma unroll
          for (int i = 0; i < 16; ++i) dk[t][i] += red[(t * 16 + i) * 64];
          store_row(dkb, a.dk_st, key, T, 32 * t, dk[t], a.scale, h);
        }
      }
      __syncthreads();
      if (qh == 1) {
#pragma unroll
        for (int t = 0; t < DT; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i) red[(t * 16 + i) * 64] = dv[t][i];
      }
      __syncthreads();
      if (qh == 0) {
#pragma unroll
        for (int t = 0; t < DT; ++t) {
#pragma unroll
          for (int i = 0; i < 16; ++i) dv[t][i] += red[(t * 16 + i) * 64];
          store_row(dvb, a.dv_st, key, T, 32 * t, dv[t], 1.f, h);
        }
      }
    }
  }
  // dS rows / columns past T: keys >= T got P = 0 above, queries >= T have lse = +inf; rows of
  // the image past T were never written -- zero them for the phase-2 reads
  for (int i = threadIdx.x; i < (kFbT - T) * kFbP; i += blockDim.x) dSs[T * kFbP + i] = 0.f;
  __syncthreads();  // phase 1 done: Q rows free, dS complete

  // ---- phase 2: Kt[d][key] in the Q rows' LDS; lane = query
  float* Kt = Qs;
  for (int i = threadIdx.x; i < kFbT * (D / 4); i += blockDim.x) {
    const int key = i % kFbT, c4 = i / kFbT;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (key < T) v = *reinterpret_cast<const float4*>(kb + int64_t(key) * a.k_st + 4 * c4);
    Kt[(4 * c4 + 0) * kFbP + key] = v.x;
    Kt[(4 * c4 + 1) * kFbP + key] = v.y;
    Kt[(4 * c4 + 2) * kFbP + key] = v.z;
    Kt[(4 * c4 + 3) * kFbP + key] = v.w;
  }
  __syncthreads();
  {
    // wave w: queries 32 (w & 3).., d tile w >> 2
    constexpr int TT = 1;
    const int q = 32 * (w & 3) + r;
    const int t0 = w >> 2;
    f32x16 dq[TT];
#pragma unroll
    for (int t = 0; t < TT; ++t) dq[t] = zero16();
    const float* brow = dSs + q * kFbP + 4 * h;
#pragma unroll 4
    for (int j = 0; j < kFbT / 8; ++j) {
      const float4 bv = *reinterpret_cast<const float4*>(brow + 8 * j);
#pragma unroll
      for (int t = 0; t < TT; ++t) {
        const float4 av = *reinterpret_cast<const float4*>(Kt + (32 * (t0 + t) + r) * kFbP + 8 * j + 4 * h);
        dq[t] = mfma(av.x, bv.x, dq[t]);
        dq[t] = mfma(av.y, bv.y, dq[t]);
        dq[t] = mfma(av.z, bv.z, dq[t]);
        dq[t] = mfma(av.w, bv.w, dq[t]);
      }
    }
    float* base = a.out + b * a.out_sb + hh * a.out_sh;
#pragma unroll
    for (int t = 0; t < TT; ++t) store_row(base, a.out_st, q, T, 32 * (t0 + t), dq[t], a.scale, h);
  }
}

template <typename F>
void dispatch_d32(int D, F&& f) {
  if (D == 32) f(std::integral_constant<int, 32>{});
  else if (D == 64) f(std::integral_constant<int, 64>{});
  else if (D == 128) f(std::integral_constant<int, 128>{});
  else if (D == 256) f(std::integral_constant<int, 256>{});
  else throw std::invalid_argument("attention (fp32): unsupported head dim");
}

// waves per workgroup (32 rows each): enough for the rows, at most 4.  Removed in round 5 after
// their recorded losses: a resident-head T <= 128 forward (K / V staged once, 67.7 KB LDS, two
// workgroups per CU, unrolled key tiles: 58.3 vs 48.3 us per BERT-base layer,
// profiles/r5/attn_fused_bwd_modes.json); a register prefetch of the next K / V tile in the forward and dQ passes
// (fwd 48.0 -> 51.2 us, dQ 75.9 -> 81.6 us per BERT-base layer) and an LDS-DMA ring for the D = 64
// forward (53.5 vs 48.3 us: its swizzled addressing cost a wave per SIMD; profiles/r4/README.md,
// r4ad)
template <typename F>
void dispatch_w32(int rows, F&& f) {
  if (rows <= 32) f(std::integral_constant<int, 1>{});
  else if (rows <= 64) f(std::integral_constant<int, 2>{});
  else f(std::integral_constant<int, 4>{});
}

AttnArgsF make_args_f(const std::vector<int64_t>& t, int B, int H, int Tq, int Tk, float scale, bool causal) {
  AttnArgsF a;
  auto P = [&](int g) { return reinterpret_cast<float*>(uintptr_t(t[4 * g])); };
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

int g_fused_bwd_f32 = 1;  // attn_f32_set_fused_bwd: 0 = the two-pass backward (tests, A/B)

bool attn_f32_fused_bwd_ok(int D, int Tq, int Tk) {
  return g_fused_bwd_f32 != 0 && D == 64 && Tq == Tk && Tq >= 1 && Tq <= kFbT;
}

bool f32_shape_ok(int D, int Tq, int Tk) {
  return (D == 32 || D == 64 || D == 128 || D == 256) && Tq >= 1 && Tk >= 1 && Tq <= kMaxT32 && Tk <= kMaxT32;
}

}  // namespace

void attention_fwd_f32(const std::vector<int64_t>& t, int B, int H, int Tq, int Tk, int D, float scale, bool causal,
                       uintptr_t stream) {
  VODA_CHECK(t.size() == 36, "attention_fwd_f32: bad argument vector");
  VODA_CHECK(f32_shape_ok(D, Tq, Tk), "attention_fwd_f32: unsupported shape");
  VODA_CHECK(int64_t(B) * H <= 65535, "attention_fwd_f32: B*H exceeds the grid's y dimension");
  const AttnArgsF a = make_args_f(t, B, H, Tq, Tk, scale, causal);
  dispatch_d32(D, [&](auto dc) {
    dispatch_w32(Tq, [&](auto wc) {
      constexpr int DD = decltype(dc)::value, WW = decltype(wc)::value;
      hipLaunchKernelGGL((attn_f32_fwd<DD, WW>), dim3((Tq + 32 * WW - 1) / (32 * WW), unsigned(B * H)),
                           dim3(64 * WW), 0, as_stream(stream), a);
    });
  });
  check_launch();
}

// the fused T <= 128 backward (default on); false: the dQ + dK/dV passes (A/B and tests)
void attn_f32_set_fused_bwd(int mode) { g_fused_bwd_f32 = mode; }

void attention_bwd_f32(const std::vector<int64_t>& t, int B, int H, int Tq, int Tk, int D, float scale, bool causal,
                       uintptr_t stream) {
  VODA_CHECK(t.size() == 36, "attention_bwd_f32: bad argument vector");
  VODA_CHECK(f32_shape_ok(D, Tq, Tk), "attention_bwd_f32: unsupported shape");
  VODA_CHECK(int64_t(B) * H <= 65535, "attention_bwd_f32: B*H exceeds the grid's y dimension");
  const AttnArgsF a = make_args_f(t, B, H, Tq, Tk, scale, causal);
  hipStream_t s = as_stream(stream);
  if (attn_f32_fused_bwd_ok(D, Tq, Tk)) {
    hipLaunchKernelGGL((attn_f32_bwd_fused_t128<64>), dim3(1, unsigned(B * H)), dim3(512), 0, s, a);
    check_launch();
    return;
  }
  dispatch_d32(D, [&](auto dc) {
    constexpr int DD = decltype(dc)::value;
    dispatch_w32(Tq, [&](auto wc) {
      constexpr int WW = decltype(wc)::value;
      hipLaunchKernelGGL((attn_f32_bwd_dq<DD, WW>), dim3((Tq + 32 * WW - 1) / (32 * WW), unsigned(B * H)),
                           dim3(64 * WW), 0, s, a);
    });
    dispatch_w32(Tk, [&](auto wc) {
      constexpr int WW = decltype(wc)::value;
      const dim3 grid((Tk + 32 * WW - 1) / (32 * WW), unsigned(B * H));
      if constexpr (DD >= 128) {
        hipLaunchKernelGGL((attn_f32_bwd_dkv<DD, WW, 1>), grid, dim3(64 * WW), 0, s, a);
        hipLaunchKernelGGL((attn_f32_bwd_dkv<DD, WW, 2>), grid, dim3(64 * WW), 0, s, a);
      } else {
        hipLaunchKernelGGL((attn_f32_bwd_dkv<DD, WW, 0>), grid, dim3(64 * WW), 0, s, a);
      }
    });
  });
  check_launch();
}

}  // namespace voda
