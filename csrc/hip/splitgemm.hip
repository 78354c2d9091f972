// fp32 GEMM at fp32 accuracy on the bf16 matrix cores of gfx950: exact 3-way bf16 split.
//
//   C[m][n] (+)= sum_k A(m,k) B(n,k)  [+ bias[n]]  [GELU_AUX / DGELU epilogue]
//
// Why.  The reference trains every workload in fp32 (Keras Dense / Conv2D with no mixed
// precision policy: examples/py/tensorflow2/neural_machine_translation_with_transformer.py:
// 191-315, tensorflow2_keras_cifar_elastic.py:148-158).  gfx950 has no xf32: the f32-input
// MFMA runs at the fp32 vector rate (157 TF), 1/16 of the bf16 MFMA, and hipBLASLt / MIOpen
// already sit at ~130 TF on it (docs/PERFORMANCE.md, round 5).  Every fp32 operand x splits
// EXACTLY into three bf16 values while it is staged,
//     hi = bf16(x),  mid = bf16(x - hi),  lo = bf16(x - hi - mid),   x == hi + mid + lo
// (round-to-nearest each time, so every residual is exact in fp32 and carries <= 8 more
// significant bits).  a.b = sum of the nine cross products; each bf16 x bf16 product is exact
// in fp32 and the MFMA accumulates in fp32.  The six products kept (hh, hm, mh, hl, lh, mm)
// drop terms <= ~2^-24 |a||b| with random signs, below the rounding of an fp32 FMA chain.
// Six 32x32x16 bf16 MFMAs cost 6/16 of the 32x32x2 f32 MFMAs for the same 16 k: the ceiling
// is ~2.7x the fp32 MFMA rate.  DUAL keeps the hi.hi products and the five small corrections
// in separate accumulators (the corrections' roundings are 2^-8 smaller), summed once at the
// end; NPROD 9 adds the three smallest products (error study, profiles/r6/).
//
// Design (guide §3 fragment maps, §5 GEMM anatomy, T10 transposed reads):
//  * operands are fp32 in HBM in either orientation: "K-contiguous" (rows of k, e.g. X and W
//    of a forward Linear) or "K-major" (k-rows of contiguous m / n, e.g. dY^T / X^T of a
//    weight gradient, W of an input gradient).  No transposed copies and no split copies are
//    ever written: each thread loads 8 fp32 (two 16-B loads), splits them in registers
//    (3 v_cvt_pk_bf16_f32 + 8 VALU per pair) and writes the three planes to LDS.
//  * LDS images per stage (16 k): K-contiguous -> [row][h][plane][8] with a 96-B row pitch and
//    the k-halves swapped in every other 8-row block (sx_kc_off: conflict-free), read
//    as 3 x ds_read_b128 per fragment; K-major -> [plane][k][row] with 256-B XOR-swizzled
//    rows (guide T10 layout (b)), read as 2 x ds_read_b64_tr_b16 per fragment.
//  * v_mfma_f32_32x32x16_bf16; each wave owns a 64 x 64 output sub-tile (2 x 2 MFMA tiles);
//    workgroups of 128 x 128 (4 waves, two workgroups per CU) or 256 x 128 / 128 x 256
//    (8 waves).  LDS double-buffered, register staging two stages deep (the loads of stage
//    s+2 fly while stage s is multiplied and stage s+1 is split into LDS), one barrier per
//    stage.
//  * split-K over a grid of tiles x splits: fp32 slabs + a reduce kernel that applies the
//    epilogue; XCD-aware bijective block remap, split-major logical order (guide T1).
#include "common.h"
#include "ops.h"

#include <type_traits>

namespace voda {

namespace {

typedef __bf16 sx_bf16x8 __attribute__((ext_vector_type(8)));
typedef float sx_f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 sx_bf16x4_v __attribute__((__vector_size__(4 * sizeof(__bf16))));
typedef __attribute__((address_space(3))) sx_bf16x4_v sx_lds_bf16x4;

#ifndef SX_SCHED_GROUPS
#define SX_SCHED_GROUPS 0
#endif

constexpr int kSxBK = 16;        // k per LDS stage: one 32x32x16 MFMA step
// K-contiguous image row: [h][plane][8] bf16 = 96 B.  Round 6 (SX_KC_PITCH 96): unpadded, the two
// k-halves swapped in rows with bit 3 set (sx_kc_off), which keeps the 32x32x16 fragment reads
// conflict-free (ds_read_b128 lane groups {0-3, 12-15, 20-27} / {4-11, 16-19, 28-31}: the rows of
// a group pair up by row mod 8, and each pair differs in bit 3, so the 16 reads land on 8 even and
// 8 odd 16-B bank slots) and, with 4 consecutive rows per 16-lane group (sx_kc_unit wmap 0), the
// 8-B staging writes too.  At 96 B a 128 x 128 workgroup's double-buffered images take 48 KB for
// every orientation, so three workgroups share a CU's LDS (variant 8).  112 (padded, no swap) is
// the round-5 layout, kept buildable for A/Bs.
#ifndef SX_KC_PITCH
#define SX_KC_PITCH 96
#endif
constexpr int kSxKcPitch = SX_KC_PITCH;
static_assert(kSxKcPitch == 96 || kSxKcPitch == 112, "K-contiguous pitch: 96 (swapped halves) or 112 (padded)");
constexpr bool kSxKcWmap = kSxKcPitch == 112;  // the parity row map is for the padded layout only
__device__ __forceinline__ int sx_kc_off(int r, int h) {
  return r * kSxKcPitch + 48 * (kSxKcPitch == 96 ? h ^ ((r >> 3) & 1) : h);
}

enum : int { kSxEpiNone = 0, kSxEpiGelu = 1, kSxEpiDGelu = 2 };

struct SxArgs {
  const float* a; int64_t lda;  // A(m,k) = a[m*lda + k] (K-contiguous) or a[k*lda + m] (K-major)
  const float* b; int64_t ldb;  // B(n,k) = b[n*ldb + k] (K-contiguous) or b[k*ldb + n] (K-major)
  float* c; int64_t ldc;
  const float* bias;            // [N] or null
  float* aux; int64_t ldaux;    // GELU: h = acc + bias written here (C gets gelu(h)); DGELU: h read
  float* ws;                    // split-K slabs [S][M][N], then (bsum) the row-sum slabs [S][M]
  float* bsum;                  // optional: bsum[m] += sum_k A(m, k) (a Linear's bias gradient from dY^T)
  int M, N, K, S, kps;          // kps: k per split (multiple of 16)
  int tiles_n, tiles;
  int beta, epi;
  int stagger;                  // 1: odd workgroups at issue priority 1
  int wmap;                     // K-contiguous staging unit -> row map (sx_kc_unit)
  // implicit-GEMM convolution weight gradient (B operand in CONV mode): B(n, k) = X[img][ho*cs +
  // kh - cpad][wo*cs + kw - cpad][ci] for n = (kh*ckw + kw)*cin + ci and output pixel
  // k = (img, ho, wo); zero outside the image.  X is NHWC [cn][ch][cw][cin].
  int cn, ch, cw, cin, cho, cwo, cs, cpad, ckw;
  // output row map (omap = 1, S == 1, beta == 0): GEMM row m = (img, i, j) of an ohc x owc grid is
  // stored at pixel (2i + oph, 2j + opw) of an oH x oW NHWC map -- one parity class of a stride-2
  // convolution's input gradient
  int omap, oH, oW, oph, opw, ohc, owc;
};

int g_sx_stagger = 1;
int g_sx_wmap = 1;  // conflict-free K-contiguous staging writes (sx_kc_unit)
// convolution weight gradient kernel: 0 one-role, 1 / 2 wave-specialised (lead 1 / 2), 3 one-role
// with one accumulator at three workgroups per CU
int g_sx_conv_ws = 0;
int g_sx_conv_fwd_v8 = 0;  // convolution forward: 1 = one accumulator at three workgroups per CU

// K-major images of R = 96 columns use the R = 128 layout (192-byte k-rows padded to 256 B)
template <int R> struct SxKmPitch { static constexpr int kR = R == 96 ? 128 : R == 192 ? 256 : R; };

template <int R, bool KM> struct SxImg {
  static constexpr int kBytes = KM ? 3 * kSxBK * SxKmPitch<R>::kR * 2 : R * kSxKcPitch;
};

// K-major image: byte offset of column ``col`` (a multiple of 4) of k-row ``k`` in one plane
// ([16][R] bf16).  The 16-B chunk index is XORed within each 256-B group (guide T10 (b)), which
// keeps the 8-B staging writes and the 32x32x16 transposed reads conflict-free.
template <int R>
__device__ __forceinline__ int sx_km_off(int k, int col) {
  if constexpr (R == 96) {
    return sx_km_off<128>(k, col);
  } else if constexpr (R == 192) {
    return sx_km_off<256>(k, col);
  } else if constexpr (R == 64) {
    // 128-B k-rows: k-rows 2j and 2j + 1 side by side form row j of a [8][128] image that takes
    // the 256-B swizzle (a bijection, so staging writes and fragment reads agree)
    return sx_km_off<128>(k >> 1, ((k & 1) << 6) + col);
  } else {
    const int ch = col >> 3;
    return k * (2 * R) + ((ch & ~15) << 4) + (((ch & 15) ^ (((k & 3) << 2) | ((k >> 2) & 3))) << 4) + ((col & 4) << 1);
  }
}

// K-contiguous staging: unit u -> (row r, 4-float chunk q).  Lanes 4a..4a+3 of a wave read one
// row's 64 contiguous bytes either way.  wmap 0: r = u >> 2 (16 consecutive rows per wave); the
// three-plane 8-B LDS writes (ds_write_b64: 16-lane groups, bank = dword mod 32, row pitch 28
// dwords) then collide 2-way inside every group (rows 0 and 3 of a group share banks 0-3).
// wmap 1: a 16-lane group takes rows of one parity, 2 apart ({0, 2, 4, 6}, {1, 3, 5, 7}, ...),
// whose bank shifts {0, 24, 16, 8} tile the 32 banks exactly: conflict-free writes.
__device__ __forceinline__ void sx_kc_unit(int u, bool wmap, int& r, int& q) {
  q = u & 3;
  if (!wmap) {
    r = u >> 2;
  } else {
    const int l = u & 63, g = l >> 4, a = (l >> 2) & 3;
    r = 16 * (u >> 6) + 8 * (g >> 1) + 2 * a + (g & 1);
  }
}

// exact split of fp32 values into three packed bf16 planes (x == hi + mid + lo)
typedef float sx_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 sx_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t sx_pack2(float a, float b) {  // one v_cvt_pk_bf16_f32 (RNE)
  const sx_f32x2 f = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, sx_bf16x2));
}
__device__ __forceinline__ void sx_split2(float x0, float x1, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = sx_pack2(x0, x1);
  const float r0 = x0 - __uint_as_float(h << 16), r1 = x1 - __uint_as_float(h & 0xffff0000u);
  m = sx_pack2(r0, r1);
  const float s0 = r0 - __uint_as_float(m << 16), s1 = r1 - __uint_as_float(m & 0xffff0000u);
  l = sx_pack2(s0, s1);
}
__device__ __forceinline__ void sx_split4(const float4 v, uint2& h, uint2& m, uint2& l) {
  sx_split2(v.x, v.y, h.x, m.x, l.x);
  sx_split2(v.z, v.w, h.y, m.y, l.y);
}

__device__ __forceinline__ uint2 sx_tr_read(const uint8_t* p) {
  const sx_bf16x4_v v = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((sx_lds_bf16x4*)(p));
  return __builtin_bit_cast(uint2, v);
}

__device__ __forceinline__ sx_f32x16 sx_mfma(const sx_bf16x8& a, const sx_bf16x8& b, const sx_f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// ---- one operand's staging: 2R units of 8 fp32 per 16-k stage -------------------------------
// K-contiguous unit u: k 4q..4q+3 (q = u & 3) of rows r and r + R/2 (r = u >> 2): four lanes read
//   one row's 64 contiguous bytes, a wave-load covers 16 whole 64-B row pieces.
// K-major unit u: rows 4cg..4cg+3 (cg = u % (R/4)) at k-rows kp and kp+8 (kp = u / (R/4)).
template <int R, bool KM, int T>
struct SxStage {
  static constexpr int kUnits = 2 * R;
  static constexpr int kPer = (kUnits + T - 1) / T;
  float4 v[kPer][2];
};

template <int R, bool KM, int T>
struct SxOperand {
  using Stage = SxStage<R, KM, T>;
  static constexpr int kUnits = 2 * R;
  static constexpr int kPer = (kUnits + T - 1) / T;
  const float* g[kPer];   // this thread's unit addresses at the current stage (first float4)
  const float* g2[kPer];  // second float4 (K-contiguous: row r + R/2; K-major: k-row + 8)
  int64_t step;           // floats per 16-k stage
  int woff[kPer];         // LDS byte offset of the first float4's split (plane 0)
  int woff2[kPer];        // ... of the second
  bool on[kPer];
  bool rok[kPer];         // K-major: the unit's 4 rows are inside the matrix (not clamped duplicates)

  __device__ __forceinline__ void init(const float* base, int64_t ld, int row0, int rows, int k0, int t,
                                       bool wmap = false) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int u = t + i * T;
      on[i] = (kUnits % T == 0) || u < kUnits;
      const int uu = on[i] ? u : 0;
      if (!KM) {
        int q, r;
        sx_kc_unit(uu, kSxKcWmap && wmap && (R / 2) % 16 == 0, r, q);
        const int gr = min(row0 + r, rows - 1), gr2 = min(row0 + r + R / 2, rows - 1);  // rows past the matrix: valid duplicates
        g[i] = base + int64_t(gr) * ld + k0 + 4 * q;
        g2[i] = base + int64_t(gr2) * ld + k0 + 4 * q;
        woff[i] = sx_kc_off(r, q >> 1) + 8 * (q & 1);
        woff2[i] = sx_kc_off(r + R / 2, q >> 1) + 8 * (q & 1);
      } else {
        const int cg = uu % (R / 4), kp = uu / (R / 4);
        const int gc = min(row0 + 4 * cg, rows - 4);
        rok[i] = on[i] && row0 + 4 * cg < rows;
        g[i] = base + int64_t(k0 + kp) * ld + gc;
        g2[i] = g[i] + int64_t(8) * ld;
        woff[i] = sx_km_off<R>(kp, 4 * cg);
        woff2[i] = sx_km_off<R>(kp + 8, 4 * cg);
      }
    }
    step = KM ? int64_t(kSxBK) * ld : kSxBK;
  }

  // Loads are unconditional (a finished operand re-reads its last stage): a load under a
  // runtime condition makes hipcc merge the register sets with copies right after the loads and
  // wait for them there, exposing the whole memory latency every stage (guide §5 item 4(c)).
  __device__ __forceinline__ void load(SxStage<R, KM, T>& s, bool advance) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {  // idle units (on == false) read unit 0's valid address
      s.v[i][0] = *reinterpret_cast<const float4*>(g[i]);
      s.v[i][1] = *reinterpret_cast<const float4*>(g2[i]);
      const int64_t d = advance ? step : 0;
      g[i] += d;
      g2[i] += d;
    }
  }

  // K-major operands: this thread's 4 rows summed over the stage's two k-rows (kPer == 1)
  __device__ __forceinline__ void rowsum(const SxStage<R, KM, T>& s, float4& acc) const {
    static_assert(KM && kPer == 1, "row sums: K-major operand, one unit per thread");
    if (rok[0]) {
      acc.x += s.v[0][0].x + s.v[0][1].x;
      acc.y += s.v[0][0].y + s.v[0][1].y;
      acc.z += s.v[0][0].z + s.v[0][1].z;
      acc.w += s.v[0][0].w + s.v[0][1].w;
    }
  }

  // unconditional (no branch around the split: it interleaves with the MFMAs); idle units
  // (on == false) write to a dummy slot instead of their duplicate unit's bytes.  Each float4
  // becomes three 8-byte plane pieces: K-contiguous images keep a row's planes 16 B apart,
  // K-major images a whole [16][R] plane apart.
  __device__ __forceinline__ void write(const SxStage<R, KM, T>& s, uint8_t* img, uint8_t* dummy) const {
    constexpr int kPl = KM ? kSxBK * SxKmPitch<R>::kR * 2 : 16;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      uint2 h0, m0, l0, h1, m1, l1;
      sx_split4(s.v[i][0], h0, m0, l0);
      sx_split4(s.v[i][1], h1, m1, l1);
      uint8_t* p = on[i] ? img + woff[i] : dummy;
      uint8_t* q = on[i] ? img + woff2[i] : dummy + 8;
      const int pl = on[i] ? kPl : 16;
      *reinterpret_cast<uint2*>(p) = h0;
      *reinterpret_cast<uint2*>(p + pl) = m0;
      *reinterpret_cast<uint2*>(p + 2 * pl) = l0;
      *reinterpret_cast<uint2*>(q) = h1;
      *reinterpret_cast<uint2*>(q + pl) = m1;
      *reinterpret_cast<uint2*>(q + 2 * pl) = l1;
    }
  }
};

// K-major B operand of a convolution weight gradient, gathered from the NHWC input while it is
// staged (no im2col buffer): unit u covers input channels ci..ci+3 of one filter tap (4 rows of
// the B image) at output pixels kp and kp + 8 of the stage; each of the two pixels is tracked as
// (img, ho, wo) and advanced 16 pixels per stage.  Taps falling outside the image read a valid
// address and are zeroed at the LDS write (no branch around the load).
template <int R, int T>
struct SxConvStage {
  static constexpr int kPer = (2 * R + T - 1) / T;
  float4 v[kPer][2];
  uint32_t keep;  // bit 2i + j: pixel j of unit i is inside the image
};

template <int R, int T>
struct SxConvOperand {
  using Stage = SxConvStage<R, T>;
  static constexpr int kUnits = 2 * R;
  static constexpr int kPer = (kUnits + T - 1) / T;
  const float* x;
  int img[kPer][2], ho[kPer][2], wo[kPer][2];
  int dh[kPer], dw[kPer], ci[kPer];
  int H, W, C, Ho, Wo, cs;
  int woff[kPer], woff2[kPer];
  bool on[kPer];

  __device__ __forceinline__ void init(const SxArgs& p, int n0, int k0, int t) {
    x = p.b;
    H = p.ch; W = p.cw; C = p.cin; Ho = p.cho; Wo = p.cwo; cs = p.cs;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int u = t + i * T;
      on[i] = (kUnits % T == 0) || u < kUnits;
      const int uu = on[i] ? u : 0;
      const int cg = uu % (R / 4), kp = uu / (R / 4);
      const int n = min(n0 + 4 * cg, p.N - 4);
      const int tap = n / C;
      ci[i] = n - tap * C;
      dh[i] = tap / p.ckw - p.cpad;
      dw[i] = tap % p.ckw - p.cpad;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int m = k0 + kp + 8 * j;
        const int hw = Ho * Wo;
        img[i][j] = m / hw;
        const int r = m - img[i][j] * hw;
        ho[i][j] = r / Wo;
        wo[i][j] = r - ho[i][j] * Wo;
      }
      woff[i] = sx_km_off<R>(kp, 4 * cg);
      woff2[i] = sx_km_off<R>(kp + 8, 4 * cg);
    }
  }

  __device__ __forceinline__ void load(Stage& s, bool advance) {
    s.keep = 0;
#pragma unroll
    for (int i = 0; i < kPer; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int hi = ho[i][j] * cs + dh[i], wi = wo[i][j] * cs + dw[i];
        const bool ok = hi >= 0 && hi < H && wi >= 0 && wi < W;
        const int64_t off = ok ? ((int64_t(img[i][j]) * H + hi) * W + wi) * C + ci[i] : 0;
        s.v[i][j] = *reinterpret_cast<const float4*>(x + off);
        s.keep |= uint32_t(ok) << (2 * i + j);
        if (advance) {  // next stage: 16 output pixels on
          int w2 = wo[i][j] + kSxBK, h2 = ho[i][j], n2 = img[i][j];
          while (w2 >= Wo) {
            w2 -= Wo;
            if (++h2 == Ho) { h2 = 0; ++n2; }
          }
          wo[i][j] = w2; ho[i][j] = h2; img[i][j] = n2;
        }
      }
  }

  __device__ __forceinline__ void write(const Stage& s, uint8_t* img_, uint8_t* dummy) const {
    constexpr int kPl = kSxBK * SxKmPitch<R>::kR * 2;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const uint32_t m0 = (s.keep >> (2 * i)) & 1 ? 0xffffffffu : 0u, m1 = (s.keep >> (2 * i + 1)) & 1 ? 0xffffffffu : 0u;
      const float4 a = s.v[i][0], b = s.v[i][1];
      const float4 va = make_float4(__uint_as_float(__float_as_uint(a.x) & m0), __uint_as_float(__float_as_uint(a.y) & m0),
                                    __uint_as_float(__float_as_uint(a.z) & m0), __uint_as_float(__float_as_uint(a.w) & m0));
      const float4 vb = make_float4(__uint_as_float(__float_as_uint(b.x) & m1), __uint_as_float(__float_as_uint(b.y) & m1),
                                    __uint_as_float(__float_as_uint(b.z) & m1), __uint_as_float(__float_as_uint(b.w) & m1));
      uint2 h0, md0, l0, h1, md1, l1;
      sx_split4(va, h0, md0, l0);
      sx_split4(vb, h1, md1, l1);
      uint8_t* p = on[i] ? img_ + woff[i] : dummy;
      uint8_t* q = on[i] ? img_ + woff2[i] : dummy + 8;
      const int pl = on[i] ? kPl : 16;
      *reinterpret_cast<uint2*>(p) = h0;
      *reinterpret_cast<uint2*>(p + pl) = md0;
      *reinterpret_cast<uint2*>(p + 2 * pl) = l0;
      *reinterpret_cast<uint2*>(q) = h1;
      *reinterpret_cast<uint2*>(q + pl) = md1;
      *reinterpret_cast<uint2*>(q + 2 * pl) = l1;
    }
  }
};

// K-contiguous A operand of a convolution FORWARD, gathered from the NHWC input while it is
// staged (implicit GEMM, no im2col buffer): A(m, k) = X[img][ho*cs + kh - cpad][wo*cs + kw - cpad][ci]
// for output pixel m = (img, ho, wo) and k = (kh*ckw + kw)*cin + ci.  cin % 16 == 0, so a 16-k stage
// is 16 consecutive channels of one tap: unit u (as SxOperand K-contiguous: k 4q..4q+3 of rows r and
// r + R/2) reads one float4 per row, zeroed outside the image; the tap / channel cursor advances
// one stage per load.
template <int R, int T>
struct SxConvAOperand {
  using Stage = SxConvStage<R, T>;
  static constexpr int kUnits = 2 * R;
  static constexpr int kPer = (kUnits + T - 1) / T;
  const float* x;
  int img[kPer][2], hb[kPer][2], wb[kPer][2];  // image, ho * cs - cpad, wo * cs - cpad of each row
  int q4[kPer];
  int ci0, kh, kw;                              // the next load's channel offset and tap
  int H, W, C, KW;
  int woff[kPer], woff2[kPer];
  bool on[kPer];

  __device__ __forceinline__ void init(const SxArgs& p, int m0, int k0, int t) {
    x = p.a;
    H = p.ch; W = p.cw; C = p.cin; KW = p.ckw;
    const int tap = k0 / C;
    ci0 = k0 - tap * C;
    kh = tap / KW;
    kw = tap - kh * KW;
    const int hw = p.cho * p.cwo;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int u = t + i * T;
      on[i] = (kUnits % T == 0) || u < kUnits;
      const int uu = on[i] ? u : 0;
      int q, r;
      sx_kc_unit(uu, kSxKcWmap && p.wmap && (R / 2) % 16 == 0, r, q);
      q4[i] = 4 * q;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int m = min(m0 + r + j * (R / 2), p.M - 1);  // rows past the matrix: valid duplicates
        img[i][j] = m / hw;
        const int rem = m - img[i][j] * hw;
        const int ho = rem / p.cwo, wo = rem - (rem / p.cwo) * p.cwo;
        hb[i][j] = ho * p.cs - p.cpad;
        wb[i][j] = wo * p.cs - p.cpad;
      }
      woff[i] = sx_kc_off(r, q >> 1) + 8 * (q & 1);
      woff2[i] = sx_kc_off(r + R / 2, q >> 1) + 8 * (q & 1);
    }
  }

  __device__ __forceinline__ void load(Stage& s, bool advance) {
    s.keep = 0;
#pragma unroll
    for (int i = 0; i < kPer; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int hi = hb[i][j] + kh, wi = wb[i][j] + kw;
        const bool ok = hi >= 0 && hi < H && wi >= 0 && wi < W;
        const int64_t off = ok ? ((int64_t(img[i][j]) * H + hi) * W + wi) * C + ci0 + q4[i] : 0;
        s.v[i][j] = *reinterpret_cast<const float4*>(x + off);
        s.keep |= uint32_t(ok) << (2 * i + j);
      }
    if (advance) {
      ci0 += kSxBK;
      if (ci0 >= C) {
        ci0 = 0;
        if (++kw == KW) { kw = 0; ++kh; }
      }
    }
  }

  __device__ __forceinline__ void write(const Stage& s, uint8_t* img_, uint8_t* dummy) const {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const uint32_t m0 = (s.keep >> (2 * i)) & 1 ? 0xffffffffu : 0u, m1 = (s.keep >> (2 * i + 1)) & 1 ? 0xffffffffu : 0u;
      const float4 a = s.v[i][0], b = s.v[i][1];
      const float4 va = make_float4(__uint_as_float(__float_as_uint(a.x) & m0), __uint_as_float(__float_as_uint(a.y) & m0),
                                    __uint_as_float(__float_as_uint(a.z) & m0), __uint_as_float(__float_as_uint(a.w) & m0));
      const float4 vb = make_float4(__uint_as_float(__float_as_uint(b.x) & m1), __uint_as_float(__float_as_uint(b.y) & m1),
                                    __uint_as_float(__float_as_uint(b.z) & m1), __uint_as_float(__float_as_uint(b.w) & m1));
      uint2 h0, md0, l0, h1, md1, l1;
      sx_split4(va, h0, md0, l0);
      sx_split4(vb, h1, md1, l1);
      uint8_t* pp = on[i] ? img_ + woff[i] : dummy;
      uint8_t* qq = on[i] ? img_ + woff2[i] : dummy + 8;
      *reinterpret_cast<uint2*>(pp) = h0;
      *reinterpret_cast<uint2*>(pp + 16) = md0;
      *reinterpret_cast<uint2*>(pp + 32) = l0;
      *reinterpret_cast<uint2*>(qq) = h1;
      *reinterpret_cast<uint2*>(qq + 16) = md1;
      *reinterpret_cast<uint2*>(qq + 32) = l1;
    }
  }
};

// three fragments (hi, mid, lo) of the 32-row tile starting at image row r0 for this lane
template <int R, bool KM>
__device__ __forceinline__ void sx_frag(const uint8_t* img, int r0, int lane, sx_bf16x8 (&f)[3]) {
  if (!KM) {
    const uint8_t* p = img + sx_kc_off(r0 + (lane & 31), lane >> 5);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) f[pl] = *reinterpret_cast<const sx_bf16x8*>(p + 16 * pl);
  } else {
    // guide T10: lane 4q+p of a 16-lane group g names k-row 8(g>>1) + 4j + q, columns
    // 16(g&1) + 4p .. +3 of the tile; lane i of the group receives column i
    const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const int k = 8 * (g >> 1) + q, col = r0 + 16 * (g & 1) + 4 * pp;
    const int o0 = sx_km_off<R>(k, col), o1 = sx_km_off<R>(k + 4, col);
    constexpr int kPlane = kSxBK * SxKmPitch<R>::kR * 2;
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
      const uint2 lo = sx_tr_read(img + pl * kPlane + o0);
      const uint2 hi = sx_tr_read(img + pl * kPlane + o1);
      f[pl] = __builtin_bit_cast(sx_bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
    }
  }
}

__device__ __forceinline__ int64_t sx_out_row(const SxArgs& p, int row) {
  if (!p.omap) return row;
  const int hw = p.ohc * p.owc;
  const int img = row / hw, r = row - img * hw, i = r / p.owc, j = r - (r / p.owc) * p.owc;
  return (int64_t(img) * p.oH + 2 * i + p.oph) * p.oW + 2 * j + p.opw;
}

__device__ __forceinline__ float sx_finish(const SxArgs& p, int row, int col, float v) {
  if (p.beta) v += p.c[int64_t(row) * p.ldc + col];
  if (p.bias) v += p.bias[col];
  if (p.epi == kSxEpiGelu) {
    p.aux[int64_t(row) * p.ldaux + col] = v;
    v = gelu_tanh_f(v);
  } else if (p.epi == kSxEpiDGelu) {
    v *= gelu_tanh_grad(p.aux[int64_t(row) * p.ldaux + col]);
  }
  return v;
}

// WMT / WNT: 32-row / 32-column MFMA tiles per wave (2 x 2: 64 x 64 per wave; 4 x 2: 128 x 64 per
// wave, one wave per SIMD with its accumulators in AGPRs; 1 x 3: 32 x 96, the 128 x 96 tile)
template <int BM, int BN, bool AKM, bool BKM, int NPROD, bool DUAL, bool TWO_SETS, int MINW, int WMT, bool CONV = false,
          int ORDER = 0, bool CONVA = false, int WNT = 2>
__global__ __launch_bounds__((BM / (32 * WMT)) * (BN / (32 * WNT)) * 64, MINW) void sgemm_bf16x3_kernel(SxArgs p) {
  constexpr int NWN = BN / (32 * WNT);
  constexpr int NWM = BM / (32 * WMT);
  constexpr int T = 64 * NWM * NWN;
  constexpr int kImgA = SxImg<BM, AKM>::kBytes, kImgB = SxImg<BN, BKM>::kBytes;
  constexpr int kBuf = kImgA + kImgB;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * kBuf + 64];  // + dummy slot (idle units)

  // bijective XCD remap (guide §5 'XCD swizzle must be bijective'): the blocks one XCD runs
  // are a contiguous range of logical ids; logical order is split-major, tiles row-major
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int split = lid / p.tiles, tile = lid - split * p.tiles;
  const int m0 = (tile / p.tiles_n) * BM, n0 = (tile % p.tiles_n) * BN;
  const int kb = split * p.kps;
  const int ke = min(p.K, kb + p.kps);
  const int nst = ke > kb ? (ke - kb) / kSxBK : 0;

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave / NWN, wn = wave % NWN;
  // two co-resident workgroups run the same program in lock step (MFMA phases together, VALU /
  // LDS / barrier phases together); static priority for one of them staggers the pair
  // (MI355X_MICROARCH.md 'Two waves per SIMD', items 4 and 9)
  if (__builtin_amdgcn_readfirstlane(p.stagger & blockIdx.x) & 1) __builtin_amdgcn_s_setprio(1);

  using OpA = std::conditional_t<CONVA, SxConvAOperand<BM, T>, SxOperand<BM, AKM, T>>;
  using StA = typename OpA::Stage;
  OpA opa;
  using OpB = std::conditional_t<CONV, SxConvOperand<BN, T>, SxOperand<BN, BKM, T>>;
  using StB = typename OpB::Stage;
  OpB opb;
  if constexpr (CONVA) opa.init(p, m0, kb, t);
  else opa.init(p.a, p.lda, m0, p.M, kb, t, p.wmap);
  if constexpr (CONV) opb.init(p, n0, kb, t);
  else opb.init(p.b, p.ldb, n0, p.N, kb, t, p.wmap);
  StA sa0, sa1;
  StB sb0, sb1;

  sx_f32x16 acc[WMT][WNT], cor[WMT][WNT];
#pragma unroll
  for (int i = 0; i < WMT; ++i)
#pragma unroll
    for (int j = 0; j < WNT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) { acc[i][j][r] = 0.f; cor[i][j][r] = 0.f; }

  auto compute = [&](int buf) {
    const uint8_t* A = smem + buf * kBuf;
    const uint8_t* B = A + kImgA;
    sx_bf16x8 fa[WMT][3], fb[WNT][3];
#pragma unroll
    for (int i = 0; i < WMT; ++i) sx_frag<BM, AKM>(A, wm * 32 * WMT + 32 * i, lane, fa[i]);
#pragma unroll
    for (int j = 0; j < WNT; ++j) sx_frag<BN, BKM>(B, wn * 32 * WNT + 32 * j, lane, fb[j]);
    if constexpr (ORDER == 0) {  // tile-outer: each accumulator's products back to back
#pragma unroll
      for (int i = 0; i < WMT; ++i)
#pragma unroll
        for (int j = 0; j < WNT; ++j) {
          sx_f32x16& s = DUAL ? cor[i][j] : acc[i][j];
          if (NPROD >= 9) {
            s = sx_mfma(fa[i][2], fb[j][2], s);
            s = sx_mfma(fa[i][1], fb[j][2], s);
            s = sx_mfma(fa[i][2], fb[j][1], s);
          }
          if (NPROD >= 6) {
            s = sx_mfma(fa[i][1], fb[j][1], s);
            s = sx_mfma(fa[i][0], fb[j][2], s);
            s = sx_mfma(fa[i][2], fb[j][0], s);
          }
          s = sx_mfma(fa[i][0], fb[j][1], s);
          s = sx_mfma(fa[i][1], fb[j][0], s);
          acc[i][j] = sx_mfma(fa[i][0], fb[j][0], acc[i][j]);
        }
    } else {  // product-outer: consecutive MFMAs write different accumulators
      constexpr int kPa[8] = {2, 1, 2, 1, 0, 2, 0, 1}, kPb[8] = {2, 2, 1, 1, 2, 0, 1, 0};
      constexpr int p0 = NPROD >= 9 ? 0 : NPROD >= 6 ? 3 : 6;
#pragma unroll
      for (int q = p0; q < 8; ++q)
#pragma unroll
        for (int i = 0; i < WMT; ++i)
#pragma unroll
          for (int j = 0; j < WNT; ++j) {
            sx_f32x16& s = DUAL ? cor[i][j] : acc[i][j];
            s = sx_mfma(fa[i][kPa[q]], fb[j][kPb[q]], s);
          }
#pragma unroll
      for (int i = 0; i < WMT; ++i)
#pragma unroll
        for (int j = 0; j < WNT; ++j) acc[i][j] = sx_mfma(fa[i][0], fb[j][0], acc[i][j]);
    }
  };
  // fused row sums of A (a Linear's bias gradient from dY^T): the workgroups of column tile 0
  constexpr bool kRowSum = AKM && !CONVA && SxOperand<BM, AKM, T>::kPer == 1;
  const bool do_rs = kRowSum && __builtin_amdgcn_readfirstlane(p.bsum != nullptr && n0 == 0);
  float4 rs = make_float4(0.f, 0.f, 0.f, 0.f);
  auto write = [&](const StA& sa, const StB& sb, int buf) {
    uint8_t* A = smem + buf * kBuf;
    if constexpr (kRowSum) {
      if (do_rs) opa.rowsum(sa, rs);
    }
    opa.write(sa, A, smem + 2 * kBuf);
    opb.write(sb, A + kImgA, smem + 2 * kBuf);
  };

  // stage k is read from global at load number k (clamped to the last stage), multiplied from
  // LDS buffer k & 1; the loads of stage s+2 fly while stage s is multiplied
  int nld = 0;
  auto load = [&](StA& sa, StB& sb) {
    const bool adv = ++nld < nst;
    opa.load(sa, adv);
    opb.load(sb, adv);
    // keep the loads ahead of the MFMAs: hipcc otherwise sinks them below the MFMAs into the
    // fragment registers and waits for them at once (no prefetch at all)
    __builtin_amdgcn_sched_barrier(0);
  };
  if (TWO_SETS) {
    // software pipeline: iteration s loads stage s+2, multiplies stage s and splits stage s+1
    // (loaded one iteration earlier) into the other LDS buffer; the split's VALU and LDS writes
    // are interleaved with the MFMAs (sched_group_barrier), not issued after them
    auto pipe = [&](StA& la, StB& lb, const StA& wa, const StB& wb, int buf) {
      load(la, lb);
      compute(buf);
      write(wa, wb, buf ^ 1);
#if SX_SCHED_GROUPS
      constexpr int kMf = 2 * WMT * (NPROD == 9 ? 9 : NPROD == 6 ? 6 : 3);
#pragma unroll
      for (int k = 0; k < kMf; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // then up to 4 VALU
        if ((k & 3) == 3) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // then a DS write
      }
#endif
      __syncthreads();
    };
    if (nst > 0) {
      load(sa0, sb0);
      write(sa0, sb0, 0);
      load(sa1, sb1);
    }
    __syncthreads();
    // unrolled by two so the register stage sets stay compile-time (guide §5.4 rule 20)
    for (int st = 0; st < nst; st += 2) {
      pipe(sa0, sb0, sa1, sb1, 0);
      if (st + 1 >= nst) break;
      pipe(sa1, sb1, sa0, sb0, 1);
    }
  } else {  // one register set: the loads of stage s+1 fly during the MFMAs of stage s
    if (nst > 0) {
      load(sa0, sb0);
      write(sa0, sb0, 0);
    }
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
      load(sa0, sb0);
      compute(st & 1);
      if (st + 1 < nst) write(sa0, sb0, (st + 1) & 1);
      __syncthreads();
    }
  }

  if constexpr (kRowSum) {
    if (do_rs) {  // the R/4 row groups' partials over the k-row slots, through LDS (loop ended in a barrier)
      constexpr int kGroups = BM / 4, kSlots = T / kGroups;
      float4* red = reinterpret_cast<float4*>(smem);
      red[t] = rs;
      __syncthreads();
      if (t < kGroups) {
        float4 v = red[t];
#pragma unroll
        for (int q = 1; q < kSlots; ++q) {
          const float4 w = red[q * kGroups + t];
          v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
        }
        const int row = m0 + 4 * t;
        if (row < p.M) {
          if (p.S > 1) {
            *reinterpret_cast<float4*>(p.ws + int64_t(p.S) * p.M * p.N + int64_t(split) * p.M + row) = v;
          } else {
            float4* b = reinterpret_cast<float4*>(p.bsum + row);
            float4 o = *b;
            o.x += v.x; o.y += v.y; o.z += v.z; o.w += v.w;
            *b = o;
          }
        }
      }
    }
  }

  // epilogue: C/D lane map col = lane & 31, row = (reg&3) + 8 (reg>>2) + 4 (lane>>5)
  const int h = lane >> 5;
#pragma unroll
  for (int i = 0; i < WMT; ++i)
#pragma unroll
    for (int j = 0; j < WNT; ++j) {
      const int col = n0 + wn * 32 * WNT + 32 * j + (lane & 31);
      if (col >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 32 * WMT + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row >= p.M) continue;
        const float v = DUAL ? acc[i][j][r] + cor[i][j][r] : acc[i][j][r];
        if (p.S > 1) {
          p.ws[(int64_t(split) * p.M + row) * p.N + col] = v;
        } else {
          p.c[sx_out_row(p, row) * p.ldc + col] = sx_finish(p, row, col, v);
        }
      }
    }
}

// Wave-specialised form of the kernel above (round 6): a 512-thread workgroup per 128 x 128 tile,
// waves 0-3 multiply (each a 64 x 64 sub-tile, dual accumulators, ds_read fragments + 24 MFMAs
// per 16-k stage) and waves 4-7 stage (global loads DEPTH - 1 stages ahead in registers, the
// exact split, ds_write of the three planes).  In the one-role kernel every wave alternates an
// MFMA phase with a VALU / LDS-write phase, and the two co-resident workgroups fall into step, so
// the phases add up (~3.9k cycles per stage per CU against 1.5k of MFMA, profiles/r6/); here a
// SIMD holds one MFMA wave and one staging wave, whose VALU issues in the 24 of every 32 MFMA
// cycles that the MFMA leaves free (MI355X_MICROARCH.md 'vector-instruction ISSUE cost').
// One barrier per stage, every wave executes the same nst barriers.  LEAD 1: two LDS buffers,
// barrier k publishes stage k.  LEAD 2: three buffers, the staging waves run two stages ahead and
// barrier k publishes stage k + 1, so the MFMA waves read the next stage's fragments while they
// multiply the current one (no LDS latency at the head of each stage); two fragment sets leave
// no room for the dual accumulators, so LEAD 2 keeps one (corrections first, hi.hi last).
template <bool AKM, bool BKM, bool CONV, int LEAD, int DEPTH, bool DUAL = (LEAD == 1)>
__global__ __launch_bounds__(512, 1) void sgemm_ws_kernel(SxArgs p) {
  static_assert(DEPTH % 2 == 0 && (LEAD == 1 || LEAD == 2), "stage sets / lead");
  constexpr int BM = 128, BN = 128, T = 256;
  constexpr int NB = LEAD + 1;  // LDS buffers
  constexpr int kImgA = SxImg<BM, AKM>::kBytes, kImgB = SxImg<BN, BKM>::kBytes;
  constexpr int kBuf = kImgA + kImgB;
  __shared__ __attribute__((aligned(16))) uint8_t smem[NB * kBuf + 64];

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int split = lid / p.tiles, tile = lid - split * p.tiles;
  const int m0 = (tile / p.tiles_n) * BM, n0 = (tile % p.tiles_n) * BN;
  const int kb = split * p.kps;
  const int ke = min(p.K, kb + p.kps);
  const int nst = ke > kb ? (ke - kb) / kSxBK : 0;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);

  if (wave >= 4) {  // ---------------- staging waves
    const int tp = t - T;
    SxOperand<BM, AKM, T> opa;
    using OpB = std::conditional_t<CONV, SxConvOperand<BN, T>, SxOperand<BN, BKM, T>>;
    using StB = typename OpB::Stage;
    OpB opb;
    opa.init(p.a, p.lda, m0, p.M, kb, tp, p.wmap);
    if constexpr (CONV) opb.init(p, n0, kb, tp);
    else opb.init(p.b, p.ldb, n0, p.N, kb, tp, p.wmap);
    SxStage<BM, AKM, T> sa[DEPTH];
    StB sb[DEPTH];
    int nld = 0;
    auto load = [&](SxStage<BM, AKM, T>& a_, StB& b_) {
      const bool adv = ++nld < nst;
      opa.load(a_, adv);
      opb.load(b_, adv);
    };
    auto write = [&](const SxStage<BM, AKM, T>& a_, const StB& b_, int stage) {
      uint8_t* A = smem + (stage % NB) * kBuf;
      opa.write(a_, A, smem + NB * kBuf);
      opb.write(b_, A + kImgA, smem + NB * kBuf);
    };
    // register sets: stage s lives in set s % DEPTH; stages 0 .. LEAD - 1 are written before
    // barrier 0, then each set is refilled right after its stage is written
    if (nst > 0) {
#pragma unroll
      for (int j = 0; j < DEPTH; ++j) load(sa[j], sb[j]);
#pragma unroll
      for (int j = 0; j < LEAD; ++j) {
        if (j < nst) {
          write(sa[j], sb[j], j);
          load(sa[j], sb[j]);  // stage DEPTH + j
        }
      }
    }
    // iteration k: barrier k, then stage k + LEAD into its buffer; unrolled by DEPTH so the
    // register sets stay static
    for (int k = 0; k < nst; k += DEPTH) {
#pragma unroll
      for (int u = 0; u < DEPTH; ++u) {
        if (k + u < nst) {
          __syncthreads();
          if (k + u + LEAD < nst) {
            write(sa[(u + LEAD) % DEPTH], sb[(u + LEAD) % DEPTH], k + u + LEAD);
            load(sa[(u + LEAD) % DEPTH], sb[(u + LEAD) % DEPTH]);
          }
        }
      }
    }
    return;
  }

  // ---------------- MFMA waves
  const int wm = wave >> 1, wn = wave & 1;
  sx_f32x16 acc[2][2], cor[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) { acc[i][j][r] = 0.f; cor[i][j][r] = 0.f; }
  auto frags = [&](int stage, sx_bf16x8 (&fa)[2][3], sx_bf16x8 (&fb)[2][3]) {
    const uint8_t* A = smem + (stage % NB) * kBuf;
    const uint8_t* B = A + kImgA;
    sx_frag<BM, AKM>(A, wm * 64, lane, fa[0]);
    sx_frag<BM, AKM>(A, wm * 64 + 32, lane, fa[1]);
    sx_frag<BN, BKM>(B, wn * 64, lane, fb[0]);
    sx_frag<BN, BKM>(B, wn * 64 + 32, lane, fb[1]);
  };
  auto mfmas = [&](const sx_bf16x8 (&fa)[2][3], const sx_bf16x8 (&fb)[2][3]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        sx_f32x16& s = DUAL ? cor[i][j] : acc[i][j];
        s = sx_mfma(fa[i][1], fb[j][1], s);
        s = sx_mfma(fa[i][0], fb[j][2], s);
        s = sx_mfma(fa[i][2], fb[j][0], s);
        s = sx_mfma(fa[i][0], fb[j][1], s);
        s = sx_mfma(fa[i][1], fb[j][0], s);
        acc[i][j] = sx_mfma(fa[i][0], fb[j][0], acc[i][j]);
      }
  };
  if constexpr (LEAD == 1) {
    for (int k = 0; k < nst; ++k) {
      __syncthreads();
      sx_bf16x8 fa[2][3], fb[2][3];
      frags(k, fa, fb);
      mfmas(fa, fb);
    }
  } else {
    // unrolled by two: set 0 holds even stages, set 1 odd ones
    sx_bf16x8 fa0[2][3], fb0[2][3], fa1[2][3], fb1[2][3];
    for (int k = 0; k < nst; k += 2) {
      __syncthreads();                    // barrier k: stages <= k + 1 published
      if (k == 0) frags(0, fa0, fb0);
      if (k + 1 < nst) frags(k + 1, fa1, fb1);
      mfmas(fa0, fb0);
      if (k + 1 >= nst) break;
      __syncthreads();                    // barrier k + 1
      if (k + 2 < nst) frags(k + 2, fa0, fb0);
      mfmas(fa1, fb1);
    }
  }
  const int h = lane >> 5;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + 32 * j + (lane & 31);
      if (col >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row >= p.M) continue;
        const float v = DUAL ? acc[i][j][r] + cor[i][j][r] : acc[i][j][r];
        if (p.S > 1) {
          p.ws[(int64_t(split) * p.M + row) * p.N + col] = v;
        } else {
          p.c[int64_t(row) * p.ldc + col] = sx_finish(p, row, col, v);
        }
      }
    }
}

// split-K: C = epilogue(sum over the S slabs), 4 columns per thread (N % 4 == 0).  A block is
// 64 float4 columns x GR slab groups: thread (g, c) sums slabs g, g + GR, ... of its column with
// four partial sums in flight, the GR partials meet in LDS and group 0 applies the epilogue.  With
// one group per column (the round-5 form) a small output with hundreds of slabs (ResNet-50 1x1
// weight gradients: 64 x 256 outputs over 256 slabs) ran as 16-64 blocks of long serial loops.
template <int GR>
__global__ __launch_bounds__(64 * GR) void sgemm_reduce_kernel(SxArgs p) {
  __shared__ float4 red[GR > 1 ? GR - 1 : 1][64];
  const int64_t n4 = p.N >> 2;
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t i = int64_t(blockIdx.x) * 64 + c;
  const bool ok = i < int64_t(p.M) * n4;
  const int64_t ii = ok ? i : 0;
  const int row = int(ii / n4), col = int(ii - int64_t(row) * n4) * 4;
  const int64_t slab = int64_t(p.M) * p.N;
  const float* w = p.ws + int64_t(row) * p.N + col;
  float4 s[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) s[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  int k = g;
  for (; k + 3 * GR < p.S; k += 4 * GR) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float4 v = *reinterpret_cast<const float4*>(w + (k + u * GR) * slab);
      s[u].x += v.x; s[u].y += v.y; s[u].z += v.z; s[u].w += v.w;
    }
  }
  for (; k < p.S; k += GR) {
    const float4 v = *reinterpret_cast<const float4*>(w + k * slab);
    s[0].x += v.x; s[0].y += v.y; s[0].z += v.z; s[0].w += v.w;
  }
  float4 t = make_float4((s[0].x + s[1].x) + (s[2].x + s[3].x), (s[0].y + s[1].y) + (s[2].y + s[3].y),
                         (s[0].z + s[1].z) + (s[2].z + s[3].z), (s[0].w + s[1].w) + (s[2].w + s[3].w));
  if constexpr (GR > 1) {
    if (g > 0) red[g - 1][c] = t;
    __syncthreads();
    if (g > 0) return;
#pragma unroll
    for (int q = 0; q < GR - 1; ++q) {
      const float4 v = red[q][c];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
  }
  if (!ok) return;
  float* cp = p.c + int64_t(row) * p.ldc + col;
  cp[0] = sx_finish(p, row, col, t.x);
  cp[1] = sx_finish(p, row, col + 1, t.y);
  cp[2] = sx_finish(p, row, col + 2, t.z);
  cp[3] = sx_finish(p, row, col + 3, t.w);
}

// bsum[m] += sum over the S row-sum slabs (the fused bias gradient of a split-K weight gradient)
__global__ __launch_bounds__(256) void sgemm_rowsum_reduce_kernel(SxArgs p) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= p.M) return;
  const float* w = p.ws + int64_t(p.S) * p.M * p.N + m;
  float s0 = 0.f, s1 = 0.f;
  int k = 0;
  for (; k + 1 < p.S; k += 2) {
    s0 += w[int64_t(k) * p.M];
    s1 += w[int64_t(k + 1) * p.M];
  }
  if (k < p.S) s0 += w[int64_t(k) * p.M];
  p.bsum[m] += s0 + s1;
}

// slab groups per float4 column: enough blocks for ~4 waves per SIMD chip-wide, >= 8 slabs per thread
int g_sx_reduce_groups = -1;  // < 0: automatic; else fixed (A/B)

void sx_reduce(const SxArgs& p, hipStream_t st) {
  const int64_t items = int64_t(p.M) * (p.N / 4);
  const int64_t blocks = (items + 63) / 64;
  int gr = g_sx_reduce_groups;
  if (gr < 0) {
    gr = 1;
    while (gr < 16 && blocks * gr < 4096 && p.S >= 16 * gr) gr *= 2;
  }
  const dim3 grid{unsigned(blocks)};
  switch (gr) {
    case 16: hipLaunchKernelGGL(sgemm_reduce_kernel<16>, grid, dim3(1024), 0, st, p); break;
    case 8: hipLaunchKernelGGL(sgemm_reduce_kernel<8>, grid, dim3(512), 0, st, p); break;
    case 4: hipLaunchKernelGGL(sgemm_reduce_kernel<4>, grid, dim3(256), 0, st, p); break;
    case 2: hipLaunchKernelGGL(sgemm_reduce_kernel<2>, grid, dim3(128), 0, st, p); break;
    default: hipLaunchKernelGGL(sgemm_reduce_kernel<1>, grid, dim3(64), 0, st, p); break;
  }
  check_launch();
}

template <int BM, int BN, int NPROD, bool DUAL, bool TWO, int MINW = 2, int WMT = 2, int ORDER = 0, int WNT = 2>
void sx_launch_tile(const SxArgs& a, bool akm, bool bkm, unsigned grid, hipStream_t st) {
  const dim3 blk((BM / (32 * WMT)) * (BN / (32 * WNT)) * 64);
  if (!akm && !bkm) hipLaunchKernelGGL((sgemm_bf16x3_kernel<BM, BN, false, false, NPROD, DUAL, TWO, MINW, WMT, false, ORDER, false, WNT>), grid, blk, 0, st, a);
  else if (!akm && bkm) hipLaunchKernelGGL((sgemm_bf16x3_kernel<BM, BN, false, true, NPROD, DUAL, TWO, MINW, WMT, false, ORDER, false, WNT>), grid, blk, 0, st, a);
  else if (akm && !bkm) hipLaunchKernelGGL((sgemm_bf16x3_kernel<BM, BN, true, false, NPROD, DUAL, TWO, MINW, WMT, false, ORDER, false, WNT>), grid, blk, 0, st, a);
  else hipLaunchKernelGGL((sgemm_bf16x3_kernel<BM, BN, true, true, NPROD, DUAL, TWO, MINW, WMT, false, ORDER, false, WNT>), grid, blk, 0, st, a);
}

template <int LEAD, int DEPTH>
void sx_launch_ws(const SxArgs& a, bool akm, bool bkm, unsigned grid, hipStream_t st) {
  const dim3 blk(512);
  if (!akm && !bkm) hipLaunchKernelGGL((sgemm_ws_kernel<false, false, false, LEAD, DEPTH>), grid, blk, 0, st, a);
  else if (!akm && bkm) hipLaunchKernelGGL((sgemm_ws_kernel<false, true, false, LEAD, DEPTH>), grid, blk, 0, st, a);
  else if (akm && !bkm) hipLaunchKernelGGL((sgemm_ws_kernel<true, false, false, LEAD, DEPTH>), grid, blk, 0, st, a);
  else hipLaunchKernelGGL((sgemm_ws_kernel<true, true, false, LEAD, DEPTH>), grid, blk, 0, st, a);
}

constexpr int kSxTileM[8] = {128, 256, 128, 256, 256, 64, 256, 128};
constexpr int kSxTileN[8] = {128, 128, 256, 128, 128, 256, 64, 96};

}  // namespace

void sgemm_f32_set_stagger(int on) { g_sx_stagger = on ? 1 : 0; }
void sgemm_set_write_map(int on) { g_sx_wmap = on ? 1 : 0; }
void sgemm_conv_fwd_set_v8(int on) { g_sx_conv_fwd_v8 = on ? 1 : 0; }
void sgemm_conv_wgrad_set_ws(int mode) { g_sx_conv_ws = mode < 0 || mode > 3 ? 0 : mode; }
void sgemm_set_reduce_groups(int g) { g_sx_reduce_groups = (g == 1 || g == 2 || g == 4 || g == 8 || g == 16) ? g : -1; }

int64_t sgemm_f32_workspace_floats(int M, int N, int splits) {
  return splits > 1 ? int64_t(splits) * M * N + int64_t(splits) * M : 0;  // + the row-sum slabs
}

// variant: 0 = 6 products, dual accumulators, one register stage set (the shipped math);
// 1 = 6 products, one accumulator, software-pipelined split (two register sets); 2 = 9
// products; 3 = 3 products (hi.hi + hi.mid + mid.hi: ~16-bit, error study only); 4 = variant 0
// software-pipelined at one wave per SIMD (512 VGPRs; the dual accumulators do not fit the
// pipeline at two waves per SIMD: 400+ bytes of spills); 5 = variant 0 with the products issued
// product-outer (consecutive MFMAs on different accumulators); 6 = variant 0's math in the
// wave-specialised kernel (sgemm_ws_kernel: 4 MFMA + 4 staging waves, one workgroup per CU);
// 7 = 6 with three LDS buffers, the staging waves two stages ahead and the MFMA waves reading
// the next stage's fragments during the current stage's MFMAs (one accumulator); 8 = one
// accumulator at three workgroups per CU (<= 168 VGPRs; K-major images fit 3 x 49 KB of LDS).  Variants 1-7: 128 x 128 only.
void sgemm_f32(uintptr_t a, int64_t lda, bool a_kmajor, uintptr_t b, int64_t ldb, bool b_kmajor, uintptr_t c,
               int64_t ldc, int M, int N, int K, bool beta, uintptr_t bias, int epi, uintptr_t aux, int64_t ldaux,
               int tile, int splits, int variant, uintptr_t ws, int64_t ws_floats, uintptr_t stream, uintptr_t bsum) {
  VODA_CHECK(M > 0 && N > 0 && K > 0, "sgemm_f32: empty GEMM");
  VODA_CHECK(bsum == 0 || (a_kmajor && (tile == 0 || tile == 7) && (variant == 0 || variant == 8) && bsum % 16 == 0),
             "sgemm_f32: fused row sums need a K-major A on tile 0 / 7, variant 0 / 8, 16-B aligned");
  VODA_CHECK(K % kSxBK == 0, "sgemm_f32: K must be a multiple of 16");
  VODA_CHECK(M % 4 == 0 && N % 4 == 0, "sgemm_f32: M and N must be multiples of 4");
  VODA_CHECK(tile >= 0 && tile < 8, "sgemm_f32: bad tile id");
  VODA_CHECK(variant >= 0 && variant <= 8 && (variant == 0 || tile == 0 || (variant == 8 && tile == 7)),
             "sgemm_f32: bad math variant");
  VODA_CHECK(epi >= kSxEpiNone && epi <= kSxEpiDGelu && (epi == kSxEpiNone || aux != 0), "sgemm_f32: bad epilogue");
  VODA_CHECK(a % 16 == 0 && b % 16 == 0 && lda % 4 == 0 && ldb % 4 == 0, "sgemm_f32: operands need 16-B rows");
  VODA_CHECK(lda >= (a_kmajor ? M : K) && ldb >= (b_kmajor ? N : K) && ldc >= N, "sgemm_f32: leading dims");
  const int BM = kSxTileM[tile], BN = kSxTileN[tile];
  SxArgs p{};
  p.a = reinterpret_cast<const float*>(a); p.lda = lda;
  p.b = reinterpret_cast<const float*>(b); p.ldb = ldb;
  p.c = reinterpret_cast<float*>(c); p.ldc = ldc;
  p.bias = reinterpret_cast<const float*>(bias);
  p.aux = reinterpret_cast<float*>(aux); p.ldaux = ldaux;
  p.M = M; p.N = N; p.K = K;
  const int kst = K / kSxBK;
  int S = splits < 1 ? 1 : splits;
  if (S > kst) S = kst;
  p.kps = ((kst + S - 1) / S) * kSxBK;
  S = (K + p.kps - 1) / p.kps;  // no empty split
  p.S = S;
  p.tiles_n = (N + BN - 1) / BN;
  p.tiles = ((M + BM - 1) / BM) * p.tiles_n;
  p.beta = beta ? 1 : 0;
  p.epi = epi;
  p.stagger = g_sx_stagger;
  p.wmap = g_sx_wmap;
  p.bsum = reinterpret_cast<float*>(bsum);
  if (S > 1) {
    VODA_CHECK(ws != 0 && ws_floats >= sgemm_f32_workspace_floats(M, N, S), "sgemm_f32: split-K workspace too small");
    VODA_CHECK(c % 16 == 0 && ldc % 4 == 0, "sgemm_f32: split-K output needs 16-B rows");
    p.ws = reinterpret_cast<float*>(ws);
  }
  const int64_t nwg = int64_t(p.tiles) * S;
  VODA_CHECK(nwg < (int64_t(1) << 31), "sgemm_f32: grid too large");
  const unsigned grid = unsigned(nwg);
  hipStream_t st = as_stream(stream);
  if (tile == 0) {
    if (variant == 0) sx_launch_tile<128, 128, 6, true, false>(p, a_kmajor, b_kmajor, grid, st);
    else if (variant == 1) sx_launch_tile<128, 128, 6, false, true>(p, a_kmajor, b_kmajor, grid, st);
    else if (variant == 2) sx_launch_tile<128, 128, 9, true, false>(p, a_kmajor, b_kmajor, grid, st);
    else if (variant == 3) sx_launch_tile<128, 128, 3, true, false>(p, a_kmajor, b_kmajor, grid, st);
    else if (variant == 4) sx_launch_tile<128, 128, 6, true, true, 1>(p, a_kmajor, b_kmajor, grid, st);
    else if (variant == 5) sx_launch_tile<128, 128, 6, true, false, 2, 2, 1>(p, a_kmajor, b_kmajor, grid, st);
    else if (variant == 6) sx_launch_ws<1, 2>(p, a_kmajor, b_kmajor, grid, st);
    else if (variant == 7) sx_launch_ws<2, 2>(p, a_kmajor, b_kmajor, grid, st);
    else sx_launch_tile<128, 128, 6, false, false, 3>(p, a_kmajor, b_kmajor, grid, st);
  } else if (tile == 1) {
    sx_launch_tile<256, 128, 6, true, false>(p, a_kmajor, b_kmajor, grid, st);
  } else if (tile == 2) {
    sx_launch_tile<128, 256, 6, true, false>(p, a_kmajor, b_kmajor, grid, st);
  } else if (tile == 7) {  // 128 x 96 (4 waves of 32 x 96): N = 768 outputs as 8 column tiles, so
                           // 8192 x 768 runs 512 workgroups (two per CU) instead of 384
    if (variant == 8)  // one accumulator at three workgroups per CU (43 KB of LDS each)
      sx_launch_tile<128, 96, 6, false, false, 3, 1, 0, 3>(p, a_kmajor, b_kmajor, grid, st);
    else
      sx_launch_tile<128, 96, 6, true, false, 2, 1, 0, 3>(p, a_kmajor, b_kmajor, grid, st);
  } else if (tile == 5) {  // 64 x 256 (4 waves along N): outputs with 64 rows (no half-empty tiles)
    sx_launch_tile<64, 256, 6, true, false>(p, a_kmajor, b_kmajor, grid, st);
  } else if (tile == 6) {  // 256 x 64 (4 waves along M): outputs with 64 columns
    sx_launch_tile<256, 64, 6, true, false>(p, a_kmajor, b_kmajor, grid, st);
  } else if (tile == 3) {  // 4 waves of 128 x 64, one per SIMD, software-pipelined split
    sx_launch_tile<256, 128, 6, true, true, 1, 4>(p, a_kmajor, b_kmajor, grid, st);
  } else {                 // the same without the pipeline (A/B)
    sx_launch_tile<256, 128, 6, true, false, 1, 4>(p, a_kmajor, b_kmajor, grid, st);
  }
  check_launch();
  if (S > 1) {
    sx_reduce(p, st);
    if (bsum) {
      hipLaunchKernelGGL(sgemm_rowsum_reduce_kernel, dim3(unsigned((M + 255) / 256)), dim3(256), 0, st, p);
      check_launch();
    }
  }
}

// Convolution weight gradient dW[co][kh][kw][ci] (+)= sum over output pixels of dY[pix][co] *
// X[pix shifted by the tap][ci] as ONE implicit GEMM on the split-bf16 MFMA kernel: A = dY^T
// (K-major, [pixels][Cout]), B gathered from the NHWC input per tap (CONV operand), C = the
// channels_last filter gradient viewed [Cout][KH*KW*Cin] (ResNet-50 fp32: replaces MIOpen's
// igemm_wrw for the 3x3 layers with C >= 128, including the stride-2 ones).
void sgemm_conv_wgrad_f32(uintptr_t dy, uintptr_t x, uintptr_t gw, int n, int H, int W, int Cin, int Ho, int Wo,
                          int Cout, int KH, int KW, int stride, int pad, int splits, bool accumulate, uintptr_t ws,
                          int64_t ws_floats, uintptr_t stream, int tile) {
  VODA_CHECK(tile == 0 || tile == 8, "sgemm_conv_wgrad_f32: tile 0 (128 x 128) or 8 (64 x 192)");
  const int BM = tile == 8 ? 64 : 128, BN = tile == 8 ? 192 : 128;
  const int64_t K = int64_t(n) * Ho * Wo;
  const int N = KH * KW * Cin;
  VODA_CHECK(n > 0 && Cout > 0 && Cin > 0 && K > 0 && K < (int64_t(1) << 31), "sgemm_conv_wgrad_f32: bad shape");
  VODA_CHECK(K % kSxBK == 0, "sgemm_conv_wgrad_f32: output pixels must be a multiple of 16");
  VODA_CHECK(Cout % 4 == 0 && Cin % 4 == 0, "sgemm_conv_wgrad_f32: channels must be multiples of 4");
  VODA_CHECK(dy % 16 == 0 && x % 16 == 0, "sgemm_conv_wgrad_f32: operands need 16-B alignment");
  VODA_CHECK(Ho == (H + 2 * pad - KH) / stride + 1 && Wo == (W + 2 * pad - KW) / stride + 1,
             "sgemm_conv_wgrad_f32: output size mismatch");
  SxArgs p{};
  p.a = reinterpret_cast<const float*>(dy); p.lda = Cout;
  p.b = reinterpret_cast<const float*>(x); p.ldb = Cin;
  p.c = reinterpret_cast<float*>(gw); p.ldc = N;
  p.M = Cout; p.N = N; p.K = int(K);
  p.cn = n; p.ch = H; p.cw = W; p.cin = Cin; p.cho = Ho; p.cwo = Wo; p.cs = stride; p.cpad = pad; p.ckw = KW;
  const int kst = int(K / kSxBK);
  int S = splits < 1 ? 1 : splits;
  if (S > kst) S = kst;
  p.kps = ((kst + S - 1) / S) * kSxBK;
  S = int((K + p.kps - 1) / p.kps);
  p.S = S;
  p.tiles_n = (N + BN - 1) / BN;
  p.tiles = ((Cout + BM - 1) / BM) * p.tiles_n;
  p.beta = accumulate ? 1 : 0;
  p.stagger = g_sx_stagger;
  p.wmap = g_sx_wmap;
  if (S > 1) {
    VODA_CHECK(ws != 0 && ws_floats >= sgemm_f32_workspace_floats(Cout, N, S), "sgemm_conv_wgrad_f32: workspace too small");
    VODA_CHECK(gw % 16 == 0, "sgemm_conv_wgrad_f32: split-K output needs 16-B rows");
    p.ws = reinterpret_cast<float*>(ws);
  }
  const int64_t nwg = int64_t(p.tiles) * S;
  VODA_CHECK(nwg < (int64_t(1) << 31), "sgemm_conv_wgrad_f32: grid too large");
  hipStream_t st = as_stream(stream);
  if (tile == 8)  // 64 x 192: 64-channel layers (N = 9 x 64 = 3 tiles exactly), 3 waves of 64 x 64
    hipLaunchKernelGGL((sgemm_bf16x3_kernel<64, 192, true, true, 6, true, false, 2, 2, true>), dim3(unsigned(nwg)),
                       dim3(192), 0, st, p);
  else if (g_sx_conv_ws == 1)
    hipLaunchKernelGGL((sgemm_ws_kernel<true, true, true, 1, 2>), dim3(unsigned(nwg)), dim3(512), 0, st, p);
  else if (g_sx_conv_ws == 2)
    hipLaunchKernelGGL((sgemm_ws_kernel<true, true, true, 2, 2>), dim3(unsigned(nwg)), dim3(512), 0, st, p);
  else if (g_sx_conv_ws == 3)  // one accumulator at three workgroups per CU (as GEMM variant 8)
    hipLaunchKernelGGL((sgemm_bf16x3_kernel<128, 128, true, true, 6, false, false, 3, 2, true>), dim3(unsigned(nwg)),
                       dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL((sgemm_bf16x3_kernel<128, 128, true, true, 6, true, false, 2, 2, true>), dim3(unsigned(nwg)),
                       dim3(256), 0, st, p);
  check_launch();
  if (S > 1) sx_reduce(p, st);
}

// Convolution forward Y[pix][Cout] = sum_{tap, ci} X[pix shifted by the tap][ci] W[co][tap][ci] as ONE
// implicit GEMM on the split-bf16 MFMA kernel: A gathered per tap from the NHWC input (CONVA
// operand), B = the channels_last filter [Cout][KH*KW*Cin] (K-contiguous), C = the NHWC output
// (ResNet-50 fp32: the three stride-2 3x3 layers, which the Winograd kernel does not take).
void sgemm_conv_fwd_f32(uintptr_t x, uintptr_t w, uintptr_t y, int n, int H, int W, int Cin, int Ho, int Wo, int Cout,
                        int KH, int KW, int stride, int pad, uintptr_t stream) {
  const int64_t M = int64_t(n) * Ho * Wo;
  const int K = KH * KW * Cin;
  VODA_CHECK(n > 0 && Cout > 0 && Cin > 0 && M > 0 && M < (int64_t(1) << 31), "sgemm_conv_fwd_f32: bad shape");
  VODA_CHECK(Cin % kSxBK == 0, "sgemm_conv_fwd_f32: input channels must be a multiple of 16");
  VODA_CHECK(Cout % 4 == 0, "sgemm_conv_fwd_f32: output channels must be a multiple of 4");
  VODA_CHECK(x % 16 == 0 && w % 16 == 0 && y % 16 == 0, "sgemm_conv_fwd_f32: operands need 16-B alignment");
  VODA_CHECK(Ho == (H + 2 * pad - KH) / stride + 1 && Wo == (W + 2 * pad - KW) / stride + 1,
             "sgemm_conv_fwd_f32: output size mismatch");
  SxArgs p{};
  p.a = reinterpret_cast<const float*>(x); p.lda = Cin;
  p.b = reinterpret_cast<const float*>(w); p.ldb = K;
  p.c = reinterpret_cast<float*>(y); p.ldc = Cout;
  p.M = int(M); p.N = Cout; p.K = K;
  p.cn = n; p.ch = H; p.cw = W; p.cin = Cin; p.cho = Ho; p.cwo = Wo; p.cs = stride; p.cpad = pad; p.ckw = KW;
  p.S = 1;
  p.kps = K;
  p.tiles_n = (Cout + 127) / 128;
  p.tiles = int((M + 127) / 128) * p.tiles_n;
  p.stagger = g_sx_stagger;
  p.wmap = g_sx_wmap;
  if (g_sx_conv_fwd_v8)  // one accumulator at three workgroups per CU (as GEMM variant 8)
    hipLaunchKernelGGL((sgemm_bf16x3_kernel<128, 128, false, false, 6, false, false, 3, 2, false, 0, true>),
                       dim3(unsigned(p.tiles)), dim3(256), 0, as_stream(stream), p);
  else
    hipLaunchKernelGGL((sgemm_bf16x3_kernel<128, 128, false, false, 6, true, false, 2, 2, false, 0, true>),
                       dim3(unsigned(p.tiles)), dim3(256), 0, as_stream(stream), p);
  check_launch();
}

// One parity class (ph, pw) of the input gradient of a stride-2, pad-1 3x3 convolution:
//   dX[img][2i + ph][2j + pw][ci] = sum_{taps (th, tw) of the class} sum_co dY[img][i + th][j + tw][co] Wc[tap][co][ci]
// the class's taps are 1 (even) or 2 (odd) per dimension: even rows take kh = 1, odd rows kh = 2
// (th = 0) and kh = 0 (th = 1); Wc = [nth * ntw][Cout][Cin] holds W[:, :, kh, kw] of the class's taps
// in that order (ops/splitgemm.conv_dgrad_s2).  A = dY gathered per tap (CONVA, stride 1, no pad,
// zero past the map), B = Wc (K-major), C rows mapped onto the class's pixels of dX.
void sgemm_conv_dgrad_s2_class(uintptr_t dy, uintptr_t wc, uintptr_t dx, int n, int Ho, int Wo, int Cout, int H, int W,
                               int Cin, int ph, int pw, uintptr_t stream) {
  const int nth = ph ? 2 : 1, ntw = pw ? 2 : 1;
  const int hc = (H - ph + 1) / 2, wcn = (W - pw + 1) / 2;  // class rows / columns
  const int64_t M = int64_t(n) * hc * wcn;
  const int K = nth * ntw * Cout;
  VODA_CHECK(n > 0 && Cin > 0 && Cout > 0 && M > 0 && M < (int64_t(1) << 31), "sgemm_conv_dgrad_s2: bad shape");
  VODA_CHECK(Cout % kSxBK == 0 && Cin % 4 == 0, "sgemm_conv_dgrad_s2: Cout % 16 and Cin % 4 required");
  VODA_CHECK(Ho == (H - 1) / 2 + 1 && Wo == (W - 1) / 2 + 1, "sgemm_conv_dgrad_s2: output size mismatch");
  VODA_CHECK(hc <= Ho && wcn <= Wo && (ph == 0 || ph == 1) && (pw == 0 || pw == 1), "sgemm_conv_dgrad_s2: class");
  VODA_CHECK(dy % 16 == 0 && wc % 16 == 0 && dx % 16 == 0, "sgemm_conv_dgrad_s2: operands need 16-B alignment");
  SxArgs p{};
  p.a = reinterpret_cast<const float*>(dy); p.lda = Cout;
  p.b = reinterpret_cast<const float*>(wc); p.ldb = Cin;
  p.c = reinterpret_cast<float*>(dx); p.ldc = Cin;
  p.M = int(M); p.N = Cin; p.K = K;
  p.cn = n; p.ch = Ho; p.cw = Wo; p.cin = Cout; p.cho = hc; p.cwo = wcn; p.cs = 1; p.cpad = 0; p.ckw = ntw;
  p.omap = 1; p.oH = H; p.oW = W; p.oph = ph; p.opw = pw; p.ohc = hc; p.owc = wcn;
  p.S = 1;
  p.kps = K;
  p.tiles_n = (Cin + 127) / 128;
  p.tiles = int((M + 127) / 128) * p.tiles_n;
  p.stagger = g_sx_stagger;
  p.wmap = g_sx_wmap;
  if (g_sx_conv_fwd_v8)  // as the forward: one accumulator at three workgroups per CU
    hipLaunchKernelGGL((sgemm_bf16x3_kernel<128, 128, false, true, 6, false, false, 3, 2, false, 0, true>),
                     dim3(unsigned(p.tiles)), dim3(256), 0, as_stream(stream), p);
  else
    hipLaunchKernelGGL((sgemm_bf16x3_kernel<128, 128, false, true, 6, true, false, 2, 2, false, 0, true>),
                     dim3(unsigned(p.tiles)), dim3(256), 0, as_stream(stream), p);
  check_launch();
}

}  // namespace voda
