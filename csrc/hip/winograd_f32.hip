// Winograd F(2x2, 3x3) forward convolution, fp32, on the f32-input MFMA of gfx950
// (v_mfma_f32_32x32x2_f32), for ResNet-50's 3x3 stride-1 pad-1 layers in NHWC.
//
// A 2x2 output tile needs a 4x4 input patch d; per channel the patch is transformed to
// V = B^T d B, the filter to U = G g G^T, and the 16 products M = sum_ci V[p] U[p] (one GEMM per
// transform position p = 4r + c, over the input channels) are transformed back, Y = A^T M A.
// The 16 GEMMs do 16 x 2 x tiles x Cin x Cout FLOPs: 2.25x fewer than the direct convolution
// (the igemm MIOpen runs: 59.2 GF per ResNet-50 3x3 layer at batch 256).  Nothing transformed
// goes to HBM (unfused, the 4x-expanded V and M tensors would cost more traffic than the FLOPs
// save):
//   * a workgroup (4 waves) owns 32 consecutive tiles x 32 output channels;
//   * per 32-channel chunk every thread loads one tile's 4x4 patch of 4 channels (16 float4,
//     zero outside the image), transforms it in registers and writes V[p][tile][ci] to LDS;
//   * wave w owns positions 4w .. 4w+3: its MFMAs read V as 16-byte LDS rows (lane half h takes
//     ci = 8q + 4h + s for MFMA s = 0..3, the permuted-k order of conv1x1_f32.hip) and U as
//     16-byte global reads of the pre-transformed filter U[p][ci/8][co][ci%8] (L2-resident, <= 16 MB);
//   * after the last chunk the 16 accumulators of every (tile, channel) meet in LDS and each
//     thread applies A^T M A to four of them and stores the 2x2 outputs.
// The filter transform (wino_f23_filter) runs once per use; the weights change every step.
//
// SX (round 6): the 16 tile GEMMs at fp32 accuracy on the bf16 matrix cores
// (v_mfma_f32_32x32x16_bf16), the exact 3-way bf16 split of splitgemm.hip: the filter transform
// writes U split into hi / mid / lo bf16 planes ([p][plane][C/8][Co][8]); each wave reads its V
// fragment (8 consecutive channels of one tile, 2 x 16-B LDS reads) as fp32, splits it in registers
// and accumulates the six significant cross products (hh, hm, mh, hl, lh, mm) into one fp32
// accumulator per position: 6 x 32 cycles per 16 channels instead of 8 x 64 for the f32 MFMA.
// Staging, V layout, exchange and inverse transform are the f32 kernel's.
#include "common.h"
#include "ops.h"

#include <algorithm>

namespace voda {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 wmfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

typedef __bf16 wsx_bf16x8 __attribute__((ext_vector_type(8)));
typedef float wsx_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 wsx_bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t wsx_pack2(float a, float b) {  // one v_cvt_pk_bf16_f32 (RNE)
  const wsx_f32x2 f = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, wsx_bf16x2));
}
// exact split of 8 fp32 values into three bf16x8 planes (x == hi + mid + lo)
__device__ __forceinline__ void wsx_split8(const float4 v0, const float4 v1, uint4& h, uint4& m, uint4& l) {
  const float x[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  uint32_t hh[4], mm[4], ll[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    hh[i] = wsx_pack2(x[2 * i], x[2 * i + 1]);
    const float r0 = x[2 * i] - __uint_as_float(hh[i] << 16), r1 = x[2 * i + 1] - __uint_as_float(hh[i] & 0xffff0000u);
    mm[i] = wsx_pack2(r0, r1);
    const float q0 = r0 - __uint_as_float(mm[i] << 16), q1 = r1 - __uint_as_float(mm[i] & 0xffff0000u);
    ll[i] = wsx_pack2(q0, q1);
  }
  h = make_uint4(hh[0], hh[1], hh[2], hh[3]);
  m = make_uint4(mm[0], mm[1], mm[2], mm[3]);
  l = make_uint4(ll[0], ll[1], ll[2], ll[3]);
}
__device__ __forceinline__ f32x16 wsx_mfma(const uint4 a, const uint4 b, const f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(wsx_bf16x8, a), __builtin_bit_cast(wsx_bf16x8, b),
                                                 c, 0, 0, 0);
}

#ifndef WSX_PREFETCH
#define WSX_PREFETCH 1
#endif

constexpr int kWT = 32;           // tiles per workgroup
constexpr int kWN = 32;           // output channels per workgroup
constexpr int kWK = 32;           // input channels per chunk
constexpr int kWP = kWK + 4;      // LDS row pitch of V (floats)
constexpr int kWThreads = 256;

struct WinoArgs {
  const float* x;  // [N][H][W][C]
  const float* u;  // [16][C / 8][Co][8]; SX: bf16 [16][3][C / 8][Co][8]
  float* y;        // [N][H][W][Co]
  float* part;     // [2][G][Co] BN partial sums (sum, sum of squares) of y, or null
  int N, H, W, C, Co;
  int th, tw;      // tiles per column / row
  int64_t T;       // N * th * tw
  int G;           // workgroups along the tiles (gridDim.x); each walks tile blocks x, x + G, ...
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wino_patch_rsrc(const WinoArgs& a) {
  const float* base = a.x - (int64_t(a.W) + 1) * a.C;
  const int64_t bytes = (int64_t(a.N) * a.H * a.W * a.C + (int64_t(a.W) + 1) * a.C) * 4;
  const uint64_t pb = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(pb)), hi = __builtin_amdgcn_readfirstlane(uint32_t(pb >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uint64_t(hi) << 32) | lo), 0,
                                           __builtin_amdgcn_readfirstlane(int(bytes)), 0x00020000);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wino_u_rsrc(const WinoArgs& a) {
  const uint64_t pb = reinterpret_cast<uint64_t>(a.u);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(pb)), hi = __builtin_amdgcn_readfirstlane(uint32_t(pb >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uint64_t(hi) << 32) | lo), 0,
                                           __builtin_amdgcn_readfirstlane(int(int64_t(96) * a.C * a.Co)), 0x00020000);
}

// ONEPOS (SX only): the split tile GEMMs one position at a time (V split of one row, its 6 MFMAs,
// the next position's U prefetched: 12 + 12 registers instead of 24 + 24) -- the position-pair form
// runs at 256 VGPRs with 116 bytes of scratch per lane
template <bool SX, bool ONEPOS = false>
__global__ __launch_bounds__(kWThreads, 2) void wino_f23_fwd_kernel(WinoArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[16 * kWT * kWP];  // V chunk, then M exchange
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lc = lane & 31, lh = lane >> 5;
  const int co0 = blockIdx.y * kWN;
  const int64_t nblk = (a.T + kWT - 1) / kWT;

  // this thread's staging task: tile (tid >> 3) of the block, channels 4 * (tid & 7) .. + 3
  const int st = tid >> 3, sq = tid & 7;  // 8 lanes read one pixel's 32 channels: 128 contiguous bytes
  bool tok = false;
  int h0 = 0, w0 = 0;
  const float* xn = a.x;
  // SX: buffer loads of the patch (voffset + uniform soffset, zero-fill out of range) instead of
  // 16 hoisted 64-bit pointers.  The resource starts at pixel (-1, -1) of image 0, so every offset
  // of a (-1-padded) patch is >= 0; a pixel outside the image gets an out-of-range voffset.
  const __amdgpu_buffer_rsrc_t xr = wino_patch_rsrc(a);
  // SX: U fragments by buffer loads too: lane (lc, lh) reads 16 B at (lh * Co + lc) * 16 from a
  // wave-uniform (position, plane, 8-channel block, co0) origin
  const __amdgpu_buffer_rsrc_t ur = wino_u_rsrc(a);
  const uint32_t uvo = uint32_t((lh * a.Co + lc) * 16);
  uint32_t vb = 0, okm = 0;  // byte offset of the patch origin + 16 sq; validity bits 4i + j
  auto tile_setup = [&](int64_t blk) {
    const int64_t tg = blk * kWT + st;
    tok = tg < a.T;
    const int64_t tt = tok ? tg : 0;
    const int n = int(tt / (int64_t(a.th) * a.tw));
    const int trem = int(tt - int64_t(n) * a.th * a.tw);
    const int ty = trem / a.tw, tx = trem - (trem / a.tw) * a.tw;
    h0 = 2 * ty - 1;
    w0 = 2 * tx - 1;
    xn = a.x + int64_t(n) * a.H * a.W * a.C;
    if constexpr (SX) {
      vb = uint32_t(((int64_t(n) * a.H + h0 + 1) * a.W + w0 + 1) * a.C * 4 + 16 * sq);
      okm = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int hh = h0 + i, ww = w0 + j;
          okm |= uint32_t(tok && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W) << (4 * i + j);
        }
    }
  };
  // 4x4 patch (4 channels) of this thread's tile, chunk c0 (zero outside the image)
  float4 d[16];
  auto load_patch = [&](int c0) {
    if constexpr (SX) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t vo = (okm >> (4 * i + j)) & 1u ? vb : 0x80000000u;
          const int so = __builtin_amdgcn_readfirstlane(((i * a.W + j) * a.C + c0) * 4);
          const auto v = __builtin_amdgcn_raw_buffer_load_b128(xr, int(vo), so, 0);
          d[4 * i + j] = make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
                                     __uint_as_float(v[3]));
        }
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int hh = h0 + i, ww = w0 + j;
        const bool ok = tok && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
        d[4 * i + j] = ok ? *reinterpret_cast<const float4*>(xn + (int64_t(hh) * a.W + ww) * a.C + c0 + 4 * sq)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
      }
  };
  const int64_t ups = int64_t(a.Co) * a.C;  // floats per transform position of U
  float s1 = 0.f, s2 = 0.f;                 // BN statistics of channel co0 + (tid & 31)

  int64_t blk = blockIdx.x;
  if (blk < nblk) {
    tile_setup(blk);
    load_patch(0);
  }
  for (; blk < nblk; blk += a.G) {
    f32x16 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x16{};
    for (int c0 = 0; c0 < a.C; c0 += kWK) {
      // U rows of this wave's first position for the chunk (issued before the barriers; the next
      // position's rows load during the MFMAs of the current one)
      const float* ub = a.u + ((int64_t(4 * wave) * (a.C / 8) + c0 / 8) * a.Co + co0 + lc) * 8 + 4 * lh;
      const int64_t uq = int64_t(8) * a.Co;  // floats per 8-channel block of U
      float4 bp[2][kWK / 8], bq[2][kWK / 8];  // U of the current / next position pair
      // SX: bf16 U fragments (hi / mid / lo) of one (16-channel step, position pair): step
      // s = 2 kk + pair covers channels c0 + 16 kk .. + 15 of positions 4 wave + 2 pair + {0, 1}
      uint4 sp[2][3], sn[2][3];
      auto sx_uload = [&](int st, uint4 (&dst)[2][3]) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) {
            const int pos = 4 * wave + 2 * (st & 1) + j;
            const int so = __builtin_amdgcn_readfirstlane(
                int(((int64_t(pos * 3 + pl) * (a.C / 8) + c0 / 8 + 2 * (st >> 1)) * a.Co + co0) * 16));
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(ur, int(uvo), so, 0);
            dst[j][pl] = make_uint4(v[0], v[1], v[2], v[3]);
          }
      };
      if constexpr (SX) {
        sx_uload(0, sp);
      } else {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int q = 0; q < kWK / 8; ++q) bp[j][q] = *reinterpret_cast<const float4*>(ub + j * ups + q * uq);
      }
      // ---- V = B^T d B in registers, in place (rows, then columns)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 a0 = d[j], a1 = d[4 + j], a2 = d[8 + j], a3 = d[12 + j];
        d[j] = make_float4(a0.x - a2.x, a0.y - a2.y, a0.z - a2.z, a0.w - a2.w);
        d[4 + j] = make_float4(a1.x + a2.x, a1.y + a2.y, a1.z + a2.z, a1.w + a2.w);
        d[8 + j] = make_float4(a2.x - a1.x, a2.y - a1.y, a2.z - a1.z, a2.w - a1.w);
        d[12 + j] = make_float4(a1.x - a3.x, a1.y - a3.y, a1.z - a3.z, a1.w - a3.w);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float4 a0 = d[4 * i], a1 = d[4 * i + 1], a2 = d[4 * i + 2], a3 = d[4 * i + 3];
        d[4 * i] = make_float4(a0.x - a2.x, a0.y - a2.y, a0.z - a2.z, a0.w - a2.w);
        d[4 * i + 1] = make_float4(a1.x + a2.x, a1.y + a2.y, a1.z + a2.z, a1.w + a2.w);
        d[4 * i + 2] = make_float4(a2.x - a1.x, a2.y - a1.y, a2.z - a1.z, a2.w - a1.w);
        d[4 * i + 3] = make_float4(a1.x - a3.x, a1.y - a3.y, a1.z - a3.z, a1.w - a3.w);
      }
      __syncthreads();  // the previous chunk's V reads (or the previous block's M reads) are done
#pragma unroll
      for (int p = 0; p < 16; ++p) *reinterpret_cast<float4*>(lds + (p * kWT + st) * kWP + 4 * sq) = d[p];
      __syncthreads();
      // in flight during this chunk's MFMAs: the next chunk, or the next block's first chunk
      if (c0 + kWK < a.C) {
        load_patch(c0 + kWK);
      } else if (blk + a.G < nblk) {
        tile_setup(blk + a.G);
        load_patch(0);
      }
      if constexpr (SX && ONEPOS) {
        // ---- 8 sub-steps (16-channel half h, position j of the wave's four) x 6 products; the next
        // sub-step's U (3 planes) loads during the current one's MFMAs
        auto uload1 = [&](int q, uint4 (&dst)[3]) {
          const int pos = 4 * wave + (q & 3), hh = q >> 2;
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) {
            const int so = __builtin_amdgcn_readfirstlane(
                int(((int64_t(pos * 3 + pl) * (a.C / 8) + c0 / 8 + 2 * hh) * a.Co + co0) * 16));
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(ur, int(uvo), so, 0);
            dst[pl] = make_uint4(v[0], v[1], v[2], v[3]);
          }
        };
        auto sub = [&](int q, const uint4 (&u)[3]) {
          const float* vr = lds + ((4 * wave + (q & 3)) * kWT + lc) * kWP + 16 * (q >> 2) + 8 * lh;
          uint4 vh, vm, vl;
          wsx_split8(*reinterpret_cast<const float4*>(vr), *reinterpret_cast<const float4*>(vr + 4), vh, vm, vl);
          f32x16& r = acc[q & 3];
          r = wsx_mfma(vm, u[1], r);
          r = wsx_mfma(vh, u[2], r);
          r = wsx_mfma(vl, u[0], r);
          r = wsx_mfma(vh, u[1], r);
          r = wsx_mfma(vm, u[0], r);
          r = wsx_mfma(vh, u[0], r);
        };
        uint4 ua[3], ub[3];
        uload1(0, ua);
#pragma unroll
        for (int q = 0; q < 8; q += 2) {
          uload1(q + 1, ub);
          sub(q, ua);
          if (q + 2 < 8) uload1(q + 2, ua);
          sub(q + 1, ub);
        }
        continue;
      }
      if constexpr (SX) {
        // ---- 4 steps x 2 positions x 6 products of 32x32x16 bf16; the next step's U loads meanwhile
#pragma unroll
        for (int st = 0; st < 4; ++st) {
#if WSX_PREFETCH
          if (st < 3) sx_uload(st + 1, sn);
#else
          if (st > 0) sx_uload(st, sp);
#endif
          __builtin_amdgcn_sched_barrier(0);  // keep each step's V reads / splits with its MFMAs
          uint4 vh[2], vm[2], vl[2];
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const float* vr = lds + ((4 * wave + 2 * (st & 1) + j) * kWT + lc) * kWP + 16 * (st >> 1) + 8 * lh;
            wsx_split8(*reinterpret_cast<const float4*>(vr), *reinterpret_cast<const float4*>(vr + 4), vh[j], vm[j],
                       vl[j]);
          }
          f32x16& c0r = acc[2 * (st & 1)];
          f32x16& c1r = acc[2 * (st & 1) + 1];
          // small products first; the two positions' chains interleave
          c0r = wsx_mfma(vm[0], sp[0][1], c0r);
          c1r = wsx_mfma(vm[1], sp[1][1], c1r);
          c0r = wsx_mfma(vh[0], sp[0][2], c0r);
          c1r = wsx_mfma(vh[1], sp[1][2], c1r);
          c0r = wsx_mfma(vl[0], sp[0][0], c0r);
          c1r = wsx_mfma(vl[1], sp[1][0], c1r);
          c0r = wsx_mfma(vh[0], sp[0][1], c0r);
          c1r = wsx_mfma(vh[1], sp[1][1], c1r);
          c0r = wsx_mfma(vm[0], sp[0][0], c0r);
          c1r = wsx_mfma(vm[1], sp[1][0], c1r);
          c0r = wsx_mfma(vh[0], sp[0][0], c0r);
          c1r = wsx_mfma(vh[1], sp[1][0], c1r);
#if WSX_PREFETCH
          if (st < 3) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
              for (int pl = 0; pl < 3; ++pl) sp[j][pl] = sn[j][pl];
          }
#endif
        }
        continue;
      }
      // ---- 4 positions per wave: acc[j] (tiles x co) += V[p] (tiles x ci) . U[p] (ci x co), in
      // pairs of positions whose two MFMA chains interleave; the next pair's U loads meanwhile
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        if (pr == 0) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < kWK / 8; ++q) bq[j][q] = *reinterpret_cast<const float4*>(ub + (2 + j) * ups + q * uq);
        }
#pragma unroll
        for (int q = 0; q < kWK / 8; ++q) {
          const float4 a0 = *reinterpret_cast<const float4*>(lds + ((4 * wave + 2 * pr) * kWT + lc) * kWP + 8 * q + 4 * lh);
          const float4 a1 = *reinterpret_cast<const float4*>(lds + ((4 * wave + 2 * pr + 1) * kWT + lc) * kWP + 8 * q + 4 * lh);
          f32x16& c0r = acc[2 * pr];
          f32x16& c1r = acc[2 * pr + 1];
          c0r = wmfma(a0.x, bp[0][q].x, c0r);
          c1r = wmfma(a1.x, bp[1][q].x, c1r);
          c0r = wmfma(a0.y, bp[0][q].y, c0r);
          c1r = wmfma(a1.y, bp[1][q].y, c1r);
          c0r = wmfma(a0.z, bp[0][q].z, c0r);
          c1r = wmfma(a1.z, bp[1][q].z, c1r);
          c0r = wmfma(a0.w, bp[0][q].w, c0r);
          c1r = wmfma(a1.w, bp[1][q].w, c1r);
        }
        if (pr == 0) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < kWK / 8; ++q) bp[j][q] = bq[j][q];
        }
      }
    }
    __syncthreads();
    // ---- exchange: M[p][tile][co] (pitch 32) in LDS
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = 4 * wave + j;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
        lds[(p * kWT + row) * kWN + lc] = acc[j][r];
      }
    }
    __syncthreads();
    // ---- inverse transform: Y = A^T M A, thread -> channel tid & 31, tiles tid >> 5 + 8k
    const int co = tid & 31;
    const int64_t t0 = blk * kWT;
#pragma unroll
    for (int k = 0; k < kWT / 8; ++k) {
      const int tl = (tid >> 5) + 8 * k;
      const int64_t tgo = t0 + tl;
      if (tgo >= a.T) continue;
      float m[16];
#pragma unroll
      for (int p = 0; p < 16; ++p) m[p] = lds[(p * kWT + tl) * kWN + co];
      float r0[4], r1[4];  // A^T M: rows
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        r0[c] = m[c] + m[4 + c] + m[8 + c];
        r1[c] = m[4 + c] - m[8 + c] - m[12 + c];
      }
      const float y00 = r0[0] + r0[1] + r0[2], y01 = r0[1] - r0[2] - r0[3];
      const float y10 = r1[0] + r1[1] + r1[2], y11 = r1[1] - r1[2] - r1[3];
      const int no = int(tgo / (int64_t(a.th) * a.tw));
      const int rem = int(tgo - int64_t(no) * a.th * a.tw);
      const int oy = 2 * (rem / a.tw), ox = 2 * (rem - (rem / a.tw) * a.tw);
      float* yb = a.y + (int64_t(no) * a.H * a.W) * a.Co + co0 + co;
      const bool xr = ox + 1 < a.W, yr = oy + 1 < a.H;
      yb[(int64_t(oy) * a.W + ox) * a.Co] = y00;
      s1 += y00;
      s2 = fmaf(y00, y00, s2);
      if (xr) {
        yb[(int64_t(oy) * a.W + ox + 1) * a.Co] = y01;
        s1 += y01;
        s2 = fmaf(y01, y01, s2);
      }
      if (yr) {
        yb[(int64_t(oy + 1) * a.W + ox) * a.Co] = y10;
        s1 += y10;
        s2 = fmaf(y10, y10, s2);
        if (xr) {
          yb[(int64_t(oy + 1) * a.W + ox + 1) * a.Co] = y11;
          s1 += y11;
          s2 = fmaf(y11, y11, s2);
        }
      }
    }
  }
  if (a.part == nullptr) return;
  // BN partials of this workgroup: the 8 threads of each channel through LDS, one row per x block
  __syncthreads();
  float* red = lds;
  red[tid] = s1;
  red[kWThreads + tid] = s2;
  __syncthreads();
  if (tid < kWN) {
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int g = 0; g < kWThreads / kWN; ++g) {
      t1 += red[g * kWN + tid];
      t2 += red[kWThreads + g * kWN + tid];
    }
    a.part[int64_t(blockIdx.x) * a.Co + co0 + tid] = t1;
    a.part[int64_t(a.G) * a.Co + int64_t(blockIdx.x) * a.Co + co0 + tid] = t2;
  }
}

// ---------------------------------------------------------------------------------------------
// SX2 (round 6): the split-bf16 kernel above at 64 output channels per workgroup.  With 32, each
// wave splits a V fragment (8 fp32 -> 3 bf16 planes, ~44 VALU) for 6 MFMAs, ~7 VALU per MFMA:
// VALU-bound, and every 32-channel column of the grid re-loads and re-transforms the same patches.
// Here a workgroup is 8 waves over 32 tiles x 64 output channels: wave w owns positions 2w, 2w + 1
// and both 32-channel column tiles, so one split feeds 12 MFMAs (2 column tiles x 6 products), and
// the patch loads / transforms per output halve.  Staging: 16 lanes read one pixel's 32 channels
// (two per lane, 8-byte buffer loads); the M exchange runs in two 32-channel halves through the V
// buffer.  One workgroup per CU (8 waves, ~220 VGPRs each).
// ---------------------------------------------------------------------------------------------
constexpr int kW2N = 64;
constexpr int kW2Threads = 512;

__global__ __launch_bounds__(kW2Threads, 1) void wino_f23_fwd_sx2_kernel(WinoArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[16 * kWT * kWP];  // V chunk, then M exchange halves
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lc = lane & 31, lh = lane >> 5;
  const int co0 = blockIdx.y * kW2N;
  const int64_t nblk = (a.T + kWT - 1) / kWT;

  // staging task: tile (tid >> 4) of the block, channels 2 * (tid & 15) .. + 1 of the chunk
  const int st = tid >> 4, sq = tid & 15;
  const __amdgpu_buffer_rsrc_t xr = wino_patch_rsrc(a);
  const __amdgpu_buffer_rsrc_t ur = wino_u_rsrc(a);
  const uint32_t uvo = uint32_t((lh * a.Co + lc) * 16);
  uint32_t vb = 0, okm = 0;
  auto tile_setup = [&](int64_t blk) {
    const int64_t tg = blk * kWT + st;
    const bool tok = tg < a.T;
    const int64_t tt = tok ? tg : 0;
    const int n = int(tt / (int64_t(a.th) * a.tw));
    const int trem = int(tt - int64_t(n) * a.th * a.tw);
    const int ty = trem / a.tw, tx = trem - (trem / a.tw) * a.tw;
    const int h0 = 2 * ty - 1, w0 = 2 * tx - 1;
    vb = uint32_t(((int64_t(n) * a.H + h0 + 1) * a.W + w0 + 1) * a.C * 4 + 8 * sq);
    okm = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int hh = h0 + i, ww = w0 + j;
        okm |= uint32_t(tok && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W) << (4 * i + j);
      }
  };
  float2 d[16];
  auto load_patch = [&](int c0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t vo = (okm >> (4 * i + j)) & 1u ? vb : 0x80000000u;
        const int so = __builtin_amdgcn_readfirstlane(((i * a.W + j) * a.C + c0) * 4);
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(xr, int(vo), so, 0);
        d[4 * i + j] = make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
      }
  };
  // bf16 U fragments (hi / mid / lo) of one 16-channel step s and one column tile c for this
  // wave's two positions: dst[j][plane]
  auto uload = [&](int c0, int s, int c, uint4 (&dst)[2][3]) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        const int pos = 2 * wave + j;
        const int so = __builtin_amdgcn_readfirstlane(
            int(((int64_t(pos * 3 + pl) * (a.C / 8) + c0 / 8 + 2 * s) * a.Co + co0 + 32 * c) * 16));
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(ur, int(uvo), so, 0);
        dst[j][pl] = make_uint4(v[0], v[1], v[2], v[3]);
      }
  };
  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f};  // BN statistics of channels co0 + 32 h + (tid & 31)

  int64_t blk = blockIdx.x;
  if (blk < nblk) {
    tile_setup(blk);
    load_patch(0);
  }
  for (; blk < nblk; blk += a.G) {
    f32x16 acc[2][2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int c = 0; c < 2; ++c) acc[j][c] = f32x16{};
    for (int c0 = 0; c0 < a.C; c0 += kWK) {
      uint4 ua[2][3], ub[2][3];  // U of the current / next (step, column tile)
      uload(c0, 0, 0, ua);       // in flight across the transform and the barriers
      // ---- V = B^T d B in registers (rows, then columns)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float2 a0 = d[j], a1 = d[4 + j], a2 = d[8 + j], a3 = d[12 + j];
        d[j] = make_float2(a0.x - a2.x, a0.y - a2.y);
        d[4 + j] = make_float2(a1.x + a2.x, a1.y + a2.y);
        d[8 + j] = make_float2(a2.x - a1.x, a2.y - a1.y);
        d[12 + j] = make_float2(a1.x - a3.x, a1.y - a3.y);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float2 a0 = d[4 * i], a1 = d[4 * i + 1], a2 = d[4 * i + 2], a3 = d[4 * i + 3];
        d[4 * i] = make_float2(a0.x - a2.x, a0.y - a2.y);
        d[4 * i + 1] = make_float2(a1.x + a2.x, a1.y + a2.y);
        d[4 * i + 2] = make_float2(a2.x - a1.x, a2.y - a1.y);
        d[4 * i + 3] = make_float2(a1.x - a3.x, a1.y - a3.y);
      }
      __syncthreads();  // the previous chunk's V reads (or the previous block's M reads) are done
#pragma unroll
      for (int p = 0; p < 16; ++p) *reinterpret_cast<float2*>(lds + (p * kWT + st) * kWP + 2 * sq) = d[p];
      __syncthreads();
      if (c0 + kWK < a.C) {
        load_patch(c0 + kWK);
      } else if (blk + a.G < nblk) {
        tile_setup(blk + a.G);
        load_patch(0);
      }
      // ---- 2 steps x 2 column tiles x 2 positions x 6 products of 32x32x16 bf16; each V split
      // (per step and position) feeds both column tiles; the U of the next (step, column tile)
      // loads during the current one's MFMAs
      uint4 vh[2], vm[2], vl[2];
      auto split = [&](int s) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float* vr = lds + ((2 * wave + j) * kWT + lc) * kWP + 16 * s + 8 * lh;
          wsx_split8(*reinterpret_cast<const float4*>(vr), *reinterpret_cast<const float4*>(vr + 4), vh[j], vm[j],
                     vl[j]);
        }
      };
      auto mfmas = [&](int c, const uint4 (&u)[2][3]) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {  // small products first
          f32x16& r = acc[j][c];
          r = wsx_mfma(vm[j], u[j][1], r);
          r = wsx_mfma(vh[j], u[j][2], r);
          r = wsx_mfma(vl[j], u[j][0], r);
          r = wsx_mfma(vh[j], u[j][1], r);
          r = wsx_mfma(vm[j], u[j][0], r);
          r = wsx_mfma(vh[j], u[j][0], r);
        }
      };
      split(0);
      uload(c0, 0, 1, ub);
      mfmas(0, ua);
      uload(c0, 1, 0, ua);
      mfmas(1, ub);
      split(1);
      uload(c0, 1, 1, ub);
      mfmas(0, ua);
      mfmas(1, ub);
    }
    // ---- exchange + inverse transform, one 32-channel half at a time through the V buffer
    const int co = tid & 31;
    const int64_t t0 = blk * kWT;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      __syncthreads();  // V reads (hf 0) / the previous half's M reads (hf 1) are done
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int p = 2 * wave + j;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
          lds[(p * kWT + row) * 32 + lc] = acc[j][hf][r];
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kWT / 16; ++k) {
        const int tl = (tid >> 5) + 16 * k;
        const int64_t tgo = t0 + tl;
        if (tgo >= a.T) continue;
        float m[16];
#pragma unroll
        for (int p = 0; p < 16; ++p) m[p] = lds[(p * kWT + tl) * 32 + co];
        float r0[4], r1[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          r0[c] = m[c] + m[4 + c] + m[8 + c];
          r1[c] = m[4 + c] - m[8 + c] - m[12 + c];
        }
        const float y00 = r0[0] + r0[1] + r0[2], y01 = r0[1] - r0[2] - r0[3];
        const float y10 = r1[0] + r1[1] + r1[2], y11 = r1[1] - r1[2] - r1[3];
        const int no = int(tgo / (int64_t(a.th) * a.tw));
        const int rem = int(tgo - int64_t(no) * a.th * a.tw);
        const int oy = 2 * (rem / a.tw), ox = 2 * (rem - (rem / a.tw) * a.tw);
        float* yb = a.y + (int64_t(no) * a.H * a.W) * a.Co + co0 + 32 * hf + co;
        const bool xr2 = ox + 1 < a.W, yr2 = oy + 1 < a.H;
        yb[(int64_t(oy) * a.W + ox) * a.Co] = y00;
        s1[hf] += y00;
        s2[hf] = fmaf(y00, y00, s2[hf]);
        if (xr2) {
          yb[(int64_t(oy) * a.W + ox + 1) * a.Co] = y01;
          s1[hf] += y01;
          s2[hf] = fmaf(y01, y01, s2[hf]);
        }
        if (yr2) {
          yb[(int64_t(oy + 1) * a.W + ox) * a.Co] = y10;
          s1[hf] += y10;
          s2[hf] = fmaf(y10, y10, s2[hf]);
          if (xr2) {
            yb[(int64_t(oy + 1) * a.W + ox + 1) * a.Co] = y11;
            s1[hf] += y11;
            s2[hf] = fmaf(y11, y11, s2[hf]);
          }
        }
      }
    }
  }
  if (a.part == nullptr) return;
  // BN partials of this workgroup: the 16 threads of each channel through LDS
  __syncthreads();
  float* red = lds;
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    red[(2 * hf) * kW2Threads + tid] = s1[hf];
    red[(2 * hf + 1) * kW2Threads + tid] = s2[hf];
  }
  __syncthreads();
  if (tid < kW2N) {
    const int hf = tid >> 5, c = tid & 31;
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int g = 0; g < kW2Threads / 32; ++g) {
      t1 += red[(2 * hf) * kW2Threads + g * 32 + c];
      t2 += red[(2 * hf + 1) * kW2Threads + g * 32 + c];
    }
    a.part[int64_t(blockIdx.x) * a.Co + co0 + tid] = t1;
    a.part[int64_t(a.G) * a.Co + int64_t(blockIdx.x) * a.Co + co0 + tid] = t2;
  }
}

// U[p][co][ci] = (G g G^T)[p] for g = w[co][ci] (3x3, any strides); one thread per (co, ci).
// flip: the filter of the input gradient as a forward convolution, g = w[ci][co] rotated by 180
// degrees (w is the layer's [Cout][Cin] filter; here co runs over its Cin and ci over its Cout).
// SX: u is bf16 [p][plane][ci / 8][co][ci % 8], the exact hi / mid / lo split of each value.
template <bool SX>
__global__ __launch_bounds__(256) void wino_f23_filter_kernel(const float* __restrict__ w, int64_t s0, int64_t s1,
                                                              int64_t s2, int64_t s3, float* __restrict__ u, int Co,
                                                              int C, int flip) {
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= int64_t(Co) * C) return;
  const int co = int(i / C), ci = int(i - int64_t(co) * C);
  float g[3][3];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      g[r][c] = flip ? w[ci * s0 + co * s1 + (2 - r) * s2 + (2 - c) * s3] : w[co * s0 + ci * s1 + r * s2 + c * s3];
  float t[4][3];  // G g: G = [[1,0,0],[.5,.5,.5],[.5,-.5,.5],[0,0,1]]
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    t[0][c] = g[0][c];
    t[1][c] = 0.5f * (g[0][c] + g[1][c] + g[2][c]);
    t[2][c] = 0.5f * (g[0][c] - g[1][c] + g[2][c]);
    t[3][c] = g[2][c];
  }
  // layout [p][ci / 8][co][ci % 8]: a wave's U reads (32 channels co, one 8-channel block) are
  // 1 KB contiguous instead of 32 rows of C floats
  const int64_t pstride = int64_t(Co) * C;
  const int64_t o = (int64_t(ci >> 3) * Co + co) * 8 + (ci & 7);
#pragma unroll
  for (int r = 0; r < 4; ++r) {  // (G g) G^T
    const float v[4] = {t[r][0], 0.5f * (t[r][0] + t[r][1] + t[r][2]), 0.5f * (t[r][0] - t[r][1] + t[r][2]), t[r][2]};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if constexpr (SX) {
        uint16_t* ub = reinterpret_cast<uint16_t*>(u) + int64_t(4 * r + c) * 3 * pstride + o;
        const uint32_t h = wsx_pack2(v[c], 0.f);
        const float r1 = v[c] - __uint_as_float(h << 16);
        const uint32_t m = wsx_pack2(r1, 0.f);
        const float r2 = r1 - __uint_as_float(m << 16);
        const uint32_t l = wsx_pack2(r2, 0.f);
        ub[0] = uint16_t(h & 0xffffu);
        ub[pstride] = uint16_t(m & 0xffffu);
        ub[2 * pstride] = uint16_t(l & 0xffffu);
      } else {
        u[(4 * r + c) * pstride + o] = v[c];
      }
    }
  }
}

}  // namespace

int g_wino_onepos = 1;
void wino_f23_set_onepos(int on) { g_wino_onepos = on ? 1 : 0; }

bool wino_f23_supported(int C, int Co) { return C > 0 && Co > 0 && C % kWK == 0 && Co % kWN == 0; }

void wino_f23_filter(uintptr_t w, int64_t s0, int64_t s1, int64_t s2, int64_t s3, uintptr_t u, int Co, int C,
                     bool flip, bool sx, uintptr_t stream) {
  VODA_CHECK(Co > 0 && C > 0, "wino_f23_filter: empty filter");
  const int64_t n = int64_t(Co) * C;
  auto kern = sx ? wino_f23_filter_kernel<true> : wino_f23_filter_kernel<false>;
  hipLaunchKernelGGL(kern, dim3(unsigned((n + 255) / 256)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float*>(w), s0, s1, s2, s3, reinterpret_cast<float*>(u), Co, C,
                     int(flip));
  check_launch();
}

int wino_cus() {
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

// workgroups along the tiles; the BN partials have one row per such workgroup.  With 64 input
// channels (two chunks) a workgroup's fixed costs -- the first patch load, the exchange and the
// stores -- are as long as its MFMAs, so two workgroups per CU walk several 32-tile blocks each and
// prefetch the next block during the epilogue (499 vs 508 us per ResNet-50 stage-1 layer).  From
// 128 channels on one block per workgroup balances better: a persistent grid left a one-block tail
// (C = 256: 433 vs 402 us, profiles/r5/winograd_f23_vs_miopen.jsonl).
int wino_f23_groups(int N, int H, int W, int C, int Co) {
  const int64_t nblk = (int64_t(N) * ((H + 1) / 2) * ((W + 1) / 2) + kWT - 1) / kWT;
  if (C >= 128) return int(nblk);
  const int ncol = std::max(1, Co / kWN);
  return int(std::max<int64_t>(1, std::min<int64_t>(nblk, (2 * wino_cus() + ncol - 1) / ncol)));
}

void wino_f23_fwd(uintptr_t x, uintptr_t u, uintptr_t y, uintptr_t part, int N, int H, int W, int C, int Co, int G,
                  bool sx, uintptr_t stream) {
  VODA_CHECK(N > 0 && H > 0 && W > 0, "wino_f23_fwd: empty input");
  VODA_CHECK(wino_f23_supported(C, Co), "wino_f23_fwd: channels must be multiples of 32");
  VODA_CHECK(x % 16 == 0 && u % 16 == 0 && y % 4 == 0 && part % 4 == 0, "wino_f23_fwd: misaligned operands");
  VODA_CHECK(G == wino_f23_groups(N, H, W, C, Co), "wino_f23_fwd: group count mismatch");
  WinoArgs a{reinterpret_cast<const float*>(x), reinterpret_cast<const float*>(u), reinterpret_cast<float*>(y),
             reinterpret_cast<float*>(part), N, H, W, C, Co, (H + 1) / 2, (W + 1) / 2, 0, G};
  a.T = int64_t(N) * a.th * a.tw;
  const dim3 grid(unsigned(G), unsigned(Co / kWN));
  void (*kern)(WinoArgs) = sx ? (g_wino_onepos ? wino_f23_fwd_kernel<true, true> : wino_f23_fwd_kernel<true, false>)
                              : wino_f23_fwd_kernel<false, false>;
  hipLaunchKernelGGL(kern, grid, dim3(kWThreads), 0,
                     as_stream(stream), a);
  check_launch();
}

// SX2: 64 output channels and one 8-wave workgroup per CU; with 64 input channels the persistent
// walk keeps one workgroup per CU, from 128 on one block per workgroup (as wino_f23_groups)
bool wino_f23_sx2_supported(int C, int Co) { return C > 0 && Co > 0 && C % kWK == 0 && Co % kW2N == 0; }

int wino_f23_groups2(int N, int H, int W, int C, int Co) {
  const int64_t nblk = (int64_t(N) * ((H + 1) / 2) * ((W + 1) / 2) + kWT - 1) / kWT;
  if (C >= 128) return int(nblk);
  const int ncol = std::max(1, Co / kW2N);
  return int(std::max<int64_t>(1, std::min<int64_t>(nblk, (wino_cus() + ncol - 1) / ncol)));
}

void wino_f23_fwd2(uintptr_t x, uintptr_t u, uintptr_t y, uintptr_t part, int N, int H, int W, int C, int Co, int G,
                   uintptr_t stream) {
  VODA_CHECK(N > 0 && H > 0 && W > 0, "wino_f23_fwd2: empty input");
  VODA_CHECK(wino_f23_sx2_supported(C, Co), "wino_f23_fwd2: channels must be multiples of 32 (in) / 64 (out)");
  VODA_CHECK(x % 16 == 0 && u % 16 == 0 && y % 4 == 0 && part % 4 == 0, "wino_f23_fwd2: misaligned operands");
  VODA_CHECK(G == wino_f23_groups2(N, H, W, C, Co), "wino_f23_fwd2: group count mismatch");
  WinoArgs a{reinterpret_cast<const float*>(x), reinterpret_cast<const float*>(u), reinterpret_cast<float*>(y),
             reinterpret_cast<float*>(part), N, H, W, C, Co, (H + 1) / 2, (W + 1) / 2, 0, G};
  a.T = int64_t(N) * a.th * a.tw;
  const dim3 grid(unsigned(G), unsigned(Co / kW2N));
  hipLaunchKernelGGL(wino_f23_fwd_sx2_kernel, grid, dim3(kW2Threads), 0, as_stream(stream), a);
  check_launch();
}

}  // namespace voda
