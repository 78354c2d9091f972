// Scaled + masked row softmax, forward and backward (CDNA4 / gfx950).
//
// Mirrors the vendored Keras MultiHeadAttention masked softmax used by the reference
// Transformer workload: softmax(scale * S + (1 - mask) * -1e9) with a padding mask and
// a causal mask (reference examples/py/tensorflow2/layers_tf25.py:421-463,
// advanced_activations_tf25.py:300-318, neural_machine_translation_with_transformer.py
// :263-295).  It is the generic path for attention shapes the fused MFMA attention
// kernel does not cover.  One wave64 per row, the row held in registers, one HBM read
// and one write per element; the masked logits are computed on the fly from an
// optional [B, Tq|1, S] key mask (nonzero = keep) and a causal flag.
#include "common.h"
#include "ops.h"

namespace voda {

struct SoftmaxShape {
  int64_t rows;       // B * H * Tq
  int S;              // row length (keys)
  int H, Tq;          // to decode (b, q) from the row index
  int64_t mask_bstride, mask_qstride;  // element strides of the keep-mask (q stride 0 = broadcast)
  int causal;
  float scale;
};

template <typename T, typename MT, int MAXITER>
__global__ __launch_bounds__(256) void softmax_fwd_kernel(const T* __restrict__ x, const MT* __restrict__ mask,
                                                          T* __restrict__ y, SoftmaxShape sh) {
  const int lane = threadIdx.x & 63;
  const int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= sh.rows) return;
  const int q = int(row % sh.Tq);
  const int64_t b = row / (int64_t(sh.Tq) * sh.H);
  const int S4 = sh.S >> 2;
  const int causal_lim = q + (sh.S - sh.Tq);  // keys > causal_lim are masked
  float4 v[MAXITER];
  float m = -INFINITY;
#pragma unroll
  for (int it = 0; it < MAXITER; ++it) {
    const int c4 = it * 64 + lane;
    if (c4 < S4) {
      float4 t = Vec4<T>::load(x + row * sh.S, c4);
      float e[4] = {t.x * sh.scale, t.y * sh.scale, t.z * sh.scale, t.w * sh.scale};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int col = c4 * 4 + k;
        bool keep = !(sh.causal && col > causal_lim);
        if (mask) keep = keep && (Vec4<MT>::load1(mask, b * sh.mask_bstride + int64_t(q) * sh.mask_qstride + col) != 0.f);
        if (!keep) e[k] = -1e9f;  // same additive constant as the Keras reference
        m = fmaxf(m, e[k]);
      }
      v[it] = make_float4(e[0], e[1], e[2], e[3]);
    } else {
      v[it] = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    }
  }
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int it = 0; it < MAXITER; ++it) {
    v[it].x = __expf(v[it].x - m); v[it].y = __expf(v[it].y - m);
    v[it].z = __expf(v[it].z - m); v[it].w = __expf(v[it].w - m);
    s += (v[it].x + v[it].y) + (v[it].z + v[it].w);
  }
  const float inv = 1.f / wave_sum(s);
#pragma unroll
  for (int it = 0; it < MAXITER; ++it) {
    const int c4 = it * 64 + lane;
    if (c4 < S4)
      Vec4<T>::store(y + row * sh.S, c4, make_float4(v[it].x * inv, v[it].y * inv, v[it].z * inv, v[it].w * inv));
  }
}

// dx = scale * y * (dy - sum(dy * y))
template <typename T, int MAXITER>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const T* __restrict__ y, const T* __restrict__ dy,
                                                          T* __restrict__ dx, int64_t rows, int S, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int S4 = S >> 2;
  float4 yv[MAXITER], dv[MAXITER];
  float s = 0.f;
#pragma unroll
  for (int it = 0; it < MAXITER; ++it) {
    const int c4 = it * 64 + lane;
    if (c4 < S4) {
      yv[it] = Vec4<T>::load(y + row * S, c4);
      dv[it] = Vec4<T>::load(dy + row * S, c4);
      s += (yv[it].x * dv[it].x + yv[it].y * dv[it].y) + (yv[it].z * dv[it].z + yv[it].w * dv[it].w);
    } else {
      yv[it] = dv[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  s = wave_sum(s);
#pragma unroll
  for (int it = 0; it < MAXITER; ++it) {
    const int c4 = it * 64 + lane;
    if (c4 < S4) {
      float4 o;
      o.x = scale * yv[it].x * (dv[it].x - s);
      o.y = scale * yv[it].y * (dv[it].y - s);
      o.z = scale * yv[it].z * (dv[it].z - s);
      o.w = scale * yv[it].w * (dv[it].w - s);
      Vec4<T>::store(dx + row * S, c4, o);
    }
  }
}

#define SM_DISPATCH_ITER(S, ...)                                  \
  [&] {                                                           \
    const int _it = (S + 255) / 256;                              \
    if (_it <= 1) { constexpr int MI = 1; __VA_ARGS__(); }        \
    else if (_it <= 2) { constexpr int MI = 2; __VA_ARGS__(); }   \
    else if (_it <= 4) { constexpr int MI = 4; __VA_ARGS__(); }   \
    else { constexpr int MI = 8; __VA_ARGS__(); }                 \
  }()

#define SM_DISPATCH_T(DT, ...)                                    \
  [&] {                                                           \
    if (DT == kF32) { using T = float; __VA_ARGS__(); }           \
    else if (DT == kBF16) { using T = BF16; __VA_ARGS__(); }      \
    else { using T = F16; __VA_ARGS__(); }                        \
  }()

void masked_softmax_fwd(uintptr_t x, uintptr_t mask, int mask_dt, uintptr_t y, int64_t B, int H, int Tq, int S,
                        int64_t mask_bstride, int64_t mask_qstride, bool causal, float scale, int dt,
                        uintptr_t stream) {
  VODA_CHECK(S > 0 && S % 4 == 0 && S <= kSoftmaxMaxS, "masked_softmax: S must be a multiple of 4 and <= 2048");
  SoftmaxShape sh{B * H * Tq, S, H, Tq, mask_bstride, mask_qstride, causal ? 1 : 0, scale};
  if (sh.rows == 0) return;
  const unsigned grid = unsigned((sh.rows + 3) / 4);
  SM_DISPATCH_T(dt, [&] {
    SM_DISPATCH_ITER(S, [&] {
      if (mask_dt == kF32 || mask == 0) {
        hipLaunchKernelGGL((softmax_fwd_kernel<T, float, MI>), dim3(grid), dim3(256), 0, as_stream(stream),
                           reinterpret_cast<const T*>(x), reinterpret_cast<const float*>(mask),
                           reinterpret_cast<T*>(y), sh);
      } else if (mask_dt == kBF16) {
        hipLaunchKernelGGL((softmax_fwd_kernel<T, BF16, MI>), dim3(grid), dim3(256), 0, as_stream(stream),
                           reinterpret_cast<const T*>(x), reinterpret_cast<const BF16*>(mask),
                           reinterpret_cast<T*>(y), sh);
      } else {
        hipLaunchKernelGGL((softmax_fwd_kernel<T, F16, MI>), dim3(grid), dim3(256), 0, as_stream(stream),
                           reinterpret_cast<const T*>(x), reinterpret_cast<const F16*>(mask),
                           reinterpret_cast<T*>(y), sh);
      }
    });
  });
  check_launch();
}

void masked_softmax_bwd(uintptr_t y, uintptr_t dy, uintptr_t dx, int64_t rows, int S, float scale, int dt,
                        uintptr_t stream) {
  VODA_CHECK(S > 0 && S % 4 == 0 && S <= kSoftmaxMaxS, "masked_softmax: S must be a multiple of 4 and <= 2048");
  if (rows == 0) return;
  const unsigned grid = unsigned((rows + 3) / 4);
  SM_DISPATCH_T(dt, [&] {
    SM_DISPATCH_ITER(S, [&] {
      hipLaunchKernelGGL((softmax_bwd_kernel<T, MI>), dim3(grid), dim3(256), 0, as_stream(stream),
                         reinterpret_cast<const T*>(y), reinterpret_cast<const T*>(dy), reinterpret_cast<T*>(dx),
                         rows, S, scale);
    });
  });
  check_launch();
}

}  // namespace voda
