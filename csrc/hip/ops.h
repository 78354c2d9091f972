// Host-side entry points of the _vodahip extension (all launches are stream-ordered).
#pragma once

#include <cstdint>
#include <cstring>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

struct ncclComm;
typedef struct ncclComm* ncclComm_t;

namespace voda {

constexpr int kLayerNormMaxN = 4096;
constexpr int kSoftmaxMaxS = 2048;

// ---- fused optimizers (optim.hip) ----
void sgd_step(uintptr_t p, uintptr_t g, int g_dtype, uintptr_t mom_buf, uintptr_t p_lp, int lp_dtype, int64_t n,
              float lr, float momentum, float dampening, float wd, bool nesterov, bool first_step, float grad_scale,
              uintptr_t stream);
void adam_step(uintptr_t p, uintptr_t g, int g_dtype, uintptr_t m, uintptr_t v, uintptr_t p_lp, int lp_dtype,
               int64_t n, float lr, float beta1, float beta2, float eps, float wd, bool adamw, int64_t step,
               float grad_scale, uintptr_t step_ptr, uintptr_t stream);
void rmsprop_step(uintptr_t p, uintptr_t g, int g_dtype, uintptr_t sq, uintptr_t mom_buf, uintptr_t gavg,
                  uintptr_t p_lp, int lp_dtype, int64_t n, float lr, float alpha, float eps, float wd, float momentum,
                  bool centered, float grad_scale, uintptr_t stream);

// ---- bucket pack / cast (bucket.hip) ----
void cast_scale(uintptr_t src, int src_dt, uintptr_t dst, int dst_dt, int64_t n, float scale, uintptr_t stream);
void multi_tensor_copy(const std::vector<uintptr_t>& srcs, const std::vector<uintptr_t>& dsts,
                       const std::vector<int64_t>& ns, int src_dt, int dst_dt, float scale, uintptr_t stream);

// ---- Adasum segmented pairwise combine (adasum.hip) ----
void adasum_combine(uintptr_t a, uintptr_t b, uintptr_t out, int dt, uintptr_t meta, int64_t nblk, int64_t nseg,
                    uintptr_t partials, uintptr_t stream);

// ---- Linear weight-gradient GEMM + fused bias gradient, split-K MFMA (wgrad.hip) ----
int64_t wgrad_conv_workspace_floats(int M, int Cout, int Cin, int taps, int splits);
void wgrad_conv(uintptr_t dy, uintptr_t x, uintptr_t dw, int Nimg, int H, int W, int Cin, int Ho, int Wo, int Cout,
                int KH, int KW, int stride, int pad, int splits, uintptr_t ws, bool accumulate, uintptr_t zero,
                int out_dt, uintptr_t stream);
int64_t wgrad_workspace_floats(int M, int N, int K, int splits);
void wgrad_gemm(uintptr_t dy, int64_t ldy, uintptr_t x, int64_t ldx, uintptr_t dw, int64_t ldw, uintptr_t db, int M,
                int N, int K, int splits, uintptr_t ws, bool accumulate, uintptr_t zero, int variant,
                int out_dt, uintptr_t stream);

// ---- tanh GELU (activation.hip); bwd may run in place (dh == dy) ----
void gelu_tanh_fwd(uintptr_t h, uintptr_t y, int64_t n, int dt, uintptr_t stream);
void gelu_tanh_bwd(uintptr_t h, uintptr_t dy, uintptr_t dh, int64_t n, int dt, uintptr_t stream);

// ---- LayerNorm (layernorm.hip) ----
void layernorm_fwd(uintptr_t x, uintptr_t gamma, uintptr_t beta, uintptr_t y, uintptr_t mean, uintptr_t rstd,
                   int64_t M, int N, float eps, int dt, int wdt, uintptr_t residual, uintptr_t sum, uintptr_t stream);
int layernorm_bwd_partial_rows(int64_t M);
void layernorm_set_bwd_waves(int w);
void layernorm_bwd(uintptr_t dy, uintptr_t x, uintptr_t mean, uintptr_t rstd, uintptr_t gamma, uintptr_t dx,
                   uintptr_t dgamma, uintptr_t dbeta, uintptr_t workspace, int64_t M, int N, int dt, int wdt,
                   bool accumulate, uintptr_t stream,
                   uintptr_t dbias_in = 0);

// ---- fused softmax cross-entropy (xent.hip) ----
// logits [rows][ld] (bf16 / fp32, 16-byte rows), V <= ld valid classes; per-row lse / loss /
// correct (fp32); labels int64, ``ignore`` rows contribute 0.  Backward: dx (same layout) =
// (*scale) * (softmax - onehot) over the V classes, 0 in the padding columns.
void xent_fwd(uintptr_t x, int64_t rows, int64_t ld, int V, int dt, uintptr_t labels, int64_t ignore, uintptr_t lse,
              uintptr_t loss, uintptr_t correct, uintptr_t stream);
void xent_bwd(uintptr_t x, uintptr_t dx, int64_t rows, int64_t ld, int V, int dt, uintptr_t labels, int64_t ignore,
              uintptr_t lse, uintptr_t scale, uintptr_t stream);

// ---- masked softmax (softmax.hip) ----
void masked_softmax_fwd(uintptr_t x, uintptr_t mask, int mask_dt, uintptr_t y, int64_t B, int H, int Tq, int S,
                        int64_t mask_bstride, int64_t mask_qstride, bool causal, float scale, int dt,
                        uintptr_t stream);
void masked_softmax_bwd(uintptr_t y, uintptr_t dy, uintptr_t dx, int64_t rows, int S, float scale, int dt,
                        uintptr_t stream);

// ---- fused BatchNorm(+add)(+ReLU), channels_last [M][C] (batchnorm.hip) ----
int64_t bn_workspace_floats(int64_t M, int C);
// reduction-pass tuning (deep unroll, grid cap, sweep order); negative = unchanged.  Not
// thread-safe against concurrent BN launches: set it before a run (tests, A/B benchmarks).
void bn_set_tuning(int deep, int blocks, int sweep);
std::vector<int> bn_get_tuning();
void bn_fwd_train(uintptr_t x, uintptr_t residual, uintptr_t gamma, uintptr_t beta, uintptr_t running_mean,
                  uintptr_t running_var, uintptr_t save_mean, uintptr_t save_invstd, uintptr_t y, uintptr_t mask,
                  uintptr_t workspace, int64_t M, int C, float eps, float momentum, bool relu, int dt,
                  uintptr_t stream, int pre_nb = 0);
void bn_apply(uintptr_t x, uintptr_t residual, uintptr_t ab, uintptr_t y, int64_t M, int C, bool relu, int dt,
              uintptr_t stream);
void bn_bwd(uintptr_t dy, uintptr_t mask, uintptr_t x, uintptr_t save_mean, uintptr_t save_invstd, uintptr_t gamma,
            uintptr_t dx, uintptr_t dres, uintptr_t dgamma, uintptr_t dbeta, uintptr_t workspace, int64_t M, int C,
            bool relu, bool accumulate, int dt, uintptr_t stream, uintptr_t pre_part = 0, int pre_nb = 0);
// dual BN relu?(bn(x) + bn2(x2)) (ResNet downsample blocks): one apply pass forward, one reduce +
// one apply pass backward for both BatchNorms (workspace = bn2_workspace_floats; the forward's
// two workspaces are bn_workspace_floats each, or a producing GEMM's statistics, pre_nb > 0)
int64_t bn2_workspace_floats(int64_t M, int C);
void bn2_fwd_train(uintptr_t x, uintptr_t x2, uintptr_t gamma, uintptr_t beta, uintptr_t running_mean,
                   uintptr_t running_var, uintptr_t save_mean, uintptr_t save_invstd, uintptr_t gamma2, uintptr_t beta2,
                   uintptr_t running_mean2, uintptr_t running_var2, uintptr_t save_mean2, uintptr_t save_invstd2,
                   uintptr_t y, uintptr_t mask, uintptr_t workspace, uintptr_t workspace2, int64_t M, int C, float eps,
                   float momentum, bool relu, int dt, uintptr_t stream, int pre_nb, int pre_nb2);
void bn2_bwd(uintptr_t dy, uintptr_t mask, uintptr_t x, uintptr_t x2, uintptr_t save_mean, uintptr_t save_invstd,
             uintptr_t gamma, uintptr_t save_mean2, uintptr_t save_invstd2, uintptr_t gamma2, uintptr_t dx,
             uintptr_t dx2, uintptr_t dgamma, uintptr_t dbeta, uintptr_t dgamma2, uintptr_t dbeta2,
             uintptr_t workspace, int64_t M, int C, bool relu, bool accumulate, int dt, uintptr_t stream, uintptr_t pre_part = 0,
             int pre_nb = 0);

// ---- fp32 1x1 conv GEMMs on the f32 MFMA: forward + BN statistics, split-K weight gradient
// (conv1x1_f32.hip) ----
bool gemm_f32_stats_supported(int64_t M, int N, int K);
int gemm_f32_stats_groups(int64_t M, int N, int K);
// w: [N][K], or [K][N] with w_kn (the input gradient dX = dY . W with W [Cout][Cin] as stored)
void gemm_f32_stats(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t part, int64_t M, int N, int K, int G,
                    uintptr_t stream, bool accumulate, bool w_kn);
// dX = dY . W (W stored [K = Cout][N = Cin]) + dout * relu-bits(cmask); with nsums = 2 / 3 also the
// downstream BN's backward partial sums (sum g, sum g*s1 [, sum g*s2], g = dX * bits(smask)) into
// part[nsums][G][N] (conv1x1_f32.hip gemm_f32_dgrad_bn_kernel)
bool gemm_f32_dgrad_bn_supported(int64_t M, int N, int K);
int gemm_f32_dgrad_bn_groups(int64_t M, int N, int K, int nsums);
void gemm_f32_dgrad_bn(uintptr_t dy, uintptr_t w, uintptr_t y, uintptr_t cg, uintptr_t cmask, uintptr_t smask,
                       uintptr_t s1, uintptr_t s2, uintptr_t part, int64_t M, int N, int K, int G, int nsums,
                       uintptr_t stream);

// ---- hipBLASLt GEMMs with GELU epilogues for the transformer FFN (blaslt_epi.cpp); dt: kF32 /
// kBF16 ----
int gemm_epilogue_algos(int epi, int dt, bool trans_a, int64_t m, int64_t n, int64_t k);
void gemm_gelu_aux(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t h, uintptr_t y, int64_t M, int64_t N,
                   int64_t K, int dt, uintptr_t ws, int64_t ws_bytes, uintptr_t stream);
void gemm_dgelu(uintptr_t dy, uintptr_t w, uintptr_t h, uintptr_t dh, int64_t M, int64_t N, int64_t K, int dt,
                uintptr_t ws, int64_t ws_bytes, uintptr_t stream);

// ---- 1x1 conv forward GEMM with BN statistics in the epilogue (gemm_bnstats.hip) ----
bool gemm_bnstats_supported(int64_t M, int N, int K);
int gemm_bnstats_groups(int64_t M, int N, int K);
void gemm_bnstats(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t part, int64_t M, int N, int K, int G,
                  uintptr_t stream, bool accumulate = false);

// ---- 3x3 / stride-1 conv weight gradient at 64 -> 64 channels (conv3x3_c64.hip) ----
int64_t conv3x3_c64_wgrad_workspace_floats(int N, int H);
bool wino_f23_supported(int C, int Co);
void wino_f23_filter(uintptr_t w, int64_t s0, int64_t s1, int64_t s2, int64_t s3, uintptr_t u, int Co, int C,
                     bool flip, bool sx, uintptr_t stream);
int wino_f23_groups(int N, int H, int W, int C, int Co);
bool wino_f23_sx2_supported(int C, int Co);
void wino_f23_set_onepos(int on);
int wino_f23_groups2(int N, int H, int W, int C, int Co);
void wino_f23_fwd2(uintptr_t x, uintptr_t u, uintptr_t y, uintptr_t part, int N, int H, int W, int C, int Co, int G,
                   uintptr_t stream);
void wino_f23_fwd(uintptr_t x, uintptr_t u, uintptr_t y, uintptr_t part, int N, int H, int W, int C, int Co, int G,
                  bool sx, uintptr_t stream);
void filter_flip_t(uintptr_t w, int in_dt, int64_t s0, int64_t s1, int64_t s2, int64_t s3, uintptr_t out,
                   int out_dt, int Cout, int Cin, int K, uintptr_t stream);
void conv3x3_c64_wgrad(uintptr_t x, uintptr_t dy, uintptr_t dw, int64_t s0, int64_t s1, int64_t s2, int64_t s3,
                       uintptr_t ws, int N, int H, int W, bool accumulate, int out_dt, uintptr_t stream,
                       int in_dt);  // in_dt: bf16 or fp32 activations

// ---- stride-s pixel subsampling of channels_last bf16 (gather, or dx[::s, ::s] += g) (pool.hip) ----
void subsample2d(uintptr_t src, uintptr_t dst, int N, int H, int W, int C, int s, bool add, int dt, uintptr_t stream);

// ---- global average pool backward, channels_last (pool.hip) ----
void global_avgpool_bwd(uintptr_t g, uintptr_t dx, int N, int HW, int C, float scale, int g_dt, int dt,
                        uintptr_t stream);

// ---- ResNet stem: 7x7/2 convolution + BN statistics (stem.hip) ----
int stem_partial_rows(int N, int Ho);
void stem_pack(uintptr_t x, uintptr_t x4, int N, int C, int H, int W, int64_t sN, int64_t sC, int64_t sH, int64_t sW,
               int dt, uintptr_t stream);
int64_t stem_wgrad_workspace_floats(int N, int Ho);
void stem_conv_wgrad(uintptr_t x4, uintptr_t dy, uintptr_t dw, int64_t s0, int64_t s1, int64_t s2, int64_t s3,
                     int Cin, uintptr_t ws, int N, int H, int W, int Ho, int Wo, bool accumulate, int out_dt,
                     uintptr_t stream);
// fp32 stem (stem_f32.hip): the image read through its strides (1..3 channels), [N][Ho][Wo][64] fp32
void stem_conv_fwd_f32(uintptr_t x, int64_t sN, int64_t sC, int64_t sH, int64_t sW, int Cin, uintptr_t w,
                       int64_t sw0, int64_t sw1, int64_t sw2, int64_t sw3, uintptr_t y, uintptr_t part, int nb, int N,
                       int H, int W, int Ho, int Wo, uintptr_t stream);
int64_t stem_wgrad_f32_workspace_floats(int N, int Ho);
bool stem_wgrad_f32_supported(int Wo);
void stem_conv_wgrad_f32(uintptr_t x, int64_t sN, int64_t sC, int64_t sH, int64_t sW, int Cin, uintptr_t dy,
                         uintptr_t dw, int64_t s0, int64_t s1, int64_t s2, int64_t s3, uintptr_t ws, int N, int H,
                         int W, int Ho, int Wo, bool accumulate, uintptr_t stream);
void stem_conv_fwd(uintptr_t x4, uintptr_t w, int64_t sw0, int64_t sw1, int64_t sw2, int64_t sw3, int Cin, int Cout,
                   uintptr_t y, uintptr_t part, int nb, int N, int H, int W, int Ho, int Wo, uintptr_t stream);

// ---- ResNet stem: BN(train) + ReLU + max pool fused (batchnorm.hip); pre_nb > 0: the
// workspace already holds pre_nb partial rows of sum / sum of squares (stem_conv_fwd) ----
int64_t bn_pool_workspace_floats(int N, int H, int C);
void bn_pool_fwd_train(uintptr_t x, uintptr_t gamma, uintptr_t beta, uintptr_t running_mean, uintptr_t running_var,
                       uintptr_t save_mean, uintptr_t save_invstd, uintptr_t y, uintptr_t idx, uintptr_t workspace,
                       int N, int H, int W, int C, int Ho, int Wo, int k, int s, int p, float eps, float momentum,
                       int dt, uintptr_t stream, int pre_nb = 0);
void bn_pool_bwd(uintptr_t dy, uintptr_t idx, uintptr_t x, uintptr_t save_mean, uintptr_t save_invstd,
                 uintptr_t gamma, uintptr_t dx, uintptr_t dgamma, uintptr_t dbeta, uintptr_t workspace, int N, int H,
                 int W, int C, int Ho, int Wo, int k, int s, int p, bool accumulate, int dt, uintptr_t stream);

// ---- NHWC max pooling with argmax bytes + gather backward (pool.hip) ----
void maxpool2d_fwd(uintptr_t x, uintptr_t y, uintptr_t idx, int N, int H, int W, int C, int Ho, int Wo, int k, int s,
                   int p, int dt, uintptr_t stream);
void maxpool2d_bwd(uintptr_t dy, uintptr_t idx, uintptr_t dx, int N, int H, int W, int C, int Ho, int Wo, int k, int s,
                   int p, int dt, uintptr_t stream);

// ---- Linear backward helpers (dense.hip) ----
int64_t colsum_workspace_floats(int64_t M, int N);
void colsum_accumulate(uintptr_t x, int64_t M, int N, int dt, uintptr_t out, int out_dt, bool accumulate,
                       uintptr_t workspace, uintptr_t stream);

// ---- fused MFMA attention (attention.hip) ----
// t = 8 x (ptr, batch stride, head stride, row stride) for q, k, v, o, dout, out, dk, dv
//     + lse ptr, delta ptr, key-mask ptr, key-mask batch stride
bool attention_supported(int D, int Tq, int Tk, int dt);
void attention_fwd(const std::vector<int64_t>& t, int B, int H, int Tq, int Tk, int D, float scale, bool causal,
                   uintptr_t stream);
void attention_bwd(const std::vector<int64_t>& t, int B, int H, int Tq, int Tk, int D, float scale, bool causal,
                   uintptr_t stream);
// ---- fused attention at fp32 on v_mfma_f32_32x32x2_f32 (attention_f32.hip) ----
void attention_fwd_f32(const std::vector<int64_t>& t, int B, int H, int Tq, int Tk, int D, float scale, bool causal,
                       uintptr_t stream);
void attn_f32_set_fused_bwd(int mode);
void attention_bwd_f32(const std::vector<int64_t>& t, int B, int H, int Tq, int Tk, int D, float scale, bool causal,
                       uintptr_t stream);

// ---- RCCL engine (comm.cpp) ----
std::string rccl_unique_id();
int rccl_version();

class RcclComm {
 public:
  // wait=false: return right after ncclCommInitRankConfig; poll_ready() until true (lets the
  // caller abandon an init whose membership epoch was superseded)
  RcclComm(const std::string& uid, int nranks, int rank, int device, double timeout_s, bool wait = true);
  bool poll_ready();
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  void allreduce(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int op, uintptr_t stream);
  void broadcast(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int root, uintptr_t stream);
  void allgather(uintptr_t send, uintptr_t recv, int64_t count, int dtype, uintptr_t stream);
  void reduce_scatter(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int op, uintptr_t stream);
  void alltoall(uintptr_t send, uintptr_t recv, int64_t count, int dtype, uintptr_t stream);
  void group_start();
  void group_end();
  std::string async_error() const;
  void abort();
  void destroy();
  int rank() const { return rank_; }
  int size() const { return nranks_; }
  bool alive() const { return !aborted_.load(); }

 private:
  // Every NCCL call on comm_ runs under mu_, and waits poll with the lock released between
  // polls, so abort() from a watchdog thread never frees the communicator under another
  // thread's NCCL call (it takes effect at the waiter's next poll, which then throws).
  template <typename F>
  int locked_call(F&& f);
  void wait_ready(const char* what);
  void check_live() const;
  void finish(int r, const char* what);
  mutable std::mutex mu_;
  ncclComm_t comm_ = nullptr;
  int nranks_, rank_;
  double timeout_s_;
  std::atomic<bool> aborted_{false};
};


// ---- fp32 GEMM on the bf16 MFMA via an exact 3-way bf16 split (splitgemm.hip) ----
// C[M][N] (+)= A(m,k) B(n,k) [+ bias] [epi 1: GELU (h -> aux, gelu(h) -> C), 2: DGELU (C *= gelu'(aux))];
// A K-contiguous (a[m*lda+k]) or K-major (a[k*lda+m]), likewise B; tile 0/1/2 = 128x128 /
// 256x128 / 128x256; variant 0 = 6 products dual-accumulated (others: error study).
int64_t sgemm_f32_workspace_floats(int M, int N, int splits);
void sgemm_f32_set_stagger(int on);
void sgemm_conv_wgrad_set_ws(int mode);
void sgemm_conv_fwd_set_v8(int on);
void sgemm_set_reduce_groups(int g);
void sgemm_set_write_map(int on);
void sgemm_conv_fwd_f32(uintptr_t x, uintptr_t w, uintptr_t y, int n, int H, int W, int Cin, int Ho, int Wo, int Cout,
                        int KH, int KW, int stride, int pad, uintptr_t stream);
void sgemm_conv_dgrad_s2_class(uintptr_t dy, uintptr_t wc, uintptr_t dx, int n, int Ho, int Wo, int Cout, int H, int W,
                               int Cin, int ph, int pw, uintptr_t stream);
void sgemm_conv_wgrad_f32(uintptr_t dy, uintptr_t x, uintptr_t gw, int n, int H, int W, int Cin, int Ho, int Wo,
                          int Cout, int KH, int KW, int stride, int pad, int splits, bool accumulate, uintptr_t ws,
                          int64_t ws_floats, uintptr_t stream, int tile);
void sgemm_f32(uintptr_t a, int64_t lda, bool a_kmajor, uintptr_t b, int64_t ldb, bool b_kmajor, uintptr_t c,
               int64_t ldc, int M, int N, int K, bool beta, uintptr_t bias, int epi, uintptr_t aux, int64_t ldaux,
               int tile, int splits, int variant, uintptr_t ws, int64_t ws_floats, uintptr_t stream,
               uintptr_t bsum = 0);

}  // namespace voda
