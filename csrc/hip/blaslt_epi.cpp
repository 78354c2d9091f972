// GEMMs with a fused GELU epilogue on hipBLASLt, for the transformer feed-forward block:
//
//   forward   h = X W1^T + b1 (kept for backward),  y = gelu_tanh(h)     GELU_AUX_BIAS epilogue
//   backward  dh = (dY2 W2) * gelu_tanh'(h)                              DGELU epilogue
//
// Without them the FFN runs fc1 GEMM -> GELU kernel (reads h, writes y) and fc2 input-gradient
// GEMM -> GELU-backward kernel (reads dY2 W2 and h, writes dh): at fp32 and BERT-base's 8192
// tokens x 3072 that is two launches and ~300 MB of extra HBM traffic per layer.  On gfx950
// (ROCm 7.2) hipBLASLt ships these epilogues for fp32 only (one algorithm each; bf16 has none):
// probe in profiles/r5/blaslt_epilogue_probe_fp32.jsonl and profiles/raw/r2_blaslt_epilogue_probe.jsonl.
// These are plain library GEMMs whose epilogue does elementwise work in registers, the same
// library the unfused path calls for the product itself.
//
// Row-major PyTorch operands map onto hipBLASLt's column-major convention as transposes:
//   Y[M][N] = X[M][K] . W[N][K]^T   ==  column-major Y^T (N x M) = op(A) . B with A = W
//                                        (stored K x N, op T, lda K), B = X (K x M, ldb K),
//                                        D = Y (ldd N); m = N, n = M
//   dX[M][K] = dY[M][N] . W[N][K]   ==  A = W (op N, lda K), B = dY (op N, ldb N), D = dX
//                                        (ldd K); m = K, n = M, k = N
// so the epilogue's per-row bias (length m) is the per-output-feature bias, and the aux
// matrix has D's layout (row-major [M][features]).
//
// Plans (descriptors + the heuristic's algorithm) are cached per shape and dtype; pointers are
// set per call.  The workspace comes from the caller (a torch buffer: allocator- and
// capture-safe).
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <string>
#include <tuple>

#include "common.h"
#include "ops.h"

namespace voda {

namespace {

#define VODA_LT_CHECK(expr)                                                                        \
  do {                                                                                             \
    const hipblasStatus_t st_ = (expr);                                                            \
    VODA_CHECK(st_ == HIPBLAS_STATUS_SUCCESS,                                                      \
               std::string("hipBLASLt: " #expr " failed, status ") + std::to_string(int(st_)));    \
  } while (0)

hipDataType lt_type(int dt) {
  VODA_CHECK(dt == kF32 || dt == kBF16, "GELU-epilogue GEMM: fp32 or bf16 operands");
  return dt == kF32 ? HIP_R_32F : HIP_R_16BF;
}

struct Plan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, ld = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws_needed = 0;
};

// mode, dtype, m, n, k, lda, ldb, ldd, device, ws bytes
using PlanKey = std::tuple<int, int, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int, size_t>;

std::mutex& lt_mutex() {
  static std::mutex mu;
  return mu;
}

hipblasLtHandle_t lt_handle(int dev) {
  static std::map<int, hipblasLtHandle_t> hs;
  auto it = hs.find(dev);
  if (it != hs.end()) return it->second;
  hipblasLtHandle_t h;
  VODA_LT_CHECK(hipblasLtCreate(&h));
  hs[dev] = h;
  return h;
}

// Descriptors of one epilogue GEMM: op(A) is m x k, op(B) is k x n, D (and aux) m x n
// (the heuristic finds the fp32 GELU_AUX_BIAS / DGELU kernels only when the bias / aux pointers
// are already set: they are, to the call's operands; the probe passes a scratch allocation)
void make_desc(hipblasLtMatmulDesc_t* op, hipblasLtMatrixLayout_t* la, hipblasLtMatrixLayout_t* lb,
               hipblasLtMatrixLayout_t* ld, hipblasLtEpilogue_t epi, bool trans_a, hipDataType t, int64_t m, int64_t n,
               int64_t k, int64_t lda, int64_t ldb, int64_t ldd, const void* bias, const void* aux) {
  VODA_LT_CHECK(hipblasLtMatmulDescCreate(op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const hipblasOperation_t ta = trans_a ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = HIPBLAS_OP_N;
  VODA_LT_CHECK(hipblasLtMatmulDescSetAttribute(*op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  VODA_LT_CHECK(hipblasLtMatmulDescSetAttribute(*op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  VODA_LT_CHECK(hipblasLtMatmulDescSetAttribute(*op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
  const int64_t ldaux = ldd;
  VODA_LT_CHECK(hipblasLtMatmulDescSetAttribute(*op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ldaux, sizeof(ldaux)));
  const hipDataType bt = t;
  VODA_LT_CHECK(hipblasLtMatmulDescSetAttribute(*op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  VODA_LT_CHECK(hipblasLtMatmulDescSetAttribute(*op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
  VODA_LT_CHECK(hipblasLtMatmulDescSetAttribute(*op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux)));
  if (trans_a) VODA_LT_CHECK(hipblasLtMatrixLayoutCreate(la, t, k, m, lda));
  else VODA_LT_CHECK(hipblasLtMatrixLayoutCreate(la, t, m, k, lda));
  VODA_LT_CHECK(hipblasLtMatrixLayoutCreate(lb, t, k, n, ldb));
  VODA_LT_CHECK(hipblasLtMatrixLayoutCreate(ld, t, m, n, ldd));
}

// mode 0: D = gelu(A.B + bias), aux = A.B + bias   (A = W op T, B = X op N)
// mode 1: D = (A.B) * gelu'(aux)                   (A = W op N, B = dY op N)
Plan& get_plan(hipblasLtHandle_t h, const PlanKey& key, const void* bias, const void* aux) {
  static std::map<PlanKey, Plan> plans;
  auto it = plans.find(key);
  if (it != plans.end()) return it->second;
  const auto [mode, dt, m, n, k, lda, ldb, ldd, dev, ws_bytes] = key;
  (void)dev;
  Plan p;
  make_desc(&p.op, &p.la, &p.lb, &p.ld, mode == 0 ? HIPBLASLT_EPILOGUE_GELU_AUX_BIAS : HIPBLASLT_EPILOGUE_DGELU,
            mode == 0, lt_type(dt), m, n, k, lda, ldb, ldd, bias, aux);
  hipblasLtMatmulPreference_t pref;
  VODA_LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  const uint64_t wsb = ws_bytes;
  VODA_LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb,
                                                      sizeof(wsb)));
  hipblasLtMatmulHeuristicResult_t res[1];
  int ret = 0;
  VODA_LT_CHECK(hipblasLtMatmulAlgoGetHeuristic(h, p.op, p.la, p.lb, p.ld, p.ld, pref, 1, res, &ret));
  hipblasLtMatmulPreferenceDestroy(pref);
  VODA_CHECK(ret > 0, "hipBLASLt: no algorithm for the GELU epilogue GEMM of this shape");
  p.algo = res[0].algo;
  p.ws_needed = res[0].workspaceSize;
  return plans.emplace(key, p).first->second;
}

void run(int mode, int dt, const void* A, int64_t lda, const void* B, int64_t ldb, void* D, int64_t ldd,
         const void* bias, void* aux, int64_t m, int64_t n, int64_t k, void* ws, size_t ws_bytes, hipStream_t s) {
  int dev = 0;
  VODA_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(lt_mutex());
  hipblasLtHandle_t h = lt_handle(dev);
  Plan& p = get_plan(h, PlanKey{mode, dt, m, n, k, lda, ldb, ldd, dev, ws_bytes}, bias, aux);
  VODA_CHECK(p.ws_needed <= ws_bytes, "hipBLASLt: workspace too small for the chosen algorithm");
  if (mode == 0)
    VODA_LT_CHECK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
  VODA_LT_CHECK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux)));
  const float alpha = 1.f, beta = 0.f;
  VODA_LT_CHECK(hipblasLtMatmul(h, p.op, &alpha, A, p.la, B, p.lb, &beta, D, p.ld, D, p.ld, &p.algo, ws, ws_bytes, s));
}

}  // namespace

// Number of algorithms hipBLASLt's heuristic returns for epilogue ``epi`` on a GEMM of dtype
// ``dt`` with op(A) = A^T if ``trans_a`` (m x n x k, tight leading dimensions); aux / bias are
// declared when the epilogue takes them.  Capability probe for tests and the FFN's path choice.
int gemm_epilogue_algos(int epi, int dt, bool trans_a, int64_t m, int64_t n, int64_t k) {
  int dev = 0;
  VODA_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(lt_mutex());
  hipblasLtHandle_t h = lt_handle(dev);
  static void* scratch = nullptr;  // stand-in bias / aux pointer (never dereferenced)
  if (scratch == nullptr) VODA_HIP_CHECK(hipMalloc(&scratch, 256));
  hipblasLtMatmulDesc_t op;
  hipblasLtMatrixLayout_t la, lb, ld;
  make_desc(&op, &la, &lb, &ld, hipblasLtEpilogue_t(epi), trans_a, lt_type(dt), m, n, k, trans_a ? k : m, k, m, scratch,
            scratch);
  hipblasLtMatmulPreference_t pref;
  VODA_LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  const uint64_t wsb = 32ull << 20;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
  hipblasLtMatmulHeuristicResult_t res[8];
  int ret = 0;
  const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, op, la, lb, ld, ld, pref, 8, res, &ret);
  hipblasLtMatmulPreferenceDestroy(pref);
  hipblasLtMatrixLayoutDestroy(la);
  hipblasLtMatrixLayoutDestroy(lb);
  hipblasLtMatrixLayoutDestroy(ld);
  hipblasLtMatmulDescDestroy(op);
  return st == HIPBLAS_STATUS_SUCCESS ? ret : -int(st);
}

void gemm_gelu_aux(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t h, uintptr_t y, int64_t M, int64_t N,
                   int64_t K, int dt, uintptr_t ws, int64_t ws_bytes, uintptr_t stream) {
  VODA_CHECK(M > 0 && N > 0 && K > 0 && N % 8 == 0 && K % 8 == 0, "gemm_gelu_aux: bad shape");
  VODA_CHECK(x % 16 == 0 && w % 16 == 0 && h % 16 == 0 && y % 16 == 0 && bias != 0, "gemm_gelu_aux: operands");
  // y = gelu(X W^T + b) (D), h = X W^T + b (aux); A = W [N][K] (op T), B = X [M][K]
  run(0, dt, reinterpret_cast<const void*>(w), K, reinterpret_cast<const void*>(x), K, reinterpret_cast<void*>(y), N,
      reinterpret_cast<const void*>(bias), reinterpret_cast<void*>(h), N, M, K, reinterpret_cast<void*>(ws),
      size_t(ws_bytes), as_stream(stream));
}

void gemm_dgelu(uintptr_t dy, uintptr_t w, uintptr_t h, uintptr_t dh, int64_t M, int64_t N, int64_t K, int dt,
                uintptr_t ws, int64_t ws_bytes, uintptr_t stream) {
  VODA_CHECK(M > 0 && N > 0 && K > 0 && N % 8 == 0 && K % 8 == 0, "gemm_dgelu: bad shape");
  VODA_CHECK(dy % 16 == 0 && w % 16 == 0 && h % 16 == 0 && dh % 16 == 0, "gemm_dgelu: operands");
  // dh[M][K] = (dY[M][N] . W[N][K]) * gelu'(h[M][K]); A = W (op N, lda K), B = dY (ldb N)
  run(1, dt, reinterpret_cast<const void*>(w), K, reinterpret_cast<const void*>(dy), N, reinterpret_cast<void*>(dh), K,
      nullptr, reinterpret_cast<void*>(h), K, M, N, reinterpret_cast<void*>(ws), size_t(ws_bytes), as_stream(stream));
}

}  // namespace voda
