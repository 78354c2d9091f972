// FfDL Optimizer dynamic program (reference pkg/algorithm/ffdl_optimizer.go:77-125):
//   P[j][k] = max_g speedup_j[g] + P[j-1][k-g],  g in [max(min_j,1), max_j] (and g = 0 when
//   allow_zero), P[0][*] = 0, P[j>0][*] = -10000.  O(J*K*Max) with J, K <= total GPUs.
#include "vodacore.h"

#include <stdexcept>

namespace vodacore {

std::pair<double, std::vector<int>> ffdl_dp(const std::vector<std::vector<double>>& speedups,
                                            const std::vector<int>& mins, const std::vector<int>& maxs, int K,
                                            bool allow_zero) {
  const int J = int(speedups.size());
  if (int(mins.size()) != J || int(maxs.size()) != J || K < 0) throw std::invalid_argument("ffdl_dp: bad sizes");
  const double NEG = -10000.0;
  std::vector<double> P(size_t(J + 1) * (K + 1), NEG);
  std::vector<int> SOL(size_t(J + 1) * (K + 1), 0);
  for (int k = 0; k <= K; ++k) P[k] = 0.0;
  for (int j = 1; j <= J; ++j) {
    const auto& sp = speedups[j - 1];
    const int lo = std::max(mins[j - 1], 1), hi = maxs[j - 1];
    if (hi >= int(sp.size())) throw std::invalid_argument("ffdl_dp: speedup table shorter than max");
    double* Pj = &P[size_t(j) * (K + 1)];
    const double* Pp = &P[size_t(j - 1) * (K + 1)];
    int* Sj = &SOL[size_t(j) * (K + 1)];
    for (int k = 0; k <= K; ++k) {
      if (allow_zero && Pp[k] > Pj[k]) {
        Pj[k] = Pp[k];
        Sj[k] = 0;
      }
      for (int g = lo; g <= hi && g <= k; ++g) {
        const double prev = Pp[k - g];
        if (prev <= NEG / 2) continue;
        const double p = sp[g] + prev;
        if (p > Pj[k]) {
          Pj[k] = p;
          Sj[k] = g;
        }
      }
    }
  }
  std::vector<int> alloc(J, 0);
  int k = K;
  for (int j = J; j >= 1; --j) {
    alloc[j - 1] = SOL[size_t(j) * (K + 1) + k];
    k -= alloc[j - 1];
  }
  return {P[size_t(J) * (K + 1) + K], alloc};
}

}  // namespace vodacore
