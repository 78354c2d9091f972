// Host-side native core of vodascheduler_amd (placement + allocation kernels).
#pragma once
#include <utility>
#include <vector>

namespace vodacore {
std::vector<int> linear_assignment(const std::vector<double>& cost, int rows, int cols, bool maximize);
std::pair<double, std::vector<int>> ffdl_dp(const std::vector<std::vector<double>>& speedups,
                                            const std::vector<int>& mins, const std::vector<int>& maxs, int K,
                                            bool allow_zero);
}  // namespace vodacore
