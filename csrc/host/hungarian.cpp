// Kuhn-Munkres (Hungarian) assignment, O(n^2 m) shortest-augmenting-path form with
// row/column potentials.  Replaces the external Go library github.com/heyfey/munkres used
// by the reference placement manager (pkg/placement/placement_manager.go:10,505-507),
// which maximises the number of workers that stay on their current node/GPU slot.
#include "vodacore.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <stdexcept>

namespace vodacore {

// rows <= cols required; returns col index for every row, minimising total cost.
static std::vector<int> hungarian_min_rect(const std::vector<double>& a, int n, int m) {
  const double INF = std::numeric_limits<double>::infinity();
  std::vector<double> u(n + 1, 0.0), v(m + 1, 0.0), minv(m + 1);
  std::vector<int> p(m + 1, 0), way(m + 1, 0);
  std::vector<char> used(m + 1);
  for (int i = 1; i <= n; ++i) {
    p[0] = i;
    int j0 = 0;
    std::fill(minv.begin(), minv.end(), INF);
    std::fill(used.begin(), used.end(), 0);
    do {
      used[j0] = 1;
      const int i0 = p[j0];
      double delta = INF;
      int j1 = -1;
      for (int j = 1; j <= m; ++j) {
        if (used[j]) continue;
        const double cur = a[size_t(i0 - 1) * m + (j - 1)] - u[i0] - v[j];
        if (cur < minv[j]) {
          minv[j] = cur;
          way[j] = j0;
        }
        if (minv[j] < delta) {
          delta = minv[j];
          j1 = j;
        }
      }
      if (j1 < 0) throw std::runtime_error("hungarian: no augmenting path (non-finite costs?)");
      for (int j = 0; j <= m; ++j) {
        if (used[j]) {
          u[p[j]] += delta;
          v[j] -= delta;
        } else {
          minv[j] -= delta;
        }
      }
      j0 = j1;
    } while (p[j0] != 0);
    do {
      const int j1 = way[j0];
      p[j0] = p[j1];
      j0 = j1;
    } while (j0);
  }
  std::vector<int> ans(n, -1);
  for (int j = 1; j <= m; ++j)
    if (p[j] != 0) ans[p[j] - 1] = j - 1;
  return ans;
}

std::vector<int> linear_assignment(const std::vector<double>& cost, int rows, int cols, bool maximize) {
  if (rows < 0 || cols < 0 || size_t(rows) * size_t(cols) != cost.size())
    throw std::invalid_argument("linear_assignment: cost size != rows*cols");
  for (double c : cost)
    if (!std::isfinite(c)) throw std::invalid_argument("linear_assignment: costs must be finite");
  if (rows == 0 || cols == 0) return std::vector<int>(rows, -1);
  const double sgn = maximize ? -1.0 : 1.0;
  if (rows <= cols) {
    std::vector<double> a(cost.size());
    for (size_t k = 0; k < cost.size(); ++k) a[k] = sgn * cost[k];
    return hungarian_min_rect(a, rows, cols);
  }
  // transpose so that rows <= cols, then invert the mapping
  std::vector<double> t(cost.size());
  for (int i = 0; i < rows; ++i)
    for (int j = 0; j < cols; ++j) t[size_t(j) * rows + i] = sgn * cost[size_t(i) * cols + j];
  std::vector<int> colrow = hungarian_min_rect(t, cols, rows);  // for each original col: row
  std::vector<int> ans(rows, -1);
  for (int j = 0; j < cols; ++j)
    if (colrow[j] >= 0) ans[colrow[j]] = j;
  return ans;
}

}  // namespace vodacore
