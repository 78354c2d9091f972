// Standalone self-test of the host native core, built with AddressSanitizer +
// UndefinedBehaviorSanitizer by tests/test_native_sanitize.py (the reference
// never ran a race/memory checker).  Exercises every entry point of vodacore.h on random
// problems and checks the answers against brute force:
//   * linear_assignment: square and rectangular (both orientations), min and max, against
//     enumeration of all injective row -> column maps;
//   * ffdl_dp: against enumeration of all allocations within [min, max] (or 0 when allowed).
//   * with the argument ``threads``: 8 threads call both entry points concurrently on their own
//     random problems and compare with the single-threaded answers (the Python bindings release
//     the GIL, so concurrent calls from scheduler/placement threads are real); built with
//     ThreadSanitizer for this mode.
// Exit status 0 and "selftest OK" on success.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <functional>
#include <atomic>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../vodacore.h"

namespace {

double assignment_cost(const std::vector<double>& c, int rows, int cols, const std::vector<int>& a) {
  double s = 0.0;
  for (int i = 0; i < rows; ++i)
    if (a[i] >= 0) s += c[size_t(i) * cols + a[i]];
  return s;
}

// best total over all maps assigning min(rows, cols) rows injectively to columns
double brute_assignment(const std::vector<double>& c, int rows, int cols, bool maximize) {
  const int k = std::min(rows, cols);
  double best = maximize ? -1e300 : 1e300;
  std::vector<int> used(cols, 0), pick(rows, -1);
  std::function<void(int, int, double)> rec = [&](int i, int assigned, double acc) {
    if (assigned == k) {
      best = maximize ? std::max(best, acc) : std::min(best, acc);
      return;
    }
    if (i == rows) return;
    if (rows - i > k - assigned) rec(i + 1, assigned, acc);  // leave row i unassigned
    for (int j = 0; j < cols; ++j) {
      if (used[j]) continue;
      used[j] = 1;
      rec(i + 1, assigned + 1, acc + c[size_t(i) * cols + j]);
      used[j] = 0;
    }
  };
  rec(0, 0, 0.0);
  return best;
}

int check_assignment(std::mt19937& rng) {
  std::uniform_int_distribution<int> dim(1, 6), val(0, 9);
  int bad = 0;
  for (int trial = 0; trial < 300; ++trial) {
    const int rows = dim(rng), cols = dim(rng);
    const bool maximize = trial % 2 == 0;
    std::vector<double> c(size_t(rows) * cols);
    for (double& v : c) v = val(rng);
    const std::vector<int> a = vodacore::linear_assignment(c, rows, cols, maximize);
    std::vector<int> seen(cols, 0);
    int assigned = 0;
    for (int i = 0; i < rows; ++i) {
      if (a[i] < 0) continue;
      if (a[i] >= cols || seen[a[i]]++) ++bad;
      ++assigned;
    }
    if (assigned != std::min(rows, cols)) ++bad;
    const double got = assignment_cost(c, rows, cols, a), want = brute_assignment(c, rows, cols, maximize);
    if (std::fabs(got - want) > 1e-9) {
      std::printf("assignment mismatch %dx%d max=%d: got %g want %g\n", rows, cols, int(maximize), got, want);
      ++bad;
    }
  }
  return bad;
}

int check_ffdl(std::mt19937& rng) {
  std::uniform_int_distribution<int> nj(1, 4), gpus(0, 6), lo(1, 2), span(0, 3);
  std::uniform_real_distribution<double> gain(0.1, 1.0);
  int bad = 0;
  for (int trial = 0; trial < 300; ++trial) {
    const int J = nj(rng), K = gpus(rng);
    const bool allow_zero = trial % 3 == 0;
    std::vector<std::vector<double>> sp(J);
    std::vector<int> mins(J), maxs(J);
    for (int j = 0; j < J; ++j) {
      mins[j] = lo(rng);
      maxs[j] = mins[j] + span(rng);
      sp[j].assign(maxs[j] + 1, 0.0);
      for (int g = 1; g <= maxs[j]; ++g) sp[j][g] = sp[j][g - 1] + gain(rng);  // increasing speedup
    }
    const auto res = vodacore::ffdl_dp(sp, mins, maxs, K, allow_zero);
    // brute force over all allocations
    double best = -1e300;
    std::vector<int> cur(J, 0);
    std::function<void(int, int, double)> rec = [&](int j, int left, double acc) {
      if (j == J) {
        best = std::max(best, acc);
        return;
      }
      if (allow_zero) rec(j + 1, left, acc);
      for (int g = std::max(mins[j], 1); g <= maxs[j] && g <= left; ++g) rec(j + 1, left - g, acc + sp[j][g]);
    };
    rec(0, K, 0.0);
    if (best < -1e299) continue;  // infeasible: the caller reports it, nothing to compare
    double got = 0.0;
    int used = 0;
    for (int j = 0; j < J; ++j) {
      const int g = res.second[j];
      if (g != 0 && (g < mins[j] || g > maxs[j])) ++bad;
      if (g == 0 && !allow_zero) ++bad;
      used += g;
      got += sp[j][g];
    }
    if (used > K || std::fabs(got - best) > 1e-9 || std::fabs(res.first - best) > 1e-9) {
      std::printf("ffdl mismatch J=%d K=%d zero=%d: got %g (dp %g) want %g\n", J, K, int(allow_zero), got,
                  res.first, best);
      ++bad;
    }
  }
  return bad;
}

}  // namespace

// Each thread solves the same seeded problem sequence; the answers must match the serial run.
int check_threads() {
  constexpr int kThreads = 8, kIters = 40;
  auto run = [](unsigned seed, std::vector<double>& out) {
    std::mt19937 rng(seed);
    std::uniform_real_distribution<double> u(0.0, 10.0);
    for (int it = 0; it < kIters; ++it) {
      const int rows = 2 + int(rng() % 9), cols = 2 + int(rng() % 9);
      std::vector<double> c(size_t(rows) * cols);
      for (auto& v : c) v = u(rng);
      const std::vector<int> a = vodacore::linear_assignment(c, rows, cols, (it & 1) != 0);
      out.push_back(assignment_cost(c, rows, cols, a));
      const int jobs = 1 + int(rng() % 5), gpus = 1 + int(rng() % 8);
      std::vector<std::vector<double>> sp(jobs);
      std::vector<int> mn(jobs), mx(jobs);
      for (int j = 0; j < jobs; ++j) {
        mn[j] = 1;
        mx[j] = 1 + int(rng() % gpus);
        sp[j].assign(size_t(mx[j]) + 1, 0.0);
        for (int g = 1; g <= mx[j]; ++g) sp[j][g] = sp[j][g - 1] + u(rng) / g;
      }
      out.push_back(vodacore::ffdl_dp(sp, mn, mx, gpus, true).first);
    }
  };
  std::vector<std::vector<double>> serial(kThreads), par(kThreads);
  for (int t = 0; t < kThreads; ++t) run(1000u + t, serial[t]);
  std::atomic<int> go{0};
  std::vector<std::thread> th;
  for (int t = 0; t < kThreads; ++t)
    th.emplace_back([&, t] {
      while (!go.load()) std::this_thread::yield();
      run(1000u + t, par[t]);
    });
  go.store(1);
  for (auto& x : th) x.join();
  int bad = 0;
  for (int t = 0; t < kThreads; ++t)
    if (serial[t] != par[t]) ++bad;
  return bad;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::strcmp(argv[1], "threads") == 0) {
    const int bad = check_threads();
    if (bad) {
      std::printf("selftest FAILED: %d thread(s) disagree with the serial run\n", bad);
      return 1;
    }
    std::printf("selftest OK\n");
    return 0;
  }
  std::mt19937 rng(12345);
  int bad = check_assignment(rng) + check_ffdl(rng);
  // error paths must throw, not corrupt memory
  try {
    vodacore::linear_assignment({1.0, 2.0}, 2, 2, false);
    ++bad;
  } catch (const std::exception&) {
  }
  try {
    vodacore::ffdl_dp({{0.0, 1.0}}, {1}, {3}, 4, false);  // speedup table shorter than max
    ++bad;
  } catch (const std::exception&) {
  }
  if (bad) {
    std::printf("selftest FAILED: %d problem(s)\n", bad);
    return 1;
  }
  std::printf("selftest OK\n");
  return 0;
}
