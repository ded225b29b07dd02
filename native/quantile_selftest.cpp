// Host self-test of quantile_core.h (built with ASan/UBSan by native/build.py --sanitize): rank
// error within each objective's epsilon on 200k exponential samples, window rotation dropping
// old observations, and the empty-summary NaN.
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
#include <algorithm>

#include "quantile_core.h"

int main() {
  std::vector<std::pair<double, double>> obj = {{0.5, 0.05}, {0.9, 0.01}, {0.99, 0.001}};
  amdkube::WindowedSummary s(obj, 600.0, 5, 0.0);
  if (!std::isnan(s.quantiles(0.0)[0])) { std::puts("FAIL: empty summary is not NaN"); return 1; }
  std::mt19937_64 rng(7);
  std::exponential_distribution<double> d(1.0);
  std::vector<double> xs(200000);
  for (auto& x : xs) { x = d(rng); s.observe(x, 1.0); }
  std::sort(xs.begin(), xs.end());
  auto q = s.quantiles(1.0);
  for (size_t i = 0; i < obj.size(); ++i) {
    double rank = double(std::lower_bound(xs.begin(), xs.end(), q[i]) - xs.begin()) / xs.size();
    if (std::fabs(rank - obj[i].first) > obj[i].second) {
      std::printf("FAIL: q=%.2f rank %.5f\n", obj[i].first, rank);
      return 1;
    }
  }
  // 10 minutes later every bucket that saw the old samples has been reset
  for (int i = 0; i < 100; ++i) s.observe(1000.0, 700.0);
  auto late = s.quantiles(700.0);
  if (late[0] != 1000.0) { std::printf("FAIL: window kept old samples (p50 %.3f)\n", late[0]); return 1; }
  std::printf("quantile selftest OK (head %zu tuples)\n", s.head_size());
  return 0;
}
