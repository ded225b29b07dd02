// Sanitizer self-test for the topology allocator core (built with
// -fsanitize=address,undefined by native/build.py --sanitize; run by tests/test_native.py).
// Exercises exhaustive and greedy paths on random 8/16/32-device nodes and checks the
// invariants: result size == k, indices unique, subset of the candidates, deterministic.
#include <cstdio>
#include <random>
#include <set>

#include "topo_core.h"

int main() {
  std::mt19937 rng(7);
  int checked = 0;
  for (int n : {8, 16, 32}) {
    for (int trial = 0; trial < 60; ++trial) {
      std::vector<std::vector<double>> link(n, std::vector<double>(n, 0.0));
      std::vector<int> numa(n);
      for (int i = 0; i < n; ++i) {
        numa[i] = i / (n / 2);
        for (int j = 0; j < n; ++j)
          if (i != j) link[i][j] = (numa[i] == numa[j] ? 15.0 : 30.0) + (rng() % 3);
      }
      std::vector<int> freev;
      for (int i = 0; i < n; ++i)
        if (rng() % 4) freev.push_back(i);
      int k = 1 + static_cast<int>(rng() % std::max<size_t>(1, freev.size()));
      topo::Problem p = topo::make(freev, k, link, numa, freev);
      auto r1 = topo::solve(p);
      auto r2 = topo::solve(p);
      const auto& s = std::get<0>(r1);
      std::set<int> u(s.begin(), s.end()), cand(freev.begin(), freev.end());
      if (static_cast<int>(s.size()) != k || u.size() != s.size() || s != std::get<0>(r2)) {
        std::printf("FAIL n=%d k=%d size=%zu\n", n, k, s.size());
        return 1;
      }
      for (int d : s)
        if (!cand.count(d)) {
          std::printf("FAIL: picked non-candidate %d\n", d);
          return 1;
        }
      ++checked;
    }
  }
  // partitioned nodes: 8 GPUs x {2,4,8} partitions, parent = physical GPU
  for (int parts : {2, 4, 8}) {
    const int n = 8 * parts;
    for (int trial = 0; trial < 20; ++trial) {
      std::vector<std::vector<double>> link(n, std::vector<double>(n, 0.0));
      std::vector<int> numa(n), parent(n);
      for (int i = 0; i < n; ++i) {
        parent[i] = i / parts;
        numa[i] = parent[i] / 4;
      }
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j)
          if (i != j) link[i][j] = parent[i] == parent[j] ? 5.0 : (numa[i] == numa[j] ? 15.0 : 30.0);
      std::vector<int> freev;
      for (int i = 0; i < n; ++i)
        if (rng() % 3) freev.push_back(i);
      int k = 1 + static_cast<int>(rng() % std::min<size_t>(freev.size(), 12));
      topo::Problem p = topo::make(freev, k, link, numa, freev, parent);
      auto r1 = topo::solve(p);
      const auto& s = std::get<0>(r1);
      std::set<int> u(s.begin(), s.end()), cand(freev.begin(), freev.end());
      if (static_cast<int>(s.size()) != k || u.size() != s.size()) {
        std::printf("FAIL partitioned n=%d k=%d size=%zu\n", n, k, s.size());
        return 1;
      }
      for (int d : s)
        if (!cand.count(d)) {
          std::printf("FAIL: picked non-candidate %d\n", d);
          return 1;
        }
      ++checked;
    }
  }
  std::printf("topo selftest OK (%d cases)\n", checked);
  return 0;
}
