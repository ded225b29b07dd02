// xGMI/NUMA topology-aware GPU subset allocator (core, shared by the pybind11 module _topo and the sanitizer self-test).
//
// The reference scheduler picks devices by iterating a Go map and taking the first N that
// match the attribute selector (plugin/pkg/scheduler/core/extended_resources.go:126-142):
// random order, no topology. Here the candidate set (free, healthy, selector-matching
// devices of one node) is scored exhaustively when C(n,k) is small — always true on an
// 8-GPU MI355X node (C(8,4) = 70) — and greedily otherwise, minimising
//
//   cost(S) = W_NUMA * (numa nodes spanned by S - minimum possible)
//           + W_LINK * mean pairwise link cost inside S        (xGMI hops / weights)
//           + W_FRAG * fragmentation of the devices left free   (best fit)
//
// Fragmentation keeps the remaining free GPUs concentrated in as few NUMA groups / aligned
// pairs as possible, so that after a 4-GPU gang lands on one socket the other socket is
// still whole for the next 4-GPU gang. Ties break on the
// lexicographically smallest index set, so placement is deterministic. The Python
// fallback in amdkube/ops/topology.py implements the identical function.
//
// Partitioned GPUs (MI355X CPX/QPX/DPX compute partitions): every partition is a device and
// `parent[d]` names its physical GPU. The fragmentation term then scores how whole the
// remaining physical GPUs stay (instead of aligned pairs), so small partition requests pack
// onto already-split GPUs and full-GPU-sized requests land on one GPU's partitions.
#pragma once

#include <algorithm>
#include <cmath>
#include <limits>
#include <map>
#include <set>
#include <stdexcept>
#include <tuple>
#include <vector>


namespace topo {

constexpr double W_NUMA = 100.0;
constexpr double W_LINK = 10.0;
constexpr double W_FRAG = 1.0;
constexpr long long MAX_ENUM = 200000;

struct Problem {
  std::vector<int> free;                 // candidate device indices (node-local)
  std::vector<std::vector<double>> link; // normalised link cost in [0,1], indexed by device index
  std::vector<int> numa;                 // numa group per device index
  std::vector<int> all_free;             // every free device on the node (for fragmentation)
  std::vector<int> parent;               // physical GPU per device index, dense 0..n_parents-1 (empty: unpartitioned)
  int parent_size = 1;                   // largest number of devices sharing one parent
  int n_parents = 0;
  std::vector<int> group;                // numa group per device, dense 0..n_groups-1
  int n_groups = 0;
  int k;
};

inline long long n_choose_k(int n, int k) {
  if (k < 0 || k > n) return 0;
  long long r = 1;
  for (int i = 1; i <= k; ++i) {
    r = r * (n - k + i) / i;
    if (r > MAX_ENUM * 10) return r;
  }
  return r;
}

inline int min_groups_needed(const Problem& p) {
  std::map<int, int> cnt;
  for (int d : p.free) cnt[p.numa[d]]++;
  std::vector<int> c;
  for (auto& kv : cnt) c.push_back(kv.second);
  std::sort(c.rbegin(), c.rend());
  int need = p.k, g = 0;
  for (int x : c) {
    if (need <= 0) break;
    need -= x;
    ++g;
  }
  return std::max(g, p.k > 0 ? 1 : 0);
}

inline double fragmentation(const Problem& p, const std::vector<int>& chosen) {
  // remaining free devices after taking `chosen`; flat per-device / per-group counters keep
  // this O(n) so the greedy path stays cheap on 64-partition (CPX) nodes
  const size_t n = p.numa.size();
  std::vector<char> rem(n, 0);
  for (int d : p.all_free) rem[d] = 1;
  for (int d : chosen) rem[d] = 0;
  std::vector<int> per_group(p.n_groups, 0), per_parent(p.parent_size > 1 ? p.n_parents : 0, 0);
  int total = 0;
  for (size_t d = 0; d < n; ++d)
    if (rem[d]) {
      ++total;
      per_group[p.group[d]]++;
      if (p.parent_size > 1) per_parent[p.parent[d]]++;
    }
  if (total == 0) return 0.0;
  double q = 0.0;
  for (int c : per_group) q += static_cast<double>(c) * c;
  double best_q = static_cast<double>(total) * total;  // everything in one group
  double frag_groups = 1.0 - q / best_q;
  if (p.parent_size > 1) {
    double qp = 0.0;
    for (int c : per_parent) qp += static_cast<double>(c) * c;
    double frag_parent = 1.0 - qp / (static_cast<double>(total) * std::min(total, p.parent_size));
    return 0.5 * frag_groups + 0.5 * std::max(0.0, frag_parent);
  }
  // devices left that can still form a 2-GPU gang inside one NUMA domain: on MI355X every GPU
  // pair is one xGMI hop, so the domain (the CPU socket's PCIe root), not the device index, is
  // what a future gang should not straddle
  double pairs = 0.0;
  for (int c : per_group) pairs += c / 2;
  double frag_pairs = 1.0 - (2.0 * pairs) / total;
  return 0.75 * frag_groups + 0.25 * std::max(0.0, frag_pairs);
}

inline double cost(const Problem& p, const std::vector<int>& s, int min_groups) {
  std::set<int> groups;
  for (int d : s) groups.insert(p.numa[d]);
  double link = 0.0;
  int pairs = 0;
  for (size_t a = 0; a < s.size(); ++a)
    for (size_t b = a + 1; b < s.size(); ++b) {
      link += p.link[s[a]][s[b]];
      ++pairs;
    }
  double mean_link = pairs ? link / pairs : 0.0;
  return W_NUMA * (static_cast<double>(groups.size()) - min_groups) + W_LINK * mean_link +
         W_FRAG * fragmentation(p, s);
}

inline std::tuple<std::vector<int>, double> solve(const Problem& p) {
  int n = static_cast<int>(p.free.size());
  if (p.k <= 0) return std::make_tuple(std::vector<int>{}, 0.0);
  if (p.k > n) return std::make_tuple(std::vector<int>{}, std::numeric_limits<double>::infinity());
  int mg = min_groups_needed(p);
  std::vector<int> best;
  double best_cost = std::numeric_limits<double>::infinity();
  std::vector<int> sorted_free = p.free;
  std::sort(sorted_free.begin(), sorted_free.end());
  if (n_choose_k(n, p.k) <= MAX_ENUM) {
    std::vector<int> idx(p.k);
    for (int i = 0; i < p.k; ++i) idx[i] = i;
    std::vector<int> s(p.k);
    while (true) {
      for (int i = 0; i < p.k; ++i) s[i] = sorted_free[idx[i]];
      double c = cost(p, s, mg);
      if (c < best_cost - 1e-12) {
        best_cost = c;
        best = s;
      }
      int i = p.k - 1;
      while (i >= 0 && idx[i] == n - p.k + i) --i;
      if (i < 0) break;
      ++idx[i];
      for (int j = i + 1; j < p.k; ++j) idx[j] = idx[j - 1] + 1;
    }
    return std::make_tuple(best, best_cost);
  }
  // greedy: grow from every seed, keep the cheapest. Partitions of one physical GPU are
  // interchangeable as seeds, so a partitioned node seeds once per parent (8 instead of 64).
  std::vector<int> seeds;
  std::vector<char> seeded(p.n_parents, 0);
  for (int d : sorted_free) {
    if (p.parent_size > 1) {
      if (seeded[p.parent[d]]) continue;
      seeded[p.parent[d]] = 1;
    }
    seeds.push_back(d);
  }
  for (int seed : seeds) {
    std::vector<int> s{seed};
    std::set<int> used{seed};
    while (static_cast<int>(s.size()) < p.k) {
      int pick = -1;
      double pc = std::numeric_limits<double>::infinity();
      for (int d : sorted_free) {
        if (used.count(d)) continue;
        s.push_back(d);
        double c = cost(p, s, mg);
        s.pop_back();
        if (c < pc - 1e-12) {
          pc = c;
          pick = d;
        }
      }
      s.push_back(pick);
      used.insert(pick);
    }
    std::sort(s.begin(), s.end());
    double c = cost(p, s, mg);
    if (c < best_cost - 1e-12) {
      best_cost = c;
      best = s;
    }
  }
  return std::make_tuple(best, best_cost);
}

inline Problem make(const std::vector<int>& free, int k, const std::vector<std::vector<double>>& link,
             const std::vector<int>& numa, const std::vector<int>& all_free,
             const std::vector<int>& parent = std::vector<int>{}) {
  Problem p;
  p.free = free;
  p.k = k;
  p.numa = numa;
  p.all_free = all_free.empty() ? free : all_free;
  size_t n = numa.size();
  if (link.size() != n) throw std::invalid_argument("link matrix must be N x N with N == len(numa)");
  double mx = 0.0;
  for (auto& r : link) {
    if (r.size() != n) throw std::invalid_argument("link matrix must be square");
    for (double v : r) mx = std::max(mx, v);
  }
  p.link.assign(n, std::vector<double>(n, 0.0));
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j) p.link[i][j] = mx > 0 ? link[i][j] / mx : 0.0;
  for (int d : p.free)
    if (d < 0 || static_cast<size_t>(d) >= n) throw std::out_of_range("device index out of range");
  for (int d : p.all_free)
    if (d < 0 || static_cast<size_t>(d) >= n) throw std::out_of_range("device index out of range");
  std::map<int, int> gid;
  p.group.resize(n);
  for (size_t d = 0; d < n; ++d) {
    auto it = gid.emplace(numa[d], static_cast<int>(gid.size())).first;
    p.group[d] = it->second;
  }
  p.n_groups = static_cast<int>(gid.size());
  if (!parent.empty()) {
    if (parent.size() != n) throw std::invalid_argument("parent must have one entry per device");
    std::map<int, int> pid, sz;
    std::vector<int> dense(n);
    for (size_t d = 0; d < n; ++d) {
      dense[d] = pid.emplace(parent[d], static_cast<int>(pid.size())).first->second;
      p.parent_size = std::max(p.parent_size, ++sz[parent[d]]);
    }
    if (p.parent_size > 1) {
      p.parent = dense;
      p.n_parents = static_cast<int>(pid.size());
    } else {
      p.parent_size = 1;
    }
  }
  return p;
}

inline double max_cost(int n_groups) { return W_NUMA * std::max(0, n_groups - 1) + W_LINK + W_FRAG; }

}  // namespace topo

