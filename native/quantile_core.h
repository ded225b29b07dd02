// Windowed targeted-quantile summary: the native core of amdkube.utils.quantiles.
//
// Same algorithm and constants as the Prometheus Go client the reference links
// (client_golang summary.go over beorn7/perks quantile: DefObjectives {0.5:0.05, 0.9:0.01,
// 0.99:0.001}, DefMaxAge 10 min, DefAgeBuckets 5, DefBufCap 500): CKMS biased quantiles with the
// targeted invariant f(r,n) = min_j { 2 e_j r / q_j if q_j n <= r, else 2 e_j (n - r) / (1 - q_j) }.
//
// One observation buffer is shared by the age-bucket streams: it is sorted once per 500
// observations and merged into every stream. Every max_age/age_buckets the head stream (the one
// holding the longest history) is reset and becomes the newest; quantiles are read from the head.
// Not thread-safe by itself: the Python binding runs under the GIL.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <limits>
#include <utility>
#include <vector>

namespace amdkube {

struct QSample {
  double value, width, delta;
};

class TargetedStream {
 public:
  explicit TargetedStream(const std::vector<std::pair<double, double>>* targets) : targets_(targets) {}

  double invariant(double r) const {
    double m = std::numeric_limits<double>::infinity();
    for (const auto& [q, e] : *targets_) {
      const double f = (q * n_ <= r) ? 2.0 * e * r / q : 2.0 * e * (n_ - r) / (1.0 - q);
      if (f < m) m = f;
    }
    return m;
  }

  // `sorted` must be ascending.
  void merge(const std::vector<double>& sorted) {
    if (sorted.empty()) return;
    std::vector<QSample> out;
    out.reserve(l_.size() + sorted.size());
    double r = 0;
    size_t i = 0;
    for (double v : sorted) {
      while (i < l_.size() && l_[i].value <= v) {
        r += l_[i].width;
        out.push_back(l_[i++]);
      }
      const double delta = (i < l_.size()) ? std::max(0.0, std::floor(invariant(r)) - 1.0) : 0.0;
      out.push_back({v, 1.0, delta});
      n_ += 1.0;
      r += 1.0;
    }
    while (i < l_.size()) out.push_back(l_[i++]);
    l_.swap(out);
    compress();
  }

  double query(double q) const {
    if (l_.empty()) return std::numeric_limits<double>::quiet_NaN();
    double t = std::ceil(q * n_);
    t += std::ceil(invariant(t) / 2.0);
    double r = 0;
    const QSample* p = &l_[0];
    for (size_t j = 1; j < l_.size(); ++j) {
      r += p->width;
      if (r + l_[j].width + l_[j].delta > t) return p->value;
      p = &l_[j];
    }
    return p->value;
  }

  void reset() {
    l_.clear();
    n_ = 0;
  }
  size_t size() const { return l_.size(); }
  double count() const { return n_; }

 private:
  void compress() {
    if (l_.size() < 2) return;
    // walk from the top, folding each tuple into its right neighbour while the invariant allows;
    // survivors are collected in reverse and flipped once
    std::vector<QSample> keep;
    keep.reserve(l_.size());
    QSample x = l_.back();
    double r = n_ - 1.0 - x.width;
    for (size_t k = l_.size() - 1; k-- > 0;) {
      const QSample& c = l_[k];
      if (c.width + x.width + x.delta <= invariant(r)) {
        x.width += c.width;
      } else {
        keep.push_back(x);
        x = c;
      }
      r -= c.width;
    }
    keep.push_back(x);
    std::reverse(keep.begin(), keep.end());
    l_.swap(keep);
  }

  const std::vector<std::pair<double, double>>* targets_;
  std::vector<QSample> l_;
  double n_ = 0;
};

class WindowedSummary {
 public:
  static constexpr size_t kBufCap = 500;

  WindowedSummary(std::vector<std::pair<double, double>> objectives, double max_age, int age_buckets, double now)
      : targets_(std::move(objectives)), step_(max_age / std::max(1, age_buckets)), next_rotate_(now + step_) {
    std::sort(targets_.begin(), targets_.end());
    for (int i = 0; i < std::max(1, age_buckets); ++i) streams_.emplace_back(&targets_);
    buf_.reserve(kBufCap);
  }

  void observe(double v, double now) {
    rotate(now);
    sum_ += v;
    count_ += 1;
    buf_.push_back(v);
    if (buf_.size() >= kBufCap) flush();
  }

  // quantile values in ascending objective order
  std::vector<double> quantiles(double now) {
    rotate(now);
    flush();
    std::vector<double> out;
    out.reserve(targets_.size());
    for (const auto& t : targets_) out.push_back(streams_[head_].query(t.first));
    return out;
  }

  double sum() const { return sum_; }
  unsigned long long count() const { return count_; }
  size_t head_size() const { return streams_[head_].size(); }

 private:
  void flush() {
    if (buf_.empty()) return;
    std::sort(buf_.begin(), buf_.end());
    for (auto& s : streams_) s.merge(buf_);
    buf_.clear();
  }

  void rotate(double now) {
    if (now < next_rotate_) return;
    flush();  // observations made before the rotation belong to every live stream
    while (now >= next_rotate_) {
      streams_[head_].reset();
      head_ = (head_ + 1) % streams_.size();
      next_rotate_ += step_;
    }
  }

  std::vector<std::pair<double, double>> targets_;
  std::vector<TargetedStream> streams_;
  std::vector<double> buf_;
  double step_, next_rotate_;
  size_t head_ = 0;
  double sum_ = 0;
  unsigned long long count_ = 0;
};

}  // namespace amdkube
