// Background GPU-activity sampler: the MI355X counterpart of the NVML sample buffer that the
// reference reads through gonvml's AverageGPUUtilization (vendor/github.com/mindprince/gonvml/
// bindings.go:218-260, nvmlDeviceGetSamples over a time window). cAdvisor reports that average
// over 10 s as AcceleratorStats.DutyCycle (vendor/github.com/google/cadvisor/accelerators/
// nvidia.go:216-252). amd-smi only exposes an instantaneous activity value, so one sampler
// thread per process polls every device at a fixed period into a per-device ring, and readers
// average the samples newer than `since`.
//
// Concurrency contract (checked by native/sampler_selftest.cpp under ThreadSanitizer):
//  * the source callback runs on the sampler thread only, outside the lock (a query can take
//    milliseconds); samples are published under the lock;
//  * average()/ticks()/running() may be called from any thread at any time, including while
//    start()/stop() run on another thread;
//  * stop() wakes the sampler immediately (condition variable), joins it, and is idempotent;
//    the destructor stops.
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace amdkube {

struct ActivitySample {
  int64_t t_ns = 0;  // steady clock
  uint32_t gfx = 0;  // percent
  uint32_t umc = 0;  // percent (memory controller)
  bool has_umc = false;
};

struct ActivityAverage {
  double gfx = 0.0;
  double umc = 0.0;
  size_t samples = 0;
  size_t umc_samples = 0;
  int64_t first_ns = 0;
  int64_t last_ns = 0;
};

inline int64_t steady_now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

class ActivitySampler {
 public:
  // source(dev, &sample) fills gfx/umc; returns false when the device could not be read
  // (the tick records nothing for it).
  using Source = std::function<bool(size_t, ActivitySample*)>;

  ActivitySampler() = default;
  ActivitySampler(const ActivitySampler&) = delete;
  ActivitySampler& operator=(const ActivitySampler&) = delete;
  ~ActivitySampler() { stop(); }

  // Restarts with a fresh ring if already running.
  void start(size_t ndev, Source src, int64_t period_ns, size_t capacity) {
    std::lock_guard<std::mutex> ctl(ctl_mu_);  // held across stop + restart: no interleaved start()
    stop_locked();
    {
      std::lock_guard<std::mutex> lk(mu_);
      rings_.assign(ndev, Ring{});
      for (auto& r : rings_) r.buf.resize(capacity < 2 ? 2 : capacity);
      stop_req_ = false;
      running_ = true;
      ticks_ = 0;
      period_ns_ = period_ns < 1000000 ? 1000000 : period_ns;  // >= 1 ms
    }
    src_ = std::move(src);
    th_ = std::thread([this] { loop(); });
  }

  void stop() {
    std::lock_guard<std::mutex> ctl(ctl_mu_);
    stop_locked();
  }

  bool running() const {
    std::lock_guard<std::mutex> lk(mu_);
    return running_;
  }

  uint64_t ticks() const {
    std::lock_guard<std::mutex> lk(mu_);
    return ticks_;
  }

  size_t devices() const {
    std::lock_guard<std::mutex> lk(mu_);
    return rings_.size();
  }

  // Mean of the device's samples taken at or after since_ns (steady clock).
  ActivityAverage average(size_t dev, int64_t since_ns) const {
    ActivityAverage a;
    std::lock_guard<std::mutex> lk(mu_);
    if (dev >= rings_.size()) return a;
    const Ring& r = rings_[dev];
    const size_t cap = r.buf.size();
    uint64_t gsum = 0, usum = 0;
    for (size_t k = 0; k < r.count; ++k) {  // newest first; stop at the first older sample
      const ActivitySample& s = r.buf[(r.head + cap - 1 - k) % cap];
      if (s.t_ns < since_ns) break;
      gsum += s.gfx;
      if (s.has_umc) {
        usum += s.umc;
        ++a.umc_samples;
      }
      if (a.samples == 0) a.last_ns = s.t_ns;
      a.first_ns = s.t_ns;
      ++a.samples;
    }
    if (a.samples) a.gfx = static_cast<double>(gsum) / static_cast<double>(a.samples);
    if (a.umc_samples) a.umc = static_cast<double>(usum) / static_cast<double>(a.umc_samples);
    return a;
  }

 private:
  void stop_locked() {  // caller holds ctl_mu_
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (!running_) return;
      stop_req_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
    std::lock_guard<std::mutex> lk(mu_);
    running_ = false;
  }

  struct Ring {
    std::vector<ActivitySample> buf;
    size_t head = 0;   // next write slot
    size_t count = 0;  // valid samples (<= buf.size())
  };

  void loop() {
    const size_t ndev = devices();
    std::vector<ActivitySample> tick(ndev);
    std::vector<char> ok(ndev);
    int64_t next = steady_now_ns();
    for (;;) {
      for (size_t d = 0; d < ndev; ++d) {  // outside the lock
        tick[d] = ActivitySample{};
        ok[d] = src_(d, &tick[d]) ? 1 : 0;
        tick[d].t_ns = steady_now_ns();
      }
      std::unique_lock<std::mutex> lk(mu_);
      for (size_t d = 0; d < ndev; ++d) {
        if (!ok[d]) continue;
        Ring& r = rings_[d];
        r.buf[r.head] = tick[d];
        r.head = (r.head + 1) % r.buf.size();
        if (r.count < r.buf.size()) ++r.count;
      }
      ++ticks_;
      next += period_ns_;
      const int64_t now = steady_now_ns();
      if (next < now) next = now;  // fell behind (slow source): no burst of catch-up ticks
      // wait_until on system_clock maps to pthread_cond_timedwait; libstdc++'s steady-clock
      // wait_for uses pthread_cond_clockwait, which GCC 11's ThreadSanitizer does not intercept
      // (it would report every later lock of mu_ as a double lock). The delta is < period,
      // and stop() notifies, so a wall-clock step can at most stretch one tick.
      cv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::nanoseconds(next - now),
                     [this] { return stop_req_; });
      if (stop_req_) return;
    }
  }

  mutable std::mutex mu_;  // rings_, ticks_, flags
  std::mutex ctl_mu_;      // serialises start()/stop()
  std::condition_variable cv_;
  std::vector<Ring> rings_;
  Source src_;
  std::thread th_;
  uint64_t ticks_ = 0;
  int64_t period_ns_ = 100000000;
  bool stop_req_ = false;
  bool running_ = false;
};

}  // namespace amdkube
