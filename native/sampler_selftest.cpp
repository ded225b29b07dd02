// Self-test of native/sampler_core.h, built twice: with ThreadSanitizer (sampler-selftest-tsan)
// and with ASan/UBSan (sampler-selftest-asan). Readers hammer average() while the sampler
// thread publishes and while other threads restart/stop it; the averages must equal the fake
// source's known pattern. Exit 0 and "OK" on success.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "sampler_core.h"

using amdkube::ActivitySample;
using amdkube::ActivitySampler;

#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

int main() {
  const size_t ndev = 8;
  // device d always reports gfx = 10*d, umc = d except device 3, which never has umc, and
  // device 7, which is unreadable.
  auto src = [](size_t d, ActivitySample* s) {
    if (d == 7) return false;
    s->gfx = static_cast<uint32_t>(10 * d);
    if (d != 3) {
      s->umc = static_cast<uint32_t>(d);
      s->has_umc = true;
    }
    return true;
  };

  ActivitySampler sm;
  CHECK(!sm.running());
  CHECK(sm.average(0, 0).samples == 0);  // before start: nothing, no crash
  const int64_t t0 = amdkube::steady_now_ns();
  sm.start(ndev, src, 1000000 /*1 ms*/, 16);
  while (sm.ticks() < 40) std::this_thread::sleep_for(std::chrono::milliseconds(1));

  // ring capacity bounds the sample count; values are exact
  for (size_t d = 0; d < ndev; ++d) {
    auto a = sm.average(d, t0);
    if (d == 7) {
      CHECK(a.samples == 0);
      continue;
    }
    CHECK(a.samples == 16);
    CHECK(a.gfx == 10.0 * d);
    if (d == 3) {
      CHECK(a.umc_samples == 0);
    } else {
      CHECK(a.umc_samples == 16 && a.umc == static_cast<double>(d));
    }
    CHECK(a.first_ns <= a.last_ns && a.first_ns >= t0);
  }
  CHECK(sm.average(99, 0).samples == 0);  // out-of-range device
  // a window in the future holds nothing
  CHECK(sm.average(0, amdkube::steady_now_ns() + 1000000000LL).samples == 0);

  // concurrent readers while other threads restart and stop the sampler
  std::atomic<bool> done{false};
  std::atomic<uint64_t> reads{0};
  std::vector<std::thread> readers;
  for (int k = 0; k < 4; ++k) {
    readers.emplace_back([&, k] {
      while (!done.load()) {
        size_t d = static_cast<size_t>(k) % 7;
        auto a = sm.average(d, 0);
        if (a.samples) CHECK(a.gfx == 10.0 * d);
        (void)sm.running();
        (void)sm.ticks();
        reads.fetch_add(1);
      }
    });
  }
  std::vector<std::thread> ctl;
  for (int k = 0; k < 2; ++k) {
    ctl.emplace_back([&] {
      for (int i = 0; i < 20; ++i) {
        sm.start(ndev, src, 1000000, 8);
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
        if (i % 3 == 0) sm.stop();
      }
    });
  }
  for (auto& t : ctl) t.join();
  done = true;
  for (auto& t : readers) t.join();
  CHECK(reads.load() > 0);

  sm.stop();
  sm.stop();  // idempotent
  CHECK(!sm.running());
  // stop() returns promptly even with a long period (condition-variable wake-up)
  sm.start(ndev, src, 10LL * 1000 * 1000 * 1000, 4);
  const int64_t s0 = amdkube::steady_now_ns();
  sm.stop();
  CHECK(amdkube::steady_now_ns() - s0 < 2000000000LL);
  std::printf("OK reads=%llu\n", static_cast<unsigned long long>(reads.load()));
  return 0;
}
