// Experiment (round 4): copies as grid-stride fronts (write_sweep3: a 0.5 MiB write front reaches
// 6.75 TB/s) with deeper per-lane batches (loads of U 16-byte words in flight before the stores)
// and tile-stride fronts (each workgroup moves one contiguous U x 4 KiB tile per step).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int U, bool NTL>
__global__ void cstride(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n) {
  const size_t st = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * st < n; i += U * st) {
    v4u r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = NTL ? __builtin_nontemporal_load(s + i + u * st) : s[i + u * st];
#pragma unroll
    for (int u = 0; u < U; ++u) d[i + u * st] = r[u];
  }
  for (; i < n; i += st) d[i] = s[i];
}
template <int U>
__global__ void ctile(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n) {
  const size_t tile = (size_t)U * blockDim.x, ntiles = n / tile;
  for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const size_t base = t * tile + threadIdx.x;
    v4u r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = __builtin_nontemporal_load(s + base + u * blockDim.x);
#pragma unroll
    for (int u = 0; u < U; ++u) d[base + u * blockDim.x] = r[u];
  }
}
template <typename F> float timeit(F f, int it) {
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  f(); f(); (void)hipEventRecord(a); for (int i = 0; i < it; ++i) f(); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b); return ms / it;
}
int main() {
  const size_t bytes = 1ull << 30, n = bytes / 16;
  v4u *s, *d;
  if (hipMalloc(&s, bytes) || hipMalloc(&d, bytes)) return 1;
  (void)hipMemset(s, 1, bytes); (void)hipMemset(d, 0, bytes);
  auto out = [&](const char* k, int bs, int grid, int u, double ms) {
    printf("{\"kernel\":\"%s\",\"block\":%d,\"grid\":%d,\"unroll\":%d,\"tbps\":%.3f}\n", k, bs, grid, u, 2.0 * bytes / (ms * 1e9)); fflush(stdout); };
  for (int g : {64, 128, 256, 512, 1024}) {
    out("cstride_nt", 256, g, 4, timeit([&] { hipLaunchKernelGGL((cstride<4, true>), dim3(g), dim3(256), 0, 0, s, d, n); }, 20));
    out("cstride_nt", 256, g, 8, timeit([&] { hipLaunchKernelGGL((cstride<8, true>), dim3(g), dim3(256), 0, 0, s, d, n); }, 20));
    out("cstride_nt", 256, g, 16, timeit([&] { hipLaunchKernelGGL((cstride<16, true>), dim3(g), dim3(256), 0, 0, s, d, n); }, 20));
    out("cstride_plain", 256, g, 8, timeit([&] { hipLaunchKernelGGL((cstride<8, false>), dim3(g), dim3(256), 0, 0, s, d, n); }, 20));
    out("ctile", 256, g, 8, timeit([&] { hipLaunchKernelGGL((ctile<8>), dim3(g), dim3(256), 0, 0, s, d, n); }, 20));
    out("ctile", 256, g, 16, timeit([&] { hipLaunchKernelGGL((ctile<16>), dim3(g), dim3(256), 0, 0, s, d, n); }, 20));
    out("ctile", 256, 2 * g, 16, timeit([&] { hipLaunchKernelGGL((ctile<16>), dim3(2 * g), dim3(256), 0, 0, s, d, n); }, 20));
  }
  return 0;
}
