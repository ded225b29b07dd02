// Experiment (round 4): narrower write fronts (64-128 workgroups) and read fronts, after
// write_sweep4 (hashed-pattern write, 128 workgroups x 256 lanes, 2-deep: 6.9-7.1 TB/s).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t mix32(uint32_t x) { x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x; }
__device__ __forceinline__ v4u pat(size_t i, uint32_t seed) {
  uint32_t b = (uint32_t)(i * 4) ^ seed ^ (uint32_t)(i >> 30);
  return v4u{mix32(b), mix32(b + 1), mix32(b + 2), mix32(b + 3)};
}
template <int U>
__global__ __launch_bounds__(256) void wfront(v4u* __restrict__ d, size_t n, uint32_t seed) {
  const size_t st = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * st < n; i += U * st)
#pragma unroll
    for (int u = 0; u < U; ++u) d[i + u * st] = pat(i + u * st, seed);
  for (; i < n; i += st) d[i] = pat(i, seed);
}
template <int U>
__global__ __launch_bounds__(256) void rfront(const v4u* __restrict__ s, size_t n, uint32_t* sink) {
  const size_t st = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (; i + (U - 1) * st < n; i += U * st) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(s + i + u * st);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}
__global__ __launch_bounds__(256) void rchunk(const v4u* __restrict__ s, size_t n, uint32_t* sink) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x, lo = (size_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  uint32_t acc = 0;
  size_t i = lo + threadIdx.x;
  for (; i + 7 * blockDim.x < hi; i += 8 * blockDim.x) {
    v4u v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(s + i + u * blockDim.x);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}
template <typename F> float timeit(F f, int it) {
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  f(); f(); (void)hipEventRecord(a); for (int i = 0; i < it; ++i) f(); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b); return ms / it;
}
int main() {
  uint32_t* sink; (void)hipMalloc(&sink, 64);
  for (size_t gib : {1, 4}) {
    const size_t bytes = gib << 30, n = bytes / 16;
    v4u* d;
    if (hipMalloc(&d, bytes)) return 1;
    auto out = [&](const char* k, int grid, int u, double ms) {
      printf("{\"kernel\":\"%s\",\"gib\":%zu,\"grid\":%d,\"unroll\":%d,\"tbps\":%.3f}\n", k, gib, grid, u, bytes / (ms * 1e9)); fflush(stdout); };
    for (int rep = 0; rep < 2; ++rep) {
      for (int g : {64, 96, 128, 160}) {
        out("wfront_pat", g, 2, timeit([&] { hipLaunchKernelGGL((wfront<2>), dim3(g), dim3(256), 0, 0, d, n, 7u); }, 10));
        out("wfront_pat", g, 4, timeit([&] { hipLaunchKernelGGL((wfront<4>), dim3(g), dim3(256), 0, 0, d, n, 7u); }, 10));
      }
      for (int g : {256, 512, 1024, 2048}) {
        out("rfront", g, 4, timeit([&] { hipLaunchKernelGGL((rfront<4>), dim3(g), dim3(256), 0, 0, d, n, sink); }, 10));
        out("rfront", g, 8, timeit([&] { hipLaunchKernelGGL((rfront<8>), dim3(g), dim3(256), 0, 0, d, n, sink); }, 10));
      }
      out("rchunk_32perCU", 8192, 8, timeit([&] { hipLaunchKernelGGL(rchunk, dim3(8192), dim3(256), 0, 0, d, n, sink); }, 10));
    }
    (void)hipFree(d);
  }
  return 0;
}
