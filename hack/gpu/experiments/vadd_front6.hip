// Experiment (round 4): the fp32 vector add (2 reads + 1 write per element) as grid-stride
// fronts of 128-1024 workgroups vs the per-workgroup chunks the pod workload uses.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v4f __attribute__((ext_vector_type(4)));
template <int U>
__global__ __launch_bounds__(256) void vfront(const v4f* __restrict__ a, const v4f* __restrict__ b, v4f* __restrict__ c, size_t n) {
  const size_t st = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * st < n; i += U * st) {
    v4f x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { x[u] = __builtin_nontemporal_load(a + i + u * st); y[u] = __builtin_nontemporal_load(b + i + u * st); }
#pragma unroll
    for (int u = 0; u < U; ++u) c[i + u * st] = x[u] + y[u];
  }
  for (; i < n; i += st) c[i] = a[i] + b[i];
}
__global__ __launch_bounds__(256) void vchunk(const v4f* __restrict__ a, const v4f* __restrict__ b, v4f* __restrict__ c, size_t n) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x, lo = (size_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  for (size_t i = lo + threadIdx.x; i < hi; i += blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load(a + i) + __builtin_nontemporal_load(b + i), c + i);
}
template <typename F> float timeit(F f, int it) {
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  f(); f(); (void)hipEventRecord(a); for (int i = 0; i < it; ++i) f(); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b); return ms / it;
}
int main() {
  const size_t bytes = 1ull << 30, n = bytes / 16;
  v4f *a, *b, *c;
  if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes) || hipMalloc(&c, bytes)) return 1;
  (void)hipMemset(a, 0, bytes); (void)hipMemset(b, 0, bytes);
  auto out = [&](const char* k, int grid, int u, double ms) {
    printf("{\"kernel\":\"%s\",\"grid\":%d,\"unroll\":%d,\"tbps\":%.3f}\n", k, grid, u, 3.0 * bytes / (ms * 1e9)); fflush(stdout); };
  for (int rep = 0; rep < 2; ++rep) {
    for (int g : {128, 256, 512, 1024}) {
      out("vfront", g, 1, timeit([&] { hipLaunchKernelGGL((vfront<1>), dim3(g), dim3(256), 0, 0, a, b, c, n); }, 10));
      out("vfront", g, 2, timeit([&] { hipLaunchKernelGGL((vfront<2>), dim3(g), dim3(256), 0, 0, a, b, c, n); }, 10));
      out("vfront", g, 4, timeit([&] { hipLaunchKernelGGL((vfront<4>), dim3(g), dim3(256), 0, 0, a, b, c, n); }, 10));
    }
    out("vchunk_64perCU", 16384, 1, timeit([&] { hipLaunchKernelGGL(vchunk, dim3(16384), dim3(256), 0, 0, a, b, c, n); }, 10));
  }
  return 0;
}
