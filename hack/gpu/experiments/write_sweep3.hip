// Experiment (round 4, after write_sweep2): the runtime's fill kernel (__amd_rocclr_fillBufferAligned,
// 256 workgroups x 256 lanes, 16-byte grid-stride stores: a 1 MiB "front" sweeping memory in
// order) writes at 6.6 TB/s where per-workgroup chunks stop at ~6.2. Grid-stride fronts of
// 0.5-4 MiB for writes and copies, unroll 1-4, and the chunked layouts for comparison.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int U>
__global__ void wstride(v4u* __restrict__ d, size_t n) {
  const size_t st = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const v4u v{1, 2, 3, 4};
  for (; i + (U - 1) * st < n; i += U * st)
#pragma unroll
    for (int u = 0; u < U; ++u) d[i + u * st] = v;
  for (; i < n; i += st) d[i] = v;
}
template <int U>
__global__ void cstride(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n) {
  const size_t st = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * st < n; i += U * st) {
    v4u r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = __builtin_nontemporal_load(s + i + u * st);
#pragma unroll
    for (int u = 0; u < U; ++u) d[i + u * st] = r[u];
  }
  for (; i < n; i += st) d[i] = s[i];
}
template <int U>
__global__ void cchunk(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x, lo = (size_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  size_t i = lo + threadIdx.x;
  for (; i + (U - 1) * blockDim.x < hi; i += (size_t)U * blockDim.x) {
    v4u r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = __builtin_nontemporal_load(s + i + u * blockDim.x);
#pragma unroll
    for (int u = 0; u < U; ++u) d[i + u * blockDim.x] = r[u];
  }
  for (; i < hi; i += blockDim.x) d[i] = s[i];
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
  auto out = [&](const char* k, int bs, int grid, int u, double tb) {
    printf("{\"kernel\":\"%s\",\"block\":%d,\"grid\":%d,\"unroll\":%d,\"tbps\":%.3f}\n", k, bs, grid, u, tb); fflush(stdout); };
  out("hipMemsetD32", 0, 0, 0, bytes / (timeit([&] { (void)hipMemsetD32Async((hipDeviceptr_t)d, 7, bytes / 4, 0); }, 20) * 1e9));
  out("hipMemcpyDtoD", 0, 0, 0, 2.0 * bytes / (timeit([&] { (void)hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); }, 20) * 1e9));
  for (int bs : {256, 512}) {
    for (int g : {128, 256, 512, 1024}) {
      out("wstride", bs, g, 1, bytes / (timeit([&] { hipLaunchKernelGGL((wstride<1>), dim3(g), dim3(bs), 0, 0, d, n); }, 20) * 1e9));
      out("wstride", bs, g, 2, bytes / (timeit([&] { hipLaunchKernelGGL((wstride<2>), dim3(g), dim3(bs), 0, 0, d, n); }, 20) * 1e9));
      out("wstride", bs, g, 4, bytes / (timeit([&] { hipLaunchKernelGGL((wstride<4>), dim3(g), dim3(bs), 0, 0, d, n); }, 20) * 1e9));
      out("cstride", bs, g, 1, 2.0 * bytes / (timeit([&] { hipLaunchKernelGGL((cstride<1>), dim3(g), dim3(bs), 0, 0, s, d, n); }, 20) * 1e9));
      out("cstride", bs, g, 2, 2.0 * bytes / (timeit([&] { hipLaunchKernelGGL((cstride<2>), dim3(g), dim3(bs), 0, 0, s, d, n); }, 20) * 1e9));
      out("cstride", bs, g, 4, 2.0 * bytes / (timeit([&] { hipLaunchKernelGGL((cstride<4>), dim3(g), dim3(bs), 0, 0, s, d, n); }, 20) * 1e9));
    }
  }
  for (int g : {4096, 8192, 16384}) {
    out("cchunk", 256, g, 8, 2.0 * bytes / (timeit([&] { hipLaunchKernelGGL((cchunk<8>), dim3(g), dim3(256), 0, 0, s, d, n); }, 20) * 1e9));
    out("cchunk", 256, g, 4, 2.0 * bytes / (timeit([&] { hipLaunchKernelGGL((cchunk<4>), dim3(g), dim3(256), 0, 0, s, d, n); }, 20) * 1e9));
  }
  return 0;
}
