// Experiment (round 4): why hipMemsetD32 writes 1 GiB at ~6.6 TB/s while the probe's own write
// kernels stop near 5.8. Plain vs non-temporal stores, 4- vs 16-byte lanes, block sizes, and
// per-workgroup chunks vs grid-stride; the memset itself is captured by rocprofv3's kernel trace
// (its grid and workgroup sizes are in the trace).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int U, bool NT, typename T>
__global__ void wchunk(T* __restrict__ d, size_t n) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x, lo = (size_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  size_t i = lo + threadIdx.x;
  T v; for (int k = 0; k < (int)(sizeof(T) / 4); ++k) ((unsigned*)&v)[k] = 0x01020304u + k;
  for (; i + (U - 1) * blockDim.x < hi; i += (size_t)U * blockDim.x)
#pragma unroll
    for (int u = 0; u < U; ++u) { if (NT) __builtin_nontemporal_store(v, d + i + u * blockDim.x); else d[i + u * blockDim.x] = v; }
  for (; i < hi; i += blockDim.x) d[i] = v;
}
template <int U, bool NT, typename T>
__global__ void wstride(T* __restrict__ d, size_t n) {
  const size_t st = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  T v; for (int k = 0; k < (int)(sizeof(T) / 4); ++k) ((unsigned*)&v)[k] = 0x01020304u + k;
  for (; i + (U - 1) * st < n; i += U * st)
#pragma unroll
    for (int u = 0; u < U; ++u) { if (NT) __builtin_nontemporal_store(v, d + i + u * st); else d[i + u * st] = v; }
  for (; i < n; i += st) d[i] = v;
}
template <typename F> float timeit(F f, int it) {
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  f(); f(); (void)hipEventRecord(a); for (int i = 0; i < it; ++i) f(); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b); return ms / it;
}
int main() {
  const size_t bytes = 1ull << 30;
  void* d;
  if (hipMalloc(&d, bytes)) return 1;
  (void)hipMemset(d, 0, bytes);
  bool first = true;
  auto out = [&](const char* k, int bs, int grid, double ms) {
    printf("%s{\"kernel\":\"%s\",\"block\":%d,\"grid\":%d,\"tbps\":%.3f}\n", first ? "" : "", k, bs, grid, bytes / (ms * 1e9));
    first = false; fflush(stdout); };
  out("hipMemsetD32", 0, 0, timeit([&] { (void)hipMemsetD32Async((hipDeviceptr_t)d, 7, bytes / 4, 0); }, 20));
  out("hipMemsetD8", 0, 0, timeit([&] { (void)hipMemsetAsync(d, 7, bytes, 0); }, 20));
  const size_t n4 = bytes / 16, n1 = bytes / 4;
  for (int bs : {256, 1024}) {
    for (int per_cu : {2, 4, 8, 16, 32}) {
      int g = 256 * per_cu * 256 / bs;
      if (g < 256) continue;
      out("chunk_v4_plain_u8", bs, g, timeit([&] { hipLaunchKernelGGL((wchunk<8, false, v4u>), dim3(g), dim3(bs), 0, 0, (v4u*)d, n4); }, 20));
      out("chunk_v4_nt_u8", bs, g, timeit([&] { hipLaunchKernelGGL((wchunk<8, true, v4u>), dim3(g), dim3(bs), 0, 0, (v4u*)d, n4); }, 20));
      out("chunk_u32_plain_u16", bs, g, timeit([&] { hipLaunchKernelGGL((wchunk<16, false, unsigned>), dim3(g), dim3(bs), 0, 0, (unsigned*)d, n1); }, 20));
      out("stride_v4_plain_u4", bs, g, timeit([&] { hipLaunchKernelGGL((wstride<4, false, v4u>), dim3(g), dim3(bs), 0, 0, (v4u*)d, n4); }, 20));
      out("stride_u32_plain_u4", bs, g, timeit([&] { hipLaunchKernelGGL((wstride<4, false, unsigned>), dim3(g), dim3(bs), 0, 0, (unsigned*)d, n1); }, 20));
    }
  }
  return 0;
}
