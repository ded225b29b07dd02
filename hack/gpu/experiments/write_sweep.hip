// Experiment (round 3): HBM write and vector-add layouts (grid-stride vs per-workgroup chunks),
// with the probe's hashed pattern and with a constant (pattern cost), and the fp32 vadd.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ unsigned mix32(unsigned x) { x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x; }
__device__ __forceinline__ v4u pat(size_t i, unsigned seed) {
  unsigned b = (unsigned)(i * 4) ^ seed ^ (unsigned)(i >> 30);
  return v4u{mix32(b), mix32(b + 1), mix32(b + 2), mix32(b + 3)};
}
template <int U, bool PAT>
__global__ __launch_bounds__(256) void wstride(v4u* __restrict__ d, size_t n) {
  const size_t st = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * st < n; i += U * st)
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(PAT ? pat(i + u * st, 7) : v4u{1, 2, 3, 4}, d + i + u * st);
  for (; i < n; i += st) d[i] = pat(i, 7);
}
template <int U, bool PAT>
__global__ __launch_bounds__(256) void wchunk(v4u* __restrict__ d, size_t n) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x, lo = (size_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  size_t i = lo + threadIdx.x;
  for (; i + (U - 1) * blockDim.x < hi; i += (size_t)U * blockDim.x)
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(PAT ? pat(i + u * blockDim.x, 7) : v4u{1, 2, 3, 4}, d + i + u * blockDim.x);
  for (; i < hi; i += blockDim.x) d[i] = pat(i, 7);
}
template <bool CHUNK>
__global__ __launch_bounds__(256) void vadd(const v4f* __restrict__ a, const v4f* __restrict__ b, v4f* __restrict__ c, size_t n) {
  if (CHUNK) {
    const size_t per = (n + gridDim.x - 1) / gridDim.x, lo = (size_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
    for (size_t i = lo + threadIdx.x; i < hi; i += blockDim.x)
      __builtin_nontemporal_store(__builtin_nontemporal_load(a + i) + __builtin_nontemporal_load(b + i), c + i);
  } else {
    const size_t st = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += st) c[i] = a[i] + b[i];
  }
}
template <typename F> float timeit(F f, int it) {
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  f(); (void)hipEventRecord(a); for (int i = 0; i < it; ++i) f(); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b); return ms / it;
}
int main() {
  const size_t bytes = 1ull << 30, n = bytes / 16;
  v4u* d; v4f *a, *b, *c;
  if (hipMalloc(&d, bytes) || hipMalloc(&a, bytes) || hipMalloc(&b, bytes) || hipMalloc(&c, bytes)) return 1;
  (void)hipMemset(a, 0, bytes); (void)hipMemset(b, 0, bytes);
  printf("[");
  bool first = true;
  auto out = [&](const char* k, int per_cu, double tb) { printf("%s{\"kernel\":\"%s\",\"per_cu\":%d,\"tbps\":%.3f}", first ? "" : ",", k, per_cu, tb); first = false; fflush(stdout); };
  for (int per_cu : {8, 16, 32, 64}) {
    int g = 256 * per_cu;
    out("write_stride_pat", per_cu, bytes / (timeit([&] { hipLaunchKernelGGL((wstride<8, true>), dim3(g), dim3(256), 0, 0, d, n); }, 10) * 1e9));
    out("write_stride_const", per_cu, bytes / (timeit([&] { hipLaunchKernelGGL((wstride<8, false>), dim3(g), dim3(256), 0, 0, d, n); }, 10) * 1e9));
    out("write_chunk_pat", per_cu, bytes / (timeit([&] { hipLaunchKernelGGL((wchunk<8, true>), dim3(g), dim3(256), 0, 0, d, n); }, 10) * 1e9));
    out("write_chunk_const", per_cu, bytes / (timeit([&] { hipLaunchKernelGGL((wchunk<8, false>), dim3(g), dim3(256), 0, 0, d, n); }, 10) * 1e9));
    out("vadd_stride", per_cu, 3.0 * bytes / (timeit([&] { hipLaunchKernelGGL((vadd<false>), dim3(g), dim3(256), 0, 0, a, b, c, n); }, 10) * 1e9));
    out("vadd_chunk", per_cu, 3.0 * bytes / (timeit([&] { hipLaunchKernelGGL((vadd<true>), dim3(g), dim3(256), 0, 0, a, b, c, n); }, 10) * 1e9));
  }
  out("hipMemsetD32", 0, bytes / (timeit([&] { (void)hipMemsetD32Async((hipDeviceptr_t)d, 7, bytes / 4, 0); }, 10) * 1e9));
  printf("]\n");
  return 0;
}
