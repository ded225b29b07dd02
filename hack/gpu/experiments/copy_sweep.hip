// Experiment (round 3): HBM copy layouts. Baseline = the probe's grid-stride NT copy
// (8 x 16 B per lane in flight, 32 blocks/CU). Variants: contiguous per-block chunks (DRAM page
// locality), cached loads + NT stores, NT loads + plain stores, 512-thread blocks, a
// "read-all-then-write-all" 16-deep unroll, and hipMemcpyDtoD as the library reference.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int U, int LD, int ST>   // LD/ST: 0 plain, 1 non-temporal
__global__ __launch_bounds__(512) void stride_k(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n) {
  const size_t st = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * st < n; i += U * st) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = LD ? __builtin_nontemporal_load(s + i + u * st) : s[i + u * st];
#pragma unroll
    for (int u = 0; u < U; ++u) { if (ST) __builtin_nontemporal_store(v[u], d + i + u * st); else d[i + u * st] = v[u]; }
  }
  for (; i < n; i += st) d[i] = s[i];
}

// each block owns a contiguous chunk; inside it the block walks U*blockDim-wide tiles
template <int U>
__global__ __launch_bounds__(256) void chunk_k(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  const size_t lo = (size_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  size_t i = lo + threadIdx.x;
  const size_t tile = (size_t)U * blockDim.x;
  for (; i + (U - 1) * blockDim.x < hi; i += tile) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(s + i + u * blockDim.x);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u], d + i + u * blockDim.x);
  }
  for (; i < hi; i += blockDim.x) d[i] = s[i];
}

template <typename F> float timeit(F f, int it) {
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  f(); (void)hipEventRecord(a); for (int i = 0; i < it; ++i) f(); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b); return ms / it;
}

int main() {
  const size_t bytes = 4ull << 30, n = bytes / 16;
  v4u *s, *d;
  if (hipMalloc(&s, bytes) || hipMalloc(&d, bytes)) return 1;
  (void)hipMemset(s, 1, bytes); (void)hipMemset(d, 0, bytes);
  int cus = 256;
  printf("[");
  bool first = true;
  auto out = [&](const char* name, int per_cu, int threads, float ms) {
    printf("%s{\"variant\":\"%s\",\"blocks_per_cu\":%d,\"threads\":%d,\"copy_gbps\":%.0f}", first ? "" : ",", name, per_cu,
           threads, 2.0 * bytes / (ms * 1e6));
    first = false;
    fflush(stdout);
  };
  for (int per_cu : {8, 16, 32, 64}) {
    int g = cus * per_cu;
    out("stride_nt_u8", per_cu, 256, timeit([&] { hipLaunchKernelGGL((stride_k<8, 1, 1>), dim3(g), dim3(256), 0, 0, s, d, n); }, 10));
    out("stride_nt_u16", per_cu, 256, timeit([&] { hipLaunchKernelGGL((stride_k<16, 1, 1>), dim3(g), dim3(256), 0, 0, s, d, n); }, 10));
    out("stride_ld_st_nt_u8", per_cu, 256, timeit([&] { hipLaunchKernelGGL((stride_k<8, 0, 1>), dim3(g), dim3(256), 0, 0, s, d, n); }, 10));
    out("stride_ldnt_st_u8", per_cu, 256, timeit([&] { hipLaunchKernelGGL((stride_k<8, 1, 0>), dim3(g), dim3(256), 0, 0, s, d, n); }, 10));
    out("stride_nt_u8_512", per_cu, 512, timeit([&] { hipLaunchKernelGGL((stride_k<8, 1, 1>), dim3(g / 2), dim3(512), 0, 0, s, d, n); }, 10));
    out("chunk_nt_u8", per_cu, 256, timeit([&] { hipLaunchKernelGGL((chunk_k<8>), dim3(g), dim3(256), 0, 0, s, d, n); }, 10));
    out("chunk_nt_u4", per_cu, 256, timeit([&] { hipLaunchKernelGGL((chunk_k<4>), dim3(g), dim3(256), 0, 0, s, d, n); }, 10));
  }
  out("hipMemcpyDtoD", 0, 0, timeit([&] { (void)hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); }, 10));
  printf("]\n");
  return 0;
}
