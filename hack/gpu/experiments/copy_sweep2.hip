// Experiment (round 3, second pass): cache policy of the chunked HBM copy and write kernels.
// The first sweep (copy_sweep.hip) only tried non-temporal stores in the chunked layout; the
// microarchitecture notes report plain stores at 6.0-6.2 TB/s. Variants: load policy x store
// policy (plain / nt) x unroll x blocks per CU x block size, on 1 GiB and 4 GiB buffers; plus
// write-only kernels with plain vs nt stores. One JSON object per line.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int U, int LD, int ST>
__global__ __launch_bounds__(512) void chunk_k(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  const size_t lo = (size_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  size_t i = lo + threadIdx.x;
  const size_t tile = (size_t)U * blockDim.x;
  for (; i + (U - 1) * blockDim.x < hi; i += tile) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = LD ? __builtin_nontemporal_load(s + i + u * blockDim.x) : s[i + u * blockDim.x];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (ST) __builtin_nontemporal_store(v[u], d + i + u * blockDim.x);
      else d[i + u * blockDim.x] = v[u];
    }
  }
  for (; i < hi; i += blockDim.x) d[i] = s[i];
}

template <int U, int ST>
__global__ __launch_bounds__(512) void write_k(v4u* __restrict__ d, size_t n, unsigned seed) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  const size_t lo = (size_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  size_t i = lo + threadIdx.x;
  for (; i + (U - 1) * blockDim.x < hi; i += (size_t)U * blockDim.x) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      size_t k = i + u * blockDim.x;
      v4u v = {(unsigned)k ^ seed, (unsigned)(k >> 32), seed, (unsigned)k};
      if (ST) __builtin_nontemporal_store(v, d + k);
      else d[k] = v;
    }
  }
  for (; i < hi; i += blockDim.x) d[i] = v4u{seed, seed, seed, seed};
}

template <typename F> float timeit(F f, int it) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  f();
  (void)hipEventRecord(a);
  for (int i = 0; i < it; ++i) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms / it;
}

int main() {
  const size_t max_bytes = 4ull << 30;
  v4u *s, *d;
  if (hipMalloc(&s, max_bytes) || hipMalloc(&d, max_bytes)) return 1;
  (void)hipMemset(s, 1, max_bytes);
  (void)hipMemset(d, 0, max_bytes);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  const int cus = 256;
  for (size_t bytes : {1ull << 30, 4ull << 30}) {
    const size_t n = bytes / 16;
    auto out = [&](const char* kind, const char* pol, int u, int per_cu, int thr, float ms, double mult) {
      printf("{\"kind\":\"%s\",\"policy\":\"%s\",\"unroll\":%d,\"blocks_per_cu\":%d,\"threads\":%d,\"gib\":%zu,\"tbps\":%.3f}\n",
             kind, pol, u, per_cu, thr, bytes >> 30, mult * bytes / (ms * 1e9));
      fflush(stdout);
    };
#define COPY(U, LD, ST, POL, THR)                                                                                  \
  for (int per_cu : {16, 32, 64, 128}) {                                                                         \
    int g = cus * per_cu * 256 / THR;                                                                            \
    out("copy", POL, U, per_cu, THR,                                                                             \
        timeit([&] { hipLaunchKernelGGL((chunk_k<U, LD, ST>), dim3(g), dim3(THR), 0, 0, s, d, n); }, 10), 2.0); \
  }
    COPY(8, 1, 1, "nt/nt", 256)
    COPY(8, 0, 0, "plain/plain", 256)
    COPY(8, 1, 0, "nt/plain", 256)
    COPY(8, 0, 1, "plain/nt", 256)
    COPY(4, 1, 0, "nt/plain", 256)
    COPY(4, 0, 0, "plain/plain", 256)
    COPY(16, 1, 0, "nt/plain", 256)
    COPY(4, 1, 0, "nt/plain", 512)
#define WRITE(U, ST, POL)                                                                                     \
  for (int per_cu : {16, 32, 64, 128}) {                                                                    \
    int g = cus * per_cu;                                                                                   \
    out("write", POL, U, per_cu, 256,                                                                       \
        timeit([&] { hipLaunchKernelGGL((write_k<U, ST>), dim3(g), dim3(256), 0, 0, d, n, 7u); }, 10), 1.0); \
  }
    WRITE(8, 1, "nt")
    WRITE(8, 0, "plain")
    WRITE(4, 0, "plain")
    out("copy", "hipMemcpyDtoD", 0, 0, 0, timeit([&] { (void)hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); }, 10), 2.0);
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 3;
}
