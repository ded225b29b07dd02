// Experiment (round 4): can the HBM copy pass 6 TB/s? Round 3 topped out at 5.7 with
// contiguous per-block chunks. New variants here:
//   xcd_chunk  — the chunk of block b is chosen so the 8 XCDs (blocks dispatch round-robin,
//                b % 8 = XCD) each own one contiguous eighth of the buffer: DRAM pages and
//                the XCD's L2/MALL slices see one sequential stream per XCD;
//   tile_rr    — 64 KiB tiles handed out round-robin to blocks (tile-strided, not one chunk);
//   deep       — 16 x 16 B per lane in flight (64 KiB per block);
//   memcpy     — hipMemcpyDtoD, the runtime's blit kernel, as the reference.
// Sizes 1 and 4 GiB; prints one JSON line per variant. Bounded: every loop is over checked sizes.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4u ld(const v4u* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st(v4u* p, v4u v) { __builtin_nontemporal_store(v, p); }

template <int U>
__device__ __forceinline__ void copy_range(const v4u* __restrict__ s, v4u* __restrict__ d, size_t lo, size_t hi) {
  size_t i = lo + threadIdx.x;
  for (; i + (U - 1) * blockDim.x < hi; i += (size_t)U * blockDim.x) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld(s + i + u * blockDim.x);
#pragma unroll
    for (int u = 0; u < U; ++u) st(d + i + u * blockDim.x, v[u]);
  }
  for (; i < hi; i += blockDim.x) st(d + i, ld(s + i));
}

template <int U>
__global__ __launch_bounds__(256) void chunk_k(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  const size_t lo = (size_t)blockIdx.x * per;
  copy_range<U>(s, d, lo, lo + per < n ? lo + per : n);
}

template <int U>
__global__ __launch_bounds__(256) void xcd_chunk_k(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n) {
  const unsigned g = gridDim.x, per_xcd = g / 8;          // grid is a multiple of 8 (host checks)
  const unsigned b = blockIdx.x, xcd = b % 8, k = b / 8;
  const size_t chunk = (size_t)xcd * per_xcd + k;          // XCD x owns chunks [x*per_xcd, (x+1)*per_xcd)
  const size_t per = (n + g - 1) / g;
  const size_t lo = chunk * per;
  copy_range<U>(s, d, lo < n ? lo : n, lo + per < n ? lo + per : n);
}

template <int U>
__global__ __launch_bounds__(256) void tile_rr_k(const v4u* __restrict__ s, v4u* __restrict__ d, size_t n) {
  const size_t tile = (size_t)U * blockDim.x * 4;          // 4 unrolled passes per tile
  const size_t tiles = (n + tile - 1) / tile;
  for (size_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const size_t lo = t * tile;
    copy_range<U>(s, d, lo, lo + tile < n ? lo + tile : n);
  }
}

template <typename F> float timeit(F f, int it) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  (void)hipEventRecord(a);
  for (int i = 0; i < it; ++i) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / it;
}

int main() {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
  const int cus = p.multiProcessorCount;
  for (size_t gib : {1, 4}) {
    const size_t bytes = gib << 30, n = bytes / 16;
    v4u *s, *d;
    if (hipMalloc(&s, bytes) || hipMalloc(&d, bytes)) return 1;
    (void)hipMemset(s, 1, bytes);
    (void)hipMemset(d, 0, bytes);
    auto out = [&](const char* name, int per_cu, float ms) {
      printf("{\"variant\":\"%s\",\"gib\":%zu,\"blocks_per_cu\":%d,\"copy_tbps\":%.3f}\n", name, gib, per_cu,
             2.0 * bytes / (ms * 1e9));
      fflush(stdout);
    };
    for (int per_cu : {8, 16, 32, 64}) {
      const int grid = cus * per_cu;                     // multiple of 8: 256 CUs
      if (grid % 8) return 2;
      out("chunk_u8", per_cu, timeit([&] { chunk_k<8><<<grid, 256>>>(s, d, n); }, 10));
      out("xcd_chunk_u8", per_cu, timeit([&] { xcd_chunk_k<8><<<grid, 256>>>(s, d, n); }, 10));
      out("xcd_chunk_u16", per_cu, timeit([&] { xcd_chunk_k<16><<<grid, 256>>>(s, d, n); }, 10));
      out("tile_rr_u8", per_cu, timeit([&] { tile_rr_k<8><<<grid, 256>>>(s, d, n); }, 10));
      out("deep_u16", per_cu, timeit([&] { chunk_k<16><<<grid, 256>>>(s, d, n); }, 10));
    }
    out("hipMemcpyDtoD", 0, timeit([&] { (void)hipMemcpy(d, s, bytes, hipMemcpyDeviceToDevice); }, 10));
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    (void)hipFree(s);
    (void)hipFree(d);
  }
  return 0;
}
