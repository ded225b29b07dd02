// The vector-add kernel of the GPU-pod workload, built as a bare gfx950 code object
// (native/build.py: --offload-device-only --no-gpu-bundle-output) and embedded in
// hsa-vector-add, which loads it through the HSA code-object loader.
//
// No HIP runtime builtin that reads the implicit kernel arguments (blockDim / gridDim come from
// the code-object-v5 hidden kernargs): the work-group size is the compile-time 256 the AQL
// packet also uses, and the global index comes straight from the work-group / work-item ID
// registers, so the kernarg segment is exactly the four explicit arguments (32 bytes).
#include <hip/hip_runtime.h>

constexpr unsigned kWG = 256;
typedef float v4f __attribute__((ext_vector_type(4)));

// Both kernels stream 16-byte words with non-temporal loads/stores; each work-group owns one
// contiguous chunk of the range (the chunked layout of kernels/gpu_common.h, which beats a
// grid-stride interleave on MI355X). The host passes the number of work-groups it launched, as
// gridDim would need the implicit kernargs. The < 4 trailing floats go to work-group 0.
__device__ __forceinline__ void chunk(unsigned long long n4, unsigned groups, unsigned long long* lo,
                                      unsigned long long* hi) {
  const unsigned long long per = (n4 + groups - 1) / groups;
  *lo = static_cast<unsigned long long>(__builtin_amdgcn_workgroup_id_x()) * per;
  *hi = *lo + per < n4 ? *lo + per : n4;
}

extern "C" __global__ __launch_bounds__(kWG) void amdkube_vadd(const float* __restrict__ a, const float* __restrict__ b,
                                                                 float* __restrict__ c, unsigned long long n, unsigned groups) {
  unsigned long long lo, hi;
  chunk(n / 4, groups, &lo, &hi);
  const v4f* a4 = reinterpret_cast<const v4f*>(a);
  const v4f* b4 = reinterpret_cast<const v4f*>(b);
  v4f* c4 = reinterpret_cast<v4f*>(c);
  for (unsigned long long i = lo + __builtin_amdgcn_workitem_id_x(); i < hi; i += kWG)
    __builtin_nontemporal_store(__builtin_nontemporal_load(a4 + i) + __builtin_nontemporal_load(b4 + i), c4 + i);
  if (__builtin_amdgcn_workgroup_id_x() == 0)
    for (unsigned long long k = (n & ~3ull) + __builtin_amdgcn_workitem_id_x(); k < n; k += kWG) c[k] = a[k] + b[k];
}

// The staging copies run on the same AQL queue as the add (no SDMA engine to bring up).
extern "C" __global__ __launch_bounds__(kWG) void amdkube_copy(const float* __restrict__ src, float* __restrict__ dst,
                                                                 unsigned long long n, unsigned groups) {
  unsigned long long lo, hi;
  chunk(n / 4, groups, &lo, &hi);
  const v4f* s4 = reinterpret_cast<const v4f*>(src);
  v4f* d4 = reinterpret_cast<v4f*>(dst);
  for (unsigned long long i = lo + __builtin_amdgcn_workitem_id_x(); i < hi; i += kWG)
    __builtin_nontemporal_store(__builtin_nontemporal_load(s4 + i), d4 + i);
  if (__builtin_amdgcn_workgroup_id_x() == 0)
    for (unsigned long long k = (n & ~3ull) + __builtin_amdgcn_workitem_id_x(); k < n; k += kWG) dst[k] = src[k];
}
