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

extern "C" __global__ __launch_bounds__(kWG) void amdkube_vadd(const float* __restrict__ a, const float* __restrict__ b,
                                                                 float* __restrict__ c, unsigned long long n) {
  const unsigned long long i =
      static_cast<unsigned long long>(__builtin_amdgcn_workgroup_id_x()) * kWG + __builtin_amdgcn_workitem_id_x();
  if (i < n) c[i] = a[i] + b[i];
}

// The staging copies run on the same AQL queue as the add (no SDMA engine to bring up for a
// 600 KB job): one 16-byte word per work-item, the < 4 trailing floats by the first work-item.
extern "C" __global__ __launch_bounds__(kWG) void amdkube_copy(const float* __restrict__ src, float* __restrict__ dst,
                                                                 unsigned long long n) {
  const unsigned long long i =
      static_cast<unsigned long long>(__builtin_amdgcn_workgroup_id_x()) * kWG + __builtin_amdgcn_workitem_id_x();
  typedef float v4f __attribute__((ext_vector_type(4)));
  if (i < n / 4) reinterpret_cast<v4f*>(dst)[i] = reinterpret_cast<const v4f*>(src)[i];
  if (i == 0)
    for (unsigned long long k = n & ~3ull; k < n; ++k) dst[k] = src[k];
}
