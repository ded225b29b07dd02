// Experiment: a process that keeps a HIP context (VM + one HW queue) alive on the GPU until
// stdin closes, to test whether a resident context changes the next pod's KFD open cost.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <unistd.h>
__global__ void touch(int* x) { if (threadIdx.x == 0) x[0] = 1; }
int main() {
  int* d = nullptr;
  if (hipMalloc(&d, 4096) != hipSuccess) return 2;
  hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, 0, d);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  std::printf("{\"holding\":1}\n");
  std::fflush(stdout);
  char b;
  while (read(0, &b, 1) > 0) {}
  (void)hipFree(d);
  return 0;
}
