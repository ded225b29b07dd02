// Experiment: process teardown cost of the HIP runtime (normal exit vs _exit after flush)
#include <hip/hip_runtime.h>
#include <unistd.h>
#include <cstdio>
#include <cstdlib>
__global__ void k(float* x) { x[threadIdx.x] += 1.f; }
int main(int argc, char** argv) {
  int quick = argc > 1 ? atoi(argv[1]) : 0;
  float* d = nullptr;
  if (hipMalloc(&d, 1 << 20) != hipSuccess) return 2;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  if (quick == 2) { (void)hipFree(d); }
  printf("done\n");
  fflush(stdout);
  if (quick) _exit(0);
  return 0;
}
