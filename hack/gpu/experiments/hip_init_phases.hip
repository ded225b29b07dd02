// Experiment: where does a GPU pod's process lifetime go? (HIP runtime init phases)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
static double now_ms() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
__global__ void k(float* x) { x[threadIdx.x] += 1.f; }
int main(int argc, char** argv) {
  int mode = argc > 1 ? atoi(argv[1]) : 9;
  if (mode == 0) return 0;  // dynamic loading + static init only
  double t0 = now_ms();
  int n = 0; hipGetDeviceCount(&n);
  double t1 = now_ms();
  if (mode >= 2) { hipDeviceProp_t p; hipGetDeviceProperties(&p, 0); }
  double t2 = now_ms();
  float* d = nullptr;
  if (mode >= 3) hipMalloc(&d, 1 << 20);
  double t3 = now_ms();
  if (mode >= 4) { hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d); hipDeviceSynchronize(); }
  double t4 = now_ms();
  printf("{\"count\":%.2f,\"props\":%.2f,\"malloc\":%.2f,\"kernel\":%.2f}\n", t1 - t0, t2 - t1, t3 - t2, t4 - t3);
  return 0;
}
