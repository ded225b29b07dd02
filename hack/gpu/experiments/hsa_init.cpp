// Experiment: ROCr (HSA) init cost alone, without the HIP/ROCclr layer.
#include <hsa/hsa.h>
#include <chrono>
#include <cstdio>
static double now_ms() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
static hsa_status_t cb(hsa_agent_t a, void* d) {
  hsa_device_type_t t; hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU) ++*static_cast<int*>(d);
  return HSA_STATUS_SUCCESS;
}
int main() {
  double t0 = now_ms();
  if (hsa_init() != HSA_STATUS_SUCCESS) return 2;
  double t1 = now_ms();
  int gpus = 0; hsa_iterate_agents(cb, &gpus);
  double t2 = now_ms();
  hsa_shut_down();
  double t3 = now_ms();
  printf("{\"gpus\":%d,\"init\":%.2f,\"iter\":%.2f,\"shutdown\":%.2f}\n", gpus, t1 - t0, t2 - t1, t3 - t2);
  return 0;
}
