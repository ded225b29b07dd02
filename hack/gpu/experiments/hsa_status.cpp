// hsa_init() status and agent count: tells whether ROCr skipped an unreachable render node
// (init OK, fewer GPU agents) or failed outright (init error).
#include <hsa/hsa.h>
#include <cstdio>
static hsa_status_t count(hsa_agent_t a, void* d) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU) ++*static_cast<int*>(d);
  else ++static_cast<int*>(d)[1];
  return HSA_STATUS_SUCCESS;
}
int main() {
  hsa_status_t s = hsa_init();
  const char* msg = nullptr;
  hsa_status_string(s, &msg);
  int n[2] = {0, 0};
  if (s == HSA_STATUS_SUCCESS) hsa_iterate_agents(count, n);
  std::printf("hsa_init=%d (%s) gpu_agents=%d cpu_agents=%d\n", s, msg ? msg : "?", n[0], n[1]);
  return s == HSA_STATUS_SUCCESS ? 0 : 1;
}
