// rocm-vector-add: the GPU-pod validation workload (MI355X replacement for the reference's
// cuda-vector-add test image, test/images/cuda-vector-add/Dockerfile:19-26, run by
// test/e2e/scheduling/nvidia-gpus.go:51-113: success = exit 0 and "Test PASSED").
//
// It runs on whatever GPU the runtime made visible (ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES
// set from the device plugin's InitContainer response) and prints that GPU's identity so
// e2e tests can assert the pod used exactly its assigned device.
//   rocm-vector-add [-n ELEMENTS] [--print-uuid] [--json] [--expect-devices K]
#include <cstdlib>
#include <cstring>

#include "gpu_common.h"

int main(int argc, char** argv) {
  size_t n = 50000;
  bool print_uuid = false, json = false;
  int expect = -1;
  for (int i = 1; i < argc; ++i) {
    if ((!std::strcmp(argv[i], "-n") || !std::strcmp(argv[i], "--elements")) && i + 1 < argc) n = std::strtoull(argv[++i], nullptr, 10);
    else if (!std::strcmp(argv[i], "--print-uuid")) print_uuid = true;
    else if (!std::strcmp(argv[i], "--json")) json = true;
    else if (!std::strcmp(argv[i], "--expect-devices") && i + 1 < argc) expect = std::atoi(argv[++i]);
  }
  try {
    int count = 0;
    AK_HIP(hipGetDeviceCount(&count));
    if (count < 1) {
      std::fprintf(stderr, "no GPU visible to this container\n");
      return 2;
    }
    if (expect >= 0 && count != expect) {
      std::fprintf(stderr, "expected %d visible GPU(s), found %d\n", expect, count);
      return 3;
    }
    amdkube::DevInfo d = amdkube::dev_info(0);
    if (print_uuid || !json) std::printf("GPU 0: %s %s bus=%s uuid=%s cus=%d visible=%d\n", d.name.c_str(), d.arch.c_str(),
                                         d.pci_bus_id.c_str(), d.uuid.c_str(), d.cu_count, count);
    std::printf("[Vector addition of %zu elements]\n", n);
    amdkube::VaddResult r = amdkube::run_vector_add(n, 0);
    if (json)
      std::printf("{\"ok\":%s,\"n\":%zu,\"kernel_ms\":%.4f,\"uuid\":\"%s\",\"bus\":\"%s\",\"arch\":\"%s\",\"visible\":%d}\n",
                  r.ok ? "true" : "false", n, r.kernel_ms, d.uuid.c_str(), d.pci_bus_id.c_str(), d.arch.c_str(), count);
    if (!r.ok) {
      std::printf("Result verification failed (%zu mismatches)\nTest FAILED\n", r.mismatches);
      return 1;
    }
    std::printf("Test PASSED\n");
    return 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "rocm-vector-add: %s\n", e.what());
    return 4;
  }
}
