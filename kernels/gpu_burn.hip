// gpu-burn: synthetic matrix-core load for GPU pods (density / exporter validation).
//   gpu-burn [--ms DURATION] [--device D]
// Runs register-resident bf16 MFMA chains on every CU for ~DURATION ms, prints achieved TF.
#include <cstdlib>
#include <cstring>

#include "gpu_common.h"

int main(int argc, char** argv) {
  double ms = 200;
  int dev = 0;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--ms") && i + 1 < argc) ms = std::atof(argv[++i]);
    else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) dev = std::atoi(argv[++i]);
  }
  try {
    amdkube::DevInfo d = amdkube::dev_info(dev);
    amdkube::BurnResult r = amdkube::run_mfma_burn(ms, dev);
    std::printf("{\"device\":%d,\"uuid\":\"%s\",\"ms\":%.2f,\"iters\":%lld,\"blocks\":%d,\"bf16_tflops\":%.1f}\n", dev,
                d.uuid.c_str(), r.ms, r.iters, r.blocks, r.tflops);
    return 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "gpu-burn: %s\n", e.what());
    return 4;
  }
}
