// hbm-probe: HBM3E bandwidth + pattern integrity check for one MI355X (device health probe
// run by the AMD device plugin before advertising a GPU as Healthy, and a benchmark).
//   hbm-probe [--mib M] [--iters K] [--device D] [--min-copy-gbps G]
// Prints one JSON line; exit 1 on pattern mismatches (or bandwidth below --min-copy-gbps).
#include <cstdlib>
#include <cstring>

#include "gpu_common.h"

int main(int argc, char** argv) {
  size_t mib = 1024;
  int iters = 5, dev = 0;
  double min_copy = 0;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--mib") && i + 1 < argc) mib = std::strtoull(argv[++i], nullptr, 10);
    else if (!std::strcmp(argv[i], "--iters") && i + 1 < argc) iters = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) dev = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--min-copy-gbps") && i + 1 < argc) min_copy = std::atof(argv[++i]);
  }
  try {
    amdkube::DevInfo d = amdkube::dev_info(dev);
    amdkube::HbmResult r = amdkube::run_hbm_probe(mib << 20, iters, dev);
    std::printf("{\"device\":%d,\"uuid\":\"%s\",\"arch\":\"%s\",\"bytes\":%zu,\"iters\":%d,\"write_gbps\":%.1f,"
                "\"read_gbps\":%.1f,\"copy_gbps\":%.1f,\"verify_gbps\":%.1f,\"errors\":%llu}\n",
                dev, d.uuid.c_str(), d.arch.c_str(), r.bytes, r.iters, r.write_gbps, r.read_gbps, r.copy_gbps,
                r.verify_gbps, r.errors);
    if (r.errors) return 1;
    if (min_copy > 0 && r.copy_gbps < min_copy) return 1;
    return 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "hbm-probe: %s\n", e.what());
    return 4;
  }
}
