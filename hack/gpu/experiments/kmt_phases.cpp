// Experiment: cost of the thunk (libhsakmt) phases that ROCr's hsa_init runs first.
//   kmt_phases [open|topo|full|hold]
//   open: open+close /dev/kfd only; topo: + topology snapshot; full (default): + node props;
//   hold: full, then keep /dev/kfd open until stdin closes (a "keeper" process).
#include <hsakmt/hsakmt.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <unistd.h>
static double now_ms() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "full";
  double t0 = now_ms();
  if (hsaKmtOpenKFD() != HSAKMT_STATUS_SUCCESS) return 2;
  double t1 = now_ms(), t2 = t1, t3 = t1;
  HsaSystemProperties sp{};
  unsigned caches = 0, gpus = 0;
  if (std::strcmp(mode, "open")) {
    if (hsaKmtAcquireSystemProperties(&sp) != HSAKMT_STATUS_SUCCESS) return 3;
    t2 = now_ms();
    for (unsigned n = 0; n < sp.NumNodes; ++n) {
      HsaNodeProperties np{};
      hsaKmtGetNodeProperties(n, &np);
      if (np.NumFComputeCores) ++gpus;
      caches += np.NumCaches;
    }
    t3 = now_ms();
  }
  if (!std::strcmp(mode, "hold")) {
    std::printf("{\"holding\":1}\n");
    std::fflush(stdout);
    char b;
    while (read(0, &b, 1) > 0) {}
  }
  if (std::strcmp(mode, "open")) hsaKmtReleaseSystemProperties();
  hsaKmtCloseKFD();
  double t4 = now_ms();
  printf("{\"nodes\":%u,\"gpus\":%u,\"caches\":%u,\"open\":%.2f,\"topology\":%.2f,\"props\":%.2f,\"close\":%.2f}\n",
         sp.NumNodes, gpus, caches, t1 - t0, t2 - t1, t3 - t2, t4 - t3);
}
