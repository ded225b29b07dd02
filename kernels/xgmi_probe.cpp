// xgmi-probe: RCCL-over-xGMI validation of the GPU set a pod was given.
//
// The reference has no collective or interconnect awareness at all. For
// topology-aware placement amdkube needs ground truth: this probe runs, over every GPU
// visible to the pod (one process, one communicator via ncclCommInitAll), an all-reduce
// bus-bandwidth sweep and a pairwise hipMemcpyPeer matrix. Before timing anything it checks
// the collective's RESULT: rank i fills element e with (i+1) + 0.5*(e%7) (exact in fp32), and
// after a sum all-reduce every rank must hold n(n+1)/2 + 0.5*n*(e%7) in every element. On an 8x MI355X node every GPU
// pair has one direct xGMI link (7 links x ~153 GB/s per GPU), so a ring all-reduce over k
// GPUs is per-link bound; the probe reports algbw and busbw = algbw * 2(k-1)/k.
// It also prints, per rank, the PCI bus id and UUID of the GPU the communicator opened, so the
// placement the scheduler bound (spec.extendedResources[].assigned → amd.com/pci-bus) can be
// checked against what RCCL actually ran on inside the pod.
//   xgmi-probe [--max-mib M] [--iters K] [--no-p2p]
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>
#include <sstream>

#define CHECK_HIP(x)                                                                          \
  do {                                                                                        \
    hipError_t e = (x);                                                                       \
    if (e != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e)); \
  } while (0)
#define CHECK_NCCL(x)                                                                             \
  do {                                                                                            \
    ncclResult_t r = (x);                                                                         \
    if (r != ncclSuccess) throw std::runtime_error(std::string(#x) + ": " + ncclGetErrorString(r)); \
  } while (0)

__global__ void fill_rank(float* buf, size_t count, int rank) {
  for (size_t e = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; e < count;
       e += static_cast<size_t>(gridDim.x) * blockDim.x)
    buf[e] = static_cast<float>(rank + 1) + 0.5f * static_cast<float>(e % 7);
}

__global__ void count_wrong(const float* buf, size_t count, int n, unsigned long long* bad) {
  unsigned long long b = 0;
  for (size_t e = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; e < count;
       e += static_cast<size_t>(gridDim.x) * blockDim.x) {
    float want = 0.5f * n * (n + 1) + 0.5f * n * static_cast<float>(e % 7);
    b += buf[e] != want;
  }
  if (b) atomicAdd(bad, b);
}

int main(int argc, char** argv) {
  size_t max_mib = 256;
  int iters = 10;
  bool p2p = true;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--max-mib") && i + 1 < argc) max_mib = std::strtoull(argv[++i], nullptr, 10);
    else if (!std::strcmp(argv[i], "--iters") && i + 1 < argc) iters = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--no-p2p")) p2p = false;
  }
  try {
    int n = 0;
    CHECK_HIP(hipGetDeviceCount(&n));
    if (n < 1) throw std::runtime_error("no GPUs visible");
    std::ostringstream js;   // printed once at the end: RCCL writes its banner to stdout at init
    char tmp[256];
    std::snprintf(tmp, sizeof tmp, "{\"gpus\":%d,\"devices\":[", n);
    js << tmp;
    for (int i = 0; i < n; ++i) {
      char bus[64] = {0};
      CHECK_HIP(hipDeviceGetPCIBusId(bus, sizeof bus, i));
      hipUUID u;
      CHECK_HIP(hipDeviceGetUuid(&u, i));
      char hex[33];
      for (int b = 0; b < 16; ++b) std::snprintf(hex + 2 * b, 3, "%02x", static_cast<unsigned char>(u.bytes[b]));
      std::snprintf(tmp, sizeof tmp, "%s{\"rank\":%d,\"bus\":\"%s\",\"uuid\":\"%s\"}", i ? "," : "", i, bus, hex);
      js << tmp;
    }
    js << "],";
    std::vector<ncclComm_t> comms(n);
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) devs[i] = i;
    CHECK_NCCL(ncclCommInitAll(comms.data(), n, devs.data()));
    std::vector<float*> buf(n);
    std::vector<hipStream_t> st(n);
    const size_t max_bytes = max_mib << 20;
    for (int i = 0; i < n; ++i) {
      CHECK_HIP(hipSetDevice(i));
      CHECK_HIP(hipMalloc(&buf[i], max_bytes));
      CHECK_HIP(hipMemset(buf[i], 0, max_bytes));
      CHECK_HIP(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    }
    // correctness: rank-dependent values, sum all-reduce, every element checked on every rank
    const size_t vcount = (max_bytes < (64u << 20) ? max_bytes : (64u << 20)) / sizeof(float);
    unsigned long long wrong_total = 0;
    {
      for (int i = 0; i < n; ++i) {
        CHECK_HIP(hipSetDevice(i));
        hipLaunchKernelGGL(fill_rank, dim3(1024), dim3(256), 0, st[i], buf[i], vcount, i);
        CHECK_HIP(hipGetLastError());
      }
      CHECK_NCCL(ncclGroupStart());
      for (int i = 0; i < n; ++i) CHECK_NCCL(ncclAllReduce(buf[i], buf[i], vcount, ncclFloat, ncclSum, comms[i], st[i]));
      CHECK_NCCL(ncclGroupEnd());
      for (int i = 0; i < n; ++i) {
        CHECK_HIP(hipSetDevice(i));
        unsigned long long* bad = nullptr;
        CHECK_HIP(hipMalloc(&bad, sizeof(*bad)));
        CHECK_HIP(hipMemsetAsync(bad, 0, sizeof(*bad), st[i]));
        hipLaunchKernelGGL(count_wrong, dim3(1024), dim3(256), 0, st[i], buf[i], vcount, n, bad);
        CHECK_HIP(hipGetLastError());
        unsigned long long h = 0;
        CHECK_HIP(hipMemcpyAsync(&h, bad, sizeof(h), hipMemcpyDeviceToHost, st[i]));
        CHECK_HIP(hipStreamSynchronize(st[i]));
        CHECK_HIP(hipFree(bad));
        wrong_total += h;
      }
      std::snprintf(tmp, sizeof tmp, "\"verify\":{\"elements\":%zu,\"ranks\":%d,\"wrong\":%llu},", vcount, n, wrong_total);
      js << tmp;
      for (int i = 0; i < n; ++i) {
        CHECK_HIP(hipSetDevice(i));
        CHECK_HIP(hipMemset(buf[i], 0, max_bytes));
      }
    }
    js << "\"allreduce\":[";
    bool first = true;
    for (size_t bytes = 1 << 20; bytes <= max_bytes; bytes <<= 2) {
      size_t count = bytes / sizeof(float);
      auto run = [&]() {
        CHECK_NCCL(ncclGroupStart());
        for (int i = 0; i < n; ++i) CHECK_NCCL(ncclAllReduce(buf[i], buf[i], count, ncclFloat, ncclSum, comms[i], st[i]));
        CHECK_NCCL(ncclGroupEnd());
      };
      run();
      for (int i = 0; i < n; ++i) {
        CHECK_HIP(hipSetDevice(i));
        CHECK_HIP(hipStreamSynchronize(st[i]));
      }
      auto t0 = std::chrono::steady_clock::now();
      for (int it = 0; it < iters; ++it) run();
      for (int i = 0; i < n; ++i) {
        CHECK_HIP(hipSetDevice(i));
        CHECK_HIP(hipStreamSynchronize(st[i]));
      }
      double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / iters;
      double alg = bytes / s / 1e9;
      double bus = n > 1 ? alg * 2.0 * (n - 1) / n : alg;
      std::snprintf(tmp, sizeof tmp, "%s{\"bytes\":%zu,\"us\":%.1f,\"algbw_gbps\":%.2f,\"busbw_gbps\":%.2f}", first ? "" : ",",
                    bytes, s * 1e6, alg, bus);
      js << tmp;
      first = false;
    }
    js << "],\"p2p_gbps\":[";
    for (int i = 0; i < n; ++i) {
      js << (i ? ",[" : "[");
      for (int j = 0; j < n; ++j) {
        double gbps = 0;
        if (p2p && i != j) {
          int can = 0;
          CHECK_HIP(hipDeviceCanAccessPeer(&can, i, j));
          if (can) {
            CHECK_HIP(hipSetDevice(i));
            hipDeviceEnablePeerAccess(j, 0);
            (void)hipGetLastError();
            size_t bytes = max_bytes;
            CHECK_HIP(hipMemcpyPeer(buf[j], j, buf[i], i, bytes));
            CHECK_HIP(hipDeviceSynchronize());
            auto t0 = std::chrono::steady_clock::now();
            for (int it = 0; it < 3; ++it) CHECK_HIP(hipMemcpyPeer(buf[j], j, buf[i], i, bytes));
            CHECK_HIP(hipDeviceSynchronize());
            double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / 3;
            gbps = bytes / s / 1e9;
          }
        }
        std::snprintf(tmp, sizeof tmp, "%s%.1f", j ? "," : "", gbps);
        js << tmp;
      }
      js << "]";
    }
    js << "]}";
    std::fflush(stdout);
    std::printf("%s\n", js.str().c_str());
    for (int i = 0; i < n; ++i) {
      ncclCommDestroy(comms[i]);
      hipSetDevice(i);
      hipFree(buf[i]);
      hipStreamDestroy(st[i]);
    }
    if (wrong_total) {
      std::fprintf(stderr, "xgmi-probe: all-reduce returned %llu wrong elements\n", wrong_total);
      return 5;
    }
    return 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "xgmi-probe: %s\n", e.what());
    return 4;
  }
}
