// hsa-vector-add: the GPU-pod validation workload on the bare ROCr (HSA) runtime.
//
// Same contract as rocm-vector-add (kernels/vector_add.hip; the reference's cuda-vector-add test
// image, test/images/cuda-vector-add, run by test/e2e/scheduling/nvidia-gpus.go: success = exit 0
// and "Test PASSED"), same output lines (the visible GPU's product name, ISA, PCI bus id and
// UUID, so e2e tests can check the pod ran on exactly its assigned device), same input data and
// verification. What it drops is the HIP runtime: a GPU pod's life is dominated by process
// start-up (docs/PERFORMANCE.md: ≈150 ms KFD release window + ≈50 ms ROCr init + ≈80 ms HIP init,
// work and exit), and everything the HIP layer adds on top of hsa_init — loading libamdhip64,
// device-property queries, the fat-binary registration, stream and blit-kernel set-up — is time
// the pod's GPU is held for nothing. Here the kernel (kernels/vadd_kernel.hip) is a bare gfx950
// code object embedded in this binary and loaded with the HSA code-object loader; the inputs are
// staged in host memory the GPU may access, and three AQL packets on one user-mode queue copy
// them into device memory, add, and copy the sum back (kernel copies: no SDMA engine to bring
// up, which alone cost ≈16 ms of the first version's life). On MI355X back-to-back pods of it
// live 250 ms (median of 15) against 320 ms for the HIP build (hack/exp/vadd_runtime_cmp.py,
// profiles/r3/hsa_vector_add.json). Skipping hsa_shut_down (--fast-exit) saves its ≈30 ms of
// user-space teardown but the next process then waits that much longer in the kernel's KFD
// release path, so the default shuts down cleanly.
//
//   hsa-vector-add [-n ELEMENTS] [--print-uuid] [--json] [--expect-devices K] [--fast-exit]
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#ifndef VADD_CO_PATH
#error "VADD_CO_PATH must name the gfx950 code object to embed (native/build.py)"
#endif

extern "C" const unsigned char amdkube_vadd_co[];
extern "C" const unsigned char amdkube_vadd_co_end[];
__asm__(".section .rodata\n.balign 64\n.global amdkube_vadd_co\namdkube_vadd_co:\n.incbin \"" VADD_CO_PATH
        "\"\n.global amdkube_vadd_co_end\namdkube_vadd_co_end:\n.byte 0\n.previous\n");

namespace {

constexpr uint32_t kWG = 256;             // must match kernels/vadd_kernel.hip
constexpr uint64_t kWaitNs = 10ull * 1000 * 1000 * 1000;   // every GPU wait gives up after 10 s

struct Fail {
  std::string what;
  hsa_status_t st;
};

void check(hsa_status_t st, const char* what) {
  if (st != HSA_STATUS_SUCCESS && st != HSA_STATUS_INFO_BREAK) throw Fail{what, st};
}

struct Agents {
  std::vector<hsa_agent_t> gpus;
  hsa_agent_t cpu{};
  bool have_cpu = false;
};

hsa_status_t on_agent(hsa_agent_t a, void* data) {
  auto* ag = static_cast<Agents*>(data);
  hsa_device_type_t t;
  check(hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t), "agent type");
  if (t == HSA_DEVICE_TYPE_GPU) ag->gpus.push_back(a);
  if (t == HSA_DEVICE_TYPE_CPU && !ag->have_cpu) {
    ag->cpu = a;
    ag->have_cpu = true;
  }
  return HSA_STATUS_SUCCESS;
}

struct Pools {
  hsa_amd_memory_pool_t device{}, kernarg{}, host{};
  bool have_device = false, have_kernarg = false, have_host = false;
};

hsa_status_t on_gpu_pool(hsa_amd_memory_pool_t p, void* data) {
  auto* pools = static_cast<Pools*>(data);
  hsa_amd_segment_t seg;
  uint32_t flags = 0;
  bool alloc = false;
  check(hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg), "pool segment");
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  check(hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags), "pool flags");
  check(hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc), "pool alloc");
  if (alloc && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && !pools->have_device) {
    pools->device = p;
    pools->have_device = true;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t on_cpu_pool(hsa_amd_memory_pool_t p, void* data) {
  auto* pools = static_cast<Pools*>(data);
  hsa_amd_segment_t seg;
  uint32_t flags = 0;
  bool alloc = false;
  check(hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg), "pool segment");
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  check(hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags), "pool flags");
  check(hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc), "pool alloc");
  if (!alloc) return HSA_STATUS_SUCCESS;
  if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !pools->have_kernarg) {
    pools->kernarg = p;
    pools->have_kernarg = true;
  }
  if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !pools->have_host) {
    pools->host = p;
    pools->have_host = true;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t on_isa(hsa_isa_t isa, void* data) {
  uint32_t len = 0;
  check(hsa_isa_get_info_alt(isa, HSA_ISA_INFO_NAME_LENGTH, &len), "isa name length");
  std::string name(len, '\0');
  check(hsa_isa_get_info_alt(isa, HSA_ISA_INFO_NAME, &name[0]), "isa name");
  name = name.c_str();
  const std::string pre = "amdgcn-amd-amdhsa--";
  *static_cast<std::string*>(data) = name.rfind(pre, 0) == 0 ? name.substr(pre.size()) : name;
  return HSA_STATUS_INFO_BREAK;
}

struct GpuId {
  std::string product, arch, bus, uuid;
  uint32_t cus = 0;
};

GpuId identify(hsa_agent_t g) {
  GpuId id;
  char buf[128] = {0};
  if (hsa_agent_get_info(g, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_PRODUCT_NAME), buf) == HSA_STATUS_SUCCESS)
    id.product = buf;
  if (id.product.empty()) id.product = "AMD Instinct GPU";   // the marketing name needs libdrm's amdgpu.ids
  std::memset(buf, 0, sizeof buf);
  if (hsa_agent_get_info(g, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_UUID), buf) == HSA_STATUS_SUCCESS) id.uuid = buf;
  uint32_t bdf = 0, domain = 0;
  hsa_agent_get_info(g, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf);
  hsa_agent_get_info(g, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &domain);
  std::snprintf(buf, sizeof buf, "%04x:%02x:%02x.%x", domain, (bdf >> 8) & 0xff, (bdf >> 3) & 0x1f, bdf & 0x7);
  id.bus = buf;
  hsa_agent_get_info(g, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT), &id.cus);
  hsa_agent_iterate_isas(g, on_isa, &id.arch);
  return id;
}

void wait_zero(hsa_signal_t s, const char* what) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::nanoseconds(kWaitNs);
  while (hsa_signal_wait_scacquire(s, HSA_SIGNAL_CONDITION_LT, 1, 100 * 1000 * 1000, HSA_WAIT_STATE_BLOCKED) >= 1) {
    if (std::chrono::steady_clock::now() > deadline) throw Fail{std::string(what) + ": timed out", HSA_STATUS_ERROR};
  }
}

struct Trace {  // AMDKUBE_VADD_TRACE=1: per-phase wall times on stderr
  bool on = std::getenv("AMDKUBE_VADD_TRACE") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void mark(const char* phase) {
    if (!on) return;
    auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[trace] %-14s %8.3f ms\n", phase, std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
};

struct Kernel {
  uint64_t object = 0;
  uint32_t kasz = 0, gsz = 0, psz = 0;
};

Kernel kernel(hsa_executable_t exe, hsa_agent_t gpu, const char* name) {
  hsa_executable_symbol_t sym;
  check(hsa_executable_get_symbol_by_name(exe, name, &gpu, &sym), name);
  Kernel k;
  check(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.object), "kernel object");
  check(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.kasz), "kernarg size");
  check(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.gsz), "group size");
  check(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.psz), "private size");
  return k;
}

// One AQL kernel-dispatch packet of `groups` work-groups, with the barrier bit so packets on
// the queue run in order; system-scope fences both sides.
void dispatch(hsa_queue_t* q, const Kernel& k, void* kargs, uint64_t groups, hsa_signal_t completion) {
  if (groups == 0 || groups * kWG > UINT32_MAX) throw Fail{"bad dispatch size", HSA_STATUS_ERROR};
  const uint64_t idx = hsa_queue_add_write_index_screlease(q, 1);
  while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {
  }
  auto* pkt = static_cast<hsa_kernel_dispatch_packet_t*>(q->base_address) + (idx & (q->size - 1));
  std::memset(reinterpret_cast<char*>(pkt) + 4, 0, sizeof(*pkt) - 4);
  pkt->workgroup_size_x = kWG;
  pkt->workgroup_size_y = pkt->workgroup_size_z = 1;
  pkt->grid_size_x = static_cast<uint32_t>(groups * kWG);
  pkt->grid_size_y = pkt->grid_size_z = 1;
  pkt->kernel_object = k.object;
  pkt->kernarg_address = kargs;
  pkt->private_segment_size = k.psz;
  pkt->group_segment_size = k.gsz;
  pkt->completion_signal = completion;
  const uint16_t setup = 1u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
  const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1u << HSA_PACKET_HEADER_BARRIER) |
                          (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                          (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
  __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), static_cast<uint32_t>(header) | (static_cast<uint32_t>(setup) << 16),
                   __ATOMIC_RELEASE);
  hsa_signal_store_screlease(q->doorbell_signal, static_cast<hsa_signal_value_t>(idx));
}

struct CopyArgs {  // amdkube_copy: src, dst, float count, work-groups launched
  const float* src;
  float* dst;
  unsigned long long n;
  unsigned groups;
};

struct Args {  // amdkube_vadd: a, b, c, float count, work-groups launched
  const float* a;
  const float* b;
  float* c;
  unsigned long long n;
  unsigned groups;
};

// the streaming grid: one work-group per 256 16-byte words, at most 64 per CU (gpu_common.h)
uint32_t stream_groups(uint64_t floats, uint32_t cus) {
  const uint64_t want = (floats / 4 + kWG - 1) / kWG;
  const uint64_t cap = static_cast<uint64_t>(cus ? cus : 256) * 64;
  return static_cast<uint32_t>(want < 1 ? 1 : (want < cap ? want : cap));
}

}  // namespace

int main(int argc, char** argv) {
  size_t n = 50000;
  bool print_uuid = false, json = false, shutdown = true;
  int expect = -1;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--fast-exit")) shutdown = false;
    if ((!std::strcmp(argv[i], "-n") || !std::strcmp(argv[i], "--elements")) && i + 1 < argc) n = std::strtoull(argv[++i], nullptr, 10);
    else if (!std::strcmp(argv[i], "--print-uuid")) print_uuid = true;
    else if (!std::strcmp(argv[i], "--json")) json = true;
    else if (!std::strcmp(argv[i], "--expect-devices") && i + 1 < argc) expect = std::atoi(argv[++i]);
  }
  if (n == 0) {
    std::fprintf(stderr, "hsa-vector-add: -n must be > 0\n");
    return 4;
  }
  Trace tr;
  try {
    const hsa_status_t init = hsa_init();
    if (init != HSA_STATUS_SUCCESS) {
      // no /dev/kfd (or no render node) for this container: ROCr cannot open a GPU at all
      const char* msg = nullptr;
      hsa_status_string(init, &msg);
      std::fprintf(stderr, "no GPU visible to this container (hsa_init: %s)\n", msg ? msg : "error");
      return 2;
    }
    tr.mark("hsa_init");
    Agents ag;
    check(hsa_iterate_agents(on_agent, &ag), "iterate agents");
    const int count = static_cast<int>(ag.gpus.size());
    if (count < 1) {
      std::fprintf(stderr, "no GPU visible to this container\n");
      return 2;
    }
    if (expect >= 0 && count != expect) {
      std::fprintf(stderr, "expected %d visible GPU(s), found %d\n", expect, count);
      return 3;
    }
    if (!ag.have_cpu) throw Fail{"no CPU agent", HSA_STATUS_ERROR};
    hsa_agent_t gpu = ag.gpus[0];
    GpuId id = identify(gpu);
    if (print_uuid || !json)
      std::printf("GPU 0: %s %s bus=%s uuid=%s cus=%u visible=%d\n", id.product.c_str(), id.arch.c_str(), id.bus.c_str(),
                  id.uuid.c_str(), id.cus, count);
    std::printf("[Vector addition of %zu elements]\n", n);
    tr.mark("agents");

    Pools pools;
    check(hsa_amd_agent_iterate_memory_pools(gpu, on_gpu_pool, &pools), "gpu pools");
    check(hsa_amd_agent_iterate_memory_pools(ag.cpu, on_cpu_pool, &pools), "cpu pools");
    if (!pools.have_device || !pools.have_kernarg || !pools.have_host) throw Fail{"memory pools missing", HSA_STATUS_ERROR};

    // the embedded code object → executable → kernel descriptor
    hsa_code_object_reader_t reader;
    check(hsa_code_object_reader_create_from_memory(amdkube_vadd_co, amdkube_vadd_co_end - amdkube_vadd_co, &reader),
          "code object reader");
    hsa_executable_t exe;
    check(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe), "executable");
    check(hsa_executable_load_agent_code_object(exe, gpu, reader, nullptr, nullptr), "load code object (gfx950 only)");
    check(hsa_executable_freeze(exe, nullptr), "freeze executable");
    const Kernel vadd = kernel(exe, gpu, "amdkube_vadd.kd"), copy = kernel(exe, gpu, "amdkube_copy.kd");
    if (vadd.kasz != offsetof(Args, groups) + sizeof(unsigned) || copy.kasz != offsetof(CopyArgs, groups) + sizeof(unsigned))
      throw Fail{"unexpected kernarg segment size", HSA_STATUS_ERROR};
    tr.mark("code object");

    // data: host staging (GPU-accessible system memory) and device buffers
    // a, b, c each start on a 256-byte boundary (the copy kernel moves 16-byte words)
    const size_t stride = (n + 63) & ~static_cast<size_t>(63);
    const size_t bytes = n * sizeof(float), span = 3 * stride * sizeof(float);
    float *ha = nullptr, *hb = nullptr, *hc = nullptr, *da = nullptr, *db = nullptr, *dc = nullptr;
    check(hsa_amd_memory_pool_allocate(pools.host, span, 0, reinterpret_cast<void**>(&ha)), "host alloc");
    hb = ha + stride;
    hc = hb + stride;
    check(hsa_amd_memory_pool_allocate(pools.device, span, 0, reinterpret_cast<void**>(&da)), "device alloc");
    db = da + stride;
    dc = db + stride;
    check(hsa_amd_agents_allow_access(1, &gpu, nullptr, ha), "host access");
    uint32_t s = 12345u;       // the same inputs as rocm-vector-add
    for (size_t i = 0; i < n; ++i) {
      s = s * 1664525u + 1013904223u;
      ha[i] = static_cast<float>(s >> 8) / 16777216.0f;
      s = s * 1664525u + 1013904223u;
      hb[i] = static_cast<float>(s >> 8) / 16777216.0f;
    }
    std::memset(hc, 0xff, bytes);
    tr.mark("alloc + fill");
    hsa_signal_t done;
    check(hsa_signal_create(1, 0, nullptr, &done), "signal");
    // one kernarg block for the three packets, each slot 64-byte aligned
    const size_t slot = 64 * ((std::max<uint32_t>(vadd.kasz, copy.kasz) + 63) / 64);
    char* kargs = nullptr;
    check(hsa_amd_memory_pool_allocate(pools.kernarg, 3 * slot, 0, reinterpret_cast<void**>(&kargs)), "kernarg alloc");
    check(hsa_amd_agents_allow_access(1, &gpu, nullptr, kargs), "kernarg access");
    std::memset(kargs, 0, 3 * slot);
    const uint32_t g_in = stream_groups(2 * stride, id.cus), g_add = stream_groups(n, id.cus);
    *reinterpret_cast<CopyArgs*>(kargs) = CopyArgs{ha, da, 2 * static_cast<unsigned long long>(stride), g_in};
    *reinterpret_cast<Args*>(kargs + slot) = Args{da, db, dc, static_cast<unsigned long long>(n), g_add};
    *reinterpret_cast<CopyArgs*>(kargs + 2 * slot) = CopyArgs{dc, hc, static_cast<unsigned long long>(n), g_add};

    hsa_queue_t* q = nullptr;
    check(hsa_queue_create(gpu, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q), "queue");
    tr.mark("queue");
    const auto t0 = std::chrono::steady_clock::now();
    dispatch(q, copy, kargs, g_in, hsa_signal_t{0});                     // host a,b → device
    dispatch(q, vadd, kargs + slot, g_add, hsa_signal_t{0});             // c = a + b on device memory
    dispatch(q, copy, kargs + 2 * slot, g_add, done);                    // device c → host
    wait_zero(done, "vector add");
    const double kernel_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    tr.mark("gpu work");
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i)
      if (std::fabs(ha[i] + hb[i] - hc[i]) > 1e-5f) ++bad;
    tr.mark("verify");

    if (shutdown) {
      hsa_queue_destroy(q);
      hsa_signal_destroy(done);
      hsa_amd_memory_pool_free(kargs);
      hsa_amd_memory_pool_free(da);
      hsa_amd_memory_pool_free(ha);
      hsa_executable_destroy(exe);
      hsa_code_object_reader_destroy(reader);
      hsa_shut_down();
      tr.mark("shut down");
    }
    if (json)
      std::printf("{\"ok\":%s,\"n\":%zu,\"kernel_ms\":%.4f,\"uuid\":\"%s\",\"bus\":\"%s\",\"arch\":\"%s\",\"visible\":%d,\"runtime\":\"hsa\"}\n",
                  bad ? "false" : "true", n, kernel_ms, id.uuid.c_str(), id.bus.c_str(), id.arch.c_str(), count);
    if (bad) {
      std::printf("Result verification failed (%zu mismatches)\nTest FAILED\n", bad);
      return 1;
    }
    std::printf("Test PASSED\n");
    return 0;
  } catch (const Fail& f) {
    const char* msg = nullptr;
    hsa_status_string(f.st, &msg);
    std::fprintf(stderr, "hsa-vector-add: %s: %s\n", f.what.c_str(), msg ? msg : "error");
    return 4;
  }
}
