// In-process HIP validation ops (pybind11 module amdkube._native._hipops).
//
// The AMD device plugin uses these as its health probe (HBM pattern check before a GPU
// is advertised Healthy) and the GPU test tier uses them to check the kernels against a
// host fp32 reference. Kernels live in kernels/gpu_common.h (shared with the pod binaries).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../kernels/gpu_common.h"

namespace py = pybind11;

PYBIND11_MODULE(_hipops, m) {
  m.doc() = "amdkube HIP (gfx950) validation kernels: vector add, HBM probe, MFMA burn";
  m.def("device_count", []() {
    int n = 0;
    AK_HIP(hipGetDeviceCount(&n));
    return n;
  });
  m.def(
      "device_info",
      [](int dev) {
        amdkube::DevInfo d = amdkube::dev_info(dev);
        py::dict o;
        o["device"] = d.device;
        o["name"] = d.name;
        o["arch"] = d.arch;
        o["pci_bus_id"] = d.pci_bus_id;
        o["uuid"] = d.uuid;
        o["total_mem"] = d.total_mem;
        o["cu_count"] = d.cu_count;
        return o;
      },
      py::arg("device") = 0);
  m.def(
      "vector_add",
      [](size_t n, int dev) {
        amdkube::VaddResult r;
        {
          py::gil_scoped_release nogil;
          r = amdkube::run_vector_add(n, dev);
        }
        py::dict o;
        o["ok"] = r.ok;
        o["kernel_ms"] = r.kernel_ms;
        o["mismatches"] = r.mismatches;
        return o;
      },
      py::arg("n") = 50000, py::arg("device") = 0);
  m.def(
      "hbm_probe",
      [](size_t mib, int iters, int dev) {
        amdkube::HbmResult r;
        {
          py::gil_scoped_release nogil;
          r = amdkube::run_hbm_probe(mib << 20, iters, dev);
        }
        py::dict o;
        o["bytes"] = r.bytes;
        o["iters"] = r.iters;
        o["write_gbps"] = r.write_gbps;
        o["read_gbps"] = r.read_gbps;
        o["copy_gbps"] = r.copy_gbps;
        o["verify_gbps"] = r.verify_gbps;
        o["errors"] = r.errors;
        return o;
      },
      py::arg("mib") = 1024, py::arg("iters") = 5, py::arg("device") = 0);
  m.def(
      "mfma_burn",
      [](double ms, int dev) {
        amdkube::BurnResult r;
        {
          py::gil_scoped_release nogil;
          r = amdkube::run_mfma_burn(ms, dev);
        }
        py::dict o;
        o["ms"] = r.ms;
        o["iters"] = r.iters;
        o["blocks"] = r.blocks;
        o["bf16_tflops"] = r.tflops;
        return o;
      },
      py::arg("ms") = 100.0, py::arg("device") = 0);
}
