// In-process HIP validation ops (pybind11 module amdkube._native._hipops).
//
// The AMD device plugin uses these as its health probe (HBM pattern check before a GPU
// is advertised Healthy) and the GPU test tier uses them to check the kernels against a
// host fp32 reference. Kernels live in kernels/gpu_common.h (shared with the pod binaries).
#include <pybind11/numpy.h>
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
  // caller-supplied data (numpy arrays, e.g. torch.Tensor.numpy()) → the same kernels
  m.def(
      "vector_add_arrays",
      [](py::array_t<float, py::array::c_style | py::array::forcecast> a,
         py::array_t<float, py::array::c_style | py::array::forcecast> b, int dev) {
        std::vector<float> va(a.data(), a.data() + a.size()), vb(b.data(), b.data() + b.size()), vc;
        {
          py::gil_scoped_release nogil;
          vc = amdkube::vector_add_host(va, vb, dev);
        }
        return py::array_t<float>(vc.size(), vc.data());
      },
      py::arg("a"), py::arg("b"), py::arg("device") = 0);
  m.def(
      "hbm_pattern",
      [](size_t n16, uint32_t seed, int dev) {
        std::vector<uint32_t> w;
        {
          py::gil_scoped_release nogil;
          w = amdkube::hbm_pattern_host(n16, seed, dev);
        }
        return py::array_t<uint32_t>(w.size(), w.data());
      },
      py::arg("n16"), py::arg("seed") = 0x5eedu, py::arg("device") = 0);
  m.def(
      "hbm_verify_words",
      [](py::array_t<uint32_t, py::array::c_style | py::array::forcecast> words, uint32_t seed, int dev) {
        std::vector<uint32_t> w(words.data(), words.data() + words.size());
        py::gil_scoped_release nogil;
        return amdkube::hbm_verify_host(w, seed, dev);
      },
      py::arg("words"), py::arg("seed") = 0x5eedu, py::arg("device") = 0);
  m.def(
      "hbm_copy_words",
      [](py::array_t<uint32_t, py::array::c_style | py::array::forcecast> words, int dev) {
        std::vector<uint32_t> w(words.data(), words.data() + words.size()), o;
        {
          py::gil_scoped_release nogil;
          o = amdkube::hbm_copy_host(w, dev);
        }
        return py::array_t<uint32_t>(o.size(), o.data());
      },
      py::arg("words"), py::arg("device") = 0);
  m.def(
      "mfma_tile",
      [](py::array_t<uint16_t, py::array::c_style | py::array::forcecast> a_bits,
         py::array_t<uint16_t, py::array::c_style | py::array::forcecast> b_bits, int k, int dev) {
        std::vector<uint16_t> a(a_bits.data(), a_bits.data() + a_bits.size()), b(b_bits.data(), b_bits.data() + b_bits.size());
        std::vector<float> c;
        {
          py::gil_scoped_release nogil;
          c = amdkube::mfma_tile_host(a, b, k, dev);
        }
        return py::array_t<float>({32, 32}, c.data());
      },
      py::arg("a_bits"), py::arg("b_bits"), py::arg("k"), py::arg("device") = 0);
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
