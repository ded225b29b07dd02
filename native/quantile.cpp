// pybind11 binding of quantile_core.h: amdkube._native._quantile.Summary, the per-label-set state
// behind amdkube.utils.quantiles.QuantileSummary (Prometheus Summary quantiles for the kubelet,
// device manager and apiserver latency families).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "quantile_core.h"

namespace py = pybind11;

PYBIND11_MODULE(_quantile, mod) {
  mod.doc() = "windowed CKMS targeted-quantile summaries (Prometheus Go client semantics)";
  py::class_<amdkube::WindowedSummary>(mod, "Summary")
      .def(py::init<std::vector<std::pair<double, double>>, double, int, double>(), py::arg("objectives"),
           py::arg("max_age"), py::arg("age_buckets"), py::arg("now"))
      .def("observe", &amdkube::WindowedSummary::observe, py::arg("value"), py::arg("now"))
      .def("quantiles", &amdkube::WindowedSummary::quantiles, py::arg("now"))
      .def_property_readonly("sum", &amdkube::WindowedSummary::sum)
      .def_property_readonly("count", &amdkube::WindowedSummary::count)
      .def_property_readonly("head_size", &amdkube::WindowedSummary::head_size);
}
