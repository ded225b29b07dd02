// pybind11 binding of the topology allocator (see topo_core.h for the algorithm).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "topo_core.h"

namespace py = pybind11;
using namespace topo;

PYBIND11_MODULE(_topo, m) {
  m.doc() = "xGMI/NUMA topology-aware GPU subset selection (amdkube scheduler)";
  m.def(
      "select",
      [](const std::vector<int>& free, int k, const std::vector<std::vector<double>>& link,
         const std::vector<int>& numa, const std::vector<int>& all_free, const std::vector<int>& parent) {
        Problem p = make(free, k, link, numa, all_free, parent);
        std::tuple<std::vector<int>, double> r;
        {
          py::gil_scoped_release nogil;
          r = solve(p);
        }
        return r;
      },
      py::arg("free"), py::arg("k"), py::arg("link"), py::arg("numa"), py::arg("all_free") = std::vector<int>{},
      py::arg("parent") = std::vector<int>{},
      "Best k-subset of `free` -> (sorted indices, cost); cost=inf if infeasible");
  m.def(
      "score",
      [](const std::vector<int>& free, int k, const std::vector<std::vector<double>>& link,
         const std::vector<int>& numa, const std::vector<int>& all_free, const std::vector<int>& parent) {
        Problem p = make(free, k, link, numa, all_free, parent);
        auto r = solve(p);
        double c = std::get<1>(r);
        if (!std::isfinite(c)) return 0.0;
        std::set<int> groups(numa.begin(), numa.end());
        double s = 10.0 * (1.0 - c / max_cost(static_cast<int>(groups.size())));
        return std::max(0.0, std::min(10.0, s));
      },
      py::arg("free"), py::arg("k"), py::arg("link"), py::arg("numa"), py::arg("all_free") = std::vector<int>{},
      py::arg("parent") = std::vector<int>{},
      "Node score in [0,10] for placing k devices (GPUTopologyPriority)");
  m.attr("W_NUMA") = W_NUMA;
  m.attr("W_LINK") = W_LINK;
  m.attr("W_FRAG") = W_FRAG;
  m.attr("MAX_ENUM") = MAX_ENUM;
}
