#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "vodacore.h"

namespace py = pybind11;

PYBIND11_MODULE(_vodacore, m) {
  m.doc() = "vodascheduler_amd host native core: Kuhn-Munkres assignment, FfDL DP";
  m.def("linear_assignment", &vodacore::linear_assignment, py::arg("cost"), py::arg("rows"), py::arg("cols"),
        py::arg("maximize") = false, py::call_guard<py::gil_scoped_release>(),
        "Optimal assignment of rows to columns of a dense row-major cost matrix; returns the column of each "
        "row (-1 when rows > cols and the row is unassigned).");
  m.def("ffdl_dp", &vodacore::ffdl_dp, py::arg("speedups"), py::arg("mins"), py::arg("maxs"), py::arg("K"),
        py::arg("allow_zero"), py::call_guard<py::gil_scoped_release>());
}
