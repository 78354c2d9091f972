// pybind11 bindings of the _vodahip extension.  Tensors cross the boundary as raw device
// pointers + HIP stream handles; shape/dtype/alignment validation happens in the Python
// wrappers (vodascheduler_amd/ops/*.py) BEFORE anything is launched.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "common.h"
#include "ops.h"

namespace py = pybind11;
using namespace voda;

PYBIND11_MODULE(_vodahip, m) {
  m.doc() = "vodascheduler_amd CDNA4 (gfx950) kernels + RCCL engine";
  m.attr("GPU_ARCH") = "gfx950";
  m.attr("LAYERNORM_MAX_N") = kLayerNormMaxN;
  m.attr("SOFTMAX_MAX_S") = kSoftmaxMaxS;

  m.def("sgd_step", &sgd_step);
  m.def("adam_step", &adam_step);
  m.def("rmsprop_step", &rmsprop_step);
  m.def("cast_scale", &cast_scale);
  m.def("multi_tensor_copy", &multi_tensor_copy);
  m.def("adasum_combine", &adasum_combine);
  m.def("wgrad_workspace_floats", &wgrad_workspace_floats);
  m.def("wgrad_gemm", &wgrad_gemm);
  m.def("sgemm_f32_workspace_floats", &sgemm_f32_workspace_floats);
  m.def("sgemm_f32", &sgemm_f32);
  m.def("sgemm_f32_set_stagger", &sgemm_f32_set_stagger);
  m.def("sgemm_conv_wgrad_set_ws", &sgemm_conv_wgrad_set_ws);
  m.def("sgemm_conv_fwd_set_v8", &sgemm_conv_fwd_set_v8);
  m.def("sgemm_set_reduce_groups", &sgemm_set_reduce_groups);
  m.def("sgemm_set_write_map", &sgemm_set_write_map);
  m.def("sgemm_conv_fwd_f32", &sgemm_conv_fwd_f32);
  m.def("sgemm_conv_dgrad_s2_class", &sgemm_conv_dgrad_s2_class);
  m.def("sgemm_conv_wgrad_f32", &sgemm_conv_wgrad_f32);
  m.def("wgrad_conv_workspace_floats", &wgrad_conv_workspace_floats);
  m.def("wgrad_conv", &wgrad_conv);
  m.def("gelu_tanh_fwd", &gelu_tanh_fwd);
  m.def("gelu_tanh_bwd", &gelu_tanh_bwd);
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("layernorm_bwd", &layernorm_bwd);
  m.def("layernorm_bwd_partial_rows", &layernorm_bwd_partial_rows);
  m.def("layernorm_set_bwd_waves", &layernorm_set_bwd_waves);
  m.def("masked_softmax_fwd", &masked_softmax_fwd);
  m.def("masked_softmax_bwd", &masked_softmax_bwd);
  m.def("xent_fwd", &xent_fwd);
  m.def("xent_bwd", &xent_bwd);

  m.def("bn_workspace_floats", &bn_workspace_floats);
  m.def("bn_set_tuning", &bn_set_tuning, py::arg("deep") = -1, py::arg("blocks") = -1, py::arg("sweep") = -1);
  m.def("bn_get_tuning", &bn_get_tuning);
  m.def("bn_fwd_train", &bn_fwd_train);
  m.def("bn_apply", &bn_apply);
  m.def("bn_bwd", &bn_bwd);
  m.def("bn2_workspace_floats", &bn2_workspace_floats);
  m.def("bn2_fwd_train", &bn2_fwd_train);
  m.def("bn2_bwd", &bn2_bwd);

  m.def("bn_pool_workspace_floats", &bn_pool_workspace_floats);
  m.def("bn_pool_fwd_train", &bn_pool_fwd_train);
  m.def("bn_pool_bwd", &bn_pool_bwd);
  m.def("global_avgpool_bwd", &global_avgpool_bwd);
  m.def("gemm_bnstats_supported", &gemm_bnstats_supported);
  m.def("gemm_bnstats_groups", &gemm_bnstats_groups);
  m.def("gemm_bnstats", &gemm_bnstats, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("part"), py::arg("M"),
        py::arg("N"), py::arg("K"), py::arg("G"), py::arg("stream"), py::arg("accumulate") = false);
  m.def("gemm_f32_stats_supported", &gemm_f32_stats_supported);
  m.def("gemm_f32_dgrad_bn", &gemm_f32_dgrad_bn);
  m.def("stem_conv_fwd_f32", &stem_conv_fwd_f32);
  m.def("attn_f32_set_fused_bwd", &attn_f32_set_fused_bwd);
  m.def("stem_wgrad_f32_workspace_floats", &stem_wgrad_f32_workspace_floats);
  m.def("stem_wgrad_f32_supported", &stem_wgrad_f32_supported);
  m.def("stem_conv_wgrad_f32", &stem_conv_wgrad_f32);
  m.def("gemm_epilogue_algos", &gemm_epilogue_algos);
  m.def("gemm_gelu_aux", &gemm_gelu_aux);
  m.def("gemm_dgelu", &gemm_dgelu);
  m.def("gemm_f32_dgrad_bn_supported", &gemm_f32_dgrad_bn_supported);
  m.def("gemm_f32_dgrad_bn_groups", &gemm_f32_dgrad_bn_groups);
  m.def("gemm_f32_stats_groups", &gemm_f32_stats_groups);
  m.def("gemm_f32_stats", &gemm_f32_stats, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("part"), py::arg("M"),
        py::arg("N"), py::arg("K"), py::arg("G"), py::arg("stream"), py::arg("accumulate") = false,
        py::arg("w_kn") = false);
  m.def("subsample2d", &subsample2d);
  m.def("conv3x3_c64_wgrad_workspace_floats", &conv3x3_c64_wgrad_workspace_floats);
  m.def("conv3x3_c64_wgrad", &conv3x3_c64_wgrad);
  m.def("filter_flip_t", &filter_flip_t);
  m.def("wino_f23_supported", &wino_f23_supported);
  m.def("wino_f23_filter", &wino_f23_filter);
  m.def("wino_f23_groups", &wino_f23_groups);
  m.def("wino_f23_fwd", &wino_f23_fwd);
  m.def("wino_f23_sx2_supported", &wino_f23_sx2_supported);
  m.def("wino_f23_set_onepos", &wino_f23_set_onepos);
  m.def("wino_f23_groups2", &wino_f23_groups2);
  m.def("wino_f23_fwd2", &wino_f23_fwd2);
  m.def("stem_partial_rows", &stem_partial_rows);
  m.def("stem_pack", &stem_pack);
  m.def("stem_conv_fwd", &stem_conv_fwd);
  m.def("stem_wgrad_workspace_floats", &stem_wgrad_workspace_floats);
  m.def("stem_conv_wgrad", &stem_conv_wgrad);
  m.def("maxpool2d_fwd", &maxpool2d_fwd);
  m.def("maxpool2d_bwd", &maxpool2d_bwd);
  m.def("colsum_workspace_floats", &colsum_workspace_floats);
  m.def("colsum_accumulate", &colsum_accumulate);
  m.def("attention_supported", &attention_supported);
  m.def("attention_fwd", &attention_fwd);
  m.def("attention_bwd", &attention_bwd);
  m.def("attention_fwd_f32", &attention_fwd_f32);
  m.def("attention_bwd_f32", &attention_bwd_f32);

  m.def("rccl_unique_id", [] { return py::bytes(rccl_unique_id()); });
  m.def("rccl_version", &rccl_version);

  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init([](py::bytes uid, int nranks, int rank, int device, double timeout_s, bool wait) {
             std::string id = uid;
             py::gil_scoped_release nogil;
             return new RcclComm(id, nranks, rank, device, timeout_s, wait);
           }),
           py::arg("uid"), py::arg("nranks"), py::arg("rank"), py::arg("device") = -1,
           py::arg("timeout_s") = 300.0, py::arg("wait") = true)
      .def("poll_ready", &RcclComm::poll_ready, py::call_guard<py::gil_scoped_release>())
      .def("allreduce", &RcclComm::allreduce, py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &RcclComm::broadcast, py::call_guard<py::gil_scoped_release>())
      .def("allgather", &RcclComm::allgather, py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter", &RcclComm::reduce_scatter, py::call_guard<py::gil_scoped_release>())
      .def("alltoall", &RcclComm::alltoall, py::call_guard<py::gil_scoped_release>())
      .def("group_start", &RcclComm::group_start)
      .def("group_end", &RcclComm::group_end, py::call_guard<py::gil_scoped_release>())
      .def("async_error", &RcclComm::async_error)
      .def("abort", &RcclComm::abort, py::call_guard<py::gil_scoped_release>())
      .def("destroy", &RcclComm::destroy, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("size", &RcclComm::size)
      .def_property_readonly("alive", &RcclComm::alive);
}
