// pybind11 module _hfens_hip: thin host entry points for the gfx950 kernels.
// Tensors cross the boundary as device pointers (torch.Tensor.data_ptr()) and the
// current HIP stream; the Python wrappers in hfens/ops validate shapes/dtypes.
#include <pybind11/pybind11.h>
#include <cstdint>

namespace hfens {
// infer.hip
void rbf_decision(uintptr_t Z, int n, int F, uintptr_t SVt, uintptr_t sn, uintptr_t coef, int mp,
                  double gamma, double b, uintptr_t out, uintptr_t stream);
void svc_proba1(uintptr_t dec, uintptr_t out, int n, double A, double B, uintptr_t stream);
void forest_raw(uintptr_t X, int n, int F, uintptr_t nodes, uintptr_t values, int T, int K,
                double init, double lr, uintptr_t out, uintptr_t stream);
// stack.hip
long long stack_infer_lds(int F, int mp, int nodes_total);
// liblinear_host.hip
int liblinear_l1r_lr(uintptr_t X, uintptr_t y, uintptr_t sw, int l, int n, double bias, double C0, double C1,
                     double eps, int max_newton_iter, long long seed, uintptr_t w);
// host.hip
void stack_plan_host(uintptr_t y_ptr, long long n, int n_folds, long long seed, uintptr_t folds_ptr,
                     uintptr_t rows_ptr, uintptr_t lens_ptr, uintptr_t out_ptr, uintptr_t meta_ptr);
#define HFENS_DECLS
#include "decls.inc"
#undef HFENS_DECLS
}  // namespace hfens

namespace py = pybind11;

PYBIND11_MODULE(_hfens_hip, m) {
  m.doc() = "hfens gfx950 HIP kernels (MI355X / CDNA4)";
  m.def("rbf_decision", &hfens::rbf_decision);
  m.def("svc_proba1", &hfens::svc_proba1);
  m.def("forest_raw", &hfens::forest_raw);
  m.def("stack_infer_lds", &hfens::stack_infer_lds);
  // (host-only and sequential: release the GIL so the stacking fit's six solves run in parallel threads)
  m.def("liblinear_l1r_lr", &hfens::liblinear_l1r_lr, py::call_guard<py::gil_scoped_release>());
  // (the label-only stacking plan on a helper thread while the main thread launches device work)
  m.def("stack_plan_host", &hfens::stack_plan_host, py::call_guard<py::gil_scoped_release>());
#define HFENS_DEFS
#include "decls.inc"
#undef HFENS_DEFS
  m.attr("arch") = "gfx950";
}
