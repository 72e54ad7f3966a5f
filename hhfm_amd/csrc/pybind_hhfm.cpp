// Thin pybind11 binding of the C ABI in include/hhfm.h.
// Takes raw device pointers / hipStream_t handles as integers (the Python
// layer passes tensor.data_ptr() and torch.cuda.current_stream().cuda_stream),
// releases the GIL around every launch and turns a non-zero status into an
// exception.  No torch types cross this boundary.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

#include "hhfm.h"

namespace py = pybind11;
using uptr = std::uintptr_t;

template <typename T>
static T* P(uptr p) { return reinterpret_cast<T*>(p); }
template <typename T>
static T* P_(uptr p) { return reinterpret_cast<T*>(p); }

static void check(int rc, const char* what) {
  if (rc == HHFM_OK) return;
  std::string msg = std::string(what) + ": " + hhfm_error_string(rc) +
                    " (code " + std::to_string(rc) + ")";
  if (rc == HHFM_EINVAL || rc == HHFM_EUNSUPPORTED || rc == HHFM_EWORKSPACE)
    throw py::value_error(msg);
  throw std::runtime_error(msg);
}

PYBIND11_MODULE(_hhfm, m) {
  m.doc() = "pybind11 binding of libhhfm (MI355X FM-family scoring kernels)";
  m.attr("ABI_VERSION") = HHFM_ABI_VERSION;
  m.attr("F32") = (int)HHFM_F32;
  m.attr("BF16") = (int)HHFM_BF16;
  m.attr("MODE_FM") = (int)HHFM_MODE_FM;
  m.attr("MODE_HHFM") = (int)HHFM_MODE_HHFM;
  m.attr("PLAN_EXACT_FP32") = HHFM_PLAN_EXACT_FP32;
  m.attr("PLAN_NO_SEED") = HHFM_PLAN_NO_SEED;
  m.attr("PLAN_NO_RING") = HHFM_PLAN_NO_RING;
  m.attr("PLAN_RING_ALT") = HHFM_PLAN_RING_ALT;
  m.attr("PLAN_GEMM") = HHFM_PLAN_GEMM;
  m.attr("PLAN_ROW_FM") = HHFM_PLAN_ROW_FM;
  m.attr("PLAN_UNSTAGED") = HHFM_PLAN_UNSTAGED;
  m.attr("PLAN_UNGROUPED") = HHFM_PLAN_UNGROUPED;
  m.attr("PLAN_NARROW") = HHFM_PLAN_NARROW;
  m.attr("PLAN_PER_FIELD") = HHFM_PLAN_PER_FIELD;
  m.attr("PLAN_ONE_WAVE") = HHFM_PLAN_ONE_WAVE;

  m.def("abi_version", [] { return hhfm_abi_version(); });

  m.def("fm_score_rows",
        [](uptr idx, int64_t B, int F, uptr E, int64_t M, int k, int dtype,
           uptr w, float w0, uptr out, uptr stream) {
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_fm_score_rows(P<const int32_t>(idx), B, F, P<const void>(E),
                                    M, k, dtype, P<const float>(w), w0,
                                    P<float>(out), P<void>(stream));
          }
          check(rc, "hhfm_fm_score_rows");
        });

  m.def("fm_score_rows_ex",
        [](uptr idx, int64_t B, int F, uptr E, int64_t M, int k, int dtype,
           uptr w, float w0, uptr out, int flags, uptr status, uptr stream) {
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_fm_score_rows_ex(P<const int32_t>(idx), B, F, P<const void>(E),
                                       M, k, dtype, P<const float>(w), w0,
                                       P<float>(out), flags, P<int32_t>(status),
                                       P<void>(stream));
          }
          check(rc, "hhfm_fm_score_rows_ex");
        });

  m.def("hybrid_score_rows",
        [](uptr idx, int64_t B, int ncols, int ucol, int icol, int c0, int c1,
           int t0, int t1, uptr E, int64_t M, int k, int dtype, uptr out,
           uptr status, uptr stream) {
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_hybrid_score_rows_ex(P<const int32_t>(idx), B, ncols, ucol,
                                           icol, c0, c1, t0, t1, P<const void>(E),
                                           M, k, dtype, P<float>(out), P<int32_t>(status),
                                           P<void>(stream));
          }
          check(rc, "hhfm_hybrid_score_rows_ex");
        });

  m.def("catalog_topk_workspace",
        [](int64_t B, int item_count, int k, int K) {
          size_t ws = 0;
          check(hhfm_catalog_topk_workspace(B, item_count, k, K, &ws),
                "hhfm_catalog_topk_workspace");
          return ws;
        });

  m.def("catalog_topk",
        [](uptr qidx, int64_t B, int ncols, int mode, int ucol, int c0, int c1,
           int t0, int t1, uptr E, int64_t M, int k, int dtype, uptr w,
           int item_row_begin, int item_count, int global_item_base, int K,
           uptr top_score, uptr top_idx, uptr ws, size_t ws_bytes, int plan, uptr status,
           uptr stream) {
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_catalog_topk_ex(
                P<const int32_t>(qidx), B, ncols, mode, ucol, c0, c1, t0, t1,
                P<const void>(E), M, k, dtype, P<const float>(w),
                item_row_begin, item_count, global_item_base, K,
                P<float>(top_score), P<int32_t>(top_idx), P<void>(ws), ws_bytes, plan,
                P<int32_t>(status), P<void>(stream));
          }
          check(rc, "hhfm_catalog_topk_ex");
        });

  m.def("check_ids", [](uptr idx, int64_t n, int64_t M, uptr status, uptr stream) {
    int rc;
    {
      py::gil_scoped_release nogil;
      rc = hhfm_check_ids(P<const int32_t>(idx), n, M, P<int32_t>(status), P<void>(stream));
    }
    check(rc, "hhfm_check_ids");
  });

  // returns HHFM_OK / HHFM_EINVAL as an int (the caller raises with its own message)
  m.def("status_read", [](uptr status, uptr stream) {
    int rc;
    {
      py::gil_scoped_release nogil;
      rc = hhfm_status_read(P<int32_t>(status), P<void>(stream));
    }
    if (rc != HHFM_OK && rc != HHFM_EINVAL) check(rc, "hhfm_status_read");
    return rc;
  });

  m.def("probe_stream_read", [](uptr buf, int64_t bytes, int mode, uptr sink, uptr stream) {
    int rc;
    {
      py::gil_scoped_release nogil;
      rc = hhfm_probe_stream_read(P<const void>(buf), bytes, mode, P<float>(sink),
                                  P<void>(stream));
    }
    check(rc, "hhfm_probe_stream_read");
  });

  m.def("pf_contains",
        [](uptr keys, int64_t nkeys, int key_cols, uptr codes, int64_t ncodes, uptr rows,
           int64_t B, int ncols, int item_col, uptr cand, int num, uptr out, uptr stream) {
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_pf_contains(P<const int32_t>(keys), nkeys, key_cols, P<const int64_t>(codes),
                                  ncodes, P<const int32_t>(rows), B, ncols, item_col,
                                  P<const int32_t>(cand), num, P<uint8_t>(out), P<void>(stream));
          }
          check(rc, "hhfm_pf_contains");
        });

  m.def("topk_walk",
        [](uptr pred, int64_t B, int Pn, uptr target, uptr positive, int TopK, uptr outcome,
           uptr stream) {
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_topk_walk(P<const int32_t>(pred), B, Pn, P<const int32_t>(target),
                                P<const uint8_t>(positive), TopK, P<int32_t>(outcome),
                                P<void>(stream));
          }
          check(rc, "hhfm_topk_walk");
        });

  m.def("sample_negative_workspace", [](int64_t B, int num) {
    size_t n = 0;
    check(hhfm_sample_negative_workspace(B, num, &n), "hhfm_sample_negative_workspace");
    return n;
  });

  m.def("sample_negative_workspace_ex", [](int64_t B, int num, int64_t lo, int64_t hi,
                                          int64_t nkeys) {
    size_t n = 0;
    check(hhfm_sample_negative_workspace_ex(B, num, lo, hi, nkeys, &n),
          "hhfm_sample_negative_workspace_ex");
    return n;
  });

  m.def("sample_negative",
        [](uptr state, int64_t lo, int64_t hi, uptr rows, int64_t B, int ncols, int item_col,
           int num, uptr keys, int64_t nkeys, uptr codes, int64_t ncodes, uptr samples, uptr ws,
           size_t ws_bytes, uptr stream) {
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_sample_negative(P<uint32_t>(state), lo, hi, P<const int32_t>(rows), B,
                                      ncols, item_col, num, P<const int32_t>(keys), nkeys,
                                      P<const int64_t>(codes), ncodes, P<int64_t>(samples),
                                      P<void>(ws), ws_bytes, P<void>(stream));
          }
          check(rc, "hhfm_sample_negative");
        });

  m.def("libfm_encode",
        [](py::bytes buf, int ncols, int64_t max_rows, uptr labels, uptr ids, uptr distinct) {
          std::string_view v = buf;
          int64_t rows = 0, fm = 0;
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_libfm_encode(v.data(), (int64_t)v.size(), ncols, max_rows, P<double>(labels),
                                   P<int64_t>(ids), &rows, &fm, P<int64_t>(distinct));
          }
          check(rc, "hhfm_libfm_encode");
          return py::make_tuple(rows, fm);
        });

  m.def("loader_split",
        [](uptr data, int64_t rows, int ncols, int item_col, int64_t test_size, uptr is_test) {
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_loader_split(P<const int64_t>(data), rows, ncols, item_col, test_size,
                                   P<uint8_t>(is_test));
          }
          check(rc, "hhfm_loader_split");
        });

  m.def("topk_merge",
        [](uptr in_score, uptr in_idx, int R, int64_t B, int K, uptr out_score,
           uptr out_idx, uptr stream) {
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_topk_merge(P<const float>(in_score), P<const int32_t>(in_idx),
                                 R, B, K, P<float>(out_score), P<int32_t>(out_idx),
                                 P<void>(stream));
          }
          check(rc, "hhfm_topk_merge");
        });

  m.def("dfm_forward_workspace",
        [](int64_t B, std::vector<int32_t> dims, int mlp_dtype) {
          size_t ws = 0;
          check(hhfm_dfm_forward_workspace(B, (int)dims.size(), dims.data(), mlp_dtype, &ws),
                "hhfm_dfm_forward_workspace");
          return ws;
        });

  m.def("dfm_forward_workspace_ex",
        [](int64_t B, int F, int k, int64_t M, std::vector<int32_t> dims, int mlp_dtype,
           int proj_mode) {
          size_t ws = 0;
          check(hhfm_dfm_forward_workspace_ex(B, F, k, M, (int)dims.size(), dims.data(),
                                              mlp_dtype, proj_mode, &ws),
                "hhfm_dfm_forward_workspace_ex");
          return ws;
        });

  m.def("dfm_forward",
        [](uptr idx, int64_t B, int F, uptr E, int64_t M, int k, int dtype, uptr w,
           std::vector<int32_t> dims, std::vector<uptr> Wt, std::vector<uptr> bias,
           int mlp_dtype, uptr Wp, float bp, uptr out, int proj_mode, int plan, uptr ws,
           size_t ws_bytes, uptr stream) {
          if (Wt.size() != dims.size() || bias.size() != dims.size())
            throw py::value_error("dims, Wt and bias must have the same length");
          std::vector<const void*> W(Wt.size());
          std::vector<const float*> b(bias.size());
          for (size_t i = 0; i < W.size(); ++i) {
            W[i] = P<const void>(Wt[i]);
            b[i] = P<const float>(bias[i]);
          }
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_dfm_forward_ex(P<const int32_t>(idx), B, F, P<const void>(E), M, k,
                                     dtype, P<const float>(w), (int)dims.size(), dims.data(),
                                     W.data(), b.data(), mlp_dtype, P<const float>(Wp), bp,
                                     P<float>(out), proj_mode, plan, P<void>(ws), ws_bytes,
                                     P<void>(stream));
          }
          check(rc, "hhfm_dfm_forward_ex");
        });

  m.def("dfm_catalog_topk_workspace",
        [](int64_t B, int F, int item_count, std::vector<int32_t> dims, int mlp_dtype,
           int64_t chunk_rows) {
          size_t ws = 0;
          check(hhfm_dfm_catalog_topk_workspace(B, F, item_count, (int)dims.size(), dims.data(),
                                                mlp_dtype, chunk_rows, &ws),
                "hhfm_dfm_catalog_topk_workspace");
          return ws;
        });

  m.def("dfm_catalog_topk_workspace_ex",
        [](int64_t B, int F, int k, int64_t M, int item_count, std::vector<int32_t> dims,
           int mlp_dtype, int64_t chunk_rows, int proj_mode) {
          size_t ws = 0;
          check(hhfm_dfm_catalog_topk_workspace_ex(B, F, k, M, item_count, (int)dims.size(),
                                                   dims.data(), mlp_dtype, chunk_rows, proj_mode,
                                                   &ws),
                "hhfm_dfm_catalog_topk_workspace_ex");
          return ws;
        });

  m.def("dfm_catalog_topk",
        [](uptr qidx, int64_t B, int F, int item_col, uptr E, int64_t M, int k, int dtype,
           uptr w, std::vector<int32_t> dims, std::vector<uptr> Wt, std::vector<uptr> bias,
           int mlp_dtype, uptr Wp, float bp, int item_row_begin, int item_count,
           int global_item_base, int K, int64_t chunk_rows, uptr top_score, uptr top_idx,
           int proj_mode, int plan, uptr ws, size_t ws_bytes, uptr stream) {
          if (Wt.size() != dims.size() || bias.size() != dims.size())
            throw py::value_error("dims, Wt and bias must have the same length");
          std::vector<const void*> W(Wt.size());
          std::vector<const float*> b(bias.size());
          for (size_t i = 0; i < W.size(); ++i) {
            W[i] = P<const void>(Wt[i]);
            b[i] = P<const float>(bias[i]);
          }
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_dfm_catalog_topk_ex(P<const int32_t>(qidx), B, F, item_col,
                                          P<const void>(E), M, k, dtype, P<const float>(w),
                                          (int)dims.size(), dims.data(), W.data(), b.data(),
                                          mlp_dtype, P<const float>(Wp), bp, item_row_begin,
                                          item_count, global_item_base, K, chunk_rows,
                                          P<float>(top_score), P<int32_t>(top_idx), proj_mode,
                                          plan, P<void>(ws), ws_bytes, P<void>(stream));
          }
          check(rc, "hhfm_dfm_catalog_topk_ex");
        });

  m.def("afm_forward_workspace", [](int64_t B, int F, int A) {
    size_t ws = 0;
    check(hhfm_afm_forward_workspace(B, F, A, &ws), "hhfm_afm_forward_workspace");
    return ws;
  });

  m.def("afm_forward",
        [](uptr idx, int64_t B, int F, uptr E, int64_t M, int k, int dtype, uptr w, float w0,
           uptr Wt, uptr ab, uptr ap, int A, uptr P, uptr out, int plan, uptr ws,
           size_t ws_bytes, uptr stream) {
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_afm_forward_ex(P_<const int32_t>(idx), B, F, P_<const void>(E), M, k,
                                     dtype, P_<const float>(w), w0, P_<const float>(Wt),
                                     P_<const float>(ab), P_<const float>(ap), A,
                                     P_<const float>(P), P_<float>(out), plan, P_<void>(ws),
                                     ws_bytes, P_<void>(stream));
          }
          check(rc, "hhfm_afm_forward_ex");
        });

  m.def("afm_catalog_topk_workspace",
        [](int64_t B, int F, int k, int A, int item_count, int64_t max_cols, int plan) {
          size_t ws = 0;
          check(hhfm_afm_catalog_topk_workspace_ex(B, F, k, A, item_count, max_cols, plan, &ws),
                "hhfm_afm_catalog_topk_workspace_ex");
          return ws;
        });

  m.def("afm_catalog_topk",
        [](uptr q, int64_t B, int F, uptr E, int64_t M, int k, int dtype, uptr w, uptr Wt,
           uptr ab, uptr ap, int A, uptr P, int irb, int cnt, int gbase, int K,
           int64_t max_cols, uptr ts, uptr ti, int plan, uptr ws, size_t ws_bytes,
           uptr stream) {
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_afm_catalog_topk_ex(P_<const int32_t>(q), B, F, P_<const void>(E), M, k,
                                          dtype, P_<const float>(w), P_<const float>(Wt),
                                          P_<const float>(ab), P_<const float>(ap), A,
                                          P_<const float>(P), irb, cnt, gbase, K, max_cols,
                                          P_<float>(ts), P_<int32_t>(ti), plan, P_<void>(ws),
                                          ws_bytes, P_<void>(stream));
          }
          check(rc, "hhfm_afm_catalog_topk_ex");
        });

  m.def("train_workspace", [](int64_t M, int k) { return hhfm_train_workspace(M, k); });

  m.def("fm_train_step",
        [](uptr idx, uptr y, int64_t B, int F, uptr E, uptr w, uptr w0, int64_t M, int k,
           float lr, float lam, int opt, uptr accE, uptr accw, uptr accw0, uptr ws,
           size_t ws_bytes, uptr loss, uptr stream) {
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_fm_train_step(P<const int32_t>(idx), P<const float>(y), B, F, P<float>(E),
                                    P<float>(w), P<float>(w0), M, k, lr, lam, opt,
                                    P<float>(accE), P<float>(accw), P<float>(accw0),
                                    P<void>(ws), ws_bytes, P<float>(loss), P<void>(stream));
          }
          check(rc, "hhfm_fm_train_step");
        });

  m.def("hhfm_train_step",
        [](uptr X, uptr Neg, int64_t B, int ncols, int c0, int c1, int t0, int t1, int NG,
           uptr E, int64_t M, int k, float lr, float lam, int opt, uptr accE, uptr ws,
           size_t ws_bytes, uptr loss, uptr stream) {
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_hhfm_train_step(P<const int32_t>(X), P<const int32_t>(Neg), B, ncols, c0,
                                      c1, t0, t1, NG, P<float>(E), M, k, lr, lam, opt,
                                      P<float>(accE), P<void>(ws), ws_bytes, P<float>(loss),
                                      P<void>(stream));
          }
          check(rc, "hhfm_hhfm_train_step");
        });

  m.def("dfm_train_workspace",
        [](int64_t B, int F, int k, int64_t M, std::vector<int32_t> dims) {
          size_t ws = 0;
          check(hhfm_dfm_train_workspace(B, F, k, M, (int)dims.size(), dims.data(), &ws),
                "hhfm_dfm_train_workspace");
          return ws;
        });

  m.def("dfm_train_state_bytes", [](int F, int k, int64_t M, std::vector<int32_t> dims) {
    size_t n = 0;
    check(hhfm_dfm_train_state_bytes(F, k, M, (int)dims.size(), dims.data(), &n),
          "hhfm_dfm_train_state_bytes");
    return n;
  });

  m.def("afm_train_state_bytes", [](int F, int k, int A, int64_t M) {
    size_t n = 0;
    check(hhfm_afm_train_state_bytes(F, k, A, M, &n), "hhfm_afm_train_state_bytes");
    return n;
  });

  m.def("dfm_train_step",
        [](uptr idx, uptr y, int64_t B, int F, uptr E, uptr w, int64_t M, int k,
           std::vector<int32_t> dims, std::vector<uptr> W, std::vector<uptr> bias, uptr Wp,
           uptr bp, float lr, float lam, int opt, std::vector<uptr> acc, uptr ws,
           size_t ws_bytes, uptr loss, uptr stream) {
          if (W.size() != dims.size() || bias.size() != dims.size())
            throw py::value_error("dims, W and bias must have the same length");
          if (opt != 1 && acc.size() != 2 * dims.size() + 4)
            throw py::value_error("acc needs 2 * len(dims) + 4 slot arrays");
          std::vector<float*> Wv(W.size()), bv(bias.size()), av(acc.size());
          for (size_t i = 0; i < W.size(); ++i) {
            Wv[i] = P<float>(W[i]);
            bv[i] = P<float>(bias[i]);
          }
          for (size_t i = 0; i < acc.size(); ++i) av[i] = P<float>(acc[i]);
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_dfm_train_step(P<const int32_t>(idx), P<const float>(y), B, F, P<float>(E),
                                     P<float>(w), M, k, (int)dims.size(), dims.data(), Wv.data(),
                                     bv.data(), P<float>(Wp), P<float>(bp), lr, lam, opt,
                                     av.empty() ? nullptr : av.data(), P<void>(ws), ws_bytes,
                                     P<float>(loss), P<void>(stream));
          }
          check(rc, "hhfm_dfm_train_step");
        });

  m.def("afm_train_workspace", [](int64_t B, int F, int k, int A, int64_t M) {
    size_t ws = 0;
    check(hhfm_afm_train_workspace(B, F, k, A, M, &ws), "hhfm_afm_train_workspace");
    return ws;
  });

  m.def("afm_train_step",
        [](uptr idx, uptr y, int64_t B, int F, uptr E, uptr w, uptr w0, int64_t M, int k, int A,
           uptr W, uptr b, uptr pvec, uptr Pv, float lr, float lam, int opt,
           std::vector<uptr> acc, uptr ws, size_t ws_bytes, uptr loss, uptr stream) {
          if (opt != 1 && acc.size() != 7)
            throw py::value_error("acc needs 7 slot arrays (E, w, w0, W, b, pvec, P)");
          std::vector<float*> av(acc.size());
          for (size_t i = 0; i < acc.size(); ++i) av[i] = P<float>(acc[i]);
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_afm_train_step(P<const int32_t>(idx), P<const float>(y), B, F, P<float>(E),
                                     P<float>(w), P<float>(w0), M, k, A, P<float>(W), P<float>(b),
                                     P<float>(pvec), P<float>(Pv), lr, lam, opt,
                                     av.empty() ? nullptr : av.data(), P<void>(ws), ws_bytes,
                                     P<float>(loss), P<void>(stream));
          }
          check(rc, "hhfm_afm_train_step");
        });

  m.def("topk_dense",
        [](uptr scores, int64_t B, int N, int64_t ld, int K, int base, uptr top_score,
           uptr top_idx, int plan, uptr stream) {
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_topk_dense_ex(P<const float>(scores), B, N, ld, K, base,
                                    P<float>(top_score), P<int32_t>(top_idx), plan,
                                    P<void>(stream));
          }
          check(rc, "hhfm_topk_dense_ex");
        });

  m.def("topk_merge_host",
        [](uptr in_score, uptr in_idx, int R, int64_t B, int K, uptr out_score,
           uptr out_idx) {
          int rc;
          {
            py::gil_scoped_release nogil;
            rc = hhfm_topk_merge_host(P<const float>(in_score),
                                      P<const int32_t>(in_idx), R, B, K,
                                      P<float>(out_score), P<int32_t>(out_idx));
          }
          check(rc, "hhfm_topk_merge_host");
        });
}
