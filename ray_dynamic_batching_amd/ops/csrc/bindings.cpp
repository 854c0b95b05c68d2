// pybind11 bindings of the gfx950 kernels.  Every tensor crosses the boundary
// as a raw device address (uintptr_t) plus explicit shapes/strides, and every
// launch goes on the caller's HIP stream, so the Python wrappers stay thin and
// the launches are capturable into hipGraphs (torch.cuda.graph).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace rdb {
void gemm_tn(int in_dtype, int out_dtype, uintptr_t A, int lda, uintptr_t W, int ldw, uintptr_t C,
             int ldc, uintptr_t bias, uintptr_t R, int ldr, int M, int N, int K, float alpha,
             int act, uintptr_t stream, int force_cfg);
void gemm_tn_sk(int in_dtype, int out_dtype, uintptr_t A, int lda, uintptr_t W, int ldw, uintptr_t C,
                int ldc, uintptr_t bias, uintptr_t R, int ldr, int M, int N, int K, float alpha,
                int act, uintptr_t stream, int force_cfg, uintptr_t ws, size_t ws_bytes);
size_t conv_splitk_bytes(int M, int N, int cfg, int splits);
int conv_halo_tiles(int v, int N, int H, int W, int C, int K);
size_t conv_halo_ws_bytes(int v, int N, int H, int W, int C, int K, int splits, int S);
int conv_halo_tiles_s(int v, int N, int H, int W, int C, int K, int S);
void gemm_tn_ln(uintptr_t A, int lda, uintptr_t W, int ldw, uintptr_t C, int ldc, uintptr_t bias, uintptr_t R,
                int ldr, int M, int N, int K, float alpha, int act, int mode, uintptr_t a_stats, int a_ld,
                uintptr_t a_colsum, uintptr_t a_bias, uintptr_t r_stats, int r_ld, uintptr_t r_g, uintptr_t r_b,
                uintptr_t o_stats, int o_ld, float a_inv_d, float r_inv_d, float eps, uintptr_t stream, int cfg,
                uintptr_t panel, uintptr_t err, int a_parts, int r_parts);
int gemm_stg_cfg(int cfg);
int gemm_tile_bn(int cfg);
void gemm_sk_bf16(uintptr_t A, int lda, uintptr_t W, int ldw, uintptr_t C, int ldc, uintptr_t bias, uintptr_t R,
                  int ldr, int M, int N, int K, float alpha, int act, uintptr_t workspace, int grid, int tile,
                  uintptr_t stream);
size_t gemm_sk_workspace_size(int tile, int grid);
void gemm_rowln(uintptr_t A, int lda, uintptr_t W, uintptr_t bias, uintptr_t R, int ldr, uintptr_t gamma,
                uintptr_t beta, uintptr_t C, int ldc, int M, int N, int K, float eps, uintptr_t stream);
void norm_fwd(int dtype, int mode, uintptr_t x, uintptr_t res, uintptr_t res_out, uintptr_t gamma,
              uintptr_t beta, uintptr_t y, int rows, int D, int ldx, float eps, uintptr_t stream);
void embed_ln_fwd(int dtype, uintptr_t ids, uintptr_t types, uintptr_t word, uintptr_t pos,
                  uintptr_t typ, uintptr_t gamma, uintptr_t beta, uintptr_t y, int tokens, int S,
                  int D, int vocab, float eps, uintptr_t zero_stats, int zn, int zstride, uintptr_t stream);
void attn_fwd(int dtype, uintptr_t qkv, int ld_qkv, int q_off, int k_off, int v_off, int B, int H, int Hkv,
              int S, int D, uintptr_t lens, int causal, uintptr_t out, int ld_out, float scale,
              uintptr_t stream);
void qkv_attn_fwd(int dtype, uintptr_t X, int ldx, uintptr_t Wp, uintptr_t bp, int B, int S, int H, int hidden,
                  uintptr_t lens, uintptr_t out, int ld_out, float scale, int cfg, uintptr_t stream,
                  uintptr_t colsum, uintptr_t bias_f, uintptr_t stats_out, float eps, uintptr_t key_ids, int pad,
                  uintptr_t a_stats, int a_ld, int a_parts);
void softmax_topk(uintptr_t x, int rows, int C, int k, uintptr_t probs, uintptr_t idx, uintptr_t stream);
void rope(uintptr_t qkv, int ld, int q_off, int k_off, int H, int Hkv, int D, int S, uintptr_t cos_t,
          uintptr_t sin_t, int T, int pos_offset, uintptr_t stream);
void gather_rows(uintptr_t src_ptrs, int n, int rows, int row_bytes, uintptr_t dst, uintptr_t stream);
void image_to_nhwc(uintptr_t src, int N, int HW, int Cp, uintptr_t dst, uintptr_t stream);
void image_to_s2d(uintptr_t src, int N, int H, int W, uintptr_t dst, uintptr_t zero, long zero_bytes, uintptr_t stream);
void stem_s2d_pool(uintptr_t img, int N, int H, int W, uintptr_t w, uintptr_t bias, uintptr_t out, uintptr_t zero,
                   long zero_bytes, uintptr_t stream);
void conv2d_nhwc(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t res, uintptr_t y, int N, int H,
                 int W, int C, int K, int R, int S, int stride, int pad, int P, int Q, int act,
                 uintptr_t stream, int force_cfg, uintptr_t ws, size_t ws_bytes);
void maxpool_nhwc(uintptr_t x, uintptr_t y, int N, int H, int W, int C, int k, int stride, int pad,
                  int P, int Q, uintptr_t stream);
void avgpool_nhwc(uintptr_t x, uintptr_t y, int N, int HW, int C, uintptr_t stream);
void dwconv_nhwc(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int N, int H, int W, int C,
                 int R, int stride, int pad, int P, int Q, int act, uintptr_t stream);
void shuffle_remap(uintptr_t A, int ldA, uintptr_t B, int ldB, int Ch, long pixels, uintptr_t O1, int ld1,
                   uintptr_t O2, int ld2, int split, uintptr_t stream);
void se_scale(uintptr_t x, uintptr_t s, uintptr_t y, int N, long HW, int C, uintptr_t stream);
void register_engine(py::module_& m);
void seq_lens(uintptr_t ids, int B, int S, int pad, uintptr_t lens, uintptr_t stream);
size_t xgmi_signal_bytes();
void xgmi_allreduce(int dtype, const std::vector<uintptr_t>& recv, const std::vector<uintptr_t>& gather,
                    const std::vector<uintptr_t>& sig, int rank, uintptr_t in, uintptr_t out_norm,
                    uintptr_t gamma, float eps, int T, int D, long long slot_elems, int two_shot,
                    int grid, unsigned long long timeout_ticks, uintptr_t stream, uintptr_t dbg,
                    int norm_store);
uintptr_t xgmi_alloc_uncached(size_t bytes);
void xgmi_free(uintptr_t p);
std::string xgmi_ipc_handle(uintptr_t p);
uintptr_t xgmi_ipc_open(const std::string& handle);
void xgmi_ipc_close(uintptr_t p);
uint32_t xgmi_read_error(uintptr_t sig);
unsigned long long xgmi_ticks_per_second();
}  // namespace rdb

static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

PYBIND11_MODULE(_rdb_ops, m) {
  m.doc() = "ray_dynamic_batching_amd gfx950 kernels (MFMA GEMM/conv, norm, attention, ...)";
  m.def("gemm_tn", &rdb::gemm_tn, py::call_guard<py::gil_scoped_release>());
  m.def("gemm_tn_sk", &rdb::gemm_tn_sk, py::call_guard<py::gil_scoped_release>());
  m.def("gemm_tn_ln", &rdb::gemm_tn_ln, py::arg("A"), py::arg("lda"), py::arg("W"), py::arg("ldw"), py::arg("C"),
        py::arg("ldc"), py::arg("bias"), py::arg("R"), py::arg("ldr"), py::arg("M"), py::arg("N"), py::arg("K"),
        py::arg("alpha"), py::arg("act"), py::arg("mode"), py::arg("a_stats"), py::arg("a_ld"), py::arg("a_colsum"),
        py::arg("a_bias"), py::arg("r_stats"), py::arg("r_ld"), py::arg("r_g"), py::arg("r_b"), py::arg("o_stats"),
        py::arg("o_ld"), py::arg("a_inv_d"), py::arg("r_inv_d"), py::arg("eps"), py::arg("stream"), py::arg("cfg"),
        py::arg("panel") = 0, py::arg("err") = 0, py::arg("a_parts") = 1, py::arg("r_parts") = 1,
        py::call_guard<py::gil_scoped_release>());
  m.def("gemm_stg_cfg", &rdb::gemm_stg_cfg, "tile the staged-LayerNorm modes run for a requested cfg");
  m.def("gemm_tile_bn", &rdb::gemm_tile_bn, "N extent of tile cfg (partial-statistics count = ceil(N / BN))");
  m.def("gemm_rowln", &rdb::gemm_rowln, py::call_guard<py::gil_scoped_release>());
#ifdef RDB_EXPERIMENTAL_KERNELS
  constexpr bool experimental = true;
#else
  constexpr bool experimental = false;
#endif
  m.def("experimental_kernels_built", [] { return experimental; },
        "whether the opt-in RDB_EXPERIMENTAL_KERNELS variants (stream-K, row-LN, LNOUT / staged LN) are compiled in");
  m.def("gemm_sk_bf16", &rdb::gemm_sk_bf16, py::call_guard<py::gil_scoped_release>());
  m.def("gemm_sk_workspace_size", &rdb::gemm_sk_workspace_size);
  m.def("norm_fwd", &rdb::norm_fwd, py::call_guard<py::gil_scoped_release>());
  m.def("embed_ln_fwd", &rdb::embed_ln_fwd, py::call_guard<py::gil_scoped_release>());
  m.def("attn_fwd", &rdb::attn_fwd, py::call_guard<py::gil_scoped_release>());
  m.def("qkv_attn_fwd", &rdb::qkv_attn_fwd, py::arg("dtype"), py::arg("X"), py::arg("ldx"), py::arg("Wp"),
        py::arg("bp"), py::arg("B"), py::arg("S"), py::arg("H"), py::arg("hidden"), py::arg("lens"), py::arg("out"),
        py::arg("ld_out"), py::arg("scale"), py::arg("cfg"), py::arg("stream"), py::arg("colsum") = 0,
        py::arg("bias_f") = 0, py::arg("stats_out") = 0, py::arg("eps") = 0.0f, py::arg("key_ids") = 0,
        py::arg("pad") = 0, py::arg("a_stats") = 0, py::arg("a_ld") = 0, py::arg("a_parts") = 0, py::call_guard<py::gil_scoped_release>());
  m.def("softmax_topk", &rdb::softmax_topk, py::call_guard<py::gil_scoped_release>());
  m.def("rope", &rdb::rope, py::call_guard<py::gil_scoped_release>());
  m.def("gather_rows", &rdb::gather_rows, py::call_guard<py::gil_scoped_release>());
  m.def("image_to_nhwc", &rdb::image_to_nhwc, py::call_guard<py::gil_scoped_release>());
  m.def("image_to_s2d", &rdb::image_to_s2d, py::call_guard<py::gil_scoped_release>());
  m.def("stem_s2d_pool", &rdb::stem_s2d_pool, py::call_guard<py::gil_scoped_release>());
  m.def("conv2d_nhwc", &rdb::conv2d_nhwc, py::call_guard<py::gil_scoped_release>());
  m.def("conv_splitk_bytes", &rdb::conv_splitk_bytes);
  m.def("conv_halo_tiles", &rdb::conv_halo_tiles);
  m.def("conv_halo_ws_bytes", &rdb::conv_halo_ws_bytes);
  m.def("conv_halo_tiles_s", &rdb::conv_halo_tiles_s);
  m.def("maxpool_nhwc", &rdb::maxpool_nhwc, py::call_guard<py::gil_scoped_release>());
  m.def("avgpool_nhwc", &rdb::avgpool_nhwc, py::call_guard<py::gil_scoped_release>());
  m.def("dwconv_nhwc", &rdb::dwconv_nhwc, py::call_guard<py::gil_scoped_release>());
  m.def("shuffle_remap", &rdb::shuffle_remap, py::call_guard<py::gil_scoped_release>());
  m.def("se_scale", &rdb::se_scale, py::call_guard<py::gil_scoped_release>());
  m.def("seq_lens", &rdb::seq_lens, py::call_guard<py::gil_scoped_release>());

  // Pinning of shared-memory regions so the device can read request payloads
  // in place (zero-copy H2D gather) -- the "pinned shm tensor arena".
  m.def("host_register", [](uintptr_t ptr, size_t bytes) {
    hip_check(hipHostRegister(reinterpret_cast<void*>(ptr), bytes, hipHostRegisterMapped), "hipHostRegister");
    void* dev = nullptr;
    hip_check(hipHostGetDevicePointer(&dev, reinterpret_cast<void*>(ptr), 0), "hipHostGetDevicePointer");
    return reinterpret_cast<uintptr_t>(dev);
  });
  m.def("host_unregister", [](uintptr_t ptr) {
    hip_check(hipHostUnregister(reinterpret_cast<void*>(ptr)), "hipHostUnregister");
  });
  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });

  // Custom all-reduce over xGMI peer memory (xgmi.hip) for TP groups.
  m.def("xgmi_signal_bytes", &rdb::xgmi_signal_bytes);
  m.def("xgmi_allreduce", &rdb::xgmi_allreduce, py::arg("dtype"), py::arg("recv"), py::arg("gather"),
        py::arg("sig"), py::arg("rank"), py::arg("in_ptr"), py::arg("out_norm"), py::arg("gamma"), py::arg("eps"),
        py::arg("T"), py::arg("D"), py::arg("slot_elems"), py::arg("two_shot"), py::arg("grid"),
        py::arg("timeout_ticks"), py::arg("stream"), py::arg("dbg") = 0, py::arg("norm_store") = 0,
        py::call_guard<py::gil_scoped_release>());
  m.def("xgmi_alloc_uncached", &rdb::xgmi_alloc_uncached);
  m.def("xgmi_free", &rdb::xgmi_free);
  m.def("xgmi_ipc_handle", [](uintptr_t p) { return py::bytes(rdb::xgmi_ipc_handle(p)); });
  m.def("xgmi_ipc_open", [](py::bytes h) { return rdb::xgmi_ipc_open(std::string(h)); });
  m.def("xgmi_ipc_close", &rdb::xgmi_ipc_close);
  m.def("xgmi_read_error", &rdb::xgmi_read_error);
  m.def("xgmi_ticks_per_second", &rdb::xgmi_ticks_per_second);
  rdb::register_engine(m);
}
