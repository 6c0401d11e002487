// pybind11 surface of the HIP extension `cgnn_amd._hip`.
// Every device pointer crosses the boundary as an integer (tensor.data_ptr()),
// every stream as the integer handle of torch.cuda.current_stream(); the
// extension never allocates device memory itself, PyTorch's caching allocator
// owns all buffers.
#include <hip/hip_runtime.h>
#include "cgnn_common.h"
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <stdint.h>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

extern "C" {
int cgnn_mmd_supported_d(int);
int cgnn_mmd_mfma_supported(int);
int cgnn_mmd_mfma_row_blocks(int);
int cgnn_launch_mmd_mfma_rows(int, int, const float*, const float*, const float*, const float*, float*, float*,
                              int, int, int, int, float, int, int, hipStream_t, int);
int cgnn_gen_supported_h(int);
int cgnn_gen_bwd_blocks(int);
size_t cgnn_gen_bwd_lds(int, int, int, int);
int cgnn_launch_mmd_rows(int, int, const float*, const float*, float*, float*, int, int, int, int, int,
                         float, int, int, hipStream_t, int);
int cgnn_mmd_mirror_slots(int, int);
int cgnn_launch_loss_finalize(const float*, int, float*, float*, float*, float, int, float*, int,
                              const int*, int, int, hipStream_t);
int cgnn_launch_gen_fwd(const int*, int, const float*, int, const float*, float*, float*, int, float*,
                        const uint32_t*, const int*, int, int, int, int, int, hipStream_t, int);
int cgnn_gen_bwd_variant(int, int, int, int);
int cgnn_gen_staged_supported(int, int, int);
size_t cgnn_gen_fwd_lds(int, int);
int cgnn_staged_plan(int, int, int, int, int, int*);
int cgnn_staged_tiles(int);
int cgnn_launch_gen_noise(const int*, int, const uint32_t*, const int*, int, float*, int, int, int, int, int, int,
                          hipStream_t);
int cgnn_launch_gen_fwd_staged(const int*, int, const int*, int, const float*, int, const float*, float*,
                               const float*, int, float*, int, int, int, int, int, int, int, hipStream_t, int);
int cgnn_launch_gen_bwd_staged(const int*, int, const int*, int, const float*, int, const float*, const float*, int,
                               const float*, int, int, int, int, int, int, int, int, float*, float*, hipStream_t,
                               int);
int cgnn_launch_gen_bwd(const int*, int, const float*, int, const float*, const float*, int,
                        const float*, int, int, int, int, int, int, int, float*, hipStream_t);
int cgnn_launch_adam(float*, float*, float*, const float*, int, const int*, int, int, const int*,
                     int, float, float, float, float, int, hipStream_t);
int cgnn_launch_init(float*, float*, float*, const int*, int, int, const uint32_t*, float, int,
                     hipStream_t);
int cgnn_launch_advance(int*, int, int, hipStream_t);
void* cgnn_engine_create(const int*, const float*, const void* const*, hipStream_t);
void cgnn_engine_destroy(void*);
int cgnn_engine_gen_blocks(void*);
int cgnn_engine_n_parts(void*);
void cgnn_engine_init(void*);
void cgnn_engine_tt(void*);
void cgnn_engine_run(void*, int, int, int, int);
// Fourier (random-feature) MMD
int rff_launch_freqs(float*, const uint32_t*, const int*, int, int, int, int, int, int, hipStream_t);
int rff_launch_fwd_bwd(int, const float*, const float*, const float*, float*, float*, float*, int,
                       int, int, int, int, float, hipStream_t, int, float*, int);
long rff_wide_scratch_floats(int, int, int);
// GNN track
int gnn_launch_spmm(const int*, const int*, const void*, void*, const float*, const float*, int,
                    int, int, int, int, int, int, int, const float*, int, const float*, int, int, hipStream_t);
int gnn_launch_spmm_fan(const int*, const int*, const void*, void*, const float*, int, int, int, int, long, long, int,
                        hipStream_t);
int gnn_launch_spmm_ce(const int*, const int*, const void*, const float*, const float*,
                       const int*, const uint8_t*, float*, void*, const float*, int, int, int, int, int, float,
                       const int*, int, hipStream_t);
int gnn_launch_adam(float*, float*, float*, const float*, int, float, float, float, float, float, int*, unsigned*,
                    int, hipStream_t);
int gnn_launch_cast_bf16(const float*, void*, long, hipStream_t);
int gnn_spmm_ce_blocks(int, int);
int gnn_launch_ell_build(const int*, const int*, int*, int, hipStream_t);
int gnn_launch_spmm_ell(const int*, const int*, const void*, void*, const float*, int, int, int, int, long,
                        const int*, int, hipStream_t);
int gnn_slab_sum(const float*, long, int, float*, int, float*, const int*, int*, hipStream_t);
int gnn_launch_sample_neighbors(const int*, const int*, const int*, int, int, const int*, int*, uint32_t, uint32_t,
                                uint32_t, hipStream_t);
int gnn_launch_bias_relu_dropout(void*, const float*, long, int, int, float, uint32_t, uint32_t,
                                 uint32_t, uint32_t, hipStream_t);
int gnn_launch_relu_dropout_bwd(void*, const void*, long, float, hipStream_t);
int gnn_launch_dense_fwd(const void*, const float*, const float*, const float*, const float*, void*, void*,
                         int, int, int, int, int, int, float, uint32_t, uint32_t, uint32_t, uint32_t,
                         const int*, void*, hipStream_t);
long gnn_keep_image_halfwords(int, int);
int gnn_launch_keep_image(void*, int, int, float, uint32_t, uint32_t, uint32_t, uint32_t, const int*, hipStream_t);
int gnn_launch_gat_fwd(const int*, const int*, const void*, const float*, const float*, const int*, float*, float*,
                       void*, int, int, int, int, const float*, void*, int, float, uint32_t, uint32_t, uint32_t,
                       const int*, uint32_t, hipStream_t);
int gnn_gat_row_blocks();
int gnn_launch_gat_rows(int, const void*, int, const float*, const void*, const float*, const float*, const int*,
                        float*, float*, void*, int, void*, const float*, float*, float*, float, uint32_t, uint32_t,
                        uint32_t, const int*, uint32_t, int, int, int, int, hipStream_t);
int gnn_launch_gat_col(const int*, const int*, const void*, const float*, const float*, const void*, float*, float*,
                       void*, int, int, int, int, int, hipStream_t);
int gnn_gat_row_ce_waves();
int gnn_launch_gat_row_ce(const float*, int, const float*, int, const int*, const uint8_t*, float, float*, void*,
                          float*, float*, float*, float*, long, hipStream_t);
int gnn_launch_gat_pack_grad(const float*, const float*, const float*, int, int, void*, int, long, hipStream_t);
int gnn_launch_halo_rows(const void*, long, const long*, void*, long, const long*, long, int, int, hipStream_t);
long gnn_sample_blocks_scratch(int, int, const int*, const int*);
long gnn_sample_flag_bytes(int);
int gnn_launch_sample_blocks(const int*, const int*, int, const int*, int, int, const int*, const int*, int* const*,
                             float* const*, int* const*, int* const*, int* const*, int* const*, int* const*,
                             int* const*, int*, uint8_t*, int*, int*, uint32_t, uint32_t, uint32_t, hipStream_t,
                             int*);
void* gnn_sw_create(int, hipStream_t, const int*, const int*, int, int, const int*, const int*, uint8_t*, int*, int*,
                    uint32_t, uint32_t);
int gnn_sw_add_slot(void*, int* const*, float* const*, int* const*, int* const*, int* const*, int* const*,
                    int* const*, int* const*, int*, int*);
long gnn_sw_submit(void*, int, const int*, int, uint32_t, const hipEvent_t*, int);
int gnn_sw_wait(void*, long, int, hipStream_t);
void gnn_sw_destroy(void*);
int gnn_fused_bwd_blocks(int);
int gnn_fused_bwd_width(int);
int gnn_fused_bwd_supported(int, int, int);
int gnn_launch_fused_bwd(const void*, const void*, const float*, const float*, const float*, const void*, float*,
                         int, int, int, int, int, int, float, hipStream_t);
int gnn_launch_dense_bwd(const void*, const float*, const void*, void*, int, int, int, int, float,
                         hipStream_t);
int gnn_launch_lin_fwd(const void*, int, int, const void*, int, int, const float*, int, const float*, void*, int,
                       int, int, float, uint32_t, uint32_t, uint32_t, uint32_t, const int*, const float*,
                       const int*, void*, float*, int, int, hipStream_t, int);
int gnn_launch_lin_bwd_data(const void*, int, const void*, int, float, int, const float*, int, int, void*, int,
                            void*, int, const float*, int, int, void*, hipStream_t);
long gnn_lin_fwd_image_bytes(int, int, int);
int gnn_lin_fwd_kc_wanted(int, int, int);
long gnn_lin_bwd_image_bytes(int, int);
int gnn_lin_wgrad_chunks(int, int, int);
int gnn_launch_lin_bwd_weight(const void*, int, int, const void*, int, int, const void*, int, const void*, int,
                              float, int, float*, float*, float*, int, const int*, hipStream_t);
}

static inline hipStream_t S(uint64_t s) { return reinterpret_cast<hipStream_t>(s); }
template <class T> static inline T* Pt(uint64_t p) { return reinterpret_cast<T*>(p); }

static void chk(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string(what) + ": HIP launch failed (code " + std::to_string(rc) + ")");
}

class PyEngine {
 public:
  PyEngine(std::vector<int> icfg, std::vector<float> fcfg, std::vector<uint64_t> ptrs, uint64_t stream) {
    if (icfg.size() < 21 || fcfg.size() < 5 || ptrs.size() < 23) throw std::invalid_argument("engine config size");
    std::vector<const void*> p(ptrs.size());
    for (size_t k = 0; k < ptrs.size(); ++k) p[k] = reinterpret_cast<const void*>(ptrs[k]);
    h_ = cgnn_engine_create(icfg.data(), fcfg.data(), p.data(), S(stream));
  }
  ~PyEngine() { if (h_) cgnn_engine_destroy(h_); }
  int gen_blocks() { return cgnn_engine_gen_blocks(h_); }
  int n_parts() { return cgnn_engine_n_parts(h_); }
  void init() { cgnn_engine_init(h_); }
  void tt() { cgnn_engine_tt(h_); }
  void run(int kind, int steps, int chunk, bool hist) { cgnn_engine_run(h_, kind, steps, chunk, hist ? 1 : 0); }
 private:
  void* h_ = nullptr;
};

PYBIND11_MODULE(_hip, m) {
  m.doc() = "cgnn_amd HIP kernels for MI355X (gfx950)";
  m.def("arch", []() { return std::string("gfx950"); });
  m.def("device_count", []() { int n = 0; if (hipGetDeviceCount(&n) != hipSuccess) return 0; return n; });
  m.def("mmd_supported_d", &cgnn_mmd_supported_d);
  m.def("mmd_mfma_supported", &cgnn_mmd_mfma_supported);
  m.def("mmd_mfma_row_blocks", &cgnn_mmd_mfma_row_blocks);
  m.def("mmd_mfma", [](int mode, int D, uint64_t xhat, uint64_t data, uint64_t xn, uint64_t yn, uint64_t gp,
                       uint64_t lp, int N, int R, int n_chunks, int tpc, float gscale, uint64_t st,
                       int row_begin, int n_rows, int wide) {
    chk(cgnn_launch_mmd_mfma_rows(mode, D, Pt<const float>(xhat), Pt<const float>(data), Pt<const float>(xn),
                                  Pt<const float>(yn), Pt<float>(gp), Pt<float>(lp), N, R, n_chunks, tpc, gscale,
                                  row_begin, n_rows < 0 ? N : n_rows, S(st), wide), "mmd_mfma");
  }, py::arg("mode"), py::arg("D"), py::arg("xhat"), py::arg("data"), py::arg("xn"), py::arg("yn"), py::arg("gp"),
     py::arg("lp"), py::arg("N"), py::arg("R"), py::arg("n_chunks"), py::arg("tpc"), py::arg("gscale"),
     py::arg("st"), py::arg("row_begin") = 0, py::arg("n_rows") = -1, py::arg("wide") = -1);
  m.def("gen_supported_h", &cgnn_gen_supported_h);
  m.def("gen_bwd_blocks", &cgnn_gen_bwd_blocks);
  m.def("gen_bwd_lds", &cgnn_gen_bwd_lds);
  m.def("gen_bwd_variant", &cgnn_gen_bwd_variant);
  m.def("gen_staged_supported", &cgnn_gen_staged_supported);
  m.def("gen_fwd_lds", &cgnn_gen_fwd_lds);
  // level-scheduled (wide-graph) generator kernels, cgnn_staged.hip
  m.def("staged_plan", [](int Dt, int H, int max_in, int W, int extra) -> py::tuple {
    int out[5];
    if (cgnn_staged_plan(Dt, H, max_in, W, extra, out) != 0) return py::tuple();
    return py::make_tuple(out[0], out[1], out[2], out[3], out[4]);
  }, py::arg("Dt"), py::arg("H"), py::arg("max_in"), py::arg("W"), py::arg("extra") = 0);
  m.def("staged_tiles", &cgnn_staged_tiles);
  m.def("gen_noise", [](uint64_t prog, int ps, uint64_t keys, uint64_t step, int off, uint64_t noise, int NS, int N,
                        int D, int Dt, int R, int row0, uint64_t st) {
    chk(cgnn_launch_gen_noise(Pt<const int>(prog), ps, Pt<const uint32_t>(keys), Pt<const int>(step), off,
                              Pt<float>(noise), NS, N, D, Dt, R, row0, S(st)), "gen_noise");
  }, py::arg("prog"), py::arg("ps"), py::arg("keys"), py::arg("step"), py::arg("off"), py::arg("noise"),
     py::arg("NS"), py::arg("N"), py::arg("D"), py::arg("Dt"), py::arg("R"), py::arg("row0"), py::arg("st"));
  m.def("gen_fwd_staged", [](uint64_t prog, int ps, uint64_t sched, int ss, uint64_t params, int P, uint64_t data,
                             uint64_t xhat, uint64_t noise, int NS, uint64_t xnorm, int N, int D, int Dt, int H,
                             int max_in, int R, int W, uint64_t st, int force) {
    chk(cgnn_launch_gen_fwd_staged(Pt<const int>(prog), ps, Pt<const int>(sched), ss, Pt<const float>(params), P,
                                   Pt<const float>(data), Pt<float>(xhat), Pt<const float>(noise), NS,
                                   Pt<float>(xnorm), N, D, Dt, H, max_in, R, W, S(st), force), "gen_fwd_staged");
  }, py::arg("prog"), py::arg("ps"), py::arg("sched"), py::arg("ss"), py::arg("params"), py::arg("P"),
     py::arg("data"), py::arg("xhat"), py::arg("noise"), py::arg("NS"), py::arg("xnorm"), py::arg("N"), py::arg("D"),
     py::arg("Dt"), py::arg("H"), py::arg("max_in"), py::arg("R"), py::arg("W"), py::arg("st"),
     py::arg("force") = -1);
  m.def("gen_bwd_staged", [](uint64_t prog, int ps, uint64_t sched, int ss, uint64_t params, int P, uint64_t xhat,
                             uint64_t noise, int NS, uint64_t gradp, int nch, int R, int N, int D, int Dt, int H,
                             int max_in, int W, uint64_t gpart, uint64_t dxs, uint64_t st, int force) {
    chk(cgnn_launch_gen_bwd_staged(Pt<const int>(prog), ps, Pt<const int>(sched), ss, Pt<const float>(params), P,
                                   Pt<const float>(xhat), Pt<const float>(noise), NS, Pt<const float>(gradp), nch,
                                   R, N, D, Dt, H, max_in, W, Pt<float>(gpart), Pt<float>(dxs), S(st), force),
        "gen_bwd_staged");
  }, py::arg("prog"), py::arg("ps"), py::arg("sched"), py::arg("ss"), py::arg("params"), py::arg("P"),
     py::arg("xhat"), py::arg("noise"), py::arg("NS"), py::arg("gradp"), py::arg("nch"), py::arg("R"), py::arg("N"),
     py::arg("D"), py::arg("Dt"), py::arg("H"), py::arg("max_in"), py::arg("W"), py::arg("gpart"), py::arg("dxs"),
     py::arg("st"), py::arg("force") = -1);

  m.def("mmd", [](int mode, int D, uint64_t xhat, uint64_t data, uint64_t gp, uint64_t lp, int N, int R,
                  int row_tiles, int n_chunks, int tpc, float gscale, uint64_t st, int row_begin, int n_rows,
                  int mirror) {
    chk(cgnn_launch_mmd_rows(mode, D, Pt<const float>(xhat), Pt<const float>(data), Pt<float>(gp),
                             Pt<float>(lp), N, R, row_tiles, n_chunks, tpc, gscale, row_begin,
                             n_rows < 0 ? N : n_rows, S(st), mirror), "mmd");
  }, py::arg("mode"), py::arg("D"), py::arg("xhat"), py::arg("data"), py::arg("gp"), py::arg("lp"), py::arg("N"),
     py::arg("R"), py::arg("row_tiles"), py::arg("n_chunks"), py::arg("tpc"), py::arg("gscale"), py::arg("st"),
     py::arg("row_begin") = 0, py::arg("n_rows") = -1, py::arg("mirror") = 0);
  // gradient slots a symmetric (mirror=1) training launch adds after its n_chunks
  m.def("mmd_mirror_slots", &cgnn_mmd_mirror_slots, py::arg("D"), py::arg("N"));
  m.def("loss_finalize", [](uint64_t lp, int n_parts, uint64_t tt, uint64_t last, uint64_t acc, float inv_n2,
                            int flags, uint64_t hist, int hist_stride, uint64_t step, int step_off, int R,
                            uint64_t st) {
    chk(cgnn_launch_loss_finalize(Pt<const float>(lp), n_parts, Pt<float>(tt), Pt<float>(last), Pt<float>(acc),
                                  inv_n2, flags, Pt<float>(hist), hist_stride, Pt<const int>(step), step_off,
                                  R, S(st)), "loss_finalize");
  });
  m.def("gen_fwd", [](uint64_t prog, int ps, uint64_t params, int P, uint64_t data, uint64_t xhat, uint64_t noise,
                      int NS, uint64_t xnorm, uint64_t keys, uint64_t step, int off, int N, int D, int H, int R,
                      uint64_t st, int row0) {
    chk(cgnn_launch_gen_fwd(Pt<const int>(prog), ps, Pt<const float>(params), P, Pt<const float>(data),
                            Pt<float>(xhat), Pt<float>(noise), NS, Pt<float>(xnorm), Pt<const uint32_t>(keys),
                            Pt<const int>(step),
                            off, N, D, H, R, S(st), row0), "gen_fwd");
  }, py::arg("prog"), py::arg("ps"), py::arg("params"), py::arg("P"), py::arg("data"), py::arg("xhat"),
     py::arg("noise"), py::arg("NS"), py::arg("xnorm"), py::arg("keys"), py::arg("step"), py::arg("off"),
     py::arg("N"), py::arg("D"), py::arg("H"), py::arg("R"), py::arg("st"), py::arg("row0") = 0);
  m.def("gen_bwd", [](uint64_t prog, int ps, uint64_t params, int P, uint64_t xhat, uint64_t noise, int NS,
                      uint64_t gradp, int nch, int R, int N, int D, int Dt, int H, int max_in, uint64_t gpart,
                      uint64_t st) {
    chk(cgnn_launch_gen_bwd(Pt<const int>(prog), ps, Pt<const float>(params), P, Pt<const float>(xhat),
                            Pt<const float>(noise), NS, Pt<const float>(gradp), nch, R, N, D, Dt, H, max_in,
                            Pt<float>(gpart), S(st)), "gen_bwd");
  }, py::arg("prog"), py::arg("ps"), py::arg("params"), py::arg("P"), py::arg("xhat"), py::arg("noise"),
     py::arg("NS"), py::arg("gradp"), py::arg("nch"), py::arg("R"), py::arg("N"), py::arg("D"), py::arg("Dt"),
     py::arg("H"), py::arg("max_in"), py::arg("gpart"), py::arg("st"));
  m.def("adam", [](uint64_t params, uint64_t mm, uint64_t vv, uint64_t gpart, int G, uint64_t prog, int ps, int P,
                   uint64_t step, int off, float lr, float b1, float b2, float eps, int R, uint64_t st) {
    chk(cgnn_launch_adam(Pt<float>(params), Pt<float>(mm), Pt<float>(vv), Pt<const float>(gpart), G,
                         Pt<const int>(prog), ps, P, Pt<const int>(step), off, lr, b1, b2, eps, R, S(st)),
        "adam");
  });
  m.def("init_params", [](uint64_t params, uint64_t mm, uint64_t vv, uint64_t prog, int ps, int P, uint64_t keys,
                          float std, int R, uint64_t st) {
    chk(cgnn_launch_init(Pt<float>(params), Pt<float>(mm), Pt<float>(vv), Pt<const int>(prog), ps, P,
                         Pt<const uint32_t>(keys), std, R, S(st)), "init_params");
  });
  m.def("advance", [](uint64_t step, int dr, int dopt, uint64_t st) {
    chk(cgnn_launch_advance(Pt<int>(step), dr, dopt, S(st)), "advance");
  });

  m.def("rff_freqs", [](uint64_t w, uint64_t keys, uint64_t step, int off, int k, int d, int n_gamma, int d_true,
                        int R, uint64_t st) {
    chk(rff_launch_freqs(Pt<float>(w), Pt<const uint32_t>(keys), Pt<const int>(step), off, k, d, n_gamma, d_true,
                         R, S(st)),
        "rff_freqs");
  });
  m.def("rff_fwd_bwd", [](int mode, uint64_t xhat, uint64_t data, uint64_t w, uint64_t feat, uint64_t loss,
                          uint64_t grad, int N, int D, int F, int R, int k, float norm, uint64_t st,
                          int force_valu, uint64_t scratch, int force_wide) {
    chk(rff_launch_fwd_bwd(mode, Pt<const float>(xhat), Pt<const float>(data), Pt<const float>(w),
                           Pt<float>(feat), Pt<float>(loss), Pt<float>(grad), N, D, F, R, k, norm, S(st),
                           force_valu, Pt<float>(scratch), force_wide),
        "rff_fwd_bwd");
  }, py::arg("mode"), py::arg("xhat"), py::arg("data"), py::arg("w"), py::arg("feat"), py::arg("loss"),
     py::arg("grad"), py::arg("N"), py::arg("D"), py::arg("F"), py::arg("R"), py::arg("k"), py::arg("norm"),
     py::arg("st"), py::arg("force_valu") = 0, py::arg("scratch") = 0, py::arg("force_wide") = 0);
  m.def("rff_wide_scratch_floats", &rff_wide_scratch_floats);

  m.def("gnn_spmm", [](uint64_t rowptr, uint64_t col, uint64_t x, uint64_t y, uint64_t rscale, uint64_t bias,
                       int n_rows, int F, int ld_x, int ld_y, int x_bf16, int y_bf16, int relu, int unit_col,
                       uint64_t st, uint64_t init, int ldi, uint64_t cscale, int init_rows, int short_rows) {
    chk(gnn_launch_spmm(Pt<const int>(rowptr), Pt<const int>(col), Pt<const void>(x), Pt<void>(y),
                        Pt<const float>(rscale), Pt<const float>(bias), n_rows, F, ld_x, ld_y, x_bf16,
                        y_bf16, relu, unit_col, Pt<const float>(init), ldi, Pt<const float>(cscale), init_rows,
                        short_rows, S(st)),
        "gnn_spmm");
  }, py::arg("rowptr"), py::arg("col"), py::arg("x"), py::arg("y"), py::arg("rscale"), py::arg("bias"),
     py::arg("n_rows"), py::arg("F"), py::arg("ld_x"), py::arg("ld_y"), py::arg("x_bf16"), py::arg("y_bf16"),
     py::arg("relu"), py::arg("unit_col"), py::arg("st"), py::arg("init") = 0, py::arg("ldi") = 0,
     py::arg("cscale") = 0, py::arg("init_rows") = -1, py::arg("short_rows") = 0);
  m.def("gnn_spmm_fan", [](uint64_t rowptr, uint64_t col, uint64_t x, uint64_t y, uint64_t rscale, int n_rows, int F,
                           int ldx, int ldy, long n_x_rows, long nnz, int max_deg, uint64_t st) {
    chk(gnn_launch_spmm_fan(Pt<const int>(rowptr), Pt<const int>(col), Pt<const void>(x), Pt<void>(y),
                            Pt<const float>(rscale), n_rows, F, ldx, ldy, n_x_rows, nnz, max_deg, S(st)),
        "gnn_spmm_fan");
  });
  m.def("gnn_spmm_ce", [](uint64_t rowptr, uint64_t col, uint64_t z, uint64_t rscale, uint64_t bias,
                          uint64_t labels, uint64_t mask, uint64_t stats, uint64_t dlogits, uint64_t init, int ldi,
                          int n_rows, int C, int ld, int mode, float inv_count, uint64_t st, uint64_t gslot,
                          int n_long) {
    chk(gnn_launch_spmm_ce(Pt<const int>(rowptr), Pt<const int>(col), Pt<const void>(z), Pt<const float>(rscale),
                           Pt<const float>(bias), Pt<const int>(labels), Pt<const uint8_t>(mask),
                           Pt<float>(stats), Pt<void>(dlogits), Pt<const float>(init), ldi, n_rows, C, ld, mode,
                           inv_count, Pt<const int>(gslot), n_long, S(st)), "gnn_spmm_ce");
  }, py::arg("rowptr"), py::arg("col"), py::arg("z"), py::arg("rscale"), py::arg("bias"), py::arg("labels"),
     py::arg("mask"), py::arg("stats"), py::arg("dlogits"), py::arg("init"), py::arg("ldi"), py::arg("n_rows"),
     py::arg("C"), py::arg("ld"), py::arg("mode"), py::arg("inv_count"), py::arg("st"), py::arg("gslot") = 0,
     py::arg("n_long") = 0);
  m.def("gnn_adam", [](uint64_t p, uint64_t mm, uint64_t vv, uint64_t g, int n, float lr, float b1, float b2,
                       float eps, float wd, uint64_t step, uint64_t st, uint64_t done, int step_done) {
    chk(gnn_launch_adam(Pt<float>(p), Pt<float>(mm), Pt<float>(vv), Pt<const float>(g), n, lr, b1, b2, eps, wd,
                        Pt<int>(step), Pt<unsigned>(done), step_done, S(st)), "gnn_adam");
  }, py::arg("p"), py::arg("m"), py::arg("v"), py::arg("g"), py::arg("n"), py::arg("lr"), py::arg("b1"),
     py::arg("b2"), py::arg("eps"), py::arg("wd"), py::arg("step"), py::arg("st"), py::arg("done") = 0,
     py::arg("step_done") = 0);
  m.def("gnn_spmm_ce_blocks", &gnn_spmm_ce_blocks);
  m.def("gnn_ell_build", [](uint64_t rowptr, uint64_t col, uint64_t ell, int n_rows, uint64_t st) {
    chk(gnn_launch_ell_build(Pt<const int>(rowptr), Pt<const int>(col), Pt<int>(ell), n_rows, S(st)), "gnn_ell_build");
  });
  m.def("gnn_spmm_ell", [](uint64_t ell, uint64_t col, uint64_t x, uint64_t y, uint64_t rscale, int n_rows, int F,
                           int ldx, int ldy, long n_x_rows, uint64_t long_rows, int n_long, uint64_t st) {
    chk(gnn_launch_spmm_ell(Pt<const int>(ell), Pt<const int>(col), Pt<const void>(x), Pt<void>(y),
                            Pt<const float>(rscale), n_rows, F, ldx, ldy, n_x_rows, Pt<const int>(long_rows),
                            n_long, S(st)), "gnn_spmm_ell");
  });
  m.def("gnn_slab_sum", [](uint64_t P, long rows, int W, uint64_t stage, int G, uint64_t out, uint64_t map,
                           uint64_t st, uint64_t bump) {
    chk(gnn_slab_sum(Pt<const float>(P), rows, W, Pt<float>(stage), G, Pt<float>(out), Pt<const int>(map),
                     Pt<int>(bump), S(st)),
        "gnn_slab_sum");
  }, py::arg("P"), py::arg("rows"), py::arg("W"), py::arg("stage"), py::arg("G"), py::arg("out"), py::arg("map"),
     py::arg("st"), py::arg("bump") = 0);
  m.def("gnn_sample_neighbors", [](uint64_t rowptr, uint64_t col, uint64_t nodes, int n, int fanout, uint64_t out_ptr,
                                   uint64_t out_col, uint32_t k0, uint32_t k1, uint32_t salt, uint64_t st) {
    chk(gnn_launch_sample_neighbors(Pt<const int>(rowptr), Pt<const int>(col), Pt<const int>(nodes), n, fanout,
                                    Pt<const int>(out_ptr), Pt<int>(out_col), k0, k1, salt, S(st)),
        "gnn_sample_neighbors");
  });
  m.def("gnn_bias_relu_dropout", [](uint64_t h, uint64_t bias, long rows, int F, int ld, float p, uint32_t k0,
                                    uint32_t k1, uint32_t step, uint32_t row0, uint64_t st) {
    chk(gnn_launch_bias_relu_dropout(Pt<void>(h), Pt<const float>(bias), rows, F, ld, p, k0, k1, step, row0, S(st)),
        "gnn_bias_relu_dropout");
  });
  m.def("gnn_relu_dropout_bwd", [](uint64_t dh, uint64_t h, long n, float p, uint64_t st) {
    chk(gnn_launch_relu_dropout_bwd(Pt<void>(dh), Pt<const void>(h), n, p, S(st)), "gnn_relu_dropout_bwd");
  });
  m.def("gnn_dense_fwd", [](uint64_t ax, uint64_t w1, uint64_t b1, uint64_t w2, uint64_t dinv, uint64_t h1,
                            uint64_t z2, int n, int F, int ldx, int HD, int C, int ldc, float p, uint32_t k0,
                            uint32_t k1, uint32_t step, uint32_t row0, uint64_t st, uint64_t stepp, uint64_t kimg) {
    return gnn_launch_dense_fwd(Pt<const void>(ax), Pt<const float>(w1), Pt<const float>(b1), Pt<const float>(w2),
                                Pt<const float>(dinv), Pt<void>(h1), Pt<void>(z2), n, F, ldx, HD, C, ldc, p, k0,
                                k1, step, row0, Pt<const int>(stepp), Pt<void>(kimg), S(st));
  }, py::arg("ax"), py::arg("w1"), py::arg("b1"), py::arg("w2"), py::arg("dinv"), py::arg("h1"), py::arg("z2"),
     py::arg("n"), py::arg("F"), py::arg("ldx"), py::arg("HD"), py::arg("C"), py::arg("ldc"), py::arg("p"),
     py::arg("k0"), py::arg("k1"), py::arg("step"), py::arg("row0"), py::arg("st"), py::arg("step_ptr") = 0,
     py::arg("kimg") = 0);
  m.def("gnn_keep_image_halfwords", &gnn_keep_image_halfwords);
  m.def("gnn_keep_image", [](uint64_t kimg, int n, int HD, float p, uint32_t k0, uint32_t k1, uint32_t step,
                             uint32_t row0, uint64_t st, uint64_t stepp) {
    return gnn_launch_keep_image(Pt<void>(kimg), n, HD, p, k0, k1, step, row0, Pt<const int>(stepp), S(st));
  }, py::arg("kimg"), py::arg("n"), py::arg("HD"), py::arg("p"), py::arg("k0"), py::arg("k1"), py::arg("step"),
     py::arg("row0"), py::arg("st"), py::arg("step_ptr") = 0);
  m.def("gnn_dense_bwd", [](uint64_t dy2, uint64_t w2, uint64_t h1, uint64_t dp1, int n, int HD, int C, int ldc,
                            float p, uint64_t st) {
    return gnn_launch_dense_bwd(Pt<const void>(dy2), Pt<const float>(w2), Pt<const void>(h1), Pt<void>(dp1), n,
                                HD, C, ldc, p, S(st));
  });
  m.def("gnn_gat_fwd", [](uint64_t rp, uint64_t col, uint64_t wh, uint64_t ss, uint64_t sd, uint64_t out,
                          uint64_t lse, int n, int K, int Fh, uint64_t st, int wbf, uint64_t dst_rows, uint64_t q,
                          uint64_t bias, uint64_t H, int ldh, float p, uint32_t k0, uint32_t k1, uint32_t step,
                          uint64_t stepp, uint32_t row0) {
    chk(gnn_launch_gat_fwd(Pt<const int>(rp), Pt<const int>(col), Pt<const void>(wh), Pt<const float>(ss),
                           Pt<const float>(sd), Pt<const int>(dst_rows), Pt<float>(out), Pt<float>(lse), Pt<void>(q),
                           n, K, Fh, wbf, Pt<const float>(bias), Pt<void>(H), ldh, p, k0, k1, step,
                           Pt<const int>(stepp), row0, S(st)),
        "gnn_gat_fwd");
  }, py::arg("rp"), py::arg("col"), py::arg("wh"), py::arg("ss"), py::arg("sd"), py::arg("out"), py::arg("lse"),
     py::arg("n"), py::arg("K"), py::arg("Fh"), py::arg("st"), py::arg("wbf") = 0, py::arg("dst_rows") = 0,
     py::arg("q") = 0, py::arg("bias") = 0, py::arg("H") = 0, py::arg("ldh") = 0, py::arg("p") = 0.f,
     py::arg("k0") = 0, py::arg("k1") = 0, py::arg("step") = 0, py::arg("stepp") = 0, py::arg("row0") = 0);
  m.def("gnn_gat_row_blocks", &gnn_gat_row_blocks);
  m.def("gnn_gat_rows", [](int act, uint64_t dout, int ldh, uint64_t out, uint64_t q, uint64_t lse, uint64_t sd,
                           uint64_t dst_rows, uint64_t rstat, uint64_t dsd, uint64_t dy, int ldy, uint64_t dout_w,
                           uint64_t bias, uint64_t bpart, uint64_t db, float p, uint32_t k0, uint32_t k1,
                           uint32_t step, uint64_t stepp, uint32_t row0, int n, int K, int Fh, int wbf, uint64_t st) {
    chk(gnn_launch_gat_rows(act, Pt<const void>(dout), ldh, Pt<const float>(out), Pt<const void>(q),
                            Pt<const float>(lse), Pt<const float>(sd), Pt<const int>(dst_rows), Pt<float>(rstat),
                            Pt<float>(dsd), Pt<void>(dy), ldy, Pt<void>(dout_w), Pt<const float>(bias),
                            Pt<float>(bpart), Pt<float>(db), p, k0, k1, step, Pt<const int>(stepp), row0, n, K, Fh,
                            wbf, S(st)), "gnn_gat_rows");
  }, py::arg("act"), py::arg("dout"), py::arg("ldh"), py::arg("out"), py::arg("q"), py::arg("lse"), py::arg("sd"),
     py::arg("dst_rows"), py::arg("rstat"), py::arg("dsd"), py::arg("dy"), py::arg("ldy"), py::arg("dout_w"),
     py::arg("bias"), py::arg("bpart"), py::arg("db"), py::arg("p"), py::arg("k0"), py::arg("k1"), py::arg("step"),
     py::arg("stepp"), py::arg("row0"), py::arg("n"), py::arg("K"), py::arg("Fh"), py::arg("wbf"), py::arg("st"));
  m.def("gnn_gat_col", [](uint64_t rpt, uint64_t colt, uint64_t wh, uint64_t ss, uint64_t rstat, uint64_t dout,
                          uint64_t dwh, uint64_t dss, uint64_t dy, int ldy, int n, int K, int Fh, uint64_t st,
                          int wbf) {
    chk(gnn_launch_gat_col(Pt<const int>(rpt), Pt<const int>(colt), Pt<const void>(wh), Pt<const float>(ss),
                           Pt<const float>(rstat), Pt<const void>(dout), Pt<float>(dwh), Pt<float>(dss), Pt<void>(dy),
                           ldy, n, K, Fh, wbf, S(st)), "gnn_gat_col");
  }, py::arg("rpt"), py::arg("colt"), py::arg("wh"), py::arg("ss"), py::arg("rstat"), py::arg("dout"),
     py::arg("dwh"), py::arg("dss"), py::arg("dy"), py::arg("ldy"), py::arg("n"), py::arg("K"), py::arg("Fh"),
     py::arg("st"), py::arg("wbf") = 1);
  // dense-side kernels of the fused GAT epoch (gnn_gat.hip)
  m.def("gnn_gat_row_ce_waves", &gnn_gat_row_ce_waves);
  m.def("gnn_gat_row_ce", [](uint64_t z, int ldz, uint64_t b, int C, uint64_t y, uint64_t mask, float inv_count,
                             uint64_t dz, uint64_t dzb, uint64_t spart, uint64_t bpart, uint64_t stats, uint64_t db,
                             long n, uint64_t st) {
    chk(gnn_launch_gat_row_ce(Pt<const float>(z), ldz, Pt<const float>(b), C, Pt<const int>(y),
                              Pt<const uint8_t>(mask), inv_count, Pt<float>(dz), Pt<void>(dzb), Pt<float>(spart),
                              Pt<float>(bpart), Pt<float>(stats), Pt<float>(db), n, S(st)), "gnn_gat_row_ce");
  });
  m.def("gnn_gat_pack_grad", [](uint64_t dwh, uint64_t dss, uint64_t dsd, int HF, int K, uint64_t dy, int ldy,
                                long n, uint64_t st) {
    chk(gnn_launch_gat_pack_grad(Pt<const float>(dwh), Pt<const float>(dss), Pt<const float>(dsd), HF, K,
                                 Pt<void>(dy), ldy, n, S(st)), "gnn_gat_pack_grad");
  });
  m.def("gnn_halo_rows", [](uint64_t src, long sp, uint64_t sidx, uint64_t dst, long dp, uint64_t didx, long rows,
                            int words, int mode, uint64_t st) {
    chk(gnn_launch_halo_rows(Pt<const void>(src), sp, Pt<const long>(sidx), Pt<void>(dst), dp, Pt<const long>(didx),
                             rows, words, mode, S(st)), "gnn_halo_rows");
  });
  m.def("gnn_sample_flag_bytes", &gnn_sample_flag_bytes);
  m.def("gnn_sample_blocks_scratch", [](int n, std::vector<int> fan, std::vector<int> nd_max) {
    if (fan.size() != nd_max.size()) throw std::runtime_error("gnn_sample_blocks_scratch: list lengths differ");
    return gnn_sample_blocks_scratch(n, (int)fan.size(), fan.data(), nd_max.data());
  });
  // whole mini-batch sampling pipeline (gnn_sampler.hip): per-level pointer lists
  m.def("gnn_sample_blocks", [](uint64_t rowptr, uint64_t col, int n, uint64_t seeds, int n_seeds,
                                std::vector<int> fan, std::vector<int> nd_max, std::vector<uint64_t> optr,
                                std::vector<uint64_t> inv_deg, std::vector<uint64_t> picks, std::vector<uint64_t> local,
                                std::vector<uint64_t> src, std::vector<uint64_t> rp_t, std::vector<uint64_t> col_t,
                                std::vector<uint64_t> cnt_t, uint64_t counts, uint64_t flag, uint64_t map,
                                uint64_t bscratch, uint32_t k0, uint32_t k1, uint32_t salt, uint64_t st,
                                uint64_t counts_host) {
    const size_t L = fan.size();
    if (nd_max.size() != L || optr.size() != L || inv_deg.size() != L || picks.size() != L || local.size() != L ||
        src.size() != L || rp_t.size() != L || col_t.size() != L || cnt_t.size() != L)
      throw std::runtime_error("gnn_sample_blocks: per-level lists differ in length");
    auto ip = [](const std::vector<uint64_t>& v) {
      std::vector<int*> o(v.size());
      for (size_t i = 0; i < v.size(); ++i) o[i] = reinterpret_cast<int*>(v[i]);
      return o;
    };
    std::vector<float*> inv(L);
    for (size_t i = 0; i < L; ++i) inv[i] = reinterpret_cast<float*>(inv_deg[i]);
    auto a = ip(optr), b = ip(picks), c = ip(local), d = ip(src), e = ip(rp_t), f = ip(col_t), g = ip(cnt_t);
    chk(gnn_launch_sample_blocks(Pt<const int>(rowptr), Pt<const int>(col), n, Pt<const int>(seeds), n_seeds,
                                 (int)L, fan.data(), nd_max.data(), a.data(), inv.data(), b.data(), c.data(),
                                 d.data(), e.data(), f.data(), g.data(), Pt<int>(counts), Pt<uint8_t>(flag),
                                 Pt<int>(map), Pt<int>(bscratch), k0, k1, salt, S(st), Pt<int>(counts_host)),
        "gnn_sample_blocks");
  }, py::arg("rowptr"), py::arg("col"), py::arg("n"), py::arg("seeds"), py::arg("n_seeds"), py::arg("fan"),
     py::arg("nd_max"), py::arg("optr"), py::arg("inv_deg"), py::arg("picks"), py::arg("local"), py::arg("src"),
     py::arg("rp_t"), py::arg("col_t"), py::arg("cnt_t"), py::arg("counts"), py::arg("flag"), py::arg("map"),
     py::arg("bscratch"), py::arg("k0"), py::arg("k1"), py::arg("salt"), py::arg("st"),
     py::arg("counts_host") = 0);
  // page-locked, device-mapped, coherent host memory a kernel can publish small results
  // to (read by the host after an event): returns (host pointer, device pointer)
  m.def("host_mapped_alloc", [](size_t nbytes) {
    void* h = nullptr;
    void* d = nullptr;
    if (hipHostMalloc(&h, nbytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess || !h)
      throw std::runtime_error("hipHostMalloc failed");
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
      (void)hipHostFree(h);
      throw std::runtime_error("hipHostGetDevicePointer failed");
    }
    std::memset(h, 0, nbytes);
    return py::make_tuple((uint64_t)(uintptr_t)h, (uint64_t)(uintptr_t)d);
  });
  // native sampling worker (gnn_sampler.hip): handle = opaque pointer
  m.def("gnn_sw_create", [](int device, uint64_t st, uint64_t rowptr, uint64_t col, int n, std::vector<int> fan,
                            std::vector<int> nd_max, uint64_t flag, uint64_t map, uint64_t bscratch, uint32_t k0,
                            uint32_t k1) {
    if (fan.size() != nd_max.size() || fan.empty()) throw std::runtime_error("gnn_sw_create: bad level lists");
    for (int f : fan)
      if (f < 1 || f > 64) throw std::runtime_error("gnn_sw_create: fanouts must be in 1..64");
    return (uint64_t)(uintptr_t)gnn_sw_create(device, S(st), Pt<const int>(rowptr), Pt<const int>(col), n,
                                              (int)fan.size(), fan.data(), nd_max.data(), Pt<uint8_t>(flag),
                                              Pt<int>(map), Pt<int>(bscratch), k0, k1);
  });
  m.def("gnn_sw_add_slot", [](uint64_t h, std::vector<uint64_t> optr, std::vector<uint64_t> inv_deg,
                              std::vector<uint64_t> picks, std::vector<uint64_t> local, std::vector<uint64_t> src,
                              std::vector<uint64_t> rp_t, std::vector<uint64_t> col_t, std::vector<uint64_t> cnt_t,
                              uint64_t counts, uint64_t host) {
    const size_t L = optr.size();
    if (inv_deg.size() != L || picks.size() != L || local.size() != L || src.size() != L || rp_t.size() != L ||
        col_t.size() != L || cnt_t.size() != L)
      throw std::runtime_error("gnn_sw_add_slot: per-level lists differ in length");
    auto ip = [](const std::vector<uint64_t>& v) {
      std::vector<int*> o(v.size());
      for (size_t i = 0; i < v.size(); ++i) o[i] = reinterpret_cast<int*>(v[i]);
      return o;
    };
    std::vector<float*> inv(L);
    for (size_t i = 0; i < L; ++i) inv[i] = reinterpret_cast<float*>(inv_deg[i]);
    auto a = ip(optr), b = ip(picks), c = ip(local), d = ip(src), e = ip(rp_t), f = ip(col_t), g = ip(cnt_t);
    const int r = gnn_sw_add_slot((void*)(uintptr_t)h, a.data(), inv.data(), b.data(), c.data(), d.data(), e.data(),
                                  f.data(), g.data(), Pt<int>(counts), Pt<int>(host));
    if (r < 0) throw std::runtime_error("gnn_sw_add_slot failed");
    return r;
  });
  m.def("gnn_sw_submit", [](uint64_t h, int slot, uint64_t seeds, int n, uint32_t salt, std::vector<uint64_t> waits) {
    std::vector<hipEvent_t> ev;
    for (uint64_t x : waits)
      if (x) ev.push_back(reinterpret_cast<hipEvent_t>(x));
    const long r = gnn_sw_submit((void*)(uintptr_t)h, slot, Pt<const int>(seeds), n, salt, ev.data(), (int)ev.size());
    if (r <= 0) throw std::runtime_error("gnn_sw_submit: bad slot or seed count");
    return r;
  });
  m.def("gnn_sw_wait", [](uint64_t h, long seq, int slot, uint64_t consumer) {
    int r;
    {
      py::gil_scoped_release nogil;
      r = gnn_sw_wait((void*)(uintptr_t)h, seq, slot, S(consumer));
    }
    chk(r, "gnn_sw_wait (sampling worker)");
  });
  m.def("gnn_sw_destroy", [](uint64_t h) {
    py::gil_scoped_release nogil;
    gnn_sw_destroy((void*)(uintptr_t)h);
  });
  m.def("host_mapped_free", [](uint64_t h) { (void)hipHostFree((void*)(uintptr_t)h); });
  // the XCD block remaps of the kernels (cgnn_common.h), evaluated on the host (tests:
  // every form is a bijection of the grid)
  m.def("xcd_remap_table", [](unsigned nwg, unsigned chunk) {
    std::vector<unsigned> out(nwg);
    for (unsigned b = 0; b < nwg; ++b)
      out[b] = chunk == 0 ? cgnn::xcd_remap(b, nwg)
               : chunk == 64 ? cgnn::xcd_remap_chunked<64>(b, nwg)
               : chunk == 512 ? cgnn::xcd_remap_chunked<512>(b, nwg)
               : throw std::runtime_error("xcd_remap_table: chunk must be 0, 64 or 512");
    return out;
  });
  m.def("gnn_fused_bwd_blocks", &gnn_fused_bwd_blocks);
  m.def("gnn_fused_bwd_width", &gnn_fused_bwd_width);
  m.def("gnn_fused_bwd_supported", &gnn_fused_bwd_supported);
  m.def("gnn_fused_bwd", [](uint64_t ax, uint64_t dy2, uint64_t w1, uint64_t b1, uint64_t w2, uint64_t kimg,
                            uint64_t gpart, int n, int F, int ldx, int HD, int C, int ldc, float p, uint64_t st) {
    return gnn_launch_fused_bwd(Pt<const void>(ax), Pt<const void>(dy2), Pt<const float>(w1), Pt<const float>(b1),
                                Pt<const float>(w2), Pt<const void>(kimg), Pt<float>(gpart), n, F, ldx, HD, C, ldc,
                                p, S(st));
  });
  // generic fused dense layers (gnn_linear.hip); return codes: 0 ok, -1 no variant, -3 bad shape
  m.def("gnn_lin_fwd", [](uint64_t x1, int ld1, int K1, uint64_t x2, int ld2, int K2, uint64_t w, int N, uint64_t b,
                          uint64_t y, int ldy, int n, int relu, float p, uint32_t k0, uint32_t k1, uint32_t step,
                          uint32_t row0, uint64_t stepp, uint64_t rscale, uint64_t st, uint64_t idx1, uint64_t wimg,
                          uint64_t yf, int nsplit, int tk, int et) {
    return gnn_launch_lin_fwd(Pt<const void>(x1), ld1, K1, Pt<const void>(x2), ld2, K2, Pt<const float>(w), N,
                              Pt<const float>(b), Pt<void>(y), ldy, n, relu, p, k0, k1, step, row0,
                              Pt<const int>(stepp), Pt<const float>(rscale), Pt<const int>(idx1), Pt<void>(wimg),
                              Pt<float>(yf), nsplit, tk, S(st), et);
  }, py::arg("x1"), py::arg("ld1"), py::arg("K1"), py::arg("x2"), py::arg("ld2"), py::arg("K2"), py::arg("w"),
     py::arg("N"), py::arg("b"), py::arg("y"), py::arg("ldy"), py::arg("n"), py::arg("relu"), py::arg("p"),
     py::arg("k0"), py::arg("k1"), py::arg("step"), py::arg("row0"), py::arg("stepp"), py::arg("rscale"),
     py::arg("st"), py::arg("idx1") = 0, py::arg("wimg") = 0, py::arg("yf") = 0, py::arg("nsplit") = 0,
     py::arg("tk") = 1, py::arg("et") = 0);
  m.def("gnn_lin_fwd_image_bytes", &gnn_lin_fwd_image_bytes);
  m.def("gnn_lin_fwd_kc_wanted", &gnn_lin_fwd_kc_wanted);
  m.def("gnn_lin_bwd_image_bytes", &gnn_lin_bwd_image_bytes);
  m.def("gnn_lin_bwd_data", [](uint64_t dy, int lddy, uint64_t ym, int ldym, float mscale, int N, uint64_t w, int K1,
                               int K2, uint64_t dx1, int ldx1, uint64_t dx2, int ldx2, uint64_t rscale, int n,
                               uint64_t st, int dx1_f32, uint64_t wimg) {
    return gnn_launch_lin_bwd_data(Pt<const void>(dy), lddy, Pt<const void>(ym), ldym, mscale, N, Pt<const float>(w),
                                   K1, K2, Pt<void>(dx1), ldx1, Pt<void>(dx2), ldx2, Pt<const float>(rscale), n,
                                   dx1_f32, Pt<void>(wimg), S(st));
  }, py::arg("dy"), py::arg("lddy"), py::arg("ym"), py::arg("ldym"), py::arg("mscale"), py::arg("N"), py::arg("w"),
     py::arg("K1"), py::arg("K2"), py::arg("dx1"), py::arg("ldx1"), py::arg("dx2"), py::arg("ldx2"),
     py::arg("rscale"), py::arg("n"), py::arg("st"), py::arg("dx1_f32") = 0, py::arg("wimg") = 0);
  m.def("gnn_lin_wgrad_chunks", &gnn_lin_wgrad_chunks, py::arg("n"), py::arg("N"), py::arg("K") = 0);
  m.def("gnn_lin_bwd_weight", [](uint64_t x1, int ld1, int K1, uint64_t x2, int ld2, int K2, uint64_t dy, int lddy,
                                 uint64_t ym, int ldym, float mscale, int N, uint64_t gpart, uint64_t dw, uint64_t db,
                                 int n, uint64_t st, uint64_t idx1) {
    return gnn_launch_lin_bwd_weight(Pt<const void>(x1), ld1, K1, Pt<const void>(x2), ld2, K2, Pt<const void>(dy), lddy,
                                     Pt<const void>(ym), ldym, mscale, N, Pt<float>(gpart), Pt<float>(dw),
                                     Pt<float>(db), n, Pt<const int>(idx1), S(st));
  }, py::arg("x1"), py::arg("ld1"), py::arg("K1"), py::arg("x2"), py::arg("ld2"), py::arg("K2"), py::arg("dy"),
     py::arg("lddy"), py::arg("ym"), py::arg("ldym"), py::arg("mscale"), py::arg("N"), py::arg("gpart"),
     py::arg("dw"), py::arg("db"), py::arg("n"), py::arg("st"), py::arg("idx1") = 0);
  m.def("gnn_cast_bf16", [](uint64_t src, uint64_t dst, long n, uint64_t st) {
    chk(gnn_launch_cast_bf16(Pt<const float>(src), Pt<void>(dst), n, S(st)), "gnn_cast_bf16");
  });

  py::class_<PyEngine>(m, "CgnnEngine")
      .def(py::init<std::vector<int>, std::vector<float>, std::vector<uint64_t>, uint64_t>())
      .def("gen_blocks", &PyEngine::gen_blocks)
      .def("n_parts", &PyEngine::n_parts)
      .def("init", &PyEngine::init)
      .def("tt", &PyEngine::tt)
      .def("run", &PyEngine::run, py::arg("kind"), py::arg("steps"), py::arg("chunk") = 0,
           py::arg("hist") = false);
}
