// Native CGNN step engine: owns the per-step launch sequence for one batch of
// R models and replays it through hipGraphs.
//
//   train step : gen_fwd -> mmd(train) -> loss_finalize -> gen_bwd -> adam
//   eval step  : gen_fwd -> mmd(eval)  -> loss_finalize(accumulate)
// (wide graphs: gen_fwd = gen_fwd_staged, which draws the step's noise itself, gen_bwd =
// gen_bwd_staged)
//
// A chunk of `chunk` steps (step offsets baked in as literals) plus one
// advance_step node is captured once per (kind, chunk) and replayed; the RNG
// and optimizer step counters live in device memory (step_base[0..1]), so every
// replay draws fresh noise.  All device buffers are owned
// by PyTorch on the Python side; the engine only holds raw pointers and is
// rebuilt whenever a buffer is reallocated.  Reusing the same engine for a new
// search candidate only requires rewriting the program/data/key buffers and
// re-running init -- the captured graphs stay valid.
#include "cgnn_common.h"
#include <map>
#include <stdexcept>
#include <string>

extern "C" {
int cgnn_launch_mmd(int, int, const float*, const float*, float*, float*, int, int, int, int, int,
                    float, hipStream_t, int);
int cgnn_launch_mmd_mfma(int, int, const float*, const float*, const float*, const float*, float*, float*,
                         int, int, int, int, float, hipStream_t);
int cgnn_mmd_mfma_row_blocks(int);
int cgnn_launch_loss_finalize(const float*, int, float*, float*, float*, float, int, float*, int,
                              const int*, int, int, hipStream_t);
int cgnn_launch_gen_fwd(const int*, int, const float*, int, const float*, float*, float*, int, float*,
                        const uint32_t*, const int*, int, int, int, int, int, hipStream_t, int);
int cgnn_launch_gen_bwd(const int*, int, const float*, int, const float*, const float*, int,
                        const float*, int, int, int, int, int, int, int, float*, hipStream_t);
int cgnn_staged_tiles(int);
int cgnn_launch_gen_noise(const int*, int, const uint32_t*, const int*, int, float*, int, int, int, int, int, int,
                          hipStream_t);
int cgnn_launch_gen_fwd_staged_draw(const int*, int, const int*, int, const float*, int, const float*, float*, float*,
                                    int, float*, int, int, int, int, int, int, int, hipStream_t, int, const uint32_t*,
                                    const int*, int, int);
int cgnn_launch_gen_fwd_staged(const int*, int, const int*, int, const float*, int, const float*, float*,
                               const float*, int, float*, int, int, int, int, int, int, int, hipStream_t, int);
int cgnn_launch_gen_bwd_staged(const int*, int, const int*, int, const float*, int, const float*, const float*, int,
                               const float*, int, int, int, int, int, int, int, int, float*, float*, hipStream_t,
                               int);
int cgnn_mmd_supported_d(int);
int cgnn_gen_bwd_blocks(int);
int cgnn_launch_adam(float*, float*, float*, const float*, int, const int*, int, int, const int*,
                     int, float, float, float, float, int, hipStream_t);
int cgnn_launch_init(float*, float*, float*, const int*, int, int, const uint32_t*, float, int,
                     hipStream_t);
int cgnn_launch_advance(int*, int, int, hipStream_t);
int rff_launch_freqs(float*, const uint32_t*, const int*, int, int, int, int, int, int, hipStream_t);
int rff_launch_fwd_bwd(int, const float*, const float*, const float*, float*, float*, float*, int,
                       int, int, int, int, float, hipStream_t, int, float*, int);
}

namespace cgnn {

struct EngineConfig {
  int R = 0, N = 0, D = 0, H = 0, P = 0, prog_stride = 0, max_in = 0;
  int row_tiles = 0, n_chunks = 0, tpc = 0;
  float lr = 0.01f, beta1 = 0.9f, beta2 = 0.999f, eps = 1e-8f, init_std = 0.05f;
  int hist_stride = 0;
  int rff_k = 0;     // > 0: random-Fourier-feature MMD with k features per bandwidth
  int d_true = 0;    // unpadded variable count (RFF draws must not depend on padding)
  int NS = 0;        // noise streams per model = D + max #confounder streams
  int mfma = 0;      // 1: train/eval MMD on the matrix cores (mmd_mfma.hip), D >= 8
  int mf_chunks = 1, mf_tpc = 0;   // its column chunking (32-wide tiles per chunk)
  int mirror = 0;    // > 0: symmetric vector-kernel training, `mirror` extra gradient slots
  int staged = 0;    // 1: level-scheduled generator kernels (wide graphs, cgnn_staged.hip)
  int sched_stride = 0, stage_w = 8;
};

struct EngineBuffers {
  const int* prog = nullptr;
  float* params = nullptr;
  float* m = nullptr;
  float* v = nullptr;
  const float* data = nullptr;
  float* xhat = nullptr;
  float* noise = nullptr;    // [R][NS][N] noise draws of the forward, reused by the backward
  float* gradp = nullptr;   // [n_chunks][R][D][N]
  float* lpart = nullptr;   // [R][n_chunks*row_tiles]
  float* gpart = nullptr;   // [R][G][P]
  float* tt = nullptr;      // [R]
  float* loss_last = nullptr;
  float* loss_acc = nullptr;
  float* loss_hist = nullptr;   // optional [R][hist_stride]
  int* step = nullptr;          // [2]
  const uint32_t* keys = nullptr;
  float* rff_w = nullptr;       // [R][7k][D+1]
  float* rff_diff = nullptr;    // [R][7k]
  float* rff_scratch = nullptr; // the wide form (engine.batch.WIDE_RFF_D): rff_wide_scratch_floats(N, 7k, R)
  float* xnorm = nullptr;       // [R][N] squared norms of xhat rows (written by gen_fwd)
  const float* ynorm = nullptr; // [R][N] squared norms of the data rows
  float* dxs = nullptr;         // [R][d_true][N] dL/dx scratch of a staged backward whose state is global
  const int* sched = nullptr;   // [R][sched_stride] stage schedules (staged kernels)
};

class Engine {
 public:
  Engine(const EngineConfig& c, const EngineBuffers& b, hipStream_t s) : c_(c), b_(b), st_(s) {
    G_ = c_.staged ? cgnn_staged_tiles(c_.N) : cgnn_gen_bwd_blocks(c_.N);
  }
  ~Engine() { clear_graphs(); }

  void clear_graphs() {
    for (auto& kv : graphs_) {
      (void)hipGraphExecDestroy(kv.second.first);
      (void)hipGraphDestroy(kv.second.second);
    }
    graphs_.clear();
  }

  static constexpr int kGammaCount = 7;
  int rff_features() const { return c_.rff_k * kGammaCount; }
  // loss partials per model of a train/eval step, and of the constant true-true pass
  int n_parts() const {
    if (c_.rff_k > 0) return (rff_features() + 255) / 256;
    if (c_.mfma) return c_.mf_chunks * cgnn_mmd_mfma_row_blocks(c_.N);
    return c_.n_chunks * c_.row_tiles;
  }
  // the vector kernel's true-true pass where it has a variant; the matrix-core one
  // (mode 2) for the wide joints only it covers
  bool tt_mfma() const { return c_.mfma && !cgnn_mmd_supported_d(c_.D); }
  int n_parts_tt() const {
    return tt_mfma() ? c_.mf_chunks * cgnn_mmd_mfma_row_blocks(c_.N) : c_.n_chunks * c_.row_tiles;
  }
  int grad_chunks() const { return c_.rff_k > 0 ? 1 : (c_.mfma ? c_.mf_chunks : c_.n_chunks + (c_.mirror > 0 ? c_.mirror : 0)); }

  // loss (+ gradient when train) of the current xhat; `need_loss` false lets the
  // matrix-core kernel skip the (unread) training loss
  void enqueue_loss(int off, bool train, bool need_loss = true) {
    if (c_.rff_k > 0) {
      check(rff_launch_freqs(b_.rff_w, b_.keys, b_.step, off, c_.rff_k, c_.D, kGammaCount, c_.d_true,
                             c_.R, st_), "rff_freqs");
      check(rff_launch_fwd_bwd(train ? 0 : 1, b_.xhat, b_.data, b_.rff_w, b_.rff_diff, b_.lpart,
                               b_.gradp, c_.N, c_.D, rff_features(), c_.R, c_.rff_k,
                               sqrtf(2.f / (float)c_.rff_k), st_, 0, b_.rff_scratch,
                               b_.rff_scratch != nullptr), "rff");
    } else if (c_.mfma) {
      const float inv = 1.f / ((float)c_.N * (float)c_.N);
      check(cgnn_launch_mmd_mfma(train ? (need_loss ? 0 : 3) : 1, c_.D, b_.xhat, b_.data, b_.xnorm, b_.ynorm,
                                 b_.gradp, b_.lpart, c_.N, c_.R,
                                 c_.mf_chunks, c_.mf_tpc, train ? 4.f * inv : 0.f, st_), "mmd_mfma");
    } else {
      const float inv = 1.f / ((float)c_.N * (float)c_.N);
      check(cgnn_launch_mmd(train ? (need_loss ? 0 : 3) : 1, c_.D, b_.xhat, b_.data, b_.gradp, b_.lpart, c_.N, c_.R,
                            c_.row_tiles, c_.n_chunks, c_.tpc, train ? 4.f * inv : 0.f, st_,
                            train && c_.mirror > 0 ? 1 : 0), "mmd");
    }
  }
  float loss_scale() const { return c_.rff_k > 0 ? 1.f : 1.f / ((float)c_.N * (float)c_.N); }
  int gen_blocks() const { return G_; }

  void check(int rc, const char* what) {
    if (rc != 0) throw std::runtime_error(std::string("cgnn engine: ") + what + " failed, code " + std::to_string(rc));
  }

  void init_params() {
    check(cgnn_launch_init(b_.params, b_.m, b_.v, b_.prog, c_.prog_stride, c_.P, b_.keys, c_.init_std, c_.R, st_), "init");
  }

  // true-true block of the MMD (constant in the parameters): once per data upload
  void compute_tt() {
    if (c_.rff_k > 0) return;   // the Fourier loss has no constant block
    const float inv = 1.f / ((float)c_.N * (float)c_.N);
    if (tt_mfma())
      check(cgnn_launch_mmd_mfma(2, c_.D, b_.xhat, b_.data, b_.xnorm, b_.ynorm, b_.gradp, b_.lpart, c_.N, c_.R,
                                 c_.mf_chunks, c_.mf_tpc, 0.f, st_), "mmd_mfma(tt)");
    else
      check(cgnn_launch_mmd(2, c_.D, b_.xhat, b_.data, b_.gradp, b_.lpart, c_.N, c_.R, c_.row_tiles,
                            c_.n_chunks, c_.tpc, 0.f, st_, 0), "mmd(tt)");
    check(cgnn_launch_loss_finalize(b_.lpart, n_parts_tt(), b_.tt, b_.loss_last, b_.loss_acc, inv, 2,
                                    nullptr, 0, b_.step, 0, c_.R, st_), "finalize(tt)");
  }

  // train: the staged forward stores its noise draws for the backward
  void enqueue_gen_fwd(int off, bool train) {
    if (c_.staged) {
      // the forward draws the step's noise itself (and stores it for the backward)
      check(cgnn_launch_gen_fwd_staged_draw(b_.prog, c_.prog_stride, b_.sched, c_.sched_stride, b_.params, c_.P,
                                            b_.data, b_.xhat, train ? b_.noise : nullptr, c_.NS, b_.xnorm, c_.N,
                                            c_.D, c_.d_true, c_.H, c_.max_in, c_.R, c_.stage_w, st_, -1, b_.keys,
                                            b_.step, off, 0),
            "gen_fwd_staged");
    } else {
      check(cgnn_launch_gen_fwd(b_.prog, c_.prog_stride, b_.params, c_.P, b_.data, b_.xhat, b_.noise, c_.NS,
                                b_.xnorm, b_.keys, b_.step, off, c_.N, c_.D, c_.H, c_.R, st_, 0), "gen_fwd");
    }
  }

  void enqueue_train_step(int off, bool record_hist) {
    const float inv = loss_scale();
    enqueue_gen_fwd(off, true);
    enqueue_loss(off, true, record_hist);
    // the training loss is only observable through the recorded history
    if (record_hist)
      check(cgnn_launch_loss_finalize(b_.lpart, n_parts(), b_.tt, b_.loss_last, b_.loss_acc, inv, 0,
                                      b_.loss_hist, c_.hist_stride, b_.step, off, c_.R, st_), "finalize");
    if (c_.staged)
      check(cgnn_launch_gen_bwd_staged(b_.prog, c_.prog_stride, b_.sched, c_.sched_stride, b_.params, c_.P, b_.xhat,
                                       b_.noise, c_.NS, b_.gradp, grad_chunks(), c_.R, c_.N, c_.D, c_.d_true, c_.H,
                                       c_.max_in, c_.stage_w, b_.gpart, b_.dxs, st_, -1), "gen_bwd_staged");
    else
      check(cgnn_launch_gen_bwd(b_.prog, c_.prog_stride, b_.params, c_.P, b_.xhat, b_.noise, c_.NS, b_.gradp,
                                grad_chunks(), c_.R, c_.N, c_.D, c_.d_true, c_.H, c_.max_in, b_.gpart, st_),
            "gen_bwd");
    check(cgnn_launch_adam(b_.params, b_.m, b_.v, b_.gpart, G_, b_.prog, c_.prog_stride, c_.P, b_.step,
                           off, c_.lr, c_.beta1, c_.beta2, c_.eps, c_.R, st_), "adam");
  }

  void enqueue_eval_step(int off) {
    const float inv = loss_scale();
    enqueue_gen_fwd(off, false);
    enqueue_loss(off, false);
    check(cgnn_launch_loss_finalize(b_.lpart, n_parts(), b_.tt, b_.loss_last, b_.loss_acc, inv, 1,
                                    nullptr, 0, b_.step, off, c_.R, st_), "finalize(eval)");
  }

  void enqueue_chunk(int kind, int n, bool hist) {
    for (int k = 0; k < n; ++k) {
      if (kind == 0) enqueue_train_step(k, hist);
      else enqueue_eval_step(k);
    }
    check(cgnn_launch_advance(b_.step, n, kind == 0 ? n : 0, st_), "advance");
  }

  // Run `steps` steps of `kind` (0 train, 1 eval).  chunk <= 0 -> eager launches.
  void run(int kind, int steps, int chunk, bool hist) {
    if (steps <= 0) return;
    if (chunk <= 0) {
      enqueue_chunk(kind, steps, hist);
      return;
    }
    chunk = std::min(chunk, steps);
    const int full = steps / chunk, rem = steps - full * chunk;
    if (full > 0) {
      hipGraphExec_t exec = get_graph(kind, chunk, hist);
      for (int k = 0; k < full; ++k) check((int)hipGraphLaunch(exec, st_), "graph launch");
    }
    if (rem > 0) enqueue_chunk(kind, rem, hist);
  }

 private:
  hipGraphExec_t get_graph(int kind, int chunk, bool hist) {
    const long key = ((long)kind << 40) | ((long)hist << 39) | chunk;
    auto it = graphs_.find(key);
    if (it != graphs_.end()) return it->second.first;
    hipGraph_t g = nullptr;
    check((int)hipStreamBeginCapture(st_, hipStreamCaptureModeThreadLocal), "begin capture");
    try {
      enqueue_chunk(kind, chunk, hist);
    } catch (...) {
      (void)hipStreamEndCapture(st_, &g);
      if (g) (void)hipGraphDestroy(g);
      throw;
    }
    check((int)hipStreamEndCapture(st_, &g), "end capture");
    hipGraphExec_t exec = nullptr;
    check((int)hipGraphInstantiate(&exec, g, nullptr, nullptr, 0), "instantiate");
    graphs_[key] = {exec, g};
    return exec;
  }

  EngineConfig c_;
  EngineBuffers b_;
  hipStream_t st_;
  int G_ = 1;
  std::map<long, std::pair<hipGraphExec_t, hipGraph_t>> graphs_;
};

}  // namespace cgnn

// ---------------------------------------------------------------- C ABI
extern "C" void* cgnn_engine_create(const int* icfg, const float* fcfg, const void* const* ptrs,
                                    hipStream_t st) {
  cgnn::EngineConfig c;
  c.R = icfg[0]; c.N = icfg[1]; c.D = icfg[2]; c.H = icfg[3]; c.P = icfg[4];
  c.prog_stride = icfg[5]; c.max_in = icfg[6]; c.row_tiles = icfg[7]; c.n_chunks = icfg[8];
  c.tpc = icfg[9]; c.hist_stride = icfg[10]; c.rff_k = icfg[11]; c.d_true = icfg[12]; c.NS = icfg[13];
  c.mfma = icfg[14]; c.mf_chunks = icfg[15]; c.mf_tpc = icfg[16]; c.mirror = icfg[17];
  c.staged = icfg[18]; c.sched_stride = icfg[19]; c.stage_w = icfg[20];
  c.lr = fcfg[0]; c.beta1 = fcfg[1]; c.beta2 = fcfg[2]; c.eps = fcfg[3]; c.init_std = fcfg[4];
  cgnn::EngineBuffers b;
  b.prog = (const int*)ptrs[0]; b.params = (float*)ptrs[1]; b.m = (float*)ptrs[2];
  b.v = (float*)ptrs[3]; b.data = (const float*)ptrs[4]; b.xhat = (float*)ptrs[5];
  b.noise = (float*)ptrs[6]; b.gradp = (float*)ptrs[7]; b.lpart = (float*)ptrs[8];
  b.gpart = (float*)ptrs[9]; b.tt = (float*)ptrs[10]; b.loss_last = (float*)ptrs[11];
  b.loss_acc = (float*)ptrs[12]; b.loss_hist = (float*)ptrs[13]; b.step = (int*)ptrs[14];
  b.keys = (const uint32_t*)ptrs[15]; b.rff_w = (float*)ptrs[16]; b.rff_diff = (float*)ptrs[17];
  b.xnorm = (float*)ptrs[18]; b.ynorm = (const float*)ptrs[19]; b.dxs = (float*)ptrs[20];
  b.sched = (const int*)ptrs[21]; b.rff_scratch = (float*)ptrs[22];
  return new cgnn::Engine(c, b, st);
}

extern "C" void cgnn_engine_destroy(void* e) { delete (cgnn::Engine*)e; }
extern "C" int cgnn_engine_gen_blocks(void* e) { return ((cgnn::Engine*)e)->gen_blocks(); }
extern "C" int cgnn_engine_n_parts(void* e) { return ((cgnn::Engine*)e)->n_parts(); }
extern "C" void cgnn_engine_init(void* e) { ((cgnn::Engine*)e)->init_params(); }
extern "C" void cgnn_engine_tt(void* e) { ((cgnn::Engine*)e)->compute_tt(); }
extern "C" void cgnn_engine_run(void* e, int kind, int steps, int chunk, int hist) {
  ((cgnn::Engine*)e)->run(kind, steps, chunk, hist != 0);
}
