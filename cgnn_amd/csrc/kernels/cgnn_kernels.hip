// CGNN device kernels for MI355X (gfx950).  One launch always serves a whole
// batch of R independent generative models ("runs x candidates"), so the
// reference's ~48k tiny TF session calls per search candidate
// become a handful of fused launches per optimisation step.
//
//   K3/K4 mmd_rbf_kernel   fused multi-bandwidth Gaussian MMD^2: loss and the
//                          analytic gradient wrt the generated samples, never
//                          materialising the [2N,2N] Gram (replaces Loss.py:12-32
//                          and its TF autodiff).
//   K1    gen_fwd_kernel   DAG generator forward: CSR-parent gather, in-kernel
//                          Philox noise, Linear->ReLU->Linear per node in
//                          topological order (CGNN.py:63-90, GNN.py:64-67,
//                          CGNN_confounders.py:66-104).
//   K2    gen_bwd_kernel   reverse-topological backward with deterministic
//                          LDS slab reduction of parameter gradients.
//   K5    adam_tf1_kernel  TF1 AdamOptimizer update (epsilon outside the bias
//                          correction) fused with the cross-workgroup gradient sum.
//
// Layouts (all fp32):
//   data, xhat, dxhat : [R][D][N]    feature-major, so a wave of 64 consecutive
//                                    samples touches 256 contiguous bytes.
//   params, m, v      : [R][P]       per-node blocks W1[nin][H], b1[H], W2[H], b2.
//   prog              : [R][stride]  int32 "DAG program", see engine/program.py.
#include "cgnn_common.h"
#include <cstdlib>

using namespace cgnn;

namespace {

constexpr float MMD_SENTINEL = 1.0e17f;   // padded columns: exp(-g*d2) == 0 exactly

}  // namespace

// ============================================================================
// K3/K4: fused MMD.  grid = (row_tiles, n_chunks, R), block = 256.
//   MODE 0: train  -> loss partial + gradient partial per column chunk
//   MODE 1: eval   -> loss partial only
//   MODE 2: const  -> true-true block (rows and columns from `data`)
// Each thread owns one row i of the generated block and streams 256-column
// tiles of the joint [pred; true] column space through LDS (broadcast reads).
// Columns are consumed in PAIRS with packed fp32 math (v_pk_add/mul/fma_f32 do
// two lanes' worth of work per issue): the LDS tile is laid out
// [T/2][D][2] so that one ds_read_b64 returns (x_j[k], x_{j+1}[k]) ready packed.
// Per column pair: 3D packed ops for distance + gradient, 10 v_exp_f32 and
// ~20 packed ops for the seven kernel values and their weights.
//   grad_i += sign * w_ij * (x_j - p_i),  sign = +1 (pred col), -1 (true col)
//   loss   += (+1 | -2) * sum_gamma exp(-gamma d2)
// dL/dp_i = 4/N^2 * grad_i  (derivation in docs/KERNELS.md).
// ============================================================================
// f2, exp2_2 and rbf7x2 live in cgnn_common.h (shared with mmd_mfma.hip)

// Rows: generated samples [row_begin, row_begin + n_rows) of the N columns (a
// sample-sharded MMD evaluates only its own rows against all columns); gradient
// partials are written with the local row stride n_rows.
//
// mirror (training, D <= MMD_SYM_MAX_D, all rows): the pred-pred block is evaluated only
// at and right of the diagonal tile.  An off-diagonal tile (a, b > a) feeds both sides:
// row i of a takes w_ij (x_j - p_i) as usual, and column j of b -- itself a generated
// row -- takes the mirrored w_ij (p_i - x_j), summed over the 256 rows of the tile.
// That column sum is done without atomics or shuffles-per-column: lane l of a wave
// visits the column pairs of a 64-pair group in the staggered order (l + s) mod 64, and
// the per-pair accumulators ride along with a full-wave DPP rotate fused into the add
// (v_add_f32_dpp wave_rol:1), so after 64 steps each lane holds the complete wave sum
// of one pair; the 4 waves' sums are added in LDS in a fixed order and written to
// grad_part slot n_chunks + a (rows of b).  Blocks (a, b <= a) zero their rows of that
// slot, so the consumer just sums n_chunks + row_tiles - 1 slots (cgnn_mmd_mirror_slots).
// Every order is a function of N only: bitwise reproducible and batch-independent.
constexpr int MMD_SYM_MAX_D = 8;

__device__ __forceinline__ float rot_next(float x) {      // lane l <- lane (l + 1) mod 64
  // a full rotate has no out-of-range source lane, so no `old` value to initialise
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x134, 0xf, 0xf, true));
}

template <int D, int MODE>
__global__ __launch_bounds__(256) void mmd_rbf_kernel(
    const float* __restrict__ xhat, const float* __restrict__ data,
    float* __restrict__ grad_part, float* __restrict__ loss_part,
    int N, int R, int tiles_per_chunk, float grad_scale, int row_begin, int n_rows, int mirror) {
  // MODE 3: training step whose loss nobody reads (no history): gradient only
  constexpr bool GRAD = MODE == 0 || MODE == 3;
  constexpr bool LOSS = MODE != 3;
  constexpr bool SYMG = GRAD && D <= MMD_SYM_MAX_D;
  constexpr int T = 256;
  __shared__ __attribute__((aligned(16))) float s_x[T * D];   // [T/2][D][2]
  __shared__ __attribute__((aligned(16))) float s_col[SYMG ? 4 * D * T : 1];   // [wave][D][T]
  __shared__ float s_red[4];

  const int rt = blockIdx.x, chunk = blockIdx.y, r = blockIdx.z;
  const int n_chunks = gridDim.y, row_tiles = gridDim.x;
  const int t = threadIdx.x;
  const int il = rt * T + t;                 // local row
  const int i = row_begin + il;              // column index of this row's sample
  const bool valid = il < n_rows;
  const size_t mbase = (size_t)r * D * N;
  const float* P = (MODE == 2 ? data : xhat) + mbase;
  const float* Tm = data + mbase;

  // padding rows sit at the sentinel: their weights against every real column are
  // exactly 0, so they add nothing to the mirrored column sums (their own row sums
  // and loss are discarded)
  f2 p[D], g[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    const float pk = valid ? P[(size_t)k * N + i] : MMD_SENTINEL;
    p[k] = f2{pk, pk};
    g[k] = f2{0.f, 0.f};
  }
  float lacc = 0.f;

  const int ct = (N + T - 1) / T;               // tiles per block
  const int n_tiles = (MODE == 2) ? ct : 2 * ct;
  const int tile_lo = chunk * tiles_per_chunk;
  const int tile_hi = min(n_tiles, tile_lo + tiles_per_chunk);
  float* my = s_x + ((t >> 1) * D) * 2 + (t & 1);

  // the pred-pred block is symmetric, so only column tiles at or right of the row tile
  // are evaluated, those strictly right counting twice in the loss (25 % fewer
  // distances; geometry fixed by N, so still bitwise reproducible and independent of
  // the batch).  Evaluation: always over all rows; training: with mirror slots.
  const bool all_rows = row_begin == 0 && n_rows == N;
  const bool msym = SYMG && mirror && all_rows;
  const bool sym = (MODE == 1 && all_rows) || msym;
  float* gmir = msym && rt < row_tiles - 1 ? grad_part + ((size_t)(n_chunks + rt) * R + r) * D * N : nullptr;
  for (int tile = tile_lo; tile < tile_hi; ++tile) {
    const bool is_pred = (MODE != 2) && tile < ct;
    if (sym && is_pred && tile <= rt && gmir) {          // this block's mirror rows of the tile: none
      const int c = tile * T + t;
      if (c < N)
#pragma unroll
        for (int k = 0; k < D; ++k) gmir[(size_t)k * N + c] = 0.f;
    }
    if (sym && is_pred && tile < rt) continue;           // block-uniform: no barrier divergence
    const float* src = is_pred ? P : Tm;
    const int col0 = (is_pred || MODE == 2 ? tile : tile - ct) * T;
    const int c = col0 + t;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < D; ++k) my[2 * k] = (c < N) ? src[(size_t)k * N + c] : MMD_SENTINEL;
    __syncthreads();
    const float lsign = (MODE == 2 || is_pred) ? ((sym && tile > rt) ? 2.f : 1.f) : -2.f;
    const float gsign = is_pred ? 1.f : -1.f;
    f2 tl = {0.f, 0.f};
    const f2* xp = reinterpret_cast<const f2*>(s_x);
    if constexpr (SYMG) {
      if (msym && is_pred && tile > rt) {                // block-uniform
        const int lane = t & 63, wv = t >> 6;
#pragma unroll 1
        for (int grp = 0; grp < 2; ++grp) {
          f2 ca[D];
#pragma unroll
          for (int k = 0; k < D; ++k) ca[k] = f2{0.f, 0.f};
#pragma unroll 2
          for (int s = 0; s < 64; ++s) {
            const f2* xj = xp + (grp * 64 + ((lane + s) & 63)) * D;
            f2 diff[D];
            f2 d2 = {0.f, 0.f};
#pragma unroll
            for (int k = 0; k < D; ++k) {
              diff[k] = xj[k] - p[k];
              d2 = diff[k] * diff[k] + d2;
            }
            f2 ks, w;
            rbf7x2(d2, ks, w);
            if (LOSS) tl += ks;
#pragma unroll
            for (int k = 0; k < D; ++k) {
              const f2 wd = w * diff[k];
              g[k] += wd;
              ca[k] = f2{rot_next(ca[k].x), rot_next(ca[k].y)} + wd;
            }
          }
          // lane l now holds the wave's sums for pair (l - 1) mod 64 of the group
          const int q = grp * 64 + ((lane + 63) & 63);
#pragma unroll
          for (int k = 0; k < D; ++k)
            *reinterpret_cast<f2*>(s_col + (wv * D + k) * T + 2 * q) = ca[k];
        }
        __syncthreads();
        if (c < N && gmir) {
#pragma unroll
          for (int k = 0; k < D; ++k) {
            const float v = (s_col[(0 * D + k) * T + t] + s_col[(1 * D + k) * T + t]) +
                            (s_col[(2 * D + k) * T + t] + s_col[(3 * D + k) * T + t]);
            gmir[(size_t)k * N + c] = -v * grad_scale;     // w_ij (p_i - x_j) = -w_ij diff_ij
          }
        }
        if (LOSS) lacc = fmaf(lsign, tl.x + tl.y, lacc);
        continue;
      }
    }
#pragma unroll 2
    for (int jj = 0; jj < T / 2; ++jj) {
      const f2* xj = xp + jj * D;
      f2 diff[D];
      f2 d2 = {0.f, 0.f};
#pragma unroll
      for (int k = 0; k < D; ++k) {
        diff[k] = xj[k] - p[k];
        d2 = diff[k] * diff[k] + d2;
      }
      f2 ks, w;
      rbf7x2(d2, ks, w);
      if (LOSS) tl += ks;
      if (GRAD) {
        const f2 sw = gsign * w;
#pragma unroll
        for (int k = 0; k < D; ++k) g[k] = sw * diff[k] + g[k];
      }
    }
    if (LOSS) lacc = fmaf(lsign, tl.x + tl.y, lacc);
  }

  // deterministic block reduction of the loss partial
  float v = valid ? lacc : 0.f;
  v = wave_sum(v);
  if ((t & 63) == 0) s_red[t >> 6] = v;
  __syncthreads();
  if (t == 0) {
    float s = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
    loss_part[((size_t)r * n_chunks + chunk) * row_tiles + rt] = s;
  }
  if (GRAD && valid) {
    float* gp = grad_part + ((size_t)chunk * R + r) * D * n_rows;
#pragma unroll
    for (int k = 0; k < D; ++k) gp[(size_t)k * n_rows + il] = (g[k].x + g[k].y) * grad_scale;
  }
}

// ============================================================================
// Loss finalize: one block per model, fixed-order sum of the partials.
//   L = (sum_partials + tt_const[r]) * inv_n2
//   flags bit0: accumulate into loss_acc (evaluation average)
//   flags bit1: write raw sum into tt_const (true-true constant pass)
// ============================================================================
__global__ __launch_bounds__(256) void loss_finalize_kernel(
    const float* __restrict__ loss_part, int n_parts, float* __restrict__ tt_const,
    float* __restrict__ loss_last, float* __restrict__ loss_acc, float inv_n2, int flags,
    float* __restrict__ loss_hist, int hist_stride, const int* __restrict__ step_base, int step_off) {
  __shared__ float s_red[4];
  const int r = blockIdx.x;
  const float* lp = loss_part + (size_t)r * n_parts;
  float s = 0.f;
  for (int k = threadIdx.x; k < n_parts; k += blockDim.x) s += lp[k];
  s = block_sum(s, s_red);
  if (threadIdx.x == 0) {
    if (flags & 2) {
      tt_const[r] = s;
    } else {
      float L = (s + tt_const[r]) * inv_n2;
      loss_last[r] = L;
      if (flags & 1) loss_acc[r] += L;
      if (loss_hist) {
        int st = step_off + (step_base ? step_base[1] : 0);
        if (st < hist_stride) loss_hist[(size_t)r * hist_stride + st] = L;
      }
    }
  }
}


// ============================================================================
// K1: generator forward.  grid = (ceil(N/256), R), one thread per sample.
// The model's DAG program is staged in LDS once, and the sample's generated
// values live in LDS (s_x[var][thread]) for the whole sweep, so a parent read is
// an LDS access rather than a dependent global round trip.  The draws of every
// noise stream are written to `noise` ([R][NS][N], NS = D + #confounder
// streams) for the backward.  Weights are read with wave-uniform (scalar) loads.
// ============================================================================
template <int H>
__global__ __launch_bounds__(256) void gen_fwd_kernel(
    const int* __restrict__ prog, int prog_stride, const float* __restrict__ params, int P,
    const float* __restrict__ data, float* __restrict__ xhat, float* __restrict__ noise, int NS,
    float* __restrict__ xnorm, const uint32_t* __restrict__ keys, const int* __restrict__ step_base,
    int step_off, int N, int D, int Hrt, int row0) {
  // row0: global index of sample 0 (a sample-sharded job keys every noise draw by the
  // GLOBAL sample, so the generated samples do not depend on the rank count)
  extern __shared__ __attribute__((aligned(16))) float s_x[];   // [D][blockDim], then program
  const int r = blockIdx.y;
  const int t = threadIdx.x, B = blockDim.x;
  const int n = blockIdx.x * B + t;
  const bool valid = n < N;
  const int nc = valid ? n : 0;
  int* s_prog = reinterpret_cast<int*>(s_x + (size_t)D * B);
  const int* pg = prog + (size_t)r * prog_stride;
  for (int i = t; i < prog_stride; i += B) s_prog[i] = pg[i];
  __syncthreads();
  const int nn = uni(s_prog);
  const uint32_t step = (uint32_t)(step_base[0] + step_off);
  const uint32_t k0 = keys[2 * r], k1 = keys[2 * r + 1];
  const float* th = params + (size_t)r * P;
  const float* dr = data + (size_t)r * D * N;
  float* nz = noise + (size_t)r * NS * N;
  const int Hh = (H > 0) ? H : Hrt;

  for (int kk = 0; kk < nn; ++kk) {
    const int* nd = s_prog + PROG_HDR + kk * NODE_REC;
    const int var = uni(nd);
    if (uni(nd + 1) == KIND_OBS) {
      s_x[var * B + t] = dr[(size_t)var * N + nc];
      continue;
    }
    const int npar = uni(nd + 2), paroff = uni(nd + 3), ncf = uni(nd + 4), cfoff = uni(nd + 5);
    const int poff = uni(nd + 6);
    const int nin = npar + 1 + ncf;
    const float* W1 = th + poff;
    const float* b1 = W1 + (size_t)nin * Hh;
    const float* W2 = b1 + Hh;
    const float b2 = W2[Hh];
    const float e = rng_normal(k0, k1, (uint32_t)(row0 + n), (uint32_t)var, step, RNG_NODE_NOISE);
    if (valid) nz[(size_t)var * N + n] = e;
    if (H > 0) {
      float pre[H > 0 ? H : 1];
#pragma unroll
      for (int q = 0; q < H; ++q) pre[q] = fmaf(W1[npar * H + q], e, b1[q]);
      for (int j = 0; j < npar; ++j) {
        const float x = s_x[uni(s_prog + paroff + j) * B + t];
#pragma unroll
        for (int q = 0; q < H; ++q) pre[q] = fmaf(W1[j * H + q], x, pre[q]);
      }
      for (int c = 0; c < ncf; ++c) {
        const int cid = uni(s_prog + cfoff + c);
        const float ec = rng_normal(k0, k1, (uint32_t)(row0 + n), (uint32_t)cid, step, RNG_CONF_NOISE);
        if (valid) nz[(size_t)(D + cid) * N + n] = ec;
#pragma unroll
        for (int q = 0; q < H; ++q) pre[q] = fmaf(W1[(npar + 1 + c) * H + q], ec, pre[q]);
      }
      float out = b2;
#pragma unroll
      for (int q = 0; q < H; ++q) out = fmaf(W2[q], fmaxf(pre[q], 0.f), out);
      s_x[var * B + t] = out;
    } else {
      // generic hidden width: hidden unit outer loop (no register array)
      float out = b2;
      for (int c = 0; c < ncf; ++c) {
        const int cid = uni(s_prog + cfoff + c);
        if (valid)
          nz[(size_t)(D + cid) * N + n] = rng_normal(k0, k1, (uint32_t)(row0 + n), (uint32_t)cid, step,
                                                     RNG_CONF_NOISE);
      }
      for (int q = 0; q < Hh; ++q) {
        float a = fmaf(W1[npar * Hh + q], e, b1[q]);
        for (int j = 0; j < npar; ++j) a = fmaf(W1[j * Hh + q], s_x[uni(s_prog + paroff + j) * B + t], a);
        for (int c = 0; c < ncf; ++c)
          a = fmaf(W1[(npar + 1 + c) * Hh + q],
                   rng_normal(k0, k1, (uint32_t)(row0 + n), (uint32_t)uni(s_prog + cfoff + c), step, RNG_CONF_NOISE),
                   a);
        out = fmaf(W2[q], fmaxf(a, 0.f), out);
      }
      s_x[var * B + t] = out;
    }
  }
  if (valid) {
    // generated sample out, plus its squared norm (program order) for the
    // matrix-core MMD's Gram-form distances
    float* xr = xhat + (size_t)r * D * N;
    float nrm = 0.f;
    for (int kk = 0; kk < nn; ++kk) {
      const int var = uni(s_prog + PROG_HDR + kk * NODE_REC);
      const float v = s_x[var * B + t];
      xr[(size_t)var * N + n] = v;
      nrm = fmaf(v, v, nrm);
    }
    if (xnorm) xnorm[(size_t)r * N + n] = nrm;
  }
}

// ============================================================================
// K2: generator backward.  grid = (G, R), block = BS = 128 samples (2 waves).
// LDS-resident per block: the samples' generated values s_x and running
// gradients s_dx ([Dt][BS], Dt = unpadded variable count).  Per node (reverse
// topological order):
//   compute  each thread rebuilds its sample's node inputs and pre-activations
//            (packed fp32), stores its input row s_in[s] = [x_0..x_{nin-1}, 1, g]
//            and mg[s][q] = g_s [pre_sq > 0] (the only per-unit value stored), and
//            pushes dL/dparent = W1 (W2 * mg) into s_dx.
//   reduce   one contraction over the block's samples gives everything:
//              Gm[j][q] = sum_s s_in[s][j] mg[s][q]           (j <= nin)
//              dW1|db1[j][q] = W2_q Gm[j][q]
//              dW2[q] = sum_s relu_sq g_s = sum_j W1ext[j][q] Gm[j][q]
//                       (relu = pre [pre > 0], pre = sum_j W1ext[j] s_in[j])
//              db2 = sum_s g_s
//            as "items" (row j, column pair): one v_pk_fma_f32 per two
//            parameters and sample.  With <= 64 items (the common case) each wave
//            takes half of the samples and hands its partial to wave 0 through LDS.
//            Fixed orders throughout: gpart[r][blk][param] is bitwise reproducible.
// Storing only mg (not dh and relu) keeps the footprint at ~300 B per sample, so
// four blocks fit per CU and the whole grid of a 256-model batch is resident at
// once.  Noise draws come from the forward's `noise` buffer, prefetched a node
// ahead; program words are wave-uniform scalar loads.
// ============================================================================
template <int H, int BS>
__global__ __launch_bounds__(BS) void gen_bwd_kernel(
    const int* __restrict__ prog, int prog_stride, const float* __restrict__ params, int P,
    const float* __restrict__ xhat, const float* __restrict__ noise, int NS,
    const float* __restrict__ grad_part, int n_chunks, int R,
    int N, int D, int Dt, int max_in, float* __restrict__ gpart) {
  static_assert(BS == 128, "two-wave reduction split assumes 128 samples per block");
  constexpr int HE = (H + 1) & ~1;       // mg rows padded to even width (pairs)
  constexpr int HP = HE / 2;             // column pairs per row
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int SI = (max_in + 2) | 1;       // odd stride: conflict-free per-thread row writes
  float* s_z = smem;                                   // [BS][HE]   mg rows (8-byte aligned)
  f2* s_red = reinterpret_cast<f2*>(s_z + BS * HE);    // [64]       wave-1 partials
  f2* s_g = s_red + 64;                                // [(max_in+1) * HP]  Gm pairs
  float* s_x = reinterpret_cast<float*>(s_g + (max_in + 1) * HP);   // [Dt][BS]
  float* s_dx = s_x + BS * Dt;                         // [Dt][BS]
  float* s_in = s_dx + BS * Dt;                        // [BS][SI]
  const int* s_prog = prog + (size_t)blockIdx.y * prog_stride;      // scalar (K$) reads

  const int r = blockIdx.y, blk = blockIdx.x, G = gridDim.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int n = blk * BS + t;
  const bool valid = n < N;
  const float* th = params + (size_t)r * P;
  const float* xr = xhat + (size_t)r * D * N;
  const float* nz = noise + (size_t)r * NS * N;
  float* gp = gpart + ((size_t)r * G + blk) * P;

  // sample state; dL/dxhat = fixed-order sum of the MMD column chunks (0 on padding rows)
  for (int v = 0; v < Dt; ++v) {
    float s = 0.f, x = 0.f;
    if (valid) {
      x = xr[(size_t)v * N + n];
      for (int c = 0; c < n_chunks; ++c) s += grad_part[(((size_t)c * R + r) * D + v) * N + n];
    }
    s_x[v * BS + t] = x;
    s_dx[v * BS + t] = s;
  }
  float* my_z = s_z + t * HE;
  float* my_in = s_in + t * SI;
  __syncthreads();
  const int nn = uni(s_prog);
  float e_cur = (nn > 0 && valid) ? nz[(size_t)uni(s_prog + PROG_HDR + (nn - 1) * NODE_REC) * N + n] : 0.f;

  for (int kk = nn - 1; kk >= 0; --kk) {
    const float e_next =
        (kk > 0 && valid) ? nz[(size_t)uni(s_prog + PROG_HDR + (kk - 1) * NODE_REC) * N + n] : 0.f;
    const int* nd = s_prog + PROG_HDR + kk * NODE_REC;
    if (uni(nd + 1) == KIND_OBS) { e_cur = e_next; continue; }
    const int var = uni(nd), npar = uni(nd + 2), paroff = uni(nd + 3), ncf = uni(nd + 4);
    const int cfoff = uni(nd + 5), poff = uni(nd + 6);
    const int nin = npar + 1 + ncf;
    const float* W1 = th + poff;
    const float* b1 = W1 + (size_t)nin * H;
    const float* W2 = b1 + H;

    // ---- compute phase (one sample per thread) ----
    const float gout = s_dx[var * BS + t];      // 0 on padding rows
    float pre[H];
#pragma unroll
    for (int q = 0; q < H; ++q) pre[q] = b1[q];
    for (int j = 0; j < nin; ++j) {
      float x;
      if (j < npar) x = s_x[uni(s_prog + paroff + j) * BS + t];
      else if (j == npar) x = e_cur;
      else x = valid ? nz[(size_t)(D + uni(s_prog + cfoff + (j - npar - 1))) * N + n] : 0.f;
      my_in[j] = x;
#pragma unroll
      for (int q = 0; q < H; ++q) pre[q] = fmaf(W1[j * H + q], x, pre[q]);
    }
    my_in[nin] = 1.f;
    my_in[nin + 1] = gout;
    float mg[HE];
#pragma unroll
    for (int q = 0; q < HE; ++q) mg[q] = (q < H && pre[q < H ? q : 0] > 0.f) ? gout : 0.f;
#pragma unroll
    for (int qp = 0; qp < HP; ++qp)
      *reinterpret_cast<f2*>(my_z + 2 * qp) = f2{mg[2 * qp], mg[2 * qp + 1]};
    for (int j = 0; j < npar; ++j) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < H; ++q) s = fmaf(W1[j * H + q] * W2[q], mg[q], s);
      s_dx[uni(s_prog + paroff + j) * BS + t] += s;
    }
    e_cur = e_next;
    __syncthreads();

    // ---- reduction phase ----
    const int n_w1 = (nin + 1) * HP;           // Gm items: rows 0..nin, column pairs
    const int n_items = n_w1 + 1;              // + db2 = sum_s g
    const bool split = n_items <= 64;          // each wave takes half of the samples
    auto item = [&](int it, int s_lo, int s_n) -> f2 {
      f2 acc0 = {0.f, 0.f}, acc1 = {0.f, 0.f};
      if (it < n_w1) {
        const int j = it / HP, qp = it - j * HP;
        const float* a = s_in + s_lo * SI + j;
        const float* zb = s_z + s_lo * HE + 2 * qp;
#pragma unroll 4
        for (int s2 = 0; s2 < s_n; s2 += 2) {
          const float a0 = a[s2 * SI], a1 = a[(s2 + 1) * SI];
          const f2 z0 = *reinterpret_cast<const f2*>(zb + s2 * HE);
          const f2 z1 = *reinterpret_cast<const f2*>(zb + (s2 + 1) * HE);
          acc0 = f2{a0, a0} * z0 + acc0;
          acc1 = f2{a1, a1} * z1 + acc1;
        }
      } else {
        const float* a = s_in + s_lo * SI + (nin + 1);
        for (int s2 = 0; s2 < s_n; s2 += 2) {
          acc0.x += a[s2 * SI];
          acc1.x += a[(s2 + 1) * SI];
        }
      }
      return acc0 + acc1;
    };
    // item -> outputs: dW1/db1 pair (scaled by W2) or db2; Gm pair kept in s_g
    auto emit = [&](int it, f2 acc) {
      if (it < n_w1) {
        const int j = it / HP, qp = it - j * HP, q = 2 * qp;
        s_g[it] = acc;
        gp[poff + j * H + q] = W2[q] * acc.x;
        if (q + 1 < H) gp[poff + j * H + q + 1] = W2[q + 1] * acc.y;
      } else {
        gp[poff + (nin + 1) * H + H] = acc.x;      // db2
      }
    };
    // dW2[q] = sum_j W1ext[j][q] Gm[j][q]  (W1ext row nin = b1), from s_g
    auto emit_w2 = [&](int q) {
      float s = 0.f;
      for (int j = 0; j <= nin; ++j) {
        const f2 gm = s_g[j * HP + (q >> 1)];
        s = fmaf(j < nin ? W1[j * H + q] : b1[q], (q & 1) ? gm.y : gm.x, s);
      }
      gp[poff + (nin + 1) * H + q] = s;
    };
    if (split) {
      f2 acc = {0.f, 0.f};
      if (lane < n_items) acc = item(lane, wave * 64, 64);
      if (wave == 1) s_red[lane] = acc;
      __syncthreads();
      if (wave == 0) {
        if (lane < n_items) emit(lane, acc + s_red[lane]);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   // s_g written by this wave
        __builtin_amdgcn_wave_barrier();
        if (lane < H) emit_w2(lane);
      }
    } else {
      for (int it = t; it < n_items; it += BS) emit(it, item(it, 0, BS));
      __syncthreads();
      if (t < H) emit_w2(t);
    }
    __syncthreads();
  }
}

// ============================================================================
// K5: TF1 Adam with fused fixed-order reduction of the G gradient slabs.
//   lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t);  theta -= lr_t * m / (sqrt(v) + eps)
// grid = (ceil(P/1024), R): four consecutive parameters per thread (P % 4 == 0,
// pack_programs), the slabs read as 16-B loads, eight in flight per thread (the round-5
// form -- one parameter per thread, one dependent load per slab -- ran at ~1 TB/s:
// 88 us per step on the 200-variable orientation slice).  Per parameter the same adds in
// the same order: bitwise the same update.
// ============================================================================
__global__ __launch_bounds__(256) void adam_tf1_kernel(
    float* __restrict__ params, float* __restrict__ m, float* __restrict__ v,
    const float* __restrict__ gpart, int G, const int* __restrict__ prog, int prog_stride, int P,
    const int* __restrict__ step_base, int step_off, float lr, float beta1, float beta2, float eps) {
  // no contraction: the float4 form otherwise fuses the moment updates into (packed)
  // FMAs the scalar round-5 kernel did not have, and the trajectories drift apart
  // (pinned example predictions, tests/test_examples_gpu.py)
#pragma clang fp contract(off)
  const int r = blockIdx.y;
  const int p0 = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
  const int Pr = prog[(size_t)r * prog_stride + 1];
  if (p0 >= Pr) return;
  const float4* gp = reinterpret_cast<const float4*>(gpart + (size_t)r * G * P + p0);
  const int P4 = P >> 2;
  float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
  for (int k = 0; k < G; ++k) {
    const float4 x = gp[(size_t)k * P4];
    g.x += x.x;
    g.y += x.y;
    g.z += x.z;
    g.w += x.w;
  }
  const float tstep = (float)(step_base[1] + step_off + 1);   // optimizer step count
  const float lr_t = lr * sqrtf(1.f - powf(beta2, tstep)) / (1.f - powf(beta1, tstep));
  const size_t idx = (size_t)r * P + p0;
  const float4 m0 = *reinterpret_cast<const float4*>(m + idx), v0 = *reinterpret_cast<const float4*>(v + idx);
  const float4 t0 = *reinterpret_cast<const float4*>(params + idx);
  const float gg[4] = {g.x, g.y, g.z, g.w}, mo[4] = {m0.x, m0.y, m0.z, m0.w}, vo[4] = {v0.x, v0.y, v0.z, v0.w};
  float to[4] = {t0.x, t0.y, t0.z, t0.w}, mn[4], vn[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    mn[q] = beta1 * mo[q] + (1.f - beta1) * gg[q];
    vn[q] = beta2 * vo[q] + (1.f - beta2) * gg[q] * gg[q];
    if (p0 + q < Pr) {
      to[q] -= lr_t * mn[q] / (sqrtf(vn[q]) + eps);
    } else {                                  // padding parameters stay untouched
      mn[q] = mo[q];
      vn[q] = vo[q];
    }
  }
  *reinterpret_cast<float4*>(m + idx) = make_float4(mn[0], mn[1], mn[2], mn[3]);
  *reinterpret_cast<float4*>(v + idx) = make_float4(vn[0], vn[1], vn[2], vn[3]);
  *reinterpret_cast<float4*>(params + idx) = make_float4(to[0], to[1], to[2], to[3]);
}

// Parameter init N(0, std^2) from Philox (weights AND biases, CGNN.py:71-74).
__global__ void init_params_kernel(float* __restrict__ params, float* __restrict__ m,
                                   float* __restrict__ v, const int* __restrict__ prog,
                                   int prog_stride, int P, const uint32_t* __restrict__ keys,
                                   float init_std) {
  const int r = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const int Pr = prog[(size_t)r * prog_stride + 1];
  const size_t idx = (size_t)r * P + p;
  params[idx] = p < Pr ? init_std * rng_normal(keys[2 * r], keys[2 * r + 1], (uint32_t)p, 0u, 0u,
                                               RNG_PARAM_INIT)
                       : 0.f;
  m[idx] = 0.f;
  v[idx] = 0.f;
}

// step_base[0]: RNG step (advances every train AND eval step);
// step_base[1]: optimizer step (advances on train steps only).
__global__ void advance_step_kernel(int* step_base, int d_rng, int d_opt) {
  step_base[0] += d_rng;
  step_base[1] += d_opt;
}

// ============================================================================
// host-side launchers (C ABI, called from the pybind11 module)
// ============================================================================
#define CGNN_CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return (int)e_; } while (0)

template <int D>
static int launch_mmd_d(int mode, const float* xhat, const float* data, float* gpart, float* lpart,
                        int row_begin, int n_rows, int N, int R, int row_tiles, int n_chunks, int tpc, float gscale,
                        int mirror, hipStream_t st) {
  dim3 grid(row_tiles, n_chunks, R), block(256);
#define MMD_ARGS xhat, data, gpart, lpart, N, R, tpc, gscale, row_begin, n_rows, mirror
  if (mode == 0) hipLaunchKernelGGL((mmd_rbf_kernel<D, 0>), grid, block, 0, st, MMD_ARGS);
  else if (mode == 3) hipLaunchKernelGGL((mmd_rbf_kernel<D, 3>), grid, block, 0, st, MMD_ARGS);
  else if (mode == 1) hipLaunchKernelGGL((mmd_rbf_kernel<D, 1>), grid, block, 0, st, MMD_ARGS);
  else hipLaunchKernelGGL((mmd_rbf_kernel<D, 2>), grid, block, 0, st, MMD_ARGS);
#undef MMD_ARGS
  return (int)hipGetLastError();
}

extern "C" int cgnn_mmd_supported_d(int D) {
  switch (D) { case 1: case 2: case 3: case 4: case 6: case 8: case 12: case 16: case 20: case 24:
    case 32: case 48: case 64: return 1; default: return 0; }
}

// extra gradient slots (after the n_chunks column chunks) a symmetric training launch
// of the vector kernel writes over all N rows: row_tiles - 1 for D <= MMD_SYM_MAX_D, else 0
extern "C" int cgnn_mmd_mirror_slots(int D, int N) {
  if (!cgnn_mmd_supported_d(D) || D > MMD_SYM_MAX_D || N < 1) return 0;
  return (N + 255) / 256 - 1;
}

// row_begin / n_rows: the rows (generated samples) this launch evaluates; (0, N)
// for the whole set.  row_tiles must cover n_rows.  mirror: symmetric training over all
// rows -- grad_part then holds n_chunks + cgnn_mmd_mirror_slots(D, N) slots.
extern "C" int cgnn_launch_mmd_rows(int mode, int D, const float* xhat, const float* data, float* gpart,
                                    float* lpart, int N, int R, int row_tiles, int n_chunks, int tpc,
                                    float gscale, int row_begin, int n_rows, hipStream_t st, int mirror) {
  if (row_begin < 0 || n_rows < 1 || row_begin + n_rows > N || (long)row_tiles * 256 < n_rows) return -2;
  if (mirror && ((mode != 0 && mode != 3) || row_begin != 0 || n_rows != N || cgnn_mmd_mirror_slots(D, N) == 0 ||
                 row_tiles != (N + 255) / 256))
    return -2;
  switch (D) {
#define CASE_D(d) case d: return launch_mmd_d<d>(mode, xhat, data, gpart, lpart, row_begin, n_rows, N, R, row_tiles, n_chunks, tpc, gscale, mirror, st);
    CASE_D(1) CASE_D(2) CASE_D(3) CASE_D(4) CASE_D(6) CASE_D(8) CASE_D(12) CASE_D(16) CASE_D(20)
    CASE_D(24) CASE_D(32) CASE_D(48) CASE_D(64)
#undef CASE_D
    default: return -1;
  }
}

extern "C" int cgnn_launch_mmd(int mode, int D, const float* xhat, const float* data, float* gpart,
                               float* lpart, int N, int R, int row_tiles, int n_chunks, int tpc,
                               float gscale, hipStream_t st, int mirror) {
  return cgnn_launch_mmd_rows(mode, D, xhat, data, gpart, lpart, N, R, row_tiles, n_chunks, tpc, gscale, 0, N, st,
                              mirror);
}

extern "C" int cgnn_launch_loss_finalize(const float* lpart, int n_parts, float* tt, float* last,
                                         float* acc, float inv_n2, int flags, float* hist,
                                         int hist_stride, const int* step_base, int step_off,
                                         int R, hipStream_t st) {
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(R), dim3(256), 0, st, lpart, n_parts, tt, last, acc,
                     inv_n2, flags, hist, hist_stride, step_base, step_off);
  return (int)hipGetLastError();
}

#define CGNN_H_LIST(X) X(1) X(2) X(3) X(4) X(5) X(6) X(8) X(10) X(12) X(16) X(20) X(24) X(30) X(32) \
  X(40) X(48) X(50) X(64)

// kernels whose dynamic LDS exceeds the default 64 KiB window must opt in
template <typename K>
static void allow_lds(K kernel, size_t lds) {
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

extern "C" int cgnn_gen_supported_h(int H) {
  switch (H) {
#define CASE_H(h) case h: return 1;
    CGNN_H_LIST(CASE_H)
#undef CASE_H
    default: return 0;
  }
}

// Samples per block of the generator forward: the widest of 256 / 128 / 64 whose
// LDS sample state [D][B] stays within 64 KiB (D = 256 variables -> 64 samples), so
// wide causal graphs keep several blocks per CU.  Every draw and sum is per sample,
// so the block size never changes a result.
static int gen_fwd_block(int D) {
  int B = 256;
  while (B > 64 && (size_t)D * B * sizeof(float) > 64 * 1024) B >>= 1;
  return B;
}

// LDS bytes of the generator forward of D (padded) variables with a program stride of
// prog_stride ints: the [D][B] sample state plus the block's program copy
extern "C" size_t cgnn_gen_fwd_lds(int D, int prog_stride) {
  return sizeof(float) * (size_t)D * gen_fwd_block(D) + sizeof(int) * (size_t)prog_stride;
}

extern "C" int cgnn_launch_gen_fwd(const int* prog, int prog_stride, const float* params, int P,
                                   const float* data, float* xhat, float* noise, int NS, float* xnorm,
                                   const uint32_t* keys, const int* step_base, int step_off, int N,
                                   int D, int H, int R, hipStream_t st, int row0) {
  const int B = gen_fwd_block(D);
  dim3 grid((N + B - 1) / B, R), block(B);
  const size_t lds = cgnn_gen_fwd_lds(D, prog_stride);
  if (lds > 160 * 1024) return -2;
  switch (H) {
#define CASE_H(h) case h: allow_lds(gen_fwd_kernel<h>, lds); hipLaunchKernelGGL((gen_fwd_kernel<h>), grid, block, lds, st, prog, prog_stride, params, P, data, xhat, noise, NS, xnorm, keys, step_base, step_off, N, D, H, row0); break;
    CGNN_H_LIST(CASE_H)
#undef CASE_H
    default:
      allow_lds(gen_fwd_kernel<0>, lds);
      hipLaunchKernelGGL((gen_fwd_kernel<0>), grid, block, lds, st, prog, prog_stride, params, P, data,
                         xhat, noise, NS, xnorm, keys, step_base, step_off, N, D, H, row0);
  }
  return (int)hipGetLastError();
}

constexpr int GEN_BWD_BS = 128;

extern "C" int cgnn_gen_bwd_blocks(int N) { return (N + GEN_BWD_BS - 1) / GEN_BWD_BS; }

// D here is the unpadded variable count (the LDS arrays hold only real variables)
extern "C" size_t cgnn_gen_bwd_lds(int H, int max_in, int D, int prog_stride) {
  const size_t HE = (size_t)((H + 1) & ~1);
  (void)prog_stride;
  return sizeof(float) * ((size_t)GEN_BWD_BS * (HE + ((max_in + 2) | 1) + 2 * (size_t)D) + 128 +
                          (size_t)(max_in + 1) * HE);
}

extern "C" int cgnn_staged_plan(int, int, int, int, int, int*);

// 1: the specialised per-sample kernel (compiled H, LDS sample state fits), 2: the
// level-scheduled kernels of cgnn_staged.hip, 0: neither fits (the caller trains this
// batch elsewhere).  The choice depends only on the arguments: the scorer evaluates it
// per program and batches programs of one family together (engine/scorer.py), so a
// model's kernels -- and its score -- do not depend on its batch-mates.
// The per-sample kernels walk the whole program in one wave, the level-scheduled ones
// share a level's nodes over W waves: above GEN_PER_SAMPLE_MAX_D variables the latter
// win.  R = 256, N = 500, H = 20, train step us, per-sample vs level-scheduled, after the
// round-5 backward changes: d = 22 326 vs 348, d = 24 375 vs 395, d = 26 520 vs 425,
// d = 28 496 vs 377 (profiles/r05_family/after_bwd; before them the crossover was
// between 28 and 30).
constexpr int GEN_PER_SAMPLE_MAX_D = 24;
extern "C" int cgnn_gen_bwd_variant(int H, int max_in, int Dt, int prog_stride) {
  const bool per_sample = cgnn_gen_supported_h(H) && cgnn_gen_bwd_lds(H, max_in, Dt, prog_stride) <= 160 * 1024;
  int plan[5];
  const bool staged = cgnn_staged_plan(Dt, H, max_in, 8, 0, plan) == 0;
  if (per_sample && (Dt <= GEN_PER_SAMPLE_MAX_D || !staged)) return 1;
  return staged ? 2 : 0;
}

// whether the level-scheduled kernels cover (Dt, H, max_in) at all (a forced staged batch)
extern "C" int cgnn_gen_staged_supported(int H, int max_in, int Dt) {
  int plan[5];
  return cgnn_staged_plan(Dt, H, max_in, 8, 0, plan) == 0;
}

// the per-sample backward (variant 1); variant 2 batches launch cgnn_launch_gen_bwd_staged
extern "C" int cgnn_launch_gen_bwd(const int* prog, int prog_stride, const float* params, int P,
                                   const float* xhat, const float* noise, int NS, const float* gradp,
                                   int n_chunks, int R, int N, int D, int Dt, int H, int max_in,
                                   float* gpart, hipStream_t st) {
  const int G = cgnn_gen_bwd_blocks(N);
  dim3 grid(G, R), block(GEN_BWD_BS);
  if (!cgnn_gen_supported_h(H)) return -1;
  const size_t lds = cgnn_gen_bwd_lds(H, max_in, Dt, prog_stride);
  if (lds > 160 * 1024) return -2;
  switch (H) {
#define CASE_H(h) case h: allow_lds(gen_bwd_kernel<h, GEN_BWD_BS>, lds); hipLaunchKernelGGL((gen_bwd_kernel<h, GEN_BWD_BS>), grid, block, lds, st, prog, prog_stride, params, P, xhat, noise, NS, gradp, n_chunks, R, N, D, Dt, max_in, gpart); break;
    CGNN_H_LIST(CASE_H)
#undef CASE_H
    default: return -1;
  }
  return (int)hipGetLastError();
}

extern "C" int cgnn_launch_adam(float* params, float* m, float* v, const float* gpart, int G,
                                const int* prog, int prog_stride, int P, const int* step_base,
                                int step_off, float lr, float b1, float b2, float eps, int R,
                                hipStream_t st) {
  if (P % 4) return -3;                       // pack_programs pads P to whole float4s
  dim3 grid((P + 1023) / 1024, R), block(256);
  hipLaunchKernelGGL(adam_tf1_kernel, grid, block, 0, st, params, m, v, gpart, G, prog, prog_stride,
                     P, step_base, step_off, lr, b1, b2, eps);
  return (int)hipGetLastError();
}

extern "C" int cgnn_launch_init(float* params, float* m, float* v, const int* prog, int prog_stride,
                                int P, const uint32_t* keys, float init_std, int R, hipStream_t st) {
  dim3 grid((P + 255) / 256, R), block(256);
  hipLaunchKernelGGL(init_params_kernel, grid, block, 0, st, params, m, v, prog, prog_stride, P, keys,
                     init_std);
  return (int)hipGetLastError();
}

extern "C" int cgnn_launch_advance(int* step_base, int d_rng, int d_opt, hipStream_t st) {
  hipLaunchKernelGGL(advance_step_kernel, dim3(1), dim3(1), 0, st, step_base, d_rng, d_opt);
  return (int)hipGetLastError();
}
