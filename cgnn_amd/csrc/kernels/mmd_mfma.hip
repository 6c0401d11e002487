// Matrix-core MMD for wide joints (D >= 8).  Both products of the fused MMD
// run on v_mfma_f32_32x32x16_f16 with a three-pass hi/lo split of every f32
// operand (x = hi + lo, both f16; hi*hi + hi*lo + lo*hi, ~22-bit operands, f32
// accumulation), 16x the f32-MFMA rate; the seven-bandwidth exponential
// epilogue runs on the vector ALUs (packed f32) and co-issues with the matrix
// cores of the other waves.  Same outputs and partial layout as the vector
// kernel (cgnn_kernels.hip, mmd_rbf_kernel); the squared distance is taken in
// the Gram form |x|^2 + |z|^2 - 2 x.z that the reference computes
// (Loss.py:17-19).
//
// Orientation (one wave = 32 generated rows i; the block's 4 waves share a
// 32-column tile j of the joint [pred; true] staged in LDS):
//   C'[j][i] = sum_d Z[j][d] X[i][d]      A = Z tile (LDS, [j][d]), B = X rows
//                                         (registers, split once)
//   -> lane l owns row i = l&31; accumulator r holds column
//      j(r, h) = (r&3) + 8(r>>2) + 4h (h = l>>5).
//   W[i][j] = s_j * sum_g g exp(-g d2_ij)  (s_j = +1 pred column, -1 true column)
//   G[i][d] += sum_j W[i][j] Z[j][d]       A = W: accumulator registers 8s..8s+7
//      are k-step s (element e <-> j = 16s + 8(e>>2) + 4h + (e&3)), B = Z read
//      from the transposed LDS image [d][j] at those j -- no lane movement.
//   dL/dp_i = 4/N^2 (G_i - p_i sum_j W_ij)
#include "cgnn_common.h"

using namespace cgnn;

namespace {

typedef float f16v __attribute__((ext_vector_type(16)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

constexpr int MT = 32;          // tile edge (rows per wave, columns per tile)
constexpr int WAVES = 4;        // rows per block = 128

// seven bandwidths for two distances, each kernel value folded into the sum
// (ks) and the weighted sum (w) as soon as it exists (values: rbf7_values).
__device__ __forceinline__ void rbf7x2_chain(f2 d2, f2& ks, f2& w) {
  f2 e[7];
  rbf7_values(d2, e);
  ks = e[0];
  w = e[0] * 0.005f;
  ks += e[1];
  w = e[1] * 0.05f + w;
  ks += e[2];
  w = e[2] * 0.25f + w;
  ks += e[3];
  w = e[3] * 0.5f + w;
  ks += e[4];
  w += e[4];
  ks += e[5];
  w = e[5] * 5.0f + w;
  ks += e[6];
  w = e[6] * 50.0f + w;
}

__device__ __forceinline__ void split16(float x, _Float16& hi, _Float16& lo) {
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}

__device__ __forceinline__ h8 cat(h4 a, h4 b) {
  return h8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

__device__ __forceinline__ f16v mma(h8 a, h8 b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <int KD, int MODE>
__global__ __launch_bounds__(256) void mmd_mfma_kernel(
    const float* __restrict__ xhat, const float* __restrict__ data,
    const float* __restrict__ xnorm, const float* __restrict__ ynorm,
    float* __restrict__ grad_part, float* __restrict__ loss_part,
    int N, int R, int tiles_per_chunk, float grad_scale, int row_begin, int n_rows) {
  // rows: generated samples [row_begin, row_begin + n_rows) (a sample-sharded
  // MMD owns a row range, columns are all N); gradient rows use stride n_rows.
  // MODE 0 train (loss + gradient), 1 eval (loss), 3 train without the loss
  // (nobody reads the training loss unless a history is recorded), 2 the constant
  // true-true block (launched with xhat = data, xnorm = ynorm: the first column part
  // only; used for the widths the vector kernel does not cover)
  constexpr bool GRAD = MODE == 0 || MODE == 3;
  constexpr bool LOSS = MODE != 3;
  constexpr int KP = (KD + 15) / 16 * 16;   // distance K padded to the MFMA k-step
  constexpr int KS = KP / 16;
  constexpr int NT = (KD + 31) / 32;        // 32-wide output tiles of the gradient
  constexpr int ZS = KP + 8;                // [j][d] image row stride (halfs): conflict-free b128
  constexpr int ZT = MT + 4;                // [d][j] image row stride (halfs): conflict-free b64
  constexpr int ZIMG = MT * ZS, TIMG = NT * 32 * ZT;
  __shared__ __attribute__((aligned(16))) _Float16 s_zh[2][ZIMG];
  __shared__ __attribute__((aligned(16))) _Float16 s_zl[2][ZIMG];
  __shared__ __attribute__((aligned(16))) _Float16 s_th[2][TIMG];
  __shared__ __attribute__((aligned(16))) _Float16 s_tl[2][TIMG];
  __shared__ __attribute__((aligned(16))) float s_n[2][MT];
  __shared__ float s_red[WAVES];

  const int rb = blockIdx.x, chunk = blockIdx.y, r = blockIdx.z;
  const int n_chunks = gridDim.y, n_rb = gridDim.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int i = row_begin + rb * (WAVES * MT) + wave * MT + li;
  const bool row_ok = i - row_begin < n_rows;
  const size_t mbase = (size_t)r * KD * N;
  const float* X = xhat + mbase;
  const float* Y = data + mbase;

  // this lane's B fragments of its row (dims 16s + 8h + e), split once; row norm
  h8 xbh[KS], xbl[KS];
  const float* XN = xnorm + (size_t)r * N;
  const float* YN = ynorm + (size_t)r * N;
  const float nx = row_ok ? XN[i] : 0.f;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int d = 16 * s + 8 * h + e;
      const float v = (row_ok && d < KD) ? X[d * N + i] : 0.f;
      _Float16 hi, lo;
      split16(v, hi, lo);
      xbh[s][e] = hi;
      xbl[s][e] = lo;
    }
  }

  const int TX = (N + MT - 1) / MT;         // column tiles per part
  const int ct = MODE == 2 ? TX : 2 * TX;
  // evaluation over all rows: the pred-pred block is symmetric -- column tiles left of
  // this block's rows are skipped, the wave's own diagonal tile counts once, tiles
  // right of it twice (and tiles left of the wave inside the block's band not at all):
  // ~25 % fewer distances per evaluation step, geometry still fixed by N
  const bool sym = (MODE == 1 || MODE == 2) && row_begin == 0 && n_rows == N;
  const int wr = rb * WAVES + wave;         // this wave's row tile (in MT columns)
  int t_begin = chunk * tiles_per_chunk;
  const int t_end = min(ct, t_begin + tiles_per_chunk);
  if (sym && t_begin < TX) t_begin = max(t_begin, min(rb * WAVES, TX));

  // zero both buffers once: padded dims / rows are never written afterwards
  for (int e = t; e < 2 * ZIMG; e += 256) { (&s_zh[0][0])[e] = (_Float16)0.f; (&s_zl[0][0])[e] = (_Float16)0.f; }
  for (int e = t; e < 2 * TIMG; e += 256) { (&s_th[0][0])[e] = (_Float16)0.f; (&s_tl[0][0])[e] = (_Float16)0.f; }
  __syncthreads();

  constexpr int LR = (MT * KD + 255) / 256;
  // staging registers: LR tile elements + (threads 0..31) the column norm
  auto load_tile = [&](int tile, float* regs) {
    const float* src = tile < TX ? X : Y;
    const int c0 = (tile < TX ? tile : tile - TX) * MT;
    regs[LR] = (t < MT && c0 + t < N) ? (tile < TX ? XN : YN)[c0 + t] : 0.f;
#pragma unroll
    for (int k = 0; k < LR; ++k) {
      const int e = t + 256 * k;
      const int d = e >> 5, jj = e & 31;
      regs[k] = (e < MT * KD && c0 + jj < N) ? src[d * N + c0 + jj] : 0.f;
    }
  };
  auto store_tile = [&](int buf, const float* regs) {
    if (t < MT) s_n[buf][t] = regs[LR];
#pragma unroll
    for (int k = 0; k < LR; ++k) {
      const int e = t + 256 * k;
      const int d = e >> 5, jj = e & 31;
      if (e < MT * KD) {
        _Float16 hi, lo;
        split16(regs[k], hi, lo);
        s_zh[buf][jj * ZS + d] = hi;
        s_zl[buf][jj * ZS + d] = lo;
        s_th[buf][d * ZT + jj] = hi;
        s_tl[buf][d * ZT + jj] = lo;
      }
    }
  };
  float stage[LR + 1];
  if (t_begin < t_end) {
    load_tile(t_begin, stage);
    store_tile(0, stage);
    if (t_begin + 1 < t_end) {
      load_tile(t_begin + 1, stage);
      store_tile(1, stage);
    }
  }
  __syncthreads();

  f16v acc_g[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q) acc_g[q] = f16v{};
  float rowsum = 0.f, lacc = 0.f;

  for (int tile = t_begin; tile < t_end; ++tile) {
    const int buf = (tile - t_begin) & 1;
    const bool pred_part = tile < TX;
    const int c0 = (pred_part ? tile : tile - TX) * MT;
    const bool more = tile + 2 < t_end;
    if (more) load_tile(tile + 2, stage);          // prefetch while this tile computes

    // ---- distance Gram C'[j][i], three passes per k-step ----
    f16v c = f16v{};
    const _Float16* zr = &s_zh[buf][li * ZS + 8 * h];
    const _Float16* zl = &s_zl[buf][li * ZS + 8 * h];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const h8 ah = *reinterpret_cast<const h8*>(zr + 16 * s);
      const h8 al = *reinterpret_cast<const h8*>(zl + 16 * s);
      c = mma(ah, xbh[s], c);
      c = mma(ah, xbl[s], c);
      c = mma(al, xbh[s], c);
    }

    // ---- epilogue (packed pairs of accumulator registers): kernel sum for the
    // loss and, when training, the signed weights W written over c in place ----
    f2 tl2 = {0.f, 0.f};
    f2 rs2 = {0.f, 0.f};
    const float sg = pred_part ? 1.f : -1.f;
    // columns j >= N - c0 are padding (only the last tile of each part): d2 -> huge
    const int jlim = N - c0 - 4 * h;               // compare j - 4h against it
    const bool ragged = N - c0 < MT;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const float4 nz4 = *reinterpret_cast<const float4*>(&s_n[buf][8 * g4 + 4 * h]);
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        const int rg = 4 * g4 + 2 * qq;
        const f2 nzp = qq ? f2{nz4.z, nz4.w} : f2{nz4.x, nz4.y};
        const f2 cc = {c[rg], c[rg + 1]};
        f2 d2 = cc * -2.f + (nzp + nx);    // Gram form, unclamped like the reference
        if (ragged) {
          const int jr = 2 * qq + 8 * g4;
          d2.x = jr < jlim ? d2.x : 1.0e30f;
          d2.y = jr + 1 < jlim ? d2.y : 1.0e30f;
        }
        f2 ks, w;
        if (GRAD) rbf7x2_chain(d2, ks, w);
        else rbf7x2(d2, ks, w);
        if (LOSS) tl2 += ks;
        if (GRAD) {
          w *= sg;
          rs2 += w;
          c[rg] = w.x;
          c[rg + 1] = w.y;
        }
      }
    }
    if (LOSS) {
      const float wgt = !pred_part ? -2.f : !sym ? 1.f : tile < wr ? 0.f : tile == wr ? 1.f : 2.f;
      lacc = fmaf(wgt, tl2.x + tl2.y, lacc);
    }

    if (GRAD) {
      rowsum += rs2.x + rs2.y;
      // ---- gradient product G[i][d] += sum_j W[i][j] Z[j][d] ----
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        h8 wh, wl;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          _Float16 hi, lo;
          split16(c[8 * s + e], hi, lo);
          wh[e] = hi;
          wl[e] = lo;
        }
#pragma unroll
        for (int q = 0; q < NT; ++q) {
          const _Float16* th = &s_th[buf][(32 * q + li) * ZT + 16 * s + 4 * h];
          const _Float16* tl = &s_tl[buf][(32 * q + li) * ZT + 16 * s + 4 * h];
          const h8 bh = cat(*reinterpret_cast<const h4*>(th), *reinterpret_cast<const h4*>(th + 8));
          const h8 bl = cat(*reinterpret_cast<const h4*>(tl), *reinterpret_cast<const h4*>(tl + 8));
          acc_g[q] = mma(wh, bh, acc_g[q]);
          acc_g[q] = mma(wh, bl, acc_g[q]);
          acc_g[q] = mma(wl, bh, acc_g[q]);
        }
      }
    }
    __syncthreads();                     // everyone is done with buffer `buf`
    if (more) store_tile(buf, stage);
    __syncthreads();
  }

  // ---- loss partial: fixed-order wave then block reduction ----
  float v = row_ok ? lacc : 0.f;
  v = wave_sum(v);
  if (lane == 0) s_red[wave] = v;
  __syncthreads();
  if (t == 0) {
    const float sum = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
    loss_part[((size_t)r * n_chunks + chunk) * n_rb + rb] = sum;
  }

  if (GRAD) {
    // sum_j W_ij: the two lane halves hold disjoint column sets of row i = l&31
    rowsum += __shfl_xor(rowsum, 32);
    float* gp = grad_part + ((size_t)chunk * R + r) * KD * n_rows;
    const int i0 = rb * (WAVES * MT) + wave * MT;           // local row
#pragma unroll
    for (int rg = 0; rg < 16; ++rg) {
      const int il = (rg & 3) + 8 * (rg >> 2) + 4 * h;   // accumulator row -> local row
      const float rs = __shfl(rowsum, il);
      const int ii = i0 + il;
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        const int d = 32 * q + li;
        if (d < KD && ii < n_rows) {
          const float p = X[d * N + row_begin + ii];
          gp[d * n_rows + ii] = (acc_g[q][rg] - p * rs) * grad_scale;
        }
      }
    }
  }
}

// ============================================================================
// Wide joints (KD >= 128): 16 generated rows per wave on v_mfma_f32_16x16x32_f16.
// The 32-row kernel above keeps KD/16 x 16 x-fragment registers and KD/32 x 16
// gradient accumulators per wave (224 + 112 at KD = 224) and a second, transposed
// copy of every column tile in LDS (123 KB at KD = 224): one wave per SIMD.  Here
// a wave holds 16 rows (x fragments KD/32 x 8 regs, accumulators KD/16 x 4), and the
// column tile is staged ONCE, row-major [j][d] (hi and lo f16 images), row j skewed
// by 2 (j & 7) 16-B chunks in a row of a whole number of 256-B bank rows, so that both
// reads are conflict-free and every address is a per-lane base plus an immediate: the
// Gram's A fragments by ds_read_b128 along d, the gradient's B fragments by
// ds_read_b64_tr_b16 along j.
//   C'[j][i] = sum_d Z[j][d] X[i][d]    two 16-column halves, A = Z (LDS), B = X
//      -> lane l: row i = l&15, columns j = 16 h + 4(l>>4) + v (half h, v = 0..3)
//   G[i][d] += sum_j W[i][j] Z[j][d]    A = the lane's own 8 W values (k-slot e <->
//      j = 4g + e for e < 4, 16 + 4g + e - 4 after; g = l>>4), B = Z^T through
//      the transposed reads of rows 4g..4g+3 and 16+4g..16+4g+3.
// Evaluation (loss only) skips the pred-pred tiles left of a row block's diagonal and
// counts those right of it twice; training evaluates the whole pred-pred block (the
// mirrored gradient would need a second, column-side accumulation).
// ============================================================================
typedef float f4v __attribute__((ext_vector_type(4)));
typedef short s4v __attribute__((ext_vector_type(4)));

constexpr int W16 = 8;          // waves per block (rows per block = 128, as the 32-row kernel)

__device__ __forceinline__ f4v mma16(h8 a, h8 b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// half offset of (row j, chunk c of 8 halfs) in a [32][ZS] image: skew 2 (j & 7) chunks
constexpr int MMD_MAX_D = 16384;

template <int ZS>
__device__ __forceinline__ int zoff(int j, int c) { return j * ZS + 8 * (c + 2 * (j & 7)); }

template <int KD, int MODE>
__global__ __launch_bounds__(512) void mmd_mfma16_kernel(
    const float* __restrict__ xhat, const float* __restrict__ data,
    const float* __restrict__ xnorm, const float* __restrict__ ynorm,
    float* __restrict__ grad_part, float* __restrict__ loss_part,
    int N, int R, int tiles_per_chunk, float grad_scale, int row_begin, int n_rows) {
  constexpr bool GRAD = MODE == 0 || MODE == 3;
  constexpr bool LOSS = MODE != 3;
  constexpr int KP = (KD + 31) / 32 * 32;   // k padded to the MFMA k-step (32)
  constexpr int KS = KP / 32;
  constexpr int NT = (KD + 15) / 16;        // 16-wide gradient tiles
  constexpr int ZS = (KP + 14 * 8 + 127) / 128 * 128;  // row (halfs): skew room, whole 256-B rows
  static_assert(KP <= 256, "wide MMD covers KD <= 256 per launch");
  constexpr int NCH = KP / 8;               // 16-B chunks per staged row
  constexpr int TASKS = MT * NCH;           // (row, chunk) staging tasks per tile
  constexpr int TPT = (TASKS + 511) / 512;  // per thread
  __shared__ __attribute__((aligned(16))) _Float16 s_zh[2][MT * ZS];
  __shared__ __attribute__((aligned(16))) _Float16 s_zl[2][MT * ZS];
  __shared__ __attribute__((aligned(16))) float s_n[2][MT];
  __shared__ float s_red[W16];

  // a model's (row block, chunk) blocks rotated by the model index: blocks are dealt
  // round-robin over the 8 XCDs, and with 4 row blocks x 2 chunks the unrotated grid put
  // every model's chunk 0 on XCDs 0-3 and chunk 1 on 4-7 -- so blocks of unequal length
  // (the symmetric evaluation below) left half the chip idle at the end
  const int n_chunks = gridDim.y, n_rb = gridDim.x, r = blockIdx.z;
  const int lid = (int)((blockIdx.x + gridDim.x * blockIdx.y + blockIdx.z) % (gridDim.x * gridDim.y));
  const int rb = lid % n_rb, chunk = lid / n_rb;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int i = row_begin + rb * (W16 * 16) + wave * 16 + li;
  const bool row_ok = i - row_begin < n_rows;
  const size_t mbase = (size_t)r * KD * N;
  const float* X = xhat + mbase;
  const float* Y = data + mbase;
  const float* XN = xnorm + (size_t)r * N;
  const float* YN = ynorm + (size_t)r * N;
  const float nx = row_ok ? XN[i] : 0.f;

  // this lane's B fragments of row i: dims 32 s + 8 g + e, split once
  h8 xbh[KS], xbl[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int d = 32 * s + 8 * g + e;
      const float v = (row_ok && d < KD) ? X[(size_t)d * N + i] : 0.f;
      _Float16 hi, lo;
      split16(v, hi, lo);
      xbh[s][e] = hi;
      xbl[s][e] = lo;
    }
  }

  const int TX = (N + MT - 1) / MT;
  const int ct = MODE == 2 ? TX : 2 * TX;
  int t_begin = chunk * tiles_per_chunk;
  const int t_end = min(ct, t_begin + tiles_per_chunk);
  // symmetric pred-pred block (loss only, all rows in this launch, a chunk of pred tiles
  // only): the row block starts at its own diagonal tile; tiles right of its 128 x 128
  // diagonal block count twice (each stands for its mirror, left of another block's
  // diagonal), the diagonal block once
  constexpr int RBT = W16 * 16 / MT;        // column tiles per row block
  // (every chunk either all pred or all true tiles, so every skipped tile's mirror is
  // counted by a symmetric block)
  const bool sym = (MODE == 1 || MODE == 2) && row_begin == 0 && n_rows == N && t_end <= TX &&
                   (MODE == 2 || TX % tiles_per_chunk == 0);
  if (sym) t_begin = max(t_begin, RBT * rb);

  // staging: task k -> (column jj = task & 31, chunk c = task >> 5): 8 consecutive dims
  float stage[TPT][8];
  float stage_n = 0.f;
  auto load_tile = [&](int tile) {
    const float* src = tile < TX ? X : Y;
    const int c0 = (tile < TX ? tile : tile - TX) * MT;
    stage_n = (t < MT && c0 + t < N) ? (tile < TX ? XN : YN)[c0 + t] : 0.f;
#pragma unroll
    for (int k = 0; k < TPT; ++k) {
      const int task = t + 512 * k;
      const int jj = task & 31, c = task >> 5;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int d = 8 * c + e;
        stage[k][e] = (task < TASKS && d < KD && c0 + jj < N) ? src[(size_t)d * N + c0 + jj] : 0.f;
      }
    }
  };
  auto store_tile = [&](int buf) {
    if (t < MT) s_n[buf][t] = stage_n;
#pragma unroll
    for (int k = 0; k < TPT; ++k) {
      const int task = t + 512 * k;
      if (task < TASKS) {
        const int jj = task & 31, c = task >> 5;
        h8 hi, lo;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          _Float16 a, b;
          split16(stage[k][e], a, b);
          hi[e] = a;
          lo[e] = b;
        }
        *reinterpret_cast<h8*>(&s_zh[buf][zoff<ZS>(jj, c)]) = hi;
        *reinterpret_cast<h8*>(&s_zl[buf][zoff<ZS>(jj, c)]) = lo;
      }
    }
  };
  if (t_begin < t_end) {
    load_tile(t_begin);
    store_tile(0);
    if (t_begin + 1 < t_end) {
      load_tile(t_begin + 1);
      store_tile(1);
    }
  }
  __syncthreads();

  f4v acc_g[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q) acc_g[q] = f4v{};
  float rowsum = 0.f, lacc = 0.f;

  for (int tile = t_begin; tile < t_end; ++tile) {
    const int buf = (tile - t_begin) & 1;
    const bool pred_part = tile < TX;
    const int c0 = (pred_part ? tile : tile - TX) * MT;
    const bool more = tile + 2 < t_end;
    if (more) load_tile(tile + 2);
    const _Float16* zh = s_zh[buf];
    const _Float16* zl = s_zl[buf];

    // ---- Gram, two 16-column halves, three passes per k-step ----
    f4v c[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      c[h] = f4v{};
      const int j = 16 * h + li;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const h8 ah = *reinterpret_cast<const h8*>(zh + zoff<ZS>(j, 4 * s + g));
        const h8 al = *reinterpret_cast<const h8*>(zl + zoff<ZS>(j, 4 * s + g));
        c[h] = mma16(ah, xbh[s], c[h]);
        c[h] = mma16(ah, xbl[s], c[h]);
        c[h] = mma16(al, xbh[s], c[h]);
      }
    }

    // ---- epilogue: lane l has row i, columns j = 16 h + 4 g + v ----
    f2 tl2 = {0.f, 0.f}, rs2 = {0.f, 0.f};
    const float sg = pred_part ? 1.f : -1.f;
    const int jlim = N - c0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 nz4 = *reinterpret_cast<const float4*>(&s_n[buf][16 * h + 4 * g]);
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        const f2 nzp = qq ? f2{nz4.z, nz4.w} : f2{nz4.x, nz4.y};
        const f2 cc = {c[h][2 * qq], c[h][2 * qq + 1]};
        f2 d2 = cc * -2.f + (nzp + nx);
        const int jr = 16 * h + 4 * g + 2 * qq;
        d2.x = jr < jlim ? d2.x : 1.0e30f;
        d2.y = jr + 1 < jlim ? d2.y : 1.0e30f;
        f2 ks, w;
        if (GRAD) rbf7x2_chain(d2, ks, w);
        else rbf7x2(d2, ks, w);
        if (LOSS) tl2 += ks;
        if (GRAD) {
          w *= sg;
          rs2 += w;
          c[h][2 * qq] = w.x;
          c[h][2 * qq + 1] = w.y;
        }
      }
    }
    if (LOSS) lacc = fmaf(pred_part ? (sym && tile >= RBT * (rb + 1) ? 2.f : 1.f) : -2.f, tl2.x + tl2.y, lacc);

    if (GRAD) {
      rowsum += rs2.x + rs2.y;
      h8 wh, wl;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 hi, lo;
        split16(c[e >> 2][e & 3], hi, lo);
        wh[e] = hi;
        wl[e] = lo;
      }
      // B fragment of tile q: rows 4g..4g+3 (slots 0..3) and 16+4g.. (slots 4..7),
      // columns 16 q .. 16 q + 15; lane 4 rr + p of each 16-lane group addresses row
      // rr, columns 4p..4p+3 (chunk 2q + (p >> 1), half (p & 1))
      const int rr = li >> 2, p = li & 3;
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        const int cq = 2 * q + (p >> 1), hq = 4 * (p & 1);
        const int o0 = zoff<ZS>(4 * g + rr, cq) + hq, o1 = zoff<ZS>(16 + 4 * g + rr, cq) + hq;
        typedef __attribute__((address_space(3))) s4v lds_s4v;
        const s4v bh0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(zh + o0));
        const s4v bh1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(zh + o1));
        const s4v bl0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(zl + o0));
        const s4v bl1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(zl + o1));
        const h8 bh = __builtin_bit_cast(h8, __builtin_shufflevector(bh0, bh1, 0, 1, 2, 3, 4, 5, 6, 7));
        const h8 bl = __builtin_bit_cast(h8, __builtin_shufflevector(bl0, bl1, 0, 1, 2, 3, 4, 5, 6, 7));
        acc_g[q] = mma16(wh, bh, acc_g[q]);
        acc_g[q] = mma16(wh, bl, acc_g[q]);
        acc_g[q] = mma16(wl, bh, acc_g[q]);
      }
    }
    __syncthreads();
    if (more) store_tile(buf);
    __syncthreads();
  }

  // ---- loss partial: fixed-order wave then block reduction ----
  float v = row_ok ? lacc : 0.f;
  v = wave_sum(v);
  if (lane == 0) s_red[wave] = v;
  __syncthreads();
  if (t == 0) {
    const float sum = ((s_red[0] + s_red[1]) + (s_red[2] + s_red[3])) + ((s_red[4] + s_red[5]) + (s_red[6] + s_red[7]));
    loss_part[((size_t)r * n_chunks + chunk) * n_rb + rb] = sum;
  }

  if (GRAD) {
    // sum_j W_ij of row i = l&15: the four lane groups hold disjoint column sets
    rowsum += __shfl_xor(rowsum, 16);
    rowsum += __shfl_xor(rowsum, 32);
    float* gp = grad_part + ((size_t)chunk * R + r) * KD * n_rows;
    const int i0 = rb * (W16 * 16) + wave * 16;       // local row of li = 0
#pragma unroll
    for (int vv = 0; vv < 4; ++vv) {
      const int il = 4 * g + vv;                      // accumulator row -> local row
      const float rs = __shfl(rowsum, il);
      const int ii = i0 + il;
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        const int d = 16 * q + li;
        if (d < KD && ii < n_rows) {
          const float pv = X[(size_t)d * N + row_begin + ii];
          gp[(size_t)d * n_rows + ii] = (acc_g[q][vv] - pv * rs) * grad_scale;
        }
      }
    }
  }
}

// ============================================================================
// Joints wider than 256 (CGNN builds one MLP per variable for any d, CGNN.py:63-90):
// the Gram and the gradient are sums over groups of 256 dimensions.  A block of 8
// waves x 16 rows computes, per 32-column tile, the Gram over every group -- group g
// staged in LDS (hi / lo f16, [32][256] skewed as above) and the wave's x fragments of
// group g loaded and split on the fly (a 512-wide x would not fit in registers) -- and
// the gradient for ONE group `dg` only (grid.x = row blocks x groups; the Gram is
// recomputed per group, the gradient accumulators stay at 16 x 4 registers).  The
// block's own group is staged last, so the gradient reads it from the same LDS image.
// Staging is synchronous (no register prefetch): two blocks per CU overlap it.
// ============================================================================
// KD (the padded joint width, a multiple of 256 here) is a launch argument: the groups
// are walked by a rolled loop, so one instantiation covers every width above 256.
template <int MODE>
__global__ __launch_bounds__(512) void mmd_mfma16g_kernel(
    const float* __restrict__ xhat, const float* __restrict__ data,
    const float* __restrict__ xnorm, const float* __restrict__ ynorm,
    float* __restrict__ grad_part, float* __restrict__ loss_part,
    int N, int R, int tiles_per_chunk, float grad_scale, int row_begin, int n_rows, int KD) {
  constexpr bool GRAD = MODE == 0 || MODE == 3;
  constexpr bool LOSS = MODE != 3;
  constexpr int KG = 256;
  const int NG = (KD + KG - 1) / KG;
  constexpr int ZS = (KG + 14 * 8 + 127) / 128 * 128;       // 384 halfs per skewed row
  constexpr int NCH = KG / 8;                                // 32 chunks per row
  constexpr int TPT = MT * NCH / 512;                        // 2 staging tasks per thread
  __shared__ __attribute__((aligned(16))) _Float16 s_zh[MT * ZS];
  __shared__ __attribute__((aligned(16))) _Float16 s_zl[MT * ZS];
  __shared__ __attribute__((aligned(16))) float s_n[MT];
  __shared__ float s_red[W16];

  const int n_rb = gridDim.x / NG;
  const int rb = blockIdx.x % n_rb, dg = blockIdx.x / n_rb;
  const int chunk = blockIdx.y, r = blockIdx.z, n_chunks = gridDim.y;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int i = row_begin + rb * (W16 * 16) + wave * 16 + li;
  const bool row_ok = i - row_begin < n_rows;
  const int ic = row_ok ? i : row_begin;
  const size_t mbase = (size_t)r * KD * N;
  const float* X = xhat + mbase;
  const float* Y = data + mbase;
  const float* XN = xnorm + (size_t)r * N;
  const float* YN = ynorm + (size_t)r * N;
  const float nx = row_ok ? XN[i] : 0.f;

  const int TX = (N + MT - 1) / MT;
  const int ct = MODE == 2 ? TX : 2 * TX;
  const int t_begin = chunk * tiles_per_chunk;
  const int t_end = min(ct, t_begin + tiles_per_chunk);

  f4v acc_g[KG / 16];
#pragma unroll
  for (int q = 0; q < KG / 16; ++q) acc_g[q] = f4v{};
  float rowsum = 0.f, lacc = 0.f;

  for (int tile = t_begin; tile < t_end; ++tile) {
    const bool pred_part = tile < TX;
    const int c0 = (pred_part ? tile : tile - TX) * MT;
    const float* src = pred_part ? X : Y;
    f4v c[2] = {f4v{}, f4v{}};
#pragma unroll 1
    for (int gi = 0; gi < NG; ++gi) {
      const int grp = (dg + 1 + gi) % NG;                    // the block's own group last
      __syncthreads();                                       // earlier readers of the image done
      if (gi == 0 && t < MT) s_n[t] = c0 + t < N ? (pred_part ? XN : YN)[c0 + t] : 0.f;
#pragma unroll
      for (int k = 0; k < TPT; ++k) {
        const int task = t + 512 * k;
        const int jj = task & 31, ch = task >> 5;
        h8 hi, lo;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int d = KG * grp + 8 * ch + e;
          const float v = (d < KD && c0 + jj < N) ? src[(size_t)d * N + c0 + jj] : 0.f;
          _Float16 a, b;
          split16(v, a, b);
          hi[e] = a;
          lo[e] = b;
        }
        *reinterpret_cast<h8*>(&s_zh[zoff<ZS>(jj, ch)]) = hi;
        *reinterpret_cast<h8*>(&s_zl[zoff<ZS>(jj, ch)]) = lo;
      }
      __syncthreads();
      // Gram over this group: x fragments of row i (dims 32 s + 8 g + e of the group)
#pragma unroll 1
      for (int s8 = 0; s8 < KG / 32; ++s8) {
        h8 xh, xl;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int d = KG * grp + 32 * s8 + 8 * g + e;
          const float v = (row_ok && d < KD) ? X[(size_t)d * N + ic] : 0.f;
          _Float16 a, b;
          split16(v, a, b);
          xh[e] = a;
          xl[e] = b;
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int j = 16 * h + li;
          const h8 ah = *reinterpret_cast<const h8*>(s_zh + zoff<ZS>(j, 4 * s8 + g));
          const h8 al = *reinterpret_cast<const h8*>(s_zl + zoff<ZS>(j, 4 * s8 + g));
          c[h] = mma16(ah, xh, c[h]);
          c[h] = mma16(ah, xl, c[h]);
          c[h] = mma16(al, xh, c[h]);
        }
      }
    }

    // ---- epilogue (as mmd_mfma16_kernel) ----
    f2 tl2 = {0.f, 0.f}, rs2 = {0.f, 0.f};
    const float sg = pred_part ? 1.f : -1.f;
    const int jlim = N - c0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 nz4 = *reinterpret_cast<const float4*>(&s_n[16 * h + 4 * g]);
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        const f2 nzp = qq ? f2{nz4.z, nz4.w} : f2{nz4.x, nz4.y};
        const f2 cc = {c[h][2 * qq], c[h][2 * qq + 1]};
        f2 d2 = cc * -2.f + (nzp + nx);
        const int jr = 16 * h + 4 * g + 2 * qq;
        d2.x = jr < jlim ? d2.x : 1.0e30f;
        d2.y = jr + 1 < jlim ? d2.y : 1.0e30f;
        f2 ks, w;
        if (GRAD) rbf7x2_chain(d2, ks, w);
        else rbf7x2(d2, ks, w);
        if (LOSS) tl2 += ks;
        if (GRAD) {
          w *= sg;
          rs2 += w;
          c[h][2 * qq] = w.x;
          c[h][2 * qq + 1] = w.y;
        }
      }
    }
    if (LOSS) lacc = fmaf(pred_part ? 1.f : -2.f, tl2.x + tl2.y, lacc);

    if (GRAD) {
      rowsum += rs2.x + rs2.y;
      h8 wh, wl;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 hi, lo;
        split16(c[e >> 2][e & 3], hi, lo);
        wh[e] = hi;
        wl[e] = lo;
      }
      // the image holds group dg (staged last)
      const int rr = li >> 2, p = li & 3;
#pragma unroll
      for (int q = 0; q < KG / 16; ++q) {
        const int cq = 2 * q + (p >> 1), hq = 4 * (p & 1);
        const int o0 = zoff<ZS>(4 * g + rr, cq) + hq, o1 = zoff<ZS>(16 + 4 * g + rr, cq) + hq;
        typedef __attribute__((address_space(3))) s4v lds_s4v;
        const s4v bh0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(s_zh + o0));
        const s4v bh1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(s_zh + o1));
        const s4v bl0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(s_zl + o0));
        const s4v bl1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(s_zl + o1));
        const h8 bh = __builtin_bit_cast(h8, __builtin_shufflevector(bh0, bh1, 0, 1, 2, 3, 4, 5, 6, 7));
        const h8 bl = __builtin_bit_cast(h8, __builtin_shufflevector(bl0, bl1, 0, 1, 2, 3, 4, 5, 6, 7));
        acc_g[q] = mma16(wh, bh, acc_g[q]);
        acc_g[q] = mma16(wh, bl, acc_g[q]);
        acc_g[q] = mma16(wl, bh, acc_g[q]);
      }
    }
  }

  // ---- loss partial (group-0 blocks only): fixed-order wave then block reduction ----
  float v = row_ok ? lacc : 0.f;
  v = wave_sum(v);
  if (lane == 0) s_red[wave] = v;
  __syncthreads();
  if (t == 0 && dg == 0) {
    const float sum = ((s_red[0] + s_red[1]) + (s_red[2] + s_red[3])) + ((s_red[4] + s_red[5]) + (s_red[6] + s_red[7]));
    loss_part[((size_t)r * n_chunks + chunk) * n_rb + rb] = sum;
  }

  if (GRAD) {
    rowsum += __shfl_xor(rowsum, 16);
    rowsum += __shfl_xor(rowsum, 32);
    float* gp = grad_part + ((size_t)chunk * R + r) * KD * n_rows;
    const int i0 = rb * (W16 * 16) + wave * 16;
#pragma unroll
    for (int vv = 0; vv < 4; ++vv) {
      const int il = 4 * g + vv;
      const float rs = __shfl(rowsum, il);
      const int ii = i0 + il;
#pragma unroll
      for (int q = 0; q < KG / 16; ++q) {
        const int d = KG * dg + 16 * q + li;
        if (d < KD && ii < n_rows) {
          const float pv = X[(size_t)d * N + row_begin + ii];
          gp[(size_t)d * n_rows + ii] = (acc_g[q][vv] - pv * rs) * grad_scale;
        }
      }
    }
  }
}

// the dimension-grouped kernel for any padded width KD > 256 (a multiple of 256)
int launch_mmd_mfma_grouped(int mode, int KD, const float* xhat, const float* data, const float* xn,
                            const float* yn, float* gpart, float* lpart, int N, int R, int n_chunks, int tpc,
                            float gscale, int row_begin, int n_rows, hipStream_t st) {
  const int n_rb = (n_rows + WAVES * MT - 1) / (WAVES * MT);
  const int NG = (KD + 255) / 256;
  dim3 grid(n_rb * NG, n_chunks, R), block(512);
#define WIDEG(M, A, B, C, D2) hipLaunchKernelGGL((mmd_mfma16g_kernel<M>), grid, block, 0, st, A, B, C, D2, gpart, lpart, N, R, tpc, gscale, row_begin, n_rows, KD)
  if (mode == 0) WIDEG(0, xhat, data, xn, yn);
  else if (mode == 3) WIDEG(3, xhat, data, xn, yn);
  else if (mode == 1) WIDEG(1, xhat, data, xn, yn);
  else if (mode == 2) WIDEG(2, data, data, yn, yn);
  else return -3;
#undef WIDEG
  return (int)hipGetLastError();
}

template <int KD>
int launch_mmd_mfma_d(int mode, const float* xhat, const float* data, const float* xn, const float* yn,
                      float* gpart, float* lpart, int N, int R, int n_chunks, int tpc, float gscale,
                      int row_begin, int n_rows, hipStream_t st, int wide) {
  const int n_rb = (n_rows + WAVES * MT - 1) / (WAVES * MT);
  if constexpr (KD > 256) {
    return launch_mmd_mfma_grouped(mode, KD, xhat, data, xn, yn, gpart, lpart, N, R, n_chunks, tpc, gscale,
                                   row_begin, n_rows, st);
  }
  if (wide < 0) wide = KD >= 128;
  if (KD >= 128 && wide) {
    if constexpr (KD >= 128 && KD <= 256) {
      dim3 grid(n_rb, n_chunks, R), block(512);
#define WIDE(M, A, B, C, D2) hipLaunchKernelGGL((mmd_mfma16_kernel<KD, M>), grid, block, 0, st, A, B, C, D2, gpart, lpart, N, R, tpc, gscale, row_begin, n_rows)
      if (mode == 0) WIDE(0, xhat, data, xn, yn);
      else if (mode == 3) WIDE(3, xhat, data, xn, yn);
      else if (mode == 1) WIDE(1, xhat, data, xn, yn);
      else if (mode == 2) WIDE(2, data, data, yn, yn);
      else return -3;
#undef WIDE
      return (int)hipGetLastError();
    }
  }
  if constexpr (KD > 256) return -1;
  else {
  dim3 grid(n_rb, n_chunks, R), block(256);
  if (mode == 0)
    hipLaunchKernelGGL((mmd_mfma_kernel<KD, 0>), grid, block, 0, st, xhat, data, xn, yn, gpart, lpart, N, R, tpc, gscale, row_begin, n_rows);
  else if (mode == 3)
    hipLaunchKernelGGL((mmd_mfma_kernel<KD, 3>), grid, block, 0, st, xhat, data, xn, yn, gpart, lpart, N, R, tpc, gscale, row_begin, n_rows);
  else if (mode == 1)
    hipLaunchKernelGGL((mmd_mfma_kernel<KD, 1>), grid, block, 0, st, xhat, data, xn, yn, gpart, lpart, N, R, tpc, gscale, row_begin, n_rows);
  else if (mode == 2)
    hipLaunchKernelGGL((mmd_mfma_kernel<KD, 2>), grid, block, 0, st, data, data, yn, yn, gpart, lpart, N, R, tpc, gscale, row_begin, n_rows);
  else
    return -3;
  return (int)hipGetLastError();
  }
}

}  // namespace

// Supported widths (the padded D of engine/batch.py SUPPORTED_D, >= 8; above 64 the
// matrix-core kernel is the only MMD; above 1024 every multiple of 256 up to MMD_MAX_D)
extern "C" int cgnn_mmd_mfma_supported(int D) {
  switch (D) {
    case 8: case 12: case 16: case 20: case 24: case 32: case 48: case 64:
    case 80: case 96: case 128: case 160: case 192: case 224: case 256:
    case 320: case 384: case 448: case 512: case 640: case 768: case 896: case 1024: return 1;
    default: return D > 1024 && D % 256 == 0 && D <= MMD_MAX_D;
  }
}

// Geometry: row blocks of 128 generated rows; `n_chunks` column chunks of
// `tpc` 32-wide tiles of the joint [pred; true] column space.
extern "C" int cgnn_mmd_mfma_row_blocks(int N) { return (N + WAVES * MT - 1) / (WAVES * MT); }

// xnorm / ynorm: [R][N] squared norms of the generated / true samples
// wide: -1 auto (the 16-row kernel from D = 128), 0 / 1 force (A/B and tests)
extern "C" int cgnn_launch_mmd_mfma_rows(int mode, int D, const float* xhat, const float* data, const float* xnorm,
                                    const float* ynorm, float* gpart, float* lpart, int N, int R, int n_chunks,
                                    int tpc, float gscale, int row_begin, int n_rows, hipStream_t st, int wide) {
  if (row_begin < 0 || n_rows < 1 || row_begin + n_rows > N) return -2;
  switch (D) {
#define CASE_D(d) case d: return launch_mmd_mfma_d<d>(mode, xhat, data, xnorm, ynorm, gpart, lpart, N, R, n_chunks, tpc, gscale, row_begin, n_rows, st, wide);
    CASE_D(8) CASE_D(12) CASE_D(16) CASE_D(20) CASE_D(24) CASE_D(32) CASE_D(48) CASE_D(64)
    CASE_D(80) CASE_D(96) CASE_D(128) CASE_D(160) CASE_D(192) CASE_D(224) CASE_D(256)
    CASE_D(320) CASE_D(384) CASE_D(448) CASE_D(512) CASE_D(640) CASE_D(768) CASE_D(896) CASE_D(1024)
#undef CASE_D
    default:
      if (D > 1024 && D % 256 == 0 && D <= MMD_MAX_D)
        return launch_mmd_mfma_grouped(mode, D, xhat, data, xnorm, ynorm, gpart, lpart, N, R, n_chunks, tpc, gscale,
                                       row_begin, n_rows, st);
      return -1;
  }
}

extern "C" int cgnn_launch_mmd_mfma(int mode, int D, const float* xhat, const float* data, const float* xnorm,
                                    const float* ynorm, float* gpart, float* lpart, int N, int R, int n_chunks,
                                    int tpc, float gscale, hipStream_t st) {
  return cgnn_launch_mmd_mfma_rows(mode, D, xhat, data, xnorm, ynorm, gpart, lpart, N, R, n_chunks, tpc, gscale,
                                   0, N, st, -1);
}
