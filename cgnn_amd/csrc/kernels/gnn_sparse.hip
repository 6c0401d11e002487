// GNN track (beyond the reference, SURVEY §0 Phase B): sparse message passing
// kernels for MI355X.
//
//   spmm_kernel     Y[i,:] = act( rscale[i] * sum_{j in N(i)} X[j,:] + bias )
//                   CSR neighbour aggregate (gather-sum).  Symmetric GCN
//                   normalisation D^-1/2 (A+I) D^-1/2 is split into a row scale
//                   here and a column scale folded into the producer of X, so
//                   no per-edge value is ever read: the kernel streams only
//                   col[] and the gathered rows.
//   spmm_ce_kernel  layer-2 aggregate fused with bias, log-softmax,
//                   cross-entropy, accuracy counting and the loss gradient
//                   (pre-scaled by rscale for the backward SpMM).
//
// Mapping: a sub-group of L lanes owns one row; each lane owns 8 consecutive
// features (one 16-byte bf16 load per gathered row).  L = 16 covers F <= 128
// (4 rows per wave64), L = 8 covers F <= 64 (8 rows per wave64).  The L column
// indices of the next L edges are fetched with one coalesced load and
// broadcast inside the sub-group with ds_bpermute; four gathered rows are kept
// in flight per lane.  Accumulation is fp32; storage is bf16.
#include "cgnn_common.h"
#include "gnn_gather.h"
#include <algorithm>
#include <cmath>
#include <cstdlib>

using namespace cgnn;
using namespace cgnn::gather;

namespace {

struct bf16x8 { uint32_t w[4]; };

}  // namespace


// Fixed-order column sums of per-block partials P [S][W] (fp32, row-major): block
// (x, y) sums rows [y * per, (y + 1) * per) of columns [64 x, 64 x + 64), blockDim / 64
// row lanes striding the rows, their sums combined in lane order -- deterministic, no
// atomics.  With gridDim.y > 1 the result is a stage [gridDim.y][W] for a second pass;
// with gridDim.y == 1 it is written to out[map[c]] (map[c] < 0: dropped; no map:
// out[c]), so the final pass also scatters the sums into their places (e.g. the weight
// gradients into the flat parameter-gradient buffer).
__global__ __launch_bounds__(1024) void slab_sum_kernel(const float* __restrict__ P, long S, int W, long per,
                                                       float* __restrict__ out, const int* __restrict__ map,
                                                       int* __restrict__ bump) {
  // bump (optional, final pass): block 0 adds 1 to *bump (a step counter advanced here
  // instead of by a launch of its own; nothing in this kernel reads it)
  if (bump && gridDim.y == 1 && blockIdx.x == 0 && threadIdx.x == 0) *bump += 1;
  __shared__ float red[16][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6, nrl = blockDim.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const long r0 = (long)blockIdx.y * per, r1 = min(S, r0 + per);
  float acc = 0.f;
  if (c < W) {
#pragma unroll 8
    for (long r = r0 + rl; r < r1; r += nrl) acc += P[r * W + c];
  }
  red[rl][cl] = acc;
  __syncthreads();
  if (rl == 0 && c < W) {
    float v = red[0][cl];
    for (int q = 1; q < nrl; ++q) v += red[q][cl];
    if (gridDim.y > 1) {
      out[(long)blockIdx.y * W + c] = v;
    } else {
      const int d = map ? map[c] : c;
      if (d >= 0) out[d] = v;
    }
  }
}

template <int L, int XBF, int YBF, int U, bool CS>
__global__ __launch_bounds__(256) void spmm_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col, const void* __restrict__ X,
    void* __restrict__ Y, const float* __restrict__ rscale, const float* __restrict__ bias,
    int n_rows, int F, int ldx, int ldy, int relu, int unit_col, int wcols,
    const float* __restrict__ init, int ldi, const float* __restrict__ cscale, int init_rows) {
  // init (optional, fp32 [init_rows][ldi]): partial sums of earlier edges (e.g. the
  // rank-local part of a split aggregation, or GraphSAGE's self-path gradient of the
  // destination rows, a prefix of the sources), added before the row scale
  // wcols: output columns this launch writes (from its base): the row stride ldy
  // for a whole-row launch, the slab width for a column-slab launch
  constexpr int RPW = 64 / L;
  const int lane = threadIdx.x & 63;
  const int sub = lane / L, sl = lane - sub * L;
  const unsigned blk = xcd_remap(blockIdx.x, gridDim.x);
  const int row = (blk * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RPW + sub;
  const bool rv = row < n_rows;
  const int f0 = sl * 8;
  const bool fv = rv && f0 < F;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int e0 = rv ? rowptr[row] : 0, e1 = rv ? rowptr[row + 1] : 0;
  gather_sum<L, XBF, U, CS>(col, X, e0, e1, ldx, f0, fv, sub * L, sl, acc, cscale);
  if (!rv || f0 >= wcols) return;
  if (init && fv && row < init_rows) {
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (f0 + q < F) acc[q] += init[(size_t)row * ldi + f0 + q];
  }
  const float rs = rscale ? rscale[row] : 1.f;
  float y[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int f = f0 + q;
    float v = acc[q] * rs + ((bias && f < F) ? bias[f] : 0.f);
    if (relu) v = fmaxf(v, 0.f);
    y[q] = f < F ? v : (f == unit_col ? 1.f : 0.f);
  }
  if (YBF == 1) {
    *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(Y) + (size_t)row * ldy + f0) = f32x8_to_bf16(y);
  } else if (YBF == 2) {
    f16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = (_Float16)y[q];
    *reinterpret_cast<f16x8*>(reinterpret_cast<uint16_t*>(Y) + (size_t)row * ldy + f0) = o;
  } else {
    float4* p = reinterpret_cast<float4*>(reinterpret_cast<float*>(Y) + (size_t)row * ldy + f0);
    p[0] = make_float4(y[0], y[1], y[2], y[3]);
    p[1] = make_float4(y[4], y[5], y[6], y[7]);
  }
}

// Short rows (average degree <= 2: the transposed blocks of sampled GraphSAGE, where
// most sources were picked once).  spmm_kernel gives each L-lane sub-group ONE row, and
// a row is a chain of dependent round trips (row bounds -> column id -> column scale
// and source row -> store) with one source row in flight per lane.  Here a sub-group
// owns RP consecutive rows: their edges are one contiguous CSR range, so one load per
// lane brings the row bounds, one more the first L column ids, and the RP rows' first
// sources load together -- RP rows per round trip.  Rows of 2-3 entries add their
// further sources one by one; rows of 4+ (or past the first L edges) take gather_sum.
// Per row the same adds in the same order as spmm_kernel (whose 1-steps they are):
// bit-identical output.  Blocks map to rows in launch order (see below).
template <int L, int XBF, int YBF, int RP, bool CS>
__global__ __launch_bounds__(256) void spmm_short_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col, const void* __restrict__ X,
    void* __restrict__ Y, const float* __restrict__ rscale, const float* __restrict__ bias,
    int n_rows, int F, int ldx, int ldy, int relu, int unit_col, int wcols,
    const float* __restrict__ init, int ldi, const float* __restrict__ cscale, int init_rows) {
  constexpr int RPW = 64 / L;
  const int lane = threadIdx.x & 63;
  const int sub = lane / L, sl = lane - sub * L, sub_base = sub * L;
  // NO XCD remap: the sources are in-edges of random destinations (no L2 locality to
  // keep), and the rows with an init (the destinations, a prefix) must spread over all
  // eight XCDs -- remapped, the first XCD alone read the whole fp32 init (+43 us of 83,
  // profiles/r05_sage)
  const unsigned blk = blockIdx.x;
  const int r0 = ((blk * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RPW + sub) * RP;
  if (r0 >= n_rows) return;                       // uniform per sub-group
  const int f0 = sl * 8;
  const bool fv = f0 < F;
  // spmm_kernel's epilogue for one row
  auto store_row = [&](int row, float* acc) {
    if (init && fv && row < init_rows) {
      const float* ip = init + (size_t)row * ldi + f0;
      if (f0 + 8 <= F && ((uintptr_t)ip & 15) == 0) {       // two 16-byte loads
        const float4 u = reinterpret_cast<const float4*>(ip)[0], v = reinterpret_cast<const float4*>(ip)[1];
        acc[0] += u.x; acc[1] += u.y; acc[2] += u.z; acc[3] += u.w;
        acc[4] += v.x; acc[5] += v.y; acc[6] += v.z; acc[7] += v.w;
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (f0 + q < F) acc[q] += ip[q];
      }
    }
    const float rs = rscale ? rscale[row] : 1.f;
    float y[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int f = f0 + q;
      float v = acc[q] * rs + ((bias && f < F) ? bias[f] : 0.f);
      if (relu) v = fmaxf(v, 0.f);
      y[q] = f < F ? v : (f == unit_col ? 1.f : 0.f);
    }
    if (YBF == 1) {
      *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(Y) + (size_t)row * ldy + f0) = f32x8_to_bf16(y);
    } else if (YBF == 2) {
      f16x8 o;
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = (_Float16)y[q];
      *reinterpret_cast<f16x8*>(reinterpret_cast<uint16_t*>(Y) + (size_t)row * ldy + f0) = o;
    } else {
      float4* p = reinterpret_cast<float4*>(reinterpret_cast<float*>(Y) + (size_t)row * ldy + f0);
      p[0] = make_float4(y[0], y[1], y[2], y[3]);
      p[1] = make_float4(y[4], y[5], y[6], y[7]);
    }
  };
  const int rpv = rowptr[min(r0 + min(sl, RP), n_rows)];
  int e[RP + 1];
#pragma unroll
  for (int r = 0; r <= RP; ++r) e[r] = __shfl(rpv, sub_base + r, 64);
  const int eb = e[0], ee = e[RP];
  const int myj = ee > eb ? col[min(eb + sl, ee - 1)] : 0;
  const float mycs = CS && ee > eb ? cscale[myj] : 1.f;
  // a row is long: 4+ entries (gather_sum's grouped steps) or past the first L edges
  auto is_long = [&](int r) { return e[r + 1] - e[r] >= 4 || e[r + 1] - eb > L; };
  float acc[RP][8];
#pragma unroll
  for (int r = 0; r < RP; ++r) {                  // every row's first source in flight at once
    const int k = min(e[r] - eb, L - 1);
    const int j = __shfl(myj, sub_base + k, 64);
    const float c = CS ? __shfl(mycs, sub_base + k, 64) : 1.f;
    float a[8];
    if (fv && ee > eb) load8<XBF>(X, (size_t)j * ldx + f0, a);     // (j is a real id then)
    const bool has = e[r + 1] > e[r];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      acc[r][q] = 0.f;
      if (fv && has) acc[r][q] = CS ? fmaf(c, a[q], acc[r][q]) : acc[r][q] + a[q];
    }
  }
#pragma unroll
  for (int r = 0; r < RP; ++r) {                  // rows of 2-3 entries: the 1-steps
    const int deg = e[r + 1] - e[r];
    if (deg <= 1 || is_long(r)) continue;
    for (int t = 1; t < deg; ++t) {
      const int k = e[r] - eb + t;
      const int j = __shfl(myj, sub_base + k, 64);
      const float c = CS ? __shfl(mycs, sub_base + k, 64) : 1.f;
      if (fv) {
        float a[8];
        load8<XBF>(X, (size_t)j * ldx + f0, a);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[r][q] = CS ? fmaf(c, a[q], acc[r][q]) : acc[r][q] + a[q];
      }
    }
  }
  // (no early exit for lanes past wcols: the long rows' gathers read every lane's ids)
  const bool wv = f0 < wcols;
#pragma unroll
  for (int r = 0; r < RP; ++r)
    if (wv && r0 + r < n_rows && !is_long(r)) store_row(r0 + r, acc[r]);
  // long rows last, one at a time (the short rows' accumulators are dead by now)
  for (int r = 0; r < RP; ++r) {
    if (r0 + r >= n_rows || !is_long(r)) continue;
    float acc1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    gather_sum<L, XBF, 8, CS>(col, X, e[r], e[r + 1], ldx, f0, fv, sub_base, sl, acc1, cscale);
    if (wv) store_row(r0 + r, acc1);
  }
}

// Short-row aggregate from an ELL image (the GCN backward's train-column adjacency: ~4
// entries per row): ell[row][0..7] holds the row's column ids (-1 past its end) or, for a
// row of more than 8 entries, {-2, e0, e1}: its range in the CSR `col`.  One 32-B load
// gives the 8-lane sub-group its whole row, so a row costs two dependent round trips
// (indices, rows) instead of three (row bounds, indices, rows).  bf16 in / out, F <= 64,
// Y[row] = rscale[row] * sum, padding columns 0.  Capped at 64 VGPRs (8 waves per SIMD
// instead of 7, no spills): 233.5 -> 216.8 us on the headline shape (profiles/r05_ell).
__global__ __launch_bounds__(256, 8) void spmm_ell_kernel(const int* __restrict__ ell, const int* __restrict__ col,
                                                       const uint16_t* __restrict__ X, uint16_t* __restrict__ Y,
                                                       const float* __restrict__ rscale, int n_rows, int F,
                                                       int ldx, int ldy) {
  constexpr int L = 8, RPW = 8;
  const int lane = threadIdx.x & 63, sub = lane / L, sl = lane - sub * L;
  const unsigned blk = xcd_remap(blockIdx.x, gridDim.x);
  const int row = (blk * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RPW + sub;
  const bool rv = row < n_rows;
  const int f0 = sl * 8;
  const bool fv = rv && f0 < F;
  const int myj = rv ? ell[(size_t)row * 8 + sl] : -1;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int j0 = __shfl(myj, sub * L, 64);
  if (j0 == -2) {                          // a long row: its CSR range
    const int e0 = __shfl(myj, sub * L + 1, 64), e1 = __shfl(myj, sub * L + 2, 64);
    gather_sum<L, 1, 8>(col, X, e0, e1, ldx, f0, fv, sub * L, sl, acc);
  } else {
    uint4 r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = __shfl(myj, sub * L + u, 64);
      r[u] = (fv && j >= 0) ? load_raw16(X, (size_t)j * ldx + f0) : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < 8; u += 2) acc_bf16_pair(acc, r[u], r[u + 1]);
  }
  if (!rv || f0 >= ldy) return;
  const float rs = rscale ? rscale[row] : 1.f;
  float y[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) y[q] = f0 + q < F ? acc[q] * rs : 0.f;
  *reinterpret_cast<uint4*>(Y + (size_t)row * ldy + f0) = f32x8_to_bf16(y);
}

// The same aggregate as a persistent grid (8 waves per SIMD on every CU) in which each
// wave loops over groups of 8 rows and loads the NEXT group's ELL indices right after
// issuing the current group's gathers: the index round trip of group k + 1 runs under
// the gathers of group k, so a group costs one exposed round trip instead of two (the
// one-shot form above is latency-bound: 217 us on the headline shape against a ~60 us
// traffic floor).  Loads and stores are counted in issue order (vmcnt), so the prefetch
// is issued AFTER the gathers (the scheduling barriers pin that order), and every
// gather and the row store go through buffer descriptors with out-of-range offsets for
// inactive lanes (the hardware returns 0 / drops the store): no branches, so the waits
// are exact counts that leave the prefetch in flight.  Rows of more than 8 entries are
// skipped in that loop (their store is dropped): a data-dependent inner loop inside it
// would make every wait of the loop a full drain.  After it, the waves sum the image's
// list of long rows, one per 8-lane sub-group, over their CSR ranges.  Same adds in the
// same order as spmm_ell_kernel: bit-identical output.  Tables below 2^31 bytes (the
// launcher checks).
__global__ __launch_bounds__(256, 8) void spmm_ell_pipe_kernel(const int* __restrict__ ell,
                                                            const int* __restrict__ col,
                                                            const int* __restrict__ long_rows, int n_long,
                                                            const uint16_t* __restrict__ X,
                                                            uint16_t* __restrict__ Y,
                                                            const float* __restrict__ rscale, int n_rows, int F,
                                                            int ldx, int ldy, uint32_t x_bytes) {
  constexpr int L = 8, RPW = 8;
  constexpr uint32_t OOB = 0x80000000u;
  typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63, sub = lane / L, sl = lane - sub * L;
  const int nw = gridDim.x * (blockDim.x >> 6);
  const int n_groups = (n_rows + RPW - 1) / RPW;
  const int f0 = sl * 8;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(X), (short)0,
                                                                      (int)x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(Y, (short)0,
                                                                      (int)((uint32_t)n_rows * (uint32_t)ldy * 2u),
                                                                      0x00020000);
  // a valid address for the row-scale load when there is no rscale (the value is unused)
  const float* rsb = rscale ? rscale : reinterpret_cast<const float*>(ell);
  // (measured: giving each XCD a contiguous eighth of the row groups, so that the
  // compact-G rows it gathers could stay in its L2, was neutral -- 174.8 vs 175.0 us)
  const int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  int g = wave;
  if (g < n_groups) {                        // uniform per wave
  // clamped, unconditional loads (a "load or -1" branches and waits at the join)
  int nj = ell[(size_t)min(g * RPW + sub, n_rows - 1) * 8 + sl];
  // a dropped store behind the first index load: the loop is entered with the same
  // count of younger operations as its back edge (the previous row store), so the loop
  // head's wait for the indices is one vmcnt(1) that never waits for a row store
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_raw_buffer_store_b32(0u, yr, OOB, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
  do {
    const int row = g * RPW + sub;
    const bool rv = row < n_rows;
    const int myj = nj;
    const int j0 = __shfl(myj, sub * L, 64);
    const bool ok = rv && j0 != -2;          // a short row of this wave's group
    const bool fv = ok && f0 < F;
    uint4 r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = __shfl(myj, sub * L + u, 64);
      const uint32_t off = (fv && j >= 0) ? ((uint32_t)j * (uint32_t)ldx + (uint32_t)f0) * 2u : OOB;
      r[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
    // the row scale is independent of the indices: loaded beside the gathers
    const float rsv = rsb[rscale ? min(row, n_rows - 1) : 0];
    __builtin_amdgcn_sched_barrier(0);
    nj = ell[(size_t)min((g + nw) * RPW + sub, n_rows - 1) * 8 + sl];
    __builtin_amdgcn_sched_barrier(0);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 8; u += 2) acc_bf16_pair(acc, r[u], r[u + 1]);
    const float rs = rscale ? rsv : 1.f;
    float y[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) y[q] = f0 + q < F ? acc[q] * rs : 0.f;
    const uint32_t yo = (ok && f0 < ldy) ? ((uint32_t)row * (uint32_t)ldy + (uint32_t)f0) * 2u : OOB;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, f32x8_to_bf16(y)), yr, yo, 0, 0);
    g += nw;
  } while (g < n_groups);
  }
  // the long rows: one per sub-group, over its CSR range (spmm_ell_kernel's long path;
  // 4-steps: for bf16 rows the same pair adds in the same order as its 8-steps -- two
  // acc_bf16_pair per 4-step -- with half the loads live, no spills at 64 VGPRs)
  for (int k = wave * RPW + sub; k < n_long; k += nw * RPW) {
    const int row = long_rows[k];
    const int e0 = ell[(size_t)row * 8 + 1], e1 = ell[(size_t)row * 8 + 2];
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    gather_sum<L, 1, 4>(col, X, e0, e1, ldx, f0, f0 < F, sub * L, sl, acc);
    const float rs = rscale ? rscale[row] : 1.f;
    float y[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) y[q] = f0 + q < F ? acc[q] * rs : 0.f;
    if (f0 < ldy) *reinterpret_cast<uint4*>(Y + (size_t)row * ldy + f0) = f32x8_to_bf16(y);
  }
}

// Rows of at most 8 entries (a sampled GraphSAGE block's input layer: one row per
// destination, min(degree, fanout) picks) as a persistent pipelined grid -- spmm_kernel
// <16> there walks three dependent round trips per row (row bounds, column ids, rows)
// with ~5 gathers each.  Each wave loops over groups of 4 rows (16 lanes per row, F <=
// 128): the gathers of group g go out with the column ids of group g + nw (whose row
// bounds arrived one iteration earlier) and the row bounds of group g + 2 nw, so a group
// costs one exposed round trip.  Gathers, column-id loads and stores use buffer
// descriptors with out-of-range offsets for inactive lanes (zeros / dropped stores, no
// branches, exact wait counts).  Per row the same adds in the same order as spmm_kernel's
// gather_sum<16, 1, 8> (an 8-step for 8 entries, else a 4-step for >= 4, then 1-steps),
// and its epilogue: bit-identical output.  Tables below 2^31 bytes (the launcher checks).
__global__ __launch_bounds__(256, 8) void spmm_fan_pipe_kernel(const int* __restrict__ rowptr,
                                                            const int* __restrict__ col,
                                                            const uint16_t* __restrict__ X, uint16_t* __restrict__ Y,
                                                            const float* __restrict__ rscale, int n_rows, int F,
                                                            int ldx, int ldy, uint32_t x_bytes, uint32_t col_bytes) {
  constexpr int L = 16, RPW = 4;
  constexpr uint32_t OOB = 0x80000000u;
  typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63, sub = lane / L, sl = lane - sub * L;
  const int nw = gridDim.x * (blockDim.x >> 6);
  const int n_groups = (n_rows + RPW - 1) / RPW;
  const int f0 = sl * 8;
  const bool fl = f0 < F;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(X), (short)0,
                                                                      (int)x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(col), (short)0,
                                                                      (int)col_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(Y, (short)0,
                                                                      (int)((uint32_t)n_rows * (uint32_t)ldy * 2u),
                                                                      0x00020000);
  const float* rsb = rscale ? rscale : reinterpret_cast<const float*>(rowptr);
  const int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  int g = wave;
  if (g < n_groups) {                        // uniform per wave
  // row bounds of this group and the next, the column ids of this group (clamped rows;
  // the ids through the descriptor: an empty row, or one at the end of col, reads zeros)
  int a0 = rowptr[min(g * RPW + sub, n_rows - 1)], b0 = rowptr[min(g * RPW + sub, n_rows - 1) + 1];
  int a1 = rowptr[min((g + nw) * RPW + sub, n_rows - 1)], b1 = rowptr[min((g + nw) * RPW + sub, n_rows - 1) + 1];
  int cj = __builtin_amdgcn_raw_buffer_load_b32(cr, sl < b0 - a0 ? (uint32_t)(a0 + sl) * 4u : OOB, 0, 0);
  // a dropped store: the loop is entered with the younger-operation count of its back edge
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_raw_buffer_store_b32(0u, yr, OOB, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
  do {
    const int row = g * RPW + sub;
    const bool rv = row < n_rows;
    const int cnt = rv ? b0 - a0 : 0;        // <= 8 (the caller's guarantee)
    const int myj = cj;
    int j[8];
    row_bcast8<0>(myj, j);
    uint4 r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t off = (fl && u < cnt) ? ((uint32_t)j[u] * (uint32_t)ldx + (uint32_t)f0) * 2u : OOB;
      r[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
    const float rsv = rsb[rscale ? min(row, n_rows - 1) : 0];
    __builtin_amdgcn_sched_barrier(0);
    // the next group's column ids (its bounds arrived last iteration), then the bounds of
    // the group after it
    const int row1 = (g + nw) * RPW + sub;
    cj = __builtin_amdgcn_raw_buffer_load_b32(cr, (row1 < n_rows && sl < b1 - a1) ? (uint32_t)(a1 + sl) * 4u : OOB,
                                              0, 0);
    a0 = a1;
    b0 = b1;
    const int row2 = min((g + 2 * nw) * RPW + sub, n_rows - 1);
    a1 = rowptr[row2];
    b1 = rowptr[row2 + 1];
    __builtin_amdgcn_sched_barrier(0);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (cnt == 8) {
#pragma unroll
      for (int u = 0; u < 8; u += 2) acc_bf16_pair(acc, r[u], r[u + 1]);
    } else {
      const int k = cnt >= 4 ? 4 : 0;
      if (cnt >= 4) {
        acc_bf16_pair(acc, r[0], r[1]);
        acc_bf16_pair(acc, r[2], r[3]);
      }
      // (u runs to 7 although cnt <= 7 here: the eighth gather is then used on both
      // paths and stays with the others, instead of sinking into the 8-entry branch
      // behind a full drain)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (u >= k && u < cnt) {
          float f[8];
          bf16x8_to_f32(r[u], f);
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[q] = acc[q] + f[q];
        }
      }
    }
    const float rs = rscale ? rsv : 1.f;
    float y[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) y[q] = f0 + q < F ? acc[q] * rs + 0.f : 0.f;
    const uint32_t yo = (rv && f0 < ldy) ? ((uint32_t)row * (uint32_t)ldy + (uint32_t)f0) * 2u : OOB;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, f32x8_to_bf16(y)), yr, yo, 0, 0);
    g += nw;
  } while (g < n_groups);
  }
}

// ell image of a CSR for spmm_ell_kernel (one thread per row)
__global__ void ell_build_kernel(const int* __restrict__ rowptr, const int* __restrict__ col, int* __restrict__ ell,
                                 int n_rows) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_rows) return;
  const int e0 = rowptr[i], e1 = rowptr[i + 1];
  int v[8];
  if (e1 - e0 > 8) {
    v[0] = -2; v[1] = e0; v[2] = e1;
#pragma unroll
    for (int u = 3; u < 8; ++u) v[u] = -1;
  } else {
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = e0 + u < e1 ? col[e0 + u] : -1;
  }
  int4* o = reinterpret_cast<int4*>(ell + (size_t)i * 8);
  o[0] = make_int4(v[0], v[1], v[2], v[3]);
  o[1] = make_int4(v[4], v[5], v[6], v[7]);
}

// Layer-2 aggregate + bias + log-softmax + NLL.  L = 8 lanes per row, C <= 64.
//   mask[i]: 0 = unused, 1 = train, 2 = valid, 3 = test
//   stats[block][4 + 64] = {sum train loss, #correct train, #correct valid, #correct test,
//                           per-class sum of dL/dlogits (= the b2 gradient, mode 0)}
//   mode 0: also write G[i,:] = rscale[i] * (softmax - onehot) / n_train  (train rows)
//   gslot (optional): G is COMPACT -- only rows with gslot[i] >= 0 (the train rows, the
//   only non-zero rows of dL/dlogits) are written, to G[gslot[i]]; the backward then
//   aggregates over the train columns of the adjacency only
//   n_long: rows [0, n_long) are long (the caller orders them first) and take a whole
//   wave each: its 8 sub-groups walk every 8th chunk of 8 edges and their sums are
//   combined across the sub-groups, so one power-law row does not hold the launch for
//   its whole length on 8 lanes (ogbn-products train rows: up to 766 entries; the
//   launch was 0.19 ms with, 0.10 ms without its longest rows)
__global__ __launch_bounds__(256, 8) void spmm_ce_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col, const void* __restrict__ Z,
    const float* __restrict__ rscale, const float* __restrict__ bias, const int* __restrict__ labels,
    const uint8_t* __restrict__ mask, float* __restrict__ stats, void* __restrict__ G,
    int n_rows, int C, int ld, int mode, float inv_count, const float* __restrict__ init, int ldi,
    const int* __restrict__ gslot, int n_long) {
  constexpr int L = 8, RPW = 8;
  __shared__ float s_red[4][4];
  __shared__ float s_cls[4][64];
  __shared__ int s_cnt;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();   // the only barrier: at entry, where the waves are still in step
  const int sub = lane / L, sl = lane - sub * L;
  const unsigned blk = xcd_remap(blockIdx.x, gridDim.x);
  const int wg = (int)blk * (int)(blockDim.x >> 6) + wid;
  const bool lmode = wg < n_long;             // wave-uniform
  const int row = lmode ? wg : n_long + (wg - n_long) * RPW + sub;
  const bool gv = row < n_rows;               // this lane gathers for `row`
  const int f0 = sl * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int e0 = gv ? rowptr[row] : 0, e1 = gv ? rowptr[row + 1] : 0;
  if (lmode) {
    for (int e = e0 + sub * L; e < e1; e += L * RPW)
      gather_sum<L, 1, 8>(col, Z, e, min(e + L, e1), ld, f0, f0 < C, sub * L, sl, acc);
#pragma unroll
    for (int q = 0; q < 8; ++q) {             // fixed-order combination over the sub-groups
      acc[q] += __shfl_xor(acc[q], 8, 64);
      acc[q] += __shfl_xor(acc[q], 16, 64);
      acc[q] += __shfl_xor(acc[q], 32, 64);
    }
  } else {
    gather_sum<L, 1, 8>(col, Z, e0, e1, ld, f0, gv && f0 < C, sub * L, sl, acc);
  }
  const bool rv = gv && (!lmode || sub == 0);   // the row's epilogue lanes
  const bool fv = rv && f0 < C;
  if (init && fv) {              // partial sums of earlier edges (split aggregation)
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (f0 + q < C) acc[q] += init[(size_t)row * ldi + f0 + q];
  }

  const float rs = rv ? rscale[row] : 0.f;
  float lg[8];
  float mx = -INFINITY;
  int amax = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int c = f0 + q;
    lg[q] = (c < C) ? acc[q] * rs + bias[c] : -INFINITY;
    if (lg[q] > mx) { mx = lg[q]; amax = c; }
  }
  // arg-max / max over the 8-lane sub-group (ties -> lowest class id)
#pragma unroll
  for (int off = 1; off < L; off <<= 1) {
    const float om = __shfl_xor(mx, off, 64);
    const int oa = __shfl_xor(amax, off, 64);
    if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
  }
  float ex[8];
  float se = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    ex[q] = (f0 + q < C) ? __expf(lg[q] - mx) : 0.f;   // reused for the softmax below
    se += ex[q];
  }
#pragma unroll
  for (int off = 1; off < L; off <<= 1) se += __shfl_xor(se, off, 64);
  const float lse = mx + __logf(se);
  const float inv_se = 1.f / se;
  const int y = rv ? labels[row] : -1;
  const int split = rv ? (int)mask[row] : 0;
  float my_loss = 0.f;
  if (split == 1 && y >= f0 && y < f0 + 8) {
#pragma unroll
    for (int q = 0; q < 8; ++q) if (f0 + q == y) my_loss = lse - lg[q];
  }
  float dl[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int c = f0 + q;
    dl[q] = (rv && split == 1 && c < C) ? (ex[q] * inv_se - (c == y ? 1.f : 0.f)) * inv_count : 0.f;
  }
  const int gr = (mode == 0 && rv) ? (gslot ? gslot[row] : row) : -1;
  if (gr >= 0 && f0 < ld) {
    float gq[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) gq[q] = dl[q] * rs;
    *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(G) + (size_t)gr * ld + f0) = f32x8_to_bf16(gq);
  }
  // Loss and per-class dL/dlogits sums are non-zero only on train rows (8 % of
  // ogbn-products): a wave with none of its 8 rows in the train split skips both
  // reductions (wave-uniform branch; dl is already zero there).
  float v0 = 0.f;
  if (__ballot(rv && split == 1)) {
    // per-class sums over the 8 rows of this wave: lanes with equal sl hold the same classes
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float v = dl[q];
      v += __shfl_xor(v, 8, 64);
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      dl[q] = v;
    }
    v0 = wave_sum(my_loss);
  }
  if (lane < 8) {
#pragma unroll
    for (int q = 0; q < 8; ++q) s_cls[wid][lane * 8 + q] = dl[q];
  }
  // accuracy counts: one vote per row (sub-group lane 0), counted by ballot + popcount
  const bool hit = rv && sl == 0 && amax == y;
  const float v1 = (float)__popcll(__ballot(hit && split == 1));
  const float v2 = (float)__popcll(__ballot(hit && split == 2));
  const float v3 = (float)__popcll(__ballot(hit && split == 3));
  if (lane == 0) { s_red[wid][0] = v0; s_red[wid][1] = v1; s_red[wid][2] = v2; s_red[wid][3] = v3; }
  // The LAST wave of the block to finish sums the four partials in fixed order
  // (deterministic) -- no end-of-block barrier, so short rows do not wait for the
  // block's longest row (power-law degrees).
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  int prev = 0;
  if (lane == 0) prev = atomicAdd(&s_cnt, 1);
  prev = __shfl(prev, 0, 64);
  if (prev == (int)(blockDim.x >> 6) - 1) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (lane < 4) {
      stats[(size_t)blk * 68 + lane] = (s_red[0][lane] + s_red[1][lane]) + (s_red[2][lane] + s_red[3][lane]);
    }
    stats[(size_t)blk * 68 + 4 + lane] = (s_cls[0][lane] + s_cls[1][lane]) + (s_cls[2][lane] + s_cls[3][lane]);
  }
}

// H = dropout(relu(P + b)) in place on a bf16 [rows][ld] matrix (F valid columns,
// F % 32 == 0).  Dropout keeps with probability 1-p (p quantised to 1/256) and scales
// kept units by 1/(1-p).  Mask of element (row, n), n = 32 t + 8 g + 4 h + i: position
// q = 4 g + i of the draw of (row, t, h) (cgnn_common.h drop_draw / drop_keep16) -- the
// layout in which the fused MFMA kernel (gnn_dense.hip) holds the values, so both
// produce the same mask.
// One thread per (row, 32-column group, half): 16 values, one draw.
__global__ __launch_bounds__(256) void bias_relu_dropout_kernel(
    uint16_t* __restrict__ Hm, const float* __restrict__ bias, long rows, int F, int ld, float p,
    uint32_t k0, uint32_t k1, uint32_t step, uint32_t thr8, uint32_t row0) {
  const int per_row = F / 16;                                // (F/32 groups) x 2 halves
  const uint32_t tpr = (uint32_t)per_row;
  const uint32_t rpb = blockDim.x / tpr;
  const uint32_t rloc = threadIdx.x / tpr;
  const long row = (long)blockIdx.y * rpb + rloc;
  if (rloc >= rpb || row >= rows) return;
  const int k = (int)(threadIdx.x - rloc * tpr);
  const int t = k >> 1, h = k & 1;
  const float scale = 1.f / (1.f - p);
  uint32_t m = 0xffffu;
  if (thr8 > 0)
    m = drop_keep16(drop_draw(row0 + (uint32_t)row, t, h, step, k0, k1, drop_bit_mode(thr8)), t, thr8,
                    drop_bit_mode(thr8));
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int n0 = 32 * t + 8 * g + 4 * h;
    uint2* ptr = reinterpret_cast<uint2*>(Hm + row * ld + n0);
    const uint2 hv = *ptr;
    float v[4] = {__uint_as_float(hv.x << 16), __uint_as_float(hv.x & 0xffff0000u),
                  __uint_as_float(hv.y << 16), __uint_as_float(hv.y & 0xffff0000u)};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = i + 4 * g;
      float x = fmaxf(v[i] + bias[n0 + i], 0.f);
      if (thr8 > 0) x = ((m >> q) & 1u) ? x * scale : 0.f;
      v[i] = x;
    }
    *ptr = make_uint2(f32_to_bf16_rne(v[0]) | (f32_to_bf16_rne(v[1]) << 16),
                      f32_to_bf16_rne(v[2]) | (f32_to_bf16_rne(v[3]) << 16));
  }
}

// dP = dH * [H > 0] * 1/(1-p)  (H already holds relu + dropout, so H > 0 iff the unit was
// active and kept).  bf16 in/out, in place on dH.
__global__ __launch_bounds__(256) void relu_dropout_bwd_kernel(
    uint16_t* __restrict__ dH, const uint16_t* __restrict__ Hm, long n8, float scale) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n8) return;
  float g[8], h[8];
  bf16x8_to_f32(reinterpret_cast<const uint4*>(dH)[idx], g);
  bf16x8_to_f32(reinterpret_cast<const uint4*>(Hm)[idx], h);
#pragma unroll
  for (int q = 0; q < 8; ++q) g[q] = h[q] > 0.f ? g[q] * scale : 0.f;
  reinterpret_cast<uint4*>(dH)[idx] = f32x8_to_bf16(g);
}

// PyTorch-semantics Adam (bias-corrected, eps inside) with optional decoupled
// weight decay, over one flat fp32 parameter buffer.  t = *step + 1.  done (optional,
// zero): the block whose arrival is counted last stores *step = t and re-zeroes *done.
// Every block has read *step into a register before its arrival (the barrier waits for
// the load), so no fence is needed -- only the count.
__global__ void gnn_adam_kernel(float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
                                const float* __restrict__ g, int n, float lr, float b1, float b2,
                                float eps, float wd, int* __restrict__ step, unsigned* __restrict__ done,
                                int step_done) {
  // step_done: *step was already advanced for this update (a slab_sum bump), t = *step
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const float t = (float)(*step + (step_done ? 0 : 1));
  if (i < n) {
    const float gi = g[i];
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float mh = mi / (1.f - powf(b1, t));
    const float vh = vi / (1.f - powf(b2, t));
    p[i] -= lr * (mh / (sqrtf(vh) + eps) + wd * p[i]);
  }
  if (!done) return;
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(done, 1u) == gridDim.x - 1) {
    *step = (int)t;
    *done = 0u;
  }
}

__global__ void cast_bf16_kernel(const float* __restrict__ src, uint16_t* __restrict__ dst, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (uint16_t)f32_to_bf16_rne(src[i]);
}

// ---------------------------------------------------------------- launchers
// Gathers unrolled 8 rows deep, the next chunk's column ids requested during the current
// chunk's gathers (round 4: headline +1-5 %, arxiv +1.2 %, profiles/r04_spmm).  Measured
// alternatives, kept out: 16 deep (2.21 vs 2.05 ms on the products layer 1, round 5: 82
// VGPRs, 5 waves / SIMD), 4 deep (slower on the products shape), and round 2's
// software-pipelined gather that combined the early column ids with non-temporal index
// loads / output stores and 16 raw rows in flight per lane: 30 % SLOWER (F = 100: 3.43 vs
// 2.64 ms) -- non-temporal stores alone double a store-heavy kernel's time (r04_lin).
template <int L, int U, int RP>
static int spmm_dispatch_u(const int* rowptr, const int* col, const void* X, void* Y, const float* rs,
                         const float* bias, int n_rows, int F, int ldx, int ldy, int xbf, int ybf,
                         int relu, int uc, int wc, const float* init, int ldi, const float* cs, int ir, hipStream_t st) {
  // RP > 0: the short-row kernel, RP rows per sub-group
  constexpr int RPB = 4 * (64 / L) * (RP > 0 ? RP : 1);   // rows per 256-thread block
  dim3 grid((n_rows + RPB - 1) / RPB), block(256);
  if (n_rows <= 0) return 0;
#define CGNN_SPMM(XT, YT, C)                                                                                    \
  do {                                                                                                         \
    if constexpr (RP > 0)                                                                                      \
      hipLaunchKernelGGL((spmm_short_kernel<L, XT, YT, RP, C>), grid, block, 0, st, rowptr, col, X, Y, rs, bias, \
                         n_rows, F, ldx, ldy, relu, uc, wc, init, ldi, cs, ir);                                \
    else                                                                                                       \
      hipLaunchKernelGGL((spmm_kernel<L, XT, YT, U, C>), grid, block, 0, st, rowptr, col, X, Y, rs, bias, n_rows, \
                         F, ldx, ldy, relu, uc, wc, init, ldi, cs, ir);                                        \
  } while (0)
  // element-type codes: 0 fp32, 1 bf16, 2 fp16 (fp16 pairs with itself or with fp32);
  // a column scale is compiled for the same-type pairs only
  if (cs) {
    if (xbf == 1 && ybf == 1) CGNN_SPMM(1, 1, true);
    else if (xbf == 2 && ybf == 2) CGNN_SPMM(2, 2, true);
    else if (xbf == 0 && ybf == 0) CGNN_SPMM(0, 0, true);
    else return -5;
  } else if (xbf == 1 && ybf == 1) CGNN_SPMM(1, 1, false);
  else if (xbf == 1 && ybf == 0) CGNN_SPMM(1, 0, false);
  else if (xbf == 0 && ybf == 1) CGNN_SPMM(0, 1, false);
  else if (xbf == 0 && ybf == 0) CGNN_SPMM(0, 0, false);
  else if (xbf == 2 && ybf == 2) CGNN_SPMM(2, 2, false);
  else if (xbf == 2 && ybf == 0) CGNN_SPMM(2, 0, false);
  else if (xbf == 0 && ybf == 2) CGNN_SPMM(0, 2, false);
  else return -5;
#undef CGNN_SPMM
  return (int)hipGetLastError();
}

template <int L>
static int spmm_dispatch(const int* rowptr, const int* col, const void* X, void* Y, const float* rs,
                         const float* bias, int n_rows, int F, int ldx, int ldy, int xbf, int ybf,
                         int relu, int uc, int wc, const float* init, int ldi, const float* cs, int ir,
                         bool short_rows, hipStream_t st) {
  if (short_rows)
    return spmm_dispatch_u<L, 8, 4>(rowptr, col, X, Y, rs, bias, n_rows, F, ldx, ldy, xbf, ybf, relu, uc, wc, init,
                                    ldi, cs, ir, st);
  return spmm_dispatch_u<L, 8, 0>(rowptr, col, X, Y, rs, bias, n_rows, F, ldx, ldy, xbf, ybf, relu, uc, wc, init,
                                  ldi, cs, ir, st);
}

// one launch writing output columns [0, wcols) of its base (wcols <= 512)
static int spmm_launch(const int* rowptr, const int* col, const void* X, void* Y, const float* rs,
                       const float* bias, int n_rows, int F, int ldx, int ldy, int xbf, int ybf, int relu,
                       int uc, int wc, const float* init, int ldi, const float* cs, int ir, bool sr,
                       hipStream_t st) {
  const int w = std::max(F, wc);
  if (w <= 64) return spmm_dispatch<8>(rowptr, col, X, Y, rs, bias, n_rows, F, ldx, ldy, xbf, ybf, relu, uc, wc, init, ldi, cs, ir, sr, st);
  if (w <= 128) return spmm_dispatch<16>(rowptr, col, X, Y, rs, bias, n_rows, F, ldx, ldy, xbf, ybf, relu, uc, wc, init, ldi, cs, ir, sr, st);
  if (w <= 256) return spmm_dispatch<32>(rowptr, col, X, Y, rs, bias, n_rows, F, ldx, ldy, xbf, ybf, relu, uc, wc, init, ldi, cs, ir, sr, st);
  if (w <= 512) return spmm_dispatch<64>(rowptr, col, X, Y, rs, bias, n_rows, F, ldx, ldy, xbf, ybf, relu, uc, wc, init, ldi, cs, ir, sr, st);
  return -1;
}

extern "C" int gnn_launch_spmm(const int* rowptr, const int* col, const void* X, void* Y,
                               const float* rscale, const float* bias, int n_rows, int F, int ldx,
                               int ldy, int xbf, int ybf, int relu, int unit_col, const float* init, int ldi,
                               const float* cscale, int init_rows, int short_rows, hipStream_t st) {
  // short_rows: the rows average <= 2 entries (spmm_short_kernel)
  constexpr int slab = 512;
  const bool sr = short_rows != 0;
  if ((ldx % 8) || (ldy % 8) || F > ldx || F > ldy) return -3;
  if (init_rows < 0) init_rows = n_rows;
  if (ldy <= slab && F <= slab)
    return spmm_launch(rowptr, col, X, Y, rscale, bias, n_rows, F, ldx, ldy, xbf, ybf, relu, unit_col, ldy, init,
                       ldi, cscale, init_rows, sr, st);
  // wide rows: column slabs of 512 output columns (16-byte aligned offsets), one launch
  // each; the last slabs also write the padding / ones columns up to ldy
  const size_t xs = xbf ? 2 : 4, ys = ybf ? 2 : 4;   // bf16 and fp16 are both 2 bytes
  for (int c0 = 0; c0 < ldy; c0 += slab) {
    const int fc = std::max(0, std::min(slab, F - c0));
    const int wc = std::min(slab, ldy - c0);
    const int rc = spmm_launch(rowptr, col, (const char*)X + (fc ? c0 * xs : 0), (char*)Y + c0 * ys, rscale,
                               bias && fc ? bias + c0 : nullptr, n_rows, fc, ldx, ldy, xbf, ybf, relu,
                               unit_col >= 0 ? unit_col - c0 : -1, wc, init && fc ? init + c0 : nullptr, ldi,
                               cscale, init_rows, sr, st);
    if (rc) return rc;
  }
  return 0;
}

// out[map[c]] = sum_r P[r][c] (fixed order).  stage: fp32 [>= G * W] scratch for the
// first of two passes when S is large (G groups of rows), or null for one pass.
extern "C" int gnn_slab_sum(const float* P, long S, int W, float* stage, int G, float* out, const int* map,
                            int* bump, hipStream_t st) {
  if (S <= 0 || W <= 0) return -3;
  const unsigned gx = (unsigned)((W + 63) / 64);
  if (stage && G > 1) {
    const long per = (S + G - 1) / G;
    hipLaunchKernelGGL(slab_sum_kernel, dim3(gx, (unsigned)G), dim3(256), 0, st, P, S, W, per, stage,
                       (const int*)nullptr, (int*)nullptr);
    hipLaunchKernelGGL(slab_sum_kernel, dim3(gx, 1), dim3(1024), 0, st, (const float*)stage, (long)G, W,
                       (long)G, out, map, bump);
  } else {
    hipLaunchKernelGGL(slab_sum_kernel, dim3(gx, 1), dim3(S >= 64 ? 1024 : 256), 0, st, P, S, W, S, out, map, bump);
  }
  return (int)hipGetLastError();
}

// n_long rows of one wave each, then the others 8 per wave; 4 waves per block
extern "C" int gnn_spmm_ce_blocks(int n_rows, int n_long) {
  const long waves = (long)n_long + (n_rows - n_long + 7) / 8;
  return (int)((waves + 3) / 4);
}

extern "C" int gnn_launch_bias_relu_dropout(void* H, const float* bias, long rows, int F, int ld,
                                            float p, uint32_t k0, uint32_t k1, uint32_t step,
                                            uint32_t row0, hipStream_t st) {
  if (F % 32 || F > ld || ld % 8 || F / 16 > 256) return -3;
  const int rpb = 256 / (F / 16);
  const long gy = (rows + rpb - 1) / rpb;
  if (gy > 2147483647L) return -4;
  const uint32_t thr8 = (uint32_t)std::min(255.0, std::floor((double)p * 256.0 + 0.5));
  hipLaunchKernelGGL(bias_relu_dropout_kernel, dim3(1, (unsigned)gy), dim3(256), 0, st,
                     (uint16_t*)H, bias, rows, F, ld, p, k0, k1, step, thr8, row0);
  return (int)hipGetLastError();
}

extern "C" int gnn_launch_relu_dropout_bwd(void* dH, const void* H, long n, float p, hipStream_t st) {
  if (n % 8) return -3;
  const long n8 = n / 8;
  hipLaunchKernelGGL(relu_dropout_bwd_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, st,
                     (uint16_t*)dH, (const uint16_t*)H, n8, 1.f / (1.f - p));
  return (int)hipGetLastError();
}

extern "C" int gnn_launch_spmm_ce(const int* rowptr, const int* col, const void* Z,
                                  const float* rscale, const float* bias, const int* labels,
                                  const uint8_t* mask, float* stats, void* G, const float* init, int ldi,
                                  int n_rows, int C, int ld, int mode, float inv_count, const int* gslot,
                                  int n_long, hipStream_t st) {
  if (C > 64 || (ld % 8) || C > ld || n_long < 0 || n_long > n_rows) return -3;
  hipLaunchKernelGGL(spmm_ce_kernel, dim3(gnn_spmm_ce_blocks(n_rows, n_long)), dim3(256), 0, st, rowptr, col,
                     Z, rscale, bias, labels, mask, stats, G, n_rows, C, ld, mode, inv_count, init, ldi, gslot,
                     n_long);
  return (int)hipGetLastError();
}

extern "C" int gnn_launch_ell_build(const int* rowptr, const int* col, int* ell, int n_rows, hipStream_t st) {
  if (n_rows <= 0) return 0;
  hipLaunchKernelGGL(ell_build_kernel, dim3((n_rows + 255) / 256), dim3(256), 0, st, rowptr, col, ell, n_rows);
  return (int)hipGetLastError();
}

extern "C" int gnn_launch_spmm_ell(const int* ell, const int* col, const void* X, void* Y, const float* rscale,
                                   int n_rows, int F, int ldx, int ldy, long n_x_rows, const int* long_rows,
                                   int n_long, hipStream_t st) {
  if (F > 64 || ldx % 8 || ldy % 8 || F > ldx) return -3;
  if (n_rows <= 0) return 0;
  // the pipelined kernel addresses X and Y through buffer descriptors (32-bit offsets);
  // larger tables (or a caller without the long-row list) take the one-shot kernel
  if (long_rows && n_x_rows * ldx * 2 < (1l << 31) && (long)n_rows * ldy * 2 < (1l << 31)) {
    const int groups = (n_rows + 7) / 8;
    const int blocks = std::max(1, std::min((groups + 3) / 4, device_cus() * 8));
    hipLaunchKernelGGL(spmm_ell_pipe_kernel, dim3(blocks), dim3(256), 0, st, ell, col, long_rows, n_long,
                       (const uint16_t*)X, (uint16_t*)Y, rscale, n_rows, F, ldx, ldy,
                       (uint32_t)(n_x_rows * ldx * 2));
  } else {
    hipLaunchKernelGGL(spmm_ell_kernel, dim3((n_rows + 31) / 32), dim3(256), 0, st, ell, col, (const uint16_t*)X,
                       (uint16_t*)Y, rscale, n_rows, F, ldx, ldy);
  }
  return (int)hipGetLastError();
}

// rows of at most max_deg <= 8 entries, bf16 X / Y, F <= 128 (spmm_fan_pipe_kernel);
// other shapes take gnn_launch_spmm.  n_x_rows: rows of X (bounds of its descriptor)
extern "C" int gnn_launch_spmm_fan(const int* rowptr, const int* col, const void* X, void* Y, const float* rscale,
                                   int n_rows, int F, int ldx, int ldy, long n_x_rows, long nnz, int max_deg,
                                   hipStream_t st) {
  if ((ldx % 8) || (ldy % 8) || F > ldx || F > ldy) return -3;
  if (n_rows <= 0) return 0;
  if (max_deg > 8 || F > 128 || ldy > 128 || n_x_rows * ldx * 2 >= (1l << 31) || nnz * 4 >= (1l << 31) ||
      (long)n_rows * ldy * 2 >= (1l << 31))
    return gnn_launch_spmm(rowptr, col, X, Y, rscale, nullptr, n_rows, F, ldx, ldy, 1, 1, 0, -1, nullptr, 0,
                           nullptr, -1, 0, st);
  const int groups = (n_rows + 3) / 4;
  const int blocks = std::max(1, std::min((groups + 3) / 4, device_cus() * 8));
  hipLaunchKernelGGL(spmm_fan_pipe_kernel, dim3(blocks), dim3(256), 0, st, rowptr, col, (const uint16_t*)X,
                     (uint16_t*)Y, rscale, n_rows, F, ldx, ldy, (uint32_t)(n_x_rows * ldx * 2), (uint32_t)(nnz * 4));
  return (int)hipGetLastError();
}

extern "C" int gnn_launch_adam(float* p, float* m, float* v, const float* g, int n, float lr,
                               float b1, float b2, float eps, float wd, int* step, unsigned* done,
                               int step_done, hipStream_t st) {
  hipLaunchKernelGGL(gnn_adam_kernel, dim3((n + 255) / 256), dim3(256), 0, st, p, m, v, g, n, lr, b1,
                     b2, eps, wd, step, step_done ? nullptr : done, step_done);
  return (int)hipGetLastError();
}

extern "C" int gnn_launch_cast_bf16(const float* src, void* dst, long n, hipStream_t st) {
  hipLaunchKernelGGL(cast_bf16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src,
                     (uint16_t*)dst, n);
  return (int)hipGetLastError();
}
