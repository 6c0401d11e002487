// Graph attention (GAT) message passing on CSR for MI355X -- GNN track, not in
// the reference (SURVEY §0 Phase B: "SDDMM edge-softmax").
//
// Per edge (i <- j) and head k:  e_ijk = LeakyReLU(s_dst[i,k] + s_src[j,k], 0.2)
//   alpha_ijk = softmax over j in N(i) of e_ijk,  out[i,k,:] = sum_j alpha_ijk Wh[j,k,:]
//
//   gat_fwd_kernel   one CSR row per L-lane sub-group, each lane 8 features of one
//                    head; single pass with an ONLINE softmax (running max and rescaled
//                    sums), so the edge scores are never materialised; writes out, the
//                    per-(row, head) log-sum-exp and (training) the LeakyReLU split q
//                    that turns the row half of the backward into a per-row product;
//                    optionally the hidden layer's activation (ELU + Philox dropout).
//   gat_row_kernel   per row: D = <dout, out>, d s_dst = -0.8 <dout, q>, the statistics
//                    (s_dst, lse, D) for the column half; optionally fused with the
//                    activation backward (dropout mask, ELU', bias gradient) -- no gather.
//   gat_col_kernel   per source row j over the TRANSPOSED CSR: alpha and the score
//                    gradient recomputed from the gathered dout_i and row statistics
//                    against the own row Wh_j: dWh[j] = sum alpha_ij dout_i, d s_src[j] =
//                    sum dscore_ij -- gathers only, no atomics; fp32 out, or bf16 straight
//                    into the projection-gradient operand dy.
// Arithmetic fp32, fixed summation orders (deterministic).
#include "cgnn_common.h"
#include <algorithm>
#include <cmath>

using namespace cgnn;

namespace {

__device__ __forceinline__ void ld8(const float* p, float* f) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
__device__ __forceinline__ void st8(float* p, const float* f) {
  *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
}
// sum over the G lanes of a head group (G = Fh/8, a power of two, groups aligned)
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int off = 1; off < G; off <<= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ float leaky(float x) { return x > 0.f ? x : 0.2f * x; }

// ---------------------------------------------------------------- aggregation
// Row layout of every aggregation kernel: L lanes per CSR row (L * 8 >= K * Fh), each
// lane 8 consecutive features of one head, G = Fh / 8 lanes per head (a power of two,
// groups aligned; one head: the row's whole sub-group).  Gathers run in batches of EC
// edges whose rows are all requested before any is consumed (EC loads of 16 B per lane
// in flight), and the next chunk's column indices are fetched one chunk ahead.
//
// LeakyReLU split.  With n_ij = [raw_ij <= 0] (the 0.2-slope side), the row half of
// the backward is
//   d s_dst[i] = sum_j alpha_ij (dalpha_ij - D_i) (1 - 0.8 n_ij)
//              = (<dout_i, out_i> - D_i) - 0.8 (<dout_i, out-_i> - D_i c-_i)
// with out-_i = sum_j n_ij alpha_ij Wh_j, c-_i = sum_j n_ij alpha_ij and D_i =
// <dout_i, out_i> (sum alpha = 1): the first bracket vanishes, so
//   d s_dst[i] = -0.8 <dout_i, q_i>,   q_i = out-_i - c-_i out_i,
// a per-row product.  The forward accumulates out- beside out (same gathered rows, one
// more FMA per feature) and stores q, so the row half needs no gather at all.
template <int WT>
__device__ __forceinline__ void ld_raw(const void* base, size_t off, uint4* r) {
  if (WT == 1) {
    r[0] = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(base) + off);
  } else {
    const uint4* p = reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(base) + off);
    r[0] = p[0];
    r[1] = p[1];
  }
}
// the same from a lane's byte base and a row's byte offset (one 64-bit multiply-add per
// gathered row: j * row_bytes + lane base)
template <int WT>
__device__ __forceinline__ void ld_raw_b(const char* lane_base, uint32_t j, uint32_t row_bytes, uint4* r) {
  const uint4* p = reinterpret_cast<const uint4*>(lane_base + (uint64_t)j * row_bytes);
  r[0] = p[0];
  if (WT == 0) r[1] = p[1];
}
template <int WT>
__device__ __forceinline__ void raw_f32(const uint4* r, float* f) {
  if (WT == 1) {
    const uint32_t w[4] = {r[0].x, r[0].y, r[0].z, r[0].w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f[2 * q] = __uint_as_float(w[q] << 16);
      f[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
    }
  } else {
    const uint32_t w[8] = {r[0].x, r[0].y, r[0].z, r[0].w, r[1].x, r[1].y, r[1].z, r[1].w};
#pragma unroll
    for (int q = 0; q < 8; ++q) f[q] = __uint_as_float(w[q]);
  }
}
__device__ __forceinline__ uint32_t bf16u(float x) { return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)x); }
__device__ __forceinline__ uint4 f8_bf16(const float* v) {
  return make_uint4(bf16u(v[0]) | (bf16u(v[1]) << 16), bf16u(v[2]) | (bf16u(v[3]) << 16),
                    bf16u(v[4]) | (bf16u(v[5]) << 16), bf16u(v[6]) | (bf16u(v[7]) << 16));
}
// 8 values stored as WT (bf16 / fp32)
template <int WT>
__device__ __forceinline__ void st_w8(void* base, size_t off, const float* v) {
  if (WT == 1) *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(base) + off) = f8_bf16(v);
  else st8(reinterpret_cast<float*>(base) + off, v);
}
template <int WT>
__device__ __forceinline__ void ld_w8(const void* base, size_t off, float* v) {
  uint4 r[2];
  ld_raw<WT>(base, off, r);
  raw_f32<WT>(r, v);
}

// Dropout convention of ops.dropout_keep_mask / the fused GCN kernels (cgnn_common.h
// drop_draw / drop_keep16): column c = 32 t + 8 g + 4 h + i is decided by position
// q = 4 g + i of the draw of (row, t, h).  A lane's 8 columns f0..f0+7 (f0 % 8 == 0) take
// positions 4 g .. 4 g + 3 of the draws for h = 0 (first 4) and h = 1 (last 4).
__device__ __forceinline__ void keep8(bool* kp, uint32_t thr8, uint32_t grow, int f0, uint32_t step, uint32_t k0,
                                      uint32_t k1) {
  if (thr8 == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) kp[i] = true;
    return;
  }
  const int t = f0 >> 5, g = (f0 & 31) >> 3;
  const bool bm = drop_bit_mode(thr8);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t m = drop_keep16(drop_draw(grow, t, h, step, k0, k1, bm), t, thr8, bm);
#pragma unroll
    for (int i = 0; i < 4; ++i) kp[4 * h + i] = (m >> (4 * g + i)) & 1u;
  }
}

}  // namespace

struct GatFwdArgs {
  const int* rowptr;
  const int* col;
  const void* Wh;          // [n_cols][HF] WT
  const float* s_src;      // [n_cols][K]
  const float* s_dst;      // [*][K], row dst_rows[i] (or i)
  const int* dst_rows;     // optional
  float* out;              // [n][HF] fp32
  float* lse;              // [n][K]
  void* q;                 // optional [n][HF] WT: out- - c- out (training)
  // optional fused hidden activation H = bf16(dropout(elu(out + bias))) (HF % 32 == 0)
  const float* bias;
  uint16_t* H;
  int ldh;
  float p;
  uint32_t k0, k1, step, thr8, row0;
  const int* stepp;
  int n, K, HF;
};

// (Occupancy of the two gather kernels: they are latency-bound, yet a register cap
// that buys waves per SIMD measured no gain; the compiler's allocation is kept.)
#define GAT_WAVES_ATTR

// Scores run in the log2 domain (LeakyReLU is positively homogeneous: leaky(c x) =
// c leaky(x) for c > 0), so every exponential is one v_exp_f32.
constexpr float L2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
__device__ __forceinline__ float leaky2(float x) { return fmaxf(x, 0.2f * x); }

template <int L, int G, int WT, int EC>
__global__ __launch_bounds__(256) GAT_WAVES_ATTR void gat_fwd_kernel(GatFwdArgs a) {
  constexpr int RPW = 64 / L;
  const int lane = threadIdx.x & 63, sub = lane / L, sl = lane - sub * L;
  const int row = (xcd_remap_chunked<64>(blockIdx.x, gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RPW + sub;
  const bool rv = row < a.n;
  const int f0 = 8 * sl, K = a.K, HF = a.HF;
  const bool fv = rv && f0 < HF;
  const int k = fv ? f0 / (8 * G) : 0;
  const int srow = rv ? (a.dst_rows ? a.dst_rows[row] : row) : 0;
  const float sd = fv ? a.s_dst[(size_t)srow * K + k] * L2E : 0.f;
  const char* wh_lane = reinterpret_cast<const char*>(a.Wh) + (size_t)f0 * (WT == 1 ? 2 : 4);
  const uint32_t wh_row = (uint32_t)HF * (WT == 1 ? 2 : 4);
  const char* ss_lane = reinterpret_cast<const char*>(a.s_src) + (size_t)k * 4;
  const uint32_t ss_row = (uint32_t)K * 4;
  float m = -INFINITY, l = 0.f, ln = 0.f;
  float acc[8], accn[8];
#pragma unroll
  for (int f = 0; f < 8; ++f) acc[f] = accn[f] = 0.f;
  const int e0 = rv ? a.rowptr[row] : 0, e1 = rv ? a.rowptr[row + 1] : 0;
  int nj = (e0 + sl < e1) ? a.col[e0 + sl] : 0;
  for (int e = e0; e < e1; e += L) {
    const int myj = nj;
    nj = (e + L + sl < e1) ? a.col[e + L + sl] : 0;       // next chunk's indices, one chunk ahead
    const int cnt = min(L, e1 - e);
    for (int q0 = 0; q0 < cnt; q0 += EC) {
      // the batch's rows: edges past the row's end re-read the batch's first row (a cache
      // hit) and get weight 0, so the loads issue back to back without branches
      int js[EC];
      const int jf = __shfl(myj, sub * L + q0, 64);
#pragma unroll
      for (int u = 0; u < EC; ++u) {
        const int j = __shfl(myj, sub * L + q0 + u, 64);
        js[u] = q0 + u < cnt ? j : jf;
      }
      if (fv) {
        uint4 raw[EC][WT == 1 ? 1 : 2];
        float sc[EC];
#pragma unroll
        for (int u = 0; u < EC; ++u) {
          ld_raw_b<WT>(wh_lane, (uint32_t)js[u], wh_row, raw[u]);
          sc[u] = *reinterpret_cast<const float*>(ss_lane + (uint64_t)(uint32_t)js[u] * ss_row);
        }
        float mx = m;
#pragma unroll
        for (int u = 0; u < EC; ++u) {
          sc[u] = (q0 + u < cnt) ? leaky2(fmaf(sc[u], L2E, sd)) : -INFINITY;
          mx = fmaxf(mx, sc[u]);
        }
        const float sa = __builtin_amdgcn_exp2f(m - mx);
        l *= sa;
        ln *= sa;
#pragma unroll
        for (int f = 0; f < 8; ++f) {
          acc[f] *= sa;
          accn[f] *= sa;
        }
#pragma unroll
        for (int u = 0; u < EC; ++u) {
          const float b = __builtin_amdgcn_exp2f(sc[u] - mx);
          const float bn = sc[u] <= 0.f ? b : 0.f;
          float w[8];
          raw_f32<WT>(raw[u], w);
#pragma unroll
          for (int f = 0; f < 8; ++f) {
            acc[f] = fmaf(b, w[f], acc[f]);
            accn[f] = fmaf(bn, w[f], accn[f]);
          }
          l += b;
          ln += bn;
        }
        m = mx;
      }
    }
  }
  if (!fv) return;
  const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
  for (int f = 0; f < 8; ++f) acc[f] *= inv;
  st8(a.out + (size_t)row * HF + f0, acc);
  if (f0 % (8 * G) == 0) a.lse[(size_t)row * K + k] = l > 0.f ? (m + __log2f(l)) * LN2 : 0.f;
  if (a.q) {
    const float cn = ln * inv;
    float qv[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) qv[f] = fmaf(accn[f], inv, -cn * acc[f]);
    st_w8<WT>(a.q, (size_t)row * HF + f0, qv);
  }
  if (a.H) {
    const uint32_t step = a.stepp ? (uint32_t)*a.stepp : a.step;
    bool kp[8];
    keep8(kp, a.thr8, a.row0 + (uint32_t)row, f0, step, a.k0, a.k1);
    const float scale = a.thr8 > 0 ? 1.f / (1.f - a.p) : 1.f;
    float hv[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      const float z = acc[f] + a.bias[f0 + f];
      const float e = z > 0.f ? z : expm1f(z);
      hv[f] = kp[f] ? e * scale : 0.f;
    }
    *reinterpret_cast<uint4*>(a.H + (size_t)row * a.ldh + f0) = f8_bf16(hv);
  }
}

// Row statistics of the backward (per destination row i, head k): D_ik = <dout_ik, out_ik>
// and d s_dst[i,k] = -0.8 <dout_ik, q_ik>; rstat[i][k] = (s_dst, lse, D, 0) for the column
// half (s_dst and lse scaled by log2 e).  dout / q as WT.  ds_dst goes to an fp32 [*][K] array (row dst_rows[i] or i) and /
// or straight into column HF + K + k of the bf16 GEMM operand dy (same row).
//
// act (hidden layer): dout is first made from the layer output's gradient dH, dout =
// dH * dropout mask * elu'(out + bias), stored as WT, and the bias gradient is summed per
// block (bpart[block][HF], fixed order) -- the activation backward and the row half in
// one pass.  Fixed grid, rows grid-strided (the per-lane column sums stay in registers).
struct GatRowArgs {
  const void* dout;        // act: the output rows' gradient dH (bf16, ldh); else dout (WT)
  int ldh;
  const float* out;
  const void* q;
  const float* lse;
  const float* s_dst;
  const int* dst_rows;
  float4* rstat;
  float* ds_dst;
  uint16_t* dy;
  int ldy;
  // act only
  void* dout_w;            // dout as WT
  const float* bias;
  float* bpart;
  float p;
  uint32_t k0, k1, step, thr8, row0;
  const int* stepp;
  int n, K, HF;
};

template <int L, int G, int WT, bool ACT>
__global__ __launch_bounds__(256) void gat_row_kernel(GatRowArgs a) {
  constexpr int RPW = 64 / L;
  __shared__ float red[4][64][8];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, sub = lane / L, sl = lane - sub * L;
  const int f0 = 8 * sl, K = a.K, HF = a.HF;
  const bool fl = f0 < HF;
  const int k = fl ? f0 / (8 * G) : 0;
  const bool lead = fl && (f0 % (8 * G) == 0);
  const long rows_per_pass = (long)gridDim.x * 4 * RPW;
  const uint32_t step = ACT ? (a.stepp ? (uint32_t)*a.stepp : a.step) : 0u;
  const float scale = (ACT && a.thr8 > 0) ? 1.f / (1.f - a.p) : 1.f;
  float bsum[8];
#pragma unroll
  for (int f = 0; f < 8; ++f) bsum[f] = 0.f;
  float bv[8];
  if (ACT) {
#pragma unroll
    for (int f = 0; f < 8; ++f) bv[f] = fl ? a.bias[f0 + f] : 0.f;
  }
  for (long base = ((long)blockIdx.x * 4 + wv) * RPW; base < a.n; base += rows_per_pass) {
    const long row = base + sub;
    const bool fv = row < a.n && fl;
    float d[8], o[8], qv[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) d[f] = o[f] = qv[f] = 0.f;
    if (fv) {
      ld8(a.out + (size_t)row * HF + f0, o);
      ld_w8<WT>(a.q, (size_t)row * HF + f0, qv);
      if (ACT) {
        float dh[8];
        ld_w8<1>(a.dout, (size_t)row * a.ldh + f0, dh);
        bool kp[8];
        keep8(kp, a.thr8, a.row0 + (uint32_t)row, f0, step, a.k0, a.k1);
#pragma unroll
        for (int f = 0; f < 8; ++f) {
          const float z = o[f] + bv[f];
          d[f] = kp[f] ? dh[f] * scale * (z > 0.f ? 1.f : __expf(z)) : 0.f;
          bsum[f] += d[f];
        }
        st_w8<WT>(a.dout_w, (size_t)row * HF + f0, d);
        if (WT == 1) {                 // the column half gathers the rounded values: use them here too
          uint4 r[1];
          r[0] = f8_bf16(d);
          raw_f32<1>(r, d);
        }
      } else {
        ld_w8<WT>(a.dout, (size_t)row * HF + f0, d);
      }
    }
    float dd = 0.f, dq = 0.f;
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      dd = fmaf(d[f], o[f], dd);
      dq = fmaf(d[f], qv[f], dq);
    }
    dd = group_sum<G>(dd);
    dq = group_sum<G>(dq);
    if (fv && f0 % (8 * G) == 0) {
      const long srow = a.dst_rows ? a.dst_rows[row] : row;
      const float dsd = -0.8f * dq;
      // (s_dst, lse) in log2 units for the column half's exp2
      a.rstat[(size_t)row * K + k] =
          make_float4(a.s_dst[(size_t)srow * K + k] * L2E, a.lse[(size_t)row * K + k] * L2E, dd, 0.f);
      if (a.ds_dst) a.ds_dst[(size_t)srow * K + k] = dsd;
      if (a.dy) a.dy[(size_t)srow * a.ldy + HF + K + k] = (uint16_t)bf16u(dsd);
    }
  }
  (void)lead;
  if (ACT) {
    // bias gradient: lanes with equal sl hold the same columns; sum the RPW sub-groups
    // (fixed xor order), then the 4 waves in order
#pragma unroll
    for (int off = L; off < 64; off <<= 1)
#pragma unroll
      for (int f = 0; f < 8; ++f) bsum[f] += __shfl_xor(bsum[f], off, 64);
    if (sub == 0) {
#pragma unroll
      for (int f = 0; f < 8; ++f) red[wv][sl][f] = bsum[f];
    }
    __syncthreads();
    if (wv == 0 && sub == 0 && fl) {
#pragma unroll
      for (int f = 0; f < 8; ++f)
        a.bpart[(size_t)blockIdx.x * HF + f0 + f] = (red[0][sl][f] + red[1][sl][f]) + (red[2][sl][f] + red[3][sl][f]);
    }
  }
}

// Column half, per SOURCE row j of the transposed CSR (the destinations i that read j,
// in increasing order) and head k: the own row Wh_j and s_src[j,k] stay in registers;
// per edge the gathered dout_i and rstat[i][k] give alpha_ij = exp(LeakyReLU(s_dst_i +
// s_src_j) - lse_i) and ds_ij = alpha_ij (<dout_i, Wh_j> - D_i) LeakyReLU':
// dWh_j = sum_i alpha_ij dout_i, d s_src[j,k] = sum_i ds_ij -- gathers only, no atomics,
// fixed order.  Output: fp32 dWh / ds_src (rows of the launch), or bf16 straight into
// columns [0, HF + K) of the GEMM operand dy (row j, stride ldy).  Rows are independent,
// so a row range is a pointer offset (halo rounds).
struct GatColArgs {
  const int* rowptr_t;
  const int* col_t;
  const void* Wh;
  const float* s_src;
  const float4* rstat;
  const void* dout;        // WT
  float* dWh;
  float* ds_src;
  uint16_t* dy;
  int ldy;
  int n, K, HF;
};

template <int L, int G, int WT, int EC>
__global__ __launch_bounds__(256) GAT_WAVES_ATTR void gat_col_kernel(GatColArgs a) {
  constexpr int RPW = 64 / L;
  const int lane = threadIdx.x & 63, sub = lane / L, sl = lane - sub * L;
  const int row = (xcd_remap_chunked<64>(blockIdx.x, gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RPW + sub;
  const bool rv = row < a.n;
  const int f0 = 8 * sl, K = a.K, HF = a.HF;
  const bool fv = rv && f0 < HF;
  const int k = fv ? f0 / (8 * G) : 0;
  float wj[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float ss = 0.f;
  if (fv) {
    ld_w8<WT>(a.Wh, (size_t)row * HF + f0, wj);
    ss = a.s_src[(size_t)row * K + k] * L2E;
  }
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float dss = 0.f;
  const char* do_lane = reinterpret_cast<const char*>(a.dout) + (size_t)f0 * (WT == 1 ? 2 : 4);
  const uint32_t do_row = (uint32_t)HF * (WT == 1 ? 2 : 4);
  const char* rs_lane = reinterpret_cast<const char*>(a.rstat) + (size_t)k * 16;
  const uint32_t rs_row = (uint32_t)K * 16;
  const int e0 = rv ? a.rowptr_t[row] : 0, e1 = rv ? a.rowptr_t[row + 1] : 0;
  int ni = (e0 + sl < e1) ? a.col_t[e0 + sl] : 0;
  for (int e = e0; e < e1; e += L) {
    const int myi = ni;
    ni = (e + L + sl < e1) ? a.col_t[e + L + sl] : 0;
    const int cnt = min(L, e1 - e);
    for (int q0 = 0; q0 < cnt; q0 += EC) {
      int is[EC];
      const int i_f = __shfl(myi, sub * L + q0, 64);
#pragma unroll
      for (int u = 0; u < EC; ++u) {
        const int i = __shfl(myi, sub * L + q0 + u, 64);
        is[u] = q0 + u < cnt ? i : i_f;
      }
      uint4 raw[EC][WT == 1 ? 1 : 2];
      float4 rs[EC];
      if (fv) {
#pragma unroll
        for (int u = 0; u < EC; ++u) {
          ld_raw_b<WT>(do_lane, (uint32_t)is[u], do_row, raw[u]);
          rs[u] = *reinterpret_cast<const float4*>(rs_lane + (uint64_t)(uint32_t)is[u] * rs_row);
        }
      } else {
#pragma unroll
        for (int u = 0; u < EC; ++u) {
          raw[u][0] = make_uint4(0u, 0u, 0u, 0u);
          if (WT == 0) raw[u][WT == 1 ? 0 : 1] = make_uint4(0u, 0u, 0u, 0u);
          rs[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
      float da[EC];
#pragma unroll
      for (int u = 0; u < EC; ++u) {
        float g[8];
        raw_f32<WT>(raw[u], g);
        float d = 0.f;
#pragma unroll
        for (int f = 0; f < 8; ++f) d = fmaf(g[f], wj[f], d);
        da[u] = d;
      }
#pragma unroll
      for (int off = 1; off < G; off <<= 1) {
#pragma unroll
        for (int u = 0; u < EC; ++u) da[u] += __shfl_xor(da[u], off, 64);
      }
      if (fv) {
#pragma unroll
        for (int u = 0; u < EC; ++u) {
          const float raw2 = rs[u].x + ss;                       // log2 units
          const float al = q0 + u < cnt ? __builtin_amdgcn_exp2f(leaky2(raw2) - rs[u].y) : 0.f;
          dss = fmaf(al * (da[u] - rs[u].z), raw2 > 0.f ? 1.f : 0.2f, dss);
          float g[8];
          raw_f32<WT>(raw[u], g);
#pragma unroll
          for (int f = 0; f < 8; ++f) acc[f] = fmaf(al, g[f], acc[f]);
        }
      }
    }
  }
  if (!fv) return;
  const bool lead = f0 % (8 * G) == 0;
  if (a.dy) {
    *reinterpret_cast<uint4*>(a.dy + (size_t)row * a.ldy + f0) = f8_bf16(acc);
    if (lead) a.dy[(size_t)row * a.ldy + HF + k] = (uint16_t)bf16u(dss);
  } else {
    st8(a.dWh + (size_t)row * HF + f0, acc);
    if (lead) a.ds_src[(size_t)row * K + k] = dss;
  }
}

// ============================================================================
// Dense-side kernels of the fused GAT epoch (gnn/gat_fused.py).  The projections
// [Wh | s_src | s_dst] = h [W | W a_src | W a_dst] run on the MFMA lin_* kernels
// (gnn_linear.hip); these cover everything between them and the aggregation:
//
//   (the hidden activation and its backward are fused into gat_fwd_kernel and
//   gat_row_kernel above)
//   gat_row_ce      logits = out + b: log-softmax, NLL, accuracy counts, and
//                   dlogits (train rows; zero elsewhere), per-wave partials of the
//                   loss statistics and of the bias gradient
//   gat_pack_grad   dy = bf16([dWh | ds_src | ds_dst]) -- the gradient of the
//                   projection output, the operand of lin_bwd_weight / lin_bwd_data
//   gat_colsum      fixed-order sum of the partials (deterministic, no atomics)
//
// Dropout mask: the convention of ops.dropout_keep_mask / the fused GCN kernels --
// thread (row, t, h) owns columns 32t + 8g + 4h + i (g, i < 4) and one Philox draw
// keyed (row0 + row, 2t + h, step), byte (i + 4g) of it, kept if >= thr8.
// ============================================================================
namespace {
__device__ __forceinline__ uint2 pack4bf(const float* v) {
  return make_uint2(bf16u(v[0]) | (bf16u(v[1]) << 16), bf16u(v[2]) | (bf16u(v[3]) << 16));
}
}  // namespace

// one wave per row (grid-stride, fixed grid); lane owns columns lane + 64 q, q < CP.
// stats[wave][4] = (sum of train NLL, correct train, correct valid, correct test);
// bpart[wave][C] = sum over the wave's train rows of dlogits (the bias gradient)
template <int CP>
__global__ __launch_bounds__(256) void gat_row_ce_kernel(const float* __restrict__ Z, int ldz,
                                                         const float* __restrict__ bias, int C,
                                                         const int* __restrict__ y, const uint8_t* __restrict__ mask,
                                                         float inv_count, float* __restrict__ dZ,
                                                         uint16_t* __restrict__ dZb, float* __restrict__ stats,
                                                         float* __restrict__ bpart, long n) {
  const int lane = threadIdx.x & 63;
  const long gw = (long)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (long)gridDim.x * 4;
  float bsum[CP], st[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < CP; ++q) bsum[q] = 0.f;
  for (long row = gw; row < n; row += nw) {
    const int m = mask[row], yi = y[row];
    float z[CP];
    float mx = -INFINITY, zy = 0.f;
    int arg = 0x7fffffff;
#pragma unroll
    for (int q = 0; q < CP; ++q) {
      const int c = lane + 64 * q;
      z[q] = c < C ? Z[(size_t)row * ldz + c] + bias[c] : -INFINITY;
      if (z[q] > mx) { mx = z[q]; arg = c; }          // first maximum of this lane
      if (c == yi) zy = z[q];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {           // (max, lowest index) over the wave
      const float om = __shfl_xor(mx, off, 64);
      const int oa = __shfl_xor(arg, off, 64);
      if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
      zy += __shfl_xor(zy, off, 64);
    }
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < CP; ++q) s += lane + 64 * q < C ? __expf(z[q] - mx) : 0.f;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    const float lse = mx + __logf(s);
    if (m == 1) st[0] += lse - zy;
    if (m >= 1 && m <= 3 && arg == yi) st[m] += 1.f;
    if (dZ || dZb) {
#pragma unroll
      for (int q = 0; q < CP; ++q) {
        const int c = lane + 64 * q;
        float d = 0.f;
        if (m == 1 && c < C) {
          d = (__expf(z[q] - lse) - (c == yi ? 1.f : 0.f)) * inv_count;
          bsum[q] += d;
        }
        if (c < ldz) {
          if (dZ) dZ[(size_t)row * ldz + c] = d;
          if (dZb) dZb[(size_t)row * ldz + c] = (uint16_t)bf16u(d);
        }
      }
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) stats[gw * 4 + i] = st[i];
  }
  if (bpart) {
#pragma unroll
    for (int q = 0; q < CP; ++q) {
      const int c = lane + 64 * q;
      if (c < C) bpart[gw * C + c] = bsum[q];
    }
  }
}

// dy[row][c] = bf16(c < HF ? dWh[row][c] : c < HF + K ? ds_src[row][c - HF] :
//                   c < HF + 2K ? ds_dst[row][c - HF - K] : 0), c < ldy; 4 columns per thread
__global__ __launch_bounds__(256) void gat_pack_grad_kernel(const float* __restrict__ dWh,
                                                            const float* __restrict__ ds_src,
                                                            const float* __restrict__ ds_dst, int HF, int K,
                                                            uint16_t* __restrict__ dy, int ldy, long n) {
  const int tpr = ldy / 4;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long row = gid / tpr;
  if (row >= n) return;
  const int c0 = 4 * (int)(gid - row * tpr);
  float v[4];
  if (c0 + 4 <= HF) {
    const float4 a = *reinterpret_cast<const float4*>(dWh + (size_t)row * HF + c0);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = c0 + e;
      v[e] = c < HF ? dWh[(size_t)row * HF + c]
           : c < HF + K ? ds_src[(size_t)row * K + (c - HF)]
           : c < HF + 2 * K ? ds_dst[(size_t)row * K + (c - HF - K)] : 0.f;
    }
  }
  *reinterpret_cast<uint2*>(dy + (size_t)row * ldy + c0) = pack4bf(v);
}

// out[c] = scale * sum_{r < rows} part[r][c] in a fixed order: 32 columns per block,
// the rows split over 8 lane groups, then the 8 partials summed in order
__global__ __launch_bounds__(256) void gat_colsum_kernel(const float* __restrict__ part, long rows, int cols,
                                                         float scale, float* __restrict__ out) {
  __shared__ float s[8][33];
  const int e = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + e;
  float acc = 0.f;
  if (c < cols)
    for (long r = grp; r < rows; r += 8) acc += part[(size_t)r * cols + c];
  s[grp][e] = acc;
  __syncthreads();
  if (grp == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) t += s[q][e];
    out[c] = t * scale;
  }
}

namespace {
int row_ce_grid() {
  int dev = 0, cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
  return 4 * cus;
}
}  // namespace

extern "C" int gnn_gat_row_ce_waves() { return 4 * row_ce_grid(); }

// stats_part: [waves][4], bpart: [waves][C] scratch; stats (optional): [4] (sums);
// db (optional): [C]; dZ / dZb (optional, training): [n][ldz] fp32 / bf16
extern "C" int gnn_launch_gat_row_ce(const float* Z, int ldz, const float* bias, int C, const int* y,
                                     const uint8_t* mask, float inv_count, float* dZ, void* dZb, float* stats_part,
                                     float* bpart, float* stats, float* db, long n, hipStream_t st) {
  if (C <= 0 || C > 256 || ldz < C) return -3;
  const int nb = row_ce_grid(), nw = 4 * nb;
  const int cp = (C + 63) / 64;
  float* bp = (dZ || dZb) ? bpart : nullptr;
  auto zb = (uint16_t*)dZb;
  switch (cp) {
    case 1: hipLaunchKernelGGL(gat_row_ce_kernel<1>, dim3(nb), dim3(256), 0, st, Z, ldz, bias, C, y, mask, inv_count, dZ, zb, stats_part, bp, n); break;
    case 2: hipLaunchKernelGGL(gat_row_ce_kernel<2>, dim3(nb), dim3(256), 0, st, Z, ldz, bias, C, y, mask, inv_count, dZ, zb, stats_part, bp, n); break;
    case 3: hipLaunchKernelGGL(gat_row_ce_kernel<3>, dim3(nb), dim3(256), 0, st, Z, ldz, bias, C, y, mask, inv_count, dZ, zb, stats_part, bp, n); break;
    default: hipLaunchKernelGGL(gat_row_ce_kernel<4>, dim3(nb), dim3(256), 0, st, Z, ldz, bias, C, y, mask, inv_count, dZ, zb, stats_part, bp, n); break;
  }
  if (stats) hipLaunchKernelGGL(gat_colsum_kernel, dim3(1), dim3(256), 0, st, stats_part, (long)nw, 4, 1.f, stats);
  if (db && bp) hipLaunchKernelGGL(gat_colsum_kernel, dim3((C + 31) / 32), dim3(256), 0, st, bpart, (long)nw, C, 1.f, db);
  return (int)hipGetLastError();
}

extern "C" int gnn_launch_gat_pack_grad(const float* dWh, const float* ds_src, const float* ds_dst, int HF, int K,
                                        void* dy, int ldy, long n, hipStream_t st) {
  if (ldy % 4 || HF % 4 || ldy < HF + 2 * K) return -3;
  if (n <= 0) return 0;
  const long threads = n * (ldy / 4);
  hipLaunchKernelGGL(gat_pack_grad_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, dWh, ds_src,
                     ds_dst, HF, K, (uint16_t*)dy, ldy, n);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- launchers
namespace {
int lanes_for(int HF) {
  const int c = (HF + 7) / 8;
  return c <= 8 ? 8 : c <= 16 ? 16 : c <= 32 ? 32 : c <= 64 ? 64 : -1;
}
}  // namespace

// edges per gather batch: 2 (measured on the products epoch: 11.80 ms at 2, 12.66 at 4,
// 13.0 at 8, 14.4 at 16 -- the gathers are latency-bound and a wider batch costs more
// occupancy than its rows in flight buy)
constexpr int GAT_EC = 2;
#define GAT_EC_OF(L) ((L) < GAT_EC ? (L) : GAT_EC)

#define GAT_SWITCH(LAUNCH)                                                                  \
  switch (L * 100 + G) {                                                                   \
    case 801: LAUNCH(8, 1); break;                                                         \
    case 802: LAUNCH(8, 2); break;                                                         \
    case 804: LAUNCH(8, 4); break;                                                         \
    case 808: LAUNCH(8, 8); break;                                                         \
    case 1601: LAUNCH(16, 1); break;                                                       \
    case 1602: LAUNCH(16, 2); break;                                                       \
    case 1604: LAUNCH(16, 4); break;                                                       \
    case 1608: LAUNCH(16, 8); break;                                                       \
    case 1616: LAUNCH(16, 16); break;                                                      \
    case 3202: LAUNCH(32, 2); break;                                                       \
    case 3204: LAUNCH(32, 4); break;                                                       \
    case 3208: LAUNCH(32, 8); break;                                                       \
    case 3216: LAUNCH(32, 16); break;                                                      \
    case 3232: LAUNCH(32, 32); break;                                                      \
    case 6404: LAUNCH(64, 4); break;                                                       \
    case 6408: LAUNCH(64, 8); break;                                                       \
    case 6416: LAUNCH(64, 16); break;                                                      \
    case 6464: LAUNCH(64, 64); break;                                                      \
    default: return -1;                                                                    \
  }

// geometry shared by the launchers: one head -> its group is the row's whole sub-group
#define GAT_GEOM                                                                            \
  const int HF = K * Fh;                                                                   \
  const int L = lanes_for(HF), G = K == 1 ? L : Fh / 8;                                    \
  if (L < 0 || Fh % 8 || (K > 1 && (G & (G - 1)))) return -3;                              \
  const int rpb = 4 * (64 / L);

namespace {
uint32_t thr8_of(float p) { return (uint32_t)std::min(255.0, std::floor((double)p * 256.0 + 0.5)); }
int act_grid() {
  int dev = 0, cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
  return 4 * cus;
}
}  // namespace

// Wh [n_cols][HF] (wbf: bf16, else fp32), s_src [n_cols][K], s_dst [*][K] (row dst_rows[i]
// or i); out [n][HF] fp32, lse [n][K]; q (optional, training) [n][HF] like Wh; H
// (optional) the fused hidden activation bf16(dropout(elu(out + bias))) with stride ldh.
extern "C" int gnn_launch_gat_fwd(const int* rowptr, const int* col, const void* Wh, const float* s_src,
                                  const float* s_dst, const int* dst_rows, float* out, float* lse, void* q, int n,
                                  int K, int Fh, int wbf, const float* bias, void* H, int ldh, float p, uint32_t k0,
                                  uint32_t k1, uint32_t step, const int* stepp, uint32_t row0, hipStream_t st) {
  GAT_GEOM
  if (H && (HF % 32 || ldh < HF || !bias)) return -3;
  if (n <= 0) return 0;
  GatFwdArgs a{rowptr, col, Wh, s_src, s_dst, dst_rows, out, lse, q, bias, (uint16_t*)H, ldh, p, k0, k1, step,
               H ? thr8_of(p) : 0u, row0, stepp, n, K, HF};
  dim3 grid((n + rpb - 1) / rpb), block(256);
#define FWD(l, g)                                                                                     \
  if (wbf) hipLaunchKernelGGL((gat_fwd_kernel<l, g, 1, GAT_EC_OF(l)>), grid, block, 0, st, a);        \
  else hipLaunchKernelGGL((gat_fwd_kernel<l, g, 0, GAT_EC_OF(l)>), grid, block, 0, st, a)
  GAT_SWITCH(FWD)
#undef FWD
  return (int)hipGetLastError();
}

extern "C" int gnn_gat_row_blocks() { return act_grid(); }

// act == 0: dout (wbf ? bf16 : fp32) given.  act == 1: dH (bf16, stride ldh) given,
// dout = dH * mask * elu'(out + bias) written to dout_w (wbf ? bf16 : fp32), bias partials
// to bpart [gnn_gat_row_blocks()][HF], db (optional) their fixed-order column sum.
extern "C" int gnn_launch_gat_rows(int act, const void* dout, int ldh, const float* out, const void* q,
                                   const float* lse, const float* s_dst, const int* dst_rows, float* rstat,
                                   float* ds_dst, void* dy, int ldy, void* dout_w, const float* bias, float* bpart,
                                   float* db, float p, uint32_t k0, uint32_t k1, uint32_t step, const int* stepp,
                                   uint32_t row0, int n, int K, int Fh, int wbf, hipStream_t st) {
  GAT_GEOM
  (void)rpb;
  if (act && (HF % 32 || !bias || !bpart || !dout_w)) return -3;
  const int nb = act_grid();
  GatRowArgs a{dout, ldh, out, q, lse, s_dst, dst_rows, reinterpret_cast<float4*>(rstat), ds_dst, (uint16_t*)dy,
               ldy, dout_w, bias, bpart, p, k0, k1, step, act ? thr8_of(p) : 0u, row0, stepp, n, K, HF};
#define ROWS(l, g)                                                                                              \
  if (act) {                                                                                                    \
    if (wbf) hipLaunchKernelGGL((gat_row_kernel<l, g, 1, true>), dim3(nb), dim3(256), 0, st, a);                \
    else hipLaunchKernelGGL((gat_row_kernel<l, g, 0, true>), dim3(nb), dim3(256), 0, st, a);                    \
  } else {                                                                                                      \
    if (wbf) hipLaunchKernelGGL((gat_row_kernel<l, g, 1, false>), dim3(nb), dim3(256), 0, st, a);               \
    else hipLaunchKernelGGL((gat_row_kernel<l, g, 0, false>), dim3(nb), dim3(256), 0, st, a);                   \
  }
  GAT_SWITCH(ROWS)
#undef ROWS
  if (act && db) hipLaunchKernelGGL(gat_colsum_kernel, dim3((HF + 31) / 32), dim3(256), 0, st, bpart, (long)nb, HF, 1.f, db);
  return (int)hipGetLastError();
}

// Wh / s_src / dWh / ds_src / dy: rows of the launch's source range; rstat / dout: all
// destination rows.  dy given: bf16 [dWh | ds_src] into its columns [0, HF + K).
extern "C" int gnn_launch_gat_col(const int* rowptr_t, const int* col_t, const void* Wh, const float* s_src,
                                  const float* rstat, const void* dout, float* dWh, float* ds_src, void* dy, int ldy,
                                  int n, int K, int Fh, int wbf, hipStream_t st) {
  GAT_GEOM
  if (dy && ldy < HF + 2 * K) return -3;
  if (n <= 0) return 0;
  GatColArgs a{rowptr_t, col_t, Wh, s_src, reinterpret_cast<const float4*>(rstat), dout, dWh, ds_src,
               (uint16_t*)dy, ldy, n, K, HF};
  dim3 grid((n + rpb - 1) / rpb), block(256);
#define COL(l, g)                                                                                     \
  if (wbf) hipLaunchKernelGGL((gat_col_kernel<l, g, 1, GAT_EC_OF(l)>), grid, block, 0, st, a);        \
  else hipLaunchKernelGGL((gat_col_kernel<l, g, 0, GAT_EC_OF(l)>), grid, block, 0, st, a)
  GAT_SWITCH(COL)
#undef COL
  return (int)hipGetLastError();
}
