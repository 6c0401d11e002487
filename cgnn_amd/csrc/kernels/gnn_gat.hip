// Graph attention (GAT) message passing on CSR for MI355X -- GNN track, not in
// the reference (SURVEY §0 Phase B: "SDDMM edge-softmax").
//
// Per edge (i <- j) and head k:  e_ijk = LeakyReLU(s_dst[i,k] + s_src[j,k], 0.2)
//   alpha_ijk = softmax over j in N(i) of e_ijk,  out[i,k,:] = sum_j alpha_ijk Wh[j,k,:]
//
//   gat_fwd_kernel      one CSR row per L-lane sub-group, each lane 8 features of one
//                       head; single pass with an ONLINE softmax (running max and
//                       rescaled sum), so the edge scores are never materialised;
//                       writes out and the per-(row, head) log-sum-exp.
//   gat_bwd_row_kernel  per row i: alpha recomputed from the lse, the SDDMM
//                       dalpha_ij = <dout_i, Wh_j> (head-group shuffle reduction),
//                       de = alpha (dalpha - <dout_i, out_i>), LeakyReLU'; the row
//                       term d s_dst[i] in registers; per (row, head) statistics
//                       (s_dst, lse, D) for the column half -- nothing per edge.
//   gat_bwd_col_kernel  per source row j over the TRANSPOSED CSR: alpha and the
//                       score gradient recomputed from the gathered dout_i and row
//                       statistics against the own row Wh_j: dWh[j] = sum alpha_ij
//                       dout_i, d s_src[j] = sum dscore_ij -- gathers only, no atomics.
// Everything fp32, fixed summation orders (deterministic).
#include "cgnn_common.h"
#include <algorithm>
#include <cmath>

using namespace cgnn;

namespace {

__device__ __forceinline__ void ld8(const float* p, float* f) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
// 8 gathered values of a row stored fp32 (WT = 0) or bf16 (WT = 1), returned as fp32
template <int WT>
__device__ __forceinline__ void ldg8(const void* base, size_t off, float* f) {
  if (WT == 1) {
    const uint4 v = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(base) + off);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f[2 * q] = __uint_as_float(w[q] << 16);
      f[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
    }
  } else {
    ld8(reinterpret_cast<const float*>(base) + off, f);
  }
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

}  // namespace

// L lanes per row (L * 8 >= K * Fh), G = Fh / 8 lanes per head.
constexpr int EB = 4;   // edges per online-softmax step (gat_fwd_kernel)

template <int L, int G, int WT>
__global__ __launch_bounds__(256) void gat_fwd_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col, const void* __restrict__ Wh,
    const float* __restrict__ s_src, const float* __restrict__ s_dst, float* __restrict__ out,
    float* __restrict__ lse, int n, int K, int HF) {
  constexpr int RPW = 64 / L;
  const int lane = threadIdx.x & 63, sub = lane / L, sl = lane - sub * L;
  const int row = (xcd_remap(blockIdx.x, gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RPW + sub;
  const bool rv = row < n;
  const int f0 = 8 * sl;
  const bool fv = rv && f0 < HF;
  const int k = fv ? f0 / (8 * G) : 0;
  const float sd = fv ? s_dst[(size_t)row * K + k] : 0.f;
  float m = -INFINITY, l = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int e0 = rv ? rowptr[row] : 0, e1 = rv ? rowptr[row + 1] : 0;
  for (int e = e0; e < e1; e += L) {
    const int myj = (e + sl < e1) ? col[e + sl] : 0;
    const int cnt = min(L, e1 - e);
    // EB edges per step: their rows are requested together, and the online softmax
    // rescales once per step (EB + 1 exponentials instead of 2 EB)
    for (int q = 0; q < cnt; q += EB) {
      int j[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) j[u] = __shfl(myj, sub * L + min(q + u, L - 1), 64);
      if (fv) {
        float w[EB][8], sc[EB];
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          ldg8<WT>(Wh, (size_t)j[u] * HF + f0, w[u]);
          sc[u] = s_src[(size_t)j[u] * K + k];
        }
        float mn = m;
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          sc[u] = (q + u < cnt) ? leaky(sd + sc[u]) : -INFINITY;
          mn = fmaxf(mn, sc[u]);
        }
        const float a = __expf(m - mn);
        float b[EB];
#pragma unroll
        for (int u = 0; u < EB; ++u) b[u] = __expf(sc[u] - mn);
#pragma unroll
        for (int f = 0; f < 8; ++f) {
          float t = acc[f] * a;
#pragma unroll
          for (int u = 0; u < EB; ++u) t = fmaf(b[u], w[u][f], t);
          acc[f] = t;
        }
        float ls = l * a;
#pragma unroll
        for (int u = 0; u < EB; ++u) ls += b[u];
        l = ls;
        m = mn;
      }
    }
  }
  if (!fv) return;
  const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] *= inv;
  st8(out + (size_t)row * HF + f0, acc);
  if (f0 % (8 * G) == 0) lse[(size_t)row * K + k] = l > 0.f ? m + __logf(l) : 0.f;
}

// Row half of the backward, per destination row i and head k: D_ik = <dout_ik, out_ik>,
// and over the row's edges the SDDMM da_ij = <dout_i, Wh_j>, the attention weight
// recomputed from the lse, ds_ij = alpha_ij (da_ij - D_ik) LeakyReLU'; their row sum is
// d s_dst[i,k].  Nothing is stored per edge: the column half recomputes alpha and ds
// from the row statistics rs[i][k] = (s_dst, lse, D, 0) (one 16-B gather per edge and
// head) -- no [nnz, K] fp32 arrays, no edge permutation.
template <int L, int G, int WT>
__global__ __launch_bounds__(256) void gat_bwd_row_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col, const void* __restrict__ Wh,
    const float* __restrict__ s_src, const float* __restrict__ s_dst, const float* __restrict__ out,
    const float* __restrict__ lse, const float* __restrict__ dout, float4* __restrict__ rstat,
    float* __restrict__ ds_dst, int n, int K, int HF) {
  constexpr int RPW = 64 / L;
  const int lane = threadIdx.x & 63, sub = lane / L, sl = lane - sub * L;
  const int row = (xcd_remap(blockIdx.x, gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RPW + sub;
  const bool rv = row < n;
  const int f0 = 8 * sl;
  const bool fv = rv && f0 < HF;
  const int k = fv ? f0 / (8 * G) : 0;
  const bool lead = fv && (f0 % (8 * G) == 0);
  float go[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float sd = 0.f, ls = 0.f;
  if (fv) {
    ld8(dout + (size_t)row * HF + f0, go);
    ld8(out + (size_t)row * HF + f0, o);
    sd = s_dst[(size_t)row * K + k];
    ls = lse[(size_t)row * K + k];
  }
  float dd = 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u) dd = fmaf(go[u], o[u], dd);
  dd = group_sum<G>(dd);                       // D_ik = <dout_ik, out_ik>
  float dsd = 0.f;
  const int e0 = rv ? rowptr[row] : 0, e1 = rv ? rowptr[row + 1] : 0;
  for (int e = e0; e < e1; e += L) {
    const int myj = (e + sl < e1) ? col[e + sl] : 0;
    const int cnt = min(L, e1 - e);
    for (int q = 0; q < cnt; q += EB) {          // EB edges' rows requested together
      int j[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) j[u] = __shfl(myj, sub * L + min(q + u, L - 1), 64);
      float w[EB][8], raw[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        if (fv) {
          ldg8<WT>(Wh, (size_t)j[u] * HF + f0, w[u]);
          raw[u] = sd + s_src[(size_t)j[u] * K + k];
        } else {
#pragma unroll
          for (int f = 0; f < 8; ++f) w[u][f] = 0.f;
          raw[u] = 0.f;
        }
      }
      float da[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        float d = 0.f;
#pragma unroll
        for (int f = 0; f < 8; ++f) d = fmaf(go[f], w[u][f], d);
        da[u] = d;
      }
#pragma unroll
      for (int off = 1; off < G; off <<= 1) {   // SDDMM: dalpha_ij = <dout_i, Wh_j>
#pragma unroll
        for (int u = 0; u < EB; ++u) da[u] += __shfl_xor(da[u], off, 64);
      }
      if (fv) {
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          if (q + u < cnt) {
            const float al = __expf(leaky(raw[u]) - ls);
            dsd += al * (da[u] - dd) * (raw[u] > 0.f ? 1.f : 0.2f);
          }
        }
      }
    }
  }
  if (lead) {
    ds_dst[(size_t)row * K + k] = dsd;
    rstat[(size_t)row * K + k] = make_float4(sd, ls, dd, 0.f);
  }
}

// Column half, per SOURCE row j of the transposed CSR (the destinations i that read j,
// in increasing order) and head k: the own row Wh_j and s_src[j,k] stay in registers;
// per edge the gathered dout_i and rs[i][k] give alpha_ij = exp(LeakyReLU(s_dst_i +
// s_src_j) - lse_i) and ds_ij = alpha_ij (<dout_i, Wh_j> - D_i) LeakyReLU':
// dWh_j = sum_i alpha_ij dout_i, d s_src[j,k] = sum_i ds_ij -- gathers only, no atomics,
// fixed order.  Rows are independent, so a row range is a pointer offset (halo rounds).
template <int L, int G, int WT>
__global__ __launch_bounds__(256) void gat_bwd_col_kernel(
    const int* __restrict__ rowptr_t, const int* __restrict__ col_t, const void* __restrict__ Wh,
    const float* __restrict__ s_src, const float4* __restrict__ rstat, const void* __restrict__ dout,
    float* __restrict__ dWh, float* __restrict__ ds_src, int n, int K, int HF) {
  constexpr int RPW = 64 / L;
  const int lane = threadIdx.x & 63, sub = lane / L, sl = lane - sub * L;
  const int row = (xcd_remap(blockIdx.x, gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RPW + sub;
  const bool rv = row < n;
  const int f0 = 8 * sl;
  const bool fv = rv && f0 < HF;
  const int k = fv ? f0 / (8 * G) : 0;
  float wj[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float ss = 0.f;
  if (fv) {
    ldg8<WT>(Wh, (size_t)row * HF + f0, wj);
    ss = s_src[(size_t)row * K + k];
  }
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float dss = 0.f;
  const int e0 = rv ? rowptr_t[row] : 0, e1 = rv ? rowptr_t[row + 1] : 0;
  for (int e = e0; e < e1; e += L) {
    const int myi = (e + sl < e1) ? col_t[e + sl] : 0;
    const int cnt = min(L, e1 - e);
    for (int q = 0; q < cnt; q += EB) {          // EB edges' rows requested together
      int i[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) i[u] = __shfl(myi, sub * L + min(q + u, L - 1), 64);
      float g[EB][8];
      float4 rs[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        if (fv) {
          ldg8<WT>(dout, (size_t)i[u] * HF + f0, g[u]);
          rs[u] = rstat[(size_t)i[u] * K + k];
        } else {
#pragma unroll
          for (int f = 0; f < 8; ++f) g[u][f] = 0.f;
          rs[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
      float da[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        float d = 0.f;
#pragma unroll
        for (int f = 0; f < 8; ++f) d = fmaf(g[u][f], wj[f], d);
        da[u] = d;
      }
#pragma unroll
      for (int off = 1; off < G; off <<= 1) {
#pragma unroll
        for (int u = 0; u < EB; ++u) da[u] += __shfl_xor(da[u], off, 64);
      }
      if (fv) {
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          if (q + u < cnt) {
            const float raw = rs[u].x + ss;
            const float al = __expf(leaky(raw) - rs[u].y);
            dss += al * (da[u] - rs[u].z) * (raw > 0.f ? 1.f : 0.2f);
#pragma unroll
            for (int f = 0; f < 8; ++f) acc[f] = fmaf(al, g[u][f], acc[f]);
          }
        }
      }
    }
  }
  if (!fv) return;
  st8(dWh + (size_t)row * HF + f0, acc);
  if (f0 % (8 * G) == 0) ds_src[(size_t)row * K + k] = dss;
}

// ---------------------------------------------------------------- launchers
namespace {
template <template <int, int> class, int, int> struct Unused {};

int lanes_for(int HF) {
  const int c = (HF + 7) / 8;
  return c <= 8 ? 8 : c <= 16 ? 16 : c <= 32 ? 32 : c <= 64 ? 64 : -1;
}
}  // namespace

#define GAT_DISPATCH(KERNEL, WT, ...)                                                                  \
  do {                                                                                             \
    /* one head: its group is the row's whole sub-group (lanes past HF add 0) */                  \
    const int L = lanes_for(HF), G = K == 1 ? L : Fh / 8;                                          \
    if (L < 0 || Fh % 8 || HF != K * Fh) return -3;                                                \
    const int rpb = 4 * (64 / L);                                                                  \
    dim3 grid((n + rpb - 1) / rpb), block(256);                                                    \
    switch (L * 100 + G) {                                                                         \
      case 801: hipLaunchKernelGGL((KERNEL<8, 1, WT>), grid, block, 0, st, __VA_ARGS__); break;        \
      case 802: hipLaunchKernelGGL((KERNEL<8, 2, WT>), grid, block, 0, st, __VA_ARGS__); break;        \
      case 804: hipLaunchKernelGGL((KERNEL<8, 4, WT>), grid, block, 0, st, __VA_ARGS__); break;        \
      case 808: hipLaunchKernelGGL((KERNEL<8, 8, WT>), grid, block, 0, st, __VA_ARGS__); break;        \
      case 1601: hipLaunchKernelGGL((KERNEL<16, 1, WT>), grid, block, 0, st, __VA_ARGS__); break;      \
      case 1602: hipLaunchKernelGGL((KERNEL<16, 2, WT>), grid, block, 0, st, __VA_ARGS__); break;      \
      case 1604: hipLaunchKernelGGL((KERNEL<16, 4, WT>), grid, block, 0, st, __VA_ARGS__); break;      \
      case 1608: hipLaunchKernelGGL((KERNEL<16, 8, WT>), grid, block, 0, st, __VA_ARGS__); break;      \
      case 1616: hipLaunchKernelGGL((KERNEL<16, 16, WT>), grid, block, 0, st, __VA_ARGS__); break;    \
      case 3202: hipLaunchKernelGGL((KERNEL<32, 2, WT>), grid, block, 0, st, __VA_ARGS__); break;      \
      case 3204: hipLaunchKernelGGL((KERNEL<32, 4, WT>), grid, block, 0, st, __VA_ARGS__); break;      \
      case 3208: hipLaunchKernelGGL((KERNEL<32, 8, WT>), grid, block, 0, st, __VA_ARGS__); break;      \
      case 3216: hipLaunchKernelGGL((KERNEL<32, 16, WT>), grid, block, 0, st, __VA_ARGS__); break;    \
      case 3232: hipLaunchKernelGGL((KERNEL<32, 32, WT>), grid, block, 0, st, __VA_ARGS__); break;    \
      case 6404: hipLaunchKernelGGL((KERNEL<64, 4, WT>), grid, block, 0, st, __VA_ARGS__); break;      \
      case 6408: hipLaunchKernelGGL((KERNEL<64, 8, WT>), grid, block, 0, st, __VA_ARGS__); break;      \
      case 6416: hipLaunchKernelGGL((KERNEL<64, 16, WT>), grid, block, 0, st, __VA_ARGS__); break;    \
      case 6464: hipLaunchKernelGGL((KERNEL<64, 64, WT>), grid, block, 0, st, __VA_ARGS__); break;    \
      default: return -1;                                                                          \
    }                                                                                              \
    return (int)hipGetLastError();                                                                 \
  } while (0)

// Wh [n][HF], s_src / s_dst / lse [n][K], HF = K * Fh, Fh % 8 == 0; HF <= 512.
// wbf: the gathered matrix (Wh in the forward and the row backward, dout in the
// column backward) is stored bf16 -- half the bytes of the edge gathers, values
// widened to fp32 in registers (all arithmetic and every other operand fp32).
extern "C" int gnn_launch_gat_fwd(const int* rowptr, const int* col, const void* Wh, const float* s_src,
                                  const float* s_dst, float* out, float* lse, int n, int K, int Fh, int wbf,
                                  hipStream_t st) {
  const int HF = K * Fh;
  if (wbf) GAT_DISPATCH(gat_fwd_kernel, 1, rowptr, col, Wh, s_src, s_dst, out, lse, n, K, HF);
  GAT_DISPATCH(gat_fwd_kernel, 0, rowptr, col, Wh, s_src, s_dst, out, lse, n, K, HF);
}

// rstat: [n][K] float4 (s_dst, lse, D, 0), written for the column half
extern "C" int gnn_launch_gat_bwd_row(const int* rowptr, const int* col, const void* Wh, const float* s_src,
                                      const float* s_dst, const float* out, const float* lse,
                                      const float* dout, float* rstat, float* ds_dst, int n, int K, int Fh, int wbf,
                                      hipStream_t st) {
  const int HF = K * Fh;
  float4* rs = reinterpret_cast<float4*>(rstat);
  if (wbf)
    GAT_DISPATCH(gat_bwd_row_kernel, 1, rowptr, col, Wh, s_src, s_dst, out, lse, dout, rs, ds_dst, n, K, HF);
  GAT_DISPATCH(gat_bwd_row_kernel, 0, rowptr, col, Wh, s_src, s_dst, out, lse, dout, rs, ds_dst, n, K, HF);
}

// Wh / s_src / dWh / ds_src: rows of the launch's source range; rstat / dout: all
// destination rows.  wbf: Wh and the gathered dout are bf16.
extern "C" int gnn_launch_gat_bwd_col(const int* rowptr_t, const int* col_t, const void* Wh, const float* s_src,
                                      const float* rstat, const void* dout, float* dWh, float* ds_src, int n, int K,
                                      int Fh, int wbf, hipStream_t st) {
  const int HF = K * Fh;
  const float4* rs = reinterpret_cast<const float4*>(rstat);
  if (wbf) GAT_DISPATCH(gat_bwd_col_kernel, 1, rowptr_t, col_t, Wh, s_src, rs, dout, dWh, ds_src, n, K, HF);
  GAT_DISPATCH(gat_bwd_col_kernel, 0, rowptr_t, col_t, Wh, s_src, rs, dout, dWh, ds_src, n, K, HF);
}

// ============================================================================
// Dense-side kernels of the fused GAT epoch (gnn/gat_fused.py).  The projections
// [Wh | s_src | s_dst] = h [W | W a_src | W a_dst] run on the MFMA lin_* kernels
// (gnn_linear.hip); these cover everything between them and the aggregation:
//
//   gat_act_fwd     h = bf16(dropout(elu(out + b)))        (hidden layer output)
//   gat_act_bwd     dout = dh * mask * elu'(out + b), fp32 + bf16 copy, and the
//                   bias gradient as per-block column partials
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
__device__ __forceinline__ uint32_t bf16u(float x) { return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)x); }
__device__ __forceinline__ uint2 pack4bf(const float* v) {
  return make_uint2(bf16u(v[0]) | (bf16u(v[1]) << 16), bf16u(v[2]) | (bf16u(v[3]) << 16));
}
__device__ __forceinline__ void dropout_words(uint32_t* w, uint32_t thr8, uint32_t grow, int t, int h,
                                              uint32_t step, uint32_t k0, uint32_t k1) {
  w[0] = w[1] = w[2] = w[3] = 0xffffffffu;
  if (thr8 > 0) {
    const u32x4 r = philox4x32_10(u32x4{grow, (uint32_t)(2 * t + h), step, RNG_DROPOUT}, k0, k1);
    w[0] = r.x; w[1] = r.y; w[2] = r.z; w[3] = r.w;
  }
}
__device__ __forceinline__ bool kept(const uint32_t* w, int q, uint32_t thr8) {
  return thr8 == 0 || ((w[q >> 2] >> (8 * (q & 3))) & 0xffu) >= thr8;
}
}  // namespace

__global__ __launch_bounds__(256) void gat_act_fwd_kernel(const float* __restrict__ out, const float* __restrict__ bias,
                                                          uint16_t* __restrict__ H, int ldh, long n, int F, float p,
                                                          uint32_t k0, uint32_t k1, uint32_t step,
                                                          const int* __restrict__ stepp, uint32_t thr8, uint32_t row0) {
  if (stepp) step = (uint32_t)*stepp;
  const int tpr = F / 16;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long row = gid / tpr;
  if (row >= n) return;
  const int k = (int)(gid - row * tpr), t = k >> 1, h = k & 1;
  const float scale = thr8 > 0 ? 1.f / (1.f - p) : 1.f;
  uint32_t w[4];
  dropout_words(w, thr8, row0 + (uint32_t)row, t, h, step, k0, k1);
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int c0 = 32 * t + 8 * g + 4 * h;
    const float4 o = *reinterpret_cast<const float4*>(out + (size_t)row * F + c0);
    const float ov[4] = {o.x, o.y, o.z, o.w};
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float z = ov[i] + bias[c0 + i];
      const float e = z > 0.f ? z : expm1f(z);
      v[i] = kept(w, i + 4 * g, thr8) ? e * scale : 0.f;
    }
    *reinterpret_cast<uint2*>(H + (size_t)row * ldh + c0) = pack4bf(v);
  }
}

// grid-stride over rows with a fixed grid: thread slot k = tid % (F/16) is constant,
// so every thread keeps the bias-gradient sums of its 16 columns in registers;
// blocks write [gridDim.x][F] partials (rows of a block summed in a fixed order)
__global__ __launch_bounds__(256) void gat_act_bwd_kernel(const uint16_t* __restrict__ dH, int ldh,
                                                          const float* __restrict__ out, const float* __restrict__ bias,
                                                          float* __restrict__ dout, uint16_t* __restrict__ doutb,
                                                          float* __restrict__ bpart, long n, int F, float p, uint32_t k0,
                                                          uint32_t k1, uint32_t step, const int* __restrict__ stepp,
                                                          uint32_t thr8, uint32_t row0) {
  __shared__ float red[256][17];
  if (stepp) step = (uint32_t)*stepp;
  const int tpr = F / 16, rpb = 256 / tpr;
  const int rl = threadIdx.x / tpr, k = threadIdx.x - rl * tpr, t = k >> 1, h = k & 1;
  const float scale = thr8 > 0 ? 1.f / (1.f - p) : 1.f;
  float bs[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) bs[q] = 0.f;
  if (rl < rpb) {
    for (long row = (long)blockIdx.x * rpb + rl; row < n; row += (long)gridDim.x * rpb) {
      uint32_t w[4];
      dropout_words(w, thr8, row0 + (uint32_t)row, t, h, step, k0, k1);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c0 = 32 * t + 8 * g + 4 * h;
        const float4 o = *reinterpret_cast<const float4*>(out + (size_t)row * F + c0);
        const uint2 hv = *reinterpret_cast<const uint2*>(dH + (size_t)row * ldh + c0);
        const float ov[4] = {o.x, o.y, o.z, o.w};
        const float gv[4] = {__uint_as_float(hv.x << 16), __uint_as_float(hv.x & 0xffff0000u),
                             __uint_as_float(hv.y << 16), __uint_as_float(hv.y & 0xffff0000u)};
        float d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float z = ov[i] + bias[c0 + i];
          d[i] = kept(w, i + 4 * g, thr8) ? gv[i] * scale * (z > 0.f ? 1.f : __expf(z)) : 0.f;
          bs[4 * g + i] += d[i];
        }
        *reinterpret_cast<float4*>(dout + (size_t)row * F + c0) = make_float4(d[0], d[1], d[2], d[3]);
        if (doutb) *reinterpret_cast<uint2*>(doutb + (size_t)row * F + c0) = pack4bf(d);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) red[threadIdx.x][q] = bs[q];
  __syncthreads();
  if (threadIdx.x < tpr) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      float s = 0.f;
      for (int r = 0; r < rpb; ++r) s += red[r * tpr + threadIdx.x][q];
      const int c = 32 * t + 8 * (q >> 2) + 4 * h + (q & 3);
      bpart[(size_t)blockIdx.x * F + c] = s;
    }
  }
}

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
int act_grid() {
  int dev = 0, cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
  return 4 * cus;
}
uint32_t thr8_of(float p) { return (uint32_t)std::min(255.0, std::floor((double)p * 256.0 + 0.5)); }
}  // namespace

extern "C" int gnn_launch_gat_act_fwd(const float* out, const float* bias, void* H, int ldh, long n, int F, float p,
                                      uint32_t k0, uint32_t k1, uint32_t step, const int* stepp, uint32_t row0,
                                      hipStream_t st) {
  if (F % 32 || ldh < F || ldh % 4) return -3;
  if (n <= 0) return 0;
  const long threads = n * (F / 16);
  hipLaunchKernelGGL(gat_act_fwd_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, out, bias,
                     (uint16_t*)H, ldh, n, F, p, k0, k1, step, stepp, thr8_of(p), row0);
  return (int)hipGetLastError();
}

extern "C" int gnn_gat_act_bwd_blocks() { return act_grid(); }

// bpart: [gnn_gat_act_bwd_blocks()][F] fp32 scratch; db (optional): [F]
extern "C" int gnn_launch_gat_act_bwd(const void* dH, int ldh, const float* out, const float* bias, float* dout,
                                      void* doutb, float* bpart, float* db, long n, int F, float p, uint32_t k0,
                                      uint32_t k1, uint32_t step, const int* stepp, uint32_t row0, hipStream_t st) {
  if (F % 32 || F > 4096 || ldh < F || ldh % 4) return -3;
  const int nb = act_grid();
  hipLaunchKernelGGL(gat_act_bwd_kernel, dim3(nb), dim3(256), 0, st, (const uint16_t*)dH, ldh, out, bias, dout,
                     (uint16_t*)doutb, bpart, n, F, p, k0, k1, step, stepp, thr8_of(p), row0);
  if (db)
    hipLaunchKernelGGL(gat_colsum_kernel, dim3((F + 31) / 32), dim3(256), 0, st, bpart, (long)nb, F, 1.f, db);
  return (int)hipGetLastError();
}

extern "C" int gnn_gat_row_ce_waves() { return 4 * act_grid(); }

// stats_part: [waves][4], bpart: [waves][C] scratch; stats (optional): [4] (sums);
// db (optional): [C]; dZ / dZb (optional, training): [n][ldz] fp32 / bf16
extern "C" int gnn_launch_gat_row_ce(const float* Z, int ldz, const float* bias, int C, const int* y,
                                     const uint8_t* mask, float inv_count, float* dZ, void* dZb, float* stats_part,
                                     float* bpart, float* stats, float* db, long n, hipStream_t st) {
  if (C <= 0 || C > 256 || ldz < C) return -3;
  const int nb = act_grid(), nw = 4 * nb;
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
