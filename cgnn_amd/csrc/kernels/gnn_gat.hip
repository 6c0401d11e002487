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
//                       term d s_dst[i] accumulates in registers; alpha and the
//                       score gradient are written per edge (one lane per head).
//   gat_bwd_col_kernel  per source row j over the TRANSPOSED CSR (edge permutation
//                       from a stable device sort): dWh[j] = sum alpha_ij dout_i,
//                       d s_src[j] = sum dscore_ij -- gathers only, no atomics.
// Everything fp32, fixed summation orders (deterministic).
#include "cgnn_common.h"
#include <algorithm>

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

template <int L, int G, int WT>
__global__ __launch_bounds__(256) void gat_bwd_row_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col, const void* __restrict__ Wh,
    const float* __restrict__ s_src, const float* __restrict__ s_dst, const float* __restrict__ out,
    const float* __restrict__ lse, const float* __restrict__ dout, float* __restrict__ alpha_e,
    float* __restrict__ dsc_e, float* __restrict__ ds_dst, int n, int K, int HF) {
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
            const float ds = al * (da[u] - dd) * (raw[u] > 0.f ? 1.f : 0.2f);
            dsd += ds;
            if (lead) {
              alpha_e[(size_t)(e + q + u) * K + k] = al;
              dsc_e[(size_t)(e + q + u) * K + k] = ds;
            }
          }
        }
      }
    }
  }
  if (lead) ds_dst[(size_t)row * K + k] = dsd;
}

template <int L, int G, int WT>
__global__ __launch_bounds__(256) void gat_bwd_col_kernel(
    const int* __restrict__ rowptr_t, const int* __restrict__ col_t, const int* __restrict__ perm,
    const float* __restrict__ alpha_e, const float* __restrict__ dsc_e, const void* __restrict__ dout,
    float* __restrict__ dWh, float* __restrict__ ds_src, int n, int K, int HF) {
  constexpr int RPW = 64 / L;
  const int lane = threadIdx.x & 63, sub = lane / L, sl = lane - sub * L;
  const int row = (xcd_remap(blockIdx.x, gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RPW + sub;
  const bool rv = row < n;
  const int f0 = 8 * sl;
  const bool fv = rv && f0 < HF;
  const int k = fv ? f0 / (8 * G) : 0;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float dss = 0.f;
  const int e0 = rv ? rowptr_t[row] : 0, e1 = rv ? rowptr_t[row + 1] : 0;
  for (int e = e0; e < e1; e += L) {
    const int myi = (e + sl < e1) ? col_t[e + sl] : 0;
    const int mye = (e + sl < e1) ? perm[e + sl] : 0;
    const int cnt = min(L, e1 - e);
    for (int q = 0; q < cnt; q += EB) {          // EB edges' rows requested together
      int i[EB], eo[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const int src = sub * L + min(q + u, L - 1);
        i[u] = __shfl(myi, src, 64);
        eo[u] = __shfl(mye, src, 64);
      }
      if (fv) {
        float g[EB][8], al[EB], dsc[EB];
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          ldg8<WT>(dout, (size_t)i[u] * HF + f0, g[u]);
          al[u] = alpha_e[(size_t)eo[u] * K + k];
          dsc[u] = dsc_e[(size_t)eo[u] * K + k];
        }
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          const float a = (q + u < cnt) ? al[u] : 0.f;
#pragma unroll
          for (int f = 0; f < 8; ++f) acc[f] = fmaf(a, g[u][f], acc[f]);
          dss += (q + u < cnt) ? dsc[u] : 0.f;
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

extern "C" int gnn_launch_gat_bwd_row(const int* rowptr, const int* col, const void* Wh, const float* s_src,
                                      const float* s_dst, const float* out, const float* lse,
                                      const float* dout, float* alpha_e, float* dsc_e, float* ds_dst, int n,
                                      int K, int Fh, int wbf, hipStream_t st) {
  const int HF = K * Fh;
  if (wbf)
    GAT_DISPATCH(gat_bwd_row_kernel, 1, rowptr, col, Wh, s_src, s_dst, out, lse, dout, alpha_e, dsc_e, ds_dst,
                 n, K, HF);
  GAT_DISPATCH(gat_bwd_row_kernel, 0, rowptr, col, Wh, s_src, s_dst, out, lse, dout, alpha_e, dsc_e, ds_dst, n,
               K, HF);
}

extern "C" int gnn_launch_gat_bwd_col(const int* rowptr_t, const int* col_t, const int* perm,
                                      const float* alpha_e, const float* dsc_e, const void* dout, float* dWh,
                                      float* ds_src, int n, int K, int Fh, int wbf, hipStream_t st) {
  const int HF = K * Fh;
  if (wbf)
    GAT_DISPATCH(gat_bwd_col_kernel, 1, rowptr_t, col_t, perm, alpha_e, dsc_e, dout, dWh, ds_src, n, K, HF);
  GAT_DISPATCH(gat_bwd_col_kernel, 0, rowptr_t, col_t, perm, alpha_e, dsc_e, dout, dWh, ds_src, n, K, HF);
}
