// Row-gather primitives of the CSR aggregation kernels (gnn_sparse.hip: spmm,
// spmm_ce, spmm_ell, ...).  One header so that every kernel summing gathered rows uses
// the same instructions in the same order: a fused kernel's aggregate is bit-identical
// to the standalone spmm's.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cgnn {
namespace gather {

template <typename T>
__device__ __forceinline__ T ld_stream(const T* p) {
  return *p;
}

__device__ __forceinline__ void bf16x8_to_f32(const uint4 v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint32_t f32_to_bf16_rne(float x) {
  uint32_t u = __float_as_uint(x);
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

__device__ __forceinline__ uint4 f32x8_to_bf16(const float* f) {
  uint4 o;
  o.x = f32_to_bf16_rne(f[0]) | (f32_to_bf16_rne(f[1]) << 16);
  o.y = f32_to_bf16_rne(f[2]) | (f32_to_bf16_rne(f[3]) << 16);
  o.z = f32_to_bf16_rne(f[4]) | (f32_to_bf16_rne(f[5]) << 16);
  o.w = f32_to_bf16_rne(f[6]) | (f32_to_bf16_rne(f[7]) << 16);
  return o;
}

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// acc[0..7] += a[0..7] + b[0..7] for two raw bf16x8 rows, two instructions per feature
// pair instead of four: v_perm_b32 pairs feature f of both rows into one dword, then
// v_dot2c_f32_bf16 against (1, 1) adds both into the fp32 accumulator
__device__ __forceinline__ void acc_bf16_pair(float* acc, const uint4 a, const uint4 b) {
  const bf16x2 one = {(__bf16)1.0f, (__bf16)1.0f};
  const uint32_t aw[4] = {a.x, a.y, a.z, a.w}, bw[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint32_t lo = __builtin_amdgcn_perm(bw[w], aw[w], 0x05040100u);   // (a.f, b.f)
    const uint32_t hi = __builtin_amdgcn_perm(bw[w], aw[w], 0x07060302u);   // (a.f+1, b.f+1)
    acc[2 * w] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, lo), one, acc[2 * w], false);
    acc[2 * w + 1] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, hi), one, acc[2 * w + 1], false);
  }
}

// the same for fp16 rows (v_dot2_f32_f16)
__device__ __forceinline__ void acc_f16_pair(float* acc, const uint4 a, const uint4 b) {
  typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
  const f16x2 one = {(_Float16)1.0f, (_Float16)1.0f};
  const uint32_t aw[4] = {a.x, a.y, a.z, a.w}, bw[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint32_t lo = __builtin_amdgcn_perm(bw[w], aw[w], 0x05040100u);
    const uint32_t hi = __builtin_amdgcn_perm(bw[w], aw[w], 0x07060302u);
    acc[2 * w] = __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, lo), one, acc[2 * w], false);
    acc[2 * w + 1] = __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, hi), one, acc[2 * w + 1], false);
  }
}

template <int XT>
__device__ __forceinline__ void acc_pair(float* acc, const uint4 a, const uint4 b) {
  if (XT == 1) acc_bf16_pair(acc, a, b);
  else acc_f16_pair(acc, a, b);
}

__device__ __forceinline__ uint4 load_raw16(const void* X, size_t off) {
  return *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(X) + off);
}

// the same with a 32-bit element offset (tables below 2^31 elements)
__device__ __forceinline__ uint4 load_raw16_u32(const void* X, uint32_t off) {
  return *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(X) + 2u * off);
}

// j[u] = v of lane u of this lane's 16-lane DPP row, u = U..15 (row_newbcast)
template <int U>
__device__ __forceinline__ void row_bcast16(int v, int* j) {
  j[U] = __builtin_amdgcn_update_dpp(0, v, 0x150 + U, 0xf, 0xf, false);
  if constexpr (U + 1 < 16) row_bcast16<U + 1>(v, j);
}

// j[u - B] = v of lane u of this lane's 16-lane DPP row, u = B..B+7
template <int B, int U = B>
__device__ __forceinline__ void row_bcast8(int v, int* j) {
  j[U - B] = __builtin_amdgcn_update_dpp(0, v, 0x150 + U, 0xf, 0xf, false);
  if constexpr (U + 1 < B + 8) row_bcast8<B, U + 1>(v, j);
}

// element types of the gathered / written matrices: 0 = fp32, 1 = bf16, 2 = fp16
template <int XT>
__device__ __forceinline__ void load8(const void* X, size_t off, float* f) {
  if (XT == 1) {
    const uint4 v = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(X) + off);
    bf16x8_to_f32(v, f);
  } else if (XT == 2) {
    const f16x8 v = *reinterpret_cast<const f16x8*>(reinterpret_cast<const uint16_t*>(X) + off);
#pragma unroll
    for (int q = 0; q < 8; ++q) f[q] = (float)v[q];
  } else {
    const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(X) + off);
    const float4 a = p[0], b = p[1];
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
}

// Sum the rows X[col[e]] for e in [e0, e1) into acc (8 features at f0).
// CS: gathered row j is scaled by cscale[j] (the column half of a symmetric
// normalisation, when the producer of X did not fold it in)
template <int L, int XBF, int U = 4, bool CS = false>
__device__ __forceinline__ void gather_sum(const int* __restrict__ col, const void* __restrict__ X,
                                           int e0, int e1, int ldx, int f0, bool fv, int sub_base,
                                           int sl, float* acc, const float* __restrict__ cscale = nullptr) {
  // the next chunk's column ids load while this chunk's rows are gathered (clamped address,
  // unconditional load: a "load or 0" would branch and wait for it at the join)
  int nxj = ld_stream(col + max(0, min(e0 + sl, e1 - 1)));
  for (int e = e0; e < e1; e += L) {
    const int myj = nxj;
    nxj = ld_stream(col + max(0, min(e + L + sl, e1 - 1)));
    const float mycs = CS ? cscale[myj] : 1.f;
    const int cnt = min(L, e1 - e);
    int k = 0;
    if (U == 16 && L >= 16 && XBF != 0 && !CS) {
      // 16 rows in flight per lane; the same pairs in the same order as two 8-steps
      if (cnt == 16) {
        // lane u of each 16-lane DPP row to the whole row (row_newbcast): a VALU move per
        // id, no LDS permute and no per-id address registers
        int j[16];
        row_bcast16<0>(myj, j);
        if (fv) {
          // 32-bit element offsets (callers guarantee a table below 2^31 elements): the
          // loads take the scalar base + one offset VGPR instead of a 64-bit address pair
          uint4 r[16];
#pragma unroll
          for (int u = 0; u < 16; ++u) r[u] = load_raw16_u32(X, (uint32_t)j[u] * (uint32_t)ldx + (uint32_t)f0);
#pragma unroll
          for (int u = 0; u < 16; u += 2) acc_pair<XBF>(acc, r[u], r[u + 1]);
        }
        k = 16;
      }
    }
    if ((U == 8 || U == 16) && L >= 8) {
      for (; k + 8 <= cnt; k += 8) {
        int j[8];
        if (L == 16 && !CS) {        // the ids by DPP row broadcast: no LDS permutes
          if (k == 0) row_bcast8<0>(myj, j);
          else row_bcast8<8>(myj, j);
        } else {
#pragma unroll
          for (int u = 0; u < 8; ++u) j[u] = __shfl(myj, sub_base + k + u, 64);
        }
        float c[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) c[u] = CS ? __shfl(mycs, sub_base + k + u, 64) : 1.f;
        if (fv && XBF != 0 && !CS) {
          uint4 r[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) r[u] = load_raw16(X, (size_t)j[u] * ldx + f0);
#pragma unroll
          for (int u = 0; u < 8; u += 2) acc_pair<XBF>(acc, r[u], r[u + 1]);
        } else if (fv) {
          float a[8][8];
#pragma unroll
          for (int u = 0; u < 8; ++u) load8<XBF>(X, (size_t)j[u] * ldx + f0, a[u]);
          if (CS) {
#pragma unroll
            for (int q = 0; q < 8; ++q)
              acc[q] += (fmaf(c[0], a[0][q], c[1] * a[1][q]) + fmaf(c[2], a[2][q], c[3] * a[3][q])) +
                        (fmaf(c[4], a[4][q], c[5] * a[5][q]) + fmaf(c[6], a[6][q], c[7] * a[7][q]));
          } else {
#pragma unroll
            for (int q = 0; q < 8; ++q)
              acc[q] += ((a[0][q] + a[1][q]) + (a[2][q] + a[3][q])) + ((a[4][q] + a[5][q]) + (a[6][q] + a[7][q]));
          }
        }
      }
    }
    for (; k + 4 <= cnt; k += 4) {
      const int j0 = __shfl(myj, sub_base + k + 0, 64);
      const int j1 = __shfl(myj, sub_base + k + 1, 64);
      const int j2 = __shfl(myj, sub_base + k + 2, 64);
      const int j3 = __shfl(myj, sub_base + k + 3, 64);
      const float c0 = CS ? __shfl(mycs, sub_base + k + 0, 64) : 1.f;
      const float c1 = CS ? __shfl(mycs, sub_base + k + 1, 64) : 1.f;
      const float c2 = CS ? __shfl(mycs, sub_base + k + 2, 64) : 1.f;
      const float c3 = CS ? __shfl(mycs, sub_base + k + 3, 64) : 1.f;
      if (fv && XBF != 0 && !CS) {
        const uint4 r0 = load_raw16(X, (size_t)j0 * ldx + f0), r1 = load_raw16(X, (size_t)j1 * ldx + f0);
        const uint4 r2 = load_raw16(X, (size_t)j2 * ldx + f0), r3 = load_raw16(X, (size_t)j3 * ldx + f0);
        acc_pair<XBF>(acc, r0, r1);
        acc_pair<XBF>(acc, r2, r3);
      } else if (fv) {
        float a[8], b[8], c[8], d[8];
        load8<XBF>(X, (size_t)j0 * ldx + f0, a);
        load8<XBF>(X, (size_t)j1 * ldx + f0, b);
        load8<XBF>(X, (size_t)j2 * ldx + f0, c);
        load8<XBF>(X, (size_t)j3 * ldx + f0, d);
        if (CS) {
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[q] += fmaf(c0, a[q], c1 * b[q]) + fmaf(c2, c[q], c3 * d[q]);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[q] += (a[q] + b[q]) + (c[q] + d[q]);
        }
      }
    }
    for (; k < cnt; ++k) {
      const int j = __shfl(myj, sub_base + k, 64);
      const float cj = CS ? __shfl(mycs, sub_base + k, 64) : 1.f;
      if (fv) {
        float a[8];
        load8<XBF>(X, (size_t)j * ldx + f0, a);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = CS ? fmaf(cj, a[q], acc[q]) : acc[q] + a[q];
      }
    }
  }
}

// gather_sum<16, 1, 8> for bf16 rows of up to 128 features with 8 lanes per row: lane sl
// owns the features f0 = 8 sl .. + 7 (acc0) and 64 + f0 .. + 7 (acc1), so a wave sums 8
// rows at once with 16 row loads in flight per lane, and each load instruction reads one
// 128-B line per row.  Chunks of 8 edges, each as 8-, 4- and 1-steps: per feature the
// same adds in the same order as gather_sum<16, 1, 8> (whose 16-edge chunks split into
// the same steps), so the sums are bit-identical.
__device__ __forceinline__ void gather_sum_x2(const int* __restrict__ col, const uint16_t* __restrict__ X,
                                              int e0, int e1, int ldx, int f0, bool fv0, bool fv1, int sub_base,
                                              int sl, float* acc0, float* acc1) {
  constexpr int L = 8;
  int nxj = ld_stream(col + max(0, min(e0 + sl, e1 - 1)));
  for (int e = e0; e < e1; e += L) {
    const int myj = nxj;
    nxj = ld_stream(col + max(0, min(e + L + sl, e1 - 1)));
    const int cnt = min(L, e1 - e);
    int k = 0;
    if (cnt == 8) {
      int j[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) j[u] = __shfl(myj, sub_base + u, 64);
      // one 32-bit byte offset per row (the table is < 4 GB): the two groups' loads share
      // it, the second at an immediate +128 B
      uint32_t o[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) o[u] = ((uint32_t)j[u] * (uint32_t)ldx + (uint32_t)f0) * 2u;
      const char* xb = reinterpret_cast<const char*>(X);
      uint4 r[8], q[8];
      if (fv0) {
#pragma unroll
        for (int u = 0; u < 8; ++u) r[u] = *reinterpret_cast<const uint4*>(xb + o[u]);
      }
      if (fv1) {
#pragma unroll
        for (int u = 0; u < 8; ++u) q[u] = *reinterpret_cast<const uint4*>(xb + o[u] + 128);
      }
      if (fv0) {
#pragma unroll
        for (int u = 0; u < 8; u += 2) acc_bf16_pair(acc0, r[u], r[u + 1]);
      }
      if (fv1) {
#pragma unroll
        for (int u = 0; u < 8; u += 2) acc_bf16_pair(acc1, q[u], q[u + 1]);
      }
      k = 8;
    }
    for (; k + 4 <= cnt; k += 4) {
      int j[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) j[u] = __shfl(myj, sub_base + k + u, 64);
      uint32_t o[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) o[u] = ((uint32_t)j[u] * (uint32_t)ldx + (uint32_t)f0) * 2u;
      const char* xb = reinterpret_cast<const char*>(X);
      uint4 r[4], q[4];
      if (fv0) {
#pragma unroll
        for (int u = 0; u < 4; ++u) r[u] = *reinterpret_cast<const uint4*>(xb + o[u]);
      }
      if (fv1) {
#pragma unroll
        for (int u = 0; u < 4; ++u) q[u] = *reinterpret_cast<const uint4*>(xb + o[u] + 128);
      }
      if (fv0) {
        acc_bf16_pair(acc0, r[0], r[1]);
        acc_bf16_pair(acc0, r[2], r[3]);
      }
      if (fv1) {
        acc_bf16_pair(acc1, q[0], q[1]);
        acc_bf16_pair(acc1, q[2], q[3]);
      }
    }
    for (; k < cnt; ++k) {
      const int j = __shfl(myj, sub_base + k, 64);
      float a[8];
      if (fv0) {
        load8<1>(X, (size_t)j * ldx + f0, a);
#pragma unroll
        for (int t = 0; t < 8; ++t) acc0[t] = acc0[t] + a[t];
      }
      if (fv1) {
        load8<1>(X, (size_t)j * ldx + 64 + f0, a);
#pragma unroll
        for (int t = 0; t < 8; ++t) acc1[t] = acc1[t] + a[t];
      }
    }
  }
}

}  // namespace gather
}  // namespace cgnn
