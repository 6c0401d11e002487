// Fused dense stages of the 2-layer GCN on MFMA (gfx950, v_mfma_f32_32x32x16_bf16).
//
// Forward (one kernel, one pass over the rows):
//     H1 = dropout(relu(AX W1 + b1))           bf16 [n][HD]  (stored: needed by the backward)
//     Z2 = dinv * (H1 W2)                      bf16 [n][ldc]
// Backward:
//     dP1 = (dY2 W2^T) * [H1 > 0] / (1 - p)    bf16 [n][HD]
//
// Both products are computed TRANSPOSED (output tile = [feature][row]) so that
//   * the B operand of the first product is AX (resp. dY2) read straight from
//     HBM in its natural row-major layout: lane l loads 16 contiguous bytes of row
//     r0 + (l & 31);
//   * the 32x32 fp32 accumulator of H1^T (feature in the registers, row on the
//     lane) is ALREADY the B operand of the second product Z2^T = W2^T H1^T: its
//     registers 8s..8s+7, converted to bf16, are the k-step-s fragment (k order
//     permuted; the A operand W2^T is read in the same permuted order) -- no LDS
//     round trip, no shuffles (cdna_hip_programming.md §3 "An accumulator tile as
//     the next MFMA's operand");
//   * each lane owns 16 values of one row: one Philox draw supplies exactly its
//     16 dropout bytes (mask keyed by (row, 2*(n/32) + (n/4)%2, step); byte
//     (n%4) + 4*((n%32)/8)), identical to the standalone kernel and the CPU mirror.
// The weights (W1^T, W2^T, b1) live in LDS for the whole persistent block; rows are
// processed in 32-row tiles, one tile per wave at a time, grid-strided.
#include "cgnn_common.h"
#include <algorithm>

using namespace cgnn;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int WAVES = 8;            // 512-thread blocks: 2 waves per SIMD share the LDS weights
constexpr int TILE = 32;

__device__ __forceinline__ bf16x8 load_bf16x8(const uint16_t* p) {
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 zero_bf16x8() {
  return __builtin_bit_cast(bf16x8, make_uint4(0u, 0u, 0u, 0u));
}

__device__ __forceinline__ uint16_t bf16_bits(float x) {
  return __builtin_bit_cast(uint16_t, (__bf16)x);
}

__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
  return make_uint2((uint32_t)bf16_bits(a) | ((uint32_t)bf16_bits(b) << 16),
                    (uint32_t)bf16_bits(c) | ((uint32_t)bf16_bits(d) << 16));
}

}  // namespace

// KS = k-steps of 16 over the input features (F <= 16*KS <= ldx rounded), HD hidden width.
template <int KS, int HD>
__global__ __launch_bounds__(WAVES * 64) void gcn_dense_fwd_kernel(
    const uint16_t* __restrict__ AX, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ W2, const float* __restrict__ dinv, uint16_t* __restrict__ H1,
    uint16_t* __restrict__ Z2, int n, int F, int ldx, int C, int ldc, float p, uint32_t k0,
    uint32_t k1, uint32_t step, uint32_t thr8, uint32_t row0) {
  constexpr int KP = KS * 16;
  constexpr int W1S = KP + 8;          // padded row strides (bank-conflict-free b128 / b64 reads)
  constexpr int W2S = HD + 8;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* sW1T = lds;                          // [HD][W1S]   W1^T
  uint16_t* sW2T = sW1T + HD * W1S;              // [64][W2S]   W2^T (rows >= C zero)
  float* sB1 = reinterpret_cast<float*>(sW2T + 64 * W2S);   // [HD]

  for (int i = threadIdx.x; i < HD * KP; i += blockDim.x) {
    const int k = i / HD, nn = i - k * HD;
    sW1T[nn * W1S + k] = bf16_bits(k < F ? W1[(size_t)k * HD + nn] : 0.f);
  }
  for (int i = threadIdx.x; i < 64 * HD; i += blockDim.x) {
    const int nn = i / 64, c = i - nn * 64;
    sW2T[c * W2S + nn] = bf16_bits(c < C ? W2[(size_t)nn * C + c] : 0.f);
  }
  for (int i = threadIdx.x; i < HD; i += blockDim.x) sB1[i] = b1[i];
  __syncthreads();

  const int lane = threadIdx.x & 63, h = lane >> 5, lr = lane & 31;
  const int wave = blockIdx.x * WAVES + (threadIdx.x >> 6);
  const int n_waves = gridDim.x * WAVES;
  const int n_tiles = (n + TILE - 1) / TILE;
  const float scale = 1.f / (1.f - p);

  for (int tile = wave; tile < n_tiles; tile += n_waves) {
    const int row = tile * TILE + lr;
    const bool rv = row < n;
    bf16x8 bx[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int f0 = 16 * s + 8 * h;
      bx[s] = (rv && f0 < ldx) ? load_bf16x8(AX + (size_t)row * ldx + f0) : zero_bf16x8();
    }
    f32x16 z0 = {}, z1 = {};
#pragma unroll 1
    for (int t = 0; t < HD / 32; ++t) {
      f32x16 acc = {};
      const uint16_t* arow = sW1T + (32 * t + lr) * W1S + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(load_bf16x8(arow + 16 * s), bx[s], acc, 0, 0, 0);
      // epilogue: bias, relu, dropout (one Philox draw = this lane's 16 bytes)
      uint32_t w[4] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
      if (thr8 > 0) {
        const u32x4 r = philox4x32_10(u32x4{row0 + (uint32_t)row, (uint32_t)(2 * t + h), step, RNG_DROPOUT}, k0, k1);
        w[0] = r.x; w[1] = r.y; w[2] = r.z; w[3] = r.w;
      }
      float v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int nn = 32 * t + (q & 3) + 8 * (q >> 2) + 4 * h;
        float x = fmaxf(acc[q] + sB1[nn], 0.f);
        if (thr8 > 0) x = (((w[q >> 2] >> (8 * (q & 3))) & 0xffu) >= thr8) ? x * scale : 0.f;
        v[q] = x;
      }
      if (rv) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<uint2*>(H1 + (size_t)row * HD + 32 * t + 8 * g + 4 * h) =
              pack4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
      }
      // second product: Z2^T += W2^T[:, 32t..32t+31] * H1^T tile (accumulator as B operand)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 xb;
#pragma unroll
        for (int j = 0; j < 8; ++j) xb[j] = (__bf16)v[8 * s2 + j];
        const int nbase = 32 * t + 16 * s2 + 4 * h;
        {
          const uint16_t* a = sW2T + lr * W2S + nbase;
          const uint2 lo = *reinterpret_cast<const uint2*>(a), hi = *reinterpret_cast<const uint2*>(a + 8);
          const bf16x8 af = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
          z0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, xb, z0, 0, 0, 0);
        }
        {
          const uint16_t* a = sW2T + (32 + lr) * W2S + nbase;
          const uint2 lo = *reinterpret_cast<const uint2*>(a), hi = *reinterpret_cast<const uint2*>(a + 8);
          const bf16x8 af = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
          z1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, xb, z1, 0, 0, 0);
        }
      }
    }
    if (rv) {
      const float ds = dinv[row];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 8 * g + 4 * h;
        if (c < ldc)
          *reinterpret_cast<uint2*>(Z2 + (size_t)row * ldc + c) =
              pack4(z0[4 * g] * ds, z0[4 * g + 1] * ds, z0[4 * g + 2] * ds, z0[4 * g + 3] * ds);
        if (32 + c < ldc)
          *reinterpret_cast<uint2*>(Z2 + (size_t)row * ldc + 32 + c) =
              pack4(z1[4 * g] * ds, z1[4 * g + 1] * ds, z1[4 * g + 2] * ds, z1[4 * g + 3] * ds);
      }
    }
  }
}

// dP1 = (dY2 W2^T) * [H1 > 0] / (1-p), computed transposed: A = W2 [n][c] from LDS,
// B = dY2 rows straight from HBM (KC k-steps of 16 over the classes).
template <int KC, int HD>
__global__ __launch_bounds__(WAVES * 64) void gcn_dense_bwd_kernel(
    const uint16_t* __restrict__ dY2, const float* __restrict__ W2, const uint16_t* __restrict__ H1,
    uint16_t* __restrict__ dP1, int n, int C, int ldc, float p) {
  constexpr int KP = KC * 16;
  constexpr int W2S = KP + 8;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* sW2 = lds;                           // [HD][W2S]
  for (int i = threadIdx.x; i < HD * KP; i += blockDim.x) {
    const int nn = i / KP, c = i - nn * KP;
    sW2[nn * W2S + c] = bf16_bits(c < C ? W2[(size_t)nn * C + c] : 0.f);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, h = lane >> 5, lr = lane & 31;
  const int wave = blockIdx.x * WAVES + (threadIdx.x >> 6);
  const int n_waves = gridDim.x * WAVES;
  const int n_tiles = (n + TILE - 1) / TILE;
  const float scale = 1.f / (1.f - p);
  for (int tile = wave; tile < n_tiles; tile += n_waves) {
    const int row = tile * TILE + lr;
    const bool rv = row < n;
    bf16x8 by[KC];
#pragma unroll
    for (int s = 0; s < KC; ++s) {
      const int c0 = 16 * s + 8 * h;
      by[s] = (rv && c0 < ldc) ? load_bf16x8(dY2 + (size_t)row * ldc + c0) : zero_bf16x8();
    }
#pragma unroll 1
    for (int t = 0; t < HD / 32; ++t) {
      f32x16 acc = {};
      const uint16_t* arow = sW2 + (32 * t + lr) * W2S + 8 * h;
#pragma unroll
      for (int s = 0; s < KC; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(load_bf16x8(arow + 16 * s), by[s], acc, 0, 0, 0);
      if (!rv) continue;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint16_t* hp = const_cast<uint16_t*>(H1) + (size_t)row * HD + 32 * t + 8 * g + 4 * h;
        const uint2 hv = *reinterpret_cast<const uint2*>(hp);
        const float m0 = (hv.x & 0x7fffu) && !(hv.x & 0x8000u) ? scale : 0.f;
        const float m1 = ((hv.x >> 16) & 0x7fffu) && !((hv.x >> 16) & 0x8000u) ? scale : 0.f;
        const float m2 = (hv.y & 0x7fffu) && !(hv.y & 0x8000u) ? scale : 0.f;
        const float m3 = ((hv.y >> 16) & 0x7fffu) && !((hv.y >> 16) & 0x8000u) ? scale : 0.f;
        *reinterpret_cast<uint2*>(dP1 + (size_t)row * HD + 32 * t + 8 * g + 4 * h) =
            pack4(acc[4 * g] * m0, acc[4 * g + 1] * m1, acc[4 * g + 2] * m2, acc[4 * g + 3] * m3);
      }
    }
  }
}

// ---------------------------------------------------------------- launchers
static int dense_grid(int n) {
  static int cached_cus[64] = {0};
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess && dev < 64) {
    if (!cached_cus[dev]) {
      hipDeviceProp_t prop;
      cached_cus[dev] = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
    }
    cus = cached_cus[dev];
  }
  const int tiles = (n + TILE - 1) / TILE;
  return std::max(1, std::min(cus, (tiles + WAVES - 1) / WAVES));
}

template <int KS, int HD>
static int fwd_launch(const uint16_t* AX, const float* W1, const float* b1, const float* W2,
                      const float* dinv, uint16_t* H1, uint16_t* Z2, int n, int F, int ldx, int C,
                      int ldc, float p, uint32_t k0, uint32_t k1, uint32_t step, uint32_t thr8,
                      uint32_t row0, hipStream_t st) {
  const size_t lds = sizeof(uint16_t) * ((size_t)HD * (KS * 16 + 8) + 64 * (size_t)(HD + 8)) + sizeof(float) * HD;
  (void)hipFuncSetAttribute((const void*)gcn_dense_fwd_kernel<KS, HD>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((gcn_dense_fwd_kernel<KS, HD>), dim3(dense_grid(n)), dim3(WAVES * 64), lds, st, AX, W1,
                     b1, W2, dinv, H1, Z2, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0);
  return (int)hipGetLastError();
}

extern "C" int gnn_launch_dense_fwd(const void* AX, const float* W1, const float* b1, const float* W2,
                                    const float* dinv, void* H1, void* Z2, int n, int F, int ldx,
                                    int HD, int C, int ldc, float p, uint32_t k0, uint32_t k1,
                                    uint32_t step, uint32_t row0, hipStream_t st) {
  if (C > 64 || ldc % 8 || ldx % 8 || ldc > 64) return -3;
  const uint32_t thr8 = (uint32_t)std::min(255.0, std::floor((double)p * 256.0 + 0.5));
  const int KS = (F + 15) / 16;
  auto* ax = (const uint16_t*)AX;
  auto* h1 = (uint16_t*)H1;
  auto* z2 = (uint16_t*)Z2;
#define FWD(ks, hd) if (KS <= ks && HD == hd) return fwd_launch<ks, hd>(ax, W1, b1, W2, dinv, h1, z2, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0, st);
  FWD(4, 256) FWD(7, 256) FWD(8, 256) FWD(4, 128) FWD(8, 128)
#undef FWD
  return -1;
}

template <int KC, int HD>
static int bwd_launch(const uint16_t* dY2, const float* W2, const uint16_t* H1, uint16_t* dP1, int n,
                      int C, int ldc, float p, hipStream_t st) {
  const size_t lds = sizeof(uint16_t) * (size_t)HD * (KC * 16 + 8);
  (void)hipFuncSetAttribute((const void*)gcn_dense_bwd_kernel<KC, HD>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((gcn_dense_bwd_kernel<KC, HD>), dim3(dense_grid(n)), dim3(WAVES * 64), lds, st, dY2,
                     W2, H1, dP1, n, C, ldc, p);
  return (int)hipGetLastError();
}

extern "C" int gnn_launch_dense_bwd(const void* dY2, const float* W2, const void* H1, void* dP1, int n,
                                    int HD, int C, int ldc, float p, hipStream_t st) {
  if (C > 64 || ldc % 8 || ldc > 64) return -3;
  const int KC = (ldc + 15) / 16;
  auto* dy = (const uint16_t*)dY2;
  auto* h1 = (const uint16_t*)H1;
  auto* dp = (uint16_t*)dP1;
#define BWD(kc, hd) if (KC <= kc && HD == hd) return bwd_launch<kc, hd>(dy, W2, h1, dp, n, C, ldc, p, st);
  BWD(3, 256) BWD(4, 256) BWD(3, 128) BWD(4, 128)
#undef BWD
  return -1;
}
