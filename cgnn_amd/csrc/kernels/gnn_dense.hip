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
#include <cstdlib>

using namespace cgnn;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int WAVES = 16;           // 1024-thread blocks: 4 waves per SIMD share the LDS weights
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

typedef short v4s __attribute__((ext_vector_type(4)));

// x with the dropout decision of keep bit q of m applied: x AND the bit sign-extended
// (v_bfe_i32 + v_and_b32; the AND is opaque so it is not turned back into a
// test / compare / select sequence of three instructions)
__device__ __forceinline__ float keep_and(float x, uint32_t m, uint32_t q) {
  const uint32_t k = (uint32_t)__builtin_amdgcn_sbfe((int)m, q, 1);
  uint32_t r;
  asm("v_and_b32 %0, %1, %2" : "=v"(r) : "v"(__float_as_uint(x)), "v"(k));
  return __uint_as_float(r);
}

// Byte offset of 16-B chunk `ch` of row `row` in a [32][256 B] staging image.  The
// XOR swizzle keeps the b128 staging writes at the 8-way minimum and makes the b128
// row reads and the ds_read_b64_tr_b16 column reads of the 32x32x16 operands
// conflict-free (cdna_hip_programming.md T10, image (b)).
__device__ __forceinline__ int stg_off(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

// Byte offset of 8-B unit `u` (0..7) of row `row` in a wave's [32 rows][32 hidden]
// H1 / dP1 image (64-B rows): the packed accumulator writes are at the 4-way minimum,
// the transposed reads conflict-free.
__device__ __forceinline__ int img_off(int row, int u) {
  return 64 * row + 8 * (u ^ ((row >> 1) & 7));
}

// ds_read_b64_tr_b16 (gfx950): lane 4q+p of a 16-lane group gives the address of
// row q, columns 4p..4p+3 of a 4x16 block; lane i receives column i of the 4 rows.
// Two reads (rows +0..3, +4..7) form one 32x32x16 operand fragment.
__device__ __forceinline__ bf16x8 tr_frag(const uint16_t* base, int off0, int off1) {
  typedef __attribute__((address_space(3))) v4s lds_v4s;
  const char* b = reinterpret_cast<const char*>(base);
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(b + off0));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(b + off1));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

}  // namespace

// KS = k-steps of 16 over the input features (F <= 16*KS <= ldx rounded), HD hidden width;
// DROP: dropout mode, a compile-time switch so the epilogue has no per-element branches:
// 0 none, 1 byte mode (any p), 2 bit mode (p = 1/2: one Philox draw per row and half for
// all eight hidden blocks, cgnn_common.h drop_draw).
//
// Latency structure (the kernel runs 4 waves / SIMD -- one 16-wave block per CU -- and
// was measured MFMA-busy ~23 %): per hidden tile t the accumulator starts as the bias
// (4 b128 LDS reads issued ahead, fp32 exact) instead of a bias add per element after
// the chain, and the KS weight fragments of the chain are read from LDS as one batch
// before the first MFMA rather than one LDS round trip per MFMA.
template <int KS, int HD, int DROP>
__global__ __launch_bounds__(WAVES * 64) void gcn_dense_fwd_kernel(
    const uint16_t* __restrict__ AX, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ W2, const float* __restrict__ dinv, uint16_t* __restrict__ H1,
    uint16_t* __restrict__ Z2, int n, int F, int ldx, int C, int ldc, float p, uint32_t k0,
    uint32_t k1, uint32_t step, uint32_t thr8, uint32_t row0, const int* __restrict__ stepp) {
  // stepp (optional): the dropout step read from device memory, so a captured hipGraph
  // replays with the current epoch's mask
  if (stepp) step = (uint32_t)*stepp;
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
  // the dropout scale 1/(1-p) of the kept units is folded into W2^T (exact for p = 1/2):
  // Z2 = (x * keep * s) W2 = (x * keep) (s W2), so the epilogue never multiplies
  const float scale = 1.f / (1.f - p);
  const float w2s = DROP != 0 ? scale : 1.f;
  for (int i = threadIdx.x; i < 64 * HD; i += blockDim.x) {
    const int nn = i / 64, c = i - nn * 64;
    sW2T[c * W2S + nn] = bf16_bits(c < C ? W2[(size_t)nn * C + c] * w2s : 0.f);
  }
  for (int i = threadIdx.x; i < HD; i += blockDim.x) sB1[i] = b1[i];
  __syncthreads();

  const int lane = threadIdx.x & 63, h = lane >> 5, lr = lane & 31;
  const int wave = blockIdx.x * WAVES + (threadIdx.x >> 6);
  const int n_waves = gridDim.x * WAVES;
  const int n_tiles = (n + TILE - 1) / TILE;

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
    static_assert(HD <= 256, "bit-mode dropout: one draw covers 8 hidden blocks");
    u32x4 rb{};
    if constexpr (DROP == 2) rb = drop_draw(row0 + (uint32_t)row, 0, h, step, k0, k1, true);
#pragma unroll 1
    for (int t = 0; t < HD / 32; ++t) {
      const uint16_t* arow = sW1T + (32 * t + lr) * W1S + 8 * h;
      bf16x8 af[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) af[s] = load_bf16x8(arow + 16 * s);
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < KS; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bx[s], acc, 0, 0, 0);
      // epilogue (registers 4g..4g+3 are hidden 32t + 8g + 4h + 0..3): bias (packed adds),
      // relu, dropout as an AND with the sign-extended keep bit (the scale is in W2^T)
      float v[16];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 bb = *reinterpret_cast<const float4*>(sB1 + 32 * t + 8 * g + 4 * h);
        const f2 lo = f2{acc[4 * g], acc[4 * g + 1]} + f2{bb.x, bb.y};
        const f2 hi = f2{acc[4 * g + 2], acc[4 * g + 3]} + f2{bb.z, bb.w};
        v[4 * g] = fmaxf(lo.x, 0.f); v[4 * g + 1] = fmaxf(lo.y, 0.f);
        v[4 * g + 2] = fmaxf(hi.x, 0.f); v[4 * g + 3] = fmaxf(hi.y, 0.f);
      }
      if constexpr (DROP != 0) {
        const uint32_t m = drop_keep16(DROP == 2 ? rb : drop_draw(row0 + (uint32_t)row, t, h, step, k0, k1, false), t,
                                       thr8, DROP == 2);
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = keep_and(v[q], m, q);
      }
      if (rv && H1) {          // H1 == nullptr: the fused backward recomputes it
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<uint2*>(H1 + (size_t)row * HD + 32 * t + 8 * g + 4 * h) =
              pack4(v[4 * g] * w2s, v[4 * g + 1] * w2s, v[4 * g + 2] * w2s, v[4 * g + 3] * w2s);
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
          const bf16x8 af2 = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
          z0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af2, xb, z0, 0, 0, 0);
        }
        {
          const uint16_t* a = sW2T + (32 + lr) * W2S + nbase;
          const uint2 lo = *reinterpret_cast<const uint2*>(a), hi = *reinterpret_cast<const uint2*>(a + 8);
          const bf16x8 af2 = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
          z1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af2, xb, z1, 0, 0, 0);
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


// ============================================================================
// Fused backward of the dense stages, H1 never stored (recomputed) and the two
// weight-gradient contractions over the rows done in the same pass:
//   P1^T = W1^T AX^T, H1 = dropout(relu(P1 + b1))      (as the forward, same Philox)
//   dP1^T = (W2 dY2^T) * [H1 > 0] / (1-p)
//   gW1^T[h][f] += sum_rows dP1^T[h][row] AX[row][f]     (f = F is the ones column: gb1)
//   gW2[h][c]   += sum_rows H1^T[h][row] dY2[row][c]
// Block = HD/32 waves, wave w owns hidden block w (32 units) for all three
// products, so its weight-gradient tiles (KF/32 + 2 of 32x32) stay in its
// accumulators for the whole persistent loop; the block walks 32-row tiles.
// Per tile: stage the AX / dY2 rows ONCE, row-major in swizzled 256-B rows: the
// recompute reads them by rows (b128), the contractions over the rows by columns
// with ds_read_b64_tr_b16 (no second, transposed copy).  The recomputed H1^T /
// dP1^T accumulators (lane = row) are stored packed, 4 hidden units per 8-B write,
// into the wave's own [row][hidden] images and read back transposed as the
// contractions' A operands.  The next tile's rows are prefetched into registers
// meanwhile.  Output: one fp32 slab per block, gpart[block][HD][KF + 64] =
// [gW1^T | gW2], summed in fixed order afterwards.
// (The round-1 form staged separate transposed images with 2-byte scattered writes
// and wrote H1^T / dP1^T one element at a time: 0.74 ms on the ogbn-products shape.)
// ============================================================================
// LDS bytes of the fused backward: weights, nbuf x two [32][128] staging images, two
// [HD/32][32][32] H1 / dP1 images, b1
constexpr size_t fused_bwd_lds(int KP, int CP, int HD, int nbuf) {
  return sizeof(uint16_t) * ((size_t)HD * (KP + 8) + (size_t)HD * (CP + 8) + (size_t)nbuf * 2 * 32 * 128 +
                             2 * (size_t)HD * 32) +
         sizeof(float) * HD;
}

template <int KS, int KC, int HD, bool DROP>
__global__ __launch_bounds__(HD * 2) void gcn_fused_bwd_kernel(
    const uint16_t* __restrict__ AX, const uint16_t* __restrict__ dY2, const float* __restrict__ W1,
    const float* __restrict__ b1, const float* __restrict__ W2, float* __restrict__ gpart, int n, int F,
    int ldx, int C, int ldc, float p, uint32_t k0, uint32_t k1, uint32_t step, uint32_t thr8,
    uint32_t row0, const int* __restrict__ stepp) {
  if (stepp) step = (uint32_t)*stepp;         // device-resident dropout step (graph replays)
  constexpr int NW = HD / 32;                 // waves per block = hidden blocks
  constexpr int NT = NW * 64;
  constexpr int KP = KS * 16;                 // layer-1 K (features + ones column), padded
  constexpr int KF = (KP + 31) / 32 * 32;     // gW1^T columns (f), padded to whole tiles
  constexpr int CP = KC * 16;                 // classes, padded
  constexpr int W1S = KP + 8, W2S = CP + 8;
  static_assert(KF <= 128 && CP <= 64, "staging rows are 256 B");
  static_assert(KC <= KS, "the dh chain is interleaved into the layer-1 chain");
  // double-buffered staging where the LDS budget allows it (HD = 256: K <= 112, C <= 48)
  constexpr int NBUF = fused_bwd_lds(KP, CP, HD, 2) <= 160 * 1024 ? 2 : 1;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* sW1T = lds;                       // [HD][W1S]
  uint16_t* sW2 = sW1T + HD * W1S;            // [HD][W2S]   W2 rows (hidden-major)
  // staging: NBUF buffers (two: tile i computes from one while tile i + 1 is written to
  // the other, one block barrier per tile), each = AX [32][128] | dY2 [32][128],
  // swizzled (stg_off), dY2 columns < 64 used
  uint16_t* sStg = sW2 + HD * W2S;
  uint16_t* sH1 = sStg + NBUF * 2 * TILE * 128;   // [NW][32][32] per-wave images (img_off)
  uint16_t* sDP = sH1 + NW * TILE * 32;       // [NW][32][32]
  float* sB1 = reinterpret_cast<float*>(sDP + NW * TILE * 32);   // [HD]

  const int tid = threadIdx.x;
  for (int i = tid; i < HD * KP; i += NT) {
    const int k = i / HD, nn = i - k * HD;
    sW1T[nn * W1S + k] = bf16_bits(k < F ? W1[(size_t)k * HD + nn] : 0.f);
  }
  for (int i = tid; i < HD * CP; i += NT) {
    const int nn = i / CP, c = i - nn * CP;
    sW2[nn * W2S + c] = bf16_bits(c < C ? W2[(size_t)nn * C + c] : 0.f);
  }
  for (int i = tid; i < HD; i += NT) sB1[i] = b1[i];
  // zero the staging images: chunks the per-tile staging never writes (columns past
  // the staged K, read by the padded contraction tiles) stay zero
  for (int i = tid; i < NBUF * 2 * TILE * 128 / 8; i += NT)
    reinterpret_cast<uint4*>(sStg)[i] = make_uint4(0u, 0u, 0u, 0u);

  const int lane = tid & 63, h = lane >> 5, lr = lane & 31;
  const int t = tid >> 6;                     // this wave's hidden block
  // transposed-read lane roles: 16-lane group, block row qq, column quad pq
  const int gb = (lane >> 4) & 1, qq = (lane >> 2) & 3, pq = lane & 3;
  uint16_t* wH1 = sH1 + t * TILE * 32;
  uint16_t* wDP = sDP + t * TILE * 32;
  const int n_tiles = (n + TILE - 1) / TILE;
  const float scale = 1.f / (1.f - p);
  // 16-byte chunks staged per row: the K columns the products read (a row pitch wider
  // than that -- rows padded to whole cache lines -- is not staged)
  const int xch = min(ldx, KP) / 8, ych = min(ldc, CP) / 8;

  f32x16 g1[KF / 32], g2[2];
#pragma unroll
  for (int q = 0; q < KF / 32; ++q) g1[q] = f32x16{};
  g2[0] = f32x16{};
  g2[1] = f32x16{};

  // prefetch registers: chunks tid, tid + NT, ... (chunk i = row i % 32, column chunk
  // i / 32) of the AX tile and of the dY2 tile
  constexpr int PFX = (TILE * (KP / 8) + NT - 1) / NT, PFY = (TILE * (CP / 8) + NT - 1) / NT;
  uint4 pax[PFX], pdy[PFY];
  auto prefetch = [&](int tile) {
    const int r0 = tile * TILE;
#pragma unroll
    for (int k = 0; k < PFX; ++k) {
      const int i = tid + k * NT;
      const int rr = i % TILE, ch = i / TILE;
      pax[k] = (i < TILE * xch && r0 + rr < n)
                   ? *reinterpret_cast<const uint4*>(AX + (size_t)(r0 + rr) * ldx + 8 * ch)
                   : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int k = 0; k < PFY; ++k) {
      const int i = tid + k * NT;
      const int rr = i % TILE, ch = i / TILE;
      pdy[k] = (i < TILE * ych && r0 + rr < n)
                   ? *reinterpret_cast<const uint4*>(dY2 + (size_t)(r0 + rr) * ldc + 8 * ch)
                   : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto stage = [&](int buf) {
    char* const bA = reinterpret_cast<char*>(sStg + buf * 2 * TILE * 128);
    char* const bD = bA + 2 * TILE * 128;
#pragma unroll
    for (int k = 0; k < PFX; ++k) {
      const int i = tid + k * NT;
      if (i < TILE * xch) *reinterpret_cast<uint4*>(bA + stg_off(i % TILE, i / TILE)) = pax[k];
    }
#pragma unroll
    for (int k = 0; k < PFY; ++k) {
      const int i = tid + k * NT;
      if (i < TILE * ych) *reinterpret_cast<uint4*>(bD + stg_off(i % TILE, i / TILE)) = pdy[k];
    }
  };
  const int G = gridDim.x;
  __syncthreads();                            // the zeroed staging images
  if ((int)blockIdx.x < n_tiles) {
    prefetch(blockIdx.x);
    if constexpr (NBUF == 2) {
      stage(0);
      if ((int)blockIdx.x + G < n_tiles) prefetch(blockIdx.x + G);
    }
  }
  __syncthreads();

  int it = 0;
  for (int tile = blockIdx.x; tile < n_tiles; tile += G, ++it) {
    int cur = 0;
    if constexpr (NBUF == 2) {
      // stage the next tile into the other buffer (read by the previous tile, which
      // every wave finished at the last barrier), prefetch the one after
      cur = it & 1;
      if (tile + G < n_tiles) {
        stage(cur ^ 1);
        if (tile + 2 * G < n_tiles) prefetch(tile + 2 * G);
      }
    } else {
      stage(0);
      if (tile + G < n_tiles) prefetch(tile + G);
      __syncthreads();
    }
    uint16_t* const sAX = sStg + cur * 2 * TILE * 128;
    uint16_t* const sDY = sAX + TILE * 128;
    char* const bAX = reinterpret_cast<char*>(sAX);
    char* const bDY = reinterpret_cast<char*>(sDY);

    // ---- recompute H1^T block t, dP1^T block t (lane = row, registers = hidden) ----
    const int row = tile * TILE + lr;
    // both chains' operands read from LDS as one batch (not one round trip per MFMA);
    // the layer-1 accumulator starts as the bias (fp32)
    f32x16 acc, dh = {};
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 bb = *reinterpret_cast<const float4*>(sB1 + 32 * t + 8 * g + 4 * h);
      acc[4 * g] = bb.x; acc[4 * g + 1] = bb.y; acc[4 * g + 2] = bb.z; acc[4 * g + 3] = bb.w;
    }
    {
      const uint16_t* arow = sW1T + (32 * t + lr) * W1S + 8 * h;
      const uint16_t* drow = sW2 + (32 * t + lr) * W2S + 8 * h;
      bf16x8 a1[KS], x1[KS], a2[KC], y2[KC];
#pragma unroll
      for (int s2 = 0; s2 < KS; ++s2) {
        a1[s2] = load_bf16x8(arow + 16 * s2);
        x1[s2] = load_bf16x8(reinterpret_cast<const uint16_t*>(bAX + stg_off(lr, 2 * s2 + h)));
      }
#pragma unroll
      for (int s2 = 0; s2 < KC; ++s2) {
        a2[s2] = load_bf16x8(drow + 16 * s2);
        y2[s2] = load_bf16x8(reinterpret_cast<const uint16_t*>(bDY + stg_off(lr, 2 * s2 + h)));
      }
#pragma unroll
      for (int s2 = 0; s2 < KS; ++s2) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[s2], x1[s2], acc, 0, 0, 0);
        if (s2 < KC) dh = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2[s2], y2[s2], dh, 0, 0, 0);
      }
    }
    uint32_t m = 0xffffu;
    if constexpr (DROP)
      m = drop_keep16(drop_draw(row0 + (uint32_t)row, t, h, step, k0, k1, drop_bit_mode(thr8)), t, thr8,
                      drop_bit_mode(thr8));
    // registers 4g..4g+3 = hidden 32t + 8g + 4h + 0..3 of this lane's row: one packed
    // 8-B write per image and g
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float xv[4], dv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = 4 * g + i;
        float x = fmaxf(acc[q], 0.f);
        if constexpr (DROP) x = ((m >> q) & 1u) ? x * scale : 0.f;
        xv[i] = x;
        dv[i] = x > 0.f ? dh[q] * scale : 0.f;
      }
      const int off = img_off(lr, 2 * g + h);
      *reinterpret_cast<uint2*>(reinterpret_cast<char*>(wH1) + off) = pack4(xv[0], xv[1], xv[2], xv[3]);
      *reinterpret_cast<uint2*>(reinterpret_cast<char*>(wDP) + off) = pack4(dv[0], dv[1], dv[2], dv[3]);
    }
    // the contraction below reads only this wave's own images: a wave-local ordering
    // of the LDS writes and reads suffices (no block barrier)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");

    // ---- contractions over the tile's 32 rows (two k-steps of 16) ----
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int ra = 16 * s2 + 8 * h + qq;      // block rows ra (+4 for the second read)
      const bf16x8 adp = tr_frag(wDP, img_off(ra, 4 * gb + pq), img_off(ra + 4, 4 * gb + pq));
      const bf16x8 ah1 = tr_frag(wH1, img_off(ra, 4 * gb + pq), img_off(ra + 4, 4 * gb + pq));
      const int cb = 2 * gb + (pq >> 1), cx = 8 * (pq & 1);
#pragma unroll
      for (int q = 0; q < KF / 32; ++q)
        g1[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            adp, tr_frag(sAX, stg_off(ra, 4 * q + cb) + cx, stg_off(ra + 4, 4 * q + cb) + cx), g1[q], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 2; ++q)
        g2[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            ah1, tr_frag(sDY, stg_off(ra, 4 * q + cb) + cx, stg_off(ra + 4, 4 * q + cb) + cx), g2[q], 0, 0, 0);
    }
    __syncthreads();      // this buffer is rewritten two tiles on; the next one is staged
  }

  // ---- this block's partial slab: rows = hidden 32t + m, columns [f | KF + c] ----
  float* gp = gpart + (size_t)blockIdx.x * HD * (KF + 64);
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int hrow = 32 * t + (q & 3) + 8 * (q >> 2) + 4 * h;
    float* dst = gp + (size_t)hrow * (KF + 64);
#pragma unroll
    for (int fb = 0; fb < KF / 32; ++fb) dst[32 * fb + lr] = g1[fb][q];
    dst[KF + lr] = g2[0][q];
    dst[KF + 32 + lr] = g2[1][q];
  }
}

// ============================================================================
// Fused backward, round-3 form: the same four products with the recompute chains
// swapped to ROWS x HIDDEN output tiles,
//   P1[row][h]  = AX[row][:] W1[:][h] (+ b1),   dP1[row][h] = dY2[row][:] W2^T[:][h],
// so that the accumulators (lane = hidden unit, registers = 16 rows of the tile) are
// ALREADY the A operands of the contractions over the rows (dP1^T, H1^T: hidden x
// rows; the k order inside a 16-row step is permuted -- rows 4h..4h+3, 8+4h..8+4h+3
// -- and the transposed B reads of AX / dY2 use the same permutation).  Against the
// round-2 form above this removes, per wave and 32-row tile:
//   * the 10 b128 LDS reads of the weight fragments: each wave owns one 32-unit hidden
//     block for the whole launch, so its W1 / W2^T B fragments (KS + KC bf16x8) are
//     loaded once into registers and the weights need no LDS at all;
//   * the H1 / dP1 images (8 packed LDS writes, 8 transposed reads, a wave barrier).
// LDS is the double-buffered AX / dY2 staging (32 KiB) and a 128-B keep-bit image per
// wave and hidden block.  The dropout mask is the forward's (cgnn_common.h drop_draw):
// each lane draws for its (row, half) as the forward does and writes its 16 keep bits
// as one halfword of the image's word `row`; every lane then reads the 16 words of its
// rows (four b128 reads) and takes its unit's bit with a sign-extending bit-field
// extract -- the keep mask as an AND mask, no ballots, no per-element branches.  As
// in the forward the 1/(1-p) of the kept units is applied once, to the weight-gradient
// slab, not per element.  The bias is added in the epilogue (packed), not as the
// accumulator's initial value.
// ============================================================================
constexpr size_t fused_bwd2_lds(int HD) { return sizeof(uint16_t) * 2 * 2 * 32 * 128 + sizeof(uint32_t) * HD; }

// TB hidden blocks per wave (1: HD/32 waves of <= 256 registers, 2 waves / SIMD; 2: HD/64
// waves of up to 512 registers -- accumulators in AGPRs -- one wave / SIMD, and every
// LDS fragment a wave reads (the AX / dY2 rows, the transposed contraction operands)
// feeds two hidden blocks' MFMAs, half the LDS traffic per tile)
template <int KS, int KC, int HD, int DROP, int TB>
__global__ __launch_bounds__(HD * 2 / TB, 1) void gcn_fused_bwd2_kernel(
    const uint16_t* __restrict__ AX, const uint16_t* __restrict__ dY2, const float* __restrict__ W1,
    const float* __restrict__ b1, const float* __restrict__ W2, float* __restrict__ gpart, int n, int F,
    int ldx, int C, int ldc, float p, uint32_t k0, uint32_t k1, uint32_t step, uint32_t thr8,
    uint32_t row0, const int* __restrict__ stepp) {
  if (stepp) step = (uint32_t)*stepp;         // device-resident dropout step (graph replays)
  constexpr int NW = HD / 32 / TB;            // waves per block; wave w owns hidden blocks w + NW b
  constexpr int NT = NW * 64;
  constexpr int KP = KS * 16;                 // layer-1 K (features + ones column), padded
  constexpr int KF = (KP + 31) / 32 * 32;     // gW1^T columns (f), padded to whole tiles
  constexpr int CP = KC * 16;                 // classes, padded
  static_assert(KF <= 128 && CP <= 64, "staging rows are 256 B");
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* sStg = lds;                       // 2 x (AX [32][128] | dY2 [32][128]), stg_off swizzle
  uint32_t* sKeep = reinterpret_cast<uint32_t*>(lds + 2 * 2 * TILE * 128);   // [NW * TB][32] words

  const int tid = threadIdx.x;
  const int lane = tid & 63, h = lane >> 5, lr = lane & 31;
  const int wv = tid >> 6;
  const int gb = (lane >> 4) & 1, qq = (lane >> 2) & 3, pq = lane & 3;

  // B fragments of the two recompute chains (lane = hidden unit, k = 16 s + 8 h + j)
  bf16x8 w1f[TB][KS], w2f[TB][KC];
  float bias[TB];
#pragma unroll
  for (int b = 0; b < TB; ++b) {
    const int hid = 32 * (wv + NW * b) + lr;  // this lane's hidden unit in block b
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 16 * s + 8 * h + j;
        const float v = W1[(size_t)min(k, F - 1) * HD + hid];
        w1f[b][s][j] = (__bf16)(k < F ? v : 0.f);
      }
#pragma unroll
    for (int s = 0; s < KC; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = 16 * s + 8 * h + j;
        const float v = W2[(size_t)hid * C + min(c, C - 1)];
        w2f[b][s][j] = (__bf16)(c < C ? v : 0.f);
      }
    bias[b] = b1[hid];
  }
  for (int i = tid; i < 2 * 2 * TILE * 128 / 8; i += NT)
    reinterpret_cast<uint4*>(sStg)[i] = make_uint4(0u, 0u, 0u, 0u);

  const int n_tiles = (n + TILE - 1) / TILE;
  const float scale = 1.f / (1.f - p);
  const int xch = min(ldx, KP) / 8, ych = min(ldc, CP) / 8;
  // this lane's hidden unit lr in the keep-bit image words: bit 16 half + q with
  // half = (lr >> 2) & 1, q = 4 (lr >> 3) + (lr & 3) (the forward's register order)
  const uint32_t kpos = 16u * ((lr >> 2) & 1) + 4u * (lr >> 3) + (lr & 3);

  f32x16 g1[TB][KF / 32], g2[TB][2];
#pragma unroll
  for (int b = 0; b < TB; ++b) {
#pragma unroll
    for (int q = 0; q < KF / 32; ++q) g1[b][q] = f32x16{};
    g2[b][0] = f32x16{};
    g2[b][1] = f32x16{};
  }

  constexpr int PFX = (TILE * (KP / 8) + NT - 1) / NT, PFY = (TILE * (CP / 8) + NT - 1) / NT;
  uint4 pax[PFX], pdy[PFY];
  auto prefetch = [&](int tile) {
    const int r0 = tile * TILE;
#pragma unroll
    for (int k = 0; k < PFX; ++k) {
      const int i = tid + k * NT;
      const int rr = i % TILE, ch = i / TILE;
      pax[k] = (i < TILE * xch && r0 + rr < n)
                   ? *reinterpret_cast<const uint4*>(AX + (size_t)(r0 + rr) * ldx + 8 * ch)
                   : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int k = 0; k < PFY; ++k) {
      const int i = tid + k * NT;
      const int rr = i % TILE, ch = i / TILE;
      pdy[k] = (i < TILE * ych && r0 + rr < n)
                   ? *reinterpret_cast<const uint4*>(dY2 + (size_t)(r0 + rr) * ldc + 8 * ch)
                   : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto stage = [&](int buf) {
    char* const bA = reinterpret_cast<char*>(sStg + buf * 2 * TILE * 128);
    char* const bD = bA + 2 * TILE * 128;
#pragma unroll
    for (int k = 0; k < PFX; ++k) {
      const int i = tid + k * NT;
      if (i < TILE * xch) *reinterpret_cast<uint4*>(bA + stg_off(i % TILE, i / TILE)) = pax[k];
    }
#pragma unroll
    for (int k = 0; k < PFY; ++k) {
      const int i = tid + k * NT;
      if (i < TILE * ych) *reinterpret_cast<uint4*>(bD + stg_off(i % TILE, i / TILE)) = pdy[k];
    }
  };
  const int G = gridDim.x;
  __syncthreads();                            // the zeroed staging images
  if ((int)blockIdx.x < n_tiles) {
    prefetch(blockIdx.x);
    stage(0);
    if ((int)blockIdx.x + G < n_tiles) prefetch(blockIdx.x + G);
  }
  __syncthreads();

  int it = 0;
  for (int tile = blockIdx.x; tile < n_tiles; tile += G, ++it) {
    const int cur = it & 1;
    if (tile + G < n_tiles) {                 // stage the next tile, prefetch the one after
      stage(cur ^ 1);
      if (tile + 2 * G < n_tiles) prefetch(tile + 2 * G);
    }
    const uint16_t* const sAX = sStg + cur * 2 * TILE * 128;
    const uint16_t* const sDY = sAX + TILE * 128;
    const char* const bAX = reinterpret_cast<const char*>(sAX);
    const char* const bDY = reinterpret_cast<const char*>(sDY);

    // ---- recompute P1 and dP1 (rows x hidden blocks; lane = hidden, regs = rows) ----
    f32x16 acc[TB], dh[TB];
#pragma unroll
    for (int b = 0; b < TB; ++b) {
      acc[b] = f32x16{};
      dh[b] = f32x16{};
    }
    {
      bf16x8 x1[KS], y2[KC];
#pragma unroll
      for (int s = 0; s < KS; ++s) x1[s] = load_bf16x8(reinterpret_cast<const uint16_t*>(bAX + stg_off(lr, 2 * s + h)));
#pragma unroll
      for (int s = 0; s < KC; ++s) y2[s] = load_bf16x8(reinterpret_cast<const uint16_t*>(bDY + stg_off(lr, 2 * s + h)));
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int b = 0; b < TB; ++b) {
          acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x1[s], w1f[b][s], acc[b], 0, 0, 0);
          if (s < KC) dh[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(y2[s], w2f[b][s], dh[b], 0, 0, 0);
        }
    }
    // H1 = dropout(relu(P1 + b1)), dP1 = dh * [H1 > 0] (both without the 1/(1-p), applied
    // to the slab), as the contractions' A operands (register 8 s + j = row
    // 16 s + 8 (j / 4) + 4 h + j % 4)
    bf16x8 ah1[TB][2], adp[TB][2];
    static_assert(HD <= 256, "bit-mode dropout: one draw covers 8 hidden blocks");
    u32x4 rb{};             // bit mode: the draw of (row lr, half h), shared by every block
    if constexpr (DROP == 2) rb = drop_draw(row0 + (uint32_t)(tile * TILE + lr), 0, h, step, k0, k1, true);
#pragma unroll
    for (int b = 0; b < TB; ++b) {
      uint4 kw[4];          // keep-bit words of rows 8 g + 4 h + 0..3
      if constexpr (DROP != 0) {
        const int t = wv + NW * b;
        const uint32_t m = drop_keep16(DROP == 2 ? rb : drop_draw(row0 + (uint32_t)(tile * TILE + lr), t, h, step,
                                                                  k0, k1, false),
                                       t, thr8, DROP == 2);
        uint32_t* img = sKeep + (wv * TB + b) * 32;
        reinterpret_cast<uint16_t*>(img)[2 * lr + h] = (uint16_t)m;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
        for (int g = 0; g < 4; ++g) kw[g] = *reinterpret_cast<const uint4*>(img + 8 * g + 4 * h);
      }
      const f2 bb = {bias[b], bias[b]};
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const f2 z = f2{acc[b][r], acc[b][r + 1]} + bb;
        float x[2] = {fmaxf(z.x, 0.f), fmaxf(z.y, 0.f)};
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int rr = r + e;
          if constexpr (DROP != 0) {
            const uint4 q4 = kw[rr >> 2];
            const uint32_t wd = (rr & 3) == 0 ? q4.x : (rr & 3) == 1 ? q4.y : (rr & 3) == 2 ? q4.z : q4.w;
            x[e] = keep_and(x[e], wd, kpos);
          }
          ah1[b][rr >> 3][rr & 7] = (__bf16)x[e];
          adp[b][rr >> 3][rr & 7] = (__bf16)(x[e] > 0.f ? dh[b][rr] : 0.f);
        }
      }
    }

    // ---- contractions over the tile's 32 rows (two k-steps of 16, permuted rows) ----
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int ra = 16 * s2 + 4 * h + qq;      // block rows ra (+8 for the second read)
      const int cb = 2 * gb + (pq >> 1), cx = 8 * (pq & 1);
#pragma unroll
      for (int q = 0; q < KF / 32; ++q) {
        const bf16x8 bx = tr_frag(sAX, stg_off(ra, 4 * q + cb) + cx, stg_off(ra + 8, 4 * q + cb) + cx);
#pragma unroll
        for (int b = 0; b < TB; ++b) g1[b][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(adp[b][s2], bx, g1[b][q], 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const bf16x8 by = tr_frag(sDY, stg_off(ra, 4 * q + cb) + cx, stg_off(ra + 8, 4 * q + cb) + cx);
#pragma unroll
        for (int b = 0; b < TB; ++b) g2[b][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah1[b][s2], by, g2[b][q], 0, 0, 0);
      }
    }
    __syncthreads();      // this buffer is rewritten two tiles on; the next one is staged
  }

  // ---- this block's partial slab: rows = hidden 32t + m, columns [f | KF + c] ----
  const float gs = DROP != 0 ? scale : 1.f;   // the kept units' 1/(1-p)
  float* gp = gpart + (size_t)blockIdx.x * HD * (KF + 64);
#pragma unroll
  for (int b = 0; b < TB; ++b) {
    const int t = wv + NW * b;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int hrow = 32 * t + (q & 3) + 8 * (q >> 2) + 4 * h;
      float* dst = gp + (size_t)hrow * (KF + 64);
#pragma unroll
      for (int fb = 0; fb < KF / 32; ++fb) dst[32 * fb + lr] = g1[b][fb][q] * gs;
      dst[KF + lr] = g2[b][0][q] * gs;
      dst[KF + 32 + lr] = g2[b][1][q] * gs;
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

template <int KS, int HD, int DROP>
static int fwd_launch_d(const uint16_t* AX, const float* W1, const float* b1, const float* W2,
                        const float* dinv, uint16_t* H1, uint16_t* Z2, int n, int F, int ldx, int C,
                        int ldc, float p, uint32_t k0, uint32_t k1, uint32_t step, uint32_t thr8,
                        uint32_t row0, const int* stepp, hipStream_t st) {
  const size_t lds = sizeof(uint16_t) * ((size_t)HD * (KS * 16 + 8) + 64 * (size_t)(HD + 8)) + sizeof(float) * HD;
  (void)hipFuncSetAttribute((const void*)gcn_dense_fwd_kernel<KS, HD, DROP>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((gcn_dense_fwd_kernel<KS, HD, DROP>), dim3(dense_grid(n)), dim3(WAVES * 64), lds, st, AX, W1,
                     b1, W2, dinv, H1, Z2, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0, stepp);
  return (int)hipGetLastError();
}

template <int KS, int HD>
static int fwd_launch(const uint16_t* AX, const float* W1, const float* b1, const float* W2,
                      const float* dinv, uint16_t* H1, uint16_t* Z2, int n, int F, int ldx, int C,
                      int ldc, float p, uint32_t k0, uint32_t k1, uint32_t step, uint32_t thr8,
                      uint32_t row0, const int* stepp, hipStream_t st) {
  if (thr8 == 128)
    return fwd_launch_d<KS, HD, 2>(AX, W1, b1, W2, dinv, H1, Z2, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0,
                                   stepp, st);
  if (thr8 > 0)
    return fwd_launch_d<KS, HD, 1>(AX, W1, b1, W2, dinv, H1, Z2, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0,
                                   stepp, st);
  return fwd_launch_d<KS, HD, 0>(AX, W1, b1, W2, dinv, H1, Z2, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0,
                                     stepp, st);
}

extern "C" int gnn_launch_dense_fwd(const void* AX, const float* W1, const float* b1, const float* W2,
                                    const float* dinv, void* H1, void* Z2, int n, int F, int ldx,
                                    int HD, int C, int ldc, float p, uint32_t k0, uint32_t k1,
                                    uint32_t step, uint32_t row0, const int* stepp, hipStream_t st) {
  if (C > 64 || ldc % 8 || ldx % 8 || ldc > 64) return -3;
  const uint32_t thr8 = (uint32_t)std::min(255.0, std::floor((double)p * 256.0 + 0.5));
  const int KS = (F + 15) / 16;
  auto* ax = (const uint16_t*)AX;
  auto* h1 = (uint16_t*)H1;
  auto* z2 = (uint16_t*)Z2;
#define FWD(ks, hd) if (KS <= ks && HD == hd) return fwd_launch<ks, hd>(ax, W1, b1, W2, dinv, h1, z2, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0, stepp, st);
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

// ---- fused backward launcher ----
extern "C" int gnn_fused_bwd_blocks(int n) {
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
  return std::max(1, std::min(cus, tiles));
}

// width of one gpart row (gW1^T columns padded to whole 32-tiles, then 64 for gW2);
// K = F + 1 (features and the ones column)
extern "C" int gnn_fused_bwd_width(int K) {
  const int KP = (K + 15) / 16 * 16;
  return (KP + 31) / 32 * 32 + 64;
}

template <int KS, int KC, int HD>
static int fused_bwd_launch(const uint16_t* AX, const uint16_t* dY2, const float* W1, const float* b1,
                            const float* W2, float* gpart, int n, int F, int ldx, int C, int ldc, float p,
                            uint32_t k0, uint32_t k1, uint32_t step, uint32_t thr8, uint32_t row0,
                            const int* stepp, hipStream_t st) {
  constexpr int KP = KS * 16, CP = KC * 16;
  // round-3 form by default; env CGNN_FUSED_BWD_V1=1 launches the round-2 form (A/B)
  static const bool v1 = [] {
    const char* e = std::getenv("CGNN_FUSED_BWD_V1");
    return e && e[0] && e[0] != '0';
  }();
  // hidden blocks per wave of the round-3 form: env CGNN_FUSED_BWD_TB (1 or 2, default 1:
  // 680 vs 772 us on the ogbn-products shape, profiles/r03_bwd)
  static const int tb = [] {
    const char* e = std::getenv("CGNN_FUSED_BWD_TB");
    return e && e[0] == '2' ? 2 : 1;
  }();
  if (!v1) {
    const size_t lds = fused_bwd2_lds(HD);
    const int dm = thr8 == 128 ? 2 : thr8 > 0 ? 1 : 0;
    auto kern = tb == 1 ? (dm == 2 ? gcn_fused_bwd2_kernel<KS, KC, HD, 2, 1>
                           : dm == 1 ? gcn_fused_bwd2_kernel<KS, KC, HD, 1, 1> : gcn_fused_bwd2_kernel<KS, KC, HD, 0, 1>)
                        : (dm == 2 ? gcn_fused_bwd2_kernel<KS, KC, HD, 2, 2>
                           : dm == 1 ? gcn_fused_bwd2_kernel<KS, KC, HD, 1, 2> : gcn_fused_bwd2_kernel<KS, KC, HD, 0, 2>);
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(gnn_fused_bwd_blocks(n)), dim3(HD * 2 / tb), lds, st,
                       AX, dY2, W1, b1, W2, gpart, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0, stepp);
    return (int)hipGetLastError();
  }
  const size_t lds2 = fused_bwd_lds(KP, CP, HD, 2);
  const size_t lds = lds2 <= 160 * 1024 ? lds2 : fused_bwd_lds(KP, CP, HD, 1);
  if (lds > 160 * 1024) return -2;
  auto kern = thr8 > 0 ? gcn_fused_bwd_kernel<KS, KC, HD, true> : gcn_fused_bwd_kernel<KS, KC, HD, false>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(gnn_fused_bwd_blocks(n)), dim3(HD * 2), lds, st,
                     AX, dY2, W1, b1, W2, gpart, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0, stepp);
  return (int)hipGetLastError();
}

// K = F + 1 (features and the ones column), C classes; the row pitches only need to
// cover them (multiples of 8)
extern "C" int gnn_fused_bwd_supported(int K, int HD, int C) {
  const int KS = (K + 15) / 16, KC = (C + 15) / 16;
  if (C > 64) return 0;
  if (HD == 256) return (KS == 4 || KS == 7 || KS == 8) && (KC == 3 || KC == 4);
  if (HD == 128) return ((KS == 7 || KS == 8 || KS == 4) && KC == 3) || (KS == 8 && KC == 4);
  return 0;
}

// AX: [n][ldx] bf16 with the ones column at F (ldx covers F + 1); dY2: [n][ldc] bf16.
// gpart: [gnn_fused_bwd_blocks(n)][HD][gnn_fused_bwd_width(ldx)] fp32.
// Returns -1 when no compiled variant covers the shape.
extern "C" int gnn_launch_fused_bwd(const void* AX, const void* dY2, const float* W1, const float* b1,
                                    const float* W2, float* gpart, int n, int F, int ldx, int HD, int C,
                                    int ldc, float p, uint32_t k0, uint32_t k1, uint32_t step, uint32_t row0,
                                    const int* stepp, hipStream_t st) {
  if (C > 64 || ldc % 8 || ldx % 8 || C > ldc || F + 1 > ldx) return -3;
  const uint32_t thr8 = (uint32_t)std::min(255.0, std::floor((double)p * 256.0 + 0.5));
  const int KS = (F + 1 + 15) / 16, KC = (C + 15) / 16;
  auto* ax = (const uint16_t*)AX;
  auto* dy = (const uint16_t*)dY2;
#define FB(ks, kc, hd) if (KS == ks && KC == kc && HD == hd) return fused_bwd_launch<ks, kc, hd>(ax, dy, W1, b1, W2, gpart, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0, stepp, st);
  FB(7, 3, 256) FB(7, 4, 256) FB(8, 3, 256) FB(8, 4, 256) FB(4, 3, 256) FB(4, 4, 256)
  FB(7, 3, 128) FB(8, 3, 128) FB(4, 3, 128) FB(8, 4, 128)
#undef FB
  return -1;
}
