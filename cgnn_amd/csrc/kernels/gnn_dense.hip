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
// DROP: dropout active (p > 0), a compile-time switch so the epilogue has no per-element
// branches.
//
// Latency structure (the kernel runs 4 waves / SIMD -- one 16-wave block per CU -- and
// was measured MFMA-busy ~23 %): per hidden tile t the accumulator starts as the bias
// (4 b128 LDS reads issued ahead, fp32 exact) instead of a bias add per element after
// the chain, and the KS weight fragments of the chain are read from LDS as one batch
// before the first MFMA rather than one LDS round trip per MFMA.
template <int KS, int HD, bool DROP>
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
      // accumulator = bias: registers 4g..4g+3 are hidden 32t + 8g + 4h + 0..3
      f32x16 acc;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 bb = *reinterpret_cast<const float4*>(sB1 + 32 * t + 8 * g + 4 * h);
        acc[4 * g] = bb.x; acc[4 * g + 1] = bb.y; acc[4 * g + 2] = bb.z; acc[4 * g + 3] = bb.w;
      }
      const uint16_t* arow = sW1T + (32 * t + lr) * W1S + 8 * h;
      bf16x8 af[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) af[s] = load_bf16x8(arow + 16 * s);
#pragma unroll
      for (int s = 0; s < KS; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bx[s], acc, 0, 0, 0);
      // epilogue: relu, dropout (one Philox draw = this lane's 16 bytes)
      float v[16];
      if constexpr (DROP) {
        const u32x4 r = philox4x32_10(u32x4{row0 + (uint32_t)row, (uint32_t)(2 * t + h), step, RNG_DROPOUT}, k0, k1);
        const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const float x = fmaxf(acc[q], 0.f);
          v[q] = (((w[q >> 2] >> (8 * (q & 3))) & 0xffu) >= thr8) ? x * scale : 0.f;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = fmaxf(acc[q], 0.f);
      }
      if (rv && H1) {          // H1 == nullptr: the fused backward recomputes it
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
    uint32_t w[4] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
    if constexpr (DROP) {
      const u32x4 r = philox4x32_10(u32x4{row0 + (uint32_t)row, (uint32_t)(2 * t + h), step, RNG_DROPOUT}, k0, k1);
      w[0] = r.x; w[1] = r.y; w[2] = r.z; w[3] = r.w;
    }
    // registers 4g..4g+3 = hidden 32t + 8g + 4h + 0..3 of this lane's row: one packed
    // 8-B write per image and g
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float xv[4], dv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = 4 * g + i;
        float x = fmaxf(acc[q], 0.f);
        if constexpr (DROP) x = (((w[g] >> (8 * i)) & 0xffu) >= thr8) ? x * scale : 0.f;
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

template <int KS, int HD, bool DROP>
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
  if (thr8 > 0)
    return fwd_launch_d<KS, HD, true>(AX, W1, b1, W2, dinv, H1, Z2, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0,
                                      stepp, st);
  return fwd_launch_d<KS, HD, false>(AX, W1, b1, W2, dinv, H1, Z2, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0,
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
