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
#include <type_traits>

using namespace cgnn;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

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

// packed bf16 epilogue helpers (cvt_pk, pk_relu, pk_mul16, pk_nz): cgnn_common.h

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
//
// Keep image (kimg, optional, training only): the dropout masks the fused backward
// applies, so that it draws no Philox of its own (bit mode: one draw per row and half
// here feeds both passes; the byte-mode launch draws the image with
// gcn_keep_image_kernel, which keeps this kernel within its register budget).  For
// 32-row tile T and hidden block t, 64 halfwords at kimg[(T * HD/32 + t) * 64]: halfword 32 uh + r = the 16 keep bits of tile row r for
// the units 32 t + 8 g + 4 uh + i (bit 4 g + i) -- halfword index = the lane that drew
// them, so each block's image is one contiguous 128-B store per wave.  Read as 32-bit
// words, word 16 uh + P holds rows 2P (low half) and 2P + 1 (high half).
//
// The next tile's AX rows are loaded right after the last hidden block's layer-1 MFMAs
// (the registers of the current rows are dead from there), so the loads fly during
// that block's epilogue, its layer-2 products and the Z2 stores.
template <int KS, int HD, int DROP>
__global__ __launch_bounds__(WAVES * 64) void gcn_dense_fwd_kernel(
    const uint16_t* __restrict__ AX, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ W2, const float* __restrict__ dinv, uint16_t* __restrict__ H1,
    uint16_t* __restrict__ Z2, int n, int F, int ldx, int C, int ldc, float p, uint32_t k0,
    uint32_t k1, uint32_t step, uint32_t thr8, uint32_t row0, const int* __restrict__ stepp,
    uint16_t* __restrict__ kimg) {
  // stepp (optional): the dropout step read from device memory, so a captured hipGraph
  // replays with the current epoch's mask
  if (stepp) step = (uint32_t)*stepp;
  constexpr int KP = KS * 16;
  constexpr int W1S = KP + 8;          // padded row strides (bank-conflict-free b128 / b64 reads)
  // W2^T rows of HD + 4 elements: a 130-dword pitch puts the 32 rows of a b64 read on
  // 32 distinct bank pairs (HD + 8 -- 132 dwords -- made rows r and r + 16 collide)
  constexpr int W2S = HD + 4;
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

  // A tile's rows.  Hoisted form: unconditional loads (a per-lane "load or zero" makes
  // hipcc branch around every load); rows past n load row n - 1 (their results are not
  // stored), and only the last k-step can pass the row pitch (F > 16 (KS - 1), ldx >= F,
  // ldx % 8 == 0): its upper half then loads the row's last chunk, which meets zero W1^T
  // rows (k >= F).
  // The hoisted next-tile loads fit the 128-register budget of 4 waves / SIMD only in
  // the bit-mode (p = 1/2) form up to 112 features: the other forms load each tile at
  // its start (and keep the per-lane "load or zero" form, which needs fewer registers)
  constexpr bool HOIST = DROP == 2 && KS <= 7;
  bf16x8 bx[KS];
  // the row's D^-1/2 is loaded with its rows: loaded at the Z2 stores it was the newest
  // load, and waiting for it meant waiting for the next tile's rows (the prefetch) too
  float dsv = 0.f;
  auto load_rows = [&](int tl) {
    dsv = dinv[min(tl * TILE + lr, n - 1)];
    if constexpr (HOIST) {
      const uint16_t* rp = AX + (size_t)min(tl * TILE + lr, n - 1) * ldx;
#pragma unroll
      for (int s = 0; s < KS - 1; ++s) bx[s] = load_bf16x8(rp + 16 * s + 8 * h);
      bx[KS - 1] = load_bf16x8(rp + min(16 * (KS - 1) + 8 * h, ldx - 8));
    } else {
      const int rw = tl * TILE + lr;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int f0 = 16 * s + 8 * h;
        bx[s] = (rw < n && f0 < ldx) ? load_bf16x8(AX + (size_t)rw * ldx + f0) : zero_bf16x8();
      }
    }
  };
  if (HOIST && wave < n_tiles) {
    load_rows(wave);
    // the first tile's rows consumed here (empty asm): with loads still pending on the
    // loop's entry edge the wait-count pass merged it into a vmcnt(0) at every tile start,
    // which also drained the previous tile's Z2 / keep-image stores
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const uint4 u = __builtin_bit_cast(uint4, bx[s]);
      asm volatile("" ::"v"(u.x), "v"(u.y), "v"(u.z), "v"(u.w));
    }
    asm volatile("" ::"v"(dsv));
  }
  for (int tile = wave; tile < n_tiles; tile += n_waves) {
    const int row = tile * TILE + lr;
    const bool rv = row < n;
    if constexpr (!HOIST) load_rows(tile);
    const float dsc = dsv;                    // this tile's (the prefetch overwrites dsv)
    f32x16 z0 = {}, z1 = {};
    static_assert(HD <= 256, "bit-mode dropout: one draw covers 8 hidden blocks");
    u32x4 rb{};
    if constexpr (DROP == 2) rb = drop_draw(row0 + (uint32_t)row, 0, h, step, k0, k1, true);
    // one hidden block: layer-1 chain, epilogue, layer-2 products; the last block is
    // peeled (LAST) so the next tile's row loads there do not keep a second set of row
    // registers live across the whole block loop
    auto hidden_block = [&](const int t, auto last_tag) {
      constexpr bool LAST = decltype(last_tag)::value;
      const uint16_t* arow = sW1T + (32 * t + lr) * W1S + 8 * h;
      // the chain's weight fragments in two LDS batches (registers: 4 waves / SIMD)
      constexpr int KA = (KS + 1) / 2;
      bf16x8 af[KA];
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < KA; ++s) af[s] = load_bf16x8(arow + 16 * s);
#pragma unroll
      for (int s = 0; s < KA; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bx[s], acc, 0, 0, 0);
#pragma unroll
      for (int s = KA; s < KS; ++s) af[s - KA] = load_bf16x8(arow + 16 * s);
#pragma unroll
      for (int s = KA; s < KS; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s - KA], bx[s], acc, 0, 0, 0);
      if constexpr (LAST && HOIST)
        if (tile + n_waves < n_tiles) load_rows(tile + n_waves);
      // epilogue (registers 4g..4g+3 are hidden 32t + 8g + 4h + 0..3) on packed bf16
      // pairs: bias (packed fp32 adds), one v_cvt_pk_bf16_f32, relu as v_pk_max_i16 and the
      // two keep bits as one v_pk_mul_lo_u16 per pair (the scale is in W2^T); the same
      // bits as relu and the keep AND in fp32 followed by the conversion
      uint32_t pk[8];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 bb = *reinterpret_cast<const float4*>(sB1 + 32 * t + 8 * g + 4 * h);
        const f2 lo = f2{acc[4 * g], acc[4 * g + 1]} + f2{bb.x, bb.y};
        const f2 hi = f2{acc[4 * g + 2], acc[4 * g + 3]} + f2{bb.z, bb.w};
        pk[2 * g] = pk_relu(cvt_pk(lo.x, lo.y));
        pk[2 * g + 1] = pk_relu(cvt_pk(hi.x, hi.y));
      }
      if constexpr (DROP != 0) {
        const uint32_t mw = keep_spread(drop_keep16(
            DROP == 2 ? rb : drop_draw(row0 + (uint32_t)row, t, h, step, k0, k1, false), t, thr8, DROP == 2));
#pragma unroll
        for (int i = 0; i < 8; ++i) pk[i] = pk_mul16(pk[i], (mw >> (2 * i)) & 0x10001u);
      }
      if (rv && H1) {          // H1 == nullptr: the fused backward recomputes it
        uint32_t o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
          o[i] = cvt_pk(__uint_as_float(pk[i] << 16) * w2s, __uint_as_float(pk[i] & 0xffff0000u) * w2s);
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<uint2*>(H1 + (size_t)row * HD + 32 * t + 8 * g + 4 * h) = make_uint2(o[2 * g], o[2 * g + 1]);
      }
      // second product: Z2^T += W2^T[:, 32t..32t+31] * H1^T tile (accumulator as B operand)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 xb = __builtin_bit_cast(bf16x8, make_uint4(pk[4 * s2], pk[4 * s2 + 1], pk[4 * s2 + 2], pk[4 * s2 + 3]));
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
    };
    if constexpr (HOIST) {
#pragma unroll 1
      for (int t = 0; t < HD / 32 - 1; ++t) hidden_block(t, std::false_type{});
      hidden_block(HD / 32 - 1, std::true_type{});
    } else {
#pragma unroll 1
      for (int t = 0; t < HD / 32; ++t) hidden_block(t, std::false_type{});
    }
    if constexpr (DROP == 2) {               // the tile's keep image, straight from the draw
      if (kimg) {
        uint16_t* kd = kimg + (size_t)tile * (HD / 32) * 64 + lane;
#pragma unroll
        for (int t = 0; t < HD / 32; ++t) kd[64 * t] = (uint16_t)drop_keep16(rb, t, thr8, true);
      }
    }
    if (rv) {
      const float ds = dsc;
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
//   P1 = AX W1 (+ b1),  H1 = dropout(relu(P1))          (the forward's masks: kimg)
//   dP1 = (dY2 W2^T) * [H1 > 0]                         (1/(1-p) applied to the slab)
//   gW1^T[h][f] += sum_rows dP1^T[h][row] AX[row][f]    (f = F, the ones column: gb1)
//   gW2[h][c]   += sum_rows H1^T[h][row] dY2[row][c]
// Block = HD/32 waves; wave w owns hidden block w (32 units) for all four products,
// so its W1 / W2^T B fragments (KS + KC bf16x8) sit in registers for the whole launch
// and its weight-gradient tiles in its accumulators.  The recompute chains
// (v_mfma_f32_32x32x16_bf16, K = 16 KS exactly) produce ROWS x HIDDEN tiles (lane =
// hidden unit, registers = 16 rows of the tile).  The contractions over the 32 rows
// run on v_mfma_f32_16x16x32_bf16 (K = 32 rows in one instruction; output tiles of
// 16 hidden x 16 features, so the gradient's feature / class padding is to 16, not 32:
// KS + KC tiles per hidden half instead of 2 (KF/32 + 2) 32x32 halves -- 9 % fewer MFMA
// cycles and 16 fewer accumulator registers).  Their A operands (16 hidden x 32 rows)
// come from the recompute accumulators by one v_permlane16_swap per packed dword pair:
// lane groups 0 / 2 keep the pairs {0, 1, 4, 5} of their 32x32 rows and trade {2, 3,
// 6, 7} with groups 1 / 3, which then hold the other hidden half -- k-slot e of lane
// group g is tile row b_g + (e & 3) + 16 (e >> 2), b_g = 8 (g & 1) + 4 (g >> 1), and
// the transposed B reads of AX / dY2 fetch those rows (conflict-free in the swizzled
// image: the rows one 32-lane half reads differ in bits 2-3).  Per 32-row tile the
// block stages the AX / dY2 rows once, row-major in swizzled 256-B rows (the recompute
// reads them by rows with b128, the contractions by columns with ds_read_b64_tr_b16),
// and the tile's keep image from the forward; double-buffered behind a register
// prefetch of the tile after next: one block barrier per tile.
// Round 6 (profiles/r06_bwd): this form 429-440 us against 445-449 for the round-5
// 32x32 contractions.  Measured slower and not kept: waves 4-7 staggered by half a tile
// (contraction of tile t - 1 before tile t's recompute; ring of three buffers; 590 us --
// two code paths, 256 VGPRs and spills), and a software pipeline in every wave (tile
// t + 1's epilogue interleaved with tile t's contractions by sched_group_barrier, the
// weight fragments moved to LDS to make room; 530 us).
// Epilogue on packed bf16 pairs (two rows per dword): relu as a signed 16-bit max, the
// keep bits and the relu derivative as 16-bit multiplies by 0 / 1 -- no compares,
// selects or per-element bit extracts, and no Philox: the forward drew the masks (a
// draw costs ~60 VALU instructions, a third of them quarter-rate 32-bit multiplies,
// and every wave of the round-3 form re-drew its tile's).
// Output: one fp32 slab per block, gpart[block][HD][KF + 64] = [gW1^T | gW2] (KF = the
// feature columns rounded up to 32; padding columns written 0), summed in fixed order
// afterwards.
// ============================================================================
// LDS bytes: two staging buffers (AX | dY2, [32][128] bf16 each) + two keep images
constexpr size_t fused_bwd_lds(int HD) { return sizeof(uint16_t) * 2 * 2 * 32 * 128 + 2 * (size_t)(HD / 32) * 128; }

template <int KS, int KC, int HD, bool DROP>
__global__ __launch_bounds__(HD * 2, 1) void gcn_fused_bwd_kernel(
    const uint16_t* __restrict__ AX, const uint16_t* __restrict__ dY2, const float* __restrict__ W1,
    const float* __restrict__ b1, const float* __restrict__ W2, const uint16_t* __restrict__ kimg,
    float* __restrict__ gpart, int n, int F, int ldx, int C, int ldc, float p) {
  constexpr int NW = HD / 32;                 // waves per block = hidden blocks
  constexpr int NT = NW * 64;
  constexpr int KP = KS * 16;                 // layer-1 K (features + ones column), padded
  constexpr int KF = (KP + 31) / 32 * 32;     // gW1^T slab columns (f), 32-aligned
  constexpr int CP = KC * 16;                 // classes, padded
  constexpr int NF = KS;                      // 16-wide feature tiles of the contraction
  constexpr int KCH = DROP ? NW * 8 : 0;      // 16-B chunks of one tile's keep image
  static_assert(KF <= 128 && CP <= 64, "staging rows are 256 B");
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* sStg = lds;                       // 2 x (AX [32][128] | dY2 [32][128]), stg_off swizzle
  uint32_t* sKeep = reinterpret_cast<uint32_t*>(lds + 2 * 2 * TILE * 128);   // 2 x [NW][32] words

  const int tid = threadIdx.x;
  const int lane = tid & 63, h = lane >> 5, lr = lane & 31;
  const int wv = tid >> 6;
  const int qq = (lane >> 2) & 3, pq = lane & 3;

  // B fragments of the two recompute chains (lane = hidden unit, k = 16 s + 8 h + j)
  bf16x8 w1f[KS], w2f[KC];
  const int hid = 32 * wv + lr;               // this lane's hidden unit
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * s + 8 * h + j;
      const float v = W1[(size_t)min(k, F - 1) * HD + hid];
      w1f[s][j] = (__bf16)(k < F ? v : 0.f);
    }
#pragma unroll
  for (int s = 0; s < KC; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = 16 * s + 8 * h + j;
      const float v = W2[(size_t)hid * C + min(c, C - 1)];
      w2f[s][j] = (__bf16)(c < C ? v : 0.f);
    }
  const f2 bb = {b1[hid], b1[hid]};
  // the stationary fragments consumed here (empty asm): otherwise the wait-count pass keeps
  // counting their ~80 loads behind the loop's prefetch loads, and the first use inside the
  // loop becomes a vmcnt(0) every tile -- draining the prefetch
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const uint4 u = __builtin_bit_cast(uint4, w1f[s]);
    asm volatile("" ::"v"(u.x), "v"(u.y), "v"(u.z), "v"(u.w));
  }
#pragma unroll
  for (int s = 0; s < KC; ++s) {
    const uint4 u = __builtin_bit_cast(uint4, w2f[s]);
    asm volatile("" ::"v"(u.x), "v"(u.y), "v"(u.z), "v"(u.w));
  }
  asm volatile("" ::"v"(bb.x));
  for (int i = tid; i < 2 * 2 * TILE * 128 / 8; i += NT)
    reinterpret_cast<uint4*>(sStg)[i] = make_uint4(0u, 0u, 0u, 0u);

  const int n_tiles = (n + TILE - 1) / TILE;
  const float scale = 1.f / (1.f - p);
  const int xch = min(ldx, KP) / 8, ych = min(ldc, CP) / 8;
  // this lane's unit in the keep image: the drawing lane's unit half uh, bit kq
  const int uh = (lr >> 2) & 1;
  const uint32_t kq = 4u * (lr >> 3) + (lr & 3);

  f32x4 g1[2][NF], g2[2][KC];                 // [hidden half][16-wide column tile]
#pragma unroll
  for (int hb = 0; hb < 2; ++hb) {
#pragma unroll
    for (int q = 0; q < NF; ++q) g1[hb][q] = f32x4{};
#pragma unroll
    for (int q = 0; q < KC; ++q) g2[hb][q] = f32x4{};
  }

  // prefetch registers: AX chunks i = tid + k NT (chunk i = row i % 32, column chunk
  // i / 32); dY2 chunks in the same form, and the tile's keep image (KCH chunks) in the
  // slots [TILE * CP / 8, + KCH) of the dY2 index space
  constexpr int KB = TILE * (CP / 8);
  constexpr int PFX = (TILE * (KP / 8) + NT - 1) / NT, PFY = (KB + KCH + NT - 1) / NT;
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
      if (i < TILE * ych && r0 + rr < n)
        pdy[k] = *reinterpret_cast<const uint4*>(dY2 + (size_t)(r0 + rr) * ldc + 8 * ch);
      else if (KCH && i >= KB && i < KB + KCH)
        pdy[k] = reinterpret_cast<const uint4*>(kimg + (size_t)tile * NW * 64)[i - KB];
      else
        pdy[k] = make_uint4(0u, 0u, 0u, 0u);
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
      if (i < TILE * ych)
        *reinterpret_cast<uint4*>(bD + stg_off(i % TILE, i / TILE)) = pdy[k];
      else if (KCH && i >= KB && i < KB + KCH)
        reinterpret_cast<uint4*>(sKeep + buf * NW * 32)[i - KB] = pdy[k];
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

    // ---- recompute P1 and dP1 (rows x hidden block; lane = hidden, regs = rows) ----
    f32x16 acc = {}, dh = {};
    {
      bf16x8 x1[KS], y2[KC];
#pragma unroll
      for (int s = 0; s < KS; ++s) x1[s] = load_bf16x8(reinterpret_cast<const uint16_t*>(bAX + stg_off(lr, 2 * s + h)));
#pragma unroll
      for (int s = 0; s < KC; ++s) y2[s] = load_bf16x8(reinterpret_cast<const uint16_t*>(bDY + stg_off(lr, 2 * s + h)));
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x1[s], w1f[s], acc, 0, 0, 0);
        if (s < KC) dh = __builtin_amdgcn_mfma_f32_32x32x16_bf16(y2[s], w2f[s], dh, 0, 0, 0);
      }
    }
    // register pair i = registers 2i, 2i + 1 = tile rows 2P, 2P + 1 with
    // P = 4 (i / 2) + 2 h + i % 2: its keep word (rows 2P / 2P + 1 in the low / high
    // half, this unit's bit at kq) is word 16 uh + P of the block's image
    uint32_t kw[8];
    if constexpr (DROP) {
      const uint32_t* img = sKeep + cur * NW * 32 + wv * 32 + uh * 16 + 2 * h;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint2 w = *reinterpret_cast<const uint2*>(img + 4 * g);
        kw[2 * g] = w.x;
        kw[2 * g + 1] = w.y;
      }
    }
    // H1 = dropout(relu(P1 + b1)) and dP1 = dh * [H1 > 0], both without the 1/(1-p)
    // (applied to the slab), as packed bf16 pairs: the contractions' A operands
    // (fragment s, dword d = register pair 4 s + d)
    uint32_t ah[8], ad[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f2 z = f2{acc[2 * i], acc[2 * i + 1]} + bb;
      uint32_t x = pk_relu(cvt_pk(z.x, z.y));
      if constexpr (DROP) x = pk_mul16(x, (kw[i] >> kq) & 0x10001u);
      ah[i] = x;
      ad[i] = pk_mul16(cvt_pk(dh[2 * i], dh[2 * i + 1]), pk_nz(x));
    }
    // 16x16x32 A operands of the two hidden halves (see the header): pairs {0, 1, 4, 5}
    // stay, {2, 3, 6, 7} go to the neighbouring lane group
    bf16x8 aH[2], aD[2];
    {
      constexpr int KEEP[4] = {0, 1, 4, 5}, SEND[4] = {2, 3, 6, 7};
      uint32_t h0[4], h1[4], d0[4], d1[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const auto sh = __builtin_amdgcn_permlane16_swap(ah[KEEP[k]], ah[SEND[k]], false, false);
        const auto sd = __builtin_amdgcn_permlane16_swap(ad[KEEP[k]], ad[SEND[k]], false, false);
        h0[k] = sh[0];
        h1[k] = sh[1];
        d0[k] = sd[0];
        d1[k] = sd[1];
      }
      aH[0] = __builtin_bit_cast(bf16x8, make_uint4(h0[0], h0[1], h0[2], h0[3]));
      aH[1] = __builtin_bit_cast(bf16x8, make_uint4(h1[0], h1[1], h1[2], h1[3]));
      aD[0] = __builtin_bit_cast(bf16x8, make_uint4(d0[0], d0[1], d0[2], d0[3]));
      aD[1] = __builtin_bit_cast(bf16x8, make_uint4(d1[0], d1[1], d1[2], d1[3]));
    }

    // ---- contractions over the tile's 32 rows: one 16x16x32 MFMA per output tile ----
    // B fragment of column tile q: rows rb and rb + 16 (k-slots 0..3 / 4..7) of lane
    // group g4, 16 columns from chunk 2q; lane 4 qq + pq addresses row qq, columns 4 pq
    {
      const int g4 = lane >> 4;
      const int rb = 8 * (g4 & 1) + 4 * (g4 >> 1) + qq;
      const int cx = 8 * (pq & 1);
#pragma unroll
      for (int q = 0; q < NF; ++q) {
        const int ch = 2 * q + (pq >> 1);
        const bf16x8 bx = tr_frag(sAX, stg_off(rb, ch) + cx, stg_off(rb + 16, ch) + cx);
        g1[0][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aD[0], bx, g1[0][q], 0, 0, 0);
        g1[1][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aD[1], bx, g1[1][q], 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < KC; ++q) {
        const int ch = 2 * q + (pq >> 1);
        const bf16x8 by = tr_frag(sDY, stg_off(rb, ch) + cx, stg_off(rb + 16, ch) + cx);
        g2[0][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aH[0], by, g2[0][q], 0, 0, 0);
        g2[1][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aH[1], by, g2[1][q], 0, 0, 0);
      }
    }
    __syncthreads();      // this buffer is rewritten two tiles on; the next one is staged
  }

  // ---- this block's partial slab: rows = hidden 32 wv + 16 hb + m, columns [f | KF + c]
  // (16x16 tile: lane = column, register v = row 4 (lane >> 4) + v); padding columns 0 ----
  const float gs = DROP ? scale : 1.f;        // the kept units' 1/(1-p)
  float* gp = gpart + (size_t)blockIdx.x * HD * (KF + 64);
  const int cl = lane & 15;
#pragma unroll
  for (int hb = 0; hb < 2; ++hb) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      float* dst = gp + (size_t)(32 * wv + 16 * hb + 4 * (lane >> 4) + v) * (KF + 64);
#pragma unroll
      for (int q = 0; q < NF; ++q) dst[16 * q + cl] = g1[hb][q][v] * gs;
#pragma unroll
      for (int q = NF; q < KF / 16; ++q) dst[16 * q + cl] = 0.f;
#pragma unroll
      for (int q = 0; q < KC; ++q) dst[KF + 16 * q + cl] = g2[hb][q][v] * gs;
#pragma unroll
      for (int q = KC; q < 4; ++q) dst[KF + 16 * q + cl] = 0.f;
    }
  }
}

// The keep image of the forward (gcn_dense_fwd_kernel, kimg) drawn on its own, for a
// backward that runs without that forward: one lane per (tile row, unit half), the
// same Philox draws.
__global__ __launch_bounds__(256) void gcn_keep_image_kernel(uint16_t* __restrict__ kimg, int n, int NB,
                                                             uint32_t thr8, uint32_t k0, uint32_t k1, uint32_t step,
                                                             uint32_t row0, const int* __restrict__ stepp) {
  if (stepp) step = (uint32_t)*stepp;
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int n_tiles = (n + TILE - 1) / TILE;
  const int tile = (int)(gid >> 6), lane = (int)(gid & 63);
  if (tile >= n_tiles) return;
  const uint32_t row = row0 + (uint32_t)(tile * TILE + (lane & 31));
  const int h = lane >> 5;
  const bool bit = drop_bit_mode(thr8);
  const u32x4 rb = drop_draw(row, 0, h, step, k0, k1, true);
  for (int t = 0; t < NB; ++t)
    kimg[(size_t)(tile * NB + t) * 64 + lane] =
        (uint16_t)drop_keep16(bit ? rb : drop_draw(row, t, h, step, k0, k1, false), t, thr8, bit);
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
                        uint32_t row0, const int* stepp, uint16_t* kimg, hipStream_t st) {
  const size_t lds = sizeof(uint16_t) * ((size_t)HD * (KS * 16 + 8) + 64 * (size_t)(HD + 4)) + sizeof(float) * HD;
  (void)hipFuncSetAttribute((const void*)gcn_dense_fwd_kernel<KS, HD, DROP>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((gcn_dense_fwd_kernel<KS, HD, DROP>), dim3(dense_grid(n)), dim3(WAVES * 64), lds, st, AX, W1,
                     b1, W2, dinv, H1, Z2, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0, stepp, kimg);
  if (DROP == 1 && kimg) {
    const long lanes = (long)((n + TILE - 1) / TILE) * 64;
    hipLaunchKernelGGL(gcn_keep_image_kernel, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, st, kimg, n,
                       HD / 32, thr8, k0, k1, step, row0, stepp);
  }
  return (int)hipGetLastError();
}

template <int KS, int HD>
static int fwd_launch(const uint16_t* AX, const float* W1, const float* b1, const float* W2,
                      const float* dinv, uint16_t* H1, uint16_t* Z2, int n, int F, int ldx, int C,
                      int ldc, float p, uint32_t k0, uint32_t k1, uint32_t step, uint32_t thr8,
                      uint32_t row0, const int* stepp, uint16_t* kimg, hipStream_t st) {
  if (thr8 == 128)
    return fwd_launch_d<KS, HD, 2>(AX, W1, b1, W2, dinv, H1, Z2, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0,
                                   stepp, kimg, st);
  if (thr8 > 0)
    return fwd_launch_d<KS, HD, 1>(AX, W1, b1, W2, dinv, H1, Z2, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0,
                                   stepp, kimg, st);
  return fwd_launch_d<KS, HD, 0>(AX, W1, b1, W2, dinv, H1, Z2, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0,
                                 stepp, kimg, st);
}

static uint32_t drop_thr8(float p) { return (uint32_t)std::min(255.0, std::floor((double)p * 256.0 + 0.5)); }

// kimg (optional): the keep image for the fused backward, gnn_keep_image_halfwords(n, HD)
// halfwords, written when the launch draws dropout masks
extern "C" int gnn_launch_dense_fwd(const void* AX, const float* W1, const float* b1, const float* W2,
                                    const float* dinv, void* H1, void* Z2, int n, int F, int ldx,
                                    int HD, int C, int ldc, float p, uint32_t k0, uint32_t k1,
                                    uint32_t step, uint32_t row0, const int* stepp, void* kimg, hipStream_t st) {
  if (C > 64 || ldc % 8 || ldx % 8 || ldc > 64) return -3;
  const uint32_t thr8 = drop_thr8(p);
  const int KS = (F + 15) / 16;
  auto* ax = (const uint16_t*)AX;
  auto* h1 = (uint16_t*)H1;
  auto* z2 = (uint16_t*)Z2;
  auto* ki = (uint16_t*)kimg;
#define FWD(ks, hd) if (KS <= ks && HD == hd) return fwd_launch<ks, hd>(ax, W1, b1, W2, dinv, h1, z2, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0, stepp, ki, st);
  FWD(4, 256) FWD(7, 256) FWD(8, 256) FWD(4, 128) FWD(8, 128)
#undef FWD
  return -1;
}

// halfwords of the keep image of n rows at HD hidden units (1 bit per element, whole tiles)
extern "C" long gnn_keep_image_halfwords(int n, int HD) { return (long)((n + TILE - 1) / TILE) * (HD / 32) * 64; }

extern "C" int gnn_launch_keep_image(void* kimg, int n, int HD, float p, uint32_t k0, uint32_t k1, uint32_t step,
                                     uint32_t row0, const int* stepp, hipStream_t st) {
  if (HD % 32 || HD > 256) return -3;
  const uint32_t thr8 = drop_thr8(p);
  if (thr8 == 0) return 0;
  const long lanes = (long)((n + TILE - 1) / TILE) * 64;
  hipLaunchKernelGGL(gcn_keep_image_kernel, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, st,
                     (uint16_t*)kimg, n, HD / 32, thr8, k0, k1, step, row0, stepp);
  return (int)hipGetLastError();
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
                            const float* W2, const uint16_t* kimg, float* gpart, int n, int F, int ldx, int C,
                            int ldc, float p, bool drop, hipStream_t st) {
  const size_t lds = fused_bwd_lds(HD);
  auto kern = drop ? gcn_fused_bwd_kernel<KS, KC, HD, true> : gcn_fused_bwd_kernel<KS, KC, HD, false>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(gnn_fused_bwd_blocks(n)), dim3(HD * 2), lds, st,
                     AX, dY2, W1, b1, W2, kimg, gpart, n, F, ldx, C, ldc, p);
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

// AX: [n][ldx] bf16 with the ones column at F (ldx covers F + 1); dY2: [n][ldc] bf16;
// kimg: the forward's keep image of the same n rows (gnn_launch_dense_fwd / _keep_image),
// required when p draws masks.  gpart: [gnn_fused_bwd_blocks(n)][HD][gnn_fused_bwd_width(ldx)]
// fp32.  Returns -1 when no compiled variant covers the shape.
extern "C" int gnn_launch_fused_bwd(const void* AX, const void* dY2, const float* W1, const float* b1,
                                    const float* W2, const void* kimg, float* gpart, int n, int F, int ldx, int HD,
                                    int C, int ldc, float p, hipStream_t st) {
  if (C > 64 || ldc % 8 || ldx % 8 || C > ldc || F + 1 > ldx) return -3;
  const bool drop = drop_thr8(p) > 0;
  if (drop && !kimg) return -3;
  const int KS = (F + 1 + 15) / 16, KC = (C + 15) / 16;
  auto* ax = (const uint16_t*)AX;
  auto* dy = (const uint16_t*)dY2;
  auto* ki = (const uint16_t*)kimg;
#define FB(ks, kc, hd) if (KS == ks && KC == kc && HD == hd) return fused_bwd_launch<ks, kc, hd>(ax, dy, W1, b1, W2, ki, gpart, n, F, ldx, C, ldc, p, drop, st);
  FB(7, 3, 256) FB(7, 4, 256) FB(8, 3, 256) FB(8, 4, 256) FB(4, 3, 256) FB(4, 4, 256)
  FB(7, 3, 128) FB(8, 3, 128) FB(4, 3, 128) FB(8, 4, 128)
#undef FB
  return -1;
}
