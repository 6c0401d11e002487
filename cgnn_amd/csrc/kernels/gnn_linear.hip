// Generic fused dense layers of the GNN track on MFMA (gfx950, v_mfma_f32_32x32x16_bf16).
//
// The dense half of every message-passing layer is a tall-skinny product: millions
// of rows, K and N of a few hundred.  Three kernels cover the forward and both
// backward products of any such layer (GraphSAGE, the GAT projection, every layer of
// the L-layer GCN), bf16 storage and fp32 accumulation throughout:
//
//   lin_fwd         Y = epi([X1 | X2] W + b)      epi: ReLU, Philox dropout, row scale
//   lin_bwd_data    [dX1 | dX2] = rs * ((dY * m) W^T)     m = [Ym > 0] / (1 - p)
//   lin_bwd_weight  [dW; db] = [X1 | X2 | 1]^T (dY * m)   split-K over row chunks
//
// [X1 | X2] is a VIRTUAL concatenation along the features (GraphSAGE's
// [h_dst | mean-aggregate] without the copy); W is the fp32 master weight
// [K1 + K2][N] (row-major), staged into LDS as bf16 once per persistent block.
// The mask m of the backward kernels is applied while the gradient rows are
// loaded: Ym is the layer's stored output (after ReLU and dropout), so Ym > 0
// marks exactly the units that were kept and active -- neither the mask nor the
// masked gradient is ever materialised.
//
// Forward / data-backward compute the output TRANSPOSED (tile = [feature][row]):
// the A operand is a weight slab in LDS, the B operand is 16 contiguous bytes of
// one row per lane, loaded from HBM in the natural row-major layout, and each
// lane ends up owning 16 features of one row -- one Philox draw per lane and
// 32-feature tile supplies exactly its 16 dropout bytes (the mask convention of
// gnn_dense.hip / ops.dropout_keep_mask: draw (row, 2*(n/32) + (n/4)%2, step),
// byte (n%4) + 4*((n%32)/8)).
//
// The weight gradient contracts over rows, so both operands must hold 8
// consecutive ROWS per lane: each 32-row tile of [X1 | X2 | 1] and of the masked
// gradient is staged in LDS transposed ([column][row]; chunks assigned
// row-fastest so a wave's 2-byte transposed writes are contiguous, no bank
// conflicts), the next tile is prefetched into registers meanwhile; every wave
// keeps its [k-tile][n-tile] accumulators for the whole row chunk and the
// per-chunk fp32 slabs are summed in a fixed order by lin_reduce (deterministic,
// no atomics).
#include "cgnn_common.h"
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

using namespace cgnn;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8v __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int TILE = 32;
// persistent blocks share one LDS weight slab: 16 waves (4 per SIMD, <= 128 VGPRs) up
// to K = 256, 8 waves (<= 256 VGPRs) for the wider variants, whose B fragments alone
// take 4 * KS registers
template <int KS> struct FwdWaves { static constexpr int value = KS <= 16 ? 16 : 8; };
constexpr int WGT_WAVES = 8;        // weight-gradient blocks
constexpr bool BWD_DATA_SEL = true;   // lin_bwd_data: branch-free gradient loader
constexpr int WS_RING = 3;             // lin_ws: register ring depth (tiles in flight; 5 measured no faster)
constexpr int FWD8_WAVES = 8;         // lin_fwd KS = 8: waves per block (prefetching 8-wave blocks, profiles/r04_lin)
constexpr int FWD16_WAVES = 8;        // lin_fwd KS = 16: waves per block (profiles/r03_waves)
constexpr int BWD16_WAVES = 8;        // lin_bwd_data KN = 16: waves per block (profiles/r03_waves)
constexpr int FWD_SEL_KS = 8;         // lin_fwd: branch-free X loader from this many k-steps up
constexpr int TR = TILE + 8;        // transposed image row: 32 rows + pad (80 B)

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8, v); }

typedef short v4s __attribute__((ext_vector_type(4)));

// ds_read_b64_tr_b16 pair -> one 32x32x16 operand fragment (lane 4q+p of a 16-lane group
// addresses row q, columns 4p..4p+3 of a 4x16 block; lane i receives column i).
__device__ __forceinline__ bf16x8 tr_frag(const uint8_t* base, int off0, int off1) {
  typedef __attribute__((address_space(3))) v4s lds_v4s;
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(base + off0));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(base + off1));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

__device__ __forceinline__ uint16_t bf16_bits(float x) { return __builtin_bit_cast(uint16_t, (__bf16)x); }

__device__ __forceinline__ float bf16_val(uint32_t bits16) { return __uint_as_float(bits16 << 16); }

__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
  return make_uint2((uint32_t)bf16_bits(a) | ((uint32_t)bf16_bits(b) << 16),
                    (uint32_t)bf16_bits(c) | ((uint32_t)bf16_bits(d) << 16));
}

// element type ET of the 16-bit operands: 0 = bf16 (training storage), 1 = fp16 (the
// fp16 inference path)
__device__ __forceinline__ uint16_t f16_bits(float x) { return __builtin_bit_cast(uint16_t, (_Float16)x); }
template <int ET>
__device__ __forceinline__ uint16_t e16_bits(float x) { return ET == 1 ? f16_bits(x) : bf16_bits(x); }
template <int ET>
__device__ __forceinline__ uint2 pack4e(float a, float b, float c, float d) {
  return make_uint2((uint32_t)e16_bits<ET>(a) | ((uint32_t)e16_bits<ET>(b) << 16),
                    (uint32_t)e16_bits<ET>(c) | ((uint32_t)e16_bits<ET>(d) << 16));
}
template <int ET>
__device__ __forceinline__ f32x16 mma16(uint4 a, uint4 b, f32x16 c) {
  if constexpr (ET == 1)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8v, a), __builtin_bit_cast(f16x8v, b), c,
                                                   0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                    0, 0, 0);
}

// zero the elements [valid, 8) of a bf16x8 chunk (padding columns may hold anything,
// and 0 * NaN would poison a product)
__device__ __forceinline__ uint4 keep_first(uint4 v, int valid) {
  if (valid >= 8) return v;
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int lo = 2 * e, hi = 2 * e + 1;
    w[e] = (lo < valid ? (w[e] & 0xffffu) : 0u) | (hi < valid ? (w[e] & 0xffff0000u) : 0u);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// branch-free form (selects only), valid may be <= 0
__device__ __forceinline__ uint4 keep_first_sel(uint4 v, int valid) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t lo = 2 * e < valid ? 0x0000ffffu : 0u, hi = 2 * e + 1 < valid ? 0xffff0000u : 0u;
    w[e] &= lo | hi;
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// 8 features [f0, f0 + 8) of row `row` of the virtual concatenation [X1 | X2]
// (K1 % 8 == 0 when X2 is given, so a chunk never straddles the two); zeros past K1 + K2
// idx1 (optional): X1 row of output row r is idx1[r] (gather-on-load: GraphSAGE's
// first layer reads the seed / frontier rows straight out of the resident features)
__device__ __forceinline__ uint4 load_cat8(const uint16_t* __restrict__ x1, int ld1, int K1,
                                           const uint16_t* __restrict__ x2, int ld2, int K2, int row, int f0,
                                           const int* __restrict__ idx1) {
  if (f0 < K1) {
    const size_t r1 = idx1 ? (size_t)idx1[row] : (size_t)row;
    return keep_first(*reinterpret_cast<const uint4*>(x1 + r1 * ld1 + f0), K1 - f0);
  }
  const int g = f0 - K1;
  if (x2 && g < K2) return keep_first(*reinterpret_cast<const uint4*>(x2 + (size_t)row * ld2 + g), K2 - g);
  return make_uint4(0u, 0u, 0u, 0u);
}

// Branch-free load_cat8 for lin_fwd's unrolled k loop: every lane loads from a valid
// address (a chunk outside both operands re-reads its row's first chunk) and the value
// is masked afterwards.  The per-lane branches of load_cat8, unrolled KS times, cost
// exec-mask saves that spilled the SGPR file (KS = 40: 1259 SGPR spills); this form has
// none up to KS = 40 and measured 365 vs 410 us on Reddit's K = 602 layer.  Since round 3
// it serves KS >= 8 too: the branchy form left lin_fwd<16> at 491 SGPR + 11 VGPR spills
// (64.1 -> 57.8 us at SAGE layer-0 shapes, products-sage3 7.96 -> 8.17 epochs/s,
// profiles/r03_linsel); KS = 4 keeps load_cat8.
__device__ __forceinline__ uint4 load_cat8_sel(const uint16_t* __restrict__ x1, int ld1, int K1,
                                               const uint16_t* __restrict__ x2, int ld2, int K2, int row, int f0,
                                               const int* __restrict__ idx1) {
  const size_t r1 = idx1 ? (size_t)idx1[row] : (size_t)row;
  const int g = f0 - K1;
  const bool in1 = f0 < K1;
  const bool in2 = x2 != nullptr && !in1 && g < K2;
  const uint16_t* p = in2 ? x2 + (size_t)row * ld2 + g : x1 + r1 * ld1 + (in1 ? f0 : 0);
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  return keep_first_sel(v, in1 ? K1 - f0 : in2 ? K2 - g : 0);
}

// g * [y > 0] * mscale per bf16 element (has_y false: g * mscale)
__device__ __forceinline__ uint4 mask8(uint4 g, uint4 y, bool has_y, float mscale) {
  uint32_t gw[4] = {g.x, g.y, g.z, g.w};
  const uint32_t yw[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    uint32_t o = 0;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const uint32_t yb = (yw[w] >> (16 * half)) & 0xffffu;
      // kept and active: y > 0 (positive, non-zero)
      const bool keep = !has_y || ((yb & 0x7fffu) != 0 && !(yb & 0x8000u));
      const float v = keep ? bf16_val((gw[w] >> (16 * half)) & 0xffffu) * mscale : 0.f;
      o |= (uint32_t)bf16_bits(v) << (16 * half);
    }
    gw[w] = o;
  }
  return make_uint4(gw[0], gw[1], gw[2], gw[3]);
}

// 8 gradient values [c0, c0 + 8) of row `row`, times the mask [Ym > 0] * mscale
__device__ __forceinline__ uint4 load_masked8(const uint16_t* __restrict__ dY, int lddy,
                                              const uint16_t* __restrict__ Ym, int ldym, float mscale,
                                              int N, int row, int c0) {
  if (c0 >= N) return make_uint4(0u, 0u, 0u, 0u);
  uint4 g = keep_first(*reinterpret_cast<const uint4*>(dY + (size_t)row * lddy + c0), N - c0);
  if (!Ym && mscale == 1.f) return g;
  const uint4 y = Ym ? *reinterpret_cast<const uint4*>(Ym + (size_t)row * ldym + c0) : make_uint4(~0u, ~0u, ~0u, ~0u);
  return mask8(g, y, Ym != nullptr, mscale);
}

// Branch-free load_masked8 (selects only, every lane loads from a valid address: the
// caller clamps `row`; `rv` false zeroes the chunk): unrolled over a k loop, the per-lane
// branches of load_masked8 cost exec-mask saves that spill the SGPR file.
__device__ __forceinline__ uint4 load_masked8_sel(const uint16_t* __restrict__ dY, int lddy,
                                                  const uint16_t* __restrict__ Ym, int ldym, float mscale,
                                                  int N, int row, int c0, bool rv) {
  const int cc = c0 < N ? c0 : 0;
  const uint4 g = keep_first_sel(*reinterpret_cast<const uint4*>(dY + (size_t)row * lddy + cc), rv ? N - c0 : 0);
  if (!Ym && mscale == 1.f) return g;
  const uint4 y = Ym ? *reinterpret_cast<const uint4*>(Ym + (size_t)row * ldym + cc) : make_uint4(~0u, ~0u, ~0u, ~0u);
  return mask8(g, y, Ym != nullptr, mscale);
}

// raw 16-byte chunk f0 of [X1 | X2] row `row`, zero outside both operands.  The padding
// columns past K1 / K2 are NOT zeroed (for products that discard those rows), so no
// instruction consumes the loaded value and the load stays in flight until it is staged.
__device__ __forceinline__ uint4 load_cat8_raw(const uint16_t* __restrict__ x1, int ld1, int K1,
                                               const uint16_t* __restrict__ x2, int ld2, int K2, int row, int f0,
                                               const int* __restrict__ idx1) {
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (f0 < K1) {
    const size_t r1 = idx1 ? (size_t)idx1[row] : (size_t)row;
    v = *reinterpret_cast<const uint4*>(x1 + r1 * ld1 + f0);
  } else if (x2 && f0 - K1 < K2) {
    v = *reinterpret_cast<const uint4*>(x2 + (size_t)row * ld2 + (f0 - K1));
  }
  return v;
}

// block-wide copy of a weight image global -> LDS with 8 loads in flight per thread: a
// plain strided loop waits on every load before its LDS store (a serial chain of L2
// round trips, ~30 us per launch for a 133 KB image -- it dominated the small layers
// of a GraphSAGE mini-batch)
__device__ __forceinline__ void copy_image(uint4* __restrict__ dst, const uint4* __restrict__ src, int n16) {
  const int bd = blockDim.x;
  int i = threadIdx.x;
  for (; i + 7 * bd < n16; i += 8 * bd) {
    uint4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[i + u * bd];
#pragma unroll
    for (int u = 0; u < 8; ++u) dst[i + u * bd] = v[u];
  }
  for (; i < n16; i += bd) dst[i] = src[i];
}

}  // namespace

// ============================================================================
// lin_fwd: Y[row][c] = epi(sum_k [X1 | X2][row][k] W[k][c] + b[c]) for the column
// slab c in [blockIdx.y * ncols, +ncols); KS k-steps of 16 cover K1 + K2.
//
// Epilogue on packed 16-bit pairs: the accumulators start from the bias (b128 LDS
// reads), the dropout scale 1/(1-p) is folded into the weight image and the bias
// (relu(z) / (1-p) = relu(z / (1-p))), so per pair of outputs the epilogue is one
// v_cvt_pk_bf16_f32, one v_pk_max_i16 (relu; identity with a floor of -32768) and one
// v_pk_mul_lo_u16 by the two keep bits.  In bit mode (p = 1/2) one Philox draw covers
// eight 32-column tiles.  The next tile's X rows load while this tile computes (KS <= 16:
// a second set of B fragments fits the VGPR budget), and the first tile's rows load
// before the weight image is staged.
// ============================================================================
// Output staging of one wave's 32-row x 32-column bf16 tile (lane (lr, h) holds row lr,
// columns 8 g + 4 h + 0..3 in pk[2 g], pk[2 g + 1]): through a per-wave LDS tile (rows of
// 80 B) so that each global store instruction writes 16 whole 64-B row segments
// (16 B per lane, 4 lanes per row) instead of 32 rows x 16 B -- every store leaves L2 as
// its own fabric requests, so the narrow pieces cost ~4x the bytes' time.  emit(r, c, v):
// global row r (< n), column offset c in {0, 8, 16, 24}, 8 bf16 values.
constexpr int OST_PITCH = 80, OST_BYTES = 32 * OST_PITCH;
template <class Emit>
__device__ __forceinline__ void out_stage(uint16_t* lds, int ost, const uint32_t (&pk)[8], int tile, int n, Emit emit) {
  const int lane = threadIdx.x & 63, h = lane >> 5, lr = lane & 31;
  uint8_t* so = reinterpret_cast<uint8_t*>(lds) + ost + (threadIdx.x >> 6) * OST_BYTES;
#pragma unroll
  for (int g = 0; g < 4; ++g) *reinterpret_cast<uint2*>(so + lr * OST_PITCH + 16 * g + 8 * h) = make_uint2(pk[2 * g], pk[2 * g + 1]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 16 * i + (lane >> 2), c = lane & 3;
    const uint4 v = *reinterpret_cast<const uint4*>(so + r * OST_PITCH + 16 * c);
    if (tile * TILE + r < n) emit(tile * TILE + r, 8 * c, v);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void st_y8(uint16_t* p, uint32_t a, uint32_t b) {
  *reinterpret_cast<uint2*>(p) = make_uint2(a, b);
}

template <int KS, int ET = 0, int FWD_WAVES = FwdWaves<KS>::value>
__global__ __launch_bounds__(FWD_WAVES * 64) void lin_fwd_kernel(
    const uint16_t* __restrict__ x1, int ld1, int K1, const uint16_t* __restrict__ x2, int ld2, int K2,
    const float* __restrict__ W, int N, const float* __restrict__ bias, uint16_t* __restrict__ Y, int ldy,
    int n, int ncols, int relu, float p, uint32_t k0, uint32_t k1, uint32_t step, uint32_t thr8,
    uint32_t row0, const int* __restrict__ stepp, const float* __restrict__ rscale, const int* __restrict__ idx1,
    const uint16_t* __restrict__ wimg, float* __restrict__ Yf, int nsplit, int tk, int ost) {
  // wimg: the bf16 LDS image of every column slab ([slabs][ncols][WS], lin_prep_fwd_kernel,
  // times 1/(1-p) when dropout is on): one vectorised copy per block instead of converting /
  // transposing the fp32 weights.
  // Yf (optional): columns c >= nsplit (nsplit % 4 == 0) are written EXACTLY, as fp32
  // planes of tk columns -- Yf[(c - nsplit) / tk][row][(c - nsplit) % tk] -- instead of
  // bf16 into Y (GAT: the attention scores s_src / s_dst folded into the projection)
  // ost >= 0: byte offset of the per-wave output staging tiles in LDS (out_stage)
  if (stepp) step = (uint32_t)*stepp;
  constexpr int KP = KS * 16;
  constexpr int WS = KP + 8;                     // padded row stride of the W^T slab
  constexpr bool PF = KS <= 16 && FWD_WAVES <= 8;   // next-tile prefetch (256 VGPRs)
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* sWT = lds;                           // [ncols][WS]
  float* sB = reinterpret_cast<float*>(sWT + (size_t)ncols * WS);   // [ncols]: bias / (1 - p)
  const int c0 = blockIdx.y * ncols;
  const int lane = threadIdx.x & 63, h = lane >> 5, lr = lane & 31;
  const int n_waves = gridDim.x * FWD_WAVES;
  const int n_tiles = (n + TILE - 1) / TILE;
  const float scale = thr8 > 0 ? 1.f / (1.f - p) : 1.f;
  const bool bit = drop_bit_mode(thr8);
  const int nt = ncols / 32;
  const uint32_t floor16 = relu ? 0u : 0x80008000u;
  const bool full = c0 + ncols <= ldy && !Yf;    // every column of the slab is stored

  // K1 % 8 == 0 and K2 % 8 == 0: every 16-byte chunk is wholly inside or wholly outside
  // [X1 | X2], and a chunk outside re-reads its row's first chunk against zero weight rows
  // of the image, so no chunk needs masking (only a chunk straddling K holds padding
  // columns, which may hold anything)
  const bool ragged = (K1 & 7) || (K2 & 7);
  auto load = [&](int tile, uint4 (&bx)[KS]) {
    const int row = tile * TILE + lr;
    const bool rv = row < n;
    if constexpr (KS >= FWD_SEL_KS) {
      // wide K: branch-free addresses (per-lane branches unrolled KS times spill the SGPRs)
      const int rr = rv ? row : n - 1;
      const uint16_t* p1 = x1 + (idx1 ? (size_t)idx1[rr] : (size_t)rr) * ld1;
      const uint16_t* p2 = x2 ? x2 + (size_t)rr * ld2 : p1;
      // fh is opaque per tile (empty asm) so the per-k-step offsets and selects derived
      // from it are recomputed next to their loads instead of being hoisted out of the
      // tile loop as 2 * KS live registers
      int fh = 8 * h;
      asm volatile("" : "+v"(fh));
      if (!ragged) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const int f0 = 16 * s + fh, g = f0 - K1;
          bx[s] = *reinterpret_cast<const uint4*>(f0 < K1 ? p1 + f0 : g < K2 ? p2 + g : p1);
        }
      } else {
#pragma unroll
        for (int s = 0; s < KS; ++s)
          bx[s] = load_cat8_sel(x1, ld1, K1, x2, ld2, K2, rr, 16 * s + fh, idx1);
      }
    } else {
#pragma unroll
      for (int s = 0; s < KS; ++s)
        bx[s] = rv ? load_cat8(x1, ld1, K1, x2, ld2, K2, row, 16 * s + 8 * h, idx1) : make_uint4(0u, 0u, 0u, 0u);
    }
  };

  auto process = [&](int tile, const uint4 (&bx)[KS]) {
    const int row = tile * TILE + lr;
    const bool rv = row < n;
    const float rs = (rv && rscale) ? rscale[row] : 1.f;
    u32x4 r = {0u, 0u, 0u, 0u};
#pragma unroll 1
    for (int t = 0; t < nt; ++t) {
      const int tg = c0 / 32 + t;                // global 32-column tile
      f32x16 acc;
      {
        const float4* bp = reinterpret_cast<const float4*>(sB + 32 * t + 4 * h);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 bb = bp[2 * g];
          acc[4 * g] = bb.x; acc[4 * g + 1] = bb.y; acc[4 * g + 2] = bb.z; acc[4 * g + 3] = bb.w;
        }
      }
      const uint16_t* arow = sWT + (32 * t + lr) * WS + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s)
        acc = mma16<ET>(*reinterpret_cast<const uint4*>(arow + 16 * s), bx[s], acc);
      // (rows past n run the epilogue too: with staged stores their lanes carry other rows)
      uint32_t m = 0xffffu;
      if (thr8 > 0) {
        if (!bit || t == 0 || (tg & 7) == 0) {
          // opaque row id: the draw stays behind its condition (hoisted, it ran every tile t)
          uint32_t gr = row0 + (uint32_t)row;
          asm volatile("" : "+v"(gr));
          r = drop_draw(gr, tg, h, step, k0, k1, bit);
        }
        m = drop_keep16(r, tg, thr8, bit);
      }
      const int cg = 32 * tg;                    // global column of this tile
      if (Yf) {
        if (!rv) continue;
        float v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          float x = acc[q];
          if (relu) x = fmaxf(x, 0.f);
          v[q] = ((m >> q) & 1u) ? x * rs : 0.f;
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = cg + 8 * g + 4 * h;
          if (c >= nsplit) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int u = c + e - nsplit;
              if (c + e < N) Yf[(size_t)(u / tk) * n * tk + (size_t)row * tk + u % tk] = v[4 * g + e];
            }
          } else if (c < ldy) {
            *reinterpret_cast<uint2*>(Y + (size_t)row * ldy + c) =
                pack4e<ET>(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
          }
        }
        continue;
      }
      uint32_t pk[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const f2 z = f2{acc[2 * i], acc[2 * i + 1]} * rs;
        pk[i] = pk_max_i16(ET == 1 ? cvt_pk_h(z.x, z.y) : cvt_pk(z.x, z.y), floor16);
      }
      if (thr8 > 0) {
        const uint32_t mw = keep_spread(m);
#pragma unroll
        for (int i = 0; i < 8; ++i) pk[i] = pk_mul16(pk[i], (mw >> (2 * i)) & 0x10001u);
      }
      if (ost >= 0) {
        out_stage(lds, ost, pk, tile, n, [&](int r, int c, uint4 v) {
          if (full || cg + c < ldy) *reinterpret_cast<uint4*>(Y + (size_t)r * ldy + cg + c) = v;
        });
        continue;
      }
      if (!rv) continue;
      uint16_t* yrow = Y + (size_t)row * ldy + cg + 4 * h;
      if (full) {
#pragma unroll
        for (int g = 0; g < 4; ++g) st_y8(yrow + 8 * g, pk[2 * g], pk[2 * g + 1]);
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g)
          if (cg + 8 * g + 4 * h < ldy) st_y8(yrow + 8 * g, pk[2 * g], pk[2 * g + 1]);
      }
    }
  };

  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int tile = blockIdx.x * FWD_WAVES + wv;
  uint4 bxa[KS], bxb[KS];
  if (tile < n_tiles) load(tile, bxa);           // in flight while the weights are staged
  {
    const uint4* src = reinterpret_cast<const uint4*>(wimg + (size_t)blockIdx.y * ncols * WS);
    uint4* dst = reinterpret_cast<uint4*>(sWT);
    copy_image(dst, src, ncols * WS / 8);
  }
  for (int c = threadIdx.x; c < ncols; c += blockDim.x) sB[c] = (bias && c0 + c < N) ? bias[c0 + c] * scale : 0.f;
  __syncthreads();

  if constexpr (PF) {
    while (tile < n_tiles) {
      if (tile + n_waves < n_tiles) load(tile + n_waves, bxb);
      process(tile, bxa);
      tile += n_waves;
      if (tile >= n_tiles) break;
      if (tile + n_waves < n_tiles) load(tile + n_waves, bxa);
      process(tile, bxb);
      tile += n_waves;
    }
  } else {
    for (bool first = true; tile < n_tiles; tile += n_waves, first = false) {
      if (!first) load(tile, bxa);
      process(tile, bxa);
    }
  }
}

// ============================================================================
// lin_fwd_kc: the same product for weights too wide to sit in LDS whole (K * N * 2 B
// beyond the budget: Reddit's first layer, K = 602 x N = 256 fp16), where the slab form
// would re-read X once per column slab.  A plain tiled GEMM instead: the weight streams
// through LDS in K chunks of 32 (double-buffered, one block barrier per chunk) while
// each wave keeps a 64-row x 128-column output block in registers (2 x 4 accumulator
// tiles: every LDS weight fragment feeds two MFMAs) and reads its X rows straight from
// HBM as MFMA B fragments, one chunk ahead.  Block = 4 waves = FG feature groups of
// 128 columns x (4 / FG) row groups of 64 rows.  Epilogue: bias, ReLU, row scale.
// No dropout / concatenation / gather (the inference path; lin_fwd keeps those).
// ============================================================================
template <int FG, int ET>
__global__ __launch_bounds__(256, 2) void lin_fwd_kc_kernel(
    const uint16_t* __restrict__ x, int ldx, int K, const uint16_t* __restrict__ img, int KPc,
    const float* __restrict__ bias, uint16_t* __restrict__ Y, int ldy, int N, int n, int relu,
    const float* __restrict__ rscale) {
  // img: W^T as [FG * 128][KPc] 16-bit (zero past K and N), KPc % 32 == 0
  constexpr int BK = 32, LS = BK + 8, NP = FG * 128;
  constexpr int RG = 4 / FG;                     // row groups of 64 rows per block
  constexpr int WCH = NP * BK / 8 / 256;         // 16-B weight chunks per thread per K chunk
  __shared__ __attribute__((aligned(16))) uint16_t sW[2][NP * LS];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, lr = lane & 31, wv = tid >> 6;
  const int fg = wv % FG, rg = wv / FG;
  const int rbase = (blockIdx.x * RG + rg) * 64;   // this wave's 64 rows: two 32-row tiles
  int rows[2];
  bool rv[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int r = rbase + 32 * u + lr;
    rv[u] = r < n;
    rows[u] = rv[u] ? r : n - 1;
  }
  // accumulators start from the bias (the same rounding as lin_fwd's, which does the same)
  f32x16 acc[2][4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    f32x16 b0 = {};
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int c = 128 * fg + 32 * t + 8 * (q >> 2) + 4 * h + (q & 3);
      b0[q] = (bias && c < N) ? bias[c] : 0.f;
    }
    acc[0][t] = b0;
    acc[1][t] = b0;
  }
  const int nch = KPc / BK;
  uint4 wr[WCH];
  auto wload = [&](int c) {
#pragma unroll
    for (int j = 0; j < WCH; ++j) {
      const int i = tid + 256 * j, rr = i / (BK / 8), cc = i % (BK / 8);
      wr[j] = *reinterpret_cast<const uint4*>(img + (size_t)rr * KPc + c * BK + 8 * cc);
    }
  };
  auto wstore = [&](int buf) {
#pragma unroll
    for (int j = 0; j < WCH; ++j) {
      const int i = tid + 256 * j, rr = i / (BK / 8), cc = i % (BK / 8);
      *reinterpret_cast<uint4*>(&sW[buf][rr * LS + 8 * cc]) = wr[j];
    }
  };
  // X fragments of chunk c: k-steps s = 0, 1 at k = 32c + 16s + 8h for both row tiles;
  // chunks past K re-read column 0 and are masked (padding columns may hold anything)
  uint4 xb[2][2], xn[2][2];
  auto xload = [&](int c, uint4 (&dst)[2][2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int k = BK * c + 16 * s + 8 * h;
      const int kk = k < K ? k : 0;
#pragma unroll
      for (int u = 0; u < 2; ++u)
        dst[u][s] = keep_first_sel(*reinterpret_cast<const uint4*>(x + (size_t)rows[u] * ldx + kk), K - k);
    }
  };
  wload(0);
  xload(0, xb);
  wstore(0);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const int buf = c & 1;
    const bool more = c + 1 < nch;
    if (more) {
      wload(c + 1);
      xload(c + 1, xn);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint4 a = *reinterpret_cast<const uint4*>(&sW[buf][(128 * fg + 32 * t + lr) * LS + 16 * s + 8 * h]);
        acc[0][t] = mma16<ET>(a, xb[0][s], acc[0][t]);
        acc[1][t] = mma16<ET>(a, xb[1][s], acc[1][t]);
      }
    }
    if (more) {
      wstore(buf ^ 1);       // the other buffer: every wave finished reading it at the last barrier
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int s = 0; s < 2; ++s) xb[u][s] = xn[u][s];
    }
    __syncthreads();
  }
  // epilogue: lane = row, registers 4g..4g+3 = columns 32t + 8g + 4h + 0..3
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (!rv[u]) continue;
    const int row = rows[u];
    const float rs = rscale ? rscale[row] : 1.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 128 * fg + 32 * t + 8 * g + 4 * h;
        if (c >= ldy) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float y = acc[u][t][4 * g + e];
          if (relu) y = fmaxf(y, 0.f);
          v[e] = y * rs;
        }
        *reinterpret_cast<uint2*>(Y + (size_t)row * ldy + c) = pack4e<ET>(v[0], v[1], v[2], v[3]);
      }
    }
  }
}

// ============================================================================
// lin_gemm: Y = epi(X W) for a weight too wide for one LDS slab (K up to thousands,
// N <= 256; Reddit's 602-wide first layer): a 256-row x 256-column output tile per
// block of 8 waves (4 x 2, each 64 rows x 128 columns: 8 accumulators), X and the W^T
// image streamed through double-buffered LDS in K chunks of 64 (the next chunk's global
// loads in flight during the current chunk's 32 MFMAs per wave, one barrier per
// chunk).  LDS rows are 128 B; 16-B chunk c of row r is stored at c ^ ((r >> 1) & 7),
// which makes the ds_read_b128 fragment reads of any 16 consecutive rows hit 16
// distinct 4-bank groups.  Output computed transposed (lane = row) as in
// lin_fwd_kc_kernel; bias, ReLU and the row scale in the epilogue.
// ============================================================================
__device__ __forceinline__ int gemm_off(int r, int ch) { return r * 64 + 8 * (ch ^ ((r >> 1) & 7)); }
constexpr int GEMM_OST_PITCH = 272, GEMM_OST_BYTES = 64 * GEMM_OST_PITCH;   // epilogue staging per wave

template <int ET>
__global__ __launch_bounds__(512, 1) void lin_gemm_kernel(
    const uint16_t* __restrict__ x, int ldx, int K, const uint16_t* __restrict__ img, int KPc,
    const float* __restrict__ bias, uint16_t* __restrict__ Y, int ldy, int N, int n, int relu,
    const float* __restrict__ rscale) {
  constexpr int BM = 256, BK = 64;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* sX = lds;                       // [2][BM * BK]
  uint16_t* sW = lds + 2 * BM * BK;         // [2][256 * BK]
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, lr = lane & 31, wv = tid >> 6;
  const int rg = wv & 3, ng = wv >> 2;
  const int row0 = blockIdx.x * BM;
  const int nch = KPc / BK;
  // the staging registers as named scalars (as arrays captured by the lambdas they were
  // kept in scratch: 4 x 16 B stored and reloaded per chunk)
  uint4 xr0, xr1, xr2, xr3, wr0, wr1, wr2, wr3;
  auto load1 = [&](int c, int j, uint4& xv, uint4& wv) {
    const int i = tid + 512 * j, r = i >> 3, ch = i & 7;
    const int k = BK * c + 8 * ch;
    const int row = row0 + r;
    // raw: the mask is applied when the chunk is stored, so the loads stay in flight
    // through the current chunk's MFMAs (masked here, every load was waited for at once)
    xv = *reinterpret_cast<const uint4*>(x + (size_t)(row < n ? row : n - 1) * ldx + (k < K ? k : 0));
    wv = *reinterpret_cast<const uint4*>(img + (size_t)r * KPc + k);
  };
  auto load = [&](int c) {
    load1(c, 0, xr0, wr0);
    load1(c, 1, xr1, wr1);
    load1(c, 2, xr2, wr2);
    load1(c, 3, xr3, wr3);
  };
  auto store1 = [&](int buf, int c, int j, const uint4& xv, const uint4& wv) {
    const int i = tid + 512 * j, r = i >> 3, ch = i & 7;
    const int k = BK * c + 8 * ch;
    *reinterpret_cast<uint4*>(sX + buf * BM * BK + gemm_off(r, ch)) = keep_first_sel(xv, row0 + r < n ? K - k : 0);
    *reinterpret_cast<uint4*>(sW + buf * 256 * BK + gemm_off(r, ch)) = wv;
  };
  auto store = [&](int buf, int c) {
    store1(buf, c, 0, xr0, wr0);
    store1(buf, c, 1, xr1, wr1);
    store1(buf, c, 2, xr2, wr2);
    store1(buf, c, 3, xr3, wr3);
  };
  f32x16 acc[2][4];                         // from the bias, as lin_fwd
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    f32x16 b0 = {};
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int c = 128 * ng + 32 * t + 8 * (q >> 2) + 4 * h + (q & 3);
      b0[q] = (bias && c < N) ? bias[c] : 0.f;
    }
    acc[0][t] = b0;
    acc[1][t] = b0;
  }
  load(0);
  store(0, 0);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const int buf = c & 1;
    load(min(c + 1, nch - 1));         // unconditional (past the end: a re-load, never stored)
    // keep the loads here, ahead of the chunk's MFMAs (the compiler sank them to their
    // LDS stores, which left nothing to overlap their latency)
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const uint16_t* bx = sX + buf * BM * BK;
    const uint16_t* bw = sW + buf * 256 * BK;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      uint4 xb[2], wa[4];
#pragma unroll
      for (int u = 0; u < 2; ++u)
        xb[u] = *reinterpret_cast<const uint4*>(bx + gemm_off(64 * rg + 32 * u + lr, 2 * s + h));
#pragma unroll
      for (int t = 0; t < 4; ++t)
        wa[t] = *reinterpret_cast<const uint4*>(bw + gemm_off(128 * ng + 32 * t + lr, 2 * s + h));
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[u][t] = mma16<ET>(wa[t], xb[u], acc[u][t]);
    }
    // the other buffer: its last reader finished at the last barrier.  Unconditional (past
    // the end: the re-loaded last chunk, never read) -- under an `if` the compiler sank the
    // loads into it, behind the MFMAs
    store(buf ^ 1, min(c + 1, nch - 1));
    __syncthreads();
  }
  // epilogue: lane = row, registers 4g..4g+3 = columns 128 ng + 32 t + 8 g + 4 h + 0..3
  const uint32_t floor16 = relu ? 0u : 0x80008000u;
  // packed 16-bit values staged through the (now free) LDS as the wave's 64-row x
  // 128-column block, then stored as whole 256-B row pieces (16 lanes per row): a store
  // instruction of the transposed layout writes 32 rows x 16 B, every piece its own
  // fabric request
  uint8_t* so = reinterpret_cast<uint8_t*>(lds) + wv * GEMM_OST_BYTES;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int row = row0 + 64 * rg + 32 * u + lr;
    const float rs = (rscale && row < n) ? rscale[row] : 1.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint32_t pk[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const f2 z = f2{acc[u][t][4 * g + 2 * e], acc[u][t][4 * g + 2 * e + 1]} * rs;
          pk[e] = pk_max_i16(ET == 1 ? cvt_pk_h(z.x, z.y) : cvt_pk(z.x, z.y), floor16);
        }
        *reinterpret_cast<uint2*>(so + (32 * u + lr) * GEMM_OST_PITCH + 2 * (32 * t + 8 * g + 4 * h)) =
            make_uint2(pk[0], pk[1]);
      }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 4
  for (int it = 0; it < 16; ++it) {
    const int r = 4 * it + (lane >> 4), ch = lane & 15;
    const int row = row0 + 64 * rg + r, col = 128 * ng + 8 * ch;
    const uint4 v = *reinterpret_cast<const uint4*>(so + r * GEMM_OST_PITCH + 16 * ch);
    if (row < n && col < ldy) *reinterpret_cast<uint4*>(Y + (size_t)row * ldy + col) = v;
  }
}

// W^T image of the K-chunked kernel: img[c][k] = W[k][c], row stride KPc, zero outside
template <int ET>
__global__ __launch_bounds__(256) void lin_prep_kc_kernel(const float* __restrict__ W, int K, int N, int KPc,
                                                          long total, uint16_t* __restrict__ img) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int k = (int)(i % KPc), c = (int)(i / KPc);
  img[i] = e16_bits<ET>(k < K && c < N ? W[(size_t)k * N + c] : 0.f);
}

// ============================================================================
// lin_bwd_data: dX^T[k][row] = sum_c W[k][c] (dY * m)[row][c] for the k slab
// [blockIdx.y * kcols, +kcols); KN k-steps of 16 cover the N gradient columns.
// Output k < K1 -> dX1, K1 <= k < K1 + K2 -> dX2; times rscale[row] (optional).
// The mask [Ym > 0] is two packed instructions per pair of gradient values
// (v_pk_max_i16 / v_pk_min_u16 -> 0 / 1, then v_pk_mul_lo_u16); mscale = 1/(1-p) rides on
// the fp32 row scale of the epilogue.  The next tile's raw dY / Ym rows load while this
// tile computes and are masked after it (KN <= 16 on 8-wave blocks: the registers fit).
// ============================================================================
template <int KN, int FWD_WAVES = FwdWaves<KN>::value>
__global__ __launch_bounds__(FWD_WAVES * 64) void lin_bwd_data_kernel(
    const uint16_t* __restrict__ dY, int lddy, const uint16_t* __restrict__ Ym, int ldym, float mscale, int N,
    const float* __restrict__ W, int K1, int K2, uint16_t* __restrict__ dX1, int ldx1, uint16_t* __restrict__ dX2,
    int ldx2, const float* __restrict__ rscale, int n, int kcols, int dx1_f32, const uint16_t* __restrict__ wimg,
    int ost) {
  // dx1_f32: dX1 is fp32 (e.g. the init partial of a following SpMM) instead of bf16;
  // ost >= 0 (bf16 outputs only): the per-wave output staging tiles in LDS (out_stage);
  // wimg: bf16 LDS image of every k slab ([slabs][kcols][WS], lin_prep_bwd_kernel)
  constexpr int NP = KN * 16;
  constexpr int WS = NP + 8;
  constexpr bool PF = KN <= 16 && FWD_WAVES <= 8;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* sW = lds;                            // [kcols][WS]: rows of W
  const int kb = blockIdx.y * kcols;
  const int lane = threadIdx.x & 63, h = lane >> 5, lr = lane & 31;
  const int n_waves = gridDim.x * FWD_WAVES;
  const int n_tiles = (n + TILE - 1) / TILE;
  const int nt = kcols / 32;

  // raw 16-byte chunks of the tile's gradient / stored-output rows (clamped row: every
  // lane loads from a valid address; a chunk past N re-reads the row's first chunk against
  // zero weight columns of the image)
  auto load = [&](int tile, uint4 (&gr)[KN], uint4 (&yr)[KN]) {
    const int row = min(tile * TILE + lr, n - 1);
    int fh = 8 * h;
    asm volatile("" : "+v"(fh));
#pragma unroll
    for (int s = 0; s < KN; ++s) {
      const int c = 16 * s + fh;
      const int cc = c < N ? c : 0;
      gr[s] = *reinterpret_cast<const uint4*>(dY + (size_t)row * lddy + cc);
      if (Ym) yr[s] = *reinterpret_cast<const uint4*>(Ym + (size_t)row * ldym + cc);
    }
  };
  // N % 8 == 0: no chunk straddles N (rows past n are never stored: no masking either)
  // chunk s* = (N & ~7) / 16 is the only one that straddles N (in the lanes of half
  // h* = (N / 8) & 1; in the other half it lies wholly past N and is zeroed as well)
  const bool ragged = N & 7;
  const int sstar = (N & ~7) / 16;
  // dY * [Ym > 0] (and zero past N when a chunk straddles it)
  auto mask1 = [&](int s, uint4 g, uint4 y, bool rag) {
    if (rag && s == sstar) g = keep_first_sel(g, N - (16 * s + 8 * h));
    if (Ym)
      g = make_uint4(pk_mul16(g.x, pk_nz(pk_relu(y.x))), pk_mul16(g.y, pk_nz(pk_relu(y.y))),
                     pk_mul16(g.z, pk_nz(pk_relu(y.z))), pk_mul16(g.w, pk_nz(pk_relu(y.w))));
    return as_bf16x8(g);
  };
  auto mask = [&](const uint4 (&gr)[KN], const uint4 (&yr)[KN], bf16x8 (&by)[KN]) {
#pragma unroll
    for (int s = 0; s < KN; ++s) by[s] = mask1(s, gr[s], yr[s], false);
  };
  // the non-prefetching form: each chunk masked as it arrives (no second register set)
  auto load_masked = [&](int tile, bf16x8 (&by)[KN]) {
    const int row = min(tile * TILE + lr, n - 1);
    int fh = 8 * h;
    asm volatile("" : "+v"(fh));
#pragma unroll
    for (int s = 0; s < KN; ++s) {
      const int c = 16 * s + fh;
      const int cc = c < N ? c : 0;
      const uint4 g = *reinterpret_cast<const uint4*>(dY + (size_t)row * lddy + cc);
      uint4 y = make_uint4(0u, 0u, 0u, 0u);
      if (Ym) y = *reinterpret_cast<const uint4*>(Ym + (size_t)row * ldym + cc);
      by[s] = mask1(s, g, y, ragged);
    }
  };
  auto process = [&](int tile, const bf16x8 (&by)[KN]) {
    const int row = tile * TILE + lr;
    const bool rv = row < n;
    const float rs = ((rv && rscale) ? rscale[row] : 1.f) * mscale;
#pragma unroll 1
    for (int t = 0; t < nt; ++t) {
      f32x16 acc = {};
      const uint16_t* arow = sW + (32 * t + lr) * WS + 8 * h;
#pragma unroll
      for (int s = 0; s < KN; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(*reinterpret_cast<const uint4*>(arow + 16 * s)),
                                                      by[s], acc, 0, 0, 0);
      if (ost >= 0) {
        uint32_t pk[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const f2 z = f2{acc[2 * i], acc[2 * i + 1]} * rs;
          pk[i] = cvt_pk(z.x, z.y);
        }
        const int kt = kb + 32 * t;
        out_stage(lds, ost, pk, tile, n, [&](int r, int c, uint4 v) {
          const int k = kt + c;                              // 8 consecutive k, never straddling K1
          if (k < K1) {
            if (k < ldx1) *reinterpret_cast<uint4*>(dX1 + (size_t)r * ldx1 + k) = v;
          } else if (dX2 && k - K1 < ldx2 && k < K1 + ldx2) {
            *reinterpret_cast<uint4*>(dX2 + (size_t)r * ldx2 + (k - K1)) = v;
          }
        });
        continue;
      }
      if (!rv) continue;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int k = kb + 32 * t + 8 * g + 4 * h;          // 4 consecutive k, never straddling K1 (K1 % 8 == 0)
        const f2 lo = f2{acc[4 * g], acc[4 * g + 1]} * rs, hi = f2{acc[4 * g + 2], acc[4 * g + 3]} * rs;
        if (k < K1) {
          if (k < ldx1) {
            if (dx1_f32)
              *reinterpret_cast<float4*>(reinterpret_cast<float*>(dX1) + (size_t)row * ldx1 + k) =
                  make_float4(lo.x, lo.y, hi.x, hi.y);
            else
              st_y8(dX1 + (size_t)row * ldx1 + k, cvt_pk(lo.x, lo.y), cvt_pk(hi.x, hi.y));
          }
        } else if (dX2 && k - K1 < ldx2 && k < K1 + ldx2) {
          st_y8(dX2 + (size_t)row * ldx2 + (k - K1), cvt_pk(lo.x, lo.y), cvt_pk(hi.x, hi.y));
        }
      }
    }
  };

  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int tile = blockIdx.x * FWD_WAVES + wv;
  auto stage = [&]() {
    const uint4* src = reinterpret_cast<const uint4*>(wimg + (size_t)blockIdx.y * kcols * WS);
    uint4* dst = reinterpret_cast<uint4*>(sW);
    copy_image(dst, src, kcols * WS / 8);
    __syncthreads();
  };
  bf16x8 by[KN];
  if (PF && !ragged) {
    uint4 gr[KN], yr[KN];
    if (tile < n_tiles) load(tile, gr, yr);      // in flight while the weights are staged
    stage();
    if (tile < n_tiles) mask(gr, yr, by);
    for (; tile < n_tiles; tile += n_waves) {
      const bool more = tile + n_waves < n_tiles;
      if (more) load(tile + n_waves, gr, yr);
      process(tile, by);
      if (more) mask(gr, yr, by);
    }
  } else {
    stage();
    for (; tile < n_tiles; tile += n_waves) {
      load_masked(tile, by);
      process(tile, by);
    }
  }
}

// ============================================================================
// lin_bwd_weight: gpart[chunk][k][c] = sum_{rows of chunk} [X1 | X2][row][k] (dY * m)[row][c]
// for the 64-column slab c in [blockIdx.y * 64, +64), and gpart[chunk][K1 + K2][c] =
// sum_rows (dY * m)[row][c] (the bias gradient, accumulated on the VALU by the threads
// that stage the gradient tile, so K = 256 is exactly 8 balanced k-tiles).  KT = k-tiles
// of 32 covering K1 + K2; wave w owns the k-tiles w, w + 8, ...
// ============================================================================
template <int KT>
__global__ __launch_bounds__(WGT_WAVES * 64) void lin_bwd_weight_kernel(
    const uint16_t* __restrict__ x1, int ld1, int K1, const uint16_t* __restrict__ x2, int ld2, int K2,
    const uint16_t* __restrict__ dY, int lddy, const uint16_t* __restrict__ Ym, int ldym, float mscale, int N,
    float* __restrict__ gpart, int n, int rows_per_chunk, const int* __restrict__ idx1) {
  constexpr int NT = WGT_WAVES * 64;
  constexpr int KROWS = KT * 32;
  constexpr int KPW = (KT + WGT_WAVES - 1) / WGT_WAVES;     // k-tiles per wave
  constexpr int XCH = KROWS / 8;                            // 16-byte chunks per staged X row
  constexpr int PFX = (TILE * XCH + NT - 1) / NT;
  constexpr int PFY = (TILE * 8 + NT - 1) / NT;             // 64 gradient columns = 8 chunks
  __shared__ __attribute__((aligned(16))) uint16_t sXt[KROWS * TR];
  __shared__ __attribute__((aligned(16))) uint16_t sDt[64 * TR];
  __shared__ float sdb[64 * 33];
  const int tid = threadIdx.x;
  const int K = K1 + K2;
  const int c0 = blockIdx.y * 64;
  const int r_begin = blockIdx.x * rows_per_chunk, r_end = min(n, r_begin + rows_per_chunk);
  const int lane = tid & 63, h = lane >> 5, lr = lane & 31, wv = tid >> 6;
  const int xch = (K + 7) / 8;                              // chunks that carry features

  f32x16 acc[KPW][2];
#pragma unroll
  for (int a = 0; a < KPW; ++a) { acc[a][0] = f32x16{}; acc[a][1] = f32x16{}; }
  float dsum[PFY][8];                                       // bias-gradient partials (staging threads)
#pragma unroll
  for (int q = 0; q < PFY; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) dsum[q][e] = 0.f;

  uint4 px[PFX], py[PFY];
  auto prefetch = [&](int r0) {
#pragma unroll
    for (int q = 0; q < PFX; ++q) {
      const int i = tid + q * NT;
      const int rr = i % TILE, ch = i / TILE;
      px[q] = (ch < xch && r0 + rr < r_end) ? load_cat8(x1, ld1, K1, x2, ld2, K2, r0 + rr, 8 * ch, idx1)
                                            : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int q = 0; q < PFY; ++q) {
      const int i = tid + q * NT;
      const int rr = i % TILE, ch = i / TILE;
      py[q] = (i < TILE * 8 && r0 + rr < r_end) ? load_masked8(dY, lddy, Ym, ldym, mscale, N, r0 + rr, c0 + 8 * ch)
                                                : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  if (r_begin < r_end) prefetch(r_begin);
  for (int r0 = r_begin; r0 < r_end; r0 += TILE) {
    __syncthreads();                                       // previous tile's images consumed
#pragma unroll
    for (int q = 0; q < PFX; ++q) {
      const int i = tid + q * NT;
      const int rr = i % TILE, ch = i / TILE;
      if (ch < XCH) {
        const uint32_t w[4] = {px[q].x, px[q].y, px[q].z, px[q].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) sXt[(8 * ch + e) * TR + rr] = (uint16_t)(w[e >> 1] >> (16 * (e & 1)));
      }
    }
#pragma unroll
    for (int q = 0; q < PFY; ++q) {
      const int i = tid + q * NT;
      const int rr = i % TILE, ch = i / TILE;
      if (i < TILE * 8) {
        const uint32_t w[4] = {py[q].x, py[q].y, py[q].z, py[q].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t b16 = (w[e >> 1] >> (16 * (e & 1))) & 0xffffu;
          sDt[(8 * ch + e) * TR + rr] = (uint16_t)b16;
          dsum[q][e] += bf16_val(b16);
        }
      }
    }
    if (r0 + TILE < r_end) prefetch(r0 + TILE);
    __syncthreads();
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 b0 = as_bf16x8(*reinterpret_cast<const uint4*>(sDt + lr * TR + 16 * s2 + 8 * h));
      const bf16x8 b1 = as_bf16x8(*reinterpret_cast<const uint4*>(sDt + (32 + lr) * TR + 16 * s2 + 8 * h));
#pragma unroll
      for (int a = 0; a < KPW; ++a) {
        const int kt = wv + WGT_WAVES * a;
        if (kt < KT) {
          const bf16x8 ax = as_bf16x8(*reinterpret_cast<const uint4*>(sXt + (32 * kt + lr) * TR + 16 * s2 + 8 * h));
          acc[a][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ax, b0, acc[a][0], 0, 0, 0);
          acc[a][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ax, b1, acc[a][1], 0, 0, 0);
        }
      }
    }
  }
  // slab of this chunk: rows k in [0, K), columns c0 + [0, 64) (lane = column: coalesced)
  float* gp = gpart + (size_t)blockIdx.x * (K + 1) * N;
#pragma unroll
  for (int a = 0; a < KPW; ++a) {
    const int kt = wv + WGT_WAVES * a;
    if (kt >= KT) continue;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k = 32 * kt + (q & 3) + 8 * (q >> 2) + 4 * h;
      if (k >= K) continue;
      if (c0 + lr < N) gp[(size_t)k * N + c0 + lr] = acc[a][0][q];
      if (c0 + 32 + lr < N) gp[(size_t)k * N + c0 + 32 + lr] = acc[a][1][q];
    }
  }
  // bias-gradient row K: the staging threads' per-(row slot, column) partials, summed over
  // the 32 row slots in a fixed order
#pragma unroll
  for (int q = 0; q < PFY; ++q) {
    const int i = tid + q * NT;
    if (i < TILE * 8) {
      const int rr = i % TILE, ch = i / TILE;
#pragma unroll
      for (int e = 0; e < 8; ++e) sdb[(8 * ch + e) * 33 + rr] = dsum[q][e];
    }
  }
  __syncthreads();
  if (tid < 64 && c0 + tid < N) {
    float t = 0.f;
    for (int r = 0; r < TILE; ++r) t += sdb[tid * 33 + r];
    gp[(size_t)K * N + c0 + tid] = t;
  }
}

// ============================================================================
// lin_bwd_weight2: the same gpart slab as lin_bwd_weight, re-laid for bandwidth.
//  * one block covers NB column tiles of 32 (all 256 hidden columns when K <= 256), so
//    X is read from HBM once per chunk instead of once per 64-column slab;
//  * both tiles are staged ROW-major with b128 writes, lanes running along a row (the
//    global loads coalesce along rows too), and both MFMA operands of the row
//    contraction come out of ds_read_b64_tr_b16 -- no 2-byte transposing writes;
//  * double-buffered images, one barrier per 32-row tile, the loads of tile t + 2 in
//    flight under tile t's MFMAs.
// Row pitch of a [32][64 * tiles B] image: a 32-lane half reads 4 consecutive rows x
// 64 B, conflict-free when the pitch is = 64 or 192 (mod 256) bytes.
// Wave map: KW = min(KT, 8) waves per column group, WPK = 8 / KW column groups; wave w
// holds k-tiles (w % KW) + KW a and column tiles (w / KW) + WPK j.
// ============================================================================
constexpr int wgt2_pitch(int tiles) { return 64 * tiles + ((tiles & 1) ? 0 : 64); }

template <int KT, int NB>
struct Wgt2 {
  static constexpr int KW = KT < 8 ? KT : 8;
  static constexpr int WPK = 8 / KW;
  static constexpr int KPW = (KT + KW - 1) / KW;
  static constexpr int CPW = (NB + WPK - 1) / WPK;
  static constexpr int PX = wgt2_pitch(KT), PY = wgt2_pitch(NB);
  static constexpr int XCH = KT * 4, YCH = NB * 4;           // 16-B chunks per staged row
  static constexpr int BUF = TILE * (PX + PY);
  static constexpr int LDS = 2 * BUF;
  static_assert(KPW * CPW <= 8, "accumulators per wave");
};

template <int KT, int NB, bool HAS_YM>
__global__ __launch_bounds__(512, 1) void lin_bwd_weight2_kernel(
    const uint16_t* __restrict__ x1, int ld1, int K1, const uint16_t* __restrict__ x2, int ld2, int K2,
    const uint16_t* __restrict__ dY, int lddy, const uint16_t* __restrict__ Ym, int ldym, float mscale, int N,
    float* __restrict__ gpart, int n, int rows_per_chunk, const int* __restrict__ idx1) {
  using C = Wgt2<KT, NB>;
  constexpr int NT = 512;
  constexpr int PFX = (TILE * C::XCH + NT - 1) / NT;
  constexpr int PFY = (TILE * C::YCH + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) uint8_t wlds[];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, lr = lane & 31, wv = tid >> 6;
  const int K = K1 + K2, xch = (K + 7) / 8;
  const int c0 = blockIdx.y * NB * 32;
  const int r_begin = blockIdx.x * rows_per_chunk, r_end = min(n, r_begin + rows_per_chunk);
  const int ntile = r_begin < r_end ? (r_end - r_begin + TILE - 1) / TILE : 0;
  const bool active = wv < C::KW * C::WPK;
  const int kw = wv % C::KW, cg = wv / C::KW;
  // gathered X1 rows (idx1): the chunk's row ids are staged in LDS once, so a prefetch
  // reads its row id from LDS instead of a dependent global load inside the ring
  int* sidx = reinterpret_cast<int*>(wlds + C::LDS);
  if (idx1) {
    for (int r = r_begin + tid; r < r_end; r += NT) sidx[r - r_begin] = idx1[r];
    __syncthreads();
  }

  f32x16 acc[C::KPW][C::CPW];
#pragma unroll
  for (int a = 0; a < C::KPW; ++a)
#pragma unroll
    for (int j = 0; j < C::CPW; ++j) acc[a][j] = f32x16{};
  float dsum[PFY][8];
#pragma unroll
  for (int q = 0; q < PFY; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) dsum[q][e] = 0.f;

  // Loads are UNCONDITIONAL (addresses clamped to the chunk's last row / the slab's first
  // column / the row's first chunk) and nothing computes on a loaded value until the
  // tile is staged, where the validity select, the mask and the scale are applied: a
  // conditional load merged with a zero (or a mask on the loaded value) would make the
  // compiler wait for the load right there (vmcnt(0)), draining the other set too.
  // Two register sets: tile j is loaded into set j & 1 and staged into LDS buffer j & 1,
  // two tiles ahead of the MFMAs.
  const bool scaled = HAS_YM || mscale != 1.f;
  uint4 px[2][PFX], py[2][PFY], pm[2][HAS_YM ? PFY : 1];
  auto prefetch = [&](auto S, int r0) {
    constexpr int st = decltype(S)::value;
#pragma unroll
    for (int q = 0; q < PFX; ++q) {
      const int i = min(tid + q * NT, TILE * C::XCH - 1);
      const int row = min(r0 + i / C::XCH, r_end - 1), f0 = 8 * (i % C::XCH);
      const size_t r1 = idx1 ? (size_t)sidx[row - r_begin] : (size_t)row;
      const uint16_t* p = f0 < K1 ? x1 + r1 * ld1 + f0
                        : (x2 && f0 - K1 < K2) ? x2 + (size_t)row * ld2 + (f0 - K1) : x1 + r1 * ld1;
      px[st][q] = *reinterpret_cast<const uint4*>(p);
    }
#pragma unroll
    for (int q = 0; q < PFY; ++q) {
      const int i = min(tid + q * NT, TILE * C::YCH - 1);
      const int row = min(r0 + i / C::YCH, r_end - 1);
      const int c = c0 + 8 * (i % C::YCH), cc = c < N ? c : c0;
      py[st][q] = *reinterpret_cast<const uint4*>(dY + (size_t)row * lddy + cc);
      if constexpr (HAS_YM) pm[st][q] = *reinterpret_cast<const uint4*>(Ym + (size_t)row * ldym + cc);
    }
  };
  auto stage = [&](auto S, int r0) {
    constexpr int st = decltype(S)::value;
    uint8_t* bx = wlds + st * C::BUF;
    uint8_t* by = bx + TILE * C::PX;
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int q = 0; q < PFX; ++q) {
      const int i = tid + q * NT;
      if (i < TILE * C::XCH) {
        const bool ok = r0 + i / C::XCH < r_end && i % C::XCH < xch;
        uint4 v = px[st][q];
        if (!ok) v = z;
        *reinterpret_cast<uint4*>(bx + (i / C::XCH) * C::PX + 16 * (i % C::XCH)) = v;
      }
    }
#pragma unroll
    for (int q = 0; q < PFY; ++q) {
      const int i = tid + q * NT;
      if (i < TILE * C::YCH) {
        const bool ok = r0 + i / C::YCH < r_end && c0 + 8 * (i % C::YCH) < N;
        uint4 v = py[st][q];
        if constexpr (HAS_YM) {
          v = mask8(v, pm[st][q], true, mscale);
        } else {
          if (scaled) v = mask8(v, z, false, mscale);
        }
        if (!ok) v = z;
        *reinterpret_cast<uint4*>(by + (i / C::YCH) * C::PY + 16 * (i % C::YCH)) = v;
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) dsum[q][e] += bf16_val((w[e >> 1] >> (16 * (e & 1))) & 0xffffu);
      }
    }
  };
  const int qq = (lane & 15) >> 2, pq = lane & 3, gb = (lane >> 4) & 1;
  auto compute = [&](int buf) {
    if (!active) return;
    const uint8_t* bx = wlds + buf * C::BUF;
    const uint8_t* by = bx + TILE * C::PX;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int ra = 16 * s2 + 8 * h + qq;                 // k slot j <-> tile row 16 s2 + 8 h + j
      const int colb = 2 * (16 * gb + 4 * pq);
      bf16x8 bf[C::CPW];
#pragma unroll
      for (int j = 0; j < C::CPW; ++j) {
        const int ct = cg + C::WPK * j;
        if (ct < NB) bf[j] = tr_frag(by, ra * C::PY + 64 * ct + colb, (ra + 4) * C::PY + 64 * ct + colb);
      }
#pragma unroll
      for (int a = 0; a < C::KPW; ++a) {
        const int kt = kw + C::KW * a;
        if (kt >= KT) continue;
        const bf16x8 ax = tr_frag(bx, ra * C::PX + 64 * kt + colb, (ra + 4) * C::PX + 64 * kt + colb);
#pragma unroll
        for (int j = 0; j < C::CPW; ++j)
          if (cg + C::WPK * j < NB) acc[a][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ax, bf[j], acc[a][j], 0, 0, 0);
      }
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  if (ntile > 0) prefetch(I0{}, r_begin);
  if (ntile > 1) prefetch(I1{}, r_begin + TILE);
  if (ntile > 0) stage(I0{}, r_begin);
  if (ntile > 2) prefetch(I0{}, r_begin + 2 * TILE);
  __syncthreads();
  for (int t = 0; t < ntile; t += 2) {
    // tile t in buffer 0; tile t + 1 (set 1) staged into buffer 1, tile t + 3 loaded into set 1
    if (t + 1 < ntile) {
      stage(I1{}, r_begin + (t + 1) * TILE);
      if (t + 3 < ntile) prefetch(I1{}, r_begin + (t + 3) * TILE);
    }
    compute(0);
    __syncthreads();
    if (t + 1 >= ntile) break;
    // tile t + 1 in buffer 1; tile t + 2 (set 0) staged into buffer 0, tile t + 4 into set 0
    if (t + 2 < ntile) {
      stage(I0{}, r_begin + (t + 2) * TILE);
      if (t + 4 < ntile) prefetch(I0{}, r_begin + (t + 4) * TILE);
    }
    compute(1);
    __syncthreads();
  }

  float* gp = gpart + (size_t)blockIdx.x * (K + 1) * N;
  if (active) {
#pragma unroll
    for (int a = 0; a < C::KPW; ++a) {
      const int kt = kw + C::KW * a;
      if (kt >= KT) continue;
#pragma unroll
      for (int j = 0; j < C::CPW; ++j) {
        const int c = c0 + 32 * (cg + C::WPK * j) + lr;
        if (cg + C::WPK * j >= NB || c >= N) continue;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int k = 32 * kt + (q & 3) + 8 * (q >> 2) + 4 * h;
          if (k < K) gp[(size_t)k * N + c] = acc[a][j][q];
        }
      }
    }
  }
  // bias-gradient row K: per-(row slot, column) partials, summed over the slots in order
  float* sdb = reinterpret_cast<float*>(wlds);               // [NB * 32][33], images consumed
#pragma unroll
  for (int q = 0; q < PFY; ++q) {
    const int i = tid + q * NT;
    if (i < TILE * C::YCH) {
      const int rr = i / C::YCH, ch = i % C::YCH;
#pragma unroll
      for (int e = 0; e < 8; ++e) sdb[(8 * ch + e) * 33 + rr] = dsum[q][e];
    }
  }
  __syncthreads();
  if (tid < NB * 32 && c0 + tid < N) {
    float s = 0.f;
    for (int r = 0; r < TILE; ++r) s += sdb[tid * 33 + r];
    gp[(size_t)K * N + c0 + tid] = s;
  }
}

// out[i] = sum_{c < chunks} gpart[c][i] (fixed order), i < count; the first k_rows * N
// go to dW, the last N (the ones row) to db when db != nullptr.  32 consecutive
// outputs per block, the chunks split over 8 lane groups (8 independent load streams
// per output instead of one serial chain), then a fixed-order sum of the 8 partials.
__global__ __launch_bounds__(256) void lin_reduce_kernel(const float* __restrict__ gpart, int chunks, long count,
                                                         int N, float* __restrict__ dW, float* __restrict__ db) {
  __shared__ float s[8][33];
  const int e = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const long i = (long)blockIdx.x * 32 + e;
  float acc = 0.f;
  if (i < count)
    for (int c = grp; c < chunks; c += 8) acc += gpart[(size_t)c * count + i];
  s[grp][e] = acc;
  __syncthreads();
  if (grp == 0 && i < count) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) t += s[q][e];
    const long kw = count - N;
    if (i < kw) dW[i] = t;
    else if (db) db[i - kw] = t;
  }
}

// The same sums (same order per output: chunks grp, grp + 8, ... of lane group grp, then
// the 8 group partials -- bitwise equal to lin_reduce_kernel) with 16-byte loads: lane e
// of a group owns outputs 4e..4e+3 of the block's 128, and each lane issues its group's
// chunk loads 4 at a time ahead of the adds.  count % 4 == 0 (16-B aligned chunk rows).
__global__ __launch_bounds__(256) void lin_reduce4_kernel(const float* __restrict__ gpart, int chunks, long count,
                                                          int N, float* __restrict__ dW, float* __restrict__ db) {
  __shared__ float4 s[8][33];
  const int e = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const long i = ((long)blockIdx.x * 32 + e) * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < count) {
    const float4* g = reinterpret_cast<const float4*>(gpart + i);
    const long cs = count >> 2;                          // chunk stride in float4
    int c = grp;
    for (; c + 24 < chunks; c += 32) {
      const float4 v0 = g[(size_t)c * cs], v1 = g[(size_t)(c + 8) * cs];
      const float4 v2 = g[(size_t)(c + 16) * cs], v3 = g[(size_t)(c + 24) * cs];
      acc.x += v0.x; acc.y += v0.y; acc.z += v0.z; acc.w += v0.w;
      acc.x += v1.x; acc.y += v1.y; acc.z += v1.z; acc.w += v1.w;
      acc.x += v2.x; acc.y += v2.y; acc.z += v2.z; acc.w += v2.w;
      acc.x += v3.x; acc.y += v3.y; acc.z += v3.z; acc.w += v3.w;
    }
    for (; c < chunks; c += 8) {
      const float4 v = g[(size_t)c * cs];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  s[grp][e] = acc;
  __syncthreads();
  if (grp == 0 && i < count) {
    float t[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 v = s[q][e];
      t[0] += v.x; t[1] += v.y; t[2] += v.z; t[3] += v.w;
    }
    const long kw = count - N;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (i + u < kw) dW[i + u] = t[u];
      else if (db) db[i + u - kw] = t[u];
    }
  }
}

// bf16 LDS images of the weights, written once per step (the blocks of the main
// kernels then copy them with 16-byte loads):
//   fwd: img[slab][c][k]  = W[k][slab * ncols + c]   (W^T, row stride WS = KP + 8)
//   bwd: img[slab][kk][c] = W[slab * kcols + kk][c]  (W rows, row stride WS = NP + 8)
// zero outside the matrix and in the pad columns
template <int ET>
__global__ __launch_bounds__(256) void lin_prep_fwd_kernel(const float* __restrict__ W, int K, int N, int ncols,
                                                           int KP, int WS, long total, float scale,
                                                           uint16_t* __restrict__ img) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int k = (int)(i % WS);
  const long rc = i / WS;                       // slab * ncols + c = global column
  const int c = (int)rc;
  img[i] = e16_bits<ET>(k < K && k < KP && c < N ? W[(size_t)k * N + c] * scale : 0.f);
}

__global__ __launch_bounds__(256) void lin_prep_bwd_kernel(const float* __restrict__ W, int K, int N, int NP, int WS,
                                                           long total, uint16_t* __restrict__ img) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % WS);
  const int k = (int)(i / WS);                  // slab * kcols + kk = global row of W
  img[i] = bf16_bits(k < K && c < N && c < NP ? W[(size_t)k * N + c] : 0.f);
}

// ============================================================================
// lin_ws: the weight-stationary form of lin_fwd (BWD = false) and lin_bwd_data (BWD =
// true) for a reduction of KP = 16 KS <= 256 and at most 256 output columns.  Block =
// NW waves; wave w owns output columns [32 w, 32 w + 32) and keeps their weight slab
// in registers (A operand, KS x 16 B per lane, read once from the image).  The block
// streams 32-row tiles of the streamed operand (X, or dY masked by [Ym > 0]) in whole
// rows: each wave loads 1/NW of a tile into a ring of R = 3 register tiles (so two tiles
// stay in flight while one is consumed), writes it to one of two XOR-swizzled LDS slots
// (chunk c of row r at c ^ (r & 15): the b128 fragment reads of 16 consecutive rows hit
// 16 distinct bank groups), and every wave reads its B fragments from the slot.  Output
// tiles are staged in LDS (double-buffered) and stored as whole rows, 16 B per lane.
// One block barrier per tile.  The slab kernels above keep the rest: fp32 tails, K
// straddling chunks, fp32 dX1, wider layers.
// ============================================================================
constexpr int WS_IDX_TILES = 64;     // tiles per block whose row ids / row scales fit their LDS stage

template <int KS, int ET, int NW, bool BWD>
__global__ __launch_bounds__(NW * 64) void lin_ws_kernel(
    const uint16_t* __restrict__ a1, int lda1, int K1, const uint16_t* __restrict__ a2, int lda2, int K2,
    const int* __restrict__ idx1, const uint16_t* __restrict__ Ym, int ldym,
    const float* __restrict__ W, int WK, int WN, const uint16_t* __restrict__ wimg, const float* __restrict__ bias,
    int N, float scale,
    uint16_t* __restrict__ Y1, int ldy1, int KO1, uint16_t* __restrict__ Y2, int ldy2,
    int n, int relu, uint32_t k0, uint32_t k1, uint32_t step, uint32_t thr8, uint32_t row0,
    const int* __restrict__ stepp, const float* __restrict__ rscale, float mscale) {
  // fwd: A = [a1 | a2] (K1 + K2 = reduction, a1 rows gathered through idx1), Y1[row][c]
  //      for c < ldy1 (N = output columns with weights, c >= N written 0);
  // bwd: A = a1 = dY (K1 = its N columns) masked by Ym, outputs c < KO1 -> Y1, else Y2.
  constexpr int KP = KS * 16, CH = KP / 8;               // 16-B chunks per tile row
  constexpr int SW = CH < 16 ? CH - 1 : 15;               // chunk swizzle mask
  constexpr int RB = KP * 2;                              // slot row bytes
  constexpr int SLOT = 32 * RB;
  constexpr int LPW = (4 * KP + 64 * NW - 1) / (64 * NW); // 16-B loads per lane per tile (ring entry)
  static_assert(LPW <= 2, "ring entries of at most two loads per lane");
  constexpr int OP = NW * 64 + 16;                        // out-staging row pitch (bytes)
  constexpr int OSZ = 32 * OP;
  constexpr int OPW = 32 * NW * 4 / (64 * NW);            // 16-B output chunks per lane per tile (2)
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* sX = smem;                                     // [2][SLOT]
  uint8_t* sO = smem + 2 * SLOT;                          // [2][OSZ]
  u32x4* sD = reinterpret_cast<u32x4*>(smem + 2 * SLOT + 2 * OSZ);   // [2][64] bit-mode draws
  int* sIdx = reinterpret_cast<int*>(smem + 2 * SLOT + 2 * OSZ + (BWD ? 0 : 2 * 64 * 16));   // [nt][32] gathered ids
  float* sRs = reinterpret_cast<float*>(sIdx + (BWD ? 0 : WS_IDX_TILES * TILE));             // [nt][32] row scales
  if (stepp) step = (uint32_t)*stepp;
  const int lane = threadIdx.x & 63, h = lane >> 5, lr = lane & 31;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n_tiles = (n + TILE - 1) / TILE;
  const int G = gridDim.x;
  const bool bit = drop_bit_mode(thr8);
  const uint32_t floor16 = relu ? 0u : 0x80008000u;

  const int nt = n_tiles > (int)blockIdx.x ? (n_tiles - 1 - (int)blockIdx.x) / G + 1 : 0;
  auto T = [&](int i) { return (int)blockIdx.x + i * G; };
  // gathered row ids and row scales of the block's tiles, staged once (a global load inside
  // the loop whose value is used at once would wait for every older ring load)
  if ((!BWD && idx1) || rscale) {
    for (int e = threadIdx.x; e < nt * TILE; e += NW * 64) {
      const int row = min(T(e / TILE) * TILE + e % TILE, n - 1);
      if (!BWD && idx1) sIdx[e] = idx1[row];
      if (rscale) sRs[e] = rscale[row];
    }
    __syncthreads();
  }
  // ring loads past the block's last tile re-read that tile (an L2 hit; no branch around the
  // loads: a conditional load into a ring register costs a copy and with it a vmcnt(0))
  auto TL = [&](int i) { return T(min(i, nt - 1)); };
  // stationary weights.  fwd: straight from the fp32 master W [WK][WN] (no image kernel):
  // A[c][k] = W[k][c] * scale (c = 32 wv + lr, k = 16 s + 8 h + j; a column of W, coalesced
  // across the lanes), zero outside W.  bwd: A[k][c] = W[k][c] from the bf16 image
  uint4 wa[KS];
  {
    const int wr = 32 * wv + lr;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      float v[8];
      if constexpr (BWD) {
        // the bf16 image of W's rows (lin_prep_bwd_kernel, row stride KP + 8): read from the
        // fp32 master instead (two float4 per k-step and lane) the kernel measured 7 us slower
        wa[s] = *reinterpret_cast<const uint4*>(wimg + (size_t)wr * (KP + 8) + 16 * s + 8 * h);
        continue;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 16 * s + 8 * h + j;
          const float x = W[(size_t)min(k, WK - 1) * WN + min(wr, WN - 1)];
          v[j] = (k < WK && wr < WN) ? x * scale : 0.f;
        }
      }
      wa[s] = ET == 1 ? make_uint4(cvt_pk_h(v[0], v[1]), cvt_pk_h(v[2], v[3]), cvt_pk_h(v[4], v[5]), cvt_pk_h(v[6], v[7]))
                      : make_uint4(cvt_pk(v[0], v[1]), cvt_pk(v[2], v[3]), cvt_pk(v[4], v[5]), cvt_pk(v[6], v[7]));
    }
  }
  f32x16 bacc = {};
  if (!BWD && bias) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int c = 32 * wv + 8 * (q >> 2) + 4 * h + (q & 3);
      bacc[q] = c < N ? bias[c] * scale : 0.f;
    }
  }

  // this lane's share of a tile: chunk q = (wv * LPW + j) * 64 + lane -> row q / CH, chunk q % CH
  // (unconditional loads -- a1 in place of a missing mask: a conditional load into a ring
  // register costs a copy and with it a vmcnt(0), i.e. every older ring load)
  auto load = [&](int tile, uint4 (&gr)[LPW], uint4 (&yr)[LPW]) {
#pragma unroll
    for (int j = 0; j < LPW; ++j) {
      // (waves past the tile's chunks re-load one of them, unused: no branch around a load)
      const int q = ((wv * LPW + j) * 64 + lane) % (4 * KP);
      const int row = min(tile * TILE + q / CH, n - 1), c = q % CH, k = 8 * c;
      if constexpr (BWD) {
        const int kk = k < K1 ? k : 0;                    // past N: chunk 0 against zero weights
        gr[j] = *reinterpret_cast<const uint4*>(a1 + (size_t)row * lda1 + kk);
        yr[j] = *reinterpret_cast<const uint4*>(Ym ? Ym + (size_t)row * ldym + kk : a1 + (size_t)row * lda1 + kk);
      } else {
        // gathered rows: their ids were staged in LDS up front (a global id load here would
        // need a vmcnt(0) -- every older ring load -- before its address is known)
        const int r1 = idx1 ? sIdx[(tile - (int)blockIdx.x) / G * TILE + q / CH] : row;
        const uint16_t* p1 = a1 + (size_t)r1 * lda1;
        const uint16_t* p2 = a2 + (size_t)row * lda2;
        const int g = k - K1;
        const uint16_t* src = k < K1 ? p1 + k : p1;
        src = (k >= K1 && g < K2) ? p2 + g : src;
        gr[j] = *reinterpret_cast<const uint4*>(src);
      }
    }
  };
  auto put = [&](int slot, const uint4 (&gr)[LPW], const uint4 (&yr)[LPW]) {
#pragma unroll
    for (int j = 0; j < LPW; ++j) {
      const int q = (wv * LPW + j) * 64 + lane;
      if (4 * KP % (64 * NW) != 0 && q >= 4 * KP) break;
      const int r = q / CH, c = q % CH;
      uint4 v = gr[j];
      if (BWD && Ym) {
        const uint4 y = yr[j];
        v = make_uint4(pk_mul16(v.x, pk_nz(pk_relu(y.x))), pk_mul16(v.y, pk_nz(pk_relu(y.y))),
                       pk_mul16(v.z, pk_nz(pk_relu(y.z))), pk_mul16(v.w, pk_nz(pk_relu(y.w))));
      }
      *reinterpret_cast<uint4*>(sX + slot * SLOT + r * RB + 16 * (c ^ (r & SW))) = v;
    }
  };
  // products of tile `tile` (slot) -> packed 16-bit outputs in out-staging buffer ob
  auto compute = [&](int tile, int slot, int ob, int i) {
    f32x16 acc = bacc;
    const uint8_t* xr = sX + slot * SLOT + lr * RB;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const uint4 b = *reinterpret_cast<const uint4*>(xr + 16 * ((2 * s + h) ^ (lr & SW)));
      acc = mma16<ET>(wa[s], b, acc);
    }
    const int row = tile * TILE + lr;
    const bool rv = row < n;
    float rs = rscale ? sRs[i * TILE + lr] : 1.f;
    if (BWD) rs *= mscale;
    uint32_t pk[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f2 z = f2{acc[2 * i], acc[2 * i + 1]} * rs;
      pk[i] = ET == 1 ? cvt_pk_h(z.x, z.y) : cvt_pk(z.x, z.y);
      if (!BWD) pk[i] = pk_max_i16(pk[i], floor16);
    }
    if (!BWD && thr8 > 0) {
      u32x4 r;
      if (bit) {
        r = sD[(slot & 1) * 64 + lane];                   // one draw per (row, half) serves all 8 waves
      } else {
        uint32_t gr32 = row0 + (uint32_t)row;
        asm volatile("" : "+v"(gr32));
        r = drop_draw(gr32, wv, h, step, k0, k1, false);
      }
      const uint32_t mw = keep_spread(drop_keep16(r, wv, thr8, bit));
#pragma unroll
      for (int i = 0; i < 8; ++i) pk[i] = pk_mul16(pk[i], (mw >> (2 * i)) & 0x10001u);
    }
    uint8_t* o = sO + ob * OSZ + lr * OP + 64 * wv + 8 * h;
#pragma unroll
    for (int g = 0; g < 4; ++g) *reinterpret_cast<uint2*>(o + 16 * g) = make_uint2(pk[2 * g], pk[2 * g + 1]);
  };
  auto store = [&](int tile, int ob) {
#pragma unroll
    for (int j = 0; j < OPW; ++j) {
      const int q = (wv * OPW + j) * 64 + lane;
      const int r = q / (NW * 4), c = 8 * (q % (NW * 4));
      const int row = tile * TILE + r;
      const uint4 v = *reinterpret_cast<const uint4*>(sO + ob * OSZ + r * OP + 16 * (q % (NW * 4)));
      if (row >= n) continue;
      if (BWD) {
        if (c < KO1) {
          if (c < ldy1) *reinterpret_cast<uint4*>(Y1 + (size_t)row * ldy1 + c) = v;
        } else if (Y2 && c - KO1 < ldy2) {
          *reinterpret_cast<uint4*>(Y2 + (size_t)row * ldy2 + (c - KO1)) = v;
        }
      } else if (c < ldy1) {
        *reinterpret_cast<uint4*>(Y1 + (size_t)row * ldy1 + c) = v;
      }
    }
  };

  // tile i of this block: blockIdx.x + i * G; ring entry i % R, LDS slot / out buffer i & 1
  constexpr int R = WS_RING;
  uint4 gq[R][LPW], yq[R][LPW];
  if (nt > 0) {
#pragma unroll
    for (int r = 0; r < R; ++r) load(TL(r), gq[r], yq[r]);
  }
  // bit-mode dropout: the 64 draws (32 rows x 2 halves) of tile i are made once, by wave
  // (i - 1) % NW during iteration i - 1, into draw buffer i & 1
  auto draws = [&](int i) {
    if (BWD || !bit || i >= nt || wv != (i + NW - 1) % NW) return;
    uint32_t gr32 = row0 + (uint32_t)(T(i) * TILE + lr);
    asm volatile("" : "+v"(gr32));
    sD[(i & 1) * 64 + lane] = drop_draw(gr32, 0, h, step, k0, k1, true);
  };
  if (nt > 0) {
    put(0, gq[0], yq[0]);
    load(TL(R), gq[0], yq[0]);
  }
  // the weights consumed here (an empty asm reading them), behind the first ring loads:
  // complete before the loop, or the wait-count pass keeps counting them behind every ring
  // load and each MFMA waits for nearly every load in flight
#pragma unroll
  for (int s = 0; s < KS; ++s) asm volatile("" ::"v"(wa[s].x), "v"(wa[s].y), "v"(wa[s].z), "v"(wa[s].w));
  if (!BWD && bit && thr8 > 0 && wv == 0 && nt > 0) {
    uint32_t gr32 = row0 + (uint32_t)(T(0) * TILE + lr);
    sD[lane] = drop_draw(gr32, 0, h, step, k0, k1, true);
  }
  __syncthreads();
  // iteration i: put tile i + 1 (ring entry (i + 1) % R), load tile i + 1 + R into it,
  // compute tile i, store the outputs of tile i - 1, barrier
  // groups of R iterations without exits (the iterations past nt compute nothing): a
  // loop body the wait-count pass can follow, so the ring loads stay in flight across it
  for (int i0 = 0; i0 < nt; i0 += R) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int i = i0 + r;
      put((i + 1) & 1, gq[(r + 1) % R], yq[(r + 1) % R]);     // past the end: a slot nobody reads
      load(TL(i + 1 + R), gq[(r + 1) % R], yq[(r + 1) % R]);
      if (thr8 > 0) draws(i + 1);
      if (i < nt) compute(T(i), i & 1, i & 1, i);
      if (i > 0 && i <= nt) store(T(i - 1), (i - 1) & 1);
      __syncthreads();
    }
  }
  if (nt > 0 && nt % R == 0) store(T(nt - 1), (nt - 1) & 1);
}

// ---------------------------------------------------------------- launchers
static int grid_rows(int n, int waves) {
  const int tiles = (n + TILE - 1) / TILE;
  return std::max(1, std::min(device_cus(), (tiles + waves - 1) / waves));
}

static int pick_ks(int K) {
  const int ks = (K + 15) / 16;
  for (int c : {4, 8, 16, 24, 32, 40, 48}) if (ks <= c) return c;
  return -1;
}

constexpr size_t LDS_MAX = 160 * 1024;

// widest slab (multiple of 32 columns) whose bf16 weight image fits the LDS budget
static int slab_cols(int N, int KP) {
  const size_t budget = 144 * 1024;
  int cols = (N + 31) / 32 * 32;
  while (cols > 32 && (size_t)cols * (KP + 8) * 2 + (size_t)cols * 4 > budget) cols -= 32;
  return cols;
}



template <int KS, int ET>
static int fwd_launch(const uint16_t* x1, int ld1, int K1, const uint16_t* x2, int ld2, int K2, const float* W, int N,
                      const float* bias, uint16_t* Y, int ldy, int n, int relu, float p, uint32_t k0, uint32_t k1,
                      uint32_t step, uint32_t thr8, uint32_t row0, const int* stepp, const float* rscale,
                      const int* idx1, uint16_t* wimg, float* Yf, int nsplit, int tk, hipStream_t st) {
  constexpr int KP = KS * 16;
  constexpr int WV = KS == 16 ? FWD16_WAVES : KS == 8 ? FWD8_WAVES : FwdWaves<KS>::value;
  const int ncols = slab_cols(std::max(N, ldy), KP);
  const size_t lds = (size_t)ncols * (KP + 8) * 2 + (size_t)ncols * 4;
  {
    const int slabs = (std::max(N, ldy) + ncols - 1) / ncols;
    const long total = (long)slabs * ncols * (KP + 8);
    const float scale = thr8 > 0 ? 1.f / (1.f - p) : 1.f;     // the dropout scale, folded into the image
    hipLaunchKernelGGL(lin_prep_fwd_kernel<ET>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, W, K1 + K2,
                       N, ncols, KP, KP + 8, total, scale, wimg);
  }
  // output staging tiles after the image when they fit beside it (every shape but the widest slabs)
  const bool tst = !Yf && lds + (size_t)WV * OST_BYTES <= LDS_MAX;
  const int ost = tst ? (int)lds : -1;
  const size_t lds_all = lds + (tst ? (size_t)WV * OST_BYTES : 0);
  (void)hipFuncSetAttribute((const void*)lin_fwd_kernel<KS, ET, WV>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds_all);
  const int slabs = (std::max(N, ldy) + ncols - 1) / ncols;
  hipLaunchKernelGGL((lin_fwd_kernel<KS, ET, WV>), dim3(grid_rows(n, WV), slabs), dim3(WV * 64), lds_all, st,
                     x1, ld1, K1, x2, ld2, K2, W, N, bias, Y, ldy, n, ncols, relu, p, k0, k1, step, thr8, row0,
                     stepp, rscale, idx1, wimg, Yf, nsplit, tk, ost);
  return (int)hipGetLastError();
}

// K-chunked form: taken when the weight does not fit LDS whole and no lin_fwd-only
// feature (dropout, concatenation, gather, fp32 tail) is asked for; N <= 256
static bool kc_wanted(int K, int N, int ldy) {
  const int Nc = std::max(N, ldy);
  if (Nc > 256) return false;
  const int ks = pick_ks(K);
  if (ks < 0) return true;
  return slab_cols(Nc, ks * 16) < (Nc + 31) / 32 * 32;
}

static int kc_pad(int K) { return (K + 63) / 64 * 64; }   // chunks of 32 (kc) and 64 (lin_gemm)

extern "C" int gnn_lin_fwd_kc_wanted(int K, int N, int ldy) { return kc_wanted(K, N, ldy) ? 1 : 0; }

template <int FG, int ET>
static int kc_launch(const uint16_t* x, int ldx, int K, const float* W, int N, const float* bias, uint16_t* Y,
                     int ldy, int n, int relu, const float* rscale, uint16_t* wimg, hipStream_t st) {
  const int KPc = kc_pad(K);
  const long total = (long)FG * 128 * KPc;
  hipLaunchKernelGGL(lin_prep_kc_kernel<ET>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, W, K, N, KPc,
                     total, wimg);
  // the 256 x 256 tiled GEMM where it applies, else the kc kernel
  if (FG == 2) {
    const size_t lds = std::max(sizeof(uint16_t) * 2 * (256 + 256) * 64, (size_t)8 * GEMM_OST_BYTES);
    (void)hipFuncSetAttribute((const void*)lin_gemm_kernel<ET>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((lin_gemm_kernel<ET>), dim3((n + 255) / 256), dim3(512), lds, st, x, ldx, K, wimg, KPc, bias, Y,
                       ldy, N, n, relu, rscale);
    return (int)hipGetLastError();
  }
  const int rows_per_block = 4 / FG * 64;
  hipLaunchKernelGGL((lin_fwd_kc_kernel<FG, ET>), dim3((n + rows_per_block - 1) / rows_per_block), dim3(256), 0, st,
                     x, ldx, K, wimg, KPc, bias, Y, ldy, N, n, relu, rscale);
  return (int)hipGetLastError();
}

// ---- weight-stationary launches (lin_ws_kernel) ----
template <int KS, int ET, int NW, bool BWD>
static int ws_launch(const uint16_t* a1, int lda1, int K1, const uint16_t* a2, int lda2, int K2, const int* idx1,
                     const uint16_t* Ym, int ldym, const float* W, int WK, int WN, const uint16_t* wimg, const float* bias,
                     int N, float scale,
                     uint16_t* Y1, int ldy1, int KO1, uint16_t* Y2, int ldy2, int n, int relu, uint32_t k0,
                     uint32_t k1, uint32_t step, uint32_t thr8, uint32_t row0, const int* stepp, const float* rscale,
                     float mscale, hipStream_t st) {
  constexpr int KP = KS * 16;
  const size_t lds = 2 * 32 * KP * 2 + 2 * 32 * (NW * 64 + 16) + (BWD ? 0 : 2 * 64 * 16 + WS_IDX_TILES * 32 * 4) +
                     WS_IDX_TILES * 32 * 4;
  auto kern = lin_ws_kernel<KS, ET, NW, BWD>;
  static int occ = 0;
  if (!occ) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, NW * 64, lds) != hipSuccess || occ < 1) occ = 1;
  }
  const int tiles = (n + TILE - 1) / TILE;
  const int grid = std::max(1, std::min(tiles, device_cus() * occ));
  if ((idx1 || rscale) && (tiles + grid - 1) / grid > WS_IDX_TILES) return -4;   // row ids / scales do not fit
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NW * 64), lds, st, a1, lda1, K1, a2, lda2, K2, idx1, Ym, ldym, W, WK, WN, wimg, bias,
                     N, scale, Y1, ldy1, KO1, Y2, ldy2, n, relu, k0, k1, step, thr8, row0, stepp, rscale, mscale);
  return (int)hipGetLastError();
}

// waves of the weight-stationary form for `cols` output columns (0: not covered)
// (the fewest of 2 / 4 / 8 covering the columns whose ring entries stay at <= 2 loads per
// lane: a narrow layer on a long reduction takes more waves than columns, the extra
// ones computing zero-weight columns that are never stored)
static int ws_waves(int KS, int cols) {
  if (KS > 16 || cols > 256) return 0;
  for (int nw : {2, 4, 8})
    if (32 * nw >= cols && (KS + nw - 1) / nw <= 2) return nw;
  return 0;
}

#define WS_DISPATCH(KSV, BWDV, ETV, ...)                                                            \
  {                                                                                                 \
    int rc_ = -4;                                                                                   \
    switch (KSV * 100 + nw) {                                                                       \
      case 402: rc_ = ws_launch<4, ETV, 2, BWDV>(__VA_ARGS__); break;                               \
      case 404: rc_ = ws_launch<4, ETV, 4, BWDV>(__VA_ARGS__); break;                               \
      case 408: rc_ = ws_launch<4, ETV, 8, BWDV>(__VA_ARGS__); break;                               \
      case 804: rc_ = ws_launch<8, ETV, 4, BWDV>(__VA_ARGS__); break;                               \
      case 808: rc_ = ws_launch<8, ETV, 8, BWDV>(__VA_ARGS__); break;                               \
      case 1608: rc_ = ws_launch<16, ETV, 8, BWDV>(__VA_ARGS__); break;                             \
      default: break;                                                                               \
    }                                                                                               \
    if (rc_ != -4) return rc_;   /* -4: not this form (the slab kernel follows) */                   \
  }

// et: element type of X / Y (0 bf16, 1 fp16: the inference path; fp16 takes K <= 768,
// no dropout or fp32 tail)
extern "C" int gnn_launch_lin_fwd(const void* x1, int ld1, int K1, const void* x2, int ld2, int K2, const float* W,
                                  int N, const float* bias, void* Y, int ldy, int n, int relu, float p, uint32_t k0,
                                  uint32_t k1, uint32_t step, uint32_t row0, const int* stepp, const float* rscale,
                                  const int* idx1, void* wimg, float* Yf, int nsplit, int tk, hipStream_t st, int et) {
  if (n <= 0) return 0;
  if ((x2 && K1 % 8) || ld1 % 8 || (x2 && (ld2 % 8)) || ldy % 8 || K1 > ld1 || (x2 && K2 > ld2))
    return -3;
  if (Yf ? (nsplit % 4 || nsplit > ldy || nsplit > N || tk <= 0 || (N - nsplit) % tk) : N > ldy) return -3;
  if (!x2) K2 = 0;
  const uint32_t thr8 = (uint32_t)std::min(255.0, std::floor((double)p * 256.0 + 0.5));
  const int ks = pick_ks(K1 + K2);
  auto a = (const uint16_t*)x1;
  auto b = (const uint16_t*)x2;
  auto y = (uint16_t*)Y;
  if (!x2 && !idx1 && !thr8 && !Yf && kc_wanted(K1, N, ldy)) {
    const int fg = std::max(N, ldy) > 128 ? 2 : 1;
    auto w = (uint16_t*)wimg;
    if (et == 1)
      return fg == 2 ? kc_launch<2, 1>(a, ld1, K1, W, N, bias, y, ldy, n, relu, rscale, w, st)
                     : kc_launch<1, 1>(a, ld1, K1, W, N, bias, y, ldy, n, relu, rscale, w, st);
    return fg == 2 ? kc_launch<2, 0>(a, ld1, K1, W, N, bias, y, ldy, n, relu, rscale, w, st)
                   : kc_launch<1, 0>(a, ld1, K1, W, N, bias, y, ldy, n, relu, rscale, w, st);
  }
  {
    const int nw = !Yf && !(K1 & 7) && !(K2 & 7) ? ws_waves(ks, std::max(N, ldy)) : 0;
    if (nw) {
      const float scale = thr8 > 0 ? 1.f / (1.f - p) : 1.f;
      if (et == 1) {
        if (thr8) return -3;
        WS_DISPATCH(ks, false, 1, a, ld1, K1, b, ld2, K2, idx1, nullptr, 0, W, K1 + K2, N, nullptr, bias, N, scale, y, ldy, 0,
                    nullptr, 0, n, relu, k0, k1, step, thr8, row0, stepp, rscale, 1.f, st)
      } else {
        WS_DISPATCH(ks, false, 0, a, ld1, K1, b, ld2, K2, idx1, nullptr, 0, W, K1 + K2, N, nullptr, bias, N, scale, y, ldy, 0,
                    nullptr, 0, n, relu, k0, k1, step, thr8, row0, stepp, rscale, 1.f, st)
      }
    }
  }
  if (et == 1) {
    if (thr8 || Yf) return -3;
#define LH(c) if (ks == c) return fwd_launch<c, 1>(a, ld1, K1, b, ld2, K2, W, N, bias, y, ldy, n, relu, p, k0, k1, step, thr8, row0, stepp, rscale, idx1, (uint16_t*)wimg, Yf, nsplit, tk, st);
    LH(4) LH(8) LH(16) LH(24) LH(32) LH(40) LH(48)
#undef LH
    return -1;
  }
#define LF(c) if (ks == c) return fwd_launch<c, 0>(a, ld1, K1, b, ld2, K2, W, N, bias, y, ldy, n, relu, p, k0, k1, step, thr8, row0, stepp, rscale, idx1, (uint16_t*)wimg, Yf, nsplit, tk, st);
  LF(4) LF(8) LF(16) LF(24) LF(32)
#undef LF
  return -1;
}

template <int KN>
static int bwd_data_launch(const uint16_t* dY, int lddy, const uint16_t* Ym, int ldym, float mscale, int N,
                           const float* W, int K1, int K2, uint16_t* dX1, int ldx1, uint16_t* dX2, int ldx2,
                           const float* rscale, int n, int dx1_f32, uint16_t* wimg, hipStream_t st) {
  constexpr int NP = KN * 16;
  const int K = K1 + K2;
  const int kcols = slab_cols(K, NP);
  const size_t lds = (size_t)kcols * (NP + 8) * 2;
  {
    const long total = (long)((K + kcols - 1) / kcols) * kcols * (NP + 8);
    hipLaunchKernelGGL(lin_prep_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, W, K, N, NP,
                       NP + 8, total, wimg);
  }
  constexpr int WV = KN == 16 ? BWD16_WAVES : FwdWaves<KN>::value;
  const bool tst = !dx1_f32 && lds + (size_t)WV * OST_BYTES <= LDS_MAX;
  const int ost = tst ? (int)lds : -1;
  const size_t lds_all = lds + (tst ? (size_t)WV * OST_BYTES : 0);
  (void)hipFuncSetAttribute((const void*)lin_bwd_data_kernel<KN, WV>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds_all);
  const int slabs = (K + kcols - 1) / kcols;
  hipLaunchKernelGGL((lin_bwd_data_kernel<KN, WV>), dim3(grid_rows(n, WV), slabs), dim3(WV * 64), lds_all, st,
                     dY, lddy, Ym, ldym, mscale, N, W, K1, K2, dX1, ldx1, dX2, ldx2, rscale, n, kcols, dx1_f32, wimg,
                     ost);
  return (int)hipGetLastError();
}

extern "C" int gnn_launch_lin_bwd_data(const void* dY, int lddy, const void* Ym, int ldym, float mscale, int N,
                                       const float* W, int K1, int K2, void* dX1, int ldx1, void* dX2, int ldx2,
                                       const float* rscale, int n, int dx1_f32, void* wimg, hipStream_t st) {
  if (n <= 0) return 0;
  if (lddy % 8 || (Ym && ldym % 8) || (dX2 && K1 % 8) || ldx1 % 8 || (dX2 && ldx2 % 8) || N > lddy) return -3;
  if (!dX2) K2 = 0;
  const int kn = pick_ks(N);
  auto d = (const uint16_t*)dY;
  auto m = (const uint16_t*)Ym;
  auto o1 = (uint16_t*)dX1;
  auto o2 = (uint16_t*)dX2;
  {
    const int nw = !dx1_f32 && !(N & 7) ? ws_waves(kn, K1 + K2) : 0;
    if (nw) {
      const int NP = kn * 16, rows = nw * 32;
      const long total = (long)rows * (NP + 8);
      hipLaunchKernelGGL(lin_prep_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, W, K1 + K2, N,
                         NP, NP + 8, total, (uint16_t*)wimg);
      WS_DISPATCH(kn, true, 0, d, lddy, N, nullptr, 0, 0, nullptr, m, ldym, W, K1 + K2, N, (const uint16_t*)wimg, nullptr,
                  N, 1.f, o1,
                  ldx1, K1, o2, ldx2, n, 0, 0u, 0u, 0u, 0u, 0u, nullptr, rscale, mscale, st)
    }
  }
#define LB(c) if (kn == c) return bwd_data_launch<c>(d, lddy, m, ldym, mscale, N, W, K1, K2, o1, ldx1, o2, ldx2, rscale, n, dx1_f32, (uint16_t*)wimg, st);
  LB(4) LB(8) LB(16) LB(24) LB(32)
#undef LB
  return -1;
}

// bytes of the weight images the launchers write (the caller provides the scratch)
// (upper bounds over every slab width the launchers may pick for any row count:
// slabs * width < columns + 256)
extern "C" long gnn_lin_fwd_image_bytes(int K, int N, int ldy) {
  const long kc = kc_wanted(K, N, ldy) ? 2L * 256 * kc_pad(K) : 0;
  const int ks = pick_ks(K);
  if (ks < 0) return kc > 0 ? kc : -1;
  const int KP = ks * 16;
  return std::max(kc, 2L * ((std::max(N, ldy) + 31) / 32 * 32 + 256) * (KP + 8));
}

extern "C" long gnn_lin_bwd_image_bytes(int K, int N) {
  const int kn = pick_ks(N);
  if (kn < 0) return -1;
  const int NP = kn * 16;
  return 2L * ((K + 31) / 32 * 32 + 256) * (NP + 8);
}

// chunk count of the split-K weight gradient for n rows and N columns (fills the chip)
// lin_bwd_weight2's column tiles per block: the widest of {2, 4, 8} the columns need whose
// accumulators fit a wave (KPW * CPW <= 8, see Wgt2)
static int wgt2_nb(int kt, int N) {
  const int kw = std::min(kt, 8), wpk = 8 / kw, kpw = (kt + kw - 1) / kw;
  int nb = N <= 64 ? 2 : N <= 128 ? 4 : 8;
  while (nb > 2 && kpw * ((nb + wpk - 1) / wpk) > 8) nb >>= 1;
  return nb;
}

// Row chunks of the split-K weight gradient (the gpart scratch's leading dimension).
// lin_bwd_weight2 (K > 0): one 8-wave block per CU over all chunks x column slabs;
// the v1 kernel: two 8-wave blocks per CU over its 64-column slabs.
extern "C" int gnn_lin_wgrad_chunks(int n, int N, int K) {
  const int tiles = std::max(1, (n + TILE - 1) / TILE);
  if (K > 0) {
    const int slabs = (N + 32 * wgt2_nb((K + 31) / 32, N) - 1) / (32 * wgt2_nb((K + 31) / 32, N));
    return std::min(tiles, std::max(1, device_cus() / std::max(slabs, 1)));
  }
  const int slabs = std::max(1, (N + 63) / 64);
  const int want = std::max(1, 2 * device_cus() / slabs);
  return std::min(tiles, want);
}

template <int KT>
static int wgt_launch(const uint16_t* x1, int ld1, int K1, const uint16_t* x2, int ld2, int K2, const uint16_t* dY,
                      int lddy, const uint16_t* Ym, int ldym, float mscale, int N, float* gpart, int n, int chunks,
                      const int* idx1, hipStream_t st) {
  const int tiles = (n + TILE - 1) / TILE;
  const int rpc = (tiles + chunks - 1) / chunks * TILE;
  hipLaunchKernelGGL((lin_bwd_weight_kernel<KT>), dim3(chunks, (N + 63) / 64), dim3(WGT_WAVES * 64), 0, st, x1, ld1,
                     K1, x2, ld2, K2, dY, lddy, Ym, ldym, mscale, N, gpart, n, rpc, idx1);
  return (int)hipGetLastError();
}

constexpr int WGT2_LDS_MAX = 160 * 1024;

// -1: the staged row ids of a gathered X1 would not fit next to the images (the caller
// falls back to v1 with the same chunking)
template <int KT, int NB, bool HAS_YM>
static int wgt2_launch_t(const uint16_t* x1, int ld1, int K1, const uint16_t* x2, int ld2, int K2, const uint16_t* dY,
                         int lddy, const uint16_t* Ym, int ldym, float mscale, int N, float* gpart, int n, int chunks,
                         const int* idx1, hipStream_t st) {
  const int tiles = (n + TILE - 1) / TILE;
  const int rpc = (tiles + chunks - 1) / chunks * TILE;
  const long lds = Wgt2<KT, NB>::LDS + (idx1 ? 4L * rpc : 0L);
  if (lds > WGT2_LDS_MAX) return -1;
  static const bool attr = [] {
    (void)hipFuncSetAttribute((const void*)lin_bwd_weight2_kernel<KT, NB, HAS_YM>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, WGT2_LDS_MAX);
    return true;
  }();
  (void)attr;
  hipLaunchKernelGGL((lin_bwd_weight2_kernel<KT, NB, HAS_YM>), dim3(chunks, (N + 32 * NB - 1) / (32 * NB)), dim3(512),
                     (size_t)lds, st, x1, ld1, K1, x2, ld2, K2, dY, lddy, Ym, ldym, mscale, N, gpart, n, rpc, idx1);
  return (int)hipGetLastError();
}

template <int KT, int NB>
static int wgt2_launch(const uint16_t* x1, int ld1, int K1, const uint16_t* x2, int ld2, int K2, const uint16_t* dY,
                       int lddy, const uint16_t* Ym, int ldym, float mscale, int N, float* gpart, int n, int chunks,
                       const int* idx1, hipStream_t st) {
  return Ym ? wgt2_launch_t<KT, NB, true>(x1, ld1, K1, x2, ld2, K2, dY, lddy, Ym, ldym, mscale, N, gpart, n, chunks,
                                          idx1, st)
            : wgt2_launch_t<KT, NB, false>(x1, ld1, K1, x2, ld2, K2, dY, lddy, Ym, ldym, mscale, N, gpart, n, chunks,
                                           idx1, st);
}

// gpart: [chunks][K1 + K2 + 1][N] fp32 scratch (chunks = gnn_lin_wgrad_chunks(n, N, K1 + K2));
// dW: [K1 + K2][N] fp32, db: [N] fp32 (optional)
extern "C" int gnn_launch_lin_bwd_weight(const void* x1, int ld1, int K1, const void* x2, int ld2, int K2,
                                         const void* dY, int lddy, const void* Ym, int ldym, float mscale, int N,
                                         float* gpart, float* dW, float* db, int n, const int* idx1, hipStream_t st) {
  if ((x2 && K1 % 8) || ld1 % 8 || (x2 && ld2 % 8) || lddy % 8 || (Ym && ldym % 8) || N > lddy) return -3;
  if (!x2) K2 = 0;
  const int K = K1 + K2;
  const int chunks = gnn_lin_wgrad_chunks(std::max(n, 1), N, K);
  if (n > 0) {
    const int kt = (K + 31) / 32;
    auto a = (const uint16_t*)x1;
    auto b = (const uint16_t*)x2;
    auto d = (const uint16_t*)dY;
    auto m = (const uint16_t*)Ym;
    int rc = -1;
    {
      const int nb = wgt2_nb(kt, N);
#define LW2(c, b_) if (rc == -1 && kt <= c && nb == b_) rc = wgt2_launch<c, b_>(a, ld1, K1, b, ld2, K2, d, lddy, m, ldym, mscale, N, gpart, n, chunks, idx1, st);
      LW2(2, 2) LW2(2, 4) LW2(2, 8) LW2(4, 2) LW2(4, 4) LW2(4, 8) LW2(5, 2) LW2(5, 4)
      LW2(8, 2) LW2(8, 4) LW2(8, 8) LW2(9, 2) LW2(9, 4) LW2(12, 2) LW2(12, 4) LW2(16, 2) LW2(16, 4) LW2(17, 2)
#undef LW2
      if (rc == -1) rc = -2;                 // no v2 form: v1 below
    }
    if (rc == -2) {
      rc = -1;
#define LW(c) if (rc == -1 && kt <= c) rc = wgt_launch<c>(a, ld1, K1, b, ld2, K2, d, lddy, m, ldym, mscale, N, gpart, n, chunks, idx1, st);
      LW(2) LW(4) LW(5) LW(8) LW(9) LW(12) LW(16) LW(17)
#undef LW
    }
    if (rc != 0) return rc;
  } else {
    (void)hipMemsetAsync(gpart, 0, sizeof(float) * (size_t)(K + 1) * N * chunks, st);
  }
  const long count = (long)(K + 1) * N;
  if (count % 4 == 0)
    hipLaunchKernelGGL(lin_reduce4_kernel, dim3((unsigned)((count + 127) / 128)), dim3(256), 0, st, gpart,
                       n > 0 ? chunks : 1, count, N, dW, db);
  else
    hipLaunchKernelGGL(lin_reduce_kernel, dim3((unsigned)((count + 31) / 32)), dim3(256), 0, st, gpart,
                       n > 0 ? chunks : 1, count, N, dW, db);
  return (int)hipGetLastError();
}
