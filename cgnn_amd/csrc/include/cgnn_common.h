// Shared device helpers for the cgnn_amd HIP kernels (gfx950 / CDNA4 only).
//
//  * Philox4x32-10 counter-based RNG.  Every random number in the framework is
//    a pure function of (key, counter): key = per-model 64-bit key derived on
//    the host from (seed, run, salt); counter = (row, stream-id, step, purpose).
//    Results therefore do not depend on batching, launch geometry or on how
//    many GPUs share the work.  The Python mirror used by
//    the CPU path lives in cgnn_amd/utils/philox.py and is bit-identical in the
//    integer part.
//  * 64-lane wave reductions (wavefront = 64 on CDNA4, never 32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CGNN_WAVE 64

namespace cgnn {

// ---------------------------------------------------------------- DAG programs
// int32 model description (engine/program.py): header, node records, index pool
constexpr int PROG_HDR = 4;      // n_nodes, n_params, n_conf, max_in
constexpr int NODE_REC = 8;      // var, kind, n_par, par_off, n_cf, cf_off, param_off, n_in
constexpr int KIND_GEN = 0;
constexpr int KIND_OBS = 1;

// wave-uniform load: the value lands in an SGPR (program words, stage tables)
__device__ __forceinline__ int uni(const int* p) { return __builtin_amdgcn_readfirstlane(*p); }

// ---------------------------------------------------------------- Philox
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ void mulhilo32(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo32(M0, c.x, hi0, lo0);
    mulhilo32(M1, c.z, hi1, lo1);
    u32x4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// uniform in (0,1): 24 random bits, centred in their bucket (never 0 or 1).
__device__ __forceinline__ float u01(uint32_t x) {
  return ((float)(x >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

// One standard normal from one Philox block (Box-Muller, cos branch).
// v_log_f32 is log2 and v_cos_f32 takes revolutions, so
//   n = sqrt(-2 ln2 * log2(u1)) * cos(2*pi*u2)  ->  two transcendental ops.
__device__ __forceinline__ float normal_from(u32x4 r) {
  float u1 = u01(r.x), u2 = u01(r.y);
  float rad = __builtin_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
  return rad * __builtin_amdgcn_cosf(u2);
}

// Two independent normals from one Philox block (cos and sin branches).
__device__ __forceinline__ void normal2_from(u32x4 r, float& n0, float& n1) {
  float u1 = u01(r.x), u2 = u01(r.y);
  float rad = __builtin_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
  n0 = rad * __builtin_amdgcn_cosf(u2);
  n1 = rad * __builtin_amdgcn_sinf(u2);
}

// RNG purposes (4th counter word).
enum RngPurpose : uint32_t {
  RNG_NODE_NOISE = 1u,   // per-node generator noise  e_v      (row, var, step)
  RNG_CONF_NOISE = 2u,   // per-skeleton-edge noise   xi_uv    (row, edge, step)
  RNG_PARAM_INIT = 3u,   // parameter init            N(0,s^2) (param, 0, 0)
  RNG_RFF_FREQ   = 4u,   // Fourier-MMD frequencies            (feat, dim, step)
  RNG_DROPOUT    = 5u,   // GNN dropout masks                  (row, col/4, step)
  RNG_SAMPLE     = 6u,   // GNN neighbour sampling             (node, salt, draw/4)
};

// ---- dropout keep masks (every GNN kernel, and ops.dropout_keep_mask on the host) ----
// Unit n of row `row` of a dropout layer: n = 32 t + 8 g + 4 h + i, q = 4 g + i; the 16
// units of one (row, t, h) share one call.  thr8 = round(256 p).
//   byte mode (any p): byte q of the draw keyed (row, 2 t + h, step) kept iff >= thr8;
//   bit mode (p = 1/2, thr8 = 128): bit 16 (t % 8) + q of the draw keyed
//   (row, DROP_BIT_CTR + 2 (t / 8) + h, step) kept iff set -- one random bit per decision,
//   so one draw covers eight 32-unit blocks (a 256-wide hidden layer draws once per
//   (row, half) instead of eight times).
constexpr uint32_t DROP_BIT_CTR = 0x80000000u;

__device__ __forceinline__ bool drop_bit_mode(uint32_t thr8) { return thr8 == 128u; }

__device__ __forceinline__ u32x4 drop_draw(uint32_t row, int t, int h, uint32_t step, uint32_t k0, uint32_t k1,
                                           bool bit_mode) {
  const uint32_t c = bit_mode ? DROP_BIT_CTR + 2u * (uint32_t)(t >> 3) + (uint32_t)h : 2u * (uint32_t)t + (uint32_t)h;
  return philox4x32_10(u32x4{row, c, step, RNG_DROPOUT}, k0, k1);
}

// the 16 keep bits (bit q) of block t from its draw
__device__ __forceinline__ uint32_t drop_keep16(const u32x4& r, int t, uint32_t thr8, bool bit_mode) {
  if (bit_mode) {
    const int wi = (t & 7) >> 1;
    const uint32_t w = wi == 0 ? r.x : wi == 1 ? r.y : wi == 2 ? r.z : r.w;
    return (w >> (16 * (t & 1))) & 0xffffu;
  }
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
  uint32_t m = 0u;
#pragma unroll
  for (int q = 0; q < 16; ++q) m |= (((w[q >> 2] >> (8 * (q & 3))) & 0xffu) >= thr8 ? 1u : 0u) << q;
  return m;
}

__device__ __forceinline__ float rng_normal(uint32_t k0, uint32_t k1, uint32_t a, uint32_t b,
                                            uint32_t step, uint32_t purpose) {
  u32x4 c = {a, b, step, purpose};
  return normal_from(philox4x32_10(c, k0, k1));
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, CGNN_WAVE);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, CGNN_WAVE));
  return v;
}

// Deterministic block sum (fixed tree), result valid in every thread.
// `scratch` needs blockDim.x / 64 floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int w = 0; w < nw; ++w) t += scratch[w];
  return t;
}

// XCD-aware block remaps (MI355X: 8 XCDs, each with its own L2; the dispatcher deals
// blocks round-robin over XCDs).  Speed only -- never correctness.
// Chunk-interleaved form: XCD x takes chunks x, x + 8, ... of C consecutive blocks --
// contiguous work within a chunk (its L2 locality), the whole range sampled by every XCD
// (its load balance when the per-row work drifts along the rows, as in a locality-
// ordered graph shard: papers100M GAT rank-0-of-8 dry run 38.8 -> 34.8 ms at scale 0.5,
// profiles/r05_gat).  Bijective; the ragged tail (< 8 C blocks) keeps its ids.
template <unsigned C>
__host__ __device__ __forceinline__ unsigned xcd_remap_chunked(unsigned b, unsigned nwg) {
  const unsigned full = nwg / (8u * C) * (8u * C);
  if (b >= full) return b;
  const unsigned xcd = b & 7u, idx = b >> 3;
  return (idx / C) * (8u * C) + xcd * C + idx % C;
}

// XCD-aware block remap (MI355X: 8 XCDs, each with its own L2; the dispatcher
// deals blocks round-robin over XCDs).  Returns a logical block id such that the
// blocks resident on one XCD process a CONTIGUOUS range of the work.  Bijective
// for any grid size (q = n/8, r = n%8).  Speed only -- never correctness.
__host__ __device__ __forceinline__ unsigned xcd_remap(unsigned b, unsigned nwg) {
  const unsigned q = nwg >> 3, r = nwg & 7u;
  const unsigned xcd = b & 7u, idx = b >> 3;
  const unsigned base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + idx;
}

// ---- packed-fp32 multi-bandwidth RBF (the seven gammas of Loss.py:10) ----
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 exp2_2(f2 x) {
  return f2{__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
}

// The seven kernel values exp(-g d2), g in {0.005, 0.05, 0.25, 0.5, 1, 5, 50},
// for two distances: two v_exp_f32
// and powering -- a = e^{-0.005 d}, a^10 = e^{-0.05 d}; c = e^{-0.25 d}, c^2, c^4,
// c^20 = e^{-5 d}, c^200 = e^{-50 d} (13 packed multiplies replace 5 exps; the
// relative error of c^200 is ~200 ulp, i.e. ~1e-5 on a term that matters only
// for d < 0.1).

__device__ __forceinline__ void rbf7_values(f2 d2, f2* e) {
  const float L2E = 1.4426950408889634f;
  const f2 a = exp2_2(d2 * (-0.005f * L2E));
  const f2 a2 = a * a, a4 = a2 * a2, a8 = a4 * a4;
  const f2 c = exp2_2(d2 * (-0.25f * L2E));
  const f2 c2 = c * c, c4 = c2 * c2, c8 = c4 * c4, c16 = c8 * c8, c20 = c16 * c4;
  const f2 c40 = c20 * c20, c80 = c40 * c40, c160 = c80 * c80;
  e[0] = a; e[1] = a8 * a2; e[2] = c; e[3] = c2; e[4] = c4; e[5] = c20; e[6] = c160 * c40;
}

// seven bandwidths for two distances at once; returns ks (kernel sum) and w
// (sum gamma * kernel) as packed pairs.
__device__ __forceinline__ void rbf7x2(f2 d2, f2& ks, f2& w) {
  f2 e[7];
  rbf7_values(d2, e);
  ks = ((e[0] + e[1]) + (e[2] + e[3])) + ((e[4] + e[5]) + e[6]);
  w = ((0.005f * e[0] + 0.05f * e[1]) + (0.25f * e[2] + 0.5f * e[3])) + ((e[4] + 5.0f * e[5]) + 50.0f * e[6]);
}

// ---- packed 16-bit epilogue helpers (two elements per dword, one instruction each) ----
// two fp32 -> two bf16 in one dword (hipcc emits v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t cvt_pk(float a, float b) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const bf16x2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}
// two fp32 -> two fp16 in one dword (round to nearest even)
__device__ __forceinline__ uint32_t cvt_pk_h(float a, float b) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  const h2 v = {(_Float16)a, (_Float16)b};
  return __builtin_bit_cast(uint32_t, v);
}
// per 16-bit half max(x, lo) as signed integers.  lo = 0 is the relu of two bf16 / fp16
// values (a negative one, -0 included, is a negative int16); lo = 0x80008000 leaves x as is
__device__ __forceinline__ uint32_t pk_max_i16(uint32_t x, uint32_t lo) {
  uint32_t r;
  asm("v_pk_max_i16 %0, %1, %2" : "=v"(r) : "v"(x), "s"(lo));
  return r;
}
__device__ __forceinline__ uint32_t pk_relu(uint32_t x) {
  uint32_t r;
  asm("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(x));
  return r;
}
// per 16-bit half: x * k (k in {0, 1}: a keep bit applied without a compare or select)
__device__ __forceinline__ uint32_t pk_mul16(uint32_t x, uint32_t k) {
  uint32_t r;
  asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(r) : "v"(x), "v"(k));
  return r;
}
// per 16-bit half: 1 if x != 0 else 0 (x a relu output, so != 0 means > 0).  The 1s
// come from a register: an inline constant of a packed instruction reaches only the low
// half (the high half of its 32-bit value, 0, feeds the high half).
__device__ __forceinline__ uint32_t pk_nz(uint32_t x) {
  uint32_t r;
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(x), "s"(0x00010001u));
  return r;
}
// the 16 keep bits m of a dropout block spread for pk_mul16: bit 2i stays, bit 2i + 1
// moves to bit 2i + 16, so (spread >> 2i) & 0x10001 is the keep pair of values 2i, 2i + 1
__device__ __forceinline__ uint32_t keep_spread(uint32_t m) { return (m & 0x5555u) | ((m & 0xaaaau) << 15); }


// CUs of the current device (cached per device; 256 on MI355X) for persistent grids
inline int device_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    hipDeviceProp_t prop;
    cached[dev] = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
  }
  return cached[dev];
}

}  // namespace cgnn
