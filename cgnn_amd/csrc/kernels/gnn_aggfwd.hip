// The GCN's layer-1 aggregation fused with its dense forward (GNN track, not in the
// reference; the headline 2-layer GCN, bench.py):
//
//     AX = D^-1/2 (A + I) Xs        gathered per 32-row tile (gnn_gather.h, the same
//                                   instructions in the same order as spmm_kernel: AX is
//                                   bit-identical), stored for the backward
//     Z2 = dinv * (dropout(relu(AX W1 + b1)) W2)     on MFMA, as gcn_dense_fwd_kernel
//
// Why: the aggregation is bound by its gather issue (114 M row gathers, 2.08 ms on the
// ogbn-products shape, MFMA idle), and the dense forward (0.28 ms, MFMA + VALU) ran
// strictly after it.  Here every wave alternates the two on its own tiles, so the 16
// waves of a CU are at different phases: while some wait on gathers, others run their
// tile's matrix products -- the dense work fills the aggregation's idle issue slots, and
// AX is read back from L2 right after it was written instead of from HBM by a second
// launch.
//
// Geometry: one persistent 16-wave block per CU (the weights W1^T / W2^T / b1 in LDS, as
// the dense kernel).  The BLOCK takes chunks of CH = 64 RPC rows (2 RPC tiles) from
// per-XCD work queues: the blocks that share an XCD (block id mod 8, dispatch order;
// speed only) take the chunks of one contiguous eighth of the rows first -- their gathers
// share that XCD's L2 -- then help the other eighths.  Each wave gathers 4 RPC rows of a
// chunk; the wave that completes a tile's rows (an LDS counter per tile) runs that
// tile's dense forward while the others move on to the next chunk.  So the rows in
// flight on an XCD stay a narrow window (~32 blocks x 2 chunks): a wave owning a whole
// 32-row tile for its gathers put 16 K rows in flight per XCD and dropped the L2 hit
// rate from 0.72 to 0.48 (profiles/r05_agg).  The last wave to finish resets the queues
// for the next launch.
#include "cgnn_common.h"
#include "gnn_gather.h"
#include <algorithm>

using namespace cgnn;
using namespace cgnn::gather;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

constexpr int WAVES = 16;
constexpr int TILE = 32;
constexpr int NQ = 8;                 // work queues (XCDs)
constexpr int RING = 4;               // chunk slots per block
constexpr int RQ = 64;                // ready-tile queue entries per block
// A/B build options (tools/build_variant.sh -D..., profiles/r05_agg): AGG_RPC = rows per
// chunk claim in units of 64 (the kept value 1); AGG_GATHER_ONLY = skip the dense tiles
// (times the gather half alone).  Neither changes the default build's results.
#ifndef AGG_RPC
#define AGG_RPC 1
#endif

__device__ __forceinline__ bf16x8 ld_bf16x8_nt(const uint16_t* p) {
  // L1-bypassing load: the rows were just stored by other lanes of this wave
  const u32x4v v = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(p));
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ uint16_t bf16_bits(float x) { return __builtin_bit_cast(uint16_t, (__bf16)x); }

__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
  return make_uint2((uint32_t)bf16_bits(a) | ((uint32_t)bf16_bits(b) << 16),
                    (uint32_t)bf16_bits(c) | ((uint32_t)bf16_bits(d) << 16));
}

// chunks [q_lo(q), q_lo(q + 1)) belong to queue q
__device__ __forceinline__ int q_lo(int q, int n_chunks, int nq) { return (int)((long)n_chunks * q / nq); }

template <typename T>
__device__ __forceinline__ T lds_load_acq(T* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <typename T>
__device__ __forceinline__ void lds_store_rel(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

}  // namespace

// ctr: int32 [NQ + 1] (queue heads, then the finished-wave count), zero before the first
// launch; the kernel leaves it zero again.  RPC: 4-row rounds per wave and chunk.
template <int KS, int HD, int DROP, int RPC>
__global__ __launch_bounds__(WAVES * 64) void gcn_agg_fwd_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col, const uint16_t* __restrict__ Xs,
    uint16_t* __restrict__ AX, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ W2, const float* __restrict__ dinv, uint16_t* __restrict__ Z2, int n, int F,
    int ldx, int C, int ldc, float p, uint32_t k0, uint32_t k1, uint32_t step, uint32_t thr8, uint32_t row0,
    const int* __restrict__ stepp, uint16_t* __restrict__ kimg, int* __restrict__ ctr) {
  constexpr int L = 16;                 // lanes per gathered row (8 features each)
  constexpr int CH = 64 * RPC;          // chunk rows
  constexpr int TPC = CH / TILE;        // tiles per chunk
  constexpr int WPT = WAVES / TPC;      // waves per tile
  constexpr int RPW = 4 * RPC;          // rows per wave and chunk
  if (stepp) step = (uint32_t)*stepp;
  constexpr int KP = KS * 16;
  constexpr int W1S = KP + 8;
  constexpr int W2S = HD + 4;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* sW1T = lds;                                     // [HD][W1S]   W1^T
  uint16_t* sW2T = sW1T + HD * W1S;                         // [64][W2S]   W2^T (rows >= C zero)
  float* sB1 = reinterpret_cast<float*>(sW2T + 64 * W2S);   // [HD]
  // chunk ring: slot k holds the chunk id of sequence s_seq[k] (< 0 while being claimed),
  // s_cons[k] = waves done with it, s_tcnt[k][t] = waves that stored their rows of tile t
  __shared__ int s_seq[RING], s_id[RING], s_cons[RING], s_tcnt[RING][TPC], s_qi;
  // ready tiles (all rows stored), tile + 1 per entry (0: empty), taken by whichever wave
  // finishes a chunk next -- the leaders, so the dense work slows the waves that are ahead
  // (when the last arriver ran it, the same laggards kept falling further behind)
  __shared__ int s_rq[RQ], s_rq_head, s_rq_tail;
  for (int i = threadIdx.x; i < HD * KP; i += blockDim.x) {
    const int k = i / HD, nn = i - k * HD;
    sW1T[nn * W1S + k] = bf16_bits(k < F ? W1[(size_t)k * HD + nn] : 0.f);
  }
  const float scale = 1.f / (1.f - p);
  const float w2s = DROP != 0 ? scale : 1.f;     // dropout scale folded into W2^T
  for (int i = threadIdx.x; i < 64 * HD; i += blockDim.x) {
    const int nn = i / 64, c = i - nn * 64;
    sW2T[c * W2S + nn] = bf16_bits(c < C ? W2[(size_t)nn * C + c] * w2s : 0.f);
  }
  for (int i = threadIdx.x; i < HD; i += blockDim.x) sB1[i] = b1[i];
  if (threadIdx.x < RING) {
    s_seq[threadIdx.x] = (int)threadIdx.x - RING;
    s_id[threadIdx.x] = -1;
    s_cons[threadIdx.x] = WAVES;
    for (int t = 0; t < TPC; ++t) s_tcnt[threadIdx.x][t] = 0;
  }
  for (int i = threadIdx.x; i < RQ; i += blockDim.x) s_rq[i] = 0;
  if (threadIdx.x == 0) {
    s_qi = 0;
    s_rq_head = 0;
    s_rq_tail = 0;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, h = lane >> 5, lr = lane & 31;
  const int wv = threadIdx.x >> 6;
  const int sub = lane / L, sl = lane - sub * L;
  const int f0 = sl * 8;
  const int n_chunks = (n + CH - 1) / CH;
  const int nq = min(NQ, (int)gridDim.x);
  const int q0 = (int)(blockIdx.x % (unsigned)nq);
  const int tic = wv / WPT;                          // this wave's tile in a chunk
  const int rbase = tic * TILE + (wv % WPT) * RPW;   // its first row in a chunk

  // the chunk id of sequence c (claimed from the queues by the first wave to need it);
  // -1 when all queues are drained
  auto chunk_of = [&](int c) -> int {
    const int slot = c % RING;
    int id = -1;
    if (lane == 0) {
      for (;;) {
        const int sq = lds_load_acq(&s_seq[slot]);
        if (sq == c) {
          id = lds_load_acq(&s_id[slot]);
          break;
        }
        if (sq == c - RING && lds_load_acq(&s_cons[slot]) == WAVES) {
          int expect = c - RING;
          if (__hip_atomic_compare_exchange_strong(&s_seq[slot], &expect, -1 - c, __ATOMIC_ACQ_REL,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
            s_cons[slot] = 0;
            for (int t = 0; t < TPC; ++t) s_tcnt[slot][t] = 0;
            int qi = lds_load_acq(&s_qi);
            while (qi < nq) {
              const int q = (q0 + qi) % nq;
              const int lo = q_lo(q, n_chunks, nq), cnt = q_lo(q + 1, n_chunks, nq) - lo;
              const int t = atomicAdd(ctr + q, 1);
              if (t < cnt) {
                id = lo + t;
                break;
              }
              __hip_atomic_fetch_max(&s_qi, qi + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              qi = max(qi + 1, lds_load_acq(&s_qi));
            }
            lds_store_rel(&s_id[slot], id);
            lds_store_rel(&s_seq[slot], c);
            break;
          }
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    return __builtin_amdgcn_readfirstlane(id);
  };

  // the dense forward of tile `tile` (gcn_dense_fwd_kernel's tile body; AX rows read
  // back from L2, bypassing L1)
  auto dense_tile = [&](const int tile) {
    const int row = tile * TILE + lr;
    const bool rv = row < n;
    bf16x8 bx[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int fb = 16 * s + 8 * h;
      bx[s] = (rv && fb < ldx) ? ld_bf16x8_nt(AX + (size_t)row * ldx + fb)
                               : __builtin_bit_cast(bf16x8, make_uint4(0u, 0u, 0u, 0u));
    }
    const float dsc = rv ? dinv[row] : 0.f;
    f32x16 z0 = {}, z1 = {};
    u32x4 rb{};
    if constexpr (DROP == 2) rb = drop_draw(row0 + (uint32_t)row, 0, h, step, k0, k1, true);
#pragma unroll 1
    for (int t = 0; t < HD / 32; ++t) {
      const uint16_t* arow = sW1T + (32 * t + lr) * W1S + 8 * h;
      // the chain's weight fragments from LDS in batches of AB (registers: 4 waves / SIMD)
      constexpr int AB = 2;
      f32x16 acc = {};
#pragma unroll
      for (int s0 = 0; s0 < KS; s0 += AB) {
        bf16x8 af[AB];
#pragma unroll
        for (int s = 0; s < AB; ++s)
          if (s0 + s < KS) af[s] = *reinterpret_cast<const bf16x8*>(arow + 16 * (s0 + s));
#pragma unroll
        for (int s = 0; s < AB; ++s)
          if (s0 + s < KS) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bx[s0 + s], acc, 0, 0, 0);
      }
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
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 xb = __builtin_bit_cast(bf16x8, make_uint4(pk[4 * s2], pk[4 * s2 + 1], pk[4 * s2 + 2], pk[4 * s2 + 3]));
        const int nbase = 32 * t + 16 * s2 + 4 * h;
        {
          const uint16_t* a = sW2T + lr * W2S + nbase;
          const uint2 lo = *reinterpret_cast<const uint2*>(a), hi = *reinterpret_cast<const uint2*>(a + 8);
          z0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y)),
                                                       xb, z0, 0, 0, 0);
        }
        {
          const uint16_t* a = sW2T + (32 + lr) * W2S + nbase;
          const uint2 lo = *reinterpret_cast<const uint2*>(a), hi = *reinterpret_cast<const uint2*>(a + 8);
          z1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y)),
                                                       xb, z1, 0, 0, 0);
        }
      }
    }
    if constexpr (DROP == 2) {
      if (kimg) {
        uint16_t* kd = kimg + (size_t)tile * (HD / 32) * 64 + lane;
#pragma unroll
        for (int t = 0; t < HD / 32; ++t) kd[64 * t] = (uint16_t)drop_keep16(rb, t, thr8, true);
      }
    }
    if (rv) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 8 * g + 4 * h;
        if (c < ldc)
          *reinterpret_cast<uint2*>(Z2 + (size_t)row * ldc + c) =
              pack4(z0[4 * g] * dsc, z0[4 * g + 1] * dsc, z0[4 * g + 2] * dsc, z0[4 * g + 3] * dsc);
        if (32 + c < ldc)
          *reinterpret_cast<uint2*>(Z2 + (size_t)row * ldc + 32 + c) =
              pack4(z1[4 * g] * dsc, z1[4 * g + 1] * dsc, z1[4 * g + 2] * dsc, z1[4 * g + 3] * dsc);
      }
    }
  };

  // next ready tile, -1 if none
  auto pop_ready = [&]() -> int {
    int t = -1;
    if (lane == 0) {
      for (;;) {
        const int hd = lds_load_acq(&s_rq_head);
        if (hd >= lds_load_acq(&s_rq_tail)) break;
        int expect = hd;
        if (__hip_atomic_compare_exchange_strong(&s_rq_head, &expect, hd + 1, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP)) {
          int v;
          while ((v = lds_load_acq(&s_rq[hd % RQ])) == 0) __builtin_amdgcn_s_sleep(1);
          s_rq[hd % RQ] = 0;
          t = v - 1;
          break;
        }
      }
    }
    return __builtin_amdgcn_readfirstlane(t);
  };

  // chunks until the queues are drained, then the remaining ready tiles; one dense call
  // site (registers)
  bool more = true;
  for (int c = 0;; ++c) {
    int own = -1;
    if (more) {
      const int chunk = chunk_of(c);
      const int slot = c % RING;
      if (chunk < 0) {
        more = false;
        if (lane == 0) __hip_atomic_fetch_add(&s_cons[slot], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else {
        // ---- aggregation of this wave's RPW rows: RPC rounds of 4 rows, 16 lanes each ----
        const int r0 = chunk * CH + rbase;
        const int rl = min(r0 + (lane & (RPW - 1)), n - 1);
        const int e_lo = rowptr[rl], e_hi = rowptr[rl + 1];
        const float dsc = dinv[rl];
#pragma unroll 1
        for (int rd = 0; rd < RPC; ++rd) {
          const int ti = 4 * rd + sub;
          const int row = r0 + ti;
          const bool rv = row < n;
          const int e0 = rv ? __shfl(e_lo, ti, 64) : 0, e1 = rv ? __shfl(e_hi, ti, 64) : 0;
          const float rs = __shfl(dsc, ti, 64);
          float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
          gather_sum<L, 1, 16, false>(col, Xs, e0, e1, ldx, f0, rv && f0 < F, sub * L, sl, acc);
          if (rv && f0 < ldx) {
            float y[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              const int f = f0 + q;
              y[q] = f < F ? acc[q] * rs + 0.f : (f == F ? 1.f : 0.f);    // the ones column (gb1) at F
            }
            *reinterpret_cast<uint4*>(AX + (size_t)row * ldx + f0) = f32x8_to_bf16(y);
          }
        }
        // the rows are stored (L2) before the tile's counter counts them
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // the tile's last rows queue its dense forward (a tile wholly past n, in the last
        // chunk, has no keep-image slot and nothing to compute); a full queue (not expected:
        // every wave takes a tile after each chunk) falls back to running it here
        if (lane == 0) {
          const int tile = chunk * TPC + tic;
          const int done =
              __hip_atomic_fetch_add(&s_tcnt[slot][tic], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (done == WPT - 1 && tile * TILE < n) {
            if (lds_load_acq(&s_rq_tail) - lds_load_acq(&s_rq_head) < RQ / 2) {
              const int t = __hip_atomic_fetch_add(&s_rq_tail, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
              lds_store_rel(&s_rq[t % RQ], tile + 1);
            } else {
              own = tile;
            }
          }
          __hip_atomic_fetch_add(&s_cons[slot], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        own = __builtin_amdgcn_readfirstlane(own);
      }
    }
#ifdef AGG_GATHER_ONLY
    if (!more) break;
#else
    const int job = own >= 0 ? own : pop_ready();
    if (job >= 0) dense_tile(job);
    else if (!more) break;
#endif
  }
  // the last wave out resets the queues (every other wave has made its final dequeue)
  if (lane == 0) {
    const int total = (int)gridDim.x * WAVES;
    if (atomicAdd(ctr + NQ, 1) == total - 1) {
      for (int q = 0; q <= NQ; ++q) atomicExch(ctr + q, 0);
    }
  }
}

// The keep image of the byte-mode dropout, drawn on its own (gnn_dense.hip)
extern "C" int gnn_launch_keep_image(void* kimg, int n, int HD, float p, uint32_t k0, uint32_t k1, uint32_t step,
                                     uint32_t row0, const int* stepp, hipStream_t st);

static int agg_grid(int n) {
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

template <int KS, int HD, int DROP, int RPC>
static int agg_launch_d(const int* rowptr, const int* col, const uint16_t* Xs, uint16_t* AX, const float* W1,
                        const float* b1, const float* W2, const float* dinv, uint16_t* Z2, int n, int F, int ldx,
                        int C, int ldc, float p, uint32_t k0, uint32_t k1, uint32_t step, uint32_t thr8,
                        uint32_t row0, const int* stepp, uint16_t* kimg, int* ctr, hipStream_t st) {
  const size_t lds = sizeof(uint16_t) * ((size_t)HD * (KS * 16 + 8) + 64 * (size_t)(HD + 4)) + sizeof(float) * HD;
  (void)hipFuncSetAttribute((const void*)gcn_agg_fwd_kernel<KS, HD, DROP, RPC>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((gcn_agg_fwd_kernel<KS, HD, DROP, RPC>), dim3(agg_grid(n)), dim3(WAVES * 64), lds, st, rowptr, col,
                     Xs, AX, W1, b1, W2, dinv, Z2, n, F, ldx, C, ldc, p, k0, k1, step, thr8, row0, stepp, kimg, ctr);
  if (DROP == 1 && kimg) return gnn_launch_keep_image(kimg, n, HD, p, k0, k1, step, row0, stepp, st);
  return (int)hipGetLastError();
}

extern "C" int gnn_agg_fwd_queue_words() { return NQ + 1; }

// rowptr / col: the layer-1 CSR of the n output rows; Xs: [*][ldx] bf16 gathered rows
// (D^-1/2 X, zero padding); AX: [n][ldx] bf16 output (the ones column at F); W1 [F][HD],
// b1 [HD], W2 [HD][C] fp32; Z2: [n][ldc] bf16.  ctr: int32[gnn_agg_fwd_queue_words()],
// zero before the first launch (left zero).  Returns -1 when no variant covers the shape.
extern "C" int gnn_launch_agg_fwd(const int* rowptr, const int* col, const void* Xs, void* AX, const float* W1,
                                  const float* b1, const float* W2, const float* dinv, void* Z2, int n, int F,
                                  int ldx, int HD, int C, int ldc, float p, uint32_t k0, uint32_t k1, uint32_t step,
                                  uint32_t row0, const int* stepp, void* kimg, int* ctr, hipStream_t st) {
  if (C > 64 || ldc % 8 || ldx % 8 || ldc > 64 || F + 1 > ldx || ldx > 128 || !ctr) return -3;
  if (n <= 0) return 0;
  const uint32_t thr8 = (uint32_t)std::min(255.0, std::floor((double)p * 256.0 + 0.5));
  const int KS = (F + 15) / 16;
  if (KS * 16 > ldx) return -1;     // the last k-step must lie inside the row pitch
  auto* xs = (const uint16_t*)Xs;
  auto* ax = (uint16_t*)AX;
  auto* z2 = (uint16_t*)Z2;
  auto* ki = (uint16_t*)kimg;
#define AGG(ks, hd, dr)                                                                                          \
  if (KS <= ks && HD == hd)                                                                                       \
    return agg_launch_d<ks, hd, dr, AGG_RPC>(rowptr, col, xs, ax, W1, b1, W2, dinv, z2, n, F, ldx, C, ldc, p, k0,  \
                                             k1, step, thr8, row0, stepp, ki, ctr, st);
  if (thr8 == 128) { AGG(4, 256, 2) AGG(7, 256, 2) AGG(8, 256, 2) AGG(4, 128, 2) AGG(8, 128, 2) }
  else if (thr8 > 0) { AGG(4, 256, 1) AGG(7, 256, 1) AGG(8, 256, 1) AGG(4, 128, 1) AGG(8, 128, 1) }
  else { AGG(4, 256, 0) AGG(7, 256, 0) AGG(8, 256, 0) AGG(4, 128, 0) AGG(8, 128, 0) }
#undef AGG
  return -1;
}
