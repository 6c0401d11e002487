// Level-scheduled generator kernels for wide causal graphs (the reference's random-graph
// generator defaults to 200 variables, generators/random_graph_generator.py:26; CGNN
// builds one MLP per variable for any d, CGNN.py:63-90).
//
// The per-sample kernels of cgnn_kernels.hip walk the whole DAG program in one wave per
// 64..256 samples: at d = 200 that is a 200-node dependent chain per wave, each node
// waiting on its scalar weight loads, with the block's [D][B] sample state limiting a
// CU to 2-3 waves.  Here a block owns ONE 64-sample tile of one model, and its W waves
// share it: the nodes of one topological level are independent, so wave w takes nodes
// w, w + W, ... of the level and the block synchronises once per level.  The dependent
// chain shrinks from d nodes to (#levels x level width / W) and every CU runs 8+ waves.
//
//   gen_noise_kernel       every Philox normal of the step (node noise and confounder
//                          streams) in one fully parallel launch, into `noise`
//                          ([R][NS][N]) -- the same draws, keyed exactly as before.
//   gen_fwd_staged_kernel  forward over the forward stages (= levels); a node's value is
//                          bitwise the per-sample kernel's (same fmaf order).
//   gen_bwd_staged_kernel  backward over the backward sub-stages: levels in reverse,
//                          split so that no two nodes of a sub-stage share a parent --
//                          every dL/dparent push is then owned by one wave and the sums
//                          are in a fixed order (no atomics; bitwise reproducible).  Per
//                          node the wave recomputes the hidden layer in 16-unit chunks and
//                          reduces the parameter gradients over its 64 samples through a
//                          per-wave LDS slab (the item scheme of gen_bwd_kernel).
//
// Sample state: x (and dL/dx in the backward) live in LDS ([Dt][64] each) while they fit,
// otherwise in global memory (xhat itself / the dxs scratch) -- the launcher picks.
// The parameter buffer must extend 64 floats (engine.batch.PARAM_PAD) past its last model (the backward's
// tail-chunk weight loads run past a node's last row and are zeroed).
// The schedule (engine/program.py stage_schedule, built by the C++ runtime):
//   [0] n_fwd_stages [1] n_bwd_stages [2] fwd_base [3] bwd_base
//   at fwd_base: starts[n_fwd + 1], then program record indices; same at bwd_base.
// Blocks are dealt XCD-contiguously (xcd_remap), so the tiles of one model share an
// L2 and its weight stream.
#include "cgnn_common.h"
#include <algorithm>

using namespace cgnn;

namespace {

constexpr int WAVE = 64;
constexpr int HZ = 16;            // hidden units per backward chunk

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(256) void gen_noise_kernel(const int* __restrict__ prog, int ps,
                                                        const uint32_t* __restrict__ keys,
                                                        const int* __restrict__ step_base, int step_off,
                                                        float* __restrict__ noise, int NS, int N, int D, int Dt,
                                                        int row0) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  const int s = blockIdx.y, r = blockIdx.z;
  if (n >= N) return;
  const uint32_t step = (uint32_t)(step_base[0] + step_off);
  const uint32_t k0 = keys[2 * r], k1 = keys[2 * r + 1];
  float* nz = noise + (size_t)r * NS * N;
  if (s < Dt) {
    nz[(size_t)s * N + n] = rng_normal(k0, k1, (uint32_t)(row0 + n), (uint32_t)s, step, RNG_NODE_NOISE);
  } else {
    const int cid = s - Dt;
    if (cid < prog[(size_t)r * ps + 2])
      nz[(size_t)(D + cid) * N + n] = rng_normal(k0, k1, (uint32_t)(row0 + n), (uint32_t)cid, step, RNG_CONF_NOISE);
  }
}

// ---------------------------------------------------------------------------- forward
template <int HC, bool XG, bool DRAW>
__global__ __launch_bounds__(512) void gen_fwd_staged_kernel(
    const int* __restrict__ prog, int ps, const int* __restrict__ sched, int ss,
    const float* __restrict__ params, int P, const float* __restrict__ data, float* __restrict__ xhat,
    float* __restrict__ noise, int NS, float* __restrict__ xnorm, int N, int D, int Dt, int H, int T,
    int max_in, const uint32_t* __restrict__ keys, const int* __restrict__ step_base, int step_off, int row0) {
  // DRAW: the node and confounder noise is drawn here (gen_noise_kernel's draws, keyed
  // the same) as the nodes consume it, and written to `noise` for the backward -- no
  // separate noise launch, no noise read in the forward
  constexpr int HCS = (HC + 3) & ~3;      // weight-slab row stride (16-B aligned rows)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int W = blockDim.x >> 6;
  const int wave = wave_id(), lane = threadIdx.x & 63;
  const int L = (int)xcd_remap(blockIdx.x, gridDim.x);
  const int r = L / T, tile = L - r * T;
  const int n = tile * WAVE + lane;
  const bool valid = n < N;
  const int nc = valid ? n : N - 1;
  // (program and schedule words are scalar loads: staging them in LDS measured slower,
  // 1.87 vs 1.47 ms for the d = 200 backward -- the LDS they take costs a block per CU)
  const int* pg = prog + (size_t)r * ps;
  const int* sc = sched + (size_t)r * ss;
  const float* th = params + (size_t)r * P;
  const float* dr = data + (size_t)r * D * N;
  // DRAW with noise == nullptr (an evaluation step): nothing reads the draws afterwards
  float* nz = noise ? noise + (size_t)r * NS * N : nullptr;
  const bool store = DRAW && noise != nullptr;
  float* xr = xhat + (size_t)r * D * N;
  uint32_t k0 = 0u, k1 = 0u, rstep = 0u;
  if constexpr (DRAW) {
    k0 = keys[2 * r];
    k1 = keys[2 * r + 1];
    rstep = (uint32_t)(step_base[0] + step_off);
  }
  auto own_noise = [&](int var) -> float {
    if constexpr (DRAW) return rng_normal(k0, k1, (uint32_t)(row0 + nc), (uint32_t)var, rstep, RNG_NODE_NOISE);
    else return nz[(size_t)var * N + nc];
  };
  float* s_x = smem;                                        // [Dt][64] (LDS state)
  float* s_w = s_x + (XG ? 0 : (size_t)Dt * WAVE) + (size_t)wave * (max_in + 2) * HCS;   // this wave's weight rows
  auto xget = [&](int v) -> float { return XG ? xr[(size_t)v * N + nc] : s_x[v * WAVE + lane]; };
  auto xput = [&](int v, float val) {
    if (XG) {
      if (valid) xr[(size_t)v * N + n] = val;
    } else {
      s_x[v * WAVE + lane] = val;
    }
  };

  const int nf = uni(sc), fb = uni(sc + 2);
  const int* starts = sc + fb;
  const int* items = starts + nf + 1;
  // software pipeline across a wave's nodes (as the backward): the next chunk's weights,
  // or the next node's first chunk and own noise, load while this chunk computes
  constexpr int WK = 8;                  // prefetched weights per lane: (nin + 2) HC <= 512
  struct Nd { int var, kind, npar, paroff, ncf, cfoff, nin; const float* W1; };
  auto node_at = [&](int idx) -> Nd {
    const int* nd = pg + PROG_HDR + uni(items + idx) * NODE_REC;
    Nd d;
    d.var = uni(nd); d.kind = uni(nd + 1); d.npar = uni(nd + 2); d.paroff = uni(nd + 3);
    d.ncf = uni(nd + 4); d.cfoff = uni(nd + 5);
    d.nin = d.npar + 1 + d.ncf;
    d.W1 = th + max(uni(nd + 6), 0);     // rows 0..nin: W1ext (row nin = b1), row nin + 1: W2
    return d;
  };
  auto load_w = [&](const Nd& d, int q0, float* w) {
    const int nel = (d.nin + 2) * HC;
#pragma unroll
    for (int k = 0; k < WK; ++k) {
      const int e = min(WAVE * k + lane, nel - 1);
      w[k] = d.W1[(e / HC) * H + q0 + e % HC];
    }
  };
  for (int st = 0; st < nf; ++st) {
    const int b = uni(starts + st), e = uni(starts + st + 1);
    float wnx[WK], enx = 0.f;
    if (b + wave < e) {
      const Nd d0 = node_at(b + wave);
      if (d0.kind != KIND_OBS) {
        load_w(d0, 0, wnx);
        enx = own_noise(d0.var);
      }
    }
    for (int i = b + wave; i < e; i += W) {
      const Nd cur = node_at(i);
      const int var = cur.var;
      if (cur.kind == KIND_OBS) {
        xput(var, dr[(size_t)var * N + nc]);
        if (i + W < e) {
          const Nd nx = node_at(i + W);
          if (nx.kind != KIND_OBS) {
            load_w(nx, 0, wnx);
            enx = own_noise(nx.var);
          }
        }
        continue;
      }
      const int npar = cur.npar, paroff = cur.paroff, ncf = cur.ncf, cfoff = cur.cfoff, nin = cur.nin;
      const float* W1 = cur.W1;
      const float e_own = enx;
      if (store && valid) nz[(size_t)var * N + n] = e_own;          // for the backward
      float out = W1[(size_t)(nin + 2) * H];                       // b2
      for (int q0 = 0; q0 < H; q0 += HC) {
        // this chunk's weights (rows 0..nin+1, HC units) into the wave's slab
        const int nel = (nin + 2) * HC;
        float wcur[WK];
#pragma unroll
        for (int k = 0; k < WK; ++k) wcur[k] = wnx[k];
        if (q0 + HC < H) {
          load_w(cur, q0 + HC, wnx);
        } else if (i + W < e) {
          const Nd nx = node_at(i + W);
          if (nx.kind != KIND_OBS) {
            load_w(nx, 0, wnx);
            enx = own_noise(nx.var);
          }
        }
#pragma unroll
        for (int k = 0; k < WK; ++k) {
          const int el = WAVE * k + lane;
          if (el < nel) s_w[(el / HC) * HCS + el % HC] = wcur[k];
        }
        for (int e0 = WK * WAVE; e0 < nel; e0 += 4 * WAVE) {     // very wide nodes: the rest now
          float wv[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int el = min(e0 + WAVE * k + lane, nel - 1);
            wv[k] = W1[(el / HC) * H + q0 + el % HC];
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int el = e0 + WAVE * k + lane;
            if (el < nel) s_w[(el / HC) * HCS + el % HC] = wv[k];
          }
        }
        wave_sync();
        // same per-unit fmaf order as gen_fwd_kernel: own noise + bias, parents, confounders
        float pre[HC];
#pragma unroll
        for (int q = 0; q < HC; ++q) pre[q] = fmaf(s_w[npar * HCS + q], e_own, s_w[nin * HCS + q]);
        // parents then confounder streams, in order; each batch of 8 inputs is loaded
        // before the first use (no load -> wait -> use chain per input)
        for (int j0 = 0; j0 < npar; j0 += 8) {
          float v[8];
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) v[jj] = xget(uni(pg + paroff + min(j0 + jj, npar - 1)));
#pragma unroll
          for (int jj = 0; jj < 8; ++jj)
            if (j0 + jj < npar) {
#pragma unroll
              for (int q = 0; q < HC; ++q) pre[q] = fmaf(s_w[(j0 + jj) * HCS + q], v[jj], pre[q]);
            }
        }
        for (int c0 = 0; c0 < ncf; c0 += 8) {
          float v[8];
          if constexpr (DRAW) {
#pragma unroll
            for (int cc = 0; cc < 8; ++cc) {
              const int cid = uni(pg + cfoff + min(c0 + cc, ncf - 1));
              v[cc] = rng_normal(k0, k1, (uint32_t)(row0 + nc), (uint32_t)cid, rstep, RNG_CONF_NOISE);
              // (the first chunk's pass writes the stream; nodes sharing it write equal values)
              if (store && q0 == 0 && valid && c0 + cc < ncf) nz[(size_t)(D + cid) * N + n] = v[cc];
            }
          } else {
#pragma unroll
            for (int cc = 0; cc < 8; ++cc)
              v[cc] = nz[(size_t)(D + uni(pg + cfoff + min(c0 + cc, ncf - 1))) * N + nc];
          }
#pragma unroll
          for (int cc = 0; cc < 8; ++cc)
            if (c0 + cc < ncf) {
#pragma unroll
              for (int q = 0; q < HC; ++q) pre[q] = fmaf(s_w[(npar + 1 + c0 + cc) * HCS + q], v[cc], pre[q]);
            }
        }
#pragma unroll
        for (int q = 0; q < HC; ++q) out = fmaf(s_w[(nin + 1) * HCS + q], fmaxf(pre[q], 0.f), out);
        wave_sync();                           // slab reads done before the next chunk's writes
      }
      xput(var, out);
    }
    __syncthreads();
  }

  if (!XG && valid)
    for (int v = wave; v < Dt; v += W) xr[(size_t)v * N + n] = s_x[v * WAVE + lane];
  if (xnorm && wave == 0) {
    // squared norm for the Gram-form MMD: one fmaf chain over the program positions in
    // order -- the per-sample kernel's order, whatever W (the block width follows the
    // widest stage of any program in the batch, so a W-dependent order would make a
    // model's loss depend on its batch-mates)
    const int nn = uni(pg);
    float nrm = 0.f;
    for (int k0 = 0; k0 < nn; k0 += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = xget(uni(pg + PROG_HDR + min(k0 + u, nn - 1) * NODE_REC));
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k0 + u < nn) nrm = fmaf(v[u], v[u], nrm);
    }
    if (valid) xnorm[(size_t)r * N + n] = nrm;
  }
}

// --------------------------------------------------------------------------- backward
// per-wave LDS slab (floats)
__host__ __device__ __forceinline__ int bwd_si(int max_in) { return (max_in + 2) | 1; }
// CW: hidden units per backward chunk (the compute width; the weight rows stay HZ = 16
// wide).  12 when it takes as many chunks as 16 (H <= 12, 17..24, 33..36): H = 20 runs
// 12 + 8 units of work instead of 16 + 16.
__host__ __device__ __forceinline__ int bwd_cw(int H) { return (H + 11) / 12 == (H + 15) / 16 ? 12 : 16; }
// parents whose dL/dparent partials a lane keeps in registers (PPR kernels): nodes of at
// most PPR_MAX parents, i.e. max_in <= PPR_MAX + 1 (an input is the own noise)
constexpr int PPR_MAX = 16;
__host__ __device__ __forceinline__ bool bwd_ppr(int max_in) { return max_in <= PPR_MAX + 1; }
__host__ __device__ __forceinline__ int bwd_slab(int max_in, int cw) {
  // [64][SI] (padded even) + [64][cw + 2] mg rows + weight rows (+ dL/dparent partials,
  // unless they live in registers: d = 200 with 400 edges (max_in 11) 12.6 -> 9.8 KB per
  // wave, 3 -> 4 four-wave blocks per CU; with 736 edges (max_in 17) 16.4 -> 12.1 KB,
  // 2 -> 3 blocks; without the Gm rows (dW2 from the MFMA registers) and with 14-float mg
  // rows at cw = 12: 9.7 KB, 4 blocks)
  return WAVE * (bwd_si(max_in) + 1) + WAVE * (cw + 2) + (max_in + 2) * HZ + (bwd_ppr(max_in) ? 0 : max_in * WAVE);
}


template <bool XG, bool DG, bool PPR, int CW>
__global__ __launch_bounds__(512) void gen_bwd_staged_kernel(
    const int* __restrict__ prog, int ps, const int* __restrict__ sched, int ss,
    const float* __restrict__ params, int P, const float* __restrict__ xhat, const float* __restrict__ noise,
    int NS, const float* __restrict__ grad_part, int n_chunks, int R, int N, int D, int Dt, int H, int max_in,
    int T, float* __restrict__ gpart, float* __restrict__ dxs) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int W = blockDim.x >> 6;
  const int wave = wave_id(), lane = threadIdx.x & 63;
  const int L = (int)xcd_remap(blockIdx.x, gridDim.x);
  const int r = L / T, tile = L - r * T;
  const int n = tile * WAVE + lane;
  const bool valid = n < N;
  const int nc = valid ? n : N - 1;
  const int* pg = prog + (size_t)r * ps;
  const int* sc = sched + (size_t)r * ss;
  const float* th = params + (size_t)r * P;
  const float* xr = xhat + (size_t)r * D * N;
  const float* nz = noise + (size_t)r * NS * N;
  float* dx = dxs + (size_t)r * Dt * N;
  float* gp = gpart + ((size_t)r * T + tile) * P;
  const int SI = bwd_si(max_in);
  float* s_x = smem;
  float* s_dx = s_x + (XG ? 0 : (size_t)Dt * WAVE);
  constexpr int ZC = CW + 2;                                 // mg row stride (even: f2 pairs)
  float* slab = s_dx + (DG ? 0 : (size_t)Dt * WAVE) + (size_t)wave * bwd_slab(max_in, CW);
  float* s_in = slab;                                        // [64][SI]
  float* s_z = slab + WAVE * (SI + 1);                       // [64][ZC]
  float* s_w = s_z + WAVE * ZC;                              // [max_in + 2][16] weight rows
  float* s_pp = s_w + (max_in + 2) * HZ;                     // [max_in][64] dL/dparent (!PPR)
  float pp[PPR ? PPR_MAX : 1];                                // dL/dparent (PPR)
  float* my_in = s_in + lane * SI;
  float* my_z = s_z + lane * ZC;

  auto xget = [&](int v) -> float { return XG ? xr[(size_t)v * N + nc] : s_x[v * WAVE + lane]; };

  // sample state: x and dL/dx = fixed-order sum of the MMD gradient chunks
  for (int v = wave; v < Dt; v += W) {
    float s = 0.f;
    if (valid)
      for (int c = 0; c < n_chunks; ++c) s += grad_part[(((size_t)c * R + r) * D + v) * N + n];
    if (DG) {
      if (valid) dx[(size_t)v * N + n] = s;
    } else {
      s_dx[v * WAVE + lane] = s;
    }
    if (!XG) s_x[v * WAVE + lane] = valid ? xr[(size_t)v * N + n] : 0.f;
  }
  __syncthreads();

  const int nb = uni(sc + 1), bb = uni(sc + 3);
  const int* starts = sc + bb;
  const int* items = starts + nb + 1;

  // ---- software pipeline across a wave's nodes: while a node's chunk computes, the
  // loads of the next chunk's weights (or of the next node's first chunk, its first 8
  // inputs and its dL/dx) are in flight.  Within a sub-stage no node writes another's
  // dL/dx (only parents, which sit at lower levels), so the next node's is final. ----
  struct Nd { int var, npar, paroff, ncf, nin; const float* W1; };
  auto node_at = [&](int idx) -> Nd {
    const int* nd = pg + PROG_HDR + uni(items + idx) * NODE_REC;
    Nd d;
    d.var = uni(nd); d.npar = uni(nd + 2); d.paroff = uni(nd + 3); d.ncf = uni(nd + 4);
    d.nin = d.npar + 1 + d.ncf;
    d.W1 = th + uni(nd + 6);               // rows 0..nin: W1ext (row nin = b1), row nin + 1: W2
    return d;
  };
  // weights of one chunk, rows 0..nin+1 x 16 units: elements 64 k + lane (the first 256)
  auto load_w = [&](const Nd& d, int q0, float* w) {
    const int nel = (d.nin + 2) * HZ;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = min(WAVE * k + lane, nel - 1);
      w[k] = d.W1[(e >> 4) * H + q0 + (e & 15)];   // tail units read past the row (padded)
    }
  };
  // inputs j0..j0+7 of a node: the pool holds the parents then the confounder ids
  // (cf_off = par_off + n_par), so input j != n_par is pool entry par_off + j (- 1 past
  // the own noise); every load is in bounds and the unused ones are discarded
  auto load_in = [&](const Nd& d, int j0, float* v) {
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int j = min(j0 + jj, d.nin - 1);
      const int pe = uni(pg + d.paroff + (j < d.npar ? j : j - 1));
      const int row = j < d.npar ? pe : (j == d.npar ? d.var : D + pe);
      if (XG) {
        const float* base = j < d.npar ? xr : nz;
        v[jj] = base[(size_t)row * N + nc];
      } else {
        const float xa = s_x[(j < d.npar ? pe : 0) * WAVE + lane];
        const float xb = nz[(size_t)row * N + nc];
        v[jj] = j < d.npar ? xa : xb;
      }
    }
  };
  auto load_g = [&](const Nd& d) -> float { return DG ? dx[(size_t)d.var * N + nc] : s_dx[d.var * WAVE + lane]; };

  for (int st = 0; st < nb; ++st) {
    const int b = uni(starts + st), e = uni(starts + st + 1);
    float wnx[4], vnx[8], gnx = 0.f;
    if (b + wave < e) {
      const Nd d0 = node_at(b + wave);
      load_w(d0, 0, wnx);
      load_in(d0, 0, vnx);
      gnx = load_g(d0);
    }
    for (int i = b + wave; i < e; i += W) {
      const Nd cur = node_at(i);
      const int var = cur.var, npar = cur.npar, paroff = cur.paroff, nin = cur.nin;
      const float* W1 = cur.W1;
      const int poff = (int)(W1 - th);
      // input row: the first 8 inputs and dL/dx were prefetched; the rest load now
#pragma unroll
      for (int jj = 0; jj < 8; ++jj)
        if (jj < nin) my_in[jj] = vnx[jj];
      for (int j0 = 8; j0 < nin; j0 += 8) {
        float v[8];
        load_in(cur, j0, v);
#pragma unroll
        for (int jj = 0; jj < 8; ++jj)
          if (j0 + jj < nin) my_in[j0 + jj] = v[jj];
      }
      my_in[nin] = 1.f;
      const float gout = valid ? gnx : 0.f;

      for (int q0 = 0; q0 < H; q0 += CW) {
        const int hc = min(CW, H - q0);
        // ---- this chunk's weights into the slab (units q >= hc of a tail chunk zeroed),
        // then the next loads go out ----
        const int nel = (nin + 2) * HZ;
        float wcur[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) wcur[k] = wnx[k];
        if (q0 + CW < H) {
          load_w(cur, q0 + CW, wnx);
        } else if (i + W < e) {
          const Nd nx = node_at(i + W);
          load_w(nx, 0, wnx);
          load_in(nx, 0, vnx);
          gnx = load_g(nx);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int el = WAVE * k + lane;
          if (el < nel) s_w[el] = (el & 15) < hc ? wcur[k] : 0.f;
        }
        for (int e0 = 4 * WAVE; e0 < nel; e0 += 4 * WAVE) {       // nin > 14: the rest now
          float wv[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int el = min(e0 + WAVE * k + lane, nel - 1);
            wv[k] = W1[(el >> 4) * H + q0 + (el & 15)];
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int el = e0 + WAVE * k + lane;
            if (el < nel) s_w[el] = (el & 15) < hc ? wv[k] : 0.f;
          }
        }
        wave_sync();
        // ---- the chunk's recompute and dL/dparent share (a 4-wide path for tail chunks
        // of <= 4 units measured slower: its registers cost the occupancy,
        // profiles/r05_cgnn_bwd) ----
        {
          static_assert(CW % 4 == 0 && CW <= HZ, "chunk width");
          auto wrow = [&](int row, float* w) {      // CW weights of a row (LDS broadcast)
#pragma unroll
            for (int c = 0; c < CW / 4; ++c) {
              const float4 v4 = *reinterpret_cast<const float4*>(s_w + row * HZ + 4 * c);
              w[4 * c] = v4.x; w[4 * c + 1] = v4.y; w[4 * c + 2] = v4.z; w[4 * c + 3] = v4.w;
            }
          };
          // recompute this chunk's pre-activations (one sample per lane)
          float pre[CW], w[CW], w2[CW];
          wrow(nin, pre);
          for (int j = 0; j < nin; ++j) {
            const float x = my_in[j];
            wrow(j, w);
#pragma unroll
            for (int q = 0; q < CW; ++q) pre[q] = fmaf(w[q], x, pre[q]);
          }
          float mg[CW];
#pragma unroll
          for (int q = 0; q < CW; ++q) mg[q] = (q < hc && pre[q] > 0.f) ? gout : 0.f;
          // this chunk's share of dL/dparent, kept until the node ends
          wrow(nin + 1, w2);
          if constexpr (PPR) {
#pragma unroll
            for (int j = 0; j < PPR_MAX; ++j)
              if (j < npar) {                  // wave-uniform
                wrow(j, w);
                float s = 0.f;
#pragma unroll
                for (int q = 0; q < CW; ++q) s = fmaf(w[q] * w2[q], mg[q], s);
                pp[j] = q0 == 0 ? s : pp[j] + s;
              }
          } else {
            for (int j = 0; j < npar; ++j) {
              wrow(j, w);
              float s = 0.f;
#pragma unroll
              for (int q = 0; q < CW; ++q) s = fmaf(w[q] * w2[q], mg[q], s);
              s_pp[j * WAVE + lane] = q0 == 0 ? s : s_pp[j * WAVE + lane] + s;
            }
          }
#pragma unroll
          for (int qp = 0; qp < CW / 2; ++qp) *reinterpret_cast<f2*>(my_z + 2 * qp) = f2{mg[2 * qp], mg[2 * qp + 1]};
        }
        wave_sync();

        // ---- Gm[j][q] = sum_s in[s][j] mg[s][q] over the 64 samples on the matrix cores
        // (v_mfma_f32_16x16x4_f32: fp32 products, fp32 accumulation): A = in^T (16 input
        // rows x 4 samples, from the input slab), B = mg (4 samples x 16 units, from the
        // mg slab; columns >= CW read the next row and are discarded), 16 k-steps for the
        // tile's 64 samples; D = 16 input rows x 16 units (lane 16 g + c: rows 4 g .. 4 g + 3,
        // unit c).  dW1 / db1 = w2 Gm straight from the accumulators, and dW2[q] =
        // sum_j W1ext[j][q] Gm[j][q] as per-lane partials over the lane's rows, summed over
        // the four row groups by two cross-lane adds (no Gm rows in LDS). ----
        {
          typedef float f32x4 __attribute__((ext_vector_type(4)));
          const int jq = lane & 15, sg = lane >> 4;
          const float w2q = s_w[(nin + 1) * HZ + jq];
          float d2 = 0.f;
          for (int j0 = 0; j0 <= nin; j0 += 16) {
            const int jr = min(j0 + jq, nin);
            const float am = j0 + jq <= nin ? 1.f : 0.f;
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
            for (int t = 0; t < WAVE / 4; ++t) {
              const int smp = 4 * t + sg;
              const float a = s_in[smp * SI + jr] * am;
              const float b = s_z[smp * ZC + jq];
              acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int j = j0 + 4 * sg + i;
              if (j <= nin) {
                d2 = fmaf(s_w[j * HZ + jq], acc[i], d2);
                if (jq < hc) gp[poff + j * H + q0 + jq] = w2q * acc[i];   // dW1 / db1
              }
            }
          }
          d2 += __shfl_xor(d2, 16, 64);
          d2 += __shfl_xor(d2, 32, 64);
          if (lane < hc) gp[poff + (nin + 1) * H + q0 + lane] = d2;       // dW2
        }
        wave_sync();
      }
      // ---- push dL/dparent (each parent is this wave's alone in the sub-stage) ----
      auto push = [&](int j0, auto part) {
        float cur[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const int pv = uni(pg + paroff + min(j0 + jj, npar - 1));
          cur[jj] = DG ? dx[(size_t)pv * N + nc] : s_dx[pv * WAVE + lane];
        }
#pragma unroll
        for (int jj = 0; jj < 8; ++jj)
          if (j0 + jj < npar) {
            const int pv = uni(pg + paroff + j0 + jj);
            const float v = cur[jj] + part(jj);
            if (DG) {
              if (valid) dx[(size_t)pv * N + n] = v;
            } else {
              s_dx[pv * WAVE + lane] = v;
            }
          }
      };
      if constexpr (PPR) {
        // static register indices: batches at 0 and 8 (PPR_MAX = 16)
        if (npar > 0) push(0, [&](int jj) { return pp[jj]; });
        if (npar > 8) push(8, [&](int jj) { return 8 + jj < PPR_MAX ? pp[(8 + jj) % PPR_MAX] : 0.f; });
      } else {
        for (int j0 = 0; j0 < npar; j0 += 8) push(j0, [&](int jj) { return s_pp[(j0 + jj) * WAVE + lane]; });
      }
      const float g2 = wave_sum(gout);                               // db2
      if (lane == 0) gp[poff + (nin + 2) * H] = g2;
    }
    __syncthreads();
  }
}

template <typename K>
void allow_lds(K kernel, size_t lds) {
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
}

constexpr size_t LDS_MAX = 160 * 1024;

int fwd_hc(int H) {
  static const int cand[] = {32, 20, 16, 12, 10, 8, 6, 5, 4, 3, 2, 1};
  for (int c : cand)
    if (H % c == 0) return c;
  return 1;
}

// extra: program + schedule ints staged in LDS
size_t fwd_lds(int Dt, int W, bool xg, int max_in, int hc, int extra) {
  const size_t hcs = (size_t)((hc + 3) & ~3);
  return sizeof(float) * ((size_t)extra + (xg ? 0 : (size_t)Dt * WAVE) + (size_t)W * (max_in + 2) * hcs);
}
size_t bwd_lds(int Dt, int W, int H, int max_in, bool xg, bool dg, int extra) {
  return sizeof(float) * ((size_t)extra + (xg ? 0 : (size_t)Dt * WAVE) + (dg ? 0 : (size_t)Dt * WAVE) +
                          (size_t)W * bwd_slab(max_in, bwd_cw(H)));
}


}  // namespace

// Plan of the staged kernels for Dt variables, hidden width H, max_in generator inputs
// and W waves per block (1..8): out = {fwd_xg, bwd_xg, bwd_dg, W_fwd, W_bwd}.  Returns 0,
// or -1 when even the all-global variant does not fit (only for absurd max_in).
// extra: further LDS ints per block (0 in the current kernels)
extern "C" int cgnn_staged_plan(int Dt, int H, int max_in, int W, int extra, int* out) {
  if (Dt < 1 || H < 1 || W < 1 || W > 8 || extra < 0) return -1;
  if (fwd_lds(Dt, W, true, max_in, fwd_hc(H), extra) > LDS_MAX) return -1;
  const int fxg = fwd_lds(Dt, W, false, max_in, fwd_hc(H), extra) <= LDS_MAX ? 0 : 1;
  // backward: latency-bound per node, so the placement that keeps the most waves per CU
  // resident wins (d = 200, H = 20: sample state in LDS at 4 waves / CU 3.76 ms, in
  // global memory at 16 waves / CU 1.59 ms; profiles/r04_cgnn_wide), at most 2 waves
  // per block (wider blocks idle on the narrow sub-stages: d = 200, H = 20 backward with
  // 1 / 2 / 4 / 8 waves per block 1421 / 995 / 1068 / 1282 us at 400 edges, 1598 / 1181 /
  // 1447 / 2121 us at 736; profiles/r05_cgnn_bwd/wsweep); ties keep the LDS state.
  // Nodes with many inputs (a slab per wave grows with max_in) take narrower blocks
  // before giving up: 2, then 1 wave per block.
  const int cap = 16;                    // ~110 VGPRs: 4 waves per SIMD
  int best = -1, best_waves = 0, wb = std::min(W, 2);
  for (; wb >= 1 && best < 0; wb /= 2) {
    for (int place = 0; place < 3; ++place) {
      const size_t lds = bwd_lds(Dt, wb, H, max_in, place >= 1, place == 2, extra);
      if (lds > LDS_MAX) continue;
      const int waves = std::min(cap, (int)(LDS_MAX / lds) * wb);
      if (waves > best_waves) { best = place; best_waves = waves; }
    }
    if (best >= 0) break;
  }
  if (best < 0) return -1;
  out[0] = fxg; out[1] = best >= 1; out[2] = best == 2; out[3] = W; out[4] = wb;
  return 0;
}

extern "C" int cgnn_staged_tiles(int N) { return (N + WAVE - 1) / WAVE; }

extern "C" int cgnn_launch_gen_noise(const int* prog, int ps, const uint32_t* keys, const int* step_base,
                                     int step_off, float* noise, int NS, int N, int D, int Dt, int R, int row0,
                                     hipStream_t st) {
  if (NS < D || Dt > D) return -2;
  dim3 grid((N + 255) / 256, Dt + (NS - D), R), block(256);
  hipLaunchKernelGGL(gen_noise_kernel, grid, block, 0, st, prog, ps, keys, step_base, step_off, noise, NS, N, D,
                     Dt, row0);
  return (int)hipGetLastError();
}

// forward of R models.  keys == nullptr: the noise was drawn (gen_noise); else the
// forward draws it itself (keys, step_base[0] + step_off, row0: gen_noise's keying) and
// writes it to `noise` for the backward (noise == nullptr: not stored).  W waves per block (1..8).  force: -1 the
// plan's state placement, 0 LDS, 1 global (tests: every placement is bitwise the same)
extern "C" int cgnn_launch_gen_fwd_staged_draw(const int* prog, int ps, const int* sched, int ss, const float* params,
                                               int P, const float* data, float* xhat, float* noise, int NS,
                                               float* xnorm, int N, int D, int Dt, int H, int max_in, int R, int W,
                                               hipStream_t st, int force, const uint32_t* keys, const int* step_base,
                                               int step_off, int row0) {
  int plan[5];
  if (cgnn_staged_plan(Dt, H, max_in, W, 0, plan) != 0) return -2;
  const int hc = fwd_hc(H);
  const bool xg = force < 0 ? plan[0] != 0 : force == 1;
  if (fwd_lds(Dt, W, xg, max_in, hc, 0) > LDS_MAX) return -2;
  const int T = cgnn_staged_tiles(N);
  const size_t lds = fwd_lds(Dt, W, xg, max_in, hc, 0);
  dim3 grid((unsigned)(T * R)), block(WAVE * W);
#define FWD(HC, XG)                                                                                           \
  {                                                                                                           \
    if (keys) {                                                                                               \
      allow_lds(gen_fwd_staged_kernel<HC, XG, true>, lds);                                                    \
      hipLaunchKernelGGL((gen_fwd_staged_kernel<HC, XG, true>), grid, block, lds, st, prog, ps, sched, ss,    \
                         params, P, data, xhat, noise, NS, xnorm, N, D, Dt, H, T, max_in, keys, step_base,     \
                         step_off, row0);                                                                     \
    } else {                                                                                                  \
      allow_lds(gen_fwd_staged_kernel<HC, XG, false>, lds);                                                   \
      hipLaunchKernelGGL((gen_fwd_staged_kernel<HC, XG, false>), grid, block, lds, st, prog, ps, sched, ss,   \
                         params, P, data, xhat, noise, NS, xnorm, N, D, Dt, H, T, max_in, keys, step_base,     \
                         step_off, row0);                                                                     \
    }                                                                                                         \
  }
#define FWD_HC(HC) case HC: if (xg) FWD(HC, true) else FWD(HC, false) break;
  switch (fwd_hc(H)) {
    FWD_HC(32) FWD_HC(20) FWD_HC(16) FWD_HC(12) FWD_HC(10) FWD_HC(8) FWD_HC(6) FWD_HC(5) FWD_HC(4) FWD_HC(3)
    FWD_HC(2) FWD_HC(1)
    default: return -1;
  }
#undef FWD_HC
#undef FWD
  return (int)hipGetLastError();
}

extern "C" int cgnn_launch_gen_fwd_staged(const int* prog, int ps, const int* sched, int ss, const float* params,
                                          int P, const float* data, float* xhat, const float* noise, int NS,
                                          float* xnorm, int N, int D, int Dt, int H, int max_in, int R, int W,
                                          hipStream_t st, int force) {
  return cgnn_launch_gen_fwd_staged_draw(prog, ps, sched, ss, params, P, data, xhat, const_cast<float*>(noise), NS,
                                         xnorm, N, D, Dt, H, max_in, R, W, st, force, nullptr, nullptr, 0, 0);
}

// backward: gpart [R][T][P] (T = cgnn_staged_tiles(N)); dxs [R][Dt][N] is needed when the
// plan puts dL/dx in global memory (plan[2]).  force: -1 the plan, 0 x and dL/dx in LDS,
// 1 x global, 2 both global (tests: every placement is bitwise the same)
extern "C" int cgnn_launch_gen_bwd_staged(const int* prog, int ps, const int* sched, int ss, const float* params,
                                          int P, const float* xhat, const float* noise, int NS, const float* gradp,
                                          int n_chunks, int R, int N, int D, int Dt, int H, int max_in, int W,
                                          float* gpart, float* dxs, hipStream_t st, int force) {
  int plan[5];
  if (cgnn_staged_plan(Dt, H, max_in, W, 0, plan) != 0) return -2;
  bool xg = plan[1] != 0, dg = plan[2] != 0;
  int wb = plan[4];
  if (force >= 0) {
    xg = force >= 1;
    dg = force == 2;
    wb = W;
    if (bwd_lds(Dt, wb, H, max_in, xg, dg, 0) > LDS_MAX) return -2;
  }
  if (dg && !dxs) return -2;
  const int T = cgnn_staged_tiles(N);
  const size_t lds = bwd_lds(Dt, wb, H, max_in, xg, dg, 0);
  dim3 grid((unsigned)(T * R)), block(WAVE * wb);
#define BWD(XG, DG, PPR, CW)                                                                                        \
  {                                                                                                               \
    allow_lds(gen_bwd_staged_kernel<XG, DG, PPR, CW>, lds);                                                       \
    hipLaunchKernelGGL((gen_bwd_staged_kernel<XG, DG, PPR, CW>), grid, block, lds, st, prog, ps, sched, ss, params, \
                       P, xhat, noise, NS, gradp, n_chunks, R, N, D, Dt, H, max_in, T, gpart, dxs);               \
  }
#define BWD_P(PPR, CW)                     \
  if (!xg) BWD(false, false, PPR, CW)      \
  else if (!dg) BWD(true, false, PPR, CW)  \
  else BWD(true, true, PPR, CW)
#define BWD_C(PPR)                  \
  if (bwd_cw(H) == 12) BWD_P(PPR, 12) \
  else BWD_P(PPR, 16)
  if (bwd_ppr(max_in)) BWD_C(true)
  else BWD_C(false)
#undef BWD_C
#undef BWD_P
#undef BWD
  return (int)hipGetLastError();
}
