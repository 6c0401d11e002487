// K6: random-Fourier-feature MMD ("Fast MMD", Loss.py:35-56), batched over R
// models, frequencies redrawn every step from Philox.
//
// Reference semantics reproduced exactly (including SURVEY §2.6 B12):
//   W in R^{(d+1) x 7k}: for bandwidth block b (k features each)
//       omega_f = 2*gamma_b * N(0, I_d),   phase_f ~ U(0, 2*pi)
//   phi(x)_f  = sqrt(2/k) * mean_n cos(omega_f . x_n + phase_f)
//   loss      = sum_f (phi(true)_f - phi(pred)_f)^2
// Gradient wrt a generated sample p_n:
//   dL/dp_n = sum_f 2 (phi_pred_f - phi_true_f) * sqrt(2/k)/N * (-sin(omega_f.p_n + phase_f)) omega_f
//
// Layouts: W [R][F][D+1] (D frequencies then the phase), diff [R][F],
// data/xhat [R][D][N], grad -> chunk 0 of the MMD gradient buffer [1][R][D][N].
//
// Default: matrix-core kernels (below); the vector kernels (one feature / one sample
// per thread) remain for W images too large for LDS (and for A/B, force_valu).
#include "cgnn_common.h"
#include <cstdlib>

using namespace cgnn;

namespace {
__device__ const float kGammas[7] = {0.005f, 0.05f, 0.25f, 0.5f, 1.f, 5.f, 50.f};

__device__ __forceinline__ float cos_rev(float x_rad) {
  // v_cos_f32 takes revolutions; reduce to [0,1) first for full-range accuracy
  float u = x_rad * 0.15915494309189535f;
  return __builtin_amdgcn_cosf(__builtin_amdgcn_fractf(u));
}
__device__ __forceinline__ float sin_rev(float x_rad) {
  float u = x_rad * 0.15915494309189535f;
  return __builtin_amdgcn_sinf(__builtin_amdgcn_fractf(u));
}
}  // namespace

__global__ void rff_freqs_kernel(float* __restrict__ W, const uint32_t* __restrict__ keys,
                                 const int* __restrict__ step_base, int step_off, int k, int D,
                                 int n_gamma, int d_true) {
  const int r = blockIdx.y;
  const int F = k * n_gamma;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;   // over F*(D+1)
  if (idx >= F * (D + 1)) return;
  const int f = idx / (D + 1), dd = idx - f * (D + 1);
  const uint32_t step = (uint32_t)step_base[0] + (uint32_t)step_off;
  // padded feature dims get zero frequency; the phase uses counter word d_true
  // so that the draw does not depend on the padding (matches the CPU oracle)
  const uint32_t cw = dd < D ? (uint32_t)dd : (uint32_t)d_true;
  u32x4 c = {(uint32_t)f, cw, step, RNG_RFF_FREQ};
  u32x4 rnd = philox4x32_10(c, keys[2 * r], keys[2 * r + 1]);
  float val;
  if (dd < d_true) val = 2.f * kGammas[f / k] * normal_from(rnd);
  else if (dd < D) val = 0.f;
  else val = 6.283185307179586f * u01(rnd.z);
  W[((size_t)r * F + f) * (D + 1) + dd] = val;
}

// per-feature means of cos for pred and true; diff_f = phi_pred - phi_true
template <int D>
__global__ __launch_bounds__(256) void rff_feat_kernel(const float* __restrict__ xhat,
                                                       const float* __restrict__ data,
                                                       const float* __restrict__ W,
                                                       float* __restrict__ diff,
                                                       float* __restrict__ loss_part, int N, int F,
                                                       float norm) {
  __shared__ float s_red[4];
  const int r = blockIdx.y;
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = f < F;
  float w[D + 1];
  const float* wf = W + ((size_t)r * F + (valid ? f : 0)) * (D + 1);
#pragma unroll
  for (int k = 0; k <= D; ++k) w[k] = wf[k];
  const float* P = xhat + (size_t)r * D * N;
  const float* T = data + (size_t)r * D * N;
  float sp = 0.f, st = 0.f;
  for (int n = 0; n < N; ++n) {   // sample index is wave-uniform -> scalar loads
    float ap = w[D], at = w[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      ap = fmaf(w[k], P[(size_t)k * N + n], ap);
      at = fmaf(w[k], T[(size_t)k * N + n], at);
    }
    sp += cos_rev(ap);
    st += cos_rev(at);
  }
  const float dlt = valid ? norm * (sp - st) / (float)N : 0.f;
  if (valid) diff[(size_t)r * F + f] = dlt;
  float v = wave_sum(dlt * dlt);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0)
    loss_part[(size_t)r * gridDim.x + blockIdx.x] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
}

template <int D>
__global__ __launch_bounds__(256) void rff_grad_kernel(const float* __restrict__ xhat,
                                                       const float* __restrict__ W,
                                                       const float* __restrict__ diff,
                                                       float* __restrict__ grad, int N, int F,
                                                       float coef) {
  const int r = blockIdx.y;
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const float* P = xhat + (size_t)r * D * N;
  float p[D], g[D];
#pragma unroll
  for (int k = 0; k < D; ++k) { p[k] = P[(size_t)k * N + n]; g[k] = 0.f; }
  const float* Wr = W + (size_t)r * F * (D + 1);
  const float* dr = diff + (size_t)r * F;
  for (int f = 0; f < F; ++f) {   // feature index is wave-uniform
    const float* wf = Wr + (size_t)f * (D + 1);
    float a = wf[D];
#pragma unroll
    for (int k = 0; k < D; ++k) a = fmaf(wf[k], p[k], a);
    const float s = -coef * dr[f] * sin_rev(a);
#pragma unroll
    for (int k = 0; k < D; ++k) g[k] = fmaf(s, wf[k], g[k]);
  }
  float* gr = grad + (size_t)r * D * N;
#pragma unroll
  for (int k = 0; k < D; ++k) gr[(size_t)k * N + n] = g[k];
}

// ============================================================================
// Matrix-core K6: the projections theta = [x | 1] W^T run on the exact-fp32
// matrix cores (v_mfma_f32_32x32x2_f32, the same bits as an fmaf chain), so the VALU
// only evaluates the cos / sin epilogue while the next tile's MFMAs issue.
//
// Forward: wave w of the block owns the 32 features f0 + [0, 32) (8 waves = 256
// features per block, the partial layout of rff_feat_kernel).  Per 32-sample tile:
// C[n][f] = sum_k A[n][k] B[k][f], A = [x | 1] (lane: sample n = l & 31, k = 2s + l/32,
// coalesced along n in the [D][N] layout), B = W^T held in registers for the whole
// loop; the lane then owns 16 samples of ONE feature, so the column means are
// in-register sums + one cross-half shuffle.
// ============================================================================
template <int D>
__global__ __launch_bounds__(512) void rff_mfma_feat_kernel(const float* __restrict__ xhat,
                                                            const float* __restrict__ data,
                                                            const float* __restrict__ W,
                                                            float* __restrict__ diff,
                                                            float* __restrict__ loss_part, int N, int F,
                                                            float norm) {
  constexpr int KS = (D + 2) / 2;          // k-steps of 2 over the D + 1 columns of [x | 1]
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  __shared__ float s_red[8];
  const int r = blockIdx.y;
  const int lane = threadIdx.x & 63, h = lane >> 5, lr = lane & 31, wv = threadIdx.x >> 6;
  const int f = (blockIdx.x * 8 + wv) * 32 + lr;
  const bool fv = f < F;
  const float* wf = W + ((size_t)r * F + (fv ? f : 0)) * (D + 1);
  float bw[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 2 * s + h;
    bw[s] = (fv && k <= D) ? wf[k] : 0.f;
  }
  float sums[2];
#pragma unroll
  for (int part = 0; part < 2; ++part) {
    const float* X = (part == 0 ? xhat : data) + (size_t)r * D * N;
    float acc = 0.f;
    for (int n0 = 0; n0 < N; n0 += 32) {
      const int n = n0 + lr;
      f32x16 c = {};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int k = 2 * s + h;
        const float a = n < N ? (k < D ? X[(size_t)k * N + n] : (k == D ? 1.f : 0.f)) : 0.f;
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bw[s], c, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int nn = n0 + (q & 3) + 8 * (q >> 2) + 4 * h;
        acc += nn < N ? cos_rev(c[q]) : 0.f;
      }
    }
    sums[part] = acc + __shfl_xor(acc, 32, 64);
  }
  const float dlt = fv ? norm * (sums[0] - sums[1]) / (float)N : 0.f;
  if (fv && h == 0) diff[(size_t)r * F + f] = dlt;
  float v = (h == 0) ? dlt * dlt : 0.f;
  v = wave_sum(v);
  if (lane == 0) s_red[wv] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) t += s_red[w];
    loss_part[(size_t)r * gridDim.x + blockIdx.x] = t;
  }
}

// Gradient: wave w owns the 32 samples n0 + [0, 32); over every 32-feature tile,
//   C'[f][n] = sum_k W[f][k] [x | 1][k][n]        (A = W rows, B = this tile's samples)
//   S'[f][n] = -coef diff_f sin(C'[f][n])          (in the accumulator registers)
//   G[k][n] += sum_f W^T[k][f] S'[f][n]            (k-step q takes register q of every
//                                                    lane as B: f = (q&3) + 8(q>>2) + 4(l/32)
//                                                    -- the accumulator IS the operand)
// W of the model is staged in LDS, FC features at a time (the whole [F][D + 1] matrix for
// narrow joints; chunks of it for wide ones -- the f order of the accumulation is the
// same either way).
template <int D>
__global__ __launch_bounds__(256) void rff_mfma_grad_kernel(const float* __restrict__ xhat,
                                                            const float* __restrict__ W,
                                                            const float* __restrict__ diff,
                                                            float* __restrict__ grad, int N, int F,
                                                            float coef, int FC) {
  constexpr int KS = (D + 2) / 2;
  constexpr int DT = (D + 31) / 32;        // 32-row tiles of the gradient's k (feature dim)
  constexpr int WS = D + 1;
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  extern __shared__ float sW[];            // [FC][WS] then diff [FC]
  float* sD = sW + (size_t)FC * WS;
  const int r = blockIdx.y;
  const float* Wr = W + (size_t)r * F * WS;
  const int lane = threadIdx.x & 63, h = lane >> 5, lr = lane & 31, wv = threadIdx.x >> 6;
  const int n0 = (blockIdx.x * 4 + wv) * 32;
  const bool active = n0 < N;               // waves past N still join every barrier
  const int n = n0 + lr;
  const float* X = xhat + (size_t)r * D * N;
  float xb[KS];                             // B of the first product: [x | 1][k = 2s + h][n]
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 2 * s + h;
    xb[s] = n < N ? (k < D ? X[(size_t)k * N + n] : (k == D ? 1.f : 0.f)) : 0.f;
  }
  f32x16 g[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) g[t] = f32x16{};
  for (int fc0 = 0; fc0 < F; fc0 += FC) {
    const int fcn = min(FC, F - fc0);
    __syncthreads();
    for (int i = threadIdx.x; i < fcn * WS; i += blockDim.x) sW[i] = Wr[(size_t)fc0 * WS + i];
    for (int i = threadIdx.x; i < fcn; i += blockDim.x) sD[i] = -coef * diff[(size_t)r * F + fc0 + i];
    __syncthreads();
    if (!active) continue;
    for (int f0 = 0; f0 < fcn; f0 += 32) {
      const int fa = f0 + lr;               // this lane's A row of the first product (chunk-local)
      f32x16 c = {};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int k = 2 * s + h;
        const float a = (fa < fcn && k <= D) ? sW[fa * WS + k] : 0.f;
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(a, xb[s], c, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ff = f0 + (q & 3) + 8 * (q >> 2) + 4 * h;
        c[q] = ff < fcn ? sD[ff] * sin_rev(c[q]) : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ff = f0 + (q & 3) + 8 * (q >> 2) + 4 * h;
#pragma unroll
        for (int t = 0; t < DT; ++t) {
          const int k = 32 * t + lr;
          const float a = (ff < fcn && k < D) ? sW[ff * WS + k] : 0.f;
          g[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, c[q], g[t], 0, 0, 0);
        }
      }
    }
  }
  if (!active || n >= N) return;
  float* gr = grad + (size_t)r * D * N;
#pragma unroll
  for (int t = 0; t < DT; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k = 32 * t + (q & 3) + 8 * (q >> 2) + 4 * h;
      if (k < D) gr[(size_t)k * N + n] = g[t][q];
    }
}

// ============================================================================
// Wide joints (D > 256; CGNN builds one MLP per variable for any d, CGNN.py:63-90): the
// per-lane W column / accumulator forms above stop at D = 256 (registers), so the
// projections go through a scratch image instead:
//   proj:   theta[n][f] = [x_n | 1] . W[f]   (matrix cores, W staged in LDS in k-chunks)
//           csum[part][nt][f] = sum over the 32 samples of tile nt of cos(theta)
//           theta of the generated samples kept for the gradient ([R][N][F])
//   reduce: diff_f = norm (sum_nt csum[0] - sum_nt csum[1]) / N in fixed order, the
//           loss partials per 256-feature group (the layout of the narrow forms)
//   grad:   G[k][n] = sum_f W[f][k] S[n][f],  S = -coef diff_f sin(theta)  (matrix cores,
//           the S tile staged in LDS per f-chunk)
// All products on v_mfma_f32_32x32x2_f32 (exact fp32, sequential k order).
// ============================================================================
namespace {
constexpr int RW_KC = 32;     // k-chunk of the staged W image (proj)
constexpr int RW_FC = 64;     // f-chunk of the staged S tile (grad)
}

// grid (ceil(F / 256), ceil(N / 32), 2 R): block = 8 waves x 32 features, one 32-sample tile
__global__ __launch_bounds__(512) void rff_wide_proj_kernel(const float* __restrict__ xhat,
                                                            const float* __restrict__ data,
                                                            const float* __restrict__ W, float* __restrict__ theta,
                                                            float* __restrict__ csum, int N, int D, int F) {
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  __shared__ float sW[256 * (RW_KC + 1)];
  const int part = blockIdx.z & 1, r = blockIdx.z >> 1, nt = blockIdx.y, fb = blockIdx.x;
  const int NT = gridDim.y;
  const int lane = threadIdx.x & 63, h = lane >> 5, lr = lane & 31, wv = threadIdx.x >> 6;
  const int f = fb * 256 + wv * 32 + lr;
  const int n = nt * 32 + lr;
  const float* X = (part == 0 ? xhat : data) + (size_t)r * D * N;
  const float* Wr = W + (size_t)r * F * (D + 1);
  f32x16 c = {};
  for (int kc = 0; kc <= D; kc += RW_KC) {
    __syncthreads();
    for (int i = threadIdx.x; i < 256 * RW_KC; i += 512) {
      const int fl = i / RW_KC, kk = i - fl * RW_KC;
      const int fg = fb * 256 + fl, k = kc + kk;
      sW[fl * (RW_KC + 1) + kk] = (fg < F && k <= D) ? Wr[(size_t)fg * (D + 1) + k] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < RW_KC / 2; ++s) {
      const int k = kc + 2 * s + h;
      const float a = n < N ? (k < D ? X[(size_t)k * N + n] : (k == D ? 1.f : 0.f)) : 0.f;
      c = __builtin_amdgcn_mfma_f32_32x32x2f32(a, sW[(wv * 32 + lr) * (RW_KC + 1) + 2 * s + h], c, 0, 0, 0);
    }
  }
  // lane = feature f, registers = 16 samples of the tile
  float acc = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int nn = nt * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
    acc += nn < N ? cos_rev(c[q]) : 0.f;
  }
  acc += __shfl_xor(acc, 32, 64);
  if (h == 0 && f < F) csum[(((size_t)r * 2 + part) * NT + nt) * F + f] = acc;
  if (part == 0 && f < F) {
    float* th = theta + (size_t)r * N * F;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int nn = nt * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
      if (nn < N) th[(size_t)nn * F + f] = c[q];
    }
  }
}

// grid (ceil(F / 256), R), 256 threads: diff and the loss partial of a 256-feature group
__global__ __launch_bounds__(256) void rff_wide_reduce_kernel(const float* __restrict__ csum,
                                                              float* __restrict__ diff,
                                                              float* __restrict__ loss_part, int N, int F, int NT,
                                                              float norm) {
  __shared__ float s_red[4];
  const int r = blockIdx.y;
  const int f = blockIdx.x * 256 + threadIdx.x;
  float dlt = 0.f;
  if (f < F) {
    const float* cp = csum + (size_t)r * 2 * NT * F + f;
    float sp = 0.f, st = 0.f;
    for (int t = 0; t < NT; ++t) {
      sp += cp[(size_t)t * F];
      st += cp[(size_t)(NT + t) * F];
    }
    dlt = norm * (sp - st) / (float)N;
    diff[(size_t)r * F + f] = dlt;
  }
  const float v = wave_sum(dlt * dlt);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0)
    loss_part[(size_t)r * gridDim.x + blockIdx.x] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
}

// grid (ceil(D / 256), ceil(N / 32), R): block = 8 waves x 32 gradient rows k, one
// 32-sample tile; G[k][n] into grad [R][D][N]
__global__ __launch_bounds__(512) void rff_wide_grad_kernel(const float* __restrict__ theta,
                                                            const float* __restrict__ W,
                                                            const float* __restrict__ diff, float* __restrict__ grad,
                                                            int N, int D, int F, float coef) {
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  __shared__ float sS[32 * (RW_FC + 1)];
  const int r = blockIdx.z, nt = blockIdx.y;
  const int lane = threadIdx.x & 63, h = lane >> 5, lr = lane & 31, wv = threadIdx.x >> 6;
  const int k0 = blockIdx.x * 256 + wv * 32;
  const float* th = theta + (size_t)r * N * F;
  const float* Wr = W + (size_t)r * F * (D + 1);
  const float* dr = diff + (size_t)r * F;
  f32x16 g = {};
  for (int fc = 0; fc < F; fc += RW_FC) {
    __syncthreads();
    for (int i = threadIdx.x; i < 32 * RW_FC; i += 512) {
      const int nl = i / RW_FC, ff = i - nl * RW_FC;
      const int nn = nt * 32 + nl, fg = fc + ff;
      sS[nl * (RW_FC + 1) + ff] = (nn < N && fg < F) ? -coef * dr[fg] * sin_rev(th[(size_t)nn * F + fg]) : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int s = 0; s < RW_FC / 2; ++s) {
      const int fg = fc + 2 * s + h, k = k0 + lr;
      const float a = (fg < F && k < D) ? Wr[(size_t)fg * (D + 1) + k] : 0.f;
      g = __builtin_amdgcn_mfma_f32_32x32x2f32(a, sS[lr * (RW_FC + 1) + 2 * s + h], g, 0, 0, 0);
    }
  }
  // lane = sample, registers = 16 gradient rows k
  const int n = nt * 32 + lr;
  if (n >= N) return;
  float* gr = grad + (size_t)r * D * N;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int k = k0 + (q & 3) + 8 * (q >> 2) + 4 * h;
    if (k < D) gr[(size_t)k * N + n] = g[q];
  }
}

// scratch floats of the wide form (theta of the generated samples + the cos-sum partials)
extern "C" long rff_wide_scratch_floats(int N, int F, int R) {
  const long NT = (N + 31) / 32;
  return (long)R * N * F + (long)R * 2 * NT * F;
}

static int rff_wide(int mode, const float* xhat, const float* data, const float* W, float* diff, float* loss_part,
                    float* grad, int N, int D, int F, int R, float norm, float* scratch, hipStream_t st) {
  if (!scratch) return -2;
  const int NT = (N + 31) / 32;
  float* theta = scratch;
  float* csum = scratch + (size_t)R * N * F;
  hipLaunchKernelGGL(rff_wide_proj_kernel, dim3((F + 255) / 256, NT, 2 * R), dim3(512), 0, st, xhat, data, W,
                     theta, csum, N, D, F);
  hipLaunchKernelGGL(rff_wide_reduce_kernel, dim3((F + 255) / 256, R), dim3(256), 0, st, csum, diff, loss_part, N,
                     F, NT, norm);
  if (mode == 0)
    hipLaunchKernelGGL(rff_wide_grad_kernel, dim3((D + 255) / 256, NT, R), dim3(512), 0, st, theta, W, diff, grad,
                       N, D, F, 2.f * norm / (float)N);
  return (int)hipGetLastError();
}

extern "C" int rff_launch_freqs(float* W, const uint32_t* keys, const int* step_base, int step_off,
                                int k, int D, int n_gamma, int d_true, int R, hipStream_t st) {
  const int tot = k * n_gamma * (D + 1);
  hipLaunchKernelGGL(rff_freqs_kernel, dim3((tot + 255) / 256, R), dim3(256), 0, st, W, keys,
                     step_base, step_off, k, D, n_gamma, d_true);
  return (int)hipGetLastError();
}

template <int D>
static int rff_fb_d(int mode, const float* xhat, const float* data, const float* W, float* diff,
                    float* loss_part, float* grad, int N, int F, int R, int k, float norm,
                    hipStream_t st, int force_valu) {
  // features staged per chunk of the gradient kernel: all of them when [F][D + 1] fits
  // in 160 KiB, else the largest multiple of 32 that does
  const size_t cap = 160 * 1024 / sizeof(float);
  const bool whole = (size_t)F * (D + 2) <= cap;
  const int FC = whole ? F : (int)(cap / (D + 2)) / 32 * 32;
  if (D > 64 || (!force_valu && whole)) {    // the vector kernels stop at D = 64
    if (FC < 32) return -2;
    const size_t glds = sizeof(float) * (size_t)FC * (D + 2);
    hipLaunchKernelGGL((rff_mfma_feat_kernel<D>), dim3((F + 255) / 256, R), dim3(512), 0, st, xhat, data, W, diff,
                       loss_part, N, F, norm);
    if (mode == 0) {
      (void)hipFuncSetAttribute((const void*)rff_mfma_grad_kernel<D>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)glds);
      hipLaunchKernelGGL((rff_mfma_grad_kernel<D>), dim3((N + 127) / 128, R), dim3(256), glds, st, xhat, W, diff,
                         grad, N, F, 2.f * norm / (float)N, FC);
    }
    return (int)hipGetLastError();
  }
  if constexpr (D <= 64) {
    hipLaunchKernelGGL((rff_feat_kernel<D>), dim3((F + 255) / 256, R), dim3(256), 0, st, xhat, data,
                       W, diff, loss_part, N, F, norm);
    if (mode == 0) {
      const float coef = 2.f * norm / (float)N;
      hipLaunchKernelGGL((rff_grad_kernel<D>), dim3((N + 255) / 256, R), dim3(256), 0, st, xhat, W,
                         diff, grad, N, F, coef);
    }
    return (int)hipGetLastError();
  }
  return -1;
}

// mode 0: loss partials + gradient; mode 1: loss partials only.  force_valu: the vector
// kernels wherever they exist (D <= 64; A/B and tests).  D > 256 (any width): the wide
// form, with `scratch` of rff_wide_scratch_floats(N, F, R) floats; force_wide = 1 takes
// it at any D (tests: the two forms agree)
extern "C" int rff_launch_fwd_bwd(int mode, const float* xhat, const float* data, const float* W,
                                  float* diff, float* loss_part, float* grad, int N, int D, int F,
                                  int R, int k, float norm, hipStream_t st, int force_valu, float* scratch,
                                  int force_wide) {
  if (D > 256 || force_wide) return rff_wide(mode, xhat, data, W, diff, loss_part, grad, N, D, F, R, norm, scratch, st);
  switch (D) {
#define CASE_D(d) case d: return rff_fb_d<d>(mode, xhat, data, W, diff, loss_part, grad, N, F, R, k, norm, st, force_valu);
    CASE_D(1) CASE_D(2) CASE_D(3) CASE_D(4) CASE_D(6) CASE_D(8) CASE_D(12) CASE_D(16) CASE_D(20)
    CASE_D(24) CASE_D(32) CASE_D(48) CASE_D(64) CASE_D(80) CASE_D(96) CASE_D(128) CASE_D(160) CASE_D(192)
    CASE_D(224) CASE_D(256)
#undef CASE_D
    default: return -1;
  }
}
