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
#include "cgnn_common.h"

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
                    hipStream_t st) {
  hipLaunchKernelGGL((rff_feat_kernel<D>), dim3((F + 255) / 256, R), dim3(256), 0, st, xhat, data,
                     W, diff, loss_part, N, F, norm);
  if (mode == 0) {
    const float coef = 2.f * norm / (float)N;
    hipLaunchKernelGGL((rff_grad_kernel<D>), dim3((N + 255) / 256, R), dim3(256), 0, st, xhat, W,
                       diff, grad, N, F, coef);
  }
  return (int)hipGetLastError();
}

// mode 0: loss partials + gradient; mode 1: loss partials only.
extern "C" int rff_launch_fwd_bwd(int mode, const float* xhat, const float* data, const float* W,
                                  float* diff, float* loss_part, float* grad, int N, int D, int F,
                                  int R, int k, float norm, hipStream_t st) {
  switch (D) {
#define CASE_D(d) case d: return rff_fb_d<d>(mode, xhat, data, W, diff, loss_part, grad, N, F, R, k, norm, st);
    CASE_D(1) CASE_D(2) CASE_D(3) CASE_D(4) CASE_D(6) CASE_D(8) CASE_D(12) CASE_D(16) CASE_D(20)
    CASE_D(24) CASE_D(32) CASE_D(48) CASE_D(64)
#undef CASE_D
    default: return -1;
  }
}
