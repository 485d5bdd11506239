// Mixup focal loss for gfx950: the whole criterion of one pass (forward value and logits gradient) in one
// launch, and its backward in one more, instead of ~50 one-element framework kernels per pass.
//
// Reference: criterion = kornia FocalLoss(alpha, gamma, reduction='mean') (src/main.py:297-305), applied as
// the mixup loss  lam * criterion(out, y_a) + (1 - lam) * criterion(out, y_b)  (src/main.py:1040-1046), divided
// by the accumulation steps (:1050). Restated by radhip.train.FocalLoss (both kornia generations):
//   per row b, class y:  lp = log_softmax(z_b)[y],  p = exp(lp),  f(z_b, y) = -a_y (1 - p)^gamma lp
//   mode 0 ('per_class'): a_y = (y == 0 ? 1 - alpha : alpha), the mean runs over B*C elements
//   mode 1 ('scalar'):    a_y = alpha, the mean runs over B rows;  alpha < 0: no factor (a = 1)
// Here  loss = scale * sum_b [ lam_b f(z_b, ya_b) + (1 - lam_b) f(z_b, yb_b) ]  with scale = 1 / (rows of one
// micro-batch * (C or 1) * accumulation) and lam_b = lam[b / rows_per_lam] (so the K micro-batches of a
// window's batched clean pass are one launch). The gradient
//   d f / d z_j = -a_y (delta_jy - p_j) [ (1 - p)^gamma - gamma (1 - p)^(gamma - 1) p lp ]
// is produced by the same launch (fp32, per unit of upstream gradient); the backward scales it by the
// upstream gradient and writes it in the logits' dtype.
#include "common.h"

namespace rdx {

constexpr int FL_THREADS = 256;
constexpr int FL_MAXC = 16;

template <typename T>
__device__ __forceinline__ float focal_row(const T* z, int C, int y, float alpha, float gamma, int mode, float wgt,
                                           float* dz) {
  float m = -INFINITY;
  for (int j = 0; j < C; ++j) m = fmaxf(m, ld(z, j));
  float s = 0.f;
  for (int j = 0; j < C; ++j) s += expf(ld(z, j) - m);
  const float lse = m + logf(s);
  const float lp = ld(z, y) - lse;
  const float p = expf(lp);
  const float omp = 1.0f - p;
  const float w = powf(omp, gamma);
  const float a = alpha < 0.f ? 1.0f : (mode == 0 ? (y == 0 ? 1.0f - alpha : alpha) : alpha);
  // d/dp of (1 - p)^gamma is 0 at gamma == 0 and taken as 0 at p == 1 (torch pow backward; no 0 * inf)
  const float k = (gamma == 0.f || omp == 0.f) ? w : w - gamma * powf(omp, gamma - 1.0f) * p * lp;
  for (int j = 0; j < C; ++j) {
    const float pj = expf(ld(z, j) - lse);
    dz[j] += wgt * (-a) * ((j == y ? 1.0f : 0.0f) - pj) * k;
  }
  return wgt * (-a * w * lp);
}

template <typename T>
__global__ __launch_bounds__(FL_THREADS) void focal_mixup_kernel(const T* __restrict__ logits, int ld_, int B, int C,
                                                                  const int64_t* __restrict__ ya,
                                                                  const int64_t* __restrict__ yb,
                                                                  const float* __restrict__ lam, int rows_per_lam,
                                                                  float alpha, float gamma, int mode, float scale,
                                                                  float* __restrict__ loss, float* __restrict__ dlog) {
  __shared__ float s_red[FL_THREADS / 64];
  float acc = 0.f;
  for (int b = threadIdx.x; b < B; b += FL_THREADS) {
    const T* z = logits + (int64_t)b * ld_;
    const float l = lam ? lam[b / rows_per_lam] : 1.0f;
    float dz[FL_MAXC];
    for (int j = 0; j < C; ++j) dz[j] = 0.f;
    acc += focal_row(z, C, (int)ya[b], alpha, gamma, mode, l * scale, dz);
    if (yb) acc += focal_row(z, C, (int)yb[b], alpha, gamma, mode, (1.0f - l) * scale, dz);
    for (int j = 0; j < C; ++j) dlog[(int64_t)b * C + j] = dz[j];
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < FL_THREADS / 64; ++k) t += s_red[k];
    loss[0] = t;
  }
}

template <typename T>
__global__ __launch_bounds__(FL_THREADS) void focal_scale_kernel(const float* __restrict__ g,
                                                                  const float* __restrict__ d32, T* __restrict__ out,
                                                                  int n) {
  const float s = g[0];
  for (int i = blockIdx.x * FL_THREADS + threadIdx.x; i < n; i += gridDim.x * FL_THREADS) st(out, i, d32[i] * s);
}

}  // namespace rdx

using namespace rdx;

extern "C" int rdx_focal_mixup_fwd(const void* logits, int logits_bf16, int ld_, int B, int C, const int64_t* ya,
                                   const int64_t* yb, const float* lam, int rows_per_lam, float alpha, float gamma,
                                   int mode, float scale, float* loss, float* dlogits, void* stream) {
  RDX_REQUIRE(logits && ya && loss && dlogits && B > 0 && C > 0 && ld_ >= C && (mode == 0 || mode == 1));
  RDX_REQUIRE(!lam || rows_per_lam > 0);
  if (C > FL_MAXC) return RDX_EUNSUPPORTED;
  hipStream_t s = as_stream(stream);
  if (logits_bf16)
    hipLaunchKernelGGL(focal_mixup_kernel<hst>, dim3(1), dim3(FL_THREADS), 0, s,
                       (const hst*)logits, ld_, B, C, ya, yb, lam, rows_per_lam, alpha, gamma, mode, scale,
                       loss, dlogits);
  else
    hipLaunchKernelGGL(focal_mixup_kernel<float>, dim3(1), dim3(FL_THREADS), 0, s, (const float*)logits, ld_, B, C, ya,
                       yb, lam, rows_per_lam, alpha, gamma, mode, scale, loss, dlogits);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_focal_mixup_bwd(const float* grad, const float* dlogits, void* out, int out_bf16, int n,
                                   void* stream) {
  RDX_REQUIRE(grad && dlogits && out && n > 0);
  hipStream_t s = as_stream(stream);
  const int blocks = (n + FL_THREADS - 1) / FL_THREADS < 64 ? (n + FL_THREADS - 1) / FL_THREADS : 64;
  if (out_bf16)
    hipLaunchKernelGGL(focal_scale_kernel<hst>, dim3(blocks), dim3(FL_THREADS), 0, s, grad, dlogits,
                       (hst*)out, n);
  else
    hipLaunchKernelGGL(focal_scale_kernel<float>, dim3(blocks), dim3(FL_THREADS), 0, s, grad, dlogits, (float*)out, n);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
