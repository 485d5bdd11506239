// AdamW step over a list of fp32 parameter tensors (torch.optim.AdamW with decoupled weight decay, the optimizer
// of src/main.py:416-457, `AdamW(param_groups, weight_decay=...)`), with the GradScaler hooks of torch's fused form:
// an optional grad scale (grads divided by it and stored back unscaled) and found_inf (the update is skipped).
//
//   p -= lr * wd * p;  m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2
//   p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)            (t = the tensor's step count, on device)
//
// torch's fused kernel deals tensors to blocks in chunks of 64 K elements: the head's ~3 M trainable parameters
// became ~50 blocks moving 1.8 MB each, ~95 us per launch, 5 launches per step. Here a block owns 4096 elements
// (256 threads x 16, float4 loads), so one launch spreads the same tensors over ~750 blocks.
#include "common.h"

namespace rdx {

constexpr int OPT_T = 256;
constexpr int OPT_EPT = 16;                       // elements per thread
constexpr int OPT_CHUNK = OPT_T * OPT_EPT;        // elements per block
constexpr int OPT_MAXP = 48;                      // tensors per launch (the table is a kernel argument)

struct AdamwTable {
  float* p[OPT_MAXP];
  float* g[OPT_MAXP];
  float* m[OPT_MAXP];
  float* v[OPT_MAXP];
  const float* step[OPT_MAXP];
  int64_t n[OPT_MAXP];
  int blk0[OPT_MAXP];
  int count;
};

__global__ __launch_bounds__(OPT_T) void adamw_many_kernel(AdamwTable t, double lr, double beta1, double beta2,
                                                           double wd, double eps, const float* __restrict__ grad_scale,
                                                           const float* __restrict__ found_inf) {
  if (found_inf && *found_inf != 0.f) return;
  int k = 0;
#pragma unroll
  for (int j = 1; j < OPT_MAXP; ++j) k = (j < t.count && (int)blockIdx.x >= t.blk0[j]) ? j : k;
  k = __builtin_amdgcn_readfirstlane(k);
  const int64_t n = t.n[k];
  const int64_t base = (int64_t)(blockIdx.x - t.blk0[k]) * OPT_CHUNK;
  float* __restrict__ P = t.p[k];
  float* __restrict__ G = t.g[k];
  float* __restrict__ M = t.m[k];
  float* __restrict__ V = t.v[k];
  // the arithmetic of torch's fused AdamW functor (ATen fused_adam_utils): hyper-parameters are doubles, so every
  // expression that involves one is evaluated in double and rounded to fp32 where the functor stores an fp32
  // value; the bias corrections come from the step count in double and are used as fp32
  const float st = *t.step[k];
  const float bc1 = (float)(1.0 - pow(beta1, (double)st));
  const float bc2_sqrt = (float)sqrt(1.0 - pow(beta2, (double)st));
  const float step_size = (float)(lr / (double)bc1);
  const double gs = grad_scale ? (double)*grad_scale : 1.0;
  const bool vec = ((((uintptr_t)P | (uintptr_t)G | (uintptr_t)M | (uintptr_t)V) & 15) == 0);
#pragma unroll
  for (int q = 0; q < OPT_EPT / 4; ++q) {
    const int64_t i = base + 4 * ((int64_t)q * OPT_T + threadIdx.x);
    if (i >= n) break;
    float pv[4], gv[4], mv[4], vv[4];
    const int cnt = (int)(n - i < 4 ? n - i : 4);
    if (vec && cnt == 4) {
      const float4 a = *reinterpret_cast<const float4*>(P + i), b = *reinterpret_cast<const float4*>(G + i);
      const float4 c = *reinterpret_cast<const float4*>(M + i), d = *reinterpret_cast<const float4*>(V + i);
      pv[0] = a.x; pv[1] = a.y; pv[2] = a.z; pv[3] = a.w;
      gv[0] = b.x; gv[1] = b.y; gv[2] = b.z; gv[3] = b.w;
      mv[0] = c.x; mv[1] = c.y; mv[2] = c.z; mv[3] = c.w;
      vv[0] = d.x; vv[1] = d.y; vv[2] = d.z; vv[3] = d.w;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pv[e] = e < cnt ? P[i + e] : 0.f;
        gv[e] = e < cnt ? G[i + e] : 0.f;
        mv[e] = e < cnt ? M[i + e] : 0.f;
        vv[e] = e < cnt ? V[i + e] : 0.f;
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (grad_scale) gv[e] = (float)((double)gv[e] / gs);   // stored back: .grad ends unscaled (torch's fused step)
      if (wd != 0.0) pv[e] = (float)((double)pv[e] - lr * wd * (double)pv[e]);
      mv[e] = (float)(beta1 * (double)mv[e] + (1.0 - beta1) * (double)gv[e]);
      vv[e] = (float)(beta2 * (double)vv[e] + (1.0 - beta2) * (double)gv[e] * (double)gv[e]);
      const float denom = (float)((double)(sqrtf(vv[e]) / bc2_sqrt) + eps);
      pv[e] -= step_size * mv[e] / denom;
    }
    if (vec && cnt == 4) {
      *reinterpret_cast<float4*>(P + i) = make_float4(pv[0], pv[1], pv[2], pv[3]);
      *reinterpret_cast<float4*>(M + i) = make_float4(mv[0], mv[1], mv[2], mv[3]);
      *reinterpret_cast<float4*>(V + i) = make_float4(vv[0], vv[1], vv[2], vv[3]);
      if (grad_scale) *reinterpret_cast<float4*>(G + i) = make_float4(gv[0], gv[1], gv[2], gv[3]);
    } else {
      for (int e = 0; e < cnt; ++e) {
        P[i + e] = pv[e];
        M[i + e] = mv[e];
        V[i + e] = vv[e];
        if (grad_scale) G[i + e] = gv[e];
      }
    }
  }
}

}  // namespace rdx

using namespace rdx;

extern "C" int rdx_adamw_many_max() { return OPT_MAXP; }

extern "C" int rdx_adamw_many(int n, float* const* params, float* const* grads, float* const* exp_avg,
                              float* const* exp_avg_sq, const float* const* step, const int64_t* numel, double lr,
                              double beta1, double beta2, double weight_decay, double eps, const float* grad_scale,
                              const float* found_inf, void* stream) {
  RDX_REQUIRE(n >= 0 && n <= OPT_MAXP);
  if (n == 0) return RDX_OK;
  RDX_REQUIRE(params && grads && exp_avg && exp_avg_sq && step && numel);
  AdamwTable t{};
  t.count = n;
  int64_t blk = 0;
  for (int k = 0; k < n; ++k) {
    RDX_REQUIRE(numel[k] >= 0 && (numel[k] == 0 || (params[k] && grads[k] && exp_avg[k] && exp_avg_sq[k])) && step[k]);
    t.p[k] = params[k];
    t.g[k] = grads[k];
    t.m[k] = exp_avg[k];
    t.v[k] = exp_avg_sq[k];
    t.step[k] = step[k];
    t.n[k] = numel[k];
    t.blk0[k] = (int)blk;
    blk += (numel[k] + OPT_CHUNK - 1) / OPT_CHUNK;
  }
  RDX_REQUIRE(blk < (1ll << 31));
  if (blk == 0) return RDX_OK;
  hipLaunchKernelGGL(adamw_many_kernel, dim3((unsigned)blk), dim3(OPT_T), 0, as_stream(stream), t, lr, beta1, beta2,
                     weight_decay, eps, grad_scale, found_inf);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
