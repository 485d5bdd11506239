// FGM adversarial perturbation for gfx950 (multi-tensor, two launches, no host sync).
//
// Reference: FGM.attack (src/main.py:85-94), applied to the parameters whose name contains
// "feature_projection" (WavLM LayerNorm(512) + Linear(512->1024), 526 336 values):
//   backup = p.clone();  norm = ||p.grad||_2;  if norm != 0 and not isnan(norm): p += eps*grad/norm
// Launch 1 writes per-block partial sums of g^2 (fp64) for every tensor; launch 2 finishes each norm
// in every block (deterministic order) and applies backup + update with grid-stride float4 streams.
#include "common.h"

namespace rdx {

constexpr int FGM_MAXT = 32;
constexpr int FGM_PART = 256;  // partial-sum slots per tensor
constexpr int FGM_THREADS = 256;

struct FgmTable {
  float* p[FGM_MAXT];
  const float* g[FGM_MAXT];
  float* bk[FGM_MAXT];
  int64_t n[FGM_MAXT];
};

__global__ __launch_bounds__(FGM_THREADS) void fgm_norm_kernel(FgmTable T, double* __restrict__ ws) {
  __shared__ double s_red[FGM_THREADS / 64];
  const int ti = blockIdx.y;
  const float* g = T.g[ti];
  const int64_t n = T.n[ti];
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * FGM_THREADS + threadIdx.x; i < n; i += (int64_t)FGM_PART * FGM_THREADS) {
    double v = (double)g[i];
    acc += v * v;
  }
  acc = wave_sum_d(acc);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int k = 0; k < FGM_THREADS / 64; ++k) s += s_red[k];
    ws[ti * FGM_PART + blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(FGM_THREADS) void fgm_apply_kernel(FgmTable T, const double* __restrict__ ws, float eps) {
  __shared__ float s_scale;
  __shared__ int s_skip;
  const int ti = blockIdx.y;
  if (threadIdx.x < 64) {
    double s = 0.0;
    for (int k = threadIdx.x; k < FGM_PART; k += 64) s += ws[ti * FGM_PART + k];
    s = wave_sum_d(s);
    if (threadIdx.x == 0) {
      const float norm = (float)sqrt(s);
      s_skip = (norm == 0.0f || isnan(norm)) ? 1 : 0;
      s_scale = norm;
    }
  }
  __syncthreads();
  float* p = T.p[ti];
  const float* g = T.g[ti];
  float* bk = T.bk[ti];
  const int64_t n = T.n[ti];
  const float norm = s_scale;
  const bool skip = s_skip != 0;
  // 4 elements per thread per round, every load of the round issued before its stores (a load-store pair per
  // iteration waited one round trip each: ~20 us for the 0.5 M-element projection on 64 blocks)
  const int64_t stride = (int64_t)gridDim.x * FGM_THREADS;
  for (int64_t i0 = (int64_t)blockIdx.x * FGM_THREADS + threadIdx.x; i0 < n; i0 += 4 * stride) {
    float pv[4], gv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = i0 + k * stride < n ? i0 + k * stride : n - 1;   // clamped: the load is unconditional
      pv[k] = p[i];
      gv[k] = g[i];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = i0 + k * stride;
      if (i < n) {
        bk[i] = pv[k];
        if (!skip) p[i] = pv[k] + eps * gv[k] / norm;
      }
    }
  }
}

}  // namespace rdx

using namespace rdx;

extern "C" int rdx_fgm_attack(int ntensors, float* const* params, const float* const* grads, float* const* backup,
                              const int64_t* numels, float eps, double* workspace, void* stream) {
  RDX_REQUIRE(params && grads && backup && numels && workspace && ntensors > 0);
  if (ntensors > FGM_MAXT) return RDX_EUNSUPPORTED;
  FgmTable T{};
  for (int i = 0; i < ntensors; ++i) {
    RDX_REQUIRE(params[i] && grads[i] && backup[i] && numels[i] > 0);
    T.p[i] = params[i];
    T.g[i] = grads[i];
    T.bk[i] = backup[i];
    T.n[i] = numels[i];
  }
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(fgm_norm_kernel, dim3(FGM_PART, ntensors), dim3(FGM_THREADS), 0, s, T, workspace);
  RDX_LAUNCH_CHECK();
  int64_t nmax = 0;
  for (int i = 0; i < ntensors; ++i) nmax = numels[i] > nmax ? numels[i] : nmax;
  const int64_t want = (nmax + 4 * FGM_THREADS - 1) / (4 * FGM_THREADS);   // one round of 4 per thread
  const unsigned gx = (unsigned)(want < 64 ? 64 : (want > 1024 ? 1024 : want));
  hipLaunchKernelGGL(fgm_apply_kernel, dim3(gx, ntensors), dim3(FGM_THREADS), 0, s, T, workspace, eps);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" const char* rdx_version(void) { return "radhip 0.1.0 (gfx950)"; }

extern "C" const char* rdx_strerror(int code) {
  if (code == RDX_OK) return "ok";
  if (code == RDX_EINVAL) return "invalid argument";
  if (code == RDX_EUNSUPPORTED) return "unsupported shape";
  if (code > 0) return hipGetErrorString((hipError_t)code);
  return "unknown error";
}
