// LayerNorm over the last dimension (C <= 1024) for the detector head of the Phase-6 model: the PN-BiMamba
// pre-norms, the fusion's stream norms and norm_f (src/models/DualStreamSEMamba.py:445-486,537-637,700-770),
// which under autocast run as fp32 layer_norm whose output the next linear casts to bf16, and whose backward is
// three kernels (input gradient, partial and final gamma/beta reductions) plus casts.
//   forward  one wave per row: mean / rstd (two-pass, biased variance, as torch), y = (x - mean) rstd gamma +
//            beta written in the requested dtype (bf16 when the consumer is a bf16 linear: the same value the
//            cast would produce), mean / rstd saved.
//   backward one wave per ROWS_PER_WAVE rows (the next row prefetched): dx = rstd (g - mean(g) - xhat mean(g xhat)), g = dy gamma;
//            dgamma = sum dy xhat, dbeta = sum dy accumulated per lane, reduced over the workgroup's waves in
//            LDS and ADDED into the fp32 gradient buffers with one atomic per (channel, workgroup).
#include <type_traits>

#include "common.h"

namespace rdx {

constexpr int RL_MAXV = 16;            // C <= 64 * 16
constexpr int RL_WAVES = 4;
#ifndef RL_RPW
#define RL_RPW 4
#endif
constexpr int RL_ROWS_PER_WAVE = RL_RPW;

template <typename T>
__device__ __forceinline__ float rl_ld(const T* p, int64_t i) {
  if constexpr (std::is_same<T, float>::value) return p[i];
  else return h2f(p[i]);
}
template <typename T>
__device__ __forceinline__ void rl_st(T* p, int64_t i, float v) {
  if constexpr (std::is_same<T, float>::value) p[i] = v;
  else p[i] = f2h(v);
}

template <typename TI, typename TO>
__global__ __launch_bounds__(RL_WAVES * 64) void row_ln_fwd_kernel(const TI* __restrict__ x, const float* __restrict__ gamma,
                                                                  const float* __restrict__ beta, float eps,
                                                                  TO* __restrict__ y, float* __restrict__ mean,
                                                                  float* __restrict__ rstd, int64_t M, int C) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * RL_WAVES + (threadIdx.x >> 6);
  if (m >= M) return;
  float v[RL_MAXV];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < RL_MAXV; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < C ? rl_ld(x, m * C + c) : 0.f;
    s += v[j];
  }
  const float mu = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < RL_MAXV; ++j) {
    const int c = lane + 64 * j;
    const float d = c < C ? v[j] - mu : 0.f;
    q += d * d;
  }
  const float rs = rsqrtf(wave_sum(q) / C + eps);
#pragma unroll
  for (int j = 0; j < RL_MAXV; ++j) {
    const int c = lane + 64 * j;
    if (c < C) rl_st(y, m * C + c, (v[j] - mu) * rs * gamma[c] + beta[c]);
  }
  if (lane == 0) {
    mean[m] = mu;
    rstd[m] = rs;
  }
}

template <typename TG, typename TX, int V>
__global__ __launch_bounds__(RL_WAVES * 64) void row_ln_bwd_kernel(const TG* __restrict__ dy, const TX* __restrict__ x,
                                                                  const float* __restrict__ mean,
                                                                  const float* __restrict__ rstd,
                                                                  const float* __restrict__ gamma, TX* __restrict__ dx,
                                                                  float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                                  int64_t M, int C) {
  // V = values per lane (C <= 64 V). The next row's dy / x are loaded while the current row is reduced, so a
  // wave's rows do not serialize on HBM latency.
  __shared__ float red[2][RL_WAVES][V * 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float dg[V], db[V], gm[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int c = lane + 64 * j;
    dg[j] = db[j] = 0.f;
    gm[j] = c < C ? gamma[c] : 0.f;
  }
  const int64_t m0 = ((int64_t)blockIdx.x * RL_WAVES + wv) * RL_ROWS_PER_WAVE;
  const int nrow = (int)(M - m0 < RL_ROWS_PER_WAVE ? (M - m0 > 0 ? M - m0 : 0) : RL_ROWS_PER_WAVE);
  float dn[V], xn[V];
  if (nrow > 0) {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = lane + 64 * j;
      dn[j] = c < C ? rl_ld(dy, m0 * C + c) : 0.f;
      xn[j] = c < C ? rl_ld(x, m0 * C + c) : 0.f;
    }
  }
  for (int rr = 0; rr < nrow; ++rr) {
    const int64_t m = m0 + rr;
    float d[V], xv[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      d[j] = dn[j];
      xv[j] = xn[j];
    }
    if (rr + 1 < nrow) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int c = lane + 64 * j;
        dn[j] = c < C ? rl_ld(dy, (m + 1) * C + c) : 0.f;
        xn[j] = c < C ? rl_ld(x, (m + 1) * C + c) : 0.f;
      }
    }
    const float mu = mean[m], rs = rstd[m];
    float xh[V], g[V];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = lane + 64 * j;
      xh[j] = c < C ? (xv[j] - mu) * rs : 0.f;
      g[j] = d[j] * gm[j];
      s1 += g[j];
      s2 += g[j] * xh[j];
      dg[j] = fmaf(d[j], xh[j], dg[j]);
      db[j] += d[j];
    }
    s1 = wave_sum(s1) / C;
    s2 = wave_sum(s2) / C;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = lane + 64 * j;
      if (c < C) rl_st(dx, m * C + c, rs * (g[j] - s1 - xh[j] * s2));
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) {
    red[0][wv][lane + 64 * j] = dg[j];
    red[1][wv][lane + 64 * j] = db[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += RL_WAVES * 64) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < RL_WAVES; ++w) {
      a += red[0][w][c];
      b += red[1][w][c];
    }
    atomicAdd(dgamma + c, a);
    atomicAdd(dbeta + c, b);
  }
}

}  // namespace rdx

using namespace rdx;

extern "C" int rdx_row_ln_fwd(int dtype_x, const void* x, const float* gamma, const float* beta, float eps,
                              int dtype_y, void* y, float* mean, float* rstd, int64_t M, int C, void* stream) {
  RDX_REQUIRE(x && gamma && beta && y && mean && rstd && M > 0 && C > 0);
  RDX_REQUIRE((dtype_x == RDX_F32 || dtype_x == RDX_BF16) && (dtype_y == RDX_F32 || dtype_y == RDX_BF16));
  if (C > 64 * RL_MAXV) return RDX_EUNSUPPORTED;
  const dim3 grid((unsigned)((M + RL_WAVES - 1) / RL_WAVES)), block(RL_WAVES * 64);
  hipStream_t st = as_stream(stream);
#define RL_FWD(TI, TO)                                                                                          \
  hipLaunchKernelGGL((row_ln_fwd_kernel<TI, TO>), grid, block, 0, st, (const TI*)x, gamma, beta, eps, (TO*)y, \
                     mean, rstd, M, C)
  if (dtype_x == RDX_F32 && dtype_y == RDX_F32) RL_FWD(float, float);
  else if (dtype_x == RDX_F32) RL_FWD(float, hst);
  else if (dtype_y == RDX_F32) RL_FWD(hst, float);
  else RL_FWD(hst, hst);
#undef RL_FWD
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_row_ln_bwd(int dtype_dy, const void* dy, int dtype_x, const void* x, const float* mean,
                              const float* rstd, const float* gamma, void* dx, float* dgamma, float* dbeta, int64_t M,
                              int C, void* stream) {
  RDX_REQUIRE(dy && x && mean && rstd && gamma && dx && dgamma && dbeta && M > 0 && C > 0);
  RDX_REQUIRE((dtype_dy == RDX_F32 || dtype_dy == RDX_BF16) && (dtype_x == RDX_F32 || dtype_x == RDX_BF16));
  if (C > 64 * RL_MAXV) return RDX_EUNSUPPORTED;
  const int64_t rows_per_block = (int64_t)RL_WAVES * RL_ROWS_PER_WAVE;
  const dim3 grid((unsigned)((M + rows_per_block - 1) / rows_per_block)), block(RL_WAVES * 64);
  hipStream_t st = as_stream(stream);
#define RL_BWD(TG, TX)                                                                                           \
  do {                                                                                                          \
    if (C <= 64 * 3)                                                                                           \
      hipLaunchKernelGGL((row_ln_bwd_kernel<TG, TX, 3>), grid, block, 0, st, (const TG*)dy, (const TX*)x, mean, \
                         rstd, gamma, (TX*)dx, dgamma, dbeta, M, C);                                          \
    else                                                                                                        \
      hipLaunchKernelGGL((row_ln_bwd_kernel<TG, TX, RL_MAXV>), grid, block, 0, st, (const TG*)dy, (const TX*)x, \
                         mean, rstd, gamma, (TX*)dx, dgamma, dbeta, M, C);                                    \
  } while (0)
  if (dtype_dy == RDX_F32 && dtype_x == RDX_F32) RL_BWD(float, float);
  else if (dtype_dy == RDX_F32) RL_BWD(float, hst);
  else if (dtype_x == RDX_F32) RL_BWD(hst, float);
  else RL_BWD(hst, hst);
#undef RL_BWD
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
