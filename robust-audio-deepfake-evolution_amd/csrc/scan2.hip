// Chunked bidirectional selective scan for gfx950 (mamba_ssm selective_scan semantics as restated by the
// reference-owned MambaBlock, src/models/modules/mamba_block.py:65-122; used twice per PN_BiMambas_Encoder,
// src/models/DualStreamSEMamba.py:467-486, direction 1 = flip(scan(flip(x))) at original positions).
//
//   h_s = a_s h_{s-1} + dt_s u_s B_s,  a_s = exp(dt_s A),  y_s = C_s . h_s + D u_s      (s in direction order)
//
// The recurrence is linear, so the steps split into NC chunks of CK = 16 (the checkpoint interval of
// csrc/bimamba.hip, same checkpoint layout) and every (direction, utterance, chunk, 32-channel group) is one
// 512-thread block (thread = channel x state, a DPP row of 16 lanes = one channel's 16 states):
//   fwd 1  each chunk from h = 0: its end state hloc_c and its decay product P_c = prod a;
//   fwd 2  carry-in h = compose(P_k, hloc_k) over the chunks before it (<= NC - 1 FMAs from L2), then the chunk
//          from the true carry: y (staged in LDS, coalesced rows) and the checkpoint at the chunk end;
//   bwd 1  each chunk's reverse carry from 0 (G_s = C_s dy_s + a_{s+1} G_{s+1}): gloc_c = a_{s0} G_{s0};
//   bwd 2  carry from the right = compose(P_k, gloc_k) over the chunks after it, states re-run from the
//          chunk's checkpoint, then every gradient of the chunk.
// At the Phase-6 shapes (B = 8, L = 201, Di = 288, N = 16, both directions) that is 2 x 8 x 13 x 9 = 1872 blocks
// per launch (csrc/bimamba.hip: 384 blocks with a 201-step serial chain staged from 24-byte row slices).
// The per-chunk products P are saved by the forward for the backward (it composes the same decays).
#include "common.h"

namespace rdx {
namespace s2 {

constexpr int N = 16;            // d_state
constexpr int CK = 16;           // steps per chunk (== SCAN_CK of bimamba.hip: same checkpoints)
constexpr int CH = 32;           // channels per block
constexpr int NT = CH * N;       // 512 threads
static_assert(NT == CK * 2 * N, "bwd 1 zeroes a chunk's dBC rows with one thread per element");
constexpr float LOG2E = 1.4426950408889634f;

struct Geo {
  int dl, n, d0, d, c, db, dir, b, s0, cnt, nc;
  bool active;
};

__device__ __forceinline__ Geo geo(int B, int L, int D) {
  Geo g;
  g.dl = threadIdx.x >> 4;
  g.n = threadIdx.x & 15;
  g.d0 = blockIdx.x * CH;
  g.d = g.d0 + g.dl;
  g.c = blockIdx.y;
  g.db = blockIdx.z;
  g.dir = g.db / B;
  g.b = g.db - g.dir * B;
  g.s0 = g.c * CK;
  g.cnt = min(CK, L - g.s0);
  g.nc = (L + CK - 1) / CK;
  g.active = g.d < D;
  return g;
}

// time index of the chunk's step i
__device__ __forceinline__ int tstep(const Geo& g, int i, int L) {
  const int s = g.s0 + i;
  return g.dir ? (L - 1 - s) : s;
}

// LDS staging of the chunk: u, dt = softplus(delta + bias) [CK][CH] (+ dy), B / C [CK][N]
// (+ with s_sig: softplus'(pre) = sigmoid(pre), the ddelta factor, once per (t, d) instead of per state)
template <typename T, bool WITH_C, bool WITH_DY>
__device__ __forceinline__ void stage(const Geo& g, const T* __restrict__ u, const T* __restrict__ delta,
                                      const float* __restrict__ dt_bias, const T* __restrict__ Bm,
                                      const T* __restrict__ Cm, int64_t ldbc, const float* __restrict__ dy,
                                      int64_t dy_dir_stride, float* s_u, float* s_dt, float* s_dy, float* s_B,
                                      float* s_C, int B, int L, int D, float* s_sig = nullptr) {
  const int tid = threadIdx.x;
  {
    const int i = tid >> 5, c = tid & 31, dd = g.d0 + c;
    float uu = 0.f, dv = 0.f, dyv = 0.f, sg = 0.f;
    if (i < g.cnt && dd < D) {
      const int t = tstep(g, i, L);
      const int64_t o = ((int64_t)g.db * L + t) * D + dd;
      uu = ld(u, o);
      const float pre = ld(delta, o) + dt_bias[dd];
      dv = softplusf_(pre);
      if (WITH_DY) {
        dyv = dy[g.dir * dy_dir_stride + ((int64_t)g.b * L + t) * D + dd];
        sg = 1.0f / (1.0f + expf(-pre));
      }
    }
    s_u[i * CH + c] = uu;
    s_dt[i * CH + c] = dv;
    if (WITH_DY) {
      s_dy[i * CH + c] = dyv;
      s_sig[i * CH + c] = sg;
    }
  }
  if (tid < CK * N) {
    const int i = tid >> 4, j = tid & 15;
    float bv = 0.f, cv = 0.f;
    if (i < g.cnt) {
      const int64_t o = ((int64_t)g.db * L + tstep(g, i, L)) * ldbc + j;
      bv = ld(Bm, o);
      if (WITH_C) cv = ld(Cm, o);
    }
    s_B[i * N + j] = bv;
    if (WITH_C) s_C[i * N + j] = cv;
  }
}

// index of per-(db, chunk, d, n) records (hloc, P, gloc, dA partials)
__device__ __forceinline__ int64_t rec(const Geo& g, int chunk, int D) {
  return (((int64_t)g.db * g.nc + chunk) * D + g.d) * N + g.n;
}

// ---- fwd 1: chunk-local end state and decay product
template <typename T>
__global__ __launch_bounds__(NT) void fwd_chunk_kernel(const T* __restrict__ u, const T* __restrict__ delta,
                                                       const float* __restrict__ A_log, const T* __restrict__ Bm,
                                                       int64_t ldbc, const float* __restrict__ dt_bias,
                                                       float* __restrict__ hloc, float* __restrict__ P, int B,
                                                       int L, int D) {
  __shared__ float s_u[CK * CH], s_dt[CK * CH], s_B[CK * N];
  const Geo g = geo(B, L, D);
  stage<T, false, false>(g, u, delta, dt_bias, Bm, nullptr, ldbc, nullptr, 0, s_u, s_dt, nullptr, s_B, nullptr, B,
                         L, D);
  __syncthreads();
  if (!g.active) return;
  const float A2 = -__expf(A_log[g.d * N + g.n]) * LOG2E;
  float h = 0.f, prod = 1.f;
#pragma unroll
  for (int i = 0; i < CK; ++i) {
    if (i < g.cnt) {
      const float dtv = s_dt[i * CH + g.dl];
      const float a = __builtin_amdgcn_exp2f(dtv * A2);
      h = fmaf(a, h, dtv * s_u[i * CH + g.dl] * s_B[i * N + g.n]);
      prod *= a;
    }
  }
  hloc[rec(g, g.c, D)] = h;
  P[rec(g, g.c, D)] = prod;
}

// ---- fwd 2: carry-in, y and the checkpoint at the chunk end
template <typename T>
__global__ __launch_bounds__(NT) void fwd_out_kernel(const T* __restrict__ u, const T* __restrict__ delta,
                                                     const float* __restrict__ A_log, const T* __restrict__ Bm,
                                                     const T* __restrict__ Cm, int64_t ldbc,
                                                     const float* __restrict__ Dp, const float* __restrict__ dt_bias,
                                                     const float* __restrict__ hloc, const float* __restrict__ P,
                                                     float* __restrict__ y, float* __restrict__ ckpt, int B, int L,
                                                     int D) {
  __shared__ float s_u[CK * CH], s_dt[CK * CH], s_B[CK * N], s_C[CK * N], s_y[CK * CH];
  const Geo g = geo(B, L, D);
  stage<T, true, false>(g, u, delta, dt_bias, Bm, Cm, ldbc, nullptr, 0, s_u, s_dt, nullptr, s_B, s_C, B, L, D);
  // carry-in from the chunks before this one, in step order: every load issued unconditionally from a clamped
  // index (a per-load runtime test makes hipcc branch and wait around each load), the unused ones masked to the
  // identity (P = 1, h = 0) in registers, then the FMA chain
  float h = 0.f;
  if (g.active) {
    const int nprev = g.c;
    for (int k0 = 0; k0 < nprev; k0 += CK) {
      const int m = min(CK, nprev - k0);
      float pk[CK], hk[CK];
#pragma unroll
      for (int k = 0; k < CK; ++k) {
        const int kk = k0 + min(k, m - 1);
        pk[k] = P[rec(g, kk, D)];
        hk[k] = hloc[rec(g, kk, D)];
      }
#pragma unroll
      for (int k = 0; k < CK; ++k) h = fmaf(k < m ? pk[k] : 1.f, h, k < m ? hk[k] : 0.f);
    }
  }
  __syncthreads();
  const float A2 = g.active ? -__expf(A_log[g.d * N + g.n]) * LOG2E : 0.f;
  const float Dd = g.active ? Dp[g.d] : 0.f;
#pragma unroll
  for (int i = 0; i < CK; ++i) {
    if (i < g.cnt) {    // block-uniform
      const float dtv = s_dt[i * CH + g.dl];
      const float uu = s_u[i * CH + g.dl];
      const float a = __builtin_amdgcn_exp2f(dtv * A2);
      h = fmaf(a, h, dtv * uu * s_B[i * N + g.n]);
      const float pv = row16_sum(s_C[i * N + g.n] * h);
      if (g.n == 0) s_y[i * CH + g.dl] = fmaf(Dd, uu, pv);
    }
  }
  if (g.active && g.c < g.nc - 1) ckpt[(((int64_t)g.db * (g.nc - 1) + g.c) * D + g.d) * N + g.n] = h;
  __syncthreads();
  {
    const int i = threadIdx.x >> 5, c = threadIdx.x & 31, dd = g.d0 + c;
    if (i < g.cnt && dd < D) y[((int64_t)g.db * L + tstep(g, i, L)) * D + dd] = s_y[i * CH + c];
  }
}

// ---- bwd 1: chunk-local reverse carry (G from 0 at the chunk end): gloc = a_{s0} G_{s0}; the first channel group's
// blocks also zero their chunk's rows of dBC, which bwd 2 accumulates into (no separate fill launch)
template <typename T>
__global__ __launch_bounds__(NT) void bwd_chunk_kernel(const T* __restrict__ delta, const float* __restrict__ A_log,
                                                       const T* __restrict__ Cm, int64_t ldbc,
                                                       const float* __restrict__ dt_bias,
                                                       const float* __restrict__ dy, int64_t dy_dir_stride,
                                                       float* __restrict__ gloc, float* __restrict__ dBC, int B, int L,
                                                       int D) {
  __shared__ float s_dt[CK * CH], s_dy[CK * CH], s_C[CK * N];
  const Geo g = geo(B, L, D);
  if (blockIdx.x == 0) {
    const int i = threadIdx.x >> 5, j = threadIdx.x & 31;   // NT = CK * 2N: one (step, dB|dC column) per thread
    if (i < g.cnt) dBC[((int64_t)g.db * L + tstep(g, i, L)) * (2 * N) + j] = 0.f;
  }
  {
    const int tid = threadIdx.x, i = tid >> 5, c = tid & 31, dd = g.d0 + c;
    float dv = 0.f, dyv = 0.f;
    if (i < g.cnt && dd < D) {
      const int t = tstep(g, i, L);
      dv = softplusf_(ld(delta, ((int64_t)g.db * L + t) * D + dd) + dt_bias[dd]);
      dyv = dy[g.dir * dy_dir_stride + ((int64_t)g.b * L + t) * D + dd];
    }
    s_dt[i * CH + c] = dv;
    s_dy[i * CH + c] = dyv;
    if (tid < CK * N) {
      const int ii = tid >> 4, j = tid & 15;
      s_C[ii * N + j] = ii < g.cnt ? ld(Cm, ((int64_t)g.db * L + tstep(g, ii, L)) * ldbc + j) : 0.f;
    }
  }
  __syncthreads();
  if (!g.active) return;
  const float A2 = -__expf(A_log[g.d * N + g.n]) * LOG2E;
  float X = 0.f;
#pragma unroll
  for (int i = CK - 1; i >= 0; --i) {
    if (i < g.cnt) {
      const float a = __builtin_amdgcn_exp2f(s_dt[i * CH + g.dl] * A2);
      X = a * fmaf(s_C[i * N + g.n], s_dy[i * CH + g.dl], X);
    }
  }
  gloc[rec(g, g.c, D)] = X;
}

// ---- bwd 2: every gradient of the chunk
//   G_s = C_s dy_s + X_s (X from the right);  ddt = sum_n G (A a h_{s-1} + B u);  du = sum_n G dt B + D dy
//   dB_s = sum_d G dt u;  dC_s = sum_d dy h_s;  dA += G dt a h_{s-1};  dD += dy u;  dbias += ddelta
// dB | dC: reduced over the block's 32 channels (2 shuffles in-wave, then the 8 waves through LDS) and added to
// dBC with one fp32 atomic per (block, t, j) (the caller zeroes dBC); dA / dD / dbias: one partial per (dir, b,
// chunk) (the caller sums them). du / ddelta go through LDS and leave as coalesced rows.
template <typename T>
__global__ __launch_bounds__(NT) void bwd_out_kernel(
    const T* __restrict__ u, const T* __restrict__ delta, const float* __restrict__ A_log, const T* __restrict__ Bm,
    const T* __restrict__ Cm, int64_t ldbc, const float* __restrict__ Dp, const float* __restrict__ dt_bias,
    const float* __restrict__ ckpt, const float* __restrict__ P, const float* __restrict__ gloc,
    const float* __restrict__ dy, int64_t dy_dir_stride, T* __restrict__ du, T* __restrict__ ddelta,
    float* __restrict__ dBC, float* __restrict__ dA_part, float* __restrict__ dD_part, float* __restrict__ dbias_part,
    int64_t ldpa, int64_t ldpd, int B, int L, int D) {
  __shared__ float s_u[CK * CH], s_dt[CK * CH], s_dy[CK * CH], s_sig[CK * CH], s_B[CK * N], s_C[CK * N];
  __shared__ float s_red[CK][8][2 * N];     // [step][wave][dB 16 | dC 16]
  const Geo g = geo(B, L, D);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, row = lane >> 4;
  stage<T, true, true>(g, u, delta, dt_bias, Bm, Cm, ldbc, dy, dy_dir_stride, s_u, s_dt, s_dy, s_B, s_C, B, L, D,
                       s_sig);
  // the carry entering from the right: compose the later chunks, nearest last
  float X = 0.f, h0 = 0.f;
  if (g.active) {
    for (int k1 = g.nc - 1; k1 > g.c; k1 -= CK) {
      const int m = min(CK, k1 - g.c);
      float pk[CK], gk[CK];
#pragma unroll
      for (int k = 0; k < CK; ++k) {      // unconditional loads from clamped indices (see fwd_out_kernel)
        const int kk = k1 - min(k, m - 1);
        pk[k] = P[rec(g, kk, D)];
        gk[k] = gloc[rec(g, kk, D)];
      }
#pragma unroll
      for (int k = 0; k < CK; ++k) X = fmaf(k < m ? pk[k] : 1.f, X, k < m ? gk[k] : 0.f);
    }
    if (g.c > 0) h0 = ckpt[(((int64_t)g.db * (g.nc - 1) + (g.c - 1)) * D + g.d) * N + g.n];
  }
  __syncthreads();
  const float Aval = g.active ? -__expf(A_log[g.d * N + g.n]) : 0.f;
  const float A2 = Aval * LOG2E;
  const float Dd = g.active ? Dp[g.d] : 0.f;
  // states of the chunk from its checkpoint
  float hs[CK];
  {
    float h = h0;
#pragma unroll
    for (int i = 0; i < CK; ++i) {
      if (i < g.cnt) {
        const float dtv = s_dt[i * CH + g.dl];
        h = fmaf(__builtin_amdgcn_exp2f(dtv * A2), h, dtv * s_u[i * CH + g.dl] * s_B[i * N + g.n]);
      }
      hs[i] = h;
    }
  }
  float dA = 0.f, dDacc = 0.f, dbacc = 0.f;
  float r_du[CK], r_dd[CK];
#pragma unroll
  for (int i = CK - 1; i >= 0; --i) {
    r_du[i] = 0.f;
    r_dd[i] = 0.f;
    if (i < g.cnt) {    // block-uniform
      const int o = i * CH + g.dl;
      const float dtv = s_dt[o], uu = s_u[o], dyv = s_dy[o];
      const float Bn = s_B[i * N + g.n], Cn = s_C[i * N + g.n];
      const float a = __builtin_amdgcn_exp2f(dtv * A2);
      const float hprev = i > 0 ? hs[i > 0 ? i - 1 : 0] : h0;
      const float G = fmaf(Cn, dyv, X);
      const float ah = a * hprev;
      float vB = g.active ? G * dtv * uu : 0.f;
      float vC = g.active ? dyv * hs[i] : 0.f;
      vB += __shfl_xor(vB, 16, 64);
      vB += __shfl_xor(vB, 32, 64);
      vC += __shfl_xor(vC, 16, 64);
      vC += __shfl_xor(vC, 32, 64);
      if (row == 0) s_red[i][wave][g.n] = vB;
      if (row == 1) s_red[i][wave][N + g.n] = vC;
      dA = fmaf(G * dtv, ah, dA);
      const float ddt = row16_sum(G * fmaf(Aval, ah, Bn * uu));
      const float dus = row16_sum(G * dtv * Bn);
      const float ddl = ddt * s_sig[o];         // softplus'(pre) = sigmoid(pre) (= 1 - exp(-dt))
      r_du[i] = fmaf(Dd, dyv, dus);
      r_dd[i] = ddl;
      dDacc = fmaf(dyv, uu, dDacc);
      dbacc += ddl;
      X = a * G;
    }
  }
  __syncthreads();                           // every read of s_u / s_dt done: reuse them for du / ddelta
  if (g.n == 0) {
#pragma unroll
    for (int i = 0; i < CK; ++i) {
      s_u[i * CH + g.dl] = r_du[i];
      s_dt[i * CH + g.dl] = r_dd[i];
    }
  }
  {
    const int tid = threadIdx.x;
    const int i = tid >> 5, j = tid & 31;      // one (step, dB|dC column) per thread
    if (i < g.cnt) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) v += s_red[i][w][j];
      atomicAdd(&dBC[((int64_t)g.db * L + tstep(g, i, L)) * (2 * N) + j], v);
    }
  }
  const int64_t part = (int64_t)g.db * g.nc + g.c;
  if (g.active) dA_part[part * ldpa + g.d * N + g.n] = dA * Aval;   // d/dA_log = dL/dA * A
  if (g.active && g.n == 0) {
    dD_part[part * ldpd + g.d] = dDacc;
    dbias_part[part * ldpd + g.d] = dbacc;
  }
  __syncthreads();
  {
    const int i = threadIdx.x >> 5, c = threadIdx.x & 31, dd = g.d0 + c;
    if (i < g.cnt && dd < D) {
      const int64_t o = ((int64_t)g.db * L + tstep(g, i, L)) * D + dd;
      st(du, o, s_u[i * CH + c]);
      st(ddelta, o, s_dt[i * CH + c]);
    }
  }
}

}  // namespace s2
}  // namespace rdx

using namespace rdx;

extern "C" int rdx_scan2_chunks(int L) { return (L + s2::CK - 1) / s2::CK; }

// per-(dir, b, chunk, d, n) record count of hloc / P / gloc / dA partials
extern "C" int64_t rdx_scan2_rec_elems(int B, int L, int D, int N, int dirs) {
  return (int64_t)dirs * B * rdx_scan2_chunks(L) * D * N;
}

extern "C" int rdx_scan2_fwd(int dtype, const void* u, const void* delta, const float* A_log, const void* Bm,
                             const void* Cm, int64_t ldbc, const float* Dp, const float* dt_bias, float* y,
                             float* ckpt, float* P, float* hloc, int B, int L, int D, int N, int dirs, void* stream) {
  RDX_REQUIRE(u && delta && A_log && Bm && Cm && Dp && dt_bias && y && ckpt && P && hloc);
  RDX_REQUIRE(B > 0 && L > 0 && D > 0 && (dirs == 1 || dirs == 2) && ldbc >= N);
  if (N != s2::N) return RDX_EUNSUPPORTED;
  const dim3 grid((D + s2::CH - 1) / s2::CH, rdx_scan2_chunks(L), dirs * B);
  hipStream_t st = as_stream(stream);
  if (dtype == RDX_BF16) {
    using T = hst;
    hipLaunchKernelGGL(s2::fwd_chunk_kernel<T>, grid, dim3(s2::NT), 0, st, (const T*)u, (const T*)delta, A_log,
                       (const T*)Bm, ldbc, dt_bias, hloc, P, B, L, D);
    RDX_LAUNCH_CHECK();
    hipLaunchKernelGGL(s2::fwd_out_kernel<T>, grid, dim3(s2::NT), 0, st, (const T*)u, (const T*)delta, A_log,
                       (const T*)Bm, (const T*)Cm, ldbc, Dp, dt_bias, hloc, P, y, ckpt, B, L, D);
  } else if (dtype == RDX_F32) {
    using T = float;
    hipLaunchKernelGGL(s2::fwd_chunk_kernel<T>, grid, dim3(s2::NT), 0, st, (const T*)u, (const T*)delta, A_log,
                       (const T*)Bm, ldbc, dt_bias, hloc, P, B, L, D);
    RDX_LAUNCH_CHECK();
    hipLaunchKernelGGL(s2::fwd_out_kernel<T>, grid, dim3(s2::NT), 0, st, (const T*)u, (const T*)delta, A_log,
                       (const T*)Bm, (const T*)Cm, ldbc, Dp, dt_bias, hloc, P, y, ckpt, B, L, D);
  } else {
    return RDX_EINVAL;
  }
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

// dA_part [dirs * B * NC][D][N], dD_part / dbias_part [dirs * B * NC][D] (NC = rdx_scan2_chunks(L)), rows of
// ld_part floats (0: dense, D * N for dA and D for dD / dbias; the caller may pack the three into one [parts][D * N +
// 2D] buffer, ld_part = D * N + 2D, and sum them with one reduction); gloc is a workspace of rdx_scan2_rec_elems
// floats; dBC [dirs][B][L][2N] is zeroed here (by the first kernel) and accumulated by the second.
extern "C" int rdx_scan2_bwd(int dtype, const void* u, const void* delta, const float* A_log, const void* Bm,
                             const void* Cm, int64_t ldbc, const float* Dp, const float* dt_bias, const float* ckpt,
                             const float* P, const float* dy, int64_t dy_dir_stride, void* du, void* ddelta,
                             float* dBC, float* dA_part, float* dD_part, float* dbias_part, int64_t ld_part,
                             float* gloc, int B, int L, int D, int N, int dirs, void* stream) {
  RDX_REQUIRE(u && delta && A_log && Bm && Cm && Dp && dt_bias && ckpt && P && dy && du && ddelta && dBC);
  RDX_REQUIRE(dA_part && dD_part && dbias_part && gloc);
  RDX_REQUIRE(B > 0 && L > 0 && D > 0 && (dirs == 1 || dirs == 2) && ldbc >= N && dy_dir_stride >= 0);
  RDX_REQUIRE(ld_part == 0 || ld_part >= (int64_t)D * N);
  if (N != s2::N) return RDX_EUNSUPPORTED;
  const int64_t ldpa = ld_part ? ld_part : (int64_t)D * N, ldpd = ld_part ? ld_part : (int64_t)D;
  const dim3 grid((D + s2::CH - 1) / s2::CH, rdx_scan2_chunks(L), dirs * B);
  hipStream_t st = as_stream(stream);
  if (dtype == RDX_BF16) {
    using T = hst;
    hipLaunchKernelGGL(s2::bwd_chunk_kernel<T>, grid, dim3(s2::NT), 0, st, (const T*)delta, A_log, (const T*)Cm,
                       ldbc, dt_bias, dy, dy_dir_stride, gloc, dBC, B, L, D);
    RDX_LAUNCH_CHECK();
    hipLaunchKernelGGL(s2::bwd_out_kernel<T>, grid, dim3(s2::NT), 0, st, (const T*)u, (const T*)delta, A_log,
                       (const T*)Bm, (const T*)Cm, ldbc, Dp, dt_bias, ckpt, P, gloc, dy, dy_dir_stride, (T*)du,
                       (T*)ddelta, dBC, dA_part, dD_part, dbias_part, ldpa, ldpd, B, L, D);
  } else if (dtype == RDX_F32) {
    using T = float;
    hipLaunchKernelGGL(s2::bwd_chunk_kernel<T>, grid, dim3(s2::NT), 0, st, (const T*)delta, A_log, (const T*)Cm,
                       ldbc, dt_bias, dy, dy_dir_stride, gloc, dBC, B, L, D);
    RDX_LAUNCH_CHECK();
    hipLaunchKernelGGL(s2::bwd_out_kernel<T>, grid, dim3(s2::NT), 0, st, (const T*)u, (const T*)delta, A_log,
                       (const T*)Bm, (const T*)Cm, ldbc, Dp, dt_bias, ckpt, P, gloc, dy, dy_dir_stride, (T*)du,
                       (T*)ddelta, dBC, dA_part, dD_part, dbias_part, ldpa, ldpd, B, L, D);
  } else {
    return RDX_EINVAL;
  }
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
