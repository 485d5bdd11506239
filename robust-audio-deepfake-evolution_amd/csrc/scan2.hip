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
//   fwd 1b carry-in of every chunk = compose(P_k, hloc_k) over the chunks before it (one thread per (dir, b, d, n),
//          in place over hloc);
//   fwd 2  the chunk from the true carry: y (staged in LDS, coalesced rows) and the checkpoint at the chunk end;
//   bwd 1  each chunk's reverse carry from 0 (G_s = C_s dy_s + a_{s+1} G_{s+1}): gloc_c = a_{s0} G_{s0};
//   bwd 1b carry from the right = compose(P_k, gloc_k) over the chunks after it (in place over gloc);
//   bwd 2  states re-run from the chunk's checkpoint, then every gradient of the chunk.
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

// The per-step sums over the 16 states (y, d dt, d u) and over the block's channels (dB, dC) do not feed the
// recurrence, so the kernels keep each step's per-lane term in registers and reduce all 16 steps at the chunk end
// in one transposed pass: 15 lane exchanges per array instead of 16 x 4 (over states), 12 instead of 16 x 2 (over a
// wave's 4 channels). The kernels are VALU-issue-bound (every step's work is per (channel, state) lane).
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// v[k] of every lane of a 16-lane row -> lane n gets the row's total of v[n] (butterfly over lane bits 3..0: xor 8
// by row_ror, xor 4 by a bit-mode ds_swizzle, xor 2 / xor 1 by quad_perm). Every exchange runs with the whole wave
// active: a DPP read of a lane that is switched off returns the bound value, so a lane-dependent choice between two
// DPP patterns (which the compiler turns into two exec-masked halves) would read zeros.
__device__ __forceinline__ float row_tr_sum16(const float* v, int n) {
  const bool b3 = n & 8, b2 = n & 4, b1 = n & 2, b0 = n & 1;
  float w8[8], w4[4], w2[2];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float keep = b3 ? v[j + 8] : v[j], send = b3 ? v[j] : v[j + 8];
    w8[j] = keep + dppf<0x128>(send);                                        // row_ror:8 = xor 8
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float keep = b2 ? w8[j + 4] : w8[j], send = b2 ? w8[j] : w8[j + 4];
    w4[j] = keep + __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(send), 0x101F));   // xor 4
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float keep = b1 ? w4[j + 2] : w4[j], send = b1 ? w4[j] : w4[j + 2];
    w2[j] = keep + dppf<0x4E>(send);                                         // quad_perm [2,3,0,1]
  }
  const float keep = b0 ? w2[1] : w2[0], send = b0 ? w2[0] : w2[1];
  return keep + dppf<0xB1>(send);                                            // quad_perm [1,0,3,2]
}
// v[k] of every lane -> x[j] = total of v[4 r + j] over the wave's 4 rows (lanes l, l ^ 16, l ^ 32, l ^ 48), in
// every lane of row r: permlane32_swap (lanes 32-63 of the first operand <-> lanes 0-31 of the second), then
// permlane16_swap (odd rows of the first <-> even rows of the second)
__device__ __forceinline__ void rows_tr_sum4(const float* v, float* x) {
  float w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[j]), __float_as_uint(v[j + 8]), false, false);
    w[j] = __uint_as_float(p[0]) + __uint_as_float(p[1]);   // lanes 0-31: index j, lanes 32-63: j + 8
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(w[j]), __float_as_uint(w[j + 4]), false, false);
    x[j] = __uint_as_float(p[0]) + __uint_as_float(p[1]);   // row r: index j + 4 r
  }
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

// ---- fwd 1b / bwd 1b: the carry entering every chunk, in place over the chunk-local records, one thread per (dir,
// b, d, n): forward rec_c <- compose(P_k, rec_k) over k < c in step order, backward over k > c nearest last (the FMA
// chains the output kernels ran per thread before: 2 loads per chunk once instead of up to 2 x 16 in each of the
// 512 threads of every block)
template <int REVERSE>     // a template argument only so that profiles tell the forward's launches from the backward's
__global__ __launch_bounds__(256) void carry_kernel(const float* __restrict__ P, float* __restrict__ recs, int64_t DN,
                                                    int nc, int64_t total) {
  constexpr bool reverse = REVERSE != 0;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= total) return;
  const int64_t db = t / DN;
  const int64_t base = db * nc * DN + (t - db * DN);   // record (db, chunk, d, n) = (db * nc + chunk) * DN + d * N + n
  float h = 0.f;
  for (int k0 = 0; k0 < nc; k0 += CK) {     // 16 chunks' loads in flight at once, then the FMA chain
    const int m = min(CK, nc - k0);
    float r[CK], p[CK];
    int64_t o[CK];
#pragma unroll
    for (int k = 0; k < CK; ++k) {
      const int kk = k0 + min(k, m - 1);
      o[k] = base + (int64_t)(reverse ? nc - 1 - kk : kk) * DN;
      r[k] = recs[o[k]];
      p[k] = P[o[k]];
    }
#pragma unroll
    for (int k = 0; k < CK; ++k) {
      if (k < m) {
        recs[o[k]] = h;
        h = fmaf(p[k], h, r[k]);
      }
    }
  }
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
  // carry-in from the chunks before this one (composed in step order by carry_kernel)
  float h = g.active ? hloc[rec(g, g.c, D)] : 0.f;
  __syncthreads();
  const float A2 = g.active ? -__expf(A_log[g.d * N + g.n]) * LOG2E : 0.f;
  const float Dd = g.active ? Dp[g.d] : 0.f;
  float pv[CK];     // this state's C_s h_s terms, summed over the states at the chunk end
#pragma unroll
  for (int i = 0; i < CK; ++i) {
    pv[i] = 0.f;
    if (i < g.cnt) {    // block-uniform
      const float dtv = s_dt[i * CH + g.dl];
      const float a = __builtin_amdgcn_exp2f(dtv * A2);
      h = fmaf(a, h, dtv * s_u[i * CH + g.dl] * s_B[i * N + g.n]);
      pv[i] = s_C[i * N + g.n] * h;
    }
  }
  if (g.active && g.c < g.nc - 1) ckpt[(((int64_t)g.db * (g.nc - 1) + g.c) * D + g.d) * N + g.n] = h;
  {
    const float yv = row_tr_sum16(pv, g.n);   // lane n: step n of channel dl
    s_y[g.n * CH + g.dl] = fmaf(Dd, s_u[g.n * CH + g.dl], yv);
  }
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
  // the carry entering from the right (the later chunks composed nearest last by carry_kernel)
  float X = 0.f, h0 = 0.f;
  if (g.active) {
    X = gloc[rec(g, g.c, D)];
    if (g.c > 0) h0 = ckpt[(((int64_t)g.db * (g.nc - 1) + (g.c - 1)) * D + g.d) * N + g.n];
  }
  __syncthreads();
  const float Aval = g.active ? -__expf(A_log[g.d * N + g.n]) : 0.f;
  const float A2 = Aval * LOG2E;
  const float Dd = g.active ? Dp[g.d] : 0.f;
  // states of the chunk from its checkpoint, and their decays
  float hs[CK], av[CK];
  {
    float h = h0;
#pragma unroll
    for (int i = 0; i < CK; ++i) {
      av[i] = 1.f;
      if (i < g.cnt) {
        const float dtv = s_dt[i * CH + g.dl];
        av[i] = __builtin_amdgcn_exp2f(dtv * A2);
        h = fmaf(av[i], h, dtv * s_u[i * CH + g.dl] * s_B[i * N + g.n]);
      }
      hs[i] = h;
    }
  }
  // per step, this lane's terms of the sums over states (d dt, d u) and over channels (dB, dC); a channel past D
  // has u = dt = dy = 0 staged and X = h = 0, so every term of it is exactly 0
  float dA = 0.f;
  float tB[CK], tC[CK], tt[CK], tu[CK];
#pragma unroll
  for (int i = CK - 1; i >= 0; --i) {
    tB[i] = tC[i] = tt[i] = tu[i] = 0.f;
    if (i < g.cnt) {    // block-uniform
      const int o = i * CH + g.dl;
      const float dtv = s_dt[o], uu = s_u[o], dyv = s_dy[o];
      const float Bn = s_B[i * N + g.n], Cn = s_C[i * N + g.n];
      const float a = av[i];
      const float hprev = i > 0 ? hs[i > 0 ? i - 1 : 0] : h0;
      const float G = fmaf(Cn, dyv, X);
      const float ah = a * hprev;
      const float Gdt = G * dtv;
      tB[i] = Gdt * uu;
      tC[i] = dyv * hs[i];
      dA = fmaf(Gdt, ah, dA);
      tt[i] = G * fmaf(Aval, ah, Bn * uu);
      tu[i] = Gdt * Bn;
      X = a * G;
    }
  }
  // lane n of each row: step n of its channel (d dt, d u over the states); lane (row r, n): steps 4 r .. 4 r + 3
  // of dB / dC[n] over the wave's 4 channels
  const float ddt = row_tr_sum16(tt, g.n);
  const float dus = row_tr_sum16(tu, g.n);
  {
    float xb[4], xc[4];
    rows_tr_sum4(tB, xb);
    rows_tr_sum4(tC, xc);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s_red[4 * row + j][wave][g.n] = xb[j];
      s_red[4 * row + j][wave][N + g.n] = xc[j];
    }
  }
  float r_du = 0.f, r_dd = 0.f, dDt = 0.f;
  if (g.n < g.cnt) {
    const int o = g.n * CH + g.dl;
    const float dyv = s_dy[o];
    r_dd = ddt * s_sig[o];         // softplus'(pre) = sigmoid(pre) (= 1 - exp(-dt))
    r_du = fmaf(Dd, dyv, dus);
    dDt = dyv * s_u[o];
  }
  const float dDacc = row16_sum(dDt);
  const float dbacc = row16_sum(r_dd);
  __syncthreads();                           // every read of s_u / s_dt done: reuse them for du / ddelta
  s_u[g.n * CH + g.dl] = r_du;
  s_dt[g.n * CH + g.dl] = r_dd;
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

__host__ inline void launch_carry(const float* P, float* recs, int B, int L, int D, int dirs, int reverse,
                                 hipStream_t st) {
  const int64_t DN = (int64_t)D * N, total = (int64_t)dirs * B * DN;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (reverse)
    hipLaunchKernelGGL(carry_kernel<1>, grid, dim3(256), 0, st, P, recs, DN, (L + CK - 1) / CK, total);
  else
    hipLaunchKernelGGL(carry_kernel<0>, grid, dim3(256), 0, st, P, recs, DN, (L + CK - 1) / CK, total);
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
    s2::launch_carry(P, hloc, B, L, D, dirs, 0, st);
    hipLaunchKernelGGL(s2::fwd_out_kernel<T>, grid, dim3(s2::NT), 0, st, (const T*)u, (const T*)delta, A_log,
                       (const T*)Bm, (const T*)Cm, ldbc, Dp, dt_bias, hloc, P, y, ckpt, B, L, D);
  } else if (dtype == RDX_F32) {
    using T = float;
    hipLaunchKernelGGL(s2::fwd_chunk_kernel<T>, grid, dim3(s2::NT), 0, st, (const T*)u, (const T*)delta, A_log,
                       (const T*)Bm, ldbc, dt_bias, hloc, P, B, L, D);
    RDX_LAUNCH_CHECK();
    s2::launch_carry(P, hloc, B, L, D, dirs, 0, st);
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
    s2::launch_carry(P, gloc, B, L, D, dirs, 1, st);
    hipLaunchKernelGGL(s2::bwd_out_kernel<T>, grid, dim3(s2::NT), 0, st, (const T*)u, (const T*)delta, A_log,
                       (const T*)Bm, (const T*)Cm, ldbc, Dp, dt_bias, ckpt, P, gloc, dy, dy_dir_stride, (T*)du,
                       (T*)ddelta, dBC, dA_part, dD_part, dbias_part, ldpa, ldpd, B, L, D);
  } else if (dtype == RDX_F32) {
    using T = float;
    hipLaunchKernelGGL(s2::bwd_chunk_kernel<T>, grid, dim3(s2::NT), 0, st, (const T*)delta, A_log, (const T*)Cm,
                       ldbc, dt_bias, dy, dy_dir_stride, gloc, dBC, B, L, D);
    RDX_LAUNCH_CHECK();
    s2::launch_carry(P, gloc, B, L, D, dirs, 1, st);
    hipLaunchKernelGGL(s2::bwd_out_kernel<T>, grid, dim3(s2::NT), 0, st, (const T*)u, (const T*)delta, A_log,
                       (const T*)Bm, (const T*)Cm, ldbc, Dp, dt_bias, ckpt, P, gloc, dy, dy_dir_stride, (T*)du,
                       (T*)ddelta, dBC, dA_part, dD_part, dbias_part, ldpa, ldpd, B, L, D);
  } else {
    return RDX_EINVAL;
  }
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
