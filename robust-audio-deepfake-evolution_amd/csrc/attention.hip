// WavLM self-attention with the gated relative-position bias, fused, on gfx950 MFMA (bf16 in, fp32
// accumulate), forward and backward.
//
// Reference: HF WavLMAttention (transformers modeling_wavlm.py) as used by WavLMFrontend
// (src/models/DualStreamSEMamba.py:292-439): per head h
//     bias[b,h,i,j] = gate[b,i,h] * pb[h,i,j]      (gated rel-pos bias; gate depends on the layer input)
//     P = softmax(Q K^T / sqrt(64) + bias),  O = dropout(P) V
// The [B,H,T,T] bias is never materialised: it is formed in registers from gate and the shared
// position bias pb, and the backward returns d gate = sum_j dS[i,j] pb[h,i,j] directly (pb comes from
// the frozen rel_attn_embed table). Dropout keeps element (b,h,i,j) iff a counter hash of
// (seed, index) >= p * 2^32, so the backward regenerates the same mask; the seed is read from device
// memory, which keeps the launch replayable inside a HIP graph.
//
// Tiling: one wave per 32-row tile; mfma_f32_32x32x16_bf16 (A: lane (r, h) holds A[r][8h + j],
// B: B[8h + j][r], C: col = lane & 31, row = (i & 3) + 8 (i >> 2) + 4h). T = 201 is covered by 7
// tiles of 32 keys; Dh = 64 = 4 k-steps.
//   forward   S^T = K Q^T (query on the lane, keys in registers), online softmax over key tiles,
//             O^T += V^T P^T with P^T taken straight from the accumulator (B operand) and V^T from LDS.
//   dK, dV    key-stationary: S = Q K^T, dP = dO V^T (query rows in registers), dV += P^T dO and
//             dK += dS^T Q with P / dS as the A operand and dO^T / Q^T from LDS.
//   dQ, dgate query-stationary: S^T, dP^T as the forward, dQ^T += K^T dS^T (K^T from LDS); the gate
//             gradient is a lane-local sum plus one cross-half exchange.
//   D         rowsum(dO o O) per (b, h, i), the softmax-backward correction.
#include "common.h"

namespace rdx {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
constexpr int AT_DH = 64;    // head dim
constexpr int AT_TILE = 32;  // rows per wave
constexpr int AT_LDP = AT_TILE + 4;  // padded LDS row (bf16) for transposed tiles
// waves per block splitting the inner (key or query) loop of each kernel
#ifndef AT_NS_FWD
#define AT_NS_FWD 4
#endif
#ifndef AT_NS_DKDV
#define AT_NS_DKDV 2
#endif
#ifndef AT_NS_DQ
#define AT_NS_DQ 4
#endif

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// C/D row held in accumulator register i by lane half h
__device__ __forceinline__ int crow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }
// k index (a row of the accumulator X) carried by element j of lane half h at k-step s when X is fed
// back as an MFMA operand (registers 8s .. 8s+7)
__device__ __forceinline__ int krow(int s, int j, int h) { return 16 * s + 8 * (j >> 2) + 4 * h + (j & 3); }

__device__ __forceinline__ bf16x8 pack8(const float* x) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)x[j];
  return r;
}
__device__ __forceinline__ bf16x8 load8(const __hip_bfloat16* p, bool ok) {
  if (!ok) {
    bf16x8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = (__bf16)0.f;
    return z;
  }
  return *reinterpret_cast<const bf16x8*>(p);
}
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// stage the 32 x 64 tile held as 4 row-fragments (lane (r, h): row r, cols 16s + 8h + j) transposed
// into LDS as t[col][row]
__device__ __forceinline__ void stage_t(__bf16 (*t)[AT_LDP], const bf16x8* f, int r, int h) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) t[16 * s + 8 * h + j][r] = f[s][j];
}
// operand fragment whose element j is t[row][krow(s, j, h)]
__device__ __forceinline__ bf16x8 read_t(const __bf16 (*t)[AT_LDP], int row, int s, int h) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = t[row][krow(s, j, h)];
  return r;
}

struct AttnArgs {
  const __hip_bfloat16 *q, *k, *v;
  int64_t ldq, ldk, ldv;
  const float* gate;  // [B, T, H]
  const float* pb;    // [H, T, T]
  const int64_t* seed_dev;
  int salt;
  uint32_t thr;   // p * 2^32 (0: no dropout)
  float inv_keep;  // 1 / (1 - p)
  float scale;
  int B, T, H;
};

// NS waves per block share one 32-query tile and split its key tiles (wave w takes kb = w, w + NS,
// ...); their online-softmax partials (m, l, O) are merged through LDS at the end. This multiplies the
// waves in flight by NS (T = 201 gives only 7 query tiles per (b, h)).
template <bool kDrop, int NS>
__global__ __launch_bounds__(64 * NS) void attn_fwd_kernel(AttnArgs a, __hip_bfloat16* __restrict__ o, int64_t ldo,
                                                           float* __restrict__ lse) {
  __shared__ __bf16 s_vt_all[NS][AT_DH][AT_LDP];
  __shared__ float s_m[AT_TILE], s_l[AT_TILE];
  __shared__ float s_o[2][16][64];
  const int w = threadIdx.x >> 6;
  __bf16 (*s_vt)[AT_LDP] = s_vt_all[w];
  const int lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int qb = blockIdx.x, head = blockIdx.y, b = blockIdx.z;
  const int T = a.T, H = a.H;
  const int qi = qb * AT_TILE + r;
  const bool qvalid = qi < T;
  const int qc = qvalid ? qi : T - 1;
  const int64_t col0 = (int64_t)head * AT_DH;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = load8(a.q + ((int64_t)b * T + qc) * a.ldq + col0 + 16 * s + 8 * hh, qvalid);
  const float g = a.gate[((int64_t)b * T + qc) * H + head];
  const float* pbrow = a.pb + ((int64_t)head * T + qc) * T;
  const uint64_t seed = kDrop ? attn_seed(a.seed_dev, a.salt) : 0;
  const uint64_t ibase = (((uint64_t)b * H + head) * T + qc) * (uint64_t)T;
  float m = -INFINITY, l = 0.f;
  f32x16 oacc[2] = {zero16(), zero16()};
  const int nkb = (T + AT_TILE - 1) / AT_TILE;
  const int niter = (nkb + NS - 1) / NS;  // equal trip counts keep the barriers uniform
  for (int it = 0; it < niter; ++it) {
    const int kb = w + NS * it;
    const int kr = kb * AT_TILE + r;
    const bool kvalid = kr < T;
    f32x16 sacc = zero16();
    bf16x8 vfr[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 kf = load8(a.k + ((int64_t)b * T + kr) * a.ldk + col0 + 16 * s + 8 * hh, kvalid);
      sacc = mfma32(kf, qf[s], sacc);
      vfr[s] = load8(a.v + ((int64_t)b * T + kr) * a.ldv + col0 + 16 * s + 8 * hh, kvalid);
    }
    stage_t(s_vt, vfr, r, hh);
    float sv[16];
    float mloc = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = kb * AT_TILE + crow(i, hh);
      float x = -INFINITY;
      if (key < T) x = fmaf(sacc[i], a.scale, g * pbrow[key]);
      sv[i] = x;
      mloc = fmaxf(mloc, x);
    }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float mnew = fmaxf(m, mloc);
    const float alpha = mnew == -INFINITY ? 1.f : __expf(m - mnew);
    float lsum = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = sv[i] == -INFINITY ? 0.f : __expf(sv[i] - mnew);
      lsum += p;
      if (kDrop) {
        const int key = kb * AT_TILE + crow(i, hh);
        sv[i] = drop_keep(seed, ibase + key, a.thr) ? p * a.inv_keep : 0.f;
      } else {
        sv[i] = p;
      }
    }
    lsum += __shfl_xor(lsum, 32, 64);
    l = l * alpha + lsum;
    m = mnew;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      oacc[0][i] *= alpha;
      oacc[1][i] *= alpha;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 pf = pack8(sv + 8 * s);
#pragma unroll
      for (int db = 0; db < 2; ++db) oacc[db] = mfma32(read_t(s_vt, db * 32 + r, s, hh), pf, oacc[db]);
    }
    __syncthreads();
  }
  // merge the NS partials into wave 0
  for (int src = 1; src < NS; ++src) {
    __syncthreads();
    if (w == src) {
      if (hh == 0) {
        s_m[r] = m;
        s_l[r] = l;
      }
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int i = 0; i < 16; ++i) s_o[db][i][lane] = oacc[db][i];
    }
    __syncthreads();
    if (w == 0) {
      const float mw = s_m[r], lw = s_l[r];
      if (mw != -INFINITY) {
        const float mnew = fmaxf(m, mw);
        const float a0 = __expf(m - mnew), a1 = __expf(mw - mnew);
        l = l * a0 + lw * a1;
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
          for (int i = 0; i < 16; ++i) oacc[db][i] = oacc[db][i] * a0 + s_o[db][i][lane] * a1;
        m = mnew;
      }
    }
  }
  if (w == 0 && qvalid) {
    const float inv = 1.f / l;
    __hip_bfloat16* orow = o + ((int64_t)b * T + qi) * ldo + col0;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int i = 0; i < 16; ++i) orow[db * 32 + crow(i, hh)] = __float2bfloat16(oacc[db][i] * inv);
    if (hh == 0) lse[((int64_t)b * H + head) * T + qi] = m + __logf(l);
  }
}

// D[b, h, i] = sum_d dO[b, i, h, d] * O[b, i, h, d]
__global__ __launch_bounds__(256) void attn_bwd_dot_kernel(const __hip_bfloat16* __restrict__ dO, int64_t lddo,
                                                           const __hip_bfloat16* __restrict__ O, int64_t ldo,
                                                           float* __restrict__ D, int B, int T, int H) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (b, i, h)
  if (t >= (int64_t)B * T * H) return;
  const int head = (int)(t % H);
  const int64_t bi = t / H;
  const int b = (int)(bi / T), i = (int)(bi - (int64_t)b * T);
  const __hip_bfloat16* x = dO + bi * lddo + head * AT_DH;
  const __hip_bfloat16* y = O + bi * ldo + head * AT_DH;
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < AT_DH / 8; ++c) {
    const bf16x8 u = *reinterpret_cast<const bf16x8*>(x + 8 * c);
    const bf16x8 w = *reinterpret_cast<const bf16x8*>(y + 8 * c);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = fmaf((float)u[j], (float)w[j], acc);
  }
  D[((int64_t)b * H + head) * T + i] = acc;
}

struct AttnBwdArgs {
  const __hip_bfloat16* dO;
  int64_t lddo;
  const float* lse;  // [B, H, T]
  const float* D;    // [B, H, T]
};

// NS waves per block share one 32-key tile and split its query tiles; dK/dV partials are summed
// through LDS at the end.
template <bool kDrop, int NS>
__global__ __launch_bounds__(64 * NS) void attn_bwd_dkdv_kernel(AttnArgs a, AttnBwdArgs g,
                                                                __hip_bfloat16* __restrict__ dk,
                                                                __hip_bfloat16* __restrict__ dv, int64_t ldg) {
  __shared__ __bf16 s_qt_all[NS][AT_DH][AT_LDP];
  __shared__ __bf16 s_dot_all[NS][AT_DH][AT_LDP];
  __shared__ float s_acc[4][16][64];
  const int w = threadIdx.x >> 6;
  __bf16 (*s_qt)[AT_LDP] = s_qt_all[w];
  __bf16 (*s_dot)[AT_LDP] = s_dot_all[w];
  const int lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int kb = blockIdx.x, head = blockIdx.y, b = blockIdx.z;
  const int T = a.T, H = a.H;
  const int key = kb * AT_TILE + r;  // this lane's key column
  const bool kvalid = key < T;
  const int64_t col0 = (int64_t)head * AT_DH;
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = load8(a.k + ((int64_t)b * T + key) * a.ldk + col0 + 16 * s + 8 * hh, kvalid);
    vf[s] = load8(a.v + ((int64_t)b * T + key) * a.ldv + col0 + 16 * s + 8 * hh, kvalid);
  }
  const uint64_t seed = kDrop ? attn_seed(a.seed_dev, a.salt) : 0;
  const int64_t bh = (int64_t)b * H + head;
  f32x16 dkacc[2] = {zero16(), zero16()}, dvacc[2] = {zero16(), zero16()};
  const int nqb = (T + AT_TILE - 1) / AT_TILE;
  const int niter = (nqb + NS - 1) / NS;
  for (int it = 0; it < niter; ++it) {
    const int qb = w + NS * it;
    const int qr = qb * AT_TILE + r;  // row loaded by this lane for the A fragments
    const bool qrv = qr < T;
    bf16x8 qa[4], da[4];
    f32x16 S = zero16(), dP = zero16();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qa[s] = load8(a.q + ((int64_t)b * T + qr) * a.ldq + col0 + 16 * s + 8 * hh, qrv);
      da[s] = load8(g.dO + ((int64_t)b * T + qr) * g.lddo + col0 + 16 * s + 8 * hh, qrv);
      S = mfma32(qa[s], kf[s], S);
      dP = mfma32(da[s], vf[s], dP);
    }
    stage_t(s_qt, qa, r, hh);
    stage_t(s_dot, da, r, hh);
    float P[16], dS[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qi = qb * AT_TILE + crow(i, hh);
      float p = 0.f, ds = 0.f;
      if (qi < T && kvalid) {
        const float gq = a.gate[((int64_t)b * T + qi) * H + head];
        const float s = fmaf(S[i], a.scale, gq * a.pb[((int64_t)head * T + qi) * T + key]);
        p = __expf(s - g.lse[bh * T + qi]);
        float mk = 1.f;
        if (kDrop) mk = drop_keep(seed, ((uint64_t)bh * T + qi) * (uint64_t)T + key, a.thr) ? a.inv_keep : 0.f;
        ds = p * (dP[i] * mk - g.D[bh * T + qi]);
        p *= mk;
      }
      P[i] = p;
      dS[i] = ds;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 xp = pack8(P + 8 * s), xs = pack8(dS + 8 * s);
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        dvacc[db] = mfma32(xp, read_t(s_dot, db * 32 + r, s, hh), dvacc[db]);
        dkacc[db] = mfma32(xs, read_t(s_qt, db * 32 + r, s, hh), dkacc[db]);
      }
    }
    __syncthreads();
  }
  for (int src = 1; src < NS; ++src) {
    __syncthreads();
    if (w == src) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        s_acc[0][i][lane] = dkacc[0][i];
        s_acc[1][i][lane] = dkacc[1][i];
        s_acc[2][i][lane] = dvacc[0][i];
        s_acc[3][i][lane] = dvacc[1][i];
      }
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        dkacc[0][i] += s_acc[0][i][lane];
        dkacc[1][i] += s_acc[1][i][lane];
        dvacc[0][i] += s_acc[2][i][lane];
        dvacc[1][i] += s_acc[3][i][lane];
      }
    }
  }
  if (w != 0) return;
  // Z[key][d]: col = d (lane), row = key (registers)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int kk = kb * AT_TILE + crow(i, hh);
    if (kk < T) {
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const int64_t off = ((int64_t)b * T + kk) * ldg + col0 + db * 32 + r;
        dk[off] = __float2bfloat16(dkacc[db][i] * a.scale);
        dv[off] = __float2bfloat16(dvacc[db][i]);
      }
    }
  }
}

// NS waves per block share one 32-query tile and split its key tiles; dQ / dgate partials are
// summed through LDS at the end.
template <bool kDrop, int NS>
__global__ __launch_bounds__(64 * NS) void attn_bwd_dq_kernel(AttnArgs a, AttnBwdArgs g,
                                                              __hip_bfloat16* __restrict__ dq, int64_t ldg,
                                                              float* __restrict__ dgate) {
  __shared__ __bf16 s_kt_all[NS][AT_DH][AT_LDP];
  __shared__ float s_acc[2][16][64];
  __shared__ float s_dg[64];
  const int w = threadIdx.x >> 6;
  __bf16 (*s_kt)[AT_LDP] = s_kt_all[w];
  const int lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int qb = blockIdx.x, head = blockIdx.y, b = blockIdx.z;
  const int T = a.T, H = a.H;
  const int qi = qb * AT_TILE + r;
  const bool qvalid = qi < T;
  const int qc = qvalid ? qi : T - 1;
  const int64_t col0 = (int64_t)head * AT_DH;
  bf16x8 qf[4], dof[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = load8(a.q + ((int64_t)b * T + qc) * a.ldq + col0 + 16 * s + 8 * hh, qvalid);
    dof[s] = load8(g.dO + ((int64_t)b * T + qc) * g.lddo + col0 + 16 * s + 8 * hh, qvalid);
  }
  const int64_t bh = (int64_t)b * H + head;
  const float gq = a.gate[((int64_t)b * T + qc) * H + head];
  const float lq = g.lse[bh * T + qc];
  const float Dq = g.D[bh * T + qc];
  const float* pbrow = a.pb + ((int64_t)head * T + qc) * T;
  const uint64_t seed = kDrop ? attn_seed(a.seed_dev, a.salt) : 0;
  const uint64_t ibase = ((uint64_t)bh * T + qc) * (uint64_t)T;
  f32x16 dqacc[2] = {zero16(), zero16()};
  float dg = 0.f;
  const int nkb = (T + AT_TILE - 1) / AT_TILE;
  const int niter = (nkb + NS - 1) / NS;
  for (int it = 0; it < niter; ++it) {
    const int kb = w + NS * it;
    const int kr = kb * AT_TILE + r;
    const bool krv = kr < T;
    bf16x8 kfr[4];
    f32x16 S = zero16(), dP = zero16();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kfr[s] = load8(a.k + ((int64_t)b * T + kr) * a.ldk + col0 + 16 * s + 8 * hh, krv);
      const bf16x8 vfr = load8(a.v + ((int64_t)b * T + kr) * a.ldv + col0 + 16 * s + 8 * hh, krv);
      S = mfma32(kfr[s], qf[s], S);
      dP = mfma32(vfr, dof[s], dP);
    }
    stage_t(s_kt, kfr, r, hh);
    float dS[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = kb * AT_TILE + crow(i, hh);
      float ds = 0.f;
      if (key < T && qvalid) {
        const float pbv = pbrow[key];
        const float p = __expf(fmaf(S[i], a.scale, gq * pbv) - lq);
        float mk = 1.f;
        if (kDrop) mk = drop_keep(seed, ibase + key, a.thr) ? a.inv_keep : 0.f;
        ds = p * (dP[i] * mk - Dq);
        dg = fmaf(ds, pbv, dg);
      }
      dS[i] = ds;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 xs = pack8(dS + 8 * s);
#pragma unroll
      for (int db = 0; db < 2; ++db) dqacc[db] = mfma32(read_t(s_kt, db * 32 + r, s, hh), xs, dqacc[db]);
    }
    __syncthreads();
  }
  for (int src = 1; src < NS; ++src) {
    __syncthreads();
    if (w == src) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        s_acc[0][i][lane] = dqacc[0][i];
        s_acc[1][i][lane] = dqacc[1][i];
      }
      s_dg[lane] = dg;
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        dqacc[0][i] += s_acc[0][i][lane];
        dqacc[1][i] += s_acc[1][i][lane];
      }
      dg += s_dg[lane];
    }
  }
  if (w != 0) return;
  dg += __shfl_xor(dg, 32, 64);
  if (qvalid) {
    __hip_bfloat16* row = dq + ((int64_t)b * T + qi) * ldg + col0;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int i = 0; i < 16; ++i) row[db * 32 + crow(i, hh)] = __float2bfloat16(dqacc[db][i] * a.scale);
    if (hh == 0) dgate[((int64_t)b * T + qi) * H + head] = dg;
  }
}

// element-wise dropout mask of the same hash (tests only): keep[b, h, i, j] in {0, 1}
__global__ void attn_mask_kernel(const int64_t* seed_dev, int salt, uint32_t thr, uint8_t* keep, int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) keep[t] = drop_keep(attn_seed(seed_dev, salt), (uint64_t)t, thr) ? 1 : 0;
}

inline AttnArgs make_args(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                          const float* gate, const float* pb, const int64_t* seed_dev, int salt, float p_drop,
                          float scale, int B, int T, int H) {
  AttnArgs a;
  a.q = (const __hip_bfloat16*)q;
  a.k = (const __hip_bfloat16*)k;
  a.v = (const __hip_bfloat16*)v;
  a.ldq = ldq;
  a.ldk = ldk;
  a.ldv = ldv;
  a.gate = gate;
  a.pb = pb;
  a.seed_dev = seed_dev;
  a.salt = salt;
  const double t = (double)p_drop * 4294967296.0;
  a.thr = p_drop > 0.f ? (uint32_t)(t >= 4294967295.0 ? 4294967295.0 : t) : 0u;
  a.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  a.scale = scale;
  a.B = B;
  a.T = T;
  a.H = H;
  return a;
}

}  // namespace rdx

using namespace rdx;

static bool attn_ok(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv, int B,
                    int T, int H) {
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  return q && k && v && al(q) && al(k) && al(v) && B > 0 && T > 0 && H > 0 && B <= 65535 && H <= 65535 &&
         ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldq >= (int64_t)H * AT_DH && ldk >= (int64_t)H * AT_DH &&
         ldv >= (int64_t)H * AT_DH;
}

extern "C" int rdx_attn_fwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                            const float* gate, const float* pos_bias, const int64_t* seed_dev, int salt,
                            float p_drop, float scale, void* o, int64_t ldo, float* lse, int B, int T, int H,
                            int head_dim, void* stream) {
  RDX_REQUIRE(attn_ok(q, ldq, k, ldk, v, ldv, B, T, H) && gate && pos_bias && o && lse && ldo >= (int64_t)H * AT_DH);
  RDX_REQUIRE(p_drop >= 0.f && p_drop < 1.f && (p_drop == 0.f || seed_dev));
  if (head_dim != AT_DH) return RDX_EUNSUPPORTED;
  const AttnArgs a = make_args(q, ldq, k, ldk, v, ldv, gate, pos_bias, seed_dev, salt, p_drop, scale, B, T, H);
  dim3 grid((T + AT_TILE - 1) / AT_TILE, H, B);
  if (a.thr)
    hipLaunchKernelGGL((attn_fwd_kernel<true, AT_NS_FWD>), grid, dim3(64 * AT_NS_FWD), 0, as_stream(stream), a,
                       (__hip_bfloat16*)o, ldo, lse);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<false, AT_NS_FWD>), grid, dim3(64 * AT_NS_FWD), 0, as_stream(stream), a,
                       (__hip_bfloat16*)o, ldo, lse);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_attn_bwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                            const float* gate, const float* pos_bias, const int64_t* seed_dev, int salt,
                            float p_drop, float scale, const void* o, int64_t ldo, const float* lse,
                            const void* dout, int64_t lddo, float* D, void* dq, void* dk, void* dv, int64_t ldg,
                            float* dgate, int B, int T, int H, int head_dim, void* stream) {
  RDX_REQUIRE(attn_ok(q, ldq, k, ldk, v, ldv, B, T, H) && gate && pos_bias && o && lse && dout && D);
  RDX_REQUIRE(dq && dk && dv && dgate && ldg >= (int64_t)H * AT_DH && ldg % 8 == 0 && lddo % 8 == 0);
  RDX_REQUIRE(p_drop >= 0.f && p_drop < 1.f && (p_drop == 0.f || seed_dev));
  if (head_dim != AT_DH) return RDX_EUNSUPPORTED;
  const AttnArgs a = make_args(q, ldq, k, ldk, v, ldv, gate, pos_bias, seed_dev, salt, p_drop, scale, B, T, H);
  hipStream_t st = as_stream(stream);
  const int64_t nrow = (int64_t)B * T * H;
  hipLaunchKernelGGL(attn_bwd_dot_kernel, dim3((unsigned)((nrow + 255) / 256)), dim3(256), 0, st,
                     (const __hip_bfloat16*)dout, lddo, (const __hip_bfloat16*)o, ldo, D, B, T, H);
  RDX_LAUNCH_CHECK();
  AttnBwdArgs g{(const __hip_bfloat16*)dout, lddo, lse, D};
  dim3 grid((T + AT_TILE - 1) / AT_TILE, H, B);
  if (a.thr) {
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<true, AT_NS_DKDV>), grid, dim3(64 * AT_NS_DKDV), 0, st, a, g,
                       (__hip_bfloat16*)dk, (__hip_bfloat16*)dv, ldg);
    hipLaunchKernelGGL((attn_bwd_dq_kernel<true, AT_NS_DQ>), grid, dim3(64 * AT_NS_DQ), 0, st, a, g,
                       (__hip_bfloat16*)dq, ldg, dgate);
  } else {
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<false, AT_NS_DKDV>), grid, dim3(64 * AT_NS_DKDV), 0, st, a, g,
                       (__hip_bfloat16*)dk, (__hip_bfloat16*)dv, ldg);
    hipLaunchKernelGGL((attn_bwd_dq_kernel<false, AT_NS_DQ>), grid, dim3(64 * AT_NS_DQ), 0, st, a, g,
                       (__hip_bfloat16*)dq, ldg, dgate);
  }
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_attn_dropout_mask(const int64_t* seed_dev, int salt, float p_drop, uint8_t* keep, int64_t n,
                                     void* stream) {
  RDX_REQUIRE(seed_dev && keep && n > 0 && p_drop >= 0.f && p_drop < 1.f);
  const AttnArgs a = make_args(nullptr, 0, nullptr, 0, nullptr, 0, nullptr, nullptr, seed_dev, salt, p_drop, 1.f, 1, 1, 1);
  hipLaunchKernelGGL(attn_mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), seed_dev,
                     salt, a.thr, keep, n);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
