// Split-precision ("x3") kernels of the fp32 scoring pass: the WavLM-Large stream of the reference's eval forward
// (src/main.py:958-995 runs model(batch_x) with no autocast, comment at :974-975; the stream is
// src/models/DualStreamSEMamba.py:392-439 over HF WavLMModel) at fp32 accuracy on gfx950's bf16 matrix cores.
//
// An fp32 value x is carried as two bf16 planes, hi = bf16(x) and lo = bf16(x - hi) (|x - hi - lo| <= 2^-17 |x|).
// The GEMMs (csrc/hgemm.hip rdx_hgemm_x3) take those planes and sum Ahi.Bhi + Alo.Bhi + Ahi.Blo in fp32; the kernels
// here produce the planes where the stream makes them and do the stream's non-GEMM arithmetic in fp32:
//   rdx_x3_split       fp32 rows -> planes (the frozen weights, once; any fp32 activation)
//   rdx_x3_ln_split    [a + b ->] LayerNorm -> planes and / or fp32, with the gated-relative-position gate of
//                      HF WavLMAttention (sigmoid of the 2 x 4 summed gru_rel_pos_linear outputs per head)
//   rdx_x3_attn_fwd    softmax((q / 8) k^T + gate * rel_bias) v in fp32 on v_mfma_f32_16x16x4_f32 (exact fp32
//                      products; the attention is ~3 % of the encoder's flops), output as planes for out_proj
//   rdx_x3_posconv_fwd h + gelu(grouped conv1d(h) + bias) (HF WavLMPositionalConvEmbedding + the encoder's add), the
//                      fp32 input split while it is staged, three bf16 MFMA products per tap
//   rdx_x3_fe_conv0    CNN layer 0 (Conv1d 1 -> 512, k 10, s 5) + LayerNorm(512) + GELU in fp32 -> planes
//   rdx_x3_fe_ln_gelu  LayerNorm(512) + GELU of the fp32 output of CNN layers 1-6 -> planes (or fp32: the last)
// libradhip.so only: libradhip_f16.so exports the same names and returns RDX_EINVAL.
#include <algorithm>

#include "common.h"

namespace rdx {
namespace x3 {

#ifndef RDX_F16
// GELU (erf form) with erf by Abramowitz & Stegun 7.1.26 (common.h gelu: |erf error| <= 1.5e-7, i.e. within about
// one fp32 rounding of the result; erff's piecewise polynomial made the LayerNorm + GELU passes VALU-bound)
__device__ __forceinline__ float gelu_exact(float x) { return gelu(x); }

// hi / lo bf16 bits of x, packed in pairs
__device__ __forceinline__ void split_pack2(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = hpack2(a, b);
  lo = hpack2(a - hlo(hi), b - hhi(hi));
}
// n consecutive floats (n % 4 == 0) -> planes at ph / pl
template <int N>
__device__ __forceinline__ void store_split(hst* ph, hst* pl, const float* v) {
  static_assert(N % 4 == 0, "store_split");
#pragma unroll
  for (int i = 0; i < N; i += 4) {
    uint32_t h0, l0, h1, l1;
    split_pack2(v[i], v[i + 1], h0, l0);
    split_pack2(v[i + 2], v[i + 3], h1, l1);
    *reinterpret_cast<uint2*>(ph + i) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(pl + i) = make_uint2(l0, l1);
  }
}

// ---- fp32 rows -> planes -----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void split_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows, int cols,
                                                    hst* __restrict__ hi, hst* __restrict__ lo, int64_t ldo) {
  const int c4 = cols / 4;
  const int64_t n = rows * c4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / c4;
    const int c = (int)(i - r * c4) * 4;
    const float4 t = *reinterpret_cast<const float4*>(x + r * ldx + c);
    const float v[4] = {t.x, t.y, t.z, t.w};
    store_split<4>(hi + r * ldo + c, lo + r * ldo + c, v);
  }
}

// ---- [a + b ->] LayerNorm -> planes / fp32 (+ gate) ------------------------------------------------------------------
struct LnArgs {
  const float* a;        // [M, E] rows (ld E)
  const float* b;        // [M, E] or null: x = a + b
  float* sum_out;        // [M, E] or null: x written here (the residual stream)
  const float* gamma;
  const float* beta;
  float eps;
  hst* hi;               // [M, ldo] planes of LN(x), or null
  hst* lo;
  int64_t ldo;
  float* y32;            // [M, E] fp32 LN(x), or null
  const float* wg;       // gate: gru_rel_pos_linear [8, 64] weight, [8] bias, [H] gru_rel_pos_const; null: no gate
  const float* bg;
  const float* gconst;
  float* gate;           // [M, H]
  int64_t M;
};

template <int VPL, bool GATE>
__global__ __launch_bounds__(256) void ln_split_kernel(LnArgs a) {
  constexpr int E = 64 * VPL;
  __shared__ __attribute__((aligned(16))) float swg[GATE ? 8 * 64 : 4];
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const bool live = m < a.M;
  const int e0 = lane * VPL;
  float v[VPL], gm[VPL], bt[VPL];
  if (live) {
#pragma unroll
    for (int i = 0; i < VPL; i += 4) {
      float4 t = *reinterpret_cast<const float4*>(a.a + m * E + e0 + i);
      if (a.b) {
        const float4 u = *reinterpret_cast<const float4*>(a.b + m * E + e0 + i);
        t = make_float4(t.x + u.x, t.y + u.y, t.z + u.z, t.w + u.w);
      }
      v[i] = t.x, v[i + 1] = t.y, v[i + 2] = t.z, v[i + 3] = t.w;
      const float4 g4 = *reinterpret_cast<const float4*>(a.gamma + e0 + i);
      const float4 b4 = *reinterpret_cast<const float4*>(a.beta + e0 + i);
      gm[i] = g4.x, gm[i + 1] = g4.y, gm[i + 2] = g4.z, gm[i + 3] = g4.w;
      bt[i] = b4.x, bt[i + 1] = b4.y, bt[i + 2] = b4.z, bt[i + 3] = b4.w;
    }
  }
  if constexpr (GATE) {
    for (int i = threadIdx.x; i < 8 * 64 / 4; i += 256)
      reinterpret_cast<float4*>(swg)[i] = reinterpret_cast<const float4*>(a.wg)[i];
    __syncthreads();
  }
  if (!live) return;
  if (a.sum_out) {
#pragma unroll
    for (int i = 0; i < VPL; i += 4)
      *reinterpret_cast<float4*>(a.sum_out + m * E + e0 + i) = make_float4(v[i], v[i + 1], v[i + 2], v[i + 3]);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) s += v[i];
  const float mean = wave_sum(s) * (1.0f / E);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const float d = v[i] - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(wave_sum(q) * (1.0f / E) + a.eps);
#pragma unroll
  for (int i = 0; i < VPL; ++i) v[i] = (v[i] - mean) * rstd * gm[i] + bt[i];
  if (a.hi) store_split<VPL>(a.hi + m * a.ldo + e0, a.lo + m * a.ldo + e0, v);
  if (a.y32) {
#pragma unroll
    for (int i = 0; i < VPL; i += 4)
      *reinterpret_cast<float4*>(a.y32 + m * E + e0 + i) = make_float4(v[i], v[i + 1], v[i + 2], v[i + 3]);
  }
  if constexpr (GATE) {
    static_assert(VPL == 16, "gate: 4 lanes per 64-dim head");
    // gate pre-activations of this lane's head (lanes 4h .. 4h + 3 hold its 64 dims)
    const int part = lane & 3;
    float z[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float* w = swg + j * 64 + part * 16;
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc = fmaf(w[i], v[i], acc);
      acc += __shfl_xor(acc, 1, 64);
      acc += __shfl_xor(acc, 2, 64);
      z[j] = acc + a.bg[j];
    }
    if (part == 0) {
      const int head = lane >> 2;
      const float ga = 1.0f / (1.0f + expf(-(z[0] + z[1] + z[2] + z[3])));
      const float gb = 1.0f / (1.0f + expf(-(z[4] + z[5] + z[6] + z[7])));
      a.gate[m * (E / 64) + head] = ga * (gb * a.gconst[head] - 1.0f) + 2.0f;
    }
  }
}

// ---- fp32 gated-relative-position attention -> planes --------------------------------------------------------------
// One workgroup per (utterance, head) [and query group], one wave per 16 query rows. K and V of the (b, h) are staged
// once in LDS (fp32, padded rows). A wave computes S^T = K Q^T (16 keys x 16 queries per 16x16x4 MFMA tile, the key
// tiles in registers), the softmax down each query column (4 registers x key tiles per lane, then lanes l ^ 16,
// l ^ 32), and O^T = V^T P^T with P^T taken straight from the S^T registers as the B operand.
constexpr int AT_KS = 68;    // K row stride in LDS (floats)
constexpr int AT_VS = 80;    // V row stride

typedef __attribute__((ext_vector_type(4))) float f4v;

template <int NTM>
__global__ __launch_bounds__(1024) void attn_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                    const float* __restrict__ v, int64_t ld,
                                                    const float* __restrict__ gate, const float* __restrict__ rel,
                                                    float scaling, hst* __restrict__ ohi, hst* __restrict__ olo,
                                                    int64_t ldo, int T, int H, int wpb) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int nt = (T + 15) >> 4;
  float* sk = sm;
  float* sv = sm + nt * 16 * AT_KS;
  const int64_t rb = (int64_t)b * T;
  for (int i = threadIdx.x; i < nt * 16 * 16; i += blockDim.x) {
    const int r = i >> 4, c4 = (i & 15) * 4;
    float4 kk = make_float4(0.f, 0.f, 0.f, 0.f), vv = kk;
    if (r < T) {
      kk = *reinterpret_cast<const float4*>(k + (rb + r) * ld + h * 64 + c4);
      vv = *reinterpret_cast<const float4*>(v + (rb + r) * ld + h * 64 + c4);
    }
    *reinterpret_cast<float4*>(sk + r * AT_KS + c4) = kk;
    *reinterpret_cast<float4*>(sv + r * AT_VS + c4) = vv;
  }
  __syncthreads();
  const int qt = blockIdx.y * wpb + (threadIdx.x >> 6);
  if (qt >= nt) return;                           // no barrier follows
  const int lane = threadIdx.x & 63, col = lane & 15, g = lane >> 4;
  const int row = qt * 16 + col;
  const bool qvalid = row < T;
  float qf[16];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (qvalid) x = *reinterpret_cast<const float4*>(q + (rb + row) * ld + h * 64 + 16 * g + 4 * t);
    qf[4 * t] = x.x * scaling, qf[4 * t + 1] = x.y * scaling, qf[4 * t + 2] = x.z * scaling,
    qf[4 * t + 3] = x.w * scaling;
  }
  f4v S[NTM];
#pragma unroll
  for (int kt = 0; kt < NTM; ++kt) {
    S[kt] = f4v{0.f, 0.f, 0.f, 0.f};
    if (kt < nt) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float4 kf = *reinterpret_cast<const float4*>(sk + (kt * 16 + col) * AT_KS + 16 * g + 4 * t);
        S[kt] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf.x, qf[4 * t], S[kt], 0, 0, 0);
        S[kt] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf.y, qf[4 * t + 1], S[kt], 0, 0, 0);
        S[kt] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf.z, qf[4 * t + 2], S[kt], 0, 0, 0);
        S[kt] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf.w, qf[4 * t + 3], S[kt], 0, 0, 0);
      }
    }
  }
  // lane holds S^T[key = kt*16 + 4g + r][query = row]: + gate * rel_bias[key - query], keys >= T masked
  const float gq = qvalid ? gate[(rb + row) * H + h] : 0.f;
  const float* relh = rel + (int64_t)h * (2 * T - 1) + (T - 1) - row;
  float mx = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < NTM; ++kt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = kt * 16 + 4 * g + r;
      float s = -INFINITY;
      if (kt < nt && key < T) s = S[kt][r] + (qvalid ? gq * relh[key] : 0.f);
      S[kt][r] = s;
      mx = fmaxf(mx, s);
    }
  }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int kt = 0; kt < NTM; ++kt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p = (kt < nt && kt * 16 + 4 * g + r < T) ? expf(S[kt][r] - mx) : 0.f;
      S[kt][r] = p;
      sum += p;
    }
  }
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
  f4v O[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) O[dt] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < NTM; ++kt) {
    if (kt < nt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float* vr = sv + (kt * 16 + 4 * g + r) * AT_VS + col;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) O[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(vr[dt * 16], S[kt][r], O[dt], 0, 0, 0);
      }
    }
  }
  if (!qvalid) return;
  const float inv = 1.0f / sum;
  // lane holds O^T[d = dt*16 + 4g + r][query = row]
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const float o4[4] = {O[dt][0] * inv, O[dt][1] * inv, O[dt][2] * inv, O[dt][3] * inv};
    const int64_t off = (rb + row) * ldo + h * 64 + dt * 16 + 4 * g;
    store_split<4>(ohi + off, olo + off, o4);
  }
}

// ---- positional convolution, split on staging -----------------------------------------------------------------------
// out[b, t, c] = h[b, t, c] + gelu(bias[c] + sum_{k<128} sum_{c'<64} h[b, t+k-64, g, c'] W[g*64+n, c', k]), c = g*64+n
// (t < T; rows outside [0, T) read as zero). Block = 4 waves = 128 output rows of one (b, g); the 255-row input
// window staged as hi / lo bf16 images; each wave 32 rows x 64 outputs as two 32x32x16 accumulators; per tap and
// k-step three MFMAs (hi.hi, lo.hi, hi.lo) against the tap's weight planes from L2.
constexpr int PC_C = 64, PC_E = 1024, PC_K = 128, PC_ROWS = 128, PC_WIN = PC_ROWS + PC_K - 1, PC_LDW = PC_C + 8;

__device__ __forceinline__ void pc_load_b(hx8* dst, const hst* wg, int k, int n, int hh) {
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int s = 0; s < 4; ++s)
      dst[nt * 4 + s] =
          *reinterpret_cast<const hx8*>(wg + ((int64_t)k * PC_C + nt * 32 + n) * PC_C + 16 * s + 8 * hh);
}

__global__ __launch_bounds__(256, 2) void posconv_kernel(const float* __restrict__ in, const hst* __restrict__ wkh,
                                                         const hst* __restrict__ wkl, const float* __restrict__ bias,
                                                         float* __restrict__ out, int T) {
  __shared__ __attribute__((aligned(16))) hel wh[PC_WIN][PC_LDW];
  __shared__ __attribute__((aligned(16))) hel wl[PC_WIN][PC_LDW];
  const int t0 = blockIdx.x * PC_ROWS, g = blockIdx.y, b = blockIdx.z;
  const int64_t base = (int64_t)b * T * PC_E + g * PC_C;
  constexpr int off = PC_K / 2;
  for (int i = threadIdx.x; i < PC_WIN * (PC_C / 4); i += 256) {
    const int wr = i >> 4, c4 = (i & 15) * 4;
    const int tr = t0 - off + wr;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tr >= 0 && tr < T) x = *reinterpret_cast<const float4*>(in + base + (int64_t)tr * PC_E + c4);
    uint32_t h0, l0, h1, l1;
    split_pack2(x.x, x.y, h0, l0);
    split_pack2(x.z, x.w, h1, l1);
    *reinterpret_cast<uint2*>(&wh[wr][c4]) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(&wl[wr][c4]) = make_uint2(l0, l1);
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  if (t0 + 32 * w >= T) return;                  // no barrier follows
  const int64_t wofs = (int64_t)g * PC_K * PC_C * PC_C;
  rdx_f32x16 acc[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[0][i] = acc[1][i] = 0.f;
  hx8 bh[8], bl[8];
#pragma unroll 2
  for (int k = 0; k < PC_K; ++k) {
    pc_load_b(bh, wkh + wofs, k, r, hh);
    pc_load_b(bl, wkl + wofs, k, r, hh);
    const hel* ah = &wh[32 * w + r + k][8 * hh];
    const hel* alo = &wl[32 * w + r + k][8 * hh];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const hx8 fh = *reinterpret_cast<const hx8*>(ah + 16 * s);
      const hx8 fl = *reinterpret_cast<const hx8*>(alo + 16 * s);
      acc[0] = mfma32x32x16(fh, bh[s], acc[0]);
      acc[1] = mfma32x32x16(fh, bh[4 + s], acc[1]);
      acc[0] = mfma32x32x16(fl, bh[s], acc[0]);
      acc[1] = mfma32x32x16(fl, bh[4 + s], acc[1]);
      acc[0] = mfma32x32x16(fh, bl[s], acc[0]);
      acc[1] = mfma32x32x16(fh, bl[4 + s], acc[1]);
    }
  }
  // C layout: column n = lane & 31 of tile nt, row (i & 3) + 8 (i >> 2) + 4 hh
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int n = nt * 32 + r;
    const float bs = bias[g * PC_C + n];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int t = t0 + 32 * w + (i & 3) + 8 * (i >> 2) + 4 * hh;
      if (t < T) {
        const int64_t o = base + (int64_t)t * PC_E + n;
        out[o] = in[o] + gelu_exact(acc[nt][i] + bs);
      }
    }
  }
}

// ---- WavLM CNN: layer 0 and the LayerNorm + GELU of layers 1-6 in fp32 ----------------------------------------------
constexpr int FE_C = 512, FE_TOK = 64;   // 16 tokens per wave: the 80 weights per lane loaded once per 64 tokens

__device__ __forceinline__ void fe_ln_gelu(float v[8], const float* __restrict__ gamma, const float* __restrict__ beta,
                                           int c0, float eps) {
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) s += v[e];
  const float mean = wave_sum(s) * (1.0f / FE_C);
  float q = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float d = v[e] - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(wave_sum(q) * (1.0f / FE_C) + eps);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = gelu_exact((v[e] - mean) * rstd * gamma[c0 + e] + beta[c0 + e]);
}

template <int K>
__global__ __launch_bounds__(256) void fe_conv0_kernel(const float* __restrict__ x, int64_t L,
                                                       const float* __restrict__ w, const float* __restrict__ bias,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float eps, int stride, hst* __restrict__ ohi,
                                                       hst* __restrict__ olo, int64_t T0) {
  extern __shared__ float s_win[];
  const int b = blockIdx.y;
  const int64_t t_base = (int64_t)blockIdx.x * FE_TOK;
  const int nwin = (FE_TOK - 1) * stride + K;
  const float* xb = x + (int64_t)b * L;
  for (int i = threadIdx.x; i < nwin; i += 256) {
    const int64_t gi = t_base * stride + i;
    s_win[i] = gi < L ? xb[gi] : 0.f;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c0 = lane * 8;
  float wr[8][K];
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int k = 0; k < K; ++k) wr[e][k] = w[(c0 + e) * K + k];
  float bs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bs[e] = bias ? bias[c0 + e] : 0.f;
  __syncthreads();
#pragma unroll 1
  for (int j = 0; j < FE_TOK / 4; ++j) {
    const int tl = wv * (FE_TOK / 4) + j;
    const int64_t t = t_base + tl;
    if (t >= T0) break;
    const float* sx = s_win + tl * stride;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float xv = sx[k];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaf(wr[e][k], xv, v[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += bs[e];
    fe_ln_gelu(v, gamma, beta, c0, eps);
    const int64_t o = ((int64_t)b * T0 + t) * FE_C + c0;
    store_split<8>(ohi + o, olo + o, v);
  }
}

__global__ __launch_bounds__(256) void fe_ln_gelu_kernel(const float* __restrict__ in, int64_t R,
                                                         const float* __restrict__ bias,
                                                         const float* __restrict__ gamma, const float* __restrict__ beta,
                                                         float eps, hst* __restrict__ ohi, hst* __restrict__ olo,
                                                         float* __restrict__ out32) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const int c0 = lane * 8;
  const float* p = in + row * FE_C + c0;
  const float4 u0 = *reinterpret_cast<const float4*>(p), u1 = *reinterpret_cast<const float4*>(p + 4);
  float v[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
  if (bias) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += bias[c0 + e];
  }
  fe_ln_gelu(v, gamma, beta, c0, eps);
  if (out32) {
    float* q = out32 + row * FE_C + c0;
    *reinterpret_cast<float4*>(q) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(q + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    store_split<8>(ohi + row * FE_C + c0, olo + row * FE_C + c0, v);
  }
}
#endif  // !RDX_F16

}  // namespace x3
}  // namespace rdx

using namespace rdx;

namespace {
[[maybe_unused]] inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
[[maybe_unused]] inline bool al8(const void* p) { return ((uintptr_t)p & 7) == 0; }
}  // namespace

#ifdef RDX_F16
#define X3_ONLY_BF16() return RDX_EINVAL
#else
#define X3_ONLY_BF16() (void)0
#endif

extern "C" int rdx_x3_split(const float* x, int64_t ldx, int64_t rows, int cols, void* hi, void* lo, int64_t ldo,
                            void* stream) {
  X3_ONLY_BF16();
#ifndef RDX_F16
  RDX_REQUIRE(x && hi && lo && rows > 0 && cols > 0 && cols % 4 == 0 && ldx >= cols && ldo >= cols);
  RDX_REQUIRE(al16(x) && ldx % 4 == 0 && al8(hi) && al8(lo) && ldo % 4 == 0);
  const int64_t n = rows * (cols / 4);
  const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 65536);
  hipLaunchKernelGGL(x3::split_kernel, dim3(grid), dim3(256), 0, as_stream(stream), x, ldx, rows, cols, (hst*)hi,
                     (hst*)lo, ldo);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
#endif
}

extern "C" int rdx_x3_ln_split(const float* a, const float* b, float* sum_out, const float* gamma, const float* beta,
                               float eps, void* hi, void* lo, int64_t ldo, float* y32, const float* wg,
                               const float* bg, const float* gconst, float* gate, int64_t M, int E, void* stream) {
  X3_ONLY_BF16();
#ifndef RDX_F16
  RDX_REQUIRE(a && gamma && beta && M > 0 && (E == 512 || E == 1024) && (hi || y32));
  RDX_REQUIRE(al16(a) && (!b || al16(b)) && (!sum_out || al16(sum_out)) && al16(gamma) && al16(beta));
  RDX_REQUIRE(!hi || (lo && al16(hi) && al16(lo) && ldo >= E && ldo % 8 == 0));
  RDX_REQUIRE(!y32 || al16(y32));
  const bool gated = wg != nullptr;
  RDX_REQUIRE(!gated || (E == 1024 && bg && gconst && gate && al16(wg)));
  x3::LnArgs args{a, b, sum_out, gamma, beta, eps, (hst*)hi, (hst*)lo, ldo, y32, wg, bg, gconst, gate, M};
  const dim3 grid((unsigned)((M + 3) / 4));
  hipStream_t st = as_stream(stream);
  if (E == 512) hipLaunchKernelGGL((x3::ln_split_kernel<8, false>), grid, dim3(256), 0, st, args);
  else if (gated) hipLaunchKernelGGL((x3::ln_split_kernel<16, true>), grid, dim3(256), 0, st, args);
  else hipLaunchKernelGGL((x3::ln_split_kernel<16, false>), grid, dim3(256), 0, st, args);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
#endif
}

extern "C" int rdx_x3_attn_fwd(const float* q, const float* k, const float* v, int64_t ld, const float* gate,
                               const float* rel, float scaling, void* ohi, void* olo, int64_t ldo, int B, int T, int H,
                               int qsplit, void* stream) {
  X3_ONLY_BF16();
#ifndef RDX_F16
  RDX_REQUIRE(q && k && v && gate && rel && ohi && olo && B > 0 && H > 0 && T > 0 && T <= 256);
  RDX_REQUIRE(al16(q) && al16(k) && al16(v) && ld % 4 == 0 && al8(ohi) && al8(olo) && ldo % 4 == 0);
  RDX_REQUIRE(ld >= (int64_t)H * 64 && ldo >= (int64_t)H * 64 && qsplit >= 1 && qsplit <= 16);
  const int nt = (T + 15) / 16;
  const int wpb = (nt + qsplit - 1) / qsplit;
  const size_t smem = (size_t)nt * 16 * (x3::AT_KS + x3::AT_VS) * sizeof(float);
  const dim3 grid((unsigned)(B * H), (unsigned)((nt + wpb - 1) / wpb));
  hipStream_t st = as_stream(stream);
  auto go = [&](auto kern) -> int {
    static bool attr = false;
    if (!attr) {
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (e != hipSuccess) return (int)e;
      attr = true;
    }
    hipLaunchKernelGGL(kern, grid, dim3(64 * wpb), smem, st, q, k, v, ld, gate, rel, scaling, (hst*)ohi, (hst*)olo,
                       ldo, T, H, wpb);
    RDX_LAUNCH_CHECK();
    return RDX_OK;
  };
  if (nt <= 4) return go(x3::attn_kernel<4>);
  if (nt <= 8) return go(x3::attn_kernel<8>);
  if (nt <= 13) return go(x3::attn_kernel<13>);
  return go(x3::attn_kernel<16>);
#endif
}

extern "C" int rdx_x3_posconv_fwd(const float* h, const void* wk_hi, const void* wk_lo, const float* bias, float* out,
                                  int B, int T, void* stream) {
  X3_ONLY_BF16();
#ifndef RDX_F16
  RDX_REQUIRE(h && wk_hi && wk_lo && bias && out && B > 0 && T > 0 && B <= 65535);
  RDX_REQUIRE(al16(h) && al16(wk_hi) && al16(wk_lo) && out != h);
  const dim3 grid((unsigned)((T + x3::PC_ROWS - 1) / x3::PC_ROWS), 16, (unsigned)B);
  hipLaunchKernelGGL(x3::posconv_kernel, grid, dim3(256), 0, as_stream(stream), h, (const hst*)wk_hi,
                     (const hst*)wk_lo, bias, out, T);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
#endif
}

extern "C" int rdx_x3_fe_conv0(const float* x, int64_t batch, int64_t len, const float* w, const float* bias,
                               const float* gamma, const float* beta, float eps, int ksize, int stride, void* out_hi,
                               void* out_lo, void* stream) {
  X3_ONLY_BF16();
#ifndef RDX_F16
  RDX_REQUIRE(x && w && gamma && beta && out_hi && out_lo && batch > 0 && batch <= 65535);
  RDX_REQUIRE(stride >= 1 && len >= ksize);
  if (ksize != 10) return RDX_EUNSUPPORTED;       // WavLM / wav2vec2 conv 0
  RDX_REQUIRE(al8(out_hi) && al8(out_lo));
  const int64_t T0 = (len - ksize) / stride + 1;
  const dim3 grid((unsigned)((T0 + x3::FE_TOK - 1) / x3::FE_TOK), (unsigned)batch);
  const size_t smem = sizeof(float) * ((x3::FE_TOK - 1) * stride + ksize);
  hipLaunchKernelGGL(x3::fe_conv0_kernel<10>, grid, dim3(256), smem, as_stream(stream), x, len, w, bias, gamma, beta,
                     eps, stride, (hst*)out_hi, (hst*)out_lo, T0);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
#endif
}

extern "C" int rdx_x3_fe_ln_gelu(const float* in, int64_t rows, const float* bias, const float* gamma,
                                 const float* beta, float eps, void* out_hi, void* out_lo, float* out32,
                                 void* stream) {
  X3_ONLY_BF16();
#ifndef RDX_F16
  RDX_REQUIRE(in && gamma && beta && rows > 0 && al16(in) && (out32 ? al16(out32) : (al8(out_hi) && al8(out_lo))));
  hipLaunchKernelGGL(x3::fe_ln_gelu_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, as_stream(stream), in,
                     rows, bias, gamma, beta, eps, (hst*)out_hi, (hst*)out_lo, out32);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
#endif
}
