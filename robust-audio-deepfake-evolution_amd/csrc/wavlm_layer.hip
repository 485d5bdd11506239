// Fused pieces of the WavLM encoder layer (stable layer norm, frozen base + LoRA q/v) for the
// Phase-6 training step: everything between the four hipBLASLt GEMMs and the MFMA attention.
//
// Reference: HF WavLMEncoderLayerStableLayerNorm / WavLMAttention / WavLMFeedForward (transformers
// modeling_wavlm.py) as run by WavLMFrontend (src/models/DualStreamSEMamba.py:292-439), with peft
// LoRA on q_proj/v_proj (src/main.py:103-158):
//     x1 = LN1(h);  gate = ga * (gb * c_h - 1) + 2,  (ga, gb) = sigmoid(sum4(Wg x1_head + bg))
//     [q k v] = x1 [Wq Wk Wv]^T + b + s * (B_q A_q drop(x1), 0, B_v A_v drop(x1))
//     h2 = h + drop(out_proj(attn(q, k, v, gate)));  x2 = LN2(h2)
//     h' = h2 + drop(W2 gelu(W1 x2 + b1) + b2)
// Layout: one wave per token row (E = 1024 = 64 lanes x 16 contiguous fp32), so a row's LN
// statistics, its 16 per-head gates (4 lanes per 64-dim head) and its 2r = 16 LoRA down-projections
// are wave reductions. The LoRA down-projection a = A drop(x1) is written next to x1 into one
// [M, E + 2r] bf16 operand, so the q/k/v GEMM (K = E + 2r against [Wqkv | s B]) applies the whole
// LoRA update with no extra GEMM; its backward returns d a in the same GEMM.
// Dropout: counter-hash masks (common.h) keyed by (layer seed, salt, m * E + e), regenerated in the
// backward; the seed lives in device memory (HIP-graph replayable).
#include "common.h"

namespace rdx {

constexpr int WL_E = 1024;
constexpr int WL_VPL = WL_E / RDX_WAVE;  // 16 fp32 per lane
constexpr int WL_R2 = 16;                // 2 * LoRA rank (q and v adapters, r = 8)

struct Drop {
  const int64_t* seed_dev;
  int salt;
  uint32_t thr;    // p * 2^32 (0: identity)
  float inv_keep;  // 1 / (1 - p)
};

__device__ __forceinline__ float drop_scale(const Drop& d, uint64_t seed, uint64_t idx) {
  return drop_keep(seed, idx, d.thr) ? d.inv_keep : 0.f;
}

__device__ __forceinline__ void load16(const float* p, float* v) {
  const float4* q = reinterpret_cast<const float4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float4 t = q[i];
    v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
  }
}
__device__ __forceinline__ void store16(float* p, const float* v) {
  float4* q = reinterpret_cast<float4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
}
__device__ __forceinline__ void load16_bf(const hst* p, float* v) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    uint4 t = q[i];
    uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[8 * i + 2 * j] = hlo(w[j]);
      v[8 * i + 2 * j + 1] = hhi(w[j]);
    }
  }
}
// raw 16 bf16 (two 16-byte loads), unpacked later: keeps the unpack from pinning a wait between a row's loads
struct Bf16x16 {
  uint4 q[2];
};
__device__ __forceinline__ Bf16x16 load16_bf_raw(const hst* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  return Bf16x16{{q[0], q[1]}};
}
__device__ __forceinline__ void unpack16_bf(const Bf16x16& t, float* v) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    uint32_t w[4] = {t.q[i].x, t.q[i].y, t.q[i].z, t.q[i].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[8 * i + 2 * j] = hlo(w[j]);
      v[8 * i + 2 * j + 1] = hhi(w[j]);
    }
  }
}
__device__ __forceinline__ void store16_bf(hst* p, const float* v) {
  uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = hbits(v[8 * i + 2 * j]) | (hbits(v[8 * i + 2 * j + 1]) << 16);
    q[i] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// mean / rstd of a row held as 16 values per lane (two-pass, biased variance like torch)
__device__ __forceinline__ void row_stats(const float* v, float eps, float& mean, float& rstd) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < WL_VPL; ++i) s += v[i];
  mean = wave_sum(s) * (1.0f / WL_E);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < WL_VPL; ++i) {
    float d = v[i] - mean;
    q += d * d;
  }
  rstd = rsqrtf(wave_sum(q) * (1.0f / WL_E) + eps);
}

// Sum 16 per-lane values over the wave with 17 shuffles: lane l ends with the total of index
// k(l) = 8 b5 + 4 b4 + 2 b3 + b2 (b = bits of l); lanes with l & 3 == 0 own distinct k.
__device__ __forceinline__ float wave_sum16(float* v, int lane) {
  float w8[8], w4[4], w2[2];
  const bool h5 = lane & 32, h4 = lane & 16, h3 = lane & 8, h2 = lane & 4;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float r = __shfl_xor(h5 ? v[j] : v[j + 8], 32, 64);
    w8[j] = (h5 ? v[j + 8] : v[j]) + r;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float r = __shfl_xor(h4 ? w8[j] : w8[j + 4], 16, 64);
    w4[j] = (h4 ? w8[j + 4] : w8[j]) + r;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    float r = __shfl_xor(h3 ? w4[j] : w4[j + 2], 8, 64);
    w2[j] = (h3 ? w4[j + 2] : w4[j]) + r;
  }
  float r = __shfl_xor(h2 ? w2[0] : w2[1], 4, 64);
  float t = (h2 ? w2[1] : w2[0]) + r;
  t += __shfl_xor(t, 2, 64);
  t += __shfl_xor(t, 1, 64);
  return t;
}
__device__ __forceinline__ int sum16_index(int lane) {
  return 8 * ((lane >> 5) & 1) + 4 * ((lane >> 4) & 1) + 2 * ((lane >> 3) & 1) + ((lane >> 2) & 1);
}

struct GateW {
  const float* wg;      // [8, 64] gru_rel_pos_linear.weight
  const float* bg;      // [8]
  const float* gconst;  // [H] gru_rel_pos_const
};

// gate pre-activations z[8] of this lane's head (4 lanes per head, 16 dims per lane); wg in LDS or global
__device__ __forceinline__ void gate_z(const GateW& g, const float* wgp, const float* x, int lane, float* z) {
  const int part = lane & 3;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float4* w = reinterpret_cast<const float4*>(wgp + j * 64 + part * 16);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float4 t = w[i];
      acc += t.x * x[4 * i] + t.y * x[4 * i + 1] + t.z * x[4 * i + 2] + t.w * x[4 * i + 3];
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    z[j] = acc + g.bg[j];
  }
}

struct Ln1Args {
  const float* h;  // [M, E] layer input (fp32 residual stream)
  const float* gamma;
  const float* beta;
  float eps;
  GateW g;
  const hst* Aq;    // [r, E] lora_A (q) in the 16-bit storage type (autocast's cast), null without LoRA
  const hst* Av;    // [r, E] lora_A (v)
  Drop dq, dv;      // LoRA dropouts (q, v)
  hst* x1;  // [M, ldx]: LN1 output in [0, E), LoRA down-projection in [E, E + 2r)
  int64_t ldx;
  float* gate;  // [M, H]
  float* mean;
  float* rstd;
  int64_t M;
  // optional residual prologue (the previous layer's last step): h = h2 + drop(delta) is computed here and
  // written to hout (h is then unused)
  const float* h2;
  const hst* delta;
  Drop dres;
  float* hout;
};

// LoRA-A of both adapters staged once per workgroup of WL_LN1_ROWS row-waves (4): [2r][E] 16-bit (the cast autocast
// applies to lora_A's weight, made once per pass by the caller), 32 KB copied with 16-byte loads. A row-wave reading
// the fp32 A from L2 itself moved 64 KB per token row and left these kernels L2-bound (26 us of the 47 us forward
// at B = 32); staging it from fp32 with the conversion here still read 64 KB per workgroup.
#ifndef WL_LN1_ROWS_DEF
#define WL_LN1_ROWS_DEF 4   // measured: 4 rows beat 8 and 2 at both pass sizes (tools/bench_wl.py)
#endif
constexpr int WL_LN1_ROWS = WL_LN1_ROWS_DEF;
constexpr int WL_LN1_THREADS = WL_LN1_ROWS * RDX_WAVE;

// WL_R2 * WL_E 16-bit values over WL_LN1_THREADS threads, 8 per 16-byte load, every load issued before the first
// store: a loop that stored each chunk as it arrived waited out one L2 round trip per chunk (8 per thread), which
// was most of the LoRA kernels' extra time over the LoRA-free variant
// The staging of a LN1 workgroup, gate weights (2 KB fp32) and LoRA-A (32 KB 16-bit), straight from global memory
// into LDS by buffer_load ... lds (16 bytes per lane, lane-linear: one wave-instruction fills 1 KB), issued before the
// rows' own loads and retired by the waitcnt ahead of the barrier: every load of the prologue in flight at once and
// no registers. (A loop that stored each chunk as it arrived waited out one L2 round trip per chunk, 8 per thread:
// most of the LoRA kernels' extra time over the LoRA-free variant; staging through registers loads-first kept the
// round trips but the compiler sank the loads back to their stores under the row kernels' register pressure.)
typedef __attribute__((ext_vector_type(4))) int wl_i32x4;
__device__ void wl_load_lds(wl_i32x4 rsrc, __attribute__((address_space(3))) uint32_t* lds, int size, int voffset,
                            int soffset, int offset, int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");
__device__ __forceinline__ wl_i32x4 wl_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  wl_i32x4 r;
  r.x = (int)(uint32_t)a;
  r.y = (int)(uint32_t)(a >> 32);
  r.z = (int)bytes;
  r.w = 0x00020000;  // raw buffer, range-checked
  return r;
}
constexpr int WL_A_INSTR = WL_R2 * WL_E * 2 / 1024 / (WL_LN1_THREADS / 64);   // LoRA-A instructions per wave (8)
static_assert(WL_A_INSTR * 1024 * (WL_LN1_THREADS / 64) == WL_R2 * WL_E * 2, "whole 1 KB instructions per wave");
template <bool kLora>
__device__ __forceinline__ void stage_dma(float* swg, hst* sA, const float* wg, const hst* Aq, const hst* Av) {
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  constexpr int NW = WL_LN1_THREADS / 64;
  if (wv == 0) {
    const wl_i32x4 rg = wl_rsrc(wg, 8 * 64 * 4);
#pragma unroll
    for (int q = 0; q < 2; ++q)
      wl_load_lds(rg, (__attribute__((address_space(3))) uint32_t*)(reinterpret_cast<char*>(swg) + 1024 * q), 16,
                  1024 * q + 16 * lane, 0, 0, 0);
  }
  if (kLora) {
    const wl_i32x4 rq = wl_rsrc(Aq, WL_R2 / 2 * WL_E * 2), rv = wl_rsrc(Av, WL_R2 / 2 * WL_E * 2);
#pragma unroll
    for (int j = 0; j < WL_A_INSTR; ++j) {
      const int q = wv + NW * j;                       // 1 KB instruction q of the [2r][E] image
      constexpr int half = WL_R2 / 2 * WL_E * 2 / 1024; // instructions per adapter (16)
      wl_load_lds(j < WL_A_INSTR / 2 ? rq : rv,         // q < half exactly when j < WL_A_INSTR / 2 (compile time)
                  (__attribute__((address_space(3))) uint32_t*)(reinterpret_cast<char*>(sA) + 1024 * q), 16,
                  1024 * (q % half) + 16 * lane, 0, 0, 0);
    }
  }
}

template <bool kLora>
__global__ __launch_bounds__(WL_LN1_THREADS) void wl_ln1_fwd_kernel(Ln1Args a) {
  __shared__ __attribute__((aligned(16))) hst sA[kLora ? WL_R2 * WL_E : 8];
  __shared__ __attribute__((aligned(16))) float swg[8 * 64];
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * WL_LN1_ROWS + (threadIdx.x >> 6);
  const bool live = m < a.M;  // no early return: the gate and LoRA parts follow a barrier
  const int e0 = lane * WL_VPL;
  float v[WL_VPL], gm[WL_VPL], bt[WL_VPL], dl[WL_VPL];
  Bf16x16 dlr;
  const uint64_t sr = (a.h2 && a.dres.thr) ? attn_seed(a.dres.seed_dev, a.dres.salt) : 0;  // with the row loads
  // every global load first (one round trip): the workgroup's staging, the row, the affine parameters
  stage_dma<kLora>(swg, sA, a.g.wg, a.Aq, a.Av);
  if (live) {
    load16(a.h2 ? a.h2 + m * WL_E + e0 : a.h + m * WL_E + e0, v);
    if (a.h2) dlr = load16_bf_raw(a.delta + m * WL_E + e0);
    load16(a.gamma + e0, gm);
    load16(a.beta + e0, bt);
  }
  __builtin_amdgcn_s_waitcnt(0);   // the staging DMA (and the row) landed
  __syncthreads();
  if (live) {
    if (a.h2) {
      unpack16_bf(dlr, dl);

#pragma unroll
      for (int i = 0; i < WL_VPL; ++i)
        v[i] += dl[i] * (a.dres.thr ? drop_scale(a.dres, sr, (uint64_t)m * WL_E + e0 + i) : 1.0f);
      store16(a.hout + m * WL_E + e0, v);
    }
    float mean, rstd;
    row_stats(v, a.eps, mean, rstd);
#pragma unroll
    for (int i = 0; i < WL_VPL; ++i) v[i] = hround((v[i] - mean) * rstd * gm[i] + bt[i]);
    store16_bf(a.x1 + m * a.ldx + e0, v);
    if (lane == 0) {
      a.mean[m] = mean;
      a.rstd[m] = rstd;
    }
    float z[8];
    gate_z(a.g, swg, v, lane, z);
    if ((lane & 3) == 0) {
      const int head = lane >> 2;
      float ga = sigmoidf_(z[0] + z[1] + z[2] + z[3]);
      float gb = sigmoidf_(z[4] + z[5] + z[6] + z[7]);
      a.gate[m * (WL_E / 64) + head] = ga * (gb * a.g.gconst[head] - 1.0f) + 2.0f;
    }
  }
  if (kLora) {
    if (!live) return;
    const uint64_t sq = a.dq.thr ? attn_seed(a.dq.seed_dev, a.dq.salt) : 0;
    const uint64_t sv = a.dv.thr ? attn_seed(a.dv.seed_dev, a.dv.salt) : 0;
    // each adapter's dropped row in the 16-bit type (the reference's dropout output: lora_A's input under autocast),
    // packed in pairs, and the down-projection as packed dot products (v_dot2c_f32_*: 8 per adapter row instead of
    // 16 unpacks + 16 FMAs; the per-row VALU work of these 2r dot products was the LoRA kernels' extra time)
    uint32_t mq[WL_VPL / 2], mv[WL_VPL / 2];
#pragma unroll
    for (int j = 0; j < WL_VPL / 2; ++j) {
      const uint64_t idx = (uint64_t)m * WL_E + e0 + 2 * j;
      mq[j] = hpack2(v[2 * j] * drop_scale(a.dq, sq, idx), v[2 * j + 1] * drop_scale(a.dq, sq, idx + 1));
      mv[j] = hpack2(v[2 * j] * drop_scale(a.dv, sv, idx), v[2 * j + 1] * drop_scale(a.dv, sv, idx + 1));
    }
    float acc[WL_R2];
#pragma unroll
    for (int k = 0; k < WL_R2; ++k) {
      const uint32_t* x = k < WL_R2 / 2 ? mq : mv;
      const uint4* wp = reinterpret_cast<const uint4*>(sA + k * WL_E + e0);
      const uint4 w0 = wp[0], w1 = wp[1];
      const uint32_t w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < WL_VPL / 2; ++j) s = hdot2(w[j], x[j], s);
      acc[k] = s;
    }
    float tot = wave_sum16(acc, lane);
    if ((lane & 3) == 0) a.x1[m * a.ldx + WL_E + sum16_index(lane)] = f2h(tot);
  }
}

// h2 = h + drop(delta) (fp32, stored), x = LN(h2) (bf16), mean / rstd saved
struct AddLnArgs {
  const float* h;
  const hst* delta;
  Drop d;
  float* h2;
  const float* gamma;
  const float* beta;
  float eps;
  hst* x;
  float* mean;
  float* rstd;
  int64_t M;
};

__global__ __launch_bounds__(256) void wl_add_ln_fwd_kernel(AddLnArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= a.M) return;
  const int e0 = lane * WL_VPL;
  float v[WL_VPL], dl[WL_VPL], gm[WL_VPL], bt[WL_VPL];
  load16(a.h + m * WL_E + e0, v);
  const Bf16x16 dlr = load16_bf_raw(a.delta + m * WL_E + e0);
  load16(a.gamma + e0, gm);   // with the row's loads: one round trip
  load16(a.beta + e0, bt);
  unpack16_bf(dlr, dl);
  const uint64_t seed = a.d.thr ? attn_seed(a.d.seed_dev, a.d.salt) : 0;
#pragma unroll
  for (int i = 0; i < WL_VPL; ++i)
    v[i] += dl[i] * (a.d.thr ? drop_scale(a.d, seed, (uint64_t)m * WL_E + e0 + i) : 1.0f);
  store16(a.h2 + m * WL_E + e0, v);
  float mean, rstd;
  row_stats(v, a.eps, mean, rstd);
#pragma unroll
  for (int i = 0; i < WL_VPL; ++i) v[i] = (v[i] - mean) * rstd * gm[i] + bt[i];
  store16_bf(a.x + m * WL_E + e0, v);
  if (lane == 0) {
    a.mean[m] = mean;
    a.rstd[m] = rstd;
  }
}

// out = h + drop(delta) over n = M * E elements (8 per thread)
__global__ __launch_bounds__(256) void wl_residual_kernel(const float* __restrict__ h,
                                                          const hst* __restrict__ delta, Drop d,
                                                          float* __restrict__ out, int64_t n) {
  const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i0 >= n) return;
  const uint64_t seed = d.thr ? attn_seed(d.seed_dev, d.salt) : 0;
  float4 a0 = reinterpret_cast<const float4*>(h + i0)[0], a1 = reinterpret_cast<const float4*>(h + i0)[1];
  float x[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  uint4 t = *reinterpret_cast<const uint4*>(delta + i0);
  uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float dv = (j & 1) ? hhi(w[j >> 1]) : hlo(w[j >> 1]);
    x[j] += dv * (d.thr ? drop_scale(d, seed, (uint64_t)(i0 + j)) : 1.0f);
  }
  reinterpret_cast<float4*>(out + i0)[0] = make_float4(x[0], x[1], x[2], x[3]);
  reinterpret_cast<float4*>(out + i0)[1] = make_float4(x[4], x[5], x[6], x[7]);
}

// grad of drop(): out = drop_mask * g (fp32 in, bf16 out), n elements (8 per thread)
__global__ __launch_bounds__(256) void wl_dropout_bwd_kernel(const float* __restrict__ g, Drop d,
                                                             hst* __restrict__ out, int64_t n) {
  const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i0 >= n) return;
  const uint64_t seed = d.thr ? attn_seed(d.seed_dev, d.salt) : 0;
  float4 a0 = reinterpret_cast<const float4*>(g + i0)[0], a1 = reinterpret_cast<const float4*>(g + i0)[1];
  float x[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  uint32_t w[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float s0 = d.thr ? drop_scale(d, seed, (uint64_t)(i0 + 2 * j)) : 1.0f;
    float s1 = d.thr ? drop_scale(d, seed, (uint64_t)(i0 + 2 * j + 1)) : 1.0f;
    w[j] = hbits(x[2 * j] * s0) | (hbits(x[2 * j + 1] * s1) << 16);
  }
  *reinterpret_cast<uint4*>(out + i0) = make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  return 0.5f * (1.0f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}

// y = gelu(u) (mode 0) or du = dy * gelu'(u) (mode 1); bf16, 8 elements per thread
template <int kMode>
__global__ __launch_bounds__(256) void wl_gelu_kernel(const hst* __restrict__ u,
                                                      const hst* __restrict__ dy,
                                                      hst* __restrict__ out, int64_t n) {
  const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i0 >= n) return;
  uint4 t = *reinterpret_cast<const uint4*>(u + i0);
  uint32_t w[4] = {t.x, t.y, t.z, t.w}, gw[4] = {0, 0, 0, 0};
  if (kMode == 1) {
    uint4 g = *reinterpret_cast<const uint4*>(dy + i0);
    gw[0] = g.x; gw[1] = g.y; gw[2] = g.z; gw[3] = g.w;
  }
  uint32_t o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float x0 = hlo(w[j]), x1 = hhi(w[j]);
    float y0, y1;
    if (kMode == 0) {
      y0 = gelu_erf(x0);
      y1 = gelu_erf(x1);
    } else {
      y0 = hlo(gw[j]) * gelu_erf_grad(x0);
      y1 = hhi(gw[j]) * gelu_erf_grad(x1);
    }
    o[j] = hbits(y0) | (hbits(y1) << 16);
  }
  *reinterpret_cast<uint4*>(out + i0) = make_uint4(o[0], o[1], o[2], o[3]);
}

// LN backward with residual: dh = dres + rstd * (g - mean(g) - xhat * mean(g xhat)), g = dx * gamma.
// Optionally also ddrop = drop_mask * dh (bf16): the gradient into the dropout that fed h.
struct LnBwdArgs {
  const hst* dx;  // [M, ldd] (first E columns used)
  int64_t ldd;
  const float* h;  // LN input [M, E]
  const float* mean;
  const float* rstd;
  const float* gamma;
  const float* dres;  // [M, E] or null
  float* dh;          // [M, E]
  Drop d;
  hst* ddrop;  // [M, E] or null
  int64_t M;
};

__device__ __forceinline__ void ln_bwd_row(const float* dx, const float* x, float mean, float rstd, const float* gm,
                                           float* out) {
  float g[WL_VPL], xh[WL_VPL], s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < WL_VPL; ++i) {
    xh[i] = (x[i] - mean) * rstd;
    g[i] = dx[i] * gm[i];
    s1 += g[i];
    s2 += g[i] * xh[i];
  }
  s1 = wave_sum(s1) * (1.0f / WL_E);
  s2 = wave_sum(s2) * (1.0f / WL_E);
#pragma unroll
  for (int i = 0; i < WL_VPL; ++i) out[i] = rstd * (g[i] - s1 - xh[i] * s2);
}

__global__ __launch_bounds__(256) void wl_ln_bwd_kernel(LnBwdArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= a.M) return;
  const int e0 = lane * WL_VPL;
  float dx[WL_VPL], x[WL_VPL], gm[WL_VPL], o[WL_VPL], r[WL_VPL];
  const uint64_t seed = (a.ddrop && a.d.thr) ? attn_seed(a.d.seed_dev, a.d.salt) : 0;
  const Bf16x16 dxr = load16_bf_raw(a.dx + m * a.ldd + e0);
  load16(a.h + m * WL_E + e0, x);
  load16(a.gamma + e0, gm);
  if (a.dres) load16(a.dres + m * WL_E + e0, r);     // every load of the row before the reductions
  unpack16_bf(dxr, dx);
  ln_bwd_row(dx, x, a.mean[m], a.rstd[m], gm, o);
  if (a.dres) {
#pragma unroll
    for (int i = 0; i < WL_VPL; ++i) o[i] += r[i];
  }
  store16(a.dh + m * WL_E + e0, o);
  if (a.ddrop) {
#pragma unroll
    for (int i = 0; i < WL_VPL; ++i)
      o[i] *= a.d.thr ? drop_scale(a.d, seed, (uint64_t)m * WL_E + e0 + i) : 1.0f;
    store16_bf(a.ddrop + m * WL_E + e0, o);
  }
}

// LN1 backward: dx1 = dX1[:, :E] + gate backward + LoRA-A backward; dh = dres + LN1_bwd(dx1).
// Also writes the dropped LN output of each adapter (xd[0] q, xd[1] v) for the dA GEMMs.
struct Ln1BwdArgs {
  const hst* dx1;  // [M, ldx] = d [x1 | a] from the qkv GEMM backward
  int64_t ldx;
  const float* dgate;  // [M, H]
  const float* h;
  const float* mean;
  const float* rstd;
  const float* gamma;
  const float* beta;
  GateW g;
  const hst* Aq;    // [r, E] 16-bit or null
  const hst* Av;
  Drop dq, dv;
  const float* dres;  // [M, E]
  float* dh;
  hst* xd;  // [2, M, E] or null
  int64_t M;
  // optional: the gradient this layer's INPUT receives as a hidden state of the layer-weighted sum,
  // sw[0] * sg (sw a device scalar: softmax(w)_l), added into dh
  const float* sg;
  const float* sw;
  // optional: ddrop = drop_prev(dh) bf16, the gradient of the previous layer's dropped FFN output
  Drop dprev;
  hst* ddrop;
};

template <bool kLora>
__global__ __launch_bounds__(WL_LN1_THREADS) void wl_ln1_bwd_kernel(Ln1BwdArgs a) {
  __shared__ __attribute__((aligned(16))) hst sA[kLora ? WL_R2 * WL_E : 8];
  __shared__ __attribute__((aligned(16))) float swg[8 * 64];
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * WL_LN1_ROWS + (threadIdx.x >> 6);
  const bool live = m < a.M;
  const int e0 = lane * WL_VPL;
  const int part = lane & 3, head = lane >> 2;
  // every row load first: h, dx1, the residual gradient, the layer-sum gradient, the affine parameters
  float x[WL_VPL], x1[WL_VPL], dx[WL_VPL], r[WL_VPL], sgv[WL_VPL], gm[WL_VPL];
  float mean = 0.f, rstd = 0.f, dg = 0.f;
  Bf16x16 dxr;
  const uint64_t sp = (a.ddrop && a.dprev.thr) ? attn_seed(a.dprev.seed_dev, a.dprev.salt) : 0;
  stage_dma<kLora>(swg, sA, a.g.wg, a.Aq, a.Av);
  if (live) {
    load16(a.h + m * WL_E + e0, x);
    dxr = load16_bf_raw(a.dx1 + m * a.ldx + e0);
    load16(a.dres + m * WL_E + e0, r);
    if (a.sg) load16(a.sg + m * WL_E + e0, sgv);
    load16(a.gamma + e0, gm);
    load16(a.beta + e0, x1);
    mean = a.mean[m];
    rstd = a.rstd[m];
    dg = a.dgate[m * (WL_E / 64) + head];
  }
  __builtin_amdgcn_s_waitcnt(0);   // the staging DMA (and the row) landed
  __syncthreads();
  if (!live) return;  // after the only barrier
  unpack16_bf(dxr, dx);
#pragma unroll
  for (int i = 0; i < WL_VPL; ++i) x1[i] = hround((x[i] - mean) * rstd * gm[i] + x1[i]);
  // gate: gate = ga (gb c - 1) + 2
  float z[8];
  gate_z(a.g, swg, x1, lane, z);
  const float ga = sigmoidf_(z[0] + z[1] + z[2] + z[3]), gb = sigmoidf_(z[4] + z[5] + z[6] + z[7]);
  const float c = a.g.gconst[head];
  const float dza = dg * (gb * c - 1.0f) * ga * (1.0f - ga);
  const float dzb = dg * ga * c * gb * (1.0f - gb);
#pragma unroll 2
  for (int j = 0; j < 8; ++j) {
    const float dz = j < 4 ? dza : dzb;
    const float4* w = reinterpret_cast<const float4*>(swg + j * 64 + part * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float4 t = w[i];
      dx[4 * i] += t.x * dz;
      dx[4 * i + 1] += t.y * dz;
      dx[4 * i + 2] += t.z * dz;
      dx[4 * i + 3] += t.w * dz;
    }
  }
  if (kLora) {
    const uint64_t sq = a.dq.thr ? attn_seed(a.dq.seed_dev, a.dq.salt) : 0;
    const uint64_t sv = a.dv.thr ? attn_seed(a.dv.seed_dev, a.dv.salt) : 0;
    if (a.xd) {  // the dropped LN output of each adapter (optional; first, so that x1 dies here)
#pragma unroll
      for (int which = 0; which < 2; ++which) {
        const Drop& dd = which ? a.dv : a.dq;
        const uint64_t sd = which ? sv : sq;
        float xm[WL_VPL];
#pragma unroll
        for (int i = 0; i < WL_VPL; ++i) xm[i] = x1[i] * drop_scale(dd, sd, (uint64_t)m * WL_E + e0 + i);
        store16_bf(a.xd + (which * a.M + m) * WL_E + e0, xm);
      }
    }
    // the 2r down-projection gradients of this row, packed in k pairs (one 32-byte broadcast read); the term
    // sum_k A[k][e] da[k] of each element e as packed dot products over k pairs: the two A rows k, k + 1 read as
    // before (32 contiguous bytes per lane, conflict-free), their 16-bit halves regrouped per element
    const uint4 dap[2] = {*reinterpret_cast<const uint4*>(a.dx1 + m * a.ldx + WL_E),
                          *reinterpret_cast<const uint4*>(a.dx1 + m * a.ldx + WL_E + 8)};
#pragma unroll
    for (int which = 0; which < 2; ++which) {
      float acc[WL_VPL];
#pragma unroll
      for (int i = 0; i < WL_VPL; ++i) acc[i] = 0.f;
      const uint32_t dk[4] = {dap[which].x, dap[which].y, dap[which].z, dap[which].w};
#pragma unroll
      for (int kp = 0; kp < WL_R2 / 4; ++kp) {
        const int k = which * (WL_R2 / 2) + 2 * kp;
        const uint4* ra = reinterpret_cast<const uint4*>(sA + k * WL_E + e0);
        const uint4* rb = reinterpret_cast<const uint4*>(sA + (k + 1) * WL_E + e0);
        const uint4 a0 = ra[0], a1 = ra[1], b0 = rb[0], b1 = rb[1];
        const uint32_t wa[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const uint32_t wb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int j = 0; j < WL_VPL / 2; ++j) {
          // v_perm_b32 (selector bytes 0-3: the second operand's bytes, 4-7: the first's)
          const uint32_t ev = __builtin_amdgcn_perm(wb[j], wa[j], 0x05040100u);   // (A[k][2j], A[k + 1][2j])
          const uint32_t od = __builtin_amdgcn_perm(wb[j], wa[j], 0x07060302u);   // (A[k][2j + 1], A[k + 1][2j + 1])
          acc[2 * j] = hdot2(ev, dk[kp], acc[2 * j]);
          acc[2 * j + 1] = hdot2(od, dk[kp], acc[2 * j + 1]);
        }
      }
      const Drop& dd = which ? a.dv : a.dq;
      const uint64_t sd = which ? sv : sq;
#pragma unroll
      for (int i = 0; i < WL_VPL; ++i) dx[i] += acc[i] * drop_scale(dd, sd, (uint64_t)m * WL_E + e0 + i);
    }
  }
  float o[WL_VPL];
  ln_bwd_row(dx, x, mean, rstd, gm, o);
#pragma unroll
  for (int i = 0; i < WL_VPL; ++i) o[i] += r[i];
  if (a.sg) {
    const float pw = a.sw[0];
#pragma unroll
    for (int i = 0; i < WL_VPL; ++i) o[i] = fmaf(pw, sgv[i], o[i]);
  }
  store16(a.dh + m * WL_E + e0, o);
  if (a.ddrop) {
#pragma unroll
    for (int i = 0; i < WL_VPL; ++i)
      o[i] *= a.dprev.thr ? drop_scale(a.dprev, sp, (uint64_t)m * WL_E + e0 + i) : 1.0f;
    store16_bf(a.ddrop + m * WL_E + e0, o);
  }
}

// LoRA weight gradients of one layer, ACCUMULATED into the fp32 .grad buffers:
//   dB_q[e, k] += s sum_m dq[m, e] a_q[m, k]        dA_q[k, e] += sum_m da_q[m, k] drop_q(x1)[m, e]
// (same for v). A block owns 128 columns and 4 * RPW rows: lane = 2 adjacent columns (bf16x2 loads,
// 256 B per wave-instruction), wave w = RPW consecutive rows whose loads are all issued before the
// FMAs (no per-row branch: rows past M read row M-1 against zeroed per-row factors). The 4 waves'
// 32 x 128 partial sums are reduced through LDS, then the block adds 4096 fp32 atomics laid out so
// each wave-instruction covers 64 consecutive dwords of dA ([r, E]) or dB ([E, r]).
constexpr int WL_LG_COLS = 128;
constexpr int WL_LG_PAD = WL_LG_COLS + 1;  // LDS row stride (floats): the dB read walks k

struct LoraGradArgs {
  const hst* dqkv;  // [M, ldq]: dq at column 0, dv at column 2E
  int64_t ldq;
  const hst* x1;    // [M, ldx]: x1 in [0, E), a in [E, E + 2r)
  int64_t ldx;
  const hst* dx1;   // [M, ldd]: d a in [E, E + 2r)
  int64_t ldd;
  Drop dq, dv;
  float scale;
  float *dAq, *dBq, *dAv, *dBv;
  int64_t M;
};

__device__ __forceinline__ float2 hx2_at(const hst* p) {
  const uint32_t u = *reinterpret_cast<const uint32_t*>(p);
  return make_float2(hlo(u), hhi(u));
}

template <int RPW>
__global__ __launch_bounds__(256, 2) void wl_lora_grad_kernel(LoraGradArgs a, int nch) {
  constexpr int ROWS = 4 * RPW;  // rows per chunk; a block walks nch chunks
  __shared__ float s_row[2][ROWS][2 * WL_R2];
  __shared__ float s_part[4][2 * WL_R2][WL_LG_PAD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e0 = blockIdx.x * WL_LG_COLS;
  const int e = e0 + 2 * lane;
  constexpr int R = WL_R2 / 2;
  float bq[2][R], bv[2][R], aq[2][R], av[2][R];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int k = 0; k < R; ++k) bq[c][k] = bv[c][k] = aq[c][k] = av[c][k] = 0.f;
  const uint64_t sq = a.dq.thr ? attn_seed(a.dq.seed_dev, a.dq.salt) : 0;
  const uint64_t sv = a.dv.thr ? attn_seed(a.dv.seed_dev, a.dv.salt) : 0;
  for (int ch = 0; ch < nch; ++ch) {
    const int64_t m0 = ((int64_t)blockIdx.y * nch + ch) * ROWS;
    float(*srow)[2 * WL_R2] = s_row[ch & 1];
    for (int t = threadIdx.x; t < ROWS * 2 * WL_R2; t += 256) {
      const int rr = t / (2 * WL_R2), c = t % (2 * WL_R2);
      const int64_t m = m0 + rr;
      float v = 0.f;
      if (m < a.M)
        v = c < WL_R2 ? h2f(a.x1[m * a.ldx + WL_E + c])
                      : h2f(a.dx1[m * a.ldd + WL_E + c - WL_R2]);
      srow[rr][c] = v;
    }
    float2 gq[RPW], gv[RPW], xx[RPW];
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int64_t m = min(m0 + w * RPW + j, a.M - 1);
      gq[j] = hx2_at(a.dqkv + m * a.ldq + e);
      gv[j] = hx2_at(a.dqkv + m * a.ldq + 2 * WL_E + e);
      xx[j] = hx2_at(a.x1 + m * a.ldx + e);
    }
    __syncthreads();  // srow staged (the other buffer is still read by nobody: one barrier per chunk)
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int rr = w * RPW + j;
      const uint64_t idx = (uint64_t)min(m0 + rr, a.M - 1) * WL_E + e;
      const float g_q[2] = {gq[j].x, gq[j].y}, g_v[2] = {gv[j].x, gv[j].y};
      const float xq[2] = {xx[j].x * drop_scale(a.dq, sq, idx), xx[j].y * drop_scale(a.dq, sq, idx + 1)};
      const float xv[2] = {xx[j].x * drop_scale(a.dv, sv, idx), xx[j].y * drop_scale(a.dv, sv, idx + 1)};
      const float* f = srow[rr];
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int k = 0; k < R; ++k) {
          bq[c][k] = fmaf(g_q[c], f[k], bq[c][k]);
          bv[c][k] = fmaf(g_v[c], f[R + k], bv[c][k]);
          aq[c][k] = fmaf(f[2 * R + k], xq[c], aq[c][k]);
          av[c][k] = fmaf(f[3 * R + k], xv[c], av[c][k]);
        }
    }
  }
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int k = 0; k < R; ++k) {
      s_part[w][k][2 * lane + c] = bq[c][k];
      s_part[w][R + k][2 * lane + c] = bv[c][k];
      s_part[w][2 * R + k][2 * lane + c] = aq[c][k];
      s_part[w][3 * R + k][2 * lane + c] = av[c][k];
    }
  __syncthreads();
  // 4096 outputs: o < 2048 -> dA (kk = o / 128 over aq then av, col = o % 128: lanes contiguous in e);
  // o >= 2048 -> dB (which = q/v, col = rem / 8, k = rem % 8: lanes contiguous in e * r + k).
#pragma unroll 4
  for (int i = 0; i < 16; ++i) {
    const int o = i * 256 + threadIdx.x;
    int row, col;
    float* dst;
    float mul = 1.f;
    if (o < 2048) {
      const int kk = o / WL_LG_COLS;
      col = o % WL_LG_COLS;
      row = 2 * R + kk;
      dst = kk < R ? a.dAq + (int64_t)kk * WL_E + e0 + col : a.dAv + (int64_t)(kk - R) * WL_E + e0 + col;
    } else {
      const int o2 = o - 2048, which = o2 / (WL_LG_COLS * R), rem = o2 % (WL_LG_COLS * R);
      col = rem / R;
      const int k = rem % R;
      row = which * R + k;
      dst = (which ? a.dBv : a.dBq) + (int64_t)(e0 + col) * R + k;
      mul = a.scale;
    }
    const float v = s_part[0][row][col] + s_part[1][row][col] + s_part[2][row][col] + s_part[3][row][col];
    atomicAdd(dst, mul * v);
  }
}

// Wext[:, E:E+2r] <- s * B (q rows 0..E-1 columns E..E+r-1, v rows 2E..3E-1 columns E+r..E+2r-1);
// one launch for every layer. Other rows of those columns stay zero.
__global__ __launch_bounds__(256) void wl_lora_pack_kernel(int nl, const float* const* bq, const float* const* bv,
                                                           hst* const* wext, int64_t ldw, int r,
                                                           float scale) {
  const int l = blockIdx.y;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;  // over 2 * E * r
  if (l >= nl || t >= 2 * (int64_t)WL_E * r) return;
  const int which = (int)(t / ((int64_t)WL_E * r));
  const int64_t rem = t % ((int64_t)WL_E * r);
  const int64_t row = rem / r;
  const int k = (int)(rem % r);
  const float* b = which ? bv[l] : bq[l];  // lora_B weight [E, r]
  const int64_t wrow = which ? 2 * WL_E + row : row;
  wext[l][wrow * ldw + WL_E + which * r + k] = f2h(scale * b[row * r + k]);
}

}  // namespace rdx

using namespace rdx;

static Drop mk_drop(const int64_t* seed_dev, int salt, float p) {
  Drop d;
  d.seed_dev = seed_dev;
  d.salt = salt;
  d.thr = (p > 0.f && seed_dev) ? (uint32_t)fminf(4294967295.0f, p * 4294967296.0f) : 0u;
  d.inv_keep = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  return d;
}

static int blocks_rows(int64_t M) { return (int)((M + 3) / 4); }
static int blocks_ln1(int64_t M) { return (int)((M + WL_LN1_ROWS - 1) / WL_LN1_ROWS); }

static int ln1_fwd_launch(const Ln1Args& a, bool lora, void* stream) {
  const int64_t M = a.M;
  if (lora)
    hipLaunchKernelGGL(wl_ln1_fwd_kernel<true>, dim3(blocks_ln1(M)), dim3(WL_LN1_THREADS), 0, as_stream(stream), a);
  else
    hipLaunchKernelGGL(wl_ln1_fwd_kernel<false>, dim3(blocks_ln1(M)), dim3(WL_LN1_THREADS), 0, as_stream(stream), a);
  RDX_LAUNCH_CHECK();
  return 0;
}


extern "C" {

int rdx_wl_ln1_fwd(const float* h, const float* gamma, const float* beta, float eps, const float* wg, const float* bg,
                   const float* gconst, const void* lora_aq, const void* lora_av, int r, const int64_t* seed_dev,
                   int salt_q, int salt_v, float p_lora, void* x1, int64_t ldx, float* gate, float* mean, float* rstd, int64_t M, int E,
                   void* stream) {
  RDX_REQUIRE(h && gamma && beta && wg && bg && gconst && x1 && gate && mean && rstd && M > 0);
  const bool lora = lora_aq != nullptr;
  RDX_REQUIRE(E == WL_E && (!lora || (2 * r == WL_R2 && lora_av)) && ldx >= E + (lora ? 2 * r : 0));
  RDX_REQUIRE(!lora || ((((uintptr_t)lora_aq | (uintptr_t)lora_av) & 15) == 0));
  RDX_REQUIRE(ldx % 8 == 0);
  Ln1Args a{h, gamma, beta, eps, GateW{wg, bg, gconst}, reinterpret_cast<const hst*>(lora_aq),
            reinterpret_cast<const hst*>(lora_av), mk_drop(seed_dev, salt_q, p_lora),
            mk_drop(seed_dev, salt_v, p_lora), reinterpret_cast<hst*>(x1), ldx, gate, mean, rstd, M,
            nullptr, nullptr, mk_drop(nullptr, 0, 0.f), nullptr};
  return ln1_fwd_launch(a, lora, stream);
}

int rdx_wl_res_ln1_fwd(const float* h2, const void* delta, int salt_res, float p_res, float* hout,
                       const float* gamma, const float* beta, float eps, const float* wg, const float* bg,
                       const float* gconst, const void* lora_aq, const void* lora_av, int r, const int64_t* seed_dev,
                       int salt_q, int salt_v, float p_lora, void* x1, int64_t ldx, float* gate, float* mean,
                       float* rstd, int64_t M, int E, void* stream) {
  RDX_REQUIRE(h2 && delta && hout && gamma && beta && wg && bg && gconst && x1 && gate && mean && rstd && M > 0);
  const bool lora = lora_aq != nullptr;
  RDX_REQUIRE(E == WL_E && (!lora || (2 * r == WL_R2 && lora_av)) && ldx >= E + (lora ? 2 * r : 0));
  RDX_REQUIRE(!lora || ((((uintptr_t)lora_aq | (uintptr_t)lora_av) & 15) == 0));
  RDX_REQUIRE(ldx % 8 == 0);
  Ln1Args a{nullptr, gamma, beta, eps, GateW{wg, bg, gconst}, reinterpret_cast<const hst*>(lora_aq),
            reinterpret_cast<const hst*>(lora_av), mk_drop(seed_dev, salt_q, p_lora),
            mk_drop(seed_dev, salt_v, p_lora), reinterpret_cast<hst*>(x1), ldx, gate, mean, rstd, M,
            h2, reinterpret_cast<const hst*>(delta), mk_drop(seed_dev, salt_res, p_res), hout};
  return ln1_fwd_launch(a, lora, stream);
}

int rdx_wl_add_ln_fwd(const float* h, const void* delta, const int64_t* seed_dev, int salt, float p, float* h2,
                      const float* gamma, const float* beta, float eps, void* x, float* mean, float* rstd, int64_t M,
                      int E, void* stream) {
  RDX_REQUIRE(h && delta && h2 && gamma && beta && x && mean && rstd && M > 0 && E == WL_E);
  AddLnArgs a{h, reinterpret_cast<const hst*>(delta), mk_drop(seed_dev, salt, p), h2, gamma, beta, eps,
              reinterpret_cast<hst*>(x), mean, rstd, M};
  hipLaunchKernelGGL(wl_add_ln_fwd_kernel, dim3(blocks_rows(M)), dim3(256), 0, as_stream(stream), a);
  RDX_LAUNCH_CHECK();
  return 0;
}

int rdx_wl_residual(const float* h, const void* delta, const int64_t* seed_dev, int salt, float p, float* out,
                    int64_t n, void* stream) {
  RDX_REQUIRE(h && delta && out && n > 0 && n % 8 == 0);
  hipLaunchKernelGGL(wl_residual_kernel, dim3((unsigned)((n / 8 + 255) / 256)), dim3(256), 0, as_stream(stream), h,
                     reinterpret_cast<const hst*>(delta), mk_drop(seed_dev, salt, p), out, n);
  RDX_LAUNCH_CHECK();
  return 0;
}

int rdx_wl_dropout_bwd(const float* g, const int64_t* seed_dev, int salt, float p, void* out, int64_t n,
                       void* stream) {
  RDX_REQUIRE(g && out && n > 0 && n % 8 == 0);
  hipLaunchKernelGGL(wl_dropout_bwd_kernel, dim3((unsigned)((n / 8 + 255) / 256)), dim3(256), 0, as_stream(stream), g,
                     mk_drop(seed_dev, salt, p), reinterpret_cast<hst*>(out), n);
  RDX_LAUNCH_CHECK();
  return 0;
}

int rdx_wl_gelu(int mode, const void* u, const void* dy, void* out, int64_t n, void* stream) {
  RDX_REQUIRE(u && out && n > 0 && n % 8 == 0 && (mode == 0 || (mode == 1 && dy)));
  const auto* U = reinterpret_cast<const hst*>(u);
  const auto* DY = reinterpret_cast<const hst*>(dy);
  auto* O = reinterpret_cast<hst*>(out);
  const dim3 grid((unsigned)((n / 8 + 255) / 256));
  if (mode == 0)
    hipLaunchKernelGGL(wl_gelu_kernel<0>, grid, dim3(256), 0, as_stream(stream), U, DY, O, n);
  else
    hipLaunchKernelGGL(wl_gelu_kernel<1>, grid, dim3(256), 0, as_stream(stream), U, DY, O, n);
  RDX_LAUNCH_CHECK();
  return 0;
}

int rdx_wl_ln_bwd(const void* dx, int64_t ldd, const float* h, const float* mean, const float* rstd,
                  const float* gamma, const float* dres, float* dh, const int64_t* seed_dev, int salt, float p,
                  void* ddrop, int64_t M, int E, void* stream) {
  RDX_REQUIRE(dx && h && mean && rstd && gamma && dh && M > 0 && E == WL_E && ldd >= E && ldd % 8 == 0);
  LnBwdArgs a{reinterpret_cast<const hst*>(dx), ldd, h, mean, rstd, gamma, dres, dh,
              mk_drop(seed_dev, salt, p), reinterpret_cast<hst*>(ddrop), M};
  hipLaunchKernelGGL(wl_ln_bwd_kernel, dim3(blocks_rows(M)), dim3(256), 0, as_stream(stream), a);
  RDX_LAUNCH_CHECK();
  return 0;
}

int rdx_wl_ln1_bwd_ex(const void* dx1, int64_t ldx, const float* dgate, const float* h, const float* mean,
                      const float* rstd, const float* gamma, const float* beta, const float* wg, const float* bg,
                      const float* gconst, const void* lora_aq, const void* lora_av, int r, const int64_t* seed_dev,
                      int salt_q, int salt_v, float p_lora, const float* dres, float* dh, void* xd,
                      const float* state_grad, const float* state_weight, int salt_prev, float p_prev,
                      void* ddrop_prev, int64_t M, int E, void* stream) {
  RDX_REQUIRE(dx1 && dgate && h && mean && rstd && gamma && beta && wg && bg && gconst && dres && dh && M > 0);
  RDX_REQUIRE((state_grad == nullptr) == (state_weight == nullptr));
  const bool lora = lora_aq != nullptr;
  RDX_REQUIRE(E == WL_E && ldx % 8 == 0 && (!lora || (2 * r == WL_R2 && lora_av && ldx >= E + 2 * r)));
  RDX_REQUIRE(!lora || ((((uintptr_t)lora_aq | (uintptr_t)lora_av) & 15) == 0));
  Ln1BwdArgs a{reinterpret_cast<const hst*>(dx1), ldx, dgate, h, mean, rstd, gamma, beta,
               GateW{wg, bg, gconst}, reinterpret_cast<const hst*>(lora_aq), reinterpret_cast<const hst*>(lora_av),
               mk_drop(seed_dev, salt_q, p_lora), mk_drop(seed_dev, salt_v, p_lora),
               dres, dh, reinterpret_cast<hst*>(xd), M, state_grad, state_weight,
               mk_drop(seed_dev, salt_prev, p_prev), reinterpret_cast<hst*>(ddrop_prev)};
  if (lora)
    hipLaunchKernelGGL(wl_ln1_bwd_kernel<true>, dim3(blocks_ln1(M)), dim3(WL_LN1_THREADS), 0, as_stream(stream), a);
  else
    hipLaunchKernelGGL(wl_ln1_bwd_kernel<false>, dim3(blocks_ln1(M)), dim3(WL_LN1_THREADS), 0, as_stream(stream), a);
  RDX_LAUNCH_CHECK();
  return 0;
}

int rdx_wl_ln1_bwd(const void* dx1, int64_t ldx, const float* dgate, const float* h, const float* mean,
                   const float* rstd, const float* gamma, const float* beta, const float* wg, const float* bg,
                   const float* gconst, const void* lora_aq, const void* lora_av, int r, const int64_t* seed_dev,
                   int salt_q, int salt_v, float p_lora, const float* dres, float* dh, void* xd, int64_t M, int E,
                   void* stream) {
  return rdx_wl_ln1_bwd_ex(dx1, ldx, dgate, h, mean, rstd, gamma, beta, wg, bg, gconst, lora_aq, lora_av, r, seed_dev,
                           salt_q, salt_v, p_lora, dres, dh, xd, nullptr, nullptr, 0, 0.f, nullptr, M, E, stream);
}

int rdx_wl_lora_grad(const void* dqkv, int64_t ldq, const void* x1, int64_t ldx, const void* dx1, int64_t ldd,
                     const int64_t* seed_dev, int salt_q, int salt_v, float p_lora, float scale, float* daq,
                     float* dbq, float* dav, float* dbv, int64_t M, int E, int r, void* stream) {
  RDX_REQUIRE(dqkv && x1 && dx1 && daq && dbq && dav && dbv && M > 0 && E == WL_E && 2 * r == WL_R2);
  RDX_REQUIRE(ldq >= 3 * (int64_t)E && ldx >= E + 2 * r && ldd >= E + 2 * r);
  RDX_REQUIRE(ldq % 2 == 0 && ldx % 2 == 0 && ((uintptr_t)dqkv & 3) == 0 && ((uintptr_t)x1 & 3) == 0);
  LoraGradArgs a{reinterpret_cast<const hst*>(dqkv), ldq, reinterpret_cast<const hst*>(x1), ldx,
                 reinterpret_cast<const hst*>(dx1), ldd, mk_drop(seed_dev, salt_q, p_lora),
                 mk_drop(seed_dev, salt_v, p_lora), scale, daq, dbq, dav, dbv, M};
  // 32-row chunks; a block walks nch of them so the 4096 fp32 atomics it ends with are amortised over
  // >= 64 rows once M allows (atomics run at ~1.3 TB/s of added bytes chip-wide), keeping >= 400 blocks.
  const int64_t nchunk = (M + 31) / 32;
  const int nch = (int)std::max<int64_t>(1, std::min<int64_t>(8, M / 2048));
  const dim3 grid(WL_E / WL_LG_COLS, (unsigned)((nchunk + nch - 1) / nch));
  hipLaunchKernelGGL(wl_lora_grad_kernel<8>, grid, dim3(256), 0, as_stream(stream), a, nch);
  RDX_LAUNCH_CHECK();
  return 0;
}

int rdx_wl_lora_pack(int nl, const float* const* bq, const float* const* bv, void* const* wext, int64_t ldw, int r,
                     float scale, int E, void* stream) {
  RDX_REQUIRE(nl > 0 && bq && bv && wext && E == WL_E && r > 0 && ldw >= E + 2 * r);
  const int64_t n = 2 * (int64_t)E * r;
  hipLaunchKernelGGL(wl_lora_pack_kernel, dim3((unsigned)((n + 255) / 256), nl), dim3(256), 0, as_stream(stream), nl,
                     bq, bv, reinterpret_cast<hst* const*>(wext), ldw, r, scale);
  RDX_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
