// WavLM-Large frozen CNN feature encoder (HF WavLMFeatureEncoder with feat_extract_norm = "layer": seven
// WavLMLayerNormConvLayer = Conv1d(bias) -> LayerNorm(512) over channels -> GELU), run once per window on the
// raw waveform by WavLMFrontend (src/models/DualStreamSEMamba.py:392-439, the frozen CNN of §8a A12).
//
// Token-major activations [B, T_l, 512] bf16 throughout, so every layer reads and writes whole 1 KB token
// rows and the final [B, 201, 512] is already the layout feature_projection consumes:
//   layer 0 (C_in = 1, K = 10, stride 5): a direct kernel, one wave per output token, 8 channels per lane
//     (80 FMAs from a sample window staged in LDS), then the 512-channel LayerNorm as a wave reduction and
//     GELU, fused: the [B, 512, 12919] conv output never exists unnormalised in HBM.
//   layers 1-6 (K = 3 or 2, stride 2): an implicit GEMM. With token-major input, output token t reads input
//     tokens 2t .. 2t+K-1, i.e. ONE contiguous K*512-element row starting at element 2t*512, so the im2col
//     matrix is the input itself with row stride 1024 (overlapping rows, never materialised). The MFMA GEMM
//     of gemm.hip runs it per utterance (grid.y) against the weight permuted to [512][K*512], bias fused.
//   LayerNorm + GELU of layers 1-6: one wave per token row, in place (bf16) or into the fp32 final output.
// Rounding follows the bf16-autocast module path: waveform, weights and bias in bf16, fp32 accumulation, the
// conv output rounded to bf16, LayerNorm/GELU in fp32, each layer's activation rounded to bf16 (the next
// conv's autocast input); the last layer's GELU output stays fp32, as autocast leaves it.
#include "common.h"

namespace rdx {

constexpr int FE_C = 512;            // conv_dim of every layer
constexpr int FE_TOK = 64;           // output tokens per 256-thread block (16 per wave: the 80 weights per lane loaded once per 64 tokens)

__device__ __forceinline__ float fe_gelu(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

// LayerNorm over the 512 channels held 8 per lane by one wave, then GELU.
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
  const float4 g0 = *reinterpret_cast<const float4*>(gamma + c0), g1 = *reinterpret_cast<const float4*>(gamma + c0 + 4);
  const float4 b0 = *reinterpret_cast<const float4*>(beta + c0), b1 = *reinterpret_cast<const float4*>(beta + c0 + 4);
  const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
  const float b[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = fe_gelu((v[e] - mean) * rstd * g[e] + b[e]);
}

__device__ __forceinline__ uint32_t fe_pack2(float a, float b) {
  hst x = f2h(a), y = f2h(b);
  return (uint32_t)(*reinterpret_cast<uint16_t*>(&x)) | ((uint32_t)(*reinterpret_cast<uint16_t*>(&y)) << 16);
}

__device__ __forceinline__ void fe_store8(hst* p, const float v[8]) {
  *reinterpret_cast<uint4*>(p) = make_uint4(fe_pack2(v[0], v[1]), fe_pack2(v[2], v[3]), fe_pack2(v[4], v[5]),
                                            fe_pack2(v[6], v[7]));
}

// ---- layer 0: x [B, L] fp32 -> out [B, T0, 512] bf16 = gelu(LN(conv(x) + bias))
// w: [512][K] fp32 holding bf16-rounded weights; bias [512] fp32 holding a bf16-rounded bias
template <int K>
__global__ __launch_bounds__(256) void fe_conv0_kernel(const float* __restrict__ x, int64_t L, const float* __restrict__ w,
                                                       const float* __restrict__ bias, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float eps, int stride,
                                                       hst* __restrict__ out, int64_t T0) {
  extern __shared__ float s_win[];
  const int b = blockIdx.y;
  const int64_t t_base = (int64_t)blockIdx.x * FE_TOK;
  const int nwin = (FE_TOK - 1) * stride + K;
  const float* xb = x + (int64_t)b * L;
  for (int i = threadIdx.x; i < nwin; i += 256) {
    const int64_t g = t_base * stride + i;
    s_win[i] = g < L ? hround(xb[g]) : 0.f;
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
  for (int e = 0; e < 8; ++e) bs[e] = bias[c0 + e];
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
    for (int e = 0; e < 8; ++e) v[e] = hround(v[e] + bs[e]);
    fe_ln_gelu(v, gamma, beta, c0, eps);
    fe_store8(out + ((int64_t)b * T0 + t) * FE_C + c0, v);
  }
}

// ---- LayerNorm(512) + GELU of rows [R, 512] bf16 (in place, or fp32 into out32)
// FE_RPW rows per wave: every row's 16-byte load issued before the first row's reductions, so a wave waits one
// memory round trip for its rows instead of one per row (one row per wave left the pass at ~1.6 TB/s)
constexpr int FE_RPW = 4;
__global__ __launch_bounds__(256) void fe_ln_gelu_kernel(hst* __restrict__ io, int64_t R,
                                                         const float* __restrict__ gamma, const float* __restrict__ beta,
                                                         float eps, float* __restrict__ out32) {
  const int lane = threadIdx.x & 63;
  const int64_t row0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * FE_RPW;
  if (row0 >= R) return;
  const int c0 = lane * 8;
  uint4 u[FE_RPW];
#pragma unroll
  for (int k = 0; k < FE_RPW; ++k) {
    const int64_t row = row0 + k < R ? row0 + k : R - 1;   // clamped: the load is unconditional
    u[k] = *reinterpret_cast<const uint4*>(io + row * FE_C + c0);
  }
#pragma unroll
  for (int k = 0; k < FE_RPW; ++k) {
    const int64_t row = row0 + k;
    if (row >= R) break;
    const uint32_t w4[4] = {u[k].x, u[k].y, u[k].z, u[k].w};
    float v[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = hlo(w4[i]);
      v[2 * i + 1] = hhi(w4[i]);
    }
    fe_ln_gelu(v, gamma, beta, c0, eps);
    if (out32) {
      float* q = out32 + row * FE_C + c0;
      *reinterpret_cast<float4*>(q) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(q + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      fe_store8(io + row * FE_C + c0, v);
    }
  }
}

}  // namespace rdx

using namespace rdx;

extern "C" int rdx_fe_conv0(const float* x, int64_t batch, int64_t len, const float* w, const float* bias,
                            const float* gamma, const float* beta, float eps, int ksize, int stride, void* out,
                            void* stream) {
  RDX_REQUIRE(x && w && bias && gamma && beta && out && batch > 0 && batch <= 65535);
  RDX_REQUIRE(stride >= 1 && len >= ksize);
  if (ksize != 10) return RDX_EUNSUPPORTED;  // WavLM / wav2vec2 conv 0
  RDX_REQUIRE(((uintptr_t)out & 15) == 0 && ((uintptr_t)gamma & 15) == 0 && ((uintptr_t)beta & 15) == 0);
  const int64_t T0 = (len - ksize) / stride + 1;
  dim3 grid((unsigned)((T0 + FE_TOK - 1) / FE_TOK), (unsigned)batch);
  const size_t smem = sizeof(float) * ((FE_TOK - 1) * stride + ksize);
  hipLaunchKernelGGL(fe_conv0_kernel<10>, grid, dim3(256), smem, as_stream(stream), x, len, w, bias, gamma, beta, eps,
                     stride, (hst*)out, T0);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_fe_ln_gelu(void* io, int64_t rows, const float* gamma, const float* beta, float eps, float* out32,
                              void* stream) {
  RDX_REQUIRE(io && gamma && beta && rows > 0 && ((uintptr_t)io & 15) == 0);
  RDX_REQUIRE(((uintptr_t)gamma & 15) == 0 && ((uintptr_t)beta & 15) == 0 && (!out32 || ((uintptr_t)out32 & 15) == 0));
  hipLaunchKernelGGL(fe_ln_gelu_kernel, dim3((unsigned)((rows + 4 * FE_RPW - 1) / (4 * FE_RPW))), dim3(256), 0,
                     as_stream(stream),
                     (hst*)io, rows, gamma, beta, eps, out32);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
