// WavLM positional convolution on gfx950 MFMA: grouped Conv1d (1024 -> 1024, 16 groups of 64 channels,
// 128 taps, padding 64, last frame dropped) + bias + GELU, forward and input gradient, bf16 operands with
// fp32 accumulation.
//
// Reference: HF WavLMPositionalConvEmbedding (transformers modeling_wavlm.py) inside the WavLM stream
// (src/models/DualStreamSEMamba.py:292-439). Its weights are frozen in Phase 6, but FGM makes
// feature_projection trainable (src/main.py:514-544), so the gradient flows back through this conv.
//   fwd   u[b,t,g,n] = bias[g*64+n] + sum_{k<128} sum_{c<64} h[b, t+k-64, g, c] * W[g*64+n, c, k]   (t < T)
//         y = gelu(u) (erf form); u is kept (bf16) for the backward
//   dgrad dh[b,s,g,c] = sum_{k'<128} sum_{n<64} du[b, s+k'-63, g, n] * W[g*64+n, c, 127-k'],  du = dy * gelu'(u)
// Both are   out[b, t, g, :] = sum_k in[b, t + k - off, g, :] . Wk[g][k]   with Wk[g][k] a 64 x 64 slice laid
// out [g][k][n][c] (permuted once on the host) and input rows outside [0, T) read as zero.
// MIOpen runs this grouped conv as per-utterance im2col + GEMM + col2im (~1.4 ms per B = 8 pass); here it is
// one launch each way.
//
// Tiling: block = 4 waves = 128 output rows of one (b, g). The input window (255 rows x 64 channels) is
// staged once in LDS (the dgrad stage forms du from dy and u). Each wave owns 32 rows x 64 outputs (two
// mfma_f32_32x32x16_bf16 accumulators) and walks 128 taps x 4 k-steps; A fragments are 16-byte LDS row reads
// (144-byte rows: conflict-free), B fragments (the tap's 64 x 64 weights) come from L2, double-buffered in
// registers one tap ahead. Waves whose 32 rows all lie past T exit after the stage.
#include "common.h"

namespace rdx {

typedef __attribute__((ext_vector_type(8))) __bf16 pc_bf16x8;
typedef __attribute__((ext_vector_type(16))) float pc_f32x16;

constexpr int PC_G = 16;                    // groups
constexpr int PC_C = 64;                    // channels per group
constexpr int PC_E = PC_G * PC_C;           // 1024
constexpr int PC_K = 128;                   // taps
constexpr int PC_ROWS = 128;                // output rows per block (4 waves x 32)
constexpr int PC_WIN = PC_ROWS + PC_K - 1;  // staged input rows
constexpr int PC_LDW = PC_C + 8;            // LDS row stride (bf16): 144 B

__device__ __forceinline__ float pc_gelu(float u) { return 0.5f * u * (1.f + erff(u * 0.70710678118654752f)); }
__device__ __forceinline__ float pc_gelu_d(float u) {
  return 0.5f * (1.f + erff(u * 0.70710678118654752f)) + u * 0.39894228040143268f * __expf(-0.5f * u * u);
}

// B fragments of tap k: [nt * 4 + s] = Wk[k][nt * 32 + n][16 s + 8 hh .. + 7] for lane (n, hh)
__device__ __forceinline__ void pc_load_b(pc_bf16x8* dst, const __hip_bfloat16* wg, int k, int n, int hh) {
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int s = 0; s < 4; ++s)
      dst[nt * 4 + s] =
          *reinterpret_cast<const pc_bf16x8*>(wg + ((int64_t)k * PC_C + nt * 32 + n) * PC_C + 16 * s + 8 * hh);
}

// one tap: acc[nt] += A (32 window rows from arow, 64 channels) x B (the tap's 64 x 32 slice nt)
__device__ __forceinline__ void pc_tap(pc_f32x16* acc, const __bf16* arow, const pc_bf16x8* bf) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const pc_bf16x8 af = *reinterpret_cast<const pc_bf16x8*>(arow + 16 * s);
    acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf[s], acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf[4 + s], acc[1], 0, 0, 0);
  }
}

template <bool kBwd>
__global__ __launch_bounds__(256) void posconv_kernel(const __hip_bfloat16* __restrict__ in,   // fwd h, bwd dy
                                                      const __hip_bfloat16* __restrict__ usave,  // bwd: u
                                                      const __hip_bfloat16* __restrict__ wk,     // [G][K][64][64]
                                                      const float* __restrict__ bias,            // fwd: [E]
                                                      __hip_bfloat16* __restrict__ out,          // fwd y, bwd dh
                                                      __hip_bfloat16* __restrict__ uout,         // fwd: u
                                                      int T, int off) {
  __shared__ __attribute__((aligned(16))) __bf16 win[PC_WIN][PC_LDW];
  const int t0 = blockIdx.x * PC_ROWS, g = blockIdx.y, b = blockIdx.z;
  const int64_t base = (int64_t)b * T * PC_E + g * PC_C;
  for (int i = threadIdx.x; i < PC_WIN * (PC_C / 8); i += 256) {
    const int wr = i >> 3, c8 = (i & 7) * 8;
    const int tr = t0 - off + wr;
    pc_bf16x8 v;
    if (tr >= 0 && tr < T) {
      const int64_t o = base + (int64_t)tr * PC_E + c8;
      if (kBwd) {
        const pc_bf16x8 d = *reinterpret_cast<const pc_bf16x8*>(in + o);
        const pc_bf16x8 u = *reinterpret_cast<const pc_bf16x8*>(usave + o);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (__bf16)((float)d[j] * pc_gelu_d((float)u[j]));
      } else {
        v = *reinterpret_cast<const pc_bf16x8*>(in + o);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__bf16)0.f;
    }
    *reinterpret_cast<pc_bf16x8*>(&win[wr][c8]) = v;
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  if (t0 + 32 * w >= T) return;  // no barrier follows
  const __hip_bfloat16* wg = wk + (int64_t)g * PC_K * PC_C * PC_C;
  pc_f32x16 acc[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[0][i] = acc[1][i] = 0.f;
  pc_bf16x8 b0[8], b1[8];
  pc_load_b(b0, wg, 0, r, hh);
  for (int k = 0; k < PC_K; k += 2) {
    pc_load_b(b1, wg, k + 1, r, hh);
    pc_tap(acc, &win[32 * w + r + k][8 * hh], b0);
    if (k + 2 < PC_K) pc_load_b(b0, wg, k + 2, r, hh);
    pc_tap(acc, &win[32 * w + r + k + 1][8 * hh], b1);
  }
  // C layout: column n = lane & 31 of tile nt, row (i & 3) + 8 (i >> 2) + 4 hh
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int n = nt * 32 + r;
    const float bs = kBwd ? 0.f : bias[g * PC_C + n];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int t = t0 + 32 * w + (i & 3) + 8 * (i >> 2) + 4 * hh;
      if (t < T) {
        const int64_t o = base + (int64_t)t * PC_E + n;
        if (kBwd) {
          out[o] = __float2bfloat16(acc[nt][i]);
        } else {
          const __hip_bfloat16 ub = __float2bfloat16(acc[nt][i] + bs);
          uout[o] = ub;
          out[o] = __float2bfloat16(pc_gelu(__bfloat162float(ub)));
        }
      }
    }
  }
}

}  // namespace rdx

using namespace rdx;

static bool pc_ok(const void* p) { return p && ((uintptr_t)p & 15) == 0; }

extern "C" int rdx_posconv_fwd(const void* h, const void* wk, const float* bias, void* y, void* u, int B, int T,
                               void* stream) {
  RDX_REQUIRE(pc_ok(h) && pc_ok(wk) && bias && pc_ok(y) && pc_ok(u) && B > 0 && T > 0 && B <= 65535);
  dim3 grid((T + PC_ROWS - 1) / PC_ROWS, PC_G, B);
  hipLaunchKernelGGL(posconv_kernel<false>, grid, dim3(256), 0, as_stream(stream), (const __hip_bfloat16*)h, nullptr,
                     (const __hip_bfloat16*)wk, bias, (__hip_bfloat16*)y, (__hip_bfloat16*)u, T, PC_K / 2);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_posconv_bwd(const void* dy, const void* u, const void* wkt, void* dh, int B, int T, void* stream) {
  RDX_REQUIRE(pc_ok(dy) && pc_ok(u) && pc_ok(wkt) && pc_ok(dh) && B > 0 && T > 0 && B <= 65535);
  dim3 grid((T + PC_ROWS - 1) / PC_ROWS, PC_G, B);
  hipLaunchKernelGGL(posconv_kernel<true>, grid, dim3(256), 0, as_stream(stream), (const __hip_bfloat16*)dy,
                     (const __hip_bfloat16*)u, (const __hip_bfloat16*)wkt, nullptr, (__hip_bfloat16*)dh, nullptr, T,
                     PC_K / 2 - 1);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
