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
__device__ __forceinline__ void pc_load_b(hx8* dst, const hst* wg, int k, int n, int hh) {
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int s = 0; s < 4; ++s)
      dst[nt * 4 + s] =
          *reinterpret_cast<const hx8*>(wg + ((int64_t)k * PC_C + nt * 32 + n) * PC_C + 16 * s + 8 * hh);
}

// one tap: acc[nt] += A (32 window rows from arow, 64 channels) x B (the tap's 64 x 32 slice nt)
__device__ __forceinline__ void pc_tap(pc_f32x16* acc, const hel* arow, const hx8* bf) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const hx8 af = *reinterpret_cast<const hx8*>(arow + 16 * s);
    acc[0] = mfma32x32x16(af, bf[s], acc[0]);
    acc[1] = mfma32x32x16(af, bf[4 + s], acc[1]);
  }
}

template <bool kBwd>
__global__ __launch_bounds__(256) void posconv_kernel(const hst* __restrict__ in,   // fwd h, bwd dy
                                                      const hst* __restrict__ usave,  // bwd: u
                                                      const hst* __restrict__ wk,     // [G][K][64][64]
                                                      const float* __restrict__ bias,            // fwd: [E]
                                                      hst* __restrict__ out,          // fwd y, bwd dh
                                                      hst* __restrict__ uout,         // fwd: u
                                                      int T, int off) {
  __shared__ __attribute__((aligned(16))) hel win[PC_WIN][PC_LDW];
  const int t0 = blockIdx.x * PC_ROWS, g = blockIdx.y, b = blockIdx.z;
  const int64_t base = (int64_t)b * T * PC_E + g * PC_C;
  for (int i = threadIdx.x; i < PC_WIN * (PC_C / 8); i += 256) {
    const int wr = i >> 3, c8 = (i & 7) * 8;
    const int tr = t0 - off + wr;
    hx8 v;
    if (tr >= 0 && tr < T) {
      const int64_t o = base + (int64_t)tr * PC_E + c8;
      if (kBwd) {
        const hx8 d = *reinterpret_cast<const hx8*>(in + o);
        const hx8 u = *reinterpret_cast<const hx8*>(usave + o);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (hel)((float)d[j] * pc_gelu_d((float)u[j]));
      } else {
        v = *reinterpret_cast<const hx8*>(in + o);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (hel)0.f;
    }
    *reinterpret_cast<hx8*>(&win[wr][c8]) = v;
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  if (t0 + 32 * w >= T) return;  // no barrier follows
  const hst* wg = wk + (int64_t)g * PC_K * PC_C * PC_C;
  pc_f32x16 acc[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[0][i] = acc[1][i] = 0.f;
  hx8 b0[8], b1[8];
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
          out[o] = f2h(acc[nt][i]);
        } else {
          const hst ub = f2h(acc[nt][i] + bs);
          uout[o] = ub;
          out[o] = f2h(pc_gelu(h2f(ub)));
        }
      }
    }
  }
}

// T <= 256: one workgroup per (b, g) covers every row, each wave 64 rows (two M tiles) x 64 outputs, so a tap's B
// fragments feed 16 MFMAs instead of 8. The tap's 64 x 64 weights (8 KB) are staged once per workgroup in a
// double-buffered LDS image (144-byte rows, conflict-free like the input window) from global loads issued two
// taps ahead, one barrier per tap, instead of every wave reading them from L2: a quarter of the weight traffic.
// Same arithmetic per output as posconv_kernel (the same taps and K order into the same fp32 accumulators).
constexpr int PC2_ROWS = 256;
constexpr int PC2_WIN = PC2_ROWS + PC_K - 1;
constexpr int PC2_WIMG = PC_C * PC_LDW;   // one tap's weight image (bf16 elements)
constexpr int PC2_LDS = (PC2_WIN * PC_LDW + 2 * PC2_WIMG) * 2;
template <bool kBwd>
__global__ __launch_bounds__(256, 2) void posconv2_kernel(const hst* __restrict__ in,
                                                          const hst* __restrict__ usave,
                                                          const hst* __restrict__ wk,
                                                          const float* __restrict__ bias,
                                                          hst* __restrict__ out,
                                                          hst* __restrict__ uout, int T, int off) {
  extern __shared__ __attribute__((aligned(16))) char pc2_lds[];
  hel (*win)[PC_LDW] = reinterpret_cast<hel (*)[PC_LDW]>(pc2_lds);
  hel* wimg = reinterpret_cast<hel*>(pc2_lds) + PC2_WIN * PC_LDW;   // [2][64 n][PC_LDW]
  const int g = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int64_t base = (int64_t)b * T * PC_E + g * PC_C;
  const hst* wg = wk + (int64_t)g * PC_K * PC_C * PC_C;
  // tap k's [64 n][64 c] slice: 512 16-byte chunks, chunks tid and tid + 256 of this thread
  const int wn0 = tid >> 3, wc0 = (tid & 7) * 8;   // chunk tid + 256: row wn0 + 32
  auto wload = [&](int k, int j) -> uint4 {
    return *reinterpret_cast<const uint4*>(wg + ((int64_t)k * PC_C + wn0 + 32 * j) * PC_C + wc0);
  };
  auto wstore = [&](int buf, uint4 v0, uint4 v1) {
    *reinterpret_cast<uint4*>(wimg + buf * PC2_WIMG + wn0 * PC_LDW + wc0) = v0;
    *reinterpret_cast<uint4*>(wimg + buf * PC2_WIMG + (wn0 + 32) * PC_LDW + wc0) = v1;
  };
  uint4 va0 = wload(0, 0), va1 = wload(0, 1), vb0 = wload(1, 0), vb1 = wload(1, 1);
  for (int i = tid; i < PC2_WIN * (PC_C / 8); i += 256) {
    const int wr = i >> 3, c8 = (i & 7) * 8;
    const int tr = wr - off;
    hx8 v;
    if (tr >= 0 && tr < T) {
      const int64_t o = base + (int64_t)tr * PC_E + c8;
      if (kBwd) {
        const hx8 d = *reinterpret_cast<const hx8*>(in + o);
        const hx8 u = *reinterpret_cast<const hx8*>(usave + o);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (hel)((float)d[j] * pc_gelu_d((float)u[j]));
      } else {
        v = *reinterpret_cast<const hx8*>(in + o);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (hel)0.f;
    }
    *reinterpret_cast<hx8*>(&win[wr][c8]) = v;
  }
  wstore(0, va0, va1);
  __syncthreads();
  const int w = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int r0 = 64 * w;
  const bool one = r0 < T, two = r0 + 32 < T;   // the wave's M tiles holding rows below T (wave-uniform)
  pc_f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[0][0][i] = acc[0][1][i] = acc[1][0][i] = acc[1][1][i] = 0.f;
  // tap kk from image buf: the B fragments [nt * 4 + s] = W[kk][nt * 32 + r][16 s + 8 hh .. + 7]
  // every LDS read of the tap (8 B fragments, both M tiles' 4 A fragments; the second tile's rows stay inside the
  // window) issued before its first MFMA, with a scheduling barrier so they are not pulled back one by one to
  // their MFMAs: the MFMAs then wait on a decreasing count instead of a full LDS round trip each
  auto tap = [&](int kk, int buf) {
    hx8 bf[8], af[2][4];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
        bf[nt * 4 + s2] =
            *reinterpret_cast<const hx8*>(wimg + buf * PC2_WIMG + (nt * 32 + r) * PC_LDW + 16 * s2 + 8 * hh);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
        af[mt][s2] = *reinterpret_cast<const hx8*>(&win[r0 + 32 * mt + r + kk][8 * hh] + 16 * s2);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      if (!(mt == 0 ? one : two)) continue;
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {   // pc_tap's order
        acc[mt][0] = mfma32x32x16(af[mt][s2], bf[s2], acc[mt][0]);
        acc[mt][1] = mfma32x32x16(af[mt][s2], bf[4 + s2], acc[mt][1]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  static_assert(PC_K % 2 == 0, "taps in pairs");
  for (int k = 0; k < PC_K; k += 2) {
    // image 0 holds tap k, vb tap k + 1; va takes tap k + 2 (the last taps re-load tap K - 1: no conditional load)
    va0 = wload(min(k + 2, PC_K - 1), 0);
    va1 = wload(min(k + 2, PC_K - 1), 1);
    tap(k, 0);
    wstore(1, vb0, vb1);
    __syncthreads();
    vb0 = wload(min(k + 3, PC_K - 1), 0);
    vb1 = wload(min(k + 3, PC_K - 1), 1);
    tap(k + 1, 1);
    wstore(0, va0, va1);
    __syncthreads();
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    if (!(mt == 0 ? one : two)) continue;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int n = nt * 32 + r;
      const float bs = kBwd ? 0.f : bias[g * PC_C + n];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int t = r0 + 32 * mt + (i & 3) + 8 * (i >> 2) + 4 * hh;
        if (t < T) {
          const int64_t o = base + (int64_t)t * PC_E + n;
          if (kBwd) {
            out[o] = f2h(acc[mt][nt][i]);
          } else {
            const hst ub = f2h(acc[mt][nt][i] + bs);
            uout[o] = ub;
            out[o] = f2h(pc_gelu(h2f(ub)));
          }
        }
      }
    }
  }
}

}  // namespace rdx

using namespace rdx;

static int pc2_launch(bool bwd, const void* in, const void* u, const void* wk, const float* bias, void* out,
                      void* uout, int B, int T, int off, hipStream_t st) {
  constexpr int smem = PC2_LDS;
  static bool attr = false;
  if (!attr) {
    for (const void* f : {reinterpret_cast<const void*>(&posconv2_kernel<false>),
                          reinterpret_cast<const void*>(&posconv2_kernel<true>)}) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
      if (e != hipSuccess) return (int)e;
    }
    attr = true;
  }
  dim3 grid(PC_G, B);
  if (bwd)
    hipLaunchKernelGGL(posconv2_kernel<true>, grid, dim3(256), smem, st, (const hst*)in,
                       (const hst*)u, (const hst*)wk, nullptr, (hst*)out, nullptr, T,
                       off);
  else
    hipLaunchKernelGGL(posconv2_kernel<false>, grid, dim3(256), smem, st, (const hst*)in, nullptr,
                       (const hst*)wk, bias, (hst*)out, (hst*)uout, T, off);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

static bool pc_ok(const void* p) { return p && ((uintptr_t)p & 15) == 0; }

extern "C" int rdx_posconv_fwd(const void* h, const void* wk, const float* bias, void* y, void* u, int B, int T,
                               void* stream) {
  RDX_REQUIRE(pc_ok(h) && pc_ok(wk) && bias && pc_ok(y) && pc_ok(u) && B > 0 && T > 0 && B <= 65535);
  if (T <= PC2_ROWS) return pc2_launch(false, h, nullptr, wk, bias, y, u, B, T, PC_K / 2, as_stream(stream));
  dim3 grid((T + PC_ROWS - 1) / PC_ROWS, PC_G, B);
  hipLaunchKernelGGL(posconv_kernel<false>, grid, dim3(256), 0, as_stream(stream), (const hst*)h, nullptr,
                     (const hst*)wk, bias, (hst*)y, (hst*)u, T, PC_K / 2);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_posconv_bwd(const void* dy, const void* u, const void* wkt, void* dh, int B, int T, void* stream) {
  RDX_REQUIRE(pc_ok(dy) && pc_ok(u) && pc_ok(wkt) && pc_ok(dh) && B > 0 && T > 0 && B <= 65535);
  if (T <= PC2_ROWS) return pc2_launch(true, dy, u, wkt, nullptr, dh, nullptr, B, T, PC_K / 2 - 1, as_stream(stream));
  dim3 grid((T + PC_ROWS - 1) / PC_ROWS, PC_G, B);
  hipLaunchKernelGGL(posconv_kernel<true>, grid, dim3(256), 0, as_stream(stream), (const hst*)dy,
                     (const hst*)u, (const hst*)wkt, nullptr, (hst*)dh, nullptr, T,
                     PC_K / 2 - 1);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
