// SincNet block 0 forward in ONE pass: Residual_block with one input channel (src/models/DualStreamSEMamba.py:
// 182-200, AASIST's first block) with frozen batch-norm (freeze_bn, src/main.py:44-51):
//     c    = conv1(x)                      (1 -> 32 channels, 2 x 3, padding (1, 1): H + 1 rows)
//     out1 = selu(bn2(c + conv1.bias))
//     a    = conv2(out1)                   (32 -> 32, 2 x 3, padding (0, 1): H rows)
//     idn  = conv_downsample(x)            (1 -> 32, 1 x 3, padding (0, 1))
//     y    = MaxPool2d((1, 3))(a + idn + conv2.bias + conv_downsample.bias)
// The unfused path (rdx_sincnet_b0_fwd + rdx_sconv_fwd + rdx_res_tail_fwd) writes c, out1, idn and a to HBM,
// four [N, H(+1), W, 32] bf16 tensors (~1 GB each at 32 utterances of 64 600 samples) and reads three of them
// back; here only x (one channel) is read and only the pooled output (a third of one tensor) and the window
// argmax bytes are written. The backward needs c / out1 / a + idn only through the argmax, and recomputes the
// rest from x.
//
// A 256-thread workgroup owns a strip of 42 pooled outputs (126 positions) of one utterance and walks its rows
// top-down. Per output row h: conv1 + BN + SELU of out1 row h + 2 into a 3-slot LDS ring (VALU, the unfused
// kernel's arithmetic and roundings: c rounded to bf16, out1 to bf16), conv2 from out1 rows h, h + 1 on
// mfma_f32_32x32x16_bf16 exactly as csrc/sconv.hip orders it (taps kh, kw, then 16-channel steps: the same fp32
// sums), a and idn rounded to bf16 as the unfused kernels store them, s = (a + idn) + bias staged in LDS, then
// the (1, 3) max pool with torch's rule (first maximum wins, NaN propagates). So y and the argmax equal the
// unfused path's bit for bit.
#include "common.h"

namespace rdx {

typedef __attribute__((ext_vector_type(8))) __bf16 bxbf16x8;
typedef __attribute__((ext_vector_type(16))) float bxf32x16;

constexpr float BX_SELU_ALPHA = 1.6732632423543772848170429916717f;
constexpr float BX_SELU_SCALE = 1.0507009873554804934193349852946f;
constexpr int BX_T = 256;
constexpr int BX_C = 32;        // channels of conv1 / conv2 / conv_downsample
constexpr int BX_J = 42;        // pooled outputs per strip
constexpr int BX_P = 3 * BX_J;  // 126 positions per strip (the pool windows it owns)
constexpr int BX_IR = 136;      // out1 image rows: positions q0 - 1 .. q0 + 128 (130 used), whole 8-row subtiles
constexpr int BX_XW = 132;      // staged x positions q0 - 2 .. q0 + 129
constexpr int BX_SP = 36;       // fp32 pitch of the pre-pool row (32 channels + 4: spreads the row stores)
constexpr int BX_IMG = BX_IR * 64;
constexpr int BX_LDS = 192 * 64 + 3 * BX_IMG + 4 * BX_XW * 4 + 128 * BX_SP * 4 + 32 * 16;

__device__ __forceinline__ float bx_selu(float u) {
  return BX_SELU_SCALE * (u > 0.f ? u : BX_SELU_ALPHA * (__expf(u) - 1.0f));
}
__device__ __forceinline__ float bx_bf16(float x) { return __bfloat162float(__float2bfloat16(x)); }
__device__ __forceinline__ uint32_t bx_pack2(float a, float b) {
  return (uint32_t)__bfloat16_as_ushort(__float2bfloat16(a)) | ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(b)) << 16);
}
// [row][32] bf16 image: 8-row x 32-channel subtiles of 512 B, the 16-byte chunk XOR-swizzled by (row >> 2) & 3
// (csrc/sconv.hip sc_img<32>)
__device__ __forceinline__ int bx_img(int row, int ch) {
  return 512 * (row >> 3) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}

struct BxFwdArgs {
  const __hip_bfloat16* x;   // [N, H, W] (the one input channel)
  const float* w1;           // [32][6] conv1 weights as autocast rounds them (bf16 values), tap kh * 3 + kw
  const float* wd;           // [32][3] conv_downsample weights (bf16 values)
  const float* bn;           // [4][32]: conv1 bias, running mean, invstd * gamma, beta
  const __hip_bfloat16* w2;  // [6][32 co][32 ci] conv2 weights, tap-major
  const float* bias;         // [32] conv2.bias + conv_downsample.bias
  __hip_bfloat16* y;         // [N, H, Wo, 32] pooled output (NHWC)
  uint8_t* arg;              // [N, H, Wo, 32] window argmax (0..2)
  int N, H, W, Wo, rows_per;
};

__global__ __launch_bounds__(BX_T, 2) void b0x_fwd_kernel(BxFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* ws = lds;                                           // conv2 weights: rows tap * 32 + co
  char* os = ws + 192 * 64;                                 // out1 ring: 3 slots
  float* xr = reinterpret_cast<float*>(os + 3 * BX_IMG);    // x ring: 4 rows of BX_XW
  float* ss = xr + 4 * BX_XW;                               // s = a + idn + bias of the current row
  float4* prec = reinterpret_cast<float4*>(ss + 128 * BX_SP);   // [32] {wd[co][0..2], bias[co]}
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int strip = blockIdx.x, n = blockIdx.y;
  const int q0 = strip * BX_P;
  const int H = a.H, W = a.W;
  const int h0 = blockIdx.z * a.rows_per, h1 = min(H, h0 + a.rows_per);
  if (h0 >= h1) return;
  for (int i = tid; i < 192 * 4; i += BX_T) {
    const int row = i >> 2, ch = i & 3;
    *reinterpret_cast<uint4*>(ws + bx_img(row, ch)) = *reinterpret_cast<const uint4*>(a.w2 + row * BX_C + ch * 8);
  }
  if (tid < 32) prec[tid] = make_float4(a.wd[tid * 3], a.wd[tid * 3 + 1], a.wd[tid * 3 + 2], a.bias[tid]);
  // this thread's out1 channels: 8 * g8 .. + 7 (its items it = tid + 256 k all have it & 3 == tid & 3)
  const int g8 = tid & 3;
  float t1[8][6], cb[8], mu[8], sg[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int co = g8 * 8 + k;
#pragma unroll
    for (int j = 0; j < 6; ++j) t1[k][j] = a.w1[co * 6 + j];
    cb[k] = a.bn[co];
    mu[k] = a.bn[BX_C + co];
    sg[k] = a.bn[2 * BX_C + co];
    sh[k] = a.bn[3 * BX_C + co];
  }
  const __hip_bfloat16* xn_base = a.x + (int64_t)n * H * W;
  auto load_x = [&](int row) -> float {   // x[row][q0 - 2 + tid], zero outside the image
    const int q = q0 - 2 + tid;
    return (tid < BX_XW && row >= 0 && row < H && q >= 0 && q < W) ? __bfloat162float(xn_base[(int64_t)row * W + q])
                                                                    : 0.f;
  };
  auto xslot = [&](int row) -> float* { return xr + (row & 3) * BX_XW; };
  auto oslot = [&](int row) -> char* { return os + (row % 3) * BX_IMG; };
  // out1 row ro (0 .. H) at positions q0 - 1 + pp, pp < 130 (zero outside [0, W): conv2's padding)
  auto make_out1 = [&](int ro) {
    const float* xa = xslot(ro - 1);
    const float* xb = xslot(ro);
    char* sl = oslot(ro);
    for (int it = tid; it < 130 * 4; it += BX_T) {
      const int pp = it >> 2;
      const int q = q0 - 1 + pp;
      const float v0[3] = {xa[pp], xa[pp + 1], xa[pp + 2]}, v1[3] = {xb[pp], xb[pp + 1], xb[pp + 2]};
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 8; k += 2) {
        float yv[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          float acc = v0[0] * t1[k + e][0];
          acc = fmaf(v0[1], t1[k + e][1], acc);
          acc = fmaf(v0[2], t1[k + e][2], acc);
          acc = fmaf(v1[0], t1[k + e][3], acc);
          acc = fmaf(v1[1], t1[k + e][4], acc);
          acc = fmaf(v1[2], t1[k + e][5], acc);
          const float cv = bx_bf16(acc);
          yv[e] = bx_selu(fmaf((cv + cb[k + e]) - mu[k + e], sg[k + e], sh[k + e]));
        }
        o[k >> 1] = (q >= 0 && q < W) ? bx_pack2(yv[0], yv[1]) : 0u;
      }
      *reinterpret_cast<uint4*>(sl + bx_img(pp, g8)) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  };
  const int pw = wv * 32 + r;   // this lane's output position q0 + pw (B operand row of the MFMA)

  {  // prologue: x rows h0 - 1 .. h0 + 2, out1 rows h0 and h0 + 1
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = load_x(h0 - 1 + i);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (tid < BX_XW) xslot(h0 - 1 + i)[tid] = v[i];
  }
  __syncthreads();
  make_out1(h0);
  make_out1(h0 + 1);
  __syncthreads();
  for (int h = h0; h < h1; ++h) {
    const float xnext = load_x(h + 3);
    bxf32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const char* xk = oslot(h + kh);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bxbf16x8 xf = *reinterpret_cast<const bxbf16x8*>(xk + bx_img(pw + kw, 2 * s + hh));
          const bxbf16x8 wf = *reinterpret_cast<const bxbf16x8*>(ws + bx_img((kh * 3 + kw) * BX_C + r, 2 * s + hh));
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf, xf, acc, 0, 0, 0);   // Y^T: rows co, columns positions
        }
    }
    if (h + 1 < h1) make_out1(h + 2);   // the next row's second input row (slot of row h - 1: read last row)
    {  // s = (a + idn) + bias at position q0 + pw, channels 8g + 4hh + e
      const float* xh = xslot(h);
      const float x0 = xh[pw + 1], x1 = xh[pw + 2], x2 = xh[pw + 3];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = 8 * g + 4 * hh + e;
          const float av = bx_bf16(acc[4 * g + e]);
          const float4 pr = prec[co];
          const float iv = bx_bf16(fmaf(x0, pr.x, fmaf(x1, pr.y, x2 * pr.z)));
          o[e] = av + iv + pr.w;
        }
        *reinterpret_cast<float4*>(ss + pw * BX_SP + 8 * g + 4 * hh) = make_float4(o[0], o[1], o[2], o[3]);
      }
    }
    if (tid < BX_XW) xslot(h + 3)[tid] = xnext;   // the slot of x row h - 1 (no reader after the last barrier)
    __syncthreads();
    if (tid < BX_J * 4) {   // pool: (window j, 8 channels) per thread, 16-byte stores of consecutive chunks
      const int j = tid >> 2, g = tid & 3;
      const int jo = strip * BX_J + j;
      if (jo < a.Wo) {
        float best[8];
        uint32_t bi[8];
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          const float* sp = ss + (3 * j + t) * BX_SP + 8 * g;
          const float4 lo = *reinterpret_cast<const float4*>(sp), hi = *reinterpret_cast<const float4*>(sp + 4);
          const float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (t == 0 || v[k] > best[k] || v[k] != v[k]) {   // torch max_pool2d: val > max || isnan(val)
              best[k] = v[k];
              bi[k] = (uint32_t)t;
            }
        }
        const int64_t o = (((int64_t)n * H + h) * a.Wo + jo) * BX_C + 8 * g;
        *reinterpret_cast<uint4*>(a.y + o) = make_uint4(bx_pack2(best[0], best[1]), bx_pack2(best[2], best[3]),
                                                        bx_pack2(best[4], best[5]), bx_pack2(best[6], best[7]));
        *reinterpret_cast<uint2*>(a.arg + o) = make_uint2(bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24),
                                                          bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24));
      }
    }
    __syncthreads();
  }
}

}  // namespace rdx

using namespace rdx;

extern "C" int rdx_b0x_fwd(const void* x, const float* w1, const float* wd, const float* bn, const void* w2,
                           const float* bias, void* y, uint8_t* arg, int N, int H, int W, void* stream) {
  RDX_REQUIRE(x && w1 && wd && bn && w2 && bias && y && arg && N > 0 && H > 0 && W >= 3);
  RDX_REQUIRE(((uintptr_t)y & 15) == 0 && ((uintptr_t)arg & 7) == 0 && ((uintptr_t)w2 & 15) == 0);
  RDX_REQUIRE(N < 65536);
  const int Wo = W / 3;
  const int strips = (Wo + BX_J - 1) / BX_J;
  // row chunks only when the (strip, utterance) grid alone cannot fill the chip (each chunk recomputes 2 rows)
  int nz = (int)((2048 + (int64_t)strips * N - 1) / ((int64_t)strips * N));
  nz = nz < 1 ? 1 : (nz > 6 ? 6 : nz);
  const int rows_per = (H + nz - 1) / nz;
  nz = (H + rows_per - 1) / rows_per;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&b0x_fwd_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, BX_LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  BxFwdArgs a{(const __hip_bfloat16*)x, w1, wd, bn, (const __hip_bfloat16*)w2, bias, (__hip_bfloat16*)y, arg,
              N, H, W, Wo, rows_per};
  hipLaunchKernelGGL(b0x_fwd_kernel, dim3((unsigned)strips, (unsigned)N, (unsigned)nz), dim3(BX_T), BX_LDS,
                     as_stream(stream), a);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

// ------------------------------------------------------------------------------------------------------------
// Backward in ONE pass: from the pooled output gradient dp (and the forward's window argmax) to dx and every
// parameter gradient of the block, recomputing c and out1 from x instead of reading the unfused path's
// intermediates (unfused: res_tail_bwd + sconv_dgrad_bnselu + sconv_wgrad + sincnet_b0_bwd, ~11 GB of HBM
// traffic at 32 utterances; here x, dp and the argmax are read and dx written):
//     ds[h, w, co]    = dp[h, w / 3, co] if w is its window's argmax (w < 3 Wo) else 0       (pool backward)
//     d(conv2.bias) = d(conv_downsample.bias) = sum ds;   d wd[co, kw] = sum ds[h, w, co] x[h, w + kw - 1]
//     d w2[co, ci, kh, kw] = sum ds[h, w, co] out1[h + kh, w + kw - 1, ci]                    (MFMA, K = w)
//     dout1[h', q, ci] = sum ds[h' + kh - 1, q + kw - 1, co] w2flip[kh, kw][ci, co]           (MFMA)
//     dc = bf16(bf16(dout1) selu'(u) s), u = (c + cb - mean) s + beta, s = invstd gamma; BN sums as
//          rdx_sconv_dgrad_bnselu (d cb = sum dc, d gamma = sum du xhat, d beta = sum du)
//     d w1[co, kh, kw] = sum dc[h', q, co] x[h' + kh - 1, q + kw - 1]
//     dx[h, w] = sum_co ( sum_{kh,kw} dc[h + 1 - kh, w + 1 - kw, co] w1[co, kh, kw] + sum_kw ds[h, w + 1 - kw, co] wd[co, kw] )
// dc and ds carry the unfused path's bf16 roundings and dout1 its MFMA order, so dc and every gradient equal
// the unfused ones up to the order of their fp32 sums.
//
// A workgroup walks units (utterance, strip of 126 positions) in a grid-stride loop and, per unit, the H + 1
// rows h' of dout1 top-down in four phases: (A) ds row h' into an LDS ring of 2 (its pooled gradient and argmax
// fetched a row ahead), out1 row h' + 1 (ring of 2); (B) dout1 row h' on the MFMA into the dc ring (2 rows) and
// the d w2 MFMAs of ds row h'; (C) the BN + SELU backward of dout1 in place, with a thread owning 8 channels
// (c recomputed from x); (D) dx row h' - 1, d w1, d wd and the bias sums, a thread owning 4 channels. Every sum counts the strip's own positions
// [126 s, 126 s + 126) (the d w2 MFMA runs K over 128 positions and zeroes the last two); with Wo / 42 + 1
// strips they partition every position that carries a gradient. Per-workgroup sums go to one fp32 partial row (the caller sums the rows: no atomics).
constexpr int BXB_DCR = 128;                         // dc image rows: positions q0 - 1 .. q0 + 126
constexpr int BXB_XW = 136;                          // staged x positions q0 - 4 .. q0 + 131
constexpr int BXB_NPART = 6 * 32 * 32 + 32 * 6 + 32 * 3 + 32 + 3 * 32;
constexpr int BXB_LDS = 192 * 64 + 3 * BX_IMG + 2 * BX_IMG + 2 * BXB_DCR * 64 + 4 * BXB_XW * 4 + 32 * 64;
constexpr int BXB_BLOCKS = 512;

typedef __attribute__((__vector_size__(4 * sizeof(__bf16)))) __bf16 bxbf16x4v;
typedef __attribute__((address_space(3))) bxbf16x4v lds_bxbf16x4v;

// MFMA operand running down a column of a bx_img image (K = positions), csrc/sconv.hip sc_read_tr<32>
__device__ __forceinline__ bxbf16x8 bx_read_tr(const char* img, int r0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int row = r0 + 16 * s + 4 * (g >> 1) + (i >> 2);
  const int col = 16 * (g & 1) + 4 * (i & 3);
  const int sub = 2 * (col & 7);
  const bxbf16x4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bxbf16x4v*)(img + bx_img(row, col >> 3) + sub));
  const bxbf16x4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bxbf16x4v*)(img + bx_img(row + 8, col >> 3) + sub));
  bxbf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = lo[j];
    r[4 + j] = hi[j];
  }
  return r;
}
// the same read from precomputed per-lane byte offsets (lo, hi) of K step 0: step s adds 1024 bytes (16 image
// rows = two 512-byte subtiles, the swizzle repeats), so the loop keeps 2 offsets live instead of 16 addresses
__device__ __forceinline__ int2 bx_tr_off(int r0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int row = r0 + 4 * (g >> 1) + (i >> 2);
  const int col = 16 * (g & 1) + 4 * (i & 3);
  const int sub = 2 * (col & 7);
  return make_int2(bx_img(row, col >> 3) + sub, bx_img(row + 8, col >> 3) + sub);
}
__device__ __forceinline__ bxbf16x8 bx_read_tr_at(const char* img, int2 off, int s) {
  const bxbf16x4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bxbf16x4v*)(img + off.x + 1024 * s));
  const bxbf16x4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bxbf16x4v*)(img + off.y + 1024 * s));
  bxbf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = lo[j];
    r[4 + j] = hi[j];
  }
  return r;
}
__device__ __forceinline__ float bx_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bx_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

struct BxBwdArgs {
  const __hip_bfloat16* x;    // [N, H, W]
  const __hip_bfloat16* dp;   // [N, H, Wo, 32] pooled-output gradient
  const uint8_t* arg;         // [N, H, Wo, 32]
  const float* w1;            // [32][6]
  const float* wd;            // [32][3]
  const float* bn;            // [5][32]: conv1 bias, mean, invstd * gamma, beta, invstd
  const __hip_bfloat16* w2f;  // [6][32 ci][32 co] conv2 weights flipped in both axes, transposed (input gradient)
  float* dx;                  // [N, H, W]
  float* part;                // [gridDim.x][BXB_NPART]: d w2 [6][32 co][32 ci], d w1 [32][6], d wd [32][3],
                              //   d bias [32], BN sums [3][32]
  int N, H, W, Wo, strips;
};

#ifdef BX_PROF
// tools/prof_b0x.hip: per-workgroup shader-cycle sums of the backward's phases (A, B, C, D, unit prologue)
__device__ unsigned long long bx_prof[BXB_BLOCKS][5];
#define BX_STAMP(k)                     \
  do {                                  \
    const long long t_ = clock64();     \
    prof_acc[k] += t_ - prof_t;         \
    prof_t = t_;                        \
  } while (0)
#else
#define BX_STAMP(k) \
  do {              \
  } while (0)
#endif

__global__ __launch_bounds__(BX_T, 2) void b0x_bwd_kernel(BxBwdArgs a) {
#ifdef BX_PROF
  long long prof_acc[5] = {0, 0, 0, 0, 0};
  long long prof_t = clock64();
#endif
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* wsf = lds;                                           // flipped conv2 weights: rows tap * 32 + ci
  char* dsr = wsf + 192 * 64;                                // ds ring (3): row i <-> position q0 - 2 + i
  char* o1r = dsr + 3 * BX_IMG;                              // out1 ring (2): row i <-> q0 - 3 + i
  char* dcr = o1r + 2 * BX_IMG;                              // dO, then dc, ring (2): row i <-> q0 - 1 + i
  float* xr = reinterpret_cast<float*>(dcr + 2 * BXB_DCR * 64);   // x ring (4): index i <-> q0 - 4 + i
  // per-channel record (four 16-byte reads): w1[0..5], wd[0..2], conv1 bias, mean, invstd * gamma, beta, invstd;
  // part j of channel co at float4 j * 32 + co (the channels one instruction reads spread over the bank slots)
  float4* prec = reinterpret_cast<float4*>(xr + 4 * BXB_XW);   // [4][32]
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int H = a.H, W = a.W, Wo = a.Wo, W3 = 3 * a.Wo;
  for (int i = tid; i < 192 * 4; i += BX_T) {
    const int row = i >> 2, ch = i & 3;
    *reinterpret_cast<uint4*>(wsf + bx_img(row, ch)) = *reinterpret_cast<const uint4*>(a.w2f + row * BX_C + ch * 8);
  }
  if (tid < 32) {
    const float* w1 = a.w1 + tid * 6;
    const float* wd = a.wd + tid * 3;
    prec[tid] = make_float4(w1[0], w1[1], w1[2], w1[3]);
    prec[32 + tid] = make_float4(w1[4], w1[5], wd[0], wd[1]);
    prec[64 + tid] = make_float4(wd[2], a.bn[tid], a.bn[BX_C + tid], a.bn[2 * BX_C + tid]);
    prec[96 + tid] = make_float4(a.bn[3 * BX_C + tid], a.bn[4 * BX_C + tid], 0.f, 0.f);
  }
  // out1 image rows 130, 131 (positions q0 + 127, q0 + 128) meet only the zeroed ds elements of the d w2 MFMA
  // (below): zeros, never stale LDS; phase C writes rows 2 .. 129
  if (tid < 16)
    *reinterpret_cast<uint4*>(o1r + (tid >> 3) * BX_IMG + bx_img(130 + ((tid >> 2) & 1), tid & 3)) =
        make_uint4(0u, 0u, 0u, 0u);
  // persistent per-thread sums. Phase C (dc) owns channels 8 c8 .. 8 c8 + 7 (c8 = tid & 3): BN sums;
  // phase D (dx) owns channels 4 g .. 4 g + 3 (g = tid & 7): d w1, d wd, d bias; the d w2 MFMA tiles
  const int c8 = tid & 3, g = tid & 7;
  float bsum[3][8];
  float aw1[4][6], awd[4][3], abias[4];
#pragma unroll
  for (int k = 0; k < 8; ++k) bsum[0][k] = bsum[1][k] = bsum[2][k] = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 6; ++j) aw1[i][j] = 0.f;
#pragma unroll
    for (int j = 0; j < 3; ++j) awd[i][j] = 0.f;
    abias[i] = 0.f;
  }
  bxf32x16 acc2[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc2[t][i] = 0.f;
  const int pw = wv * 32 + r;    // dout1 position q0 - 1 + pw of this lane in phase B
  __syncthreads();
  constexpr int DSN = (BX_IR * 4 + BX_T - 1) / BX_T;   // ds items per thread (3)
  auto ds_slot = [&](int h) -> char* { return dsr + ((h + 3) % 3) * BX_IMG; };   // h >= -3

  for (int64_t u = blockIdx.x; u < (int64_t)a.strips * a.N; u += gridDim.x) {
    const int strip = (int)(u % a.strips), n = (int)(u / a.strips);
    const int q0 = strip * BX_P;
    const __hip_bfloat16* xn = a.x + (int64_t)n * H * W;
    // x row `row` at position q0 - 4 + tid: raw bf16 bits from a clamped (always valid) address, so the load
    // carries no branch and its wait falls where the row is stored (x_val), a phase or more later
    auto x_raw = [&](int row) -> uint32_t {
      const int q = q0 - 4 + tid;
      const int rc = row < 0 ? 0 : (row >= H ? H - 1 : row);
      const int qc = q < 0 ? 0 : (q >= W ? W - 1 : q);
      return reinterpret_cast<const uint16_t*>(xn)[(int64_t)rc * W + qc];
    };
    auto x_val = [&](int row, uint32_t raw) -> float {   // zero outside the image
      const int q = q0 - 4 + tid;
      return (row >= 0 && row < H && q >= 0 && q < W) ? __uint_as_float(raw << 16) : 0.f;
    };
    auto xslot = [&](int row) -> float* { return xr + (row & 3) * BXB_XW; };
    // conv1 pre-activation c (bf16-rounded, the unfused kernel's FMA order) at x columns v0 / v1, from a record
    auto conv1c = [&](const float (&v0)[3], const float (&v1)[3], const float4& r0, const float4& r1) -> float {
      float acc = v0[0] * r0.x;
      acc = fmaf(v0[1], r0.y, acc);
      acc = fmaf(v0[2], r0.z, acc);
      acc = fmaf(v1[0], r0.w, acc);
      acc = fmaf(v1[1], r1.x, acc);
      acc = fmaf(v1[2], r1.y, acc);
      return bx_bf16(acc);
    };
    // ds row hrow: the pooled gradient where the window argmax hits, fetched a row ahead into registers
    uint4 pd[DSN];
    uint2 pa[DSN];
    auto fetch_ds = [&](int hrow) {
#pragma unroll
      for (int j = 0; j < DSN; ++j) {
        const int it = tid + BX_T * j;
        const int i = it >> 2;
        const int w = q0 - 2 + i;
        pd[j] = make_uint4(0u, 0u, 0u, 0u);
        pa[j] = make_uint2(0xffffffffu, 0xffffffffu);
        if (it < BX_IR * 4 && hrow >= 0 && hrow < H && i < 130 && w >= 0 && w < W3) {
          const int jj = w / 3;
          const int64_t off = (((int64_t)n * H + hrow) * Wo + jj) * BX_C + 8 * c8;
          pd[j] = *reinterpret_cast<const uint4*>(a.dp + off);
          pa[j] = *reinterpret_cast<const uint2*>(a.arg + off);
        }
      }
    };
    auto store_ds = [&](int hrow) {
      char* sl = ds_slot(hrow);
#pragma unroll
      for (int j = 0; j < DSN; ++j) {
        const int it = tid + BX_T * j;
        if (it < BX_IR * 4) {
          const int i = it >> 2;
          const uint32_t t = (uint32_t)((q0 - 2 + i + 3) % 3);   // window slot of position q0 - 2 + i
          const uint32_t dw[4] = {pd[j].x, pd[j].y, pd[j].z, pd[j].w};
          uint32_t ow[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const uint32_t bits = e < 2 ? pa[j].x >> (16 * e) : pa[j].y >> (16 * (e - 2));
            const uint32_t m0 = ((bits & 0xff) == t) ? 0x0000ffffu : 0u;
            const uint32_t m1 = (((bits >> 8) & 0xff) == t) ? 0xffff0000u : 0u;
            ow[e] = dw[e] & (m0 | m1);
          }
          *reinterpret_cast<uint4*>(sl + bx_img(i, c8)) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
        }
      }
    };
    __syncthreads();   // the previous unit's readers are done
    {
      uint32_t v[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) v[i] = x_raw(i - 1);
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if (tid < BXB_XW) xslot(i - 1)[tid] = x_val(i - 1, v[i]);
    }
    fetch_ds(-1);
    store_ds(-1);       // zeros
    fetch_ds(0);
    BX_STAMP(4);
    // iteration hp: dout1 / dc row hp (hp <= H), out1 row hp (phase C, used by the d w2 MFMAs of ds row hp - 1 and
    // hp - 2 in the next two iterations), dx row hp - 1, d w2 of ds row hp - 2 (hp >= 2: out1 rows hp - 2, hp - 1)
    for (int hp = 0; hp <= H + 1; ++hp) {
      const bool rowc = hp <= H;
      // ---- phase A: ds row hp (registers -> LDS), the next row's fetch, x row hp + 2 in flight
      const uint32_t xnext = x_raw(hp + 2);
      store_ds(hp);
      fetch_ds(hp + 1);
      __syncthreads();
      BX_STAMP(0);
      // ---- phase B: dout1 row hp = conv(ds rows hp - 1, hp) with the flipped weights -> bf16 into the dc slot;
      // d w2 += ds row hp - 2 x out1 rows hp - 2, hp - 1 over K = ds image rows 2 .. 129 (positions q0 .. q0 + 127);
      // rows 128 and 129 (q0 + 126, q0 + 127) belong to the next strip: their A elements are zeroed (in the last
      // K step, element j of lane l holds row 2 + 112 + 8 (j >> 2) + 4 (l >> 5) + (j & 3): elements 6, 7 of lanes
      // 32-63)
      if (rowc) {
        bxf32x16 acc;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 0.f;
        // weight rows tap * 32 + r: 2048 bytes per tap; input rows pw + kw
        const int wo0 = bx_img(r, hh), wo1 = bx_img(r, 2 + hh);
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
          const char* dk = ds_slot(hp - 1 + kh);
#pragma unroll
          for (int kw = 0; kw < 3; ++kw)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
              const bxbf16x8 xf = *reinterpret_cast<const bxbf16x8*>(dk + bx_img(pw + kw, 2 * s + hh));
              const bxbf16x8 wf = *reinterpret_cast<const bxbf16x8*>(wsf + (kh * 3 + kw) * 2048 + (s ? wo1 : wo0));
              acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf, xf, acc, 0, 0, 0);
            }
        }
        char* dcs = dcr + (hp & 1) * (BXB_DCR * 64);
#pragma unroll
        for (int gg = 0; gg < 4; ++gg)
          *reinterpret_cast<uint2*>(dcs + bx_img(pw, gg) + 8 * hh) =
              make_uint2(bx_pack2(acc[4 * gg], acc[4 * gg + 1]), bx_pack2(acc[4 * gg + 2], acc[4 * gg + 3]));
      }
      if (hp >= 2) {
        const char* dsi = ds_slot(hp - 2);
        const bool tail_lane = (lane >> 5) == 1;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int tap = wv + 4 * t;
          if (tap < 6) {
            const int kh = tap / 3, kw = tap - 3 * kh;
            const char* oi = o1r + ((hp + kh) & 1) * BX_IMG;   // out1 row hp - 2 + kh
            const int2 offa = bx_tr_off(2, lane), offb = bx_tr_off(2 + kw, lane);
#pragma unroll
            for (int s = 0; s < 8; ++s) {
              bxbf16x8 av = bx_read_tr_at(dsi, offa, s);
              if (s == 7 && tail_lane) {
                av[6] = (__bf16)0.0f;
                av[7] = (__bf16)0.0f;
              }
              acc2[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bx_read_tr_at(oi, offb, s), acc2[t], 0, 0, 0);
            }
          }
        }
      }
      __syncthreads();
      BX_STAMP(1);
      if (rowc) {
        // ---- phase C: dc row hp = bf16(dO selu'(u) s) in place (rdx_sconv_dgrad_bnselu's arithmetic on c
        // recomputed from x), BN sums over the strip's own positions; out1 row hp = selu(u) (rdx_sincnet_b0_fwd's
        // value, one exp for both) into the out1 slot of row hp - 2 (read for the last time in phase B above)
        {
          char* dcs = dcr + (hp & 1) * (BXB_DCR * 64);
          char* o1s = o1r + (hp & 1) * BX_IMG;
          const float* xa = xslot(hp - 1);
          const float* xb = xslot(hp);
#pragma unroll
          for (int jt = 0; jt < 2; ++jt) {
            const int it = tid + BX_T * jt;
            const int i = it >> 2;
            const int q = q0 - 1 + i;
            const bool inside = q >= 0 && q < W;
            const bool own = inside && i >= 1 && i <= BX_P;
            uint4* slot = reinterpret_cast<uint4*>(dcs + bx_img(i, c8));
            const uint4 dov = *slot;
            const uint32_t dw[4] = {dov.x, dov.y, dov.z, dov.w};
            const float v0[3] = {xa[i + 2], xa[i + 3], xa[i + 4]}, v1[3] = {xb[i + 2], xb[i + 3], xb[i + 4]};
            uint32_t ow[4], oo[4];
#pragma unroll
            for (int k = 0; k < 8; k += 2) {
              float dz[2], yo[2];
#pragma unroll
              for (int e = 0; e < 2; ++e) {
                const int co = 8 * c8 + k + e;
                const float4 r0 = prec[co], r1 = prec[32 + co], r2 = prec[64 + co], r3 = prec[96 + co];
                const float cv = conv1c(v0, v1, r0, r1);
                const float zc = (cv + r2.y) - r2.z;
                const float xhat = zc * r3.y;
                const float uu = fmaf(zc, r2.w, r3.x);
                const float ex = __expf(uu);
                const float sd = uu > 0.f ? BX_SELU_SCALE : BX_SELU_SCALE * BX_SELU_ALPHA * ex;
                yo[e] = BX_SELU_SCALE * (uu > 0.f ? uu : BX_SELU_ALPHA * (ex - 1.0f));   // bx_selu(uu)
                const float dov_e = e == 0 ? bx_lo(dw[k >> 1]) : bx_hi(dw[k >> 1]);
                const float du = dov_e * sd;
                dz[e] = inside ? du * r2.w : 0.f;
                if (own) {
                  bsum[0][k + e] += dz[e];
                  bsum[1][k + e] = fmaf(du, xhat, bsum[1][k + e]);
                  bsum[2][k + e] += du;
                }
              }
              ow[k >> 1] = bx_pack2(dz[0], dz[1]);
              oo[k >> 1] = inside ? bx_pack2(yo[0], yo[1]) : 0u;
            }
            *slot = make_uint4(ow[0], ow[1], ow[2], ow[3]);
            *reinterpret_cast<uint4*>(o1s + bx_img(i + 2, c8)) = make_uint4(oo[0], oo[1], oo[2], oo[3]);
          }
        }
        __syncthreads();
        BX_STAMP(2);
        // ---- phase D: dx row hp - 1, d w1 (dc row hp), d wd / d bias (ds row hp) over the strip's own positions
        {
          const char* dcA = dcr + (hp & 1) * (BXB_DCR * 64);         // dc row hp
          const char* dcB = dcr + ((hp - 1) & 1) * (BXB_DCR * 64);   // dc row hp - 1
          const char* dsP = ds_slot(hp - 1);                         // ds row hp - 1
          const char* dsC = ds_slot(hp);                             // ds row hp
          const float* xa = xslot(hp - 1);
          const float* xb = xslot(hp);
          const int gc = g >> 1, sub = 8 * (g & 1);
          for (int it = tid; it < BX_P * 8; it += BX_T) {
            const int k = it >> 3;
            const int q = q0 + k;
            const bool valid = q < W;
            float pdx = 0.f;
            if (hp >= 1 && valid) {
#pragma unroll
              for (int kw = 0; kw < 3; ++kw) {
                const uint2 A = *reinterpret_cast<const uint2*>(dcA + bx_img(k + 2 - kw, gc) + sub);
                const uint2 Bv = *reinterpret_cast<const uint2*>(dcB + bx_img(k + 2 - kw, gc) + sub);
                const uint2 D = *reinterpret_cast<const uint2*>(dsP + bx_img(k + 3 - kw, gc) + sub);
                const float av[4] = {bx_lo(A.x), bx_hi(A.x), bx_lo(A.y), bx_hi(A.y)};
                const float bv[4] = {bx_lo(Bv.x), bx_hi(Bv.x), bx_lo(Bv.y), bx_hi(Bv.y)};
                const float dv[4] = {bx_lo(D.x), bx_hi(D.x), bx_lo(D.y), bx_hi(D.y)};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const int co = 4 * g + e;
                  const float4 r0 = prec[co], r1 = prec[32 + co], r2 = prec[64 + co];
                  const float w1a[6] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y}, wda[3] = {r1.z, r1.w, r2.x};
                  pdx = fmaf(av[e], w1a[kw], pdx);
                  pdx = fmaf(bv[e], w1a[3 + kw], pdx);
                  pdx = fmaf(dv[e], wda[kw], pdx);
                }
              }
            }
            pdx += __shfl_xor(pdx, 1, 64);
            pdx += __shfl_xor(pdx, 2, 64);
            pdx += __shfl_xor(pdx, 4, 64);
            if (hp >= 1 && valid && g == 0) a.dx[((int64_t)n * H + hp - 1) * W + q] = pdx;
            if (valid) {
              const uint2 C = *reinterpret_cast<const uint2*>(dcA + bx_img(k + 1, gc) + sub);
              const float cv[4] = {bx_lo(C.x), bx_hi(C.x), bx_lo(C.y), bx_hi(C.y)};
              const float xv0[3] = {xa[k + 3], xa[k + 4], xa[k + 5]}, xv1[3] = {xb[k + 3], xb[k + 4], xb[k + 5]};
#pragma unroll
              for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int kw = 0; kw < 3; ++kw) {
                  aw1[e][kw] = fmaf(cv[e], xv0[kw], aw1[e][kw]);
                  aw1[e][3 + kw] = fmaf(cv[e], xv1[kw], aw1[e][3 + kw]);
                }
              if (hp < H) {
                const uint2 S = *reinterpret_cast<const uint2*>(dsC + bx_img(k + 2, gc) + sub);
                const float sv[4] = {bx_lo(S.x), bx_hi(S.x), bx_lo(S.y), bx_hi(S.y)};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  abias[e] += sv[e];
#pragma unroll
                  for (int kw = 0; kw < 3; ++kw) awd[e][kw] = fmaf(sv[e], xv1[kw], awd[e][kw]);
                }
              }
            }
          }
        }
      }
      // x row hp + 2 into the slot of row hp - 2 (no reader in this row)
      if (tid < BXB_XW) xslot(hp + 2)[tid] = x_val(hp + 2, xnext);
      __syncthreads();
      BX_STAMP(3);
    }
  }
#ifdef BX_PROF
  if (tid == 0)
#pragma unroll
    for (int k = 0; k < 5; ++k) bx_prof[blockIdx.x][k] = (unsigned long long)prof_acc[k];
#endif
  // ---- per-workgroup partial row (fixed-order sums: bitwise repeatable) ----
  float* out = a.part + (int64_t)blockIdx.x * BXB_NPART;
#pragma unroll
  for (int t = 0; t < 2; ++t) {   // d w2: lane owns ci = lane & 31, co = (i & 3) + 8 (i >> 2) + 4 hh
    const int tap = wv + 4 * t;
    if (tap < 6)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int co = (i & 3) + 8 * (i >> 2) + 4 * hh;
        out[(tap * BX_C + co) * BX_C + r] = acc2[t][i];
      }
  }
  float* red = reinterpret_cast<float*>(lds);   // the rings are free: [256][40] + [256][24] thread sums
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 4; ++e) {
#pragma unroll
    for (int j = 0; j < 6; ++j) red[tid * 40 + e * 6 + j] = aw1[e][j];
#pragma unroll
    for (int j = 0; j < 3; ++j) red[tid * 40 + 24 + e * 3 + j] = awd[e][j];
    red[tid * 40 + 36 + e] = abias[e];
  }
  float* bred = red + 256 * 40;
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int k = 0; k < 8; ++k) bred[tid * 24 + q * 8 + k] = bsum[q][k];
  __syncthreads();
  // d w1 [32][6], d wd [32][3], d bias [32]: channel co = 4 g + e sums the 32 threads with tid & 7 == g
  for (int i = tid; i < 32 * 10; i += BX_T) {
    const int co = i / 10, j = i % 10, gq = co >> 2, e = co & 3;
    const int slot = j < 6 ? e * 6 + j : (j < 9 ? 24 + e * 3 + (j - 6) : 36 + e);
    float s = 0.f;
    for (int t = 0; t < 32; ++t) s += red[(t * 8 + gq) * 40 + slot];
    const int dst = j < 6 ? 6144 + co * 6 + j : (j < 9 ? 6144 + 192 + co * 3 + (j - 6) : 6144 + 192 + 96 + co);
    out[dst] = s;
  }
  if (tid < 96) {   // BN sums [3][32]: channel co = 8 c8 + k sums the 64 threads with tid & 3 == c8
    const int q = tid / 32, co = tid % 32, cq = co >> 3, k = co & 7;
    float s = 0.f;
    for (int t = 0; t < 64; ++t) s += bred[(t * 4 + cq) * 24 + q * 8 + k];
    out[6144 + 192 + 96 + 32 + q * 32 + co] = s;
  }
}

extern "C" int rdx_b0x_bwd_nblk(int N, int W) {
  const int64_t units = (int64_t)(W / 3 / BX_J + 1) * N;
  return (int)(units < BXB_BLOCKS ? units : BXB_BLOCKS);
}

extern "C" int rdx_b0x_bwd(const void* x, const void* dp, const uint8_t* arg, const float* w1, const float* wd,
                           const float* bn, const void* w2f, float* dx, float* part, int N, int H, int W,
                           void* stream) {
  RDX_REQUIRE(x && dp && arg && w1 && wd && bn && w2f && dx && part && N > 0 && H > 0 && W >= 3);
  RDX_REQUIRE(((uintptr_t)dp & 15) == 0 && ((uintptr_t)arg & 7) == 0 && ((uintptr_t)w2f & 15) == 0);
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&b0x_bwd_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, BXB_LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  BxBwdArgs a{(const __hip_bfloat16*)x, (const __hip_bfloat16*)dp, arg, w1, wd, bn, (const __hip_bfloat16*)w2f,
              dx, part, N, H, W, W / 3, W / 3 / BX_J + 1};
  hipLaunchKernelGGL(b0x_bwd_kernel, dim3((unsigned)rdx_b0x_bwd_nblk(N, W)), dim3(BX_T), BXB_LDS, as_stream(stream),
                     a);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
