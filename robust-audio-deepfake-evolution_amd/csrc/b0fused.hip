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
constexpr int BX_LDS = 3 * BX_IMG + 4 * BX_XW * 4 + 128 * BX_SP * 4 + 32 * 16;   // conv2 weights: registers

__device__ __forceinline__ float bx_selu(float u) {
  return BX_SELU_SCALE * (u > 0.f ? u : BX_SELU_ALPHA * (__expf(u) - 1.0f));
}
__device__ __forceinline__ uint32_t bx_pack2(float a, float b) {
  return (uint32_t)hbits_of(f2h(a)) | ((uint32_t)hbits_of(f2h(b)) << 16);
}
// [row][32] bf16 image: 8-row x 32-channel subtiles of 512 B, the 16-byte chunk XOR-swizzled by (row >> 2) & 3
// (csrc/sconv.hip sc_img<32>)
__device__ __forceinline__ int bx_img(int row, int ch) {
  return 512 * (row >> 3) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}
__device__ __forceinline__ float bx_lo(uint32_t u) { return hlo(u); }
__device__ __forceinline__ float bx_hi(uint32_t u) { return hhi(u); }

// Two channels at once on the packed fp32 VALU (v_pk_fma / v_pk_mul / v_pk_add: per component the same IEEE
// operations, so the results keep the scalar code's bits): conv1's pre-activation c (the unfused kernel's FMA
// order), rounded to bf16
typedef float bxf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bxf2 bx_conv1_pair(const float (&v0)[3], const float (&v1)[3], const bxf2 (&w)[6]) {
  bxf2 acc = v0[0] * w[0];
  acc = __builtin_elementwise_fma((bxf2)v0[1], w[1], acc);
  acc = __builtin_elementwise_fma((bxf2)v0[2], w[2], acc);
  acc = __builtin_elementwise_fma((bxf2)v1[0], w[3], acc);
  acc = __builtin_elementwise_fma((bxf2)v1[1], w[4], acc);
  acc = __builtin_elementwise_fma((bxf2)v1[2], w[5], acc);
  const uint32_t c = bx_pack2(acc.x, acc.y);
  return (bxf2){bx_lo(c), bx_hi(c)};
}

struct BxFwdArgs {
  const hst* x;   // [N, H, W] (the one input channel)
  const float* w1;           // [32][6] conv1 weights as autocast rounds them (bf16 values), tap kh * 3 + kw
  const float* wd;           // [32][3] conv_downsample weights (bf16 values)
  const float* bn;           // [4][32]: conv1 bias, running mean, invstd * gamma, beta
  const hst* w2;  // [6][32 co][32 ci] conv2 weights, tap-major
  const float* bias;         // [32] conv2.bias + conv_downsample.bias
  hst* y;         // [N, H, Wo, 32] pooled output (NHWC)
  uint8_t* arg;              // [N, H, Wo, 32] window argmax (0..2)
  int N, H, W, Wo, rows_per;
};

#ifdef BX_PROF
// tools/prof_b0x.hip: shader-cycle sums over every workgroup of the forward's row phases (conv2 MFMAs, out1 of
// row h + 2, s = a + idn + bias staging, pool)
__device__ unsigned long long bx_prof_f[4];
#define BXF_STAMP(k)                    \
  do {                                  \
    const long long t_ = clock64();     \
    pf_acc[k] += t_ - pf_t;             \
    pf_t = t_;                          \
  } while (0)
#else
#define BXF_STAMP(k) \
  do {               \
  } while (0)
#endif

__global__ __launch_bounds__(BX_T, 2) void b0x_fwd_kernel(BxFwdArgs a) {
#ifdef BX_PROF
  long long pf_acc[4] = {0, 0, 0, 0};
  long long pf_t = clock64();
#endif
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* os = lds;                                           // out1 ring: 3 slots
  float* xr = reinterpret_cast<float*>(os + 3 * BX_IMG);    // x ring: 4 rows of BX_XW
  float* ss = xr + 4 * BX_XW;                               // s = a + idn + bias of the current row
  float4* prec = reinterpret_cast<float4*>(ss + 128 * BX_SP);   // [32] {wd[co][0..2], bias[co]}
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int strip = blockIdx.x, n = blockIdx.y;
  const int q0 = strip * BX_P;
  const int H = a.H, W = a.W;
  const int h0 = blockIdx.z * a.rows_per, h1 = min(H, h0 + a.rows_per);
  if (h0 >= h1) return;
  // conv2's A operand (the weights, rows co = lane & 31) for all 6 taps x 2 K steps, held in registers for the whole
  // walk (48 VGPRs): read from LDS per row they were half of the conv2 phase's LDS traffic (12 of 24 KB per wave)
  hx8 wreg[6][2];
#pragma unroll
  for (int t = 0; t < 6; ++t)
#pragma unroll
    for (int s = 0; s < 2; ++s)
      wreg[t][s] = *reinterpret_cast<const hx8*>(a.w2 + (t * BX_C + (tid & 31)) * BX_C + (2 * s + ((tid >> 5) & 1)) * 8);
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
  const hst* xn_base = a.x + (int64_t)n * H * W;
  // x[row][q0 - 2 + tid] as raw bf16 bits from a clamped (always valid) address: no branch around the load, so
  // its wait falls where the value is stored (x_val), after the row's MFMAs
  auto x_raw = [&](int row) -> uint32_t {
    const int q = q0 - 2 + tid;
    const int rc = row < 0 ? 0 : (row >= H ? H - 1 : row);
    const int qc = q < 0 ? 0 : (q >= W ? W - 1 : q);
    return reinterpret_cast<const uint16_t*>(xn_base)[(int64_t)rc * W + qc];
  };
  auto x_val = [&](int row, uint32_t raw) -> float {   // zero outside the image
    const int q = q0 - 2 + tid;
    return (row >= 0 && row < H && q >= 0 && q < W) ? hlo(raw) : 0.f;
  };
  auto xslot = [&](int row) -> float* { return xr + (row & 3) * BX_XW; };
  auto oslot = [&](int row) -> char* { return os + (row % 3) * BX_IMG; };
  // out1 row ro (0 .. H) at positions q0 - 1 + pp, pp < 130 (zero outside [0, W): conv2's padding)
  // one item = (position pp, this thread's 8 channels); the out-of-image positions (conv2's zero padding) are
  // masked with an AND rather than branched around, and a thread's items (2 or 3) read their x taps together
  auto out1_item = [&](const float (&v0)[3], const float (&v1)[3], int pp, char* sl) {
    const int q = q0 - 1 + pp;
    const uint32_t msk = (q >= 0 && q < W) ? 0xffffffffu : 0u;
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
        const float cv = hround(acc);
        yv[e] = bx_selu(fmaf((cv + cb[k + e]) - mu[k + e], sg[k + e], sh[k + e]));
      }
      o[k >> 1] = bx_pack2(yv[0], yv[1]) & msk;
    }
    *reinterpret_cast<uint4*>(sl + bx_img(pp, g8)) = make_uint4(o[0], o[1], o[2], o[3]);
  };
  auto make_out1 = [&](int ro) {
    const float* xa = xslot(ro - 1);
    const float* xb = xslot(ro);
    char* sl = oslot(ro);
    static_assert(2 * BX_T <= 130 * 4 && 3 * BX_T >= 130 * 4, "2 or 3 items per thread");
    const int pa = tid >> 2, pb = (tid + BX_T) >> 2, pc = (tid + 2 * BX_T) >> 2;
    const bool has_c = tid + 2 * BX_T < 130 * 4;
    const int pcc = has_c ? pc : 0;
    const float a0[3] = {xa[pa], xa[pa + 1], xa[pa + 2]}, a1[3] = {xb[pa], xb[pa + 1], xb[pa + 2]};
    const float b0[3] = {xa[pb], xa[pb + 1], xa[pb + 2]}, b1[3] = {xb[pb], xb[pb + 1], xb[pb + 2]};
    const float c0[3] = {xa[pcc], xa[pcc + 1], xa[pcc + 2]}, c1[3] = {xb[pcc], xb[pcc + 1], xb[pcc + 2]};
    out1_item(a0, a1, pa, sl);
    out1_item(b0, b1, pb, sl);
    if (has_c) out1_item(c0, c1, pc, sl);
  };
  const int pw = wv * 32 + r;   // this lane's output position q0 + pw (B operand row of the MFMA)

  {  // prologue: x rows h0 - 1 .. h0 + 2, out1 rows h0 and h0 + 1
    uint32_t v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = x_raw(h0 - 1 + i);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (tid < BX_XW) xslot(h0 - 1 + i)[tid] = x_val(h0 - 1 + i, v[i]);
  }
  __syncthreads();
  make_out1(h0);
  make_out1(h0 + 1);
  __syncthreads();
#ifdef BX_PROF
  pf_t = clock64();
#endif
  for (int h = h0; h < h1; ++h) {
    const uint32_t xnext = x_raw(h + 3);
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
          const hx8 xf = *reinterpret_cast<const hx8*>(xk + bx_img(pw + kw, 2 * s + hh));
          acc = mfma32x32x16(wreg[kh * 3 + kw][s], xf, acc);   // Y^T: rows co, columns positions
        }
    }
    BXF_STAMP(0);
    if (h + 1 < h1) make_out1(h + 2);   // the next row's second input row (slot of row h - 1: read last row)
    BXF_STAMP(1);
    {  // s = (a + idn) + bias at position q0 + pw, channels 8g + 4hh + e
      const float* xh = xslot(h);
      const float x0 = xh[pw + 1], x1 = xh[pw + 2], x2 = xh[pw + 3];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = 8 * g + 4 * hh + e;
          const float av = hround(acc[4 * g + e]);
          const float4 pr = prec[co];
          const float iv = hround(fmaf(x0, pr.x, fmaf(x1, pr.y, x2 * pr.z)));
          o[e] = av + iv + pr.w;
        }
        *reinterpret_cast<float4*>(ss + pw * BX_SP + 8 * g + 4 * hh) = make_float4(o[0], o[1], o[2], o[3]);
      }
    }
    if (tid < BX_XW) xslot(h + 3)[tid] = x_val(h + 3, xnext);   // the slot of x row h - 1 (no reader after the last barrier)
    __syncthreads();
    BXF_STAMP(2);
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
    BXF_STAMP(3);
  }
#ifdef BX_PROF
  if (tid == 0)
#pragma unroll
    for (int k = 0; k < 4; ++k) atomicAdd(&bx_prof_f[k], (unsigned long long)pf_acc[k]);
#endif
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
  BxFwdArgs a{(const hst*)x, w1, wd, bn, (const hst*)w2, bias, (hst*)y, arg,
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
// A workgroup walks units (utterance, strip of 126 positions) in a grid-stride loop and, per unit, the rows
// top-down; iteration hp has three phases between barriers:
//   (B) dx row hp - 2 from the three tap responses phase D left in LDS; dout1 row hp on the MFMA (ds rows hp - 1,
//       hp) into the dc ring (2 rows), and the d w2 MFMAs of ds row hp - 2 x out1 rows hp - 2, hp - 1 (6 taps x
//       8 K steps, 12 per wave);
//   (C) the BN + SELU backward of dout1 row hp in place and out1 row hp = selu(u) (c recomputed from x, one exp
//       for both), a thread owning 2 channels (their frozen-BN / conv1 parameters in registers) x 8 positions;
//   (D) on the MFMA: dx's three tap responses O[kw][k] = sum_co (dc rows hp, hp - 1 | ds row hp - 1) x (w1 | wd)
//       (M = kw, K = 3 images x 32 channels, N = positions), and d w1 / d wd / d bias as dc^T / ds^T x the x taps
//       (K = positions, N = taps; x kept as three bf16 copies shifted by kw); then ds row hp + 1 into the LDS
//       ring of 3 (its pooled gradient and argmax fetched a row ahead) and x row hp + 2 into the x rings.
// Every sum counts the strip's own positions [126 s, 126 s + 126) (the K = position MFMAs run over 128 positions
// and zero the last two); with Wo / 42 + 1 strips they partition every position that carries a gradient.
// Per-workgroup sums go to one fp32 partial row (the caller sums the rows: no atomics).
constexpr int BXB_DCR = 128;                         // dc image rows: positions q0 - 1 .. q0 + 126
constexpr int BXB_XW = 136;                          // staged x positions q0 - 4 .. q0 + 131
constexpr int BXB_NPART = 6 * 32 * 32 + 32 * 6 + 32 * 3 + 32 + 3 * 32;
constexpr int BXB_XS = 4 * 3 * 128 * 2;              // x rows as bf16, shifted by kw: [4 slots][3 kw][128]
constexpr int BXB_WDX = 37 * 16;                     // dx weights, the MFMA A operand: [6 K steps][2][3 kw] + zeros
constexpr int BXB_OB = 3 * 128 * 4;                  // dx tap responses [3 kw][128] fp32
constexpr int BXB_PR = 6 * 16 * 16;                  // conv1 / frozen-BN records of the 16 channel pairs
constexpr int BXB_LDS = 192 * 64 + 3 * BX_IMG + 2 * BX_IMG + 2 * BXB_DCR * 64 + 4 * BXB_XW * 4 + BXB_XS + BXB_WDX +
                        BXB_OB + BXB_PR;
constexpr int BXB_BLOCKS = 512;
constexpr int BXB_PD = 2;                            // phase B's dout1 MFMA operands read this many steps ahead
static_assert(2 * BXB_LDS <= 160 * 1024, "two workgroups per CU");


// MFMA operand running down a column of a bx_img image (K = positions), csrc/sconv.hip sc_read_tr<32>
__device__ __forceinline__ hx8 bx_read_tr(const char* img, int r0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int row = r0 + 16 * s + 4 * (g >> 1) + (i >> 2);
  const int col = 16 * (g & 1) + 4 * (i & 3);
  const int sub = 2 * (col & 7);
  const hx4v lo = ds_tr4((img + bx_img(row, col >> 3) + sub));
  const hx4v hi = ds_tr4((img + bx_img(row + 8, col >> 3) + sub));
  hx8 r;
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
__device__ __forceinline__ hx8 bx_read_tr_at(const char* img, int2 off, int s) {
  const hx4v lo = ds_tr4((img + off.x + 1024 * s));
  const hx4v hi = ds_tr4((img + off.y + 1024 * s));
  hx8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = lo[j];
    r[4 + j] = hi[j];
  }
  return r;
}
struct BxBwdArgs {
  const hst* x;    // [N, H, W]
  const hst* dp;   // [N, H, Wo, 32] pooled-output gradient
  const uint8_t* arg;         // [N, H, Wo, 32]
  const float* w1;            // [32][6]
  const float* wd;            // [32][3]
  const float* bn;            // [5][32]: conv1 bias, mean, invstd * gamma, beta, invstd
  const hst* w2f;  // [6][32 ci][32 co] conv2 weights flipped in both axes, transposed (input gradient)
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
  char* xs = reinterpret_cast<char*>(xr + 4 * BXB_XW);       // bf16 x ring (4) x kw: [kw][i] <-> q0 + i + kw - 1
  char* wdx = xs + BXB_XS;                                   // chunk (s * 2 + h) * 3 + kw; chunk 36 = zeros
  float* ob = reinterpret_cast<float*>(wdx + BXB_WDX);       // O[kw][k + 2], k = -2 .. 125
  // channel pair cp's record, part k at float4 k * 16 + cp: w1[2cp][0..3] | w1[2cp][4..5] w1[2cp+1][0..1] |
  // w1[2cp+1][2..5] | cb mean invstd*gamma beta (2cp) | invstd (2cp), cb mean invstd*gamma (2cp+1) | beta invstd
  float4* prr = reinterpret_cast<float4*>(ob + 3 * 128);
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int H = a.H, W = a.W, Wo = a.Wo, W3 = 3 * a.Wo;
  for (int i = tid; i < 192 * 4; i += BX_T) {
    const int row = i >> 2, ch = i & 3;
    *reinterpret_cast<uint4*>(wsf + bx_img(row, ch)) = *reinterpret_cast<const uint4*>(a.w2f + row * BX_C + ch * 8);
  }
  // dx weights as the MFMA A operand: chunk (s * 2 + h) * 3 + kw holds w_img[co][kw] for co = 16 (s & 1) + 8 h + j,
  // image s >> 1 (0: w1 taps kh = 0 on dc row hp; 1: w1 taps kh = 1 on dc row hp - 1; 2: wd on ds row hp - 1)
  if (tid < 36) {
    const int kw = tid % 3, h = (tid / 3) & 1, s = tid / 6, img = s >> 1;
    uint32_t pk[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int c0 = 16 * (s & 1) + 8 * h + 2 * jj;
      const float v0 = img < 2 ? a.w1[c0 * 6 + 3 * img + kw] : a.wd[c0 * 3 + kw];
      const float v1 = img < 2 ? a.w1[(c0 + 1) * 6 + 3 * img + kw] : a.wd[(c0 + 1) * 3 + kw];
      pk[jj] = bx_pack2(v0, v1);
    }
    *reinterpret_cast<uint4*>(wdx + tid * 16) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
  } else if (tid == 36) {
    *reinterpret_cast<uint4*>(wdx + 36 * 16) = make_uint4(0u, 0u, 0u, 0u);
  }
  // out1 image rows 130, 131 (positions q0 + 127, q0 + 128) meet only the zeroed ds elements of the d w2 MFMA:
  // zeros, never stale LDS; phase C writes rows 2 .. 129
  if (tid >= 64 && tid < 80) {
    const int t = tid - 64;
    *reinterpret_cast<uint4*>(o1r + (t >> 3) * BX_IMG + bx_img(130 + ((t >> 2) & 1), t & 3)) =
        make_uint4(0u, 0u, 0u, 0u);
  }
  // phase C: this thread's channels 2 cp, 2 cp + 1 (records read once per row), positions 8 pg .. 8 pg + 7
  const int cp = tid & 15, pg = tid >> 4;
  if (tid < 16) {
    const float* w0 = a.w1 + 12 * tid;   // channel 2 tid, then 2 tid + 1
    const int c0 = 2 * tid, c1 = c0 + 1;
    prr[tid] = make_float4(w0[0], w0[1], w0[2], w0[3]);
    prr[16 + tid] = make_float4(w0[4], w0[5], w0[6], w0[7]);
    prr[32 + tid] = make_float4(w0[8], w0[9], w0[10], w0[11]);
    prr[48 + tid] = make_float4(a.bn[c0], a.bn[BX_C + c0], a.bn[2 * BX_C + c0], a.bn[3 * BX_C + c0]);
    prr[64 + tid] = make_float4(a.bn[4 * BX_C + c0], a.bn[c1], a.bn[BX_C + c1], a.bn[2 * BX_C + c1]);
    prr[80 + tid] = make_float4(a.bn[3 * BX_C + c1], a.bn[4 * BX_C + c1], 0.f, 0.f);
  }
  bxf2 bsum[3];   // channels 2 cp, 2 cp + 1: d cb, d gamma, d beta
#pragma unroll
  for (int q = 0; q < 3; ++q) bsum[q] = (bxf2)0.f;
  // d w2: acc2[0] = tap wv over every K step; acc2[1] = tap 4 + (wv >> 1) over K steps 4 (wv & 1) .. + 3.
  // accw = D[co][n] over K steps 2 wv, 2 wv + 1: n < 6 d w1 (tap n, from dc), n = 8 + kw d wd and n = 11 d bias
  // (from ds): the two B operands have disjoint nonzero columns, so both products accumulate into one tile
  bxf32x16 acc2[2], accw;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc2[0][i] = acc2[1][i] = accw[i] = 0.f;
  const int pw = wv * 32 + r;    // dout1 position q0 - 1 + pw of this lane in phase B
  __syncthreads();
  constexpr int DSN = (BX_IR * 4 + BX_T - 1) / BX_T;   // ds items per thread (3)
  auto ds_slot = [&](int h) -> char* { return dsr + ((h + 3) % 3) * BX_IMG; };   // h >= -3
  const int2 off_ds = bx_tr_off(2, lane);                // ds image rows 2 + k <-> positions q0 + k
  const int2 off_dc = bx_tr_off(1, lane);                // dc image rows 1 + k <-> positions q0 + k
  const bool tail_lane = hh == 1;                        // K rows 126, 127 (next strip): elements 6, 7 at step 7

  for (int64_t u = blockIdx.x; u < (int64_t)a.strips * a.N; u += gridDim.x) {
    const int strip = (int)(u % a.strips), n = (int)(u / a.strips);
    const int q0 = strip * BX_P;
    const hst* xn = a.x + (int64_t)n * H * W;
    // x row `row` at position q0 - 4 + tid: raw bf16 bits from a clamped (always valid) address, so the load
    // carries no branch and its wait falls where the row is stored (put_x), a phase or more later
    auto x_raw = [&](int row) -> uint32_t {
      const int q = q0 - 4 + tid;
      const int rc = row < 0 ? 0 : (row >= H ? H - 1 : row);
      const int qc = q < 0 ? 0 : (q >= W ? W - 1 : q);
      return reinterpret_cast<const uint16_t*>(xn)[(int64_t)rc * W + qc];
    };
    auto xslot = [&](int row) -> float* { return xr + (row & 3) * BXB_XW; };
    auto xsslot = [&](int row) -> char* { return xs + (row & 3) * (3 * 256); };
    // x (zero outside the image) into the fp32 ring and the three kw-shifted bf16 copies
    auto put_x = [&](int row, uint32_t raw) {
      const int q = q0 - 4 + tid;
      const uint32_t b = (row >= 0 && row < H && q >= 0 && q < W) ? raw : 0u;
      if (tid < BXB_XW) {
        xslot(row)[tid] = hlo(b);
        char* xsr = xsslot(row);
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int i = tid - 3 - kw;
          if (i >= 0 && i < 128) *reinterpret_cast<uint16_t*>(xsr + kw * 256 + 2 * i) = (uint16_t)b;
        }
      }
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
          const int64_t off = (((int64_t)n * H + hrow) * Wo + jj) * BX_C + 8 * (tid & 3);
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
          *reinterpret_cast<uint4*>(sl + bx_img(i, tid & 3)) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
        }
      }
    };
    __syncthreads();   // the previous unit's readers are done
    {
      uint32_t v[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) v[i] = x_raw(i - 1);
#pragma unroll
      for (int i = 0; i < 3; ++i) put_x(i - 1, v[i]);
    }
    fetch_ds(-1);
    store_ds(-1);       // zeros
    fetch_ds(0);
    store_ds(0);
    fetch_ds(1);
    __syncthreads();
    BX_STAMP(4);
    // iteration hp: dout1 / dc row hp and out1 row hp (hp <= H), dx tap responses of row hp - 1 (stored at hp + 1),
    // d w1 / d wd of rows hp, d w2 of ds row hp - 2 (hp >= 2)
    for (int hp = 0; hp <= H + 1; ++hp) {
      const bool rowc = hp <= H;
      // x row hp + 2 in flight (stored at the end of phase D); dx row hp - 2 from the tap responses in LDS
      const uint32_t xnext = x_raw(hp + 2);
      if (hp >= 2 && tid < BX_P && q0 + tid < W)
        a.dx[((int64_t)n * H + hp - 2) * W + q0 + tid] = (ob[tid + 2] + ob[128 + tid + 1]) + ob[256 + tid];
      // ---- phase B: dout1 row hp = conv(ds rows hp - 1, hp) with the flipped weights -> bf16 into the dc slot;
      // d w2 += ds row hp - 2 x out1 rows hp - 2, hp - 1 over K = ds image rows 2 .. 129 (positions q0 ..
      // q0 + 127); rows 128, 129 (q0 + 126, q0 + 127) belong to the next strip: their A elements are zeroed
      // (in the last K step, element j of lane l holds row 2 + 112 + 8 (j >> 2) + 4 (l >> 5) + (j & 3): elements
      // 6, 7 of lanes 32-63)
      if (rowc) {
        bxf32x16 acc;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 0.f;
        // weight rows tap * 32 + r: 2048 bytes per tap; input rows pw + kw
        const int wo0 = bx_img(r, hh), wo1 = bx_img(r, 2 + hh);
        // steps (kh, kw, s) in the same order, each step's two operand reads issued BXB_PD steps ahead of its MFMA
        // (the scheduler would otherwise pull them back next to it and expose the LDS latency at every step)
        {
          constexpr int PD = BXB_PD;
          hx8 xq[12], wq[12];
#pragma unroll
          for (int q = 0; q < 12 + PD; ++q) {
            if (q < 12) {
              const int kh = q / 6, kw = (q / 2) % 3, s = q & 1;
              xq[q] = *reinterpret_cast<const hx8*>(ds_slot(hp - 1 + kh) + bx_img(pw + kw, 2 * s + hh));
              wq[q] = *reinterpret_cast<const hx8*>(wsf + (kh * 3 + kw) * 2048 + (s ? wo1 : wo0));
            }
            if (q >= PD) acc = mfma32x32x16(wq[q - PD], xq[q - PD], acc);
            __builtin_amdgcn_sched_barrier(0);
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
        const int kh0 = wv / 3, kw0 = wv - 3 * kh0;      // tap wv: (0, 0), (0, 1), (0, 2), (1, 0)
        const char* oi0 = o1r + ((hp + kh0) & 1) * BX_IMG;   // out1 row hp - 2 + kh
        const char* oi1 = o1r + ((hp + 1) & 1) * BX_IMG;     // taps 4, 5: kh = 1
        const int2 offb0 = bx_tr_off(2 + kw0, lane), offb1 = bx_tr_off(3 + (wv >> 1), lane);
        const int s1 = 4 * (wv & 1);
        // K steps s in order, their reads BXB_PD steps ahead (the taps-4/5 operand is read at every step and used
        // at the wave's four)
        constexpr int PD = BXB_PD;
        hx8 aq[8], bq0[8], bq1[8];
#pragma unroll
        for (int q = 0; q < 8 + PD; ++q) {
          if (q < 8) {
            aq[q] = bx_read_tr_at(dsi, off_ds, q);
            bq0[q] = bx_read_tr_at(oi0, offb0, q);
            bq1[q] = bx_read_tr_at(oi1, offb1, q);
          }
          if (q >= PD) {
            const int s = q - PD;
            hx8 av = aq[s];
            if (s == 7 && tail_lane) {
              av[6] = (hel)0.0f;
              av[7] = (hel)0.0f;
            }
            acc2[0] = mfma32x32x16(av, bq0[s], acc2[0]);
            if (s >= s1 && s < s1 + 4) acc2[1] = mfma32x32x16(av, bq1[s], acc2[1]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __syncthreads();
      BX_STAMP(1);
      if (rowc) {
        // ---- phase C: dc row hp = bf16(dO selu'(u) s) in place (rdx_sconv_dgrad_bnselu's arithmetic on c
        // recomputed from x), BN sums over the strip's own positions; out1 row hp = selu(u) (rdx_sincnet_b0_fwd's
        // value) into the out1 slot of row hp - 2 (read for the last time in phase B above)
        {
          char* dcs = dcr + (hp & 1) * (BXB_DCR * 64);
          char* o1s = o1r + (hp & 1) * BX_IMG;
          const int i0 = 8 * pg, cofs = 4 * (cp & 3), cch = cp >> 2;
          bxf2 pw1[6], pcb, pmu, psg, psh, pis;   // the pair's conv1 weights and frozen BN
          {
            const float4 r0 = prr[cp], r1 = prr[16 + cp], r2 = prr[32 + cp], r3 = prr[48 + cp], r4 = prr[64 + cp],
                         r5 = prr[80 + cp];
            const float w[12] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w};
#pragma unroll
            for (int k = 0; k < 6; ++k) pw1[k] = (bxf2){w[k], w[6 + k]};
            pcb = (bxf2){r3.x, r4.y};
            pmu = (bxf2){r3.y, r4.z};
            psg = (bxf2){r3.z, r4.w};
            psh = (bxf2){r3.w, r5.x};
            pis = (bxf2){r4.x, r5.y};
          }
#pragma unroll 1
          for (int half = 0; half < 2; ++half) {
          const int i4 = i0 + 4 * half;
          float xwa[8], xwb[8];   // x ring indices i4 .. i4 + 7 of rows hp - 1 / hp
#pragma unroll
          for (int v = 0; v < 2; ++v) {
            const float4 fa = *reinterpret_cast<const float4*>(xslot(hp - 1) + i4 + 4 * v);
            const float4 fb = *reinterpret_cast<const float4*>(xslot(hp) + i4 + 4 * v);
            xwa[4 * v] = fa.x;
            xwa[4 * v + 1] = fa.y;
            xwa[4 * v + 2] = fa.z;
            xwa[4 * v + 3] = fa.w;
            xwb[4 * v] = fb.x;
            xwb[4 * v + 1] = fb.y;
            xwb[4 * v + 2] = fb.z;
            xwb[4 * v + 3] = fb.w;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int i = i4 + j;   // dc image row <-> position q0 - 1 + i
            const int q = q0 - 1 + i;
            const bool inside = q >= 0 && q < W;
            const bool own = inside && i >= 1 && i <= BX_P;
            uint32_t* slot = reinterpret_cast<uint32_t*>(dcs + bx_img(i, cch) + cofs);
            const uint32_t dov = *slot;
            // c (bf16-rounded, the unfused kernel's FMA order), u, and from one exp both selu'(u) and selu(u)
            const float v0[3] = {xwa[j + 2], xwa[j + 3], xwa[j + 4]}, v1[3] = {xwb[j + 2], xwb[j + 3], xwb[j + 4]};
            const bxf2 cv = bx_conv1_pair(v0, v1, pw1);
            const bxf2 zc = (cv + pcb) - pmu;
            const bxf2 xhat = zc * pis;
            const bxf2 uu = __builtin_elementwise_fma(zc, psg, psh);
            const bxf2 ex = {__expf(uu.x), __expf(uu.y)};
            const bxf2 sdn = (BX_SELU_SCALE * BX_SELU_ALPHA) * ex;
            const bxf2 sd = {uu.x > 0.f ? BX_SELU_SCALE : sdn.x, uu.y > 0.f ? BX_SELU_SCALE : sdn.y};
            const bxf2 ng = BX_SELU_ALPHA * (ex - 1.0f);
            const bxf2 yo = BX_SELU_SCALE * (bxf2){uu.x > 0.f ? uu.x : ng.x, uu.y > 0.f ? uu.y : ng.y};   // bx_selu
            const bxf2 du = (bxf2){bx_lo(dov), bx_hi(dov)} * sd;
            const bxf2 dz = inside ? du * psg : (bxf2)0.f;
            const bxf2 b0 = bsum[0] + dz, b1 = __builtin_elementwise_fma(du, xhat, bsum[1]), b2 = bsum[2] + du;
            bsum[0] = own ? b0 : bsum[0];
            bsum[1] = own ? b1 : bsum[1];
            bsum[2] = own ? b2 : bsum[2];
            *slot = bx_pack2(dz.x, dz.y);
            *reinterpret_cast<uint32_t*>(o1s + bx_img(i + 2, cch) + cofs) = inside ? bx_pack2(yo.x, yo.y) : 0u;
          }
          }
        }
        __syncthreads();
        BX_STAMP(2);
        // ---- phase D (MFMA): dx tap responses of row hp - 1; d w1 (dc row hp x x rows hp - 1, hp), d wd and
        // d bias (ds row hp x x row hp, ones)
        {
          const char* dcA = dcr + (hp & 1) * (BXB_DCR * 64);         // dc row hp
          const char* dcB = dcr + ((hp - 1) & 1) * (BXB_DCR * 64);   // dc row hp - 1
          const char* dsP = ds_slot(hp - 1);                         // ds row hp - 1
          const char* dsC = ds_slot(hp);                             // ds row hp
          if (hp >= 1) {
            // O[kw][k'] = sum_co dcA[k' + 2] w1[., kw] + dcB[k' + 2] w1[., 3 + kw] + dsP[k' + 3] wd[., kw],
            // k' = 32 wv - 2 + r; dx[k] = O[0][k] + O[1][k - 1] + O[2][k - 2] (phase B of the next iteration)
            bxf32x16 o;
#pragma unroll
            for (int i = 0; i < 16; ++i) o[i] = 0.f;
            const int kp = 32 * wv - 2 + r;
            constexpr int PD = BXB_PD;   // reads PD steps ahead, as in phase B
            hx8 bq[6], wq[6];
#pragma unroll
            for (int q = 0; q < 6 + PD; ++q) {
              if (q < 6) {
                const int img = q >> 1;
                const char* src = img == 0 ? dcA : (img == 1 ? dcB : dsP);
                bq[q] = *reinterpret_cast<const hx8*>(src + bx_img(kp + (img == 2 ? 3 : 2), 2 * (q & 1) + hh));
                wq[q] = *reinterpret_cast<const hx8*>(wdx + (r < 3 ? (q * 6 + hh * 3 + r) * 16 : 576));
              }
              if (q >= PD) o = mfma32x32x16(wq[q - PD], bq[q - PD], o);
              __builtin_amdgcn_sched_barrier(0);
            }
            if (hh == 0) {   // D[m][n]: element i of lane n < 32 holds m = i for i < 3
              ob[kp + 2] = o[0];
              ob[128 + kp + 2] = o[1];
              ob[256 + kp + 2] = o[2];
            }
          }
          // B operand: element j of lane (n, h) = X[16 s + 8 (j >> 2) + 4 h + (j & 3)][n] (the transposed A's K order)
          const int nn1 = r < 6 ? r : 5, nn2 = r >= 8 && r < 11 ? r - 8 : 0;
          const char* xb1 = xsslot(hp - 1 + nn1 / 3) + (nn1 % 3) * 256;
          const char* xb2 = xsslot(hp) + nn2 * 256;
#pragma unroll
          for (int ss = 0; ss < 2; ++ss) {
            const int s = 2 * wv + ss;
            hx8 ac = bx_read_tr_at(dcA, off_dc, s), as = bx_read_tr_at(dsC, off_ds, s);
            if (s == 7 && tail_lane) {
              ac[6] = ac[7] = as[6] = as[7] = (hel)0.0f;
            }
            const int kb = 2 * (16 * s + 4 * hh);
            const uint2 p1a = *reinterpret_cast<const uint2*>(xb1 + kb), p1b = *reinterpret_cast<const uint2*>(xb1 + kb + 16);
            const uint2 p2a = *reinterpret_cast<const uint2*>(xb2 + kb), p2b = *reinterpret_cast<const uint2*>(xb2 + kb + 16);
            const uint32_t one2 = hpack2(1.f, 1.f);   // 1.0 pair: the bias column
            const uint4 w1v = r < 6 ? make_uint4(p1a.x, p1a.y, p1b.x, p1b.y) : make_uint4(0u, 0u, 0u, 0u);
            const uint4 w2v = (r >= 8 && r < 11) ? make_uint4(p2a.x, p2a.y, p2b.x, p2b.y)
                                                 : (r == 11 ? make_uint4(one2, one2, one2, one2) : make_uint4(0u, 0u, 0u, 0u));
            accw = mfma32x32x16(ac, __builtin_bit_cast(hx8, w1v), accw);
            accw = mfma32x32x16(as, __builtin_bit_cast(hx8, w2v), accw);
          }
        }
        // the next row's ds into the slot of row hp - 2 (read for the last time in phase B), its successor's fetch
        store_ds(hp + 1);
        fetch_ds(hp + 2);
        put_x(hp + 2, xnext);   // x row hp + 2 into the slots of row hp - 2 (no reader in this row)
        __syncthreads();
      }
      BX_STAMP(3);
    }
  }
#ifdef BX_PROF
  if (tid == 0)
#pragma unroll
    for (int k = 0; k < 5; ++k) bx_prof[blockIdx.x][k] = (unsigned long long)prof_acc[k];
#endif

  // ---- per-workgroup partial row (fixed-order sums: bitwise repeatable) ----
  // D element i of lane (n, h) is [m = (i & 3) + 8 (i >> 2) + 4 h][n]
  float* out = a.part + (int64_t)blockIdx.x * BXB_NPART;
#pragma unroll
  for (int i = 0; i < 16; ++i) {   // d w2 taps 0..3: [tap][co][ci], ci = n
    const int co = (i & 3) + 8 * (i >> 2) + 4 * hh;
    out[(wv * BX_C + co) * BX_C + r] = acc2[0][i];
  }
  float* red = reinterpret_cast<float*>(lds);   // [2 tiles][4 waves][16][64] MFMA partials, then [256][6] BN sums
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    red[((0 * 4 + wv) * 16 + i) * 64 + lane] = acc2[1][i];
    red[((1 * 4 + wv) * 16 + i) * 64 + lane] = accw[i];
  }
  float* bred = red + 2 * 4 * 16 * 64;
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int e = 0; e < 2; ++e) bred[tid * 6 + q * 2 + e] = bsum[q][e];
  __syncthreads();
  auto tile_at = [&](int t, int w, int m, int nn) -> float {   // element [m][nn] of tile t of wave w
    const int h = (m >> 2) & 1, i = (m & 3) + 4 * (m >> 3);
    return red[((t * 4 + w) * 16 + i) * 64 + nn + 32 * h];
  };
  for (int idx = tid; idx < 2 * 32 * 32; idx += BX_T) {   // d w2 taps 4 (waves 0 + 1), 5 (waves 2 + 3)
    const int tap = idx >> 10, co = (idx >> 5) & 31, ci = idx & 31;
    out[((4 + tap) * BX_C + co) * BX_C + ci] = tile_at(0, 2 * tap, co, ci) + tile_at(0, 2 * tap + 1, co, ci);
  }
  for (int idx = tid; idx < 32 * 10; idx += BX_T) {   // d w1 [32][6], d wd [32][3], d bias [32]: sum of 4 waves
    const int co = idx / 10, j = idx % 10;
    const int nn = j < 6 ? j : j + 2;
    const float s = ((tile_at(1, 0, co, nn) + tile_at(1, 1, co, nn)) + tile_at(1, 2, co, nn)) + tile_at(1, 3, co, nn);
    const int dst = j < 6 ? 6144 + co * 6 + j : (j < 9 ? 6144 + 192 + co * 3 + (j - 6) : 6144 + 192 + 96 + co);
    out[dst] = s;
  }
  if (tid < 96) {   // BN sums [3][32]: channel co = 2 cp + e sums the 16 threads with tid & 15 == cp
    const int q = tid / 32, co = tid % 32, c2 = co >> 1, e = co & 1;
    float s = 0.f;
    for (int t = 0; t < 16; ++t) s += bred[(t * 16 + c2) * 6 + q * 2 + e];
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
  BxBwdArgs a{(const hst*)x, (const hst*)dp, arg, w1, wd, bn, (const hst*)w2f,
              dx, part, N, H, W, W / 3, W / 3 / BX_J + 1};
  hipLaunchKernelGGL(b0x_bwd_kernel, dim3((unsigned)rdx_b0x_bwd_nblk(N, W)), dim3(BX_T), BXB_LDS, as_stream(stream),
                     a);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
