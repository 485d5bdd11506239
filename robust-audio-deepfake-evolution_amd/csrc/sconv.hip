// SincNet residual-stack convolutions on gfx950 MFMA: NHWC bf16, kernel (KH x 3) with KH in {1, 2}, stride 1,
// padding (ph, 1), C_in and C_out in {32, 64} — conv1 (2x3, pad (1,1)), conv2 (2x3, pad (0,1)) and
// conv_downsample (1x3, pad (0,1)) of Residual_block (src/models/DualStreamSEMamba.py:144-200) in blocks 1-5 and
// conv2 of block 0, forward, input gradient and weight gradient. They replace MIOpen's implicit-GEMM solvers
// and the layout transposes / zero-fills around them.
//
// Forward (also the input gradient: dX is the same convolution of dY with the kernel flipped in both axes,
// C_in/C_out exchanged and the row padding KH-1-ph):
//   Y[n, ho, w, co] = sum_{kh, kw, ci} X[n, ho + kh - ph, w + kw - 1, ci] * Wt[co, ci, kh, kw]
// A 256-thread workgroup owns a strip of 128 positions of one utterance and walks its output rows top-down:
// the weights [tap][co][ci] are staged in LDS once, each input row (130 positions with the two halo columns,
// zero outside the image) is read from HBM once into a ring of KH + 1 LDS row slots (16-byte chunks
// XOR-swizzled by position / output channel), prefetched a row ahead; each wave owns 32 positions and runs
// KH*3*C_in/16 mfma_f32_32x32x16_bf16 steps per 32 output channels, computing Y^T (weights as the row
// operand), so a lane holds one position and groups of 4 consecutive channels: 8-byte stores.
// Epilogue options: bf16 output (no bias: the conv biases are folded into the next fused pass, as
// radhip.ops.BnSelu / ResTail expect), or additionally the frozen-BN + SELU activation of that output (the
// conv1 -> bn2 -> selu chain), so conv2's input is produced without another pass over HBM.
//
// Weight gradient: dW[co, ci, kh, kw] = sum_{n, ho, w} dY[n, ho, w, co] * X[n, ho + kh - ph, w + kw - 1, ci].
// A workgroup walks units of (output row, 128-position strip) in a grid-stride loop, stages the dY strip and
// the KH input rows (130 positions) row-major in LDS, and accumulates (tap, co-tile, ci-tile) 32x32 MFMA tiles
// with K = positions in registers (4 waves split the tiles); both operands are read down their columns with
// ds_read_b64_tr_b16 (the tap's column shift is a row offset into the input image). One fp32 partial per
// workgroup, summed by a second kernel in a fixed order (deterministic, no atomics).
#include "common.h"

namespace rdx {

typedef __attribute__((ext_vector_type(16))) float sf32x16;
typedef __attribute__((ext_vector_type(2))) unsigned int v2u32;

constexpr int SC_T = 256;        // threads
constexpr int SC_P = 128;        // output positions per strip
constexpr int SC_PW = SC_P + 2;  // staged input positions (halo 1 each side)

__device__ __forceinline__ sf32x16 sc_mfma(hx8 a, hx8 b, sf32x16 c) {
  return mfma32x32x16(a, b, c);
}
__device__ __forceinline__ uint32_t sc_pack2(float a, float b) {
  hst x = f2h(a), y = f2h(b);
  return (uint32_t)(*reinterpret_cast<uint16_t*>(&x)) | ((uint32_t)(*reinterpret_cast<uint16_t*>(&y)) << 16);
}
__device__ __forceinline__ float sc_selu(float u) {  // as sincnet.hip selu_fast (bf16-rounded output)
  return 1.0507009873554805f * (u > 0.f ? u : 1.6732632423543772f * (__expf(u) - 1.0f));
}

// LDS byte offset of the 16-byte chunk `ch` (8 channels) of row `row` in a [rows][C] bf16 image; chunks are
// XOR-swizzled by the row so 32 lanes reading the same chunk of 32 consecutive rows spread over the banks.
template <int C>
__device__ __forceinline__ int sc_off(int row, int ch) {
  constexpr int NCH = C / 8;
  return row * (C * 2) + 16 * (ch ^ (row & (NCH - 1)));
}

struct SConvArgs {
  const hst* x;  // [N, H, W, CI]
  const hst* w;  // [KH*3][CO][CI] (tap-major, prepared on the host)
  hst* y;        // [N, Ho, W, CO]
  hst* y2;       // optional: selu(bn(y + cb)) [N, Ho, W, CO]
  const float* bn;          // [4][CO]: conv bias cb, running mean, invstd * gamma, beta (frozen BN); the
                            //   backward epilogue reads a fifth row, invstd
  const hst* c;  // backward epilogue: the saved pre-activation [N, Ho, W, CO]
  float* sums;              // backward epilogue: [3][CO] d conv_bias | d gamma | d beta (fp32 atomics)
  const hst* res;  // optional [N, Ho, W, CO]: y = bf16(bf16(conv) + res) (a residual branch's gradient)
  int N, H, W, Ho, ph;
  int rows_per;             // output rows per workgroup (grid.z chunks of the Ho rows)
};

// Input rows cycle through KH + 1 LDS slots: input row (ho - ph + kh) of output row ho lives in slot
// (ho + kh) % (KH + 1), and the row the next output row adds is loaded into registers while the current
// row's MFMAs run, then written to the slot the current row no longer needs (one barrier per row).
constexpr uint32_t SC_OOB = 0x80000000u;   // a buffer offset past every range (the host keeps ranges below it)

// raw buffer resource over `bytes` bytes at p (range-checked: an offset past it loads 0, a store there is dropped)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sc_rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

// input row hi of the utterance behind rs (positions p0 - 1 .. p0 + 128, zero outside the image) into registers:
// one unconditional buffer load per 16-byte item (an item outside the image gets an offset past the range and
// loads 0). Branch-free, so the compiler tracks the loads exactly and does not wait on them, or on the stores
// around them, before they are used.
template <int CI>
__device__ __forceinline__ void sc_load_row(uint4* regs, __amdgpu_buffer_rsrc_t rs, int hi, int H, int W, int p0) {
  constexpr int XCH = CI / 8, NV = (SC_PW * XCH + SC_T - 1) / SC_T;
  const bool rok = hi >= 0 && hi < H;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int i = threadIdx.x + SC_T * j;
    const int ch = i % XCH, pp = i / XCH, wi = p0 - 1 + pp;
    const bool ok = rok && pp < SC_PW && wi >= 0 && wi < W;
    const uint32_t off = ok ? (uint32_t)(((hi * W + wi) * CI + ch * 8) * 2) : SC_OOB;
    regs[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
  }
}
template <int CI>
__device__ __forceinline__ void sc_store_row(char* slot, const uint4* regs) {
  constexpr int XCH = CI / 8, NV = (SC_PW * XCH + SC_T - 1) / SC_T;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int i = threadIdx.x + SC_T * j;
    if (i < SC_PW * XCH) *reinterpret_cast<uint4*>(slot + sc_off<CI>(i / XCH, i % XCH)) = regs[j];
  }
}

// kBnBwd: the convolution is conv2's input gradient dO1 (the same kernel on dY with the flipped weights) and
// the epilogue continues it through the frozen BN + SELU backward of bnselu_bwd_kernel (csrc/sincnet.hip) on the
// bf16-rounded dO1, as the unfused path would: y = dc, and the per-channel sums of dc, dc/s * xhat, dc/s go
// to a.sums, so dO1 never goes through HBM.
template <int CI, int CO, int KH, bool kBnBwd = false>
__global__ __launch_bounds__(SC_T) void sconv_fwd_kernel(SConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char sc_lds[];
  constexpr int NSLOT = KH + 1, SLOT = SC_PW * CI * 2, XCH = CI / 8;
  constexpr int NV = (SC_PW * XCH + SC_T - 1) / SC_T;
  char* ws = sc_lds;                          // [KH*3*CO][CI]
  char* xs = sc_lds + KH * 3 * CO * CI * 2;   // NSLOT x [SC_PW][CI]
  // the epilogue's per-channel BN parameters (up to 5 x CO fp32) in LDS: read per output element, they were
  // global loads ordered behind the previous group's stores (y may alias bn / c for the compiler)
  float* sbn = reinterpret_cast<float*>(xs + NSLOT * SLOT);
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int n = blockIdx.y, p0 = blockIdx.x * SC_P;
  const int ho0 = blockIdx.z * a.rows_per, ho1 = min(a.Ho, ho0 + a.rows_per);
  // buffer resources over this utterance's input and output images (the host keeps each below 2 GiB)
  const int64_t ibytes = (int64_t)a.H * a.W * CI * 2, obytes = (int64_t)a.Ho * a.W * CO * 2;
  const int64_t obase_n = (int64_t)n * a.Ho * a.W * CO;
  const __amdgpu_buffer_rsrc_t rx = sc_rsrc(a.x + (int64_t)n * a.H * a.W * CI, ibytes);
  const __amdgpu_buffer_rsrc_t ry = sc_rsrc(a.y + obase_n, obytes);
  const __amdgpu_buffer_rsrc_t ry2 = sc_rsrc(a.y2 ? a.y2 + obase_n : a.y + obase_n, obytes);
  const __amdgpu_buffer_rsrc_t rc = sc_rsrc(kBnBwd ? a.c + obase_n : a.y + obase_n, obytes);
  const __amdgpu_buffer_rsrc_t rres = sc_rsrc(a.res ? a.res + obase_n : a.y + obase_n, obytes);
  {  // weights: every load issued before the first LDS store (one round trip, not one per chunk)
    constexpr int NWV = (KH * 3 * CO * XCH + SC_T - 1) / SC_T;
    const __amdgpu_buffer_rsrc_t rw = sc_rsrc(a.w, (int64_t)KH * 3 * CO * CI * 2);
    uint4 wr[NWV];
#pragma unroll
    for (int j = 0; j < NWV; ++j) {   // unconditional (past the end: an offset out of range), so wr stays in VGPRs
      const int i = tid + SC_T * j;
      const uint32_t off = i < KH * 3 * CO * XCH ? (uint32_t)(((i / XCH) * CI + (i % XCH) * 8) * 2) : SC_OOB;
      wr[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rw, off, 0, 0));
    }
#pragma unroll
    for (int j = 0; j < NWV; ++j) {
      const int i = tid + SC_T * j;  // row i / XCH = tap * CO + co
      if (i < KH * 3 * CO * XCH) *reinterpret_cast<uint4*>(ws + sc_off<CI>(i / XCH, i % XCH)) = wr[j];
    }
  }
  if (a.bn && (kBnBwd || a.y2))
    for (int i = tid; i < (kBnBwd ? 5 : 4) * CO; i += SC_T) sbn[i] = a.bn[i];
  uint4 pre[NV];
#pragma unroll
  for (int kh = 0; kh < KH; ++kh) {
    sc_load_row<CI>(pre, rx, ho0 + kh - a.ph, a.H, a.W, p0);
    sc_store_row<CI>(xs + ((ho0 + kh) % NSLOT) * SLOT, pre);
  }
  __syncthreads();
  constexpr int NT = CO / 32;
  const int pw = wv * 32 + r;  // this lane's position within the strip (B operand row)
  const int p = p0 + pw;
  const bool pv = p < a.W;
  // kBnBwd: per-lane sums [sum][t][g][e] over the rows this workgroup walks (channel t*32 + 8g + 4h + e)
  float bsum[kBnBwd ? 3 : 1][NT][4][4];
  if constexpr (kBnBwd) {
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int e = 0; e < 4; ++e) bsum[q][t][g][e] = 0.f;
  }
  // MFMA steps of a row: (kh, kw, 16-channel step s); their LDS operands are read PD steps ahead
  constexpr int SPK = CI / 16, NSTEP = KH * 3 * SPK, PD = 4;
  for (int ho = ho0; ho < ho1; ++ho) {
    const bool more = ho + 1 < ho1;
    // the next input row (rows past the last one this workgroup needs load zeros: ho1 <= Ho keeps them in range
    // or out of the image)
    sc_load_row<CI>(pre, rx, more ? ho - a.ph + KH : -1, a.H, a.W, p0);
    // this lane's output byte offset in the utterance (an offset past the range for a position past W: its loads
    // read 0 and its stores are dropped)
    const uint32_t orow = pv ? (uint32_t)(((ho * a.W + p) * CO + 4 * h) * 2) : SC_OOB;
    // kBnBwd: this row's saved pre-activations, loaded with the next input row (before the MFMAs), not one
    // round trip per channel group in the epilogue; !kBnBwd with a residual: this row's residual
    uint2 cres[NT][4];
    if (kBnBwd || a.res) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          cres[t][g] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(
                                                     kBnBwd ? rc : rres, orow + (t * 32 + 8 * g) * 2, 0, 0));
    }
    sf32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
    const char* xk0 = xs + (ho % NSLOT) * SLOT;
    const char* xk1 = xs + ((ho + 1) % NSLOT) * SLOT;
    hx8 xq[NSTEP], wq[NSTEP][NT];
#pragma unroll
    for (int q = 0; q < NSTEP + PD; ++q) {
      if (q < NSTEP) {   // issue step q's operand reads
        const int kh = q / (3 * SPK), kw = (q / SPK) % 3, s = q % SPK;
        xq[q] = *reinterpret_cast<const hx8*>((kh ? xk1 : xk0) + sc_off<CI>(pw + kw, 2 * s + h));
#pragma unroll
        for (int t = 0; t < NT; ++t)
          wq[q][t] = *reinterpret_cast<const hx8*>(ws + sc_off<CI>((kh * 3 + kw) * CO + t * 32 + r, 2 * s + h));
      }
      if (q >= PD) {     // step q - PD on the MFMA (Y^T tile: rows co, columns positions)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = sc_mfma(wq[q - PD][t], xq[q - PD], acc[t]);
      }
      // keep the reads PD steps ahead: the scheduler would otherwise pull each read back to its MFMA and expose
      // the LDS latency at every step (one wave per SIMD at 64 x 64 channels: nothing else hides it)
      __builtin_amdgcn_sched_barrier(0);
    }
    // the next input row into the slot this row does not read (its last reader, row ho - 1, is behind the previous
    // barrier), before the epilogue's stores
    if (more) sc_store_row<CI>(xs + ((ho + KH) % NSLOT) * SLOT, pre);
    // epilogue: lane owns position p, channels co = t*32 + 8g + 4h + e
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int co = t * 32 + 8 * g + 4 * h;
        const uint32_t off = orow + (t * 32 + 8 * g) * 2;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[t][4 * g + e];
        if constexpr (kBnBwd) {
          const uint2 cc = cres[t][g];
          const float cv[4] = {hlo(cc.x), hhi(cc.x), hlo(cc.y), hhi(cc.y)};
          const float4 cb = *reinterpret_cast<const float4*>(sbn + co);
          const float4 mu = *reinterpret_cast<const float4*>(sbn + CO + co);
          const float4 sg = *reinterpret_cast<const float4*>(sbn + 2 * CO + co);
          const float4 bb = *reinterpret_cast<const float4*>(sbn + 3 * CO + co);
          const float4 is = *reinterpret_cast<const float4*>(sbn + 4 * CO + co);
          const float pcb[4] = {cb.x, cb.y, cb.z, cb.w}, pmu[4] = {mu.x, mu.y, mu.z, mu.w};
          const float psg[4] = {sg.x, sg.y, sg.z, sg.w}, pbb[4] = {bb.x, bb.y, bb.z, bb.w};
          const float pis[4] = {is.x, is.y, is.z, is.w};
          float dz[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {  // the arithmetic of bnselu_bwd_kernel
            const float zc = (cv[e] + pcb[e]) - pmu[e];
            const float xhat = zc * pis[e];
            const float u = fmaf(zc, psg[e], pbb[e]);
            const float sd = u > 0.f ? 1.0507009873554805f : 1.0507009873554805f * 1.6732632423543772f * __expf(u);
            const float du = hround(v[e]) * sd;
            dz[e] = du * psg[e];
            // a position past W has no gradient (its lane's sums skip it)
            bsum[0][t][g][e] += pv ? dz[e] : 0.f;
            bsum[1][t][g][e] = pv ? fmaf(du, xhat, bsum[1][t][g][e]) : bsum[1][t][g][e];
            bsum[2][t][g][e] += pv ? du : 0.f;
          }
          __builtin_amdgcn_raw_buffer_store_b64(
              __builtin_bit_cast(v2u32, make_uint2(sc_pack2(dz[0], dz[1]), sc_pack2(dz[2], dz[3]))), ry, off, 0, 0);
          continue;
        }
        if (a.res) {   // the sum autograd would form: the bf16 convolution output plus the residual gradient
          const uint2 rr = cres[t][g];
          v[0] = hround(v[0]) + hlo(rr.x);
          v[1] = hround(v[1]) + hhi(rr.x);
          v[2] = hround(v[2]) + hlo(rr.y);
          v[3] = hround(v[3]) + hhi(rr.y);
        }
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(v2u32, make_uint2(sc_pack2(v[0], v[1]), sc_pack2(v[2], v[3]))), ry, off, 0, 0);
        if (a.y2) {
          const float4 cb = *reinterpret_cast<const float4*>(sbn + co);
          const float4 mu = *reinterpret_cast<const float4*>(sbn + CO + co);
          const float4 sg = *reinterpret_cast<const float4*>(sbn + 2 * CO + co);
          const float4 bb = *reinterpret_cast<const float4*>(sbn + 3 * CO + co);
          const float pcb[4] = {cb.x, cb.y, cb.z, cb.w}, pmu[4] = {mu.x, mu.y, mu.z, mu.w};
          const float psg[4] = {sg.x, sg.y, sg.z, sg.w}, pbb[4] = {bb.x, bb.y, bb.z, bb.w};
          float u[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)  // the arithmetic of bnselu_fwd_kernel on the bf16 conv output
            u[e] = sc_selu(fmaf((hround(v[e]) + pcb[e]) - pmu[e], psg[e], pbb[e]));
          __builtin_amdgcn_raw_buffer_store_b64(
              __builtin_bit_cast(v2u32, make_uint2(sc_pack2(u[0], u[1]), sc_pack2(u[2], u[3]))), ry2, off, 0, 0);
        }
      }
    __syncthreads();
  }
  if constexpr (kBnBwd) {
    // the 32 lanes of a half-wave hold the same channels: reduce them, then the four waves through LDS (the
    // weight image is no longer needed), then one atomic per (sum, channel) per workgroup
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float x = bsum[q][t][g][e];
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) x += __shfl_xor(x, o, 64);
            bsum[q][t][g][e] = x;
          }
    float* red = reinterpret_cast<float*>(sc_lds);  // [4 waves][3][CO]
    if (r == 0) {
#pragma unroll
      for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int e = 0; e < 4; ++e) red[(wv * 3 + q) * CO + t * 32 + 8 * g + 4 * h + e] = bsum[q][t][g][e];
    }
    __syncthreads();
    for (int i = tid; i < 3 * CO; i += SC_T)
      atomicAdd(&a.sums[i], (red[i] + red[3 * CO + i]) + (red[6 * CO + i] + red[9 * CO + i]));
  }
}

// ---------------------------------------------------------------------------- weight gradient ------
struct SWgradArgs {
  const hst* x;   // [N, H, W, CI]
  const hst* dy;  // [N, Ho, W, CO]
  float* part;               // [gridDim.x][KH*3][CO][CI]
  int N, H, W, Ho, ph;
  int64_t units;             // N * strips * nz
  int strips, nz, rows_per;  // 128-position strips, row chunks, rows per chunk
};


// Row-major [pos][C] image in LDS as 8-row x 32-channel subtiles of 512 B, the 16-byte chunk XOR-swizzled by
// (row >> 2) & 3: conflict-free for the hardware-transposed ds_read_b64_tr_b16 reads below.
template <int C>
__device__ __forceinline__ int sc_img(int row, int ch) {
  return (C * 16) * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}
// MFMA operand running down a column (K = positions): element j = IMG[r0 + 16 s + 8 (j >> 2) + 4 h + (j & 3)]
// [c0 + (lane & 31)], two ds_read_b64_tr_b16. Both operands of the weight-gradient MFMA use this same
// permuted position order, so the reduction over positions is unaffected.
template <int C>
__device__ __forceinline__ hx8 sc_read_tr(const char* img, int r0, int c0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int row = r0 + 16 * s + 4 * (g >> 1) + (i >> 2);
  const int col = c0 + 16 * (g & 1) + 4 * (i & 3);
  const int sub = 2 * (col & 7);
  const hx4v lo = ds_tr4((img + sc_img<C>(row, col >> 3) + sub));
  const hx4v hi = ds_tr4((img + sc_img<C>(row + 8, col >> 3) + sub));
  hx8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = lo[j];
    r[4 + j] = hi[j];
  }
  return r;
}

constexpr int SC_XR = 136;  // staged input rows per kernel row: 130 used, padded to whole 8-row subtiles

// A unit is (utterance, strip, chunk of output rows); the unit walks its rows top-down. Input rows cycle
// through KH + 1 image slots (row (ho - ph + kh) in slot (ho + kh) % (KH + 1)) and dY rows through two, so
// each input row is read from HBM once per unit and one barrier per row separates the writes of row ho from
// the MFMA reads of row ho - 1 (they never touch the same slot).
template <int CI, int CO, int KH>
__global__ __launch_bounds__(SC_T) void sconv_wgrad_kernel(SWgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char sc_lds[];
  constexpr int NSLOT = KH + 1, XSLOT = SC_XR * CI * 2, DSLOT = SC_P * CO * 2;
  char* dyi = sc_lds;                       // 2 x [SC_P][CO]
  char* xi = sc_lds + 2 * DSLOT;            // NSLOT x [SC_XR][CI]
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  constexpr int NTAP = KH * 3, TCO = CO / 32, TCI = CI / 32;
  constexpr int NTILE = NTAP * TCO * TCI;
  constexpr int PER = (NTILE + 3) / 4;  // tiles per wave
  sf32x16 acc[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
  // one staged row per thread-slice: X rows (SC_XR x CI) and dY rows (SC_P x CO) as 16-byte vectors, loaded
  // into registers one row ahead and written to their LDS slot after the current row's MFMAs
  constexpr int XV = SC_XR * (CI / 8), XN = (XV + SC_T - 1) / SC_T;
  constexpr int DV = SC_P * (CO / 8), DN = (DV + SC_T - 1) / SC_T;
  auto load_x = [&](uint4 (&r)[XN], int n, int hi, int p0) {
#pragma unroll
    for (int j = 0; j < XN; ++j) {
      const int i = tid + SC_T * j;
      const int ch = i % (CI / 8), pp = i / (CI / 8), wi = p0 - 1 + pp;
      r[j] = make_uint4(0, 0, 0, 0);
      if (i < XV && pp < SC_PW && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W)
        r[j] = *reinterpret_cast<const uint4*>(a.x + (((int64_t)n * a.H + hi) * a.W + wi) * CI + ch * 8);
    }
  };
  auto store_x = [&](char* slot, const uint4 (&r)[XN]) {
#pragma unroll
    for (int j = 0; j < XN; ++j) {
      const int i = tid + SC_T * j;
      if (i < XV) *reinterpret_cast<uint4*>(slot + sc_img<CI>(i / (CI / 8), i % (CI / 8))) = r[j];
    }
  };
  auto load_dy = [&](uint4 (&r)[DN], int n, int ho, int p0) {
#pragma unroll
    for (int j = 0; j < DN; ++j) {
      const int i = tid + SC_T * j;
      const int ch = i % (CO / 8), pp = i / (CO / 8), wi = p0 + pp;
      r[j] = make_uint4(0, 0, 0, 0);
      if (i < DV && ho < a.Ho && wi < a.W)
        r[j] = *reinterpret_cast<const uint4*>(a.dy + (((int64_t)n * a.Ho + ho) * a.W + wi) * CO + ch * 8);
    }
  };
  auto store_dy = [&](char* slot, const uint4 (&r)[DN]) {
#pragma unroll
    for (int j = 0; j < DN; ++j) {
      const int i = tid + SC_T * j;
      if (i < DV) *reinterpret_cast<uint4*>(slot + sc_img<CO>(i / (CO / 8), i % (CO / 8))) = r[j];
    }
  };
  uint4 rx[XN], rd[DN];
  for (int64_t u = blockIdx.x; u < a.units; u += gridDim.x) {
    const int zc = (int)(u % a.nz);
    const int64_t us = u / a.nz;
    const int strip = (int)(us % a.strips), n = (int)(us / a.strips);
    const int p0 = strip * SC_P;
    const int ho0 = zc * a.rows_per, ho1 = min(a.Ho, ho0 + a.rows_per);
    __syncthreads();  // the previous unit's reads are done
    for (int kh = 0; kh < KH; ++kh) {  // input rows of output row ho0, and its dY row
      load_x(rx, n, ho0 + kh - a.ph, p0);
      store_x(xi + ((ho0 + kh) % NSLOT) * XSLOT, rx);
    }
    load_dy(rd, n, ho0, p0);
    store_dy(dyi + (ho0 & 1) * DSLOT, rd);
    if (ho0 + 1 < ho1) {  // prefetch the rows output row ho0 + 1 adds
      load_x(rx, n, ho0 + 1 - a.ph + KH - 1, p0);
      load_dy(rd, n, ho0 + 1, p0);
    }
    for (int ho = ho0; ho < ho1; ++ho) {
      __syncthreads();
      const char* dys = dyi + (ho & 1) * DSLOT;
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int tile = wv + 4 * j;
        if (tile >= NTILE) break;
        const int tap = tile / (TCO * TCI), tco = (tile / TCI) % TCO, tci = tile % TCI;
        const int kh = tap / 3, kw = tap % 3;
        const char* xk = xi + ((ho + kh) % NSLOT) * XSLOT;
#pragma unroll
        for (int s = 0; s < SC_P / 16; ++s) {
          // output position pl pairs with staged input row pl + kw (input column p0 + pl + kw - 1)
          acc[j] = sc_mfma(sc_read_tr<CO>(dys, 0, tco * 32, s, lane), sc_read_tr<CI>(xk, kw, tci * 32, s, lane),
                           acc[j]);
        }
      }
      if (ho + 1 < ho1) {
        // the slots of rows ho - 1 (X) and ho - 1 (dY) are free: every wave passed this row's barrier
        store_x(xi + ((ho + KH) % NSLOT) * XSLOT, rx);
        store_dy(dyi + ((ho + 1) & 1) * DSLOT, rd);
        if (ho + 2 < ho1) {
          load_x(rx, n, ho + 2 - a.ph + KH - 1, p0);
          load_dy(rd, n, ho + 2, p0);
        }
      }
    }
  }
  // partial: lane owns ci column (lane & 31) of its tile, co rows (i & 3) + 8 (i >> 2) + 4 h
  const int r = lane & 31, h = lane >> 5;
  float* out = a.part + (int64_t)blockIdx.x * NTAP * CO * CI;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int tile = wv + 4 * j;
    if (tile >= NTILE) break;
    const int tap = tile / (TCO * TCI), tco = (tile / TCI) % TCO, tci = tile % TCI;
    const int ci = tci * 32 + r;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int co = tco * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
      out[((int64_t)tap * CO + co) * CI + ci] = acc[j][i];
    }
  }
}

// Fixed-order reduction of the per-workgroup partials [nblk][n]: stage 1 sums slice z of SC_RS slices of the
// partial rows (8 independent loads in flight per thread) into part2 [SC_RS][n]; stage 2 sums the slices.
constexpr int SC_RS = 16;
__global__ void sconv_wgrad_reduce1_kernel(const float* __restrict__ part, int nblk, int64_t n, float* __restrict__ part2) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int per = (nblk + SC_RS - 1) / SC_RS, b0 = blockIdx.y * per, b1 = min(nblk, b0 + per);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int b = b0;
  for (; b + 8 <= b1; b += 8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] += part[(int64_t)(b + k) * n + i];
  }
  for (; b < b1; ++b) s[0] += part[(int64_t)b * n + i];
  part2[(int64_t)blockIdx.y * n + i] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}
__global__ void sconv_wgrad_reduce2_kernel(const float* __restrict__ part2, int64_t n, float* __restrict__ dw) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
#pragma unroll
  for (int z = 0; z < SC_RS; ++z) s += part2[(int64_t)z * n + i];
  dw[i] = s;
}

template <int CI, int CO, int KH, bool kBnBwd = false>
static int sconv_fwd_launch(const SConvArgs& a, hipStream_t st) {
  // the kernel's per-utterance buffer ranges and 32-bit offsets (the sentinel SC_OOB must lie past every range)
  if ((int64_t)a.H * a.W * CI * 2 >= (int64_t)SC_OOB - 4096 || (int64_t)a.Ho * a.W * CO * 2 >= (int64_t)SC_OOB - 4096)
    return RDX_EUNSUPPORTED;
  const size_t smem = (size_t)(KH + 1) * SC_PW * CI * 2 + (size_t)KH * 3 * CO * CI * 2 + 5 * CO * sizeof(float);
  const int strips = (a.W + SC_P - 1) / SC_P;
  // one round of resident workgroups (256 CUs x the workgroups the LDS image allows per CU: 4 at 32 x 32
  // channels, 1 at 64 x 64): split the rows when strips x N alone is fewer (each split restages the weights
  // and KH - 1 halo rows), never more (a second round would restage for nothing)
  const int per_cu = (int)((160 * 1024) / smem) < 1 ? 1 : ((int)((160 * 1024) / smem) > 4 ? 4 : (int)((160 * 1024) / smem));
  const int64_t slots = 256 * (int64_t)per_cu, pairs = (int64_t)strips * a.N;
  // the row split that minimises rounds x (rows per workgroup + the restaging, ~KH + 1 row-equivalents)
  int nz = 1;
  int64_t best = -1;
  for (int z = 1; z <= a.Ho && z <= 64; ++z) {
    const int rp = (a.Ho + z - 1) / z;
    if (z > 1 && (a.Ho + rp - 1) / rp < z) continue;  // the same split as a smaller z
    const int64_t cost = ((pairs * z + slots - 1) / slots) * (rp + KH + 1);
    if (best < 0 || cost < best) {
      best = cost;
      nz = z;
    }
  }
  SConvArgs b = a;
  b.rows_per = (a.Ho + nz - 1) / nz;
  dim3 grid((unsigned)strips, (unsigned)a.N, (unsigned)((a.Ho + b.rows_per - 1) / b.rows_per));
  hipLaunchKernelGGL((sconv_fwd_kernel<CI, CO, KH, kBnBwd>), grid, dim3(SC_T), smem, st, b);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

template <int CI, int CO, int KH>
static int sconv_wgrad_launch(const SWgradArgs& a, int nblk, hipStream_t st) {
  const size_t smem = (2 * (size_t)SC_P * CO + (size_t)(KH + 1) * SC_XR * CI) * 2;
  hipLaunchKernelGGL((sconv_wgrad_kernel<CI, CO, KH>), dim3((unsigned)nblk), dim3(SC_T), smem, st, a);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

}  // namespace rdx

using namespace rdx;

#define SC_DISPATCH(FN, ...)                                                                   \
  if (ci == 32 && co == 32 && kh == 2) return FN<32, 32, 2>(__VA_ARGS__);                      \
  if (ci == 32 && co == 64 && kh == 2) return FN<32, 64, 2>(__VA_ARGS__);                      \
  if (ci == 64 && co == 32 && kh == 2) return FN<64, 32, 2>(__VA_ARGS__);                      \
  if (ci == 64 && co == 64 && kh == 2) return FN<64, 64, 2>(__VA_ARGS__);                      \
  if (ci == 32 && co == 64 && kh == 1) return FN<32, 64, 1>(__VA_ARGS__);                      \
  if (ci == 64 && co == 32 && kh == 1) return FN<64, 32, 1>(__VA_ARGS__);                      \
  if (ci == 32 && co == 32 && kh == 1) return FN<32, 32, 1>(__VA_ARGS__);                      \
  if (ci == 64 && co == 64 && kh == 1) return FN<64, 64, 1>(__VA_ARGS__);                      \
  return RDX_EUNSUPPORTED;

// y[N, Ho, W, co] = conv(x[N, H, W, ci], w) with Ho = H + 2*ph - kh + 1; w is tap-major [kh*3][co][ci] bf16.
// With y2 (and bn = [cb | mean | invstd*gamma | beta], 4 x co fp32) also
//   y2 = bf16(selu(((bf16(y) + cb) - mean) * invstd*gamma + beta)), exactly radhip.ops.BnSelu's forward.
extern "C" int rdx_sconv_fwd(const void* x, const void* w, void* y, void* y2, const float* bn, int N, int H, int W,
                             int ci, int co, int kh, int ph, void* stream) {
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  RDX_REQUIRE(x && w && y && N > 0 && H > 0 && W > 0 && (kh == 1 || kh == 2) && ph >= 0 && ph <= kh);
  RDX_REQUIRE(al(x) && al(w) && al(y) && (!y2 || (al(y2) && bn)));
  SConvArgs a;
  a.x = (const hst*)x;
  a.w = (const hst*)w;
  a.y = (hst*)y;
  a.y2 = (hst*)y2;
  a.bn = bn;
  a.c = nullptr;
  a.sums = nullptr;
  a.res = nullptr;
  a.N = N;
  a.H = H;
  a.W = W;
  a.ph = ph;
  a.Ho = H + 2 * ph - kh + 1;
  RDX_REQUIRE(a.Ho > 0 && N <= 65535);
  hipStream_t st = as_stream(stream);
  SC_DISPATCH(sconv_fwd_launch, a, st)
}

// The same convolution with a residual added in the epilogue: y = bf16(bf16(conv(x, w)) + res), res [N, Ho, W, co]
// bf16 — a residual block's input gradient, conv1's input gradient plus the identity branch's, in one pass
// (autograd's separate add reads both and writes the sum: the same bits, one full-size round trip less).
extern "C" int rdx_sconv_fwd_res(const void* x, const void* w, void* y, const void* res, int N, int H, int W, int ci,
                                 int co, int kh, int ph, void* stream) {
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  RDX_REQUIRE(x && w && y && res && N > 0 && H > 0 && W > 0 && (kh == 1 || kh == 2) && ph >= 0 && ph <= kh);
  RDX_REQUIRE(al(x) && al(w) && al(y) && al(res));
  SConvArgs a;
  a.x = (const hst*)x;
  a.w = (const hst*)w;
  a.y = (hst*)y;
  a.y2 = nullptr;
  a.bn = nullptr;
  a.c = nullptr;
  a.sums = nullptr;
  a.res = (const hst*)res;
  a.N = N;
  a.H = H;
  a.W = W;
  a.ph = ph;
  a.Ho = H + 2 * ph - kh + 1;
  RDX_REQUIRE(a.Ho > 0 && N <= 65535);
  hipStream_t st = as_stream(stream);
  SC_DISPATCH(sconv_fwd_launch, a, st)
}

// conv2's input gradient continued through conv1's frozen BN + SELU backward (Residual_block, the 32- and
// 64-channel blocks): dO1 = conv(dy[N, H, W, ci], w) (w: the flipped, transposed kernel, tap-major [kh*3][co][ci]; ph:
// kh - 1 - conv2's row padding), never stored; dc[N, Ho, W, co] = bf16(dO1) * selu'(u) * s with the saved
// pre-activation c, and sums[3][co] += (sum dc, sum dc/s * xhat, sum dc/s) — exactly rdx_bnselu_bwd on the
// unfused dO1. bn = [cb | mean | invstd*gamma | beta | invstd] (5 x co fp32); sums zeroed by the caller.
extern "C" int rdx_sconv_dgrad_bnselu(const void* dy, const void* w, const void* c, void* dc, const float* bn,
                                      float* sums, int N, int H, int W, int ci, int co, int kh, int ph, void* stream) {
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  RDX_REQUIRE(dy && w && c && dc && bn && sums && N > 0 && H > 0 && W > 0 && ph >= 0 && ph <= kh);
  RDX_REQUIRE(al(dy) && al(w) && al(c) && al(dc) && N <= 65535);
  if (!((ci == 32 && co == 32) || (ci == 64 && co == 64)) || kh != 2) return RDX_EUNSUPPORTED;
  SConvArgs a;
  a.x = (const hst*)dy;
  a.w = (const hst*)w;
  a.y = (hst*)dc;
  a.y2 = nullptr;
  a.bn = bn;
  a.c = (const hst*)c;
  a.sums = sums;
  a.res = nullptr;
  a.N = N;
  a.H = H;
  a.W = W;
  a.ph = ph;
  a.Ho = H + 2 * ph - kh + 1;
  RDX_REQUIRE(a.Ho > 0);
  if (ci == 64) return sconv_fwd_launch<64, 64, 2, true>(a, as_stream(stream));
  return sconv_fwd_launch<32, 32, 2, true>(a, as_stream(stream));
}

// Both 16-bit operand layouts of up to SC_WP_MAX convolution weights [co][ci][kh][3] (fp32) in one launch: wf
// [kh*3][co][ci] (forward, tap-major) and wd [kh*3][ci][co] of the kernel flipped in both axes (input gradient).
// The per-window preparation of the SincNet stack's weights (radhip/window.py) was four torch launches per weight
// (cast, permute-copy, flip, permute-copy).
constexpr int SC_WP_MAX = 32;
struct WPrepTable {
  const float* src[SC_WP_MAX];
  hst* wf[SC_WP_MAX];
  hst* wd[SC_WP_MAX];
  int co[SC_WP_MAX], ci[SC_WP_MAX], kh[SC_WP_MAX];
};
__global__ __launch_bounds__(256) void sconv_wprep_many_kernel(WPrepTable t) {
  const int k = blockIdx.y;
  const int co = t.co[k], ci = t.ci[k], kh = t.kh[k];
  const int n = co * ci * kh * 3;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int kw = i % 3, r = i / 3, h = r % kh, r2 = r / kh, c = r2 % ci, o = r2 / ci;   // src [o][c][h][kw]
    const hst v = f2h(t.src[k][i]);
    t.wf[k][((int64_t)(h * 3 + kw) * co + o) * ci + c] = v;
    t.wd[k][((int64_t)((kh - 1 - h) * 3 + (2 - kw)) * ci + c) * co + o] = v;
  }
}

extern "C" int rdx_sconv_wprep_many(int n, const float* const* src, void* const* wf, void* const* wd, const int* co,
                                    const int* ci, const int* kh, void* stream) {
  RDX_REQUIRE(n >= 0 && (n == 0 || (src && wf && wd && co && ci && kh)));
  if (n > SC_WP_MAX) return RDX_EUNSUPPORTED;
  if (n == 0) return RDX_OK;
  WPrepTable t{};
  int mx = 1;
  for (int k = 0; k < n; ++k) {
    RDX_REQUIRE(src[k] && wf[k] && wd[k] && co[k] > 0 && ci[k] > 0 && (kh[k] == 1 || kh[k] == 2));
    t.src[k] = src[k];
    t.wf[k] = reinterpret_cast<hst*>(wf[k]);
    t.wd[k] = reinterpret_cast<hst*>(wd[k]);
    t.co[k] = co[k];
    t.ci[k] = ci[k];
    t.kh[k] = kh[k];
    const int e = co[k] * ci[k] * kh[k] * 3;
    mx = e > mx ? e : mx;
  }
  const int bx = (mx + 255) / 256;
  hipLaunchKernelGGL(sconv_wprep_many_kernel, dim3((unsigned)(bx < 128 ? bx : 128), (unsigned)n), dim3(256), 0,
                     as_stream(stream), t);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

// row chunks of the weight-gradient units: about 4 rows each, at least 2048 units where the shape allows
static int sc_wgrad_nz(int N, int Ho, int W) {
  const int64_t su = (int64_t)N * ((W + SC_P - 1) / SC_P);
  int nz = (int)((2048 + su - 1) / su);
  if (nz < (Ho + 3) / 4) nz = (Ho + 3) / 4;
  return nz > Ho ? Ho : nz;
}

static int sc_wgrad_blocks(int N, int Ho, int W) {
  const int nz = sc_wgrad_nz(N, Ho, W);
  const int64_t units = (int64_t)N * ((W + SC_P - 1) / SC_P) * nz;
  return (int)(units < 1024 ? units : 1024);
}

// rows of kh*3*co*ci fp32 the weight-gradient scratch needs: one partial per workgroup + the reduction slices
extern "C" int rdx_sconv_wgrad_nblk(int N, int Ho, int W) { return sc_wgrad_blocks(N, Ho, W) + SC_RS; }

// dw [kh*3][co][ci] fp32 = sum over positions of dy (x) shifted x; part: [nblk][kh*3*co*ci] fp32 scratch,
// nblk = rdx_sconv_wgrad_nblk(N, Ho, W).
extern "C" int rdx_sconv_wgrad(const void* x, const void* dy, float* dw, float* part, int N, int H, int W, int ci,
                               int co, int kh, int ph, void* stream) {
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  RDX_REQUIRE(x && dy && dw && part && N > 0 && H > 0 && W > 0 && (kh == 1 || kh == 2) && ph >= 0 && ph <= kh);
  RDX_REQUIRE(al(x) && al(dy));
  SWgradArgs a;
  a.x = (const hst*)x;
  a.dy = (const hst*)dy;
  a.part = part;
  a.N = N;
  a.H = H;
  a.W = W;
  a.ph = ph;
  a.Ho = H + 2 * ph - kh + 1;
  RDX_REQUIRE(a.Ho > 0);
  a.strips = (W + SC_P - 1) / SC_P;
  a.nz = sc_wgrad_nz(N, a.Ho, W);
  a.rows_per = (a.Ho + a.nz - 1) / a.nz;
  a.nz = (a.Ho + a.rows_per - 1) / a.rows_per;
  a.units = (int64_t)N * a.strips * a.nz;
  // one resident round of workgroups (the LDS image sets how many fit on a CU), each walking several units:
  // fewer workgroups write fewer fp32 partials (kh*3*co*ci each: 96 KB at 64 x 64 channels) for the reduction
  const int64_t smem = (2 * (int64_t)SC_P * co + (int64_t)(kh + 1) * SC_XR * ci) * 2;
  const int per_cu = (int)((160 * 1024) / smem) < 1 ? 1 : ((int)((160 * 1024) / smem) > 4 ? 4 : (int)((160 * 1024) / smem));
  const int cap = sc_wgrad_blocks(N, a.Ho, W);
  const int nblk = cap < 256 * per_cu ? cap : 256 * per_cu;
  hipStream_t st = as_stream(stream);
  int rc = RDX_EUNSUPPORTED;
  if (ci == 32 && co == 32 && kh == 2) rc = sconv_wgrad_launch<32, 32, 2>(a, nblk, st);
  else if (ci == 32 && co == 64 && kh == 2) rc = sconv_wgrad_launch<32, 64, 2>(a, nblk, st);
  else if (ci == 64 && co == 32 && kh == 2) rc = sconv_wgrad_launch<64, 32, 2>(a, nblk, st);
  else if (ci == 64 && co == 64 && kh == 2) rc = sconv_wgrad_launch<64, 64, 2>(a, nblk, st);
  else if (ci == 32 && co == 64 && kh == 1) rc = sconv_wgrad_launch<32, 64, 1>(a, nblk, st);
  else if (ci == 64 && co == 32 && kh == 1) rc = sconv_wgrad_launch<64, 32, 1>(a, nblk, st);
  else if (ci == 32 && co == 32 && kh == 1) rc = sconv_wgrad_launch<32, 32, 1>(a, nblk, st);
  else if (ci == 64 && co == 64 && kh == 1) rc = sconv_wgrad_launch<64, 64, 1>(a, nblk, st);
  if (rc != RDX_OK) return rc;
  const int64_t n = (int64_t)kh * 3 * co * ci;
  float* part2 = part + (int64_t)nblk * n;  // SC_RS more rows of the scratch
  hipLaunchKernelGGL(sconv_wgrad_reduce1_kernel, dim3((unsigned)((n + 255) / 256), SC_RS), dim3(256), 0, st, part, nblk,
                     n, part2);
  hipLaunchKernelGGL(sconv_wgrad_reduce2_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, part2, n, dw);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
