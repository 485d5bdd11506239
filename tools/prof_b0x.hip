// Phase profile of the one-pass block-0 backward (csrc/b0fused.hip built with BX_PROF): synthetic inputs at the
// bench's shape (N = 32 utterances, H = 23, W = 21490), HIP-event time per launch and the per-workgroup
// shader-cycle sums of phases A (ds / out1 staging), B (MFMAs), C (BN + SELU backward), D (dx / d w1 / d wd) and
// the unit prologues. Tools only.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DBX_PROF -I../include tools/prof_b0x.hip -o tools/prof_b0x
#include "../robust-audio-deepfake-evolution_amd/csrc/b0fused.hip"

#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

static uint16_t bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? std::atoi(argv[1]) : 32, H = 23, W = 21490, Wo = W / 3;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
  std::srand(1);
  auto rnd = [] { return (float)std::rand() / (float)RAND_MAX * 2.f - 1.f; };
  std::vector<uint16_t> hx((size_t)N * H * W), hdp((size_t)N * H * Wo * 32), hw2((size_t)6 * 32 * 32);
  std::vector<uint8_t> harg(hdp.size());
  for (auto& v : hx) v = bf(rnd());
  for (auto& v : hdp) v = bf(0.01f * rnd());
  for (auto& v : harg) v = (uint8_t)(std::rand() % 3);
  for (auto& v : hw2) v = bf(0.1f * rnd());
  std::vector<float> hw1(32 * 6), hwd(32 * 3), hbn(5 * 32);
  for (auto& v : hw1) v = 0.3f * rnd();
  for (auto& v : hwd) v = 0.3f * rnd();
  for (int c = 0; c < 32; ++c) {
    hbn[c] = 0.1f * rnd();
    hbn[32 + c] = 0.1f * rnd();
    hbn[64 + c] = 1.f + 0.2f * rnd();
    hbn[96 + c] = 0.1f * rnd();
    hbn[128 + c] = 1.f;
  }
  void *x, *dp, *w2f;
  uint8_t* arg;
  float *w1, *wd, *bn, *dx, *part;
  CK(hipMalloc(&x, hx.size() * 2));
  CK(hipMalloc(&dp, hdp.size() * 2));
  CK(hipMalloc(&arg, harg.size()));
  CK(hipMalloc(&w2f, hw2.size() * 2));
  CK(hipMalloc(&w1, hw1.size() * 4));
  CK(hipMalloc(&wd, hwd.size() * 4));
  CK(hipMalloc(&bn, hbn.size() * 4));
  CK(hipMalloc(&dx, (size_t)N * H * W * 4));
  const int nblk = rdx_b0x_bwd_nblk(N, W);
  CK(hipMalloc(&part, (size_t)nblk * BXB_NPART * 4));
  CK(hipMemcpy(x, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dp, hdp.data(), hdp.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(arg, harg.data(), harg.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(w2f, hw2.data(), hw2.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(w1, hw1.data(), hw1.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(wd, hwd.data(), hwd.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(bn, hbn.data(), hbn.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int rc = rdx_b0x_bwd(x, dp, arg, w1, wd, bn, w2f, dx, part, N, H, W, nullptr);
  CK(hipDeviceSynchronize());
  if (rc) {
    std::fprintf(stderr, "rc %d\n", rc);
    return 1;
  }
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) rdx_b0x_bwd(x, dp, arg, w1, wd, bn, w2f, dx, part, N, H, W, nullptr);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  {  // the forward at the same shape: y, argmax from x (conv2 weights / bias reuse the buffers above)
    void* y;
    uint8_t* yarg;
    CK(hipMalloc(&y, (size_t)N * H * Wo * 32 * 2));
    CK(hipMalloc(&yarg, (size_t)N * H * Wo * 32));
    rc = rdx_b0x_fwd(x, w1, wd, bn, w2f, bn, y, yarg, N, H, W, nullptr);
    CK(hipDeviceSynchronize());
    if (rc) {
      std::fprintf(stderr, "fwd rc %d\n", rc);
      return 1;
    }
    std::vector<unsigned long long> zf(4, 0);
    CK(hipMemcpyToSymbol(HIP_SYMBOL(rdx::bx_prof_f), zf.data(), 4 * 8));
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) rdx_b0x_fwd(x, w1, wd, bn, w2f, bn, y, yarg, N, H, W, nullptr);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float fms;
    CK(hipEventElapsedTime(&fms, e0, e1));
    std::printf("forward ms/launch %.4f\n", fms / reps);
    CK(hipMemcpyFromSymbol(zf.data(), HIP_SYMBOL(rdx::bx_prof_f), 4 * 8));
    const double frows = (double)reps * N * ((Wo + BX_J - 1) / BX_J) * H;
    const char* fn[4] = {"conv2 MFMA", "out1 h+2", "s staging", "pool"};
    for (int k = 0; k < 4; ++k) std::printf("forward %-10s cycles/row %8.0f\n", fn[k], (double)zf[k] / frows);
  }
  std::vector<unsigned long long> prof((size_t)BXB_BLOCKS * 5);
  CK(hipMemcpyFromSymbol(prof.data(), HIP_SYMBOL(bx_prof), prof.size() * 8));
  double sum[5] = {0, 0, 0, 0, 0};
  for (int b = 0; b < nblk; ++b)
    for (int k = 0; k < 5; ++k) sum[k] += (double)prof[(size_t)b * 5 + k];
  const double units = (double)(W / 3 / BX_J + 1) * N, rows = units * (H + 1);
  std::printf("N %d blocks %d ms/launch %.4f\n", N, nblk, ms / reps);
  const char* nm[5] = {"(unused)", "B", "C", "D", "prologue"};
  double tot = 0;
  for (int k = 0; k < 5; ++k) tot += sum[k];
  for (int k = 0; k < 5; ++k)
    std::printf("phase %-8s cycles/row %8.0f  share %.3f\n", nm[k], sum[k] / rows, sum[k] / tot);
  std::printf("total cycles/row %.0f  (per workgroup, last launch)\n", tot / rows);
  return 0;
}
