// Device-clock stamps for timing kernels inside replayed HIP graphs (where HIP events cannot be
// recorded as nodes on ROCm). A one-lane kernel adds sign * wall_clock64() to acc[0] and, for the
// closing stamp, 1 to acc[1]: bracketing a launch with sign -1 / +1 accumulates its duration (in
// wall-clock ticks, constant rate rdx_wallclock_khz) and its count over every replay.
#include "common.h"

namespace rdx {

__global__ void ts_acc_kernel(int64_t* acc, int sign) {
  const int64_t t = (int64_t)wall_clock64();
  acc[0] += sign * t;
  if (sign > 0) acc[1] += 1;
}

}  // namespace rdx

using namespace rdx;

extern "C" int rdx_timestamp_acc(int64_t* acc, int sign, void* stream) {
  RDX_REQUIRE(acc && (sign == 1 || sign == -1));
  hipLaunchKernelGGL(ts_acc_kernel, dim3(1), dim3(1), 0, as_stream(stream), acc, sign);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_wallclock_khz(int device) {
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess) return -1;
  return khz;
}
